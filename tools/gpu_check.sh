#!/bin/bash
# GPU-box check: build, gpu tests, smoke, bench, rocprof.  Each GPU step has its own time limit;
# a crash/timeout (anything but exit 0/1) stops the script before the next GPU step.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
export PYTHONUNBUFFERED=1
step build 600 python -c "import __graft_entry__ as g; g.build()"
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu ${TEST_T:-900} python -m pytest tests -m gpu -x -q -p no:cacheprovider
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 900 python bench.py ${BENCH_ARGS:-}
if [ "${PROF:-0}" = 1 ]; then
  export TMPDIR=/tmp
  step rocprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --cpu-budget 0 --no-traffic ${BENCH_ARGS:-}
fi
echo "== done"
