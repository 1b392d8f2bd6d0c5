# round 5: the passes' claim heads off the levels' count lines: every GPU test, config 5 frames under
# a kernel trace (k_first / k_shade at level 0), then the headline and config 5 benches
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v53
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 tools/shade_lit_probe.py > $OUT/probe.log 2>&1 || exit $?
bl() {  # tag config extra-args...
  local tag=$1 cfg=$2; shift 2
  timeout -k 10 400 python3 bench.py --config $cfg --no-js --cpu-budget 0 --no-profile "$@" > $OUT/bench_${cfg}_$tag.log 2>&1 || return 1
  grep '^{' $OUT/bench_${cfg}_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $cfg', d['value'], d['ms_per_step'], d['serial']['value'] if d.get('serial') else '')"
}
bl unlit config3 && bl unlit config5 && bl lit config5 --lights 2 && bl lit config3 --lights 2
