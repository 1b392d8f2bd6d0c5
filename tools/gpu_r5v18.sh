# round 5: grid resolution from the cube root of the list entries; parity of the kept changes (early
# matte deferral, f32 slot-exit screen, shadow grid) over the whole GPU suite, then lit benches
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v18
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for c in config3 config5; do
  timeout -k 10 400 python3 bench.py --config $c --lights 2 --no-js --cpu-budget 0 --no-profile > $OUT/bench_${c}l.log 2>&1 || exit 1
  grep '^{' $OUT/bench_${c}l.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c+2 lights', d['value'], d['ms_per_step'])"
done
