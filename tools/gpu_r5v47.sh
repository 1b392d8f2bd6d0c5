# round 5: light maps with the large-list limit at 1024 cells: shadow / host-frame parity, then the
# lit benches with their rocprofv3 passes and CPU baselines (as tools/gpu_round.sh PART=2)
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v47
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_shadow_rays.py tests/test_host_stream.py > $OUT/pytest_shadow.log 2>&1 || { tail -40 $OUT/pytest_shadow.log; exit 1; }
tail -2 $OUT/pytest_shadow.log
timeout -k 10 480 python3 bench.py --config config5 --lights 2 --no-js --cpu-budget 10 --profile-out "$OUT/prof5l" > "$OUT/bench_config5_lights2.log" 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config config3 --lights 2 --no-js --cpu-budget 10 --profile-out "$OUT/prof3l" > "$OUT/bench_config3_lights2.log" 2>&1 || exit $?
for f in bench_config5_lights2 bench_config3_lights2; do grep '^{' $OUT/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
