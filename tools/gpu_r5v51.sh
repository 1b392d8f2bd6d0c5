# round 5: the deferred-record counter on its own line: every GPU test, smoke, the headline bench and
# the lit benches with their rocprofv3 passes and CPU baselines
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v51
mkdir -p $OUT
OUT=$OUT PART=1 bash tools/gpu_round.sh || exit $?
tail -1 $OUT/pytest_gpu.log
timeout -k 10 480 python3 bench.py --config config5 --lights 2 --no-js --cpu-budget 10 --profile-out "$OUT/prof5l" > "$OUT/bench_config5_lights2.log" 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config config3 --lights 2 --no-js --cpu-budget 10 --profile-out "$OUT/prof3l" > "$OUT/bench_config3_lights2.log" 2>&1 || exit $?
for f in bench bench_config5_lights2 bench_config3_lights2; do grep '^{' $OUT/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
