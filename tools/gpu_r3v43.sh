set -u
OUT=gpurun_out/r3v43
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 bench.py --config config4 --no-js --cpu-budget 0 --profile-out $OUT/prof4 > $OUT/bench_config4.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --config config2 --no-js --cpu-budget 0 --no-profile > $OUT/bench_config2.log 2>&1 || exit $?
timeout -k 10 300 python tools/pipeline_probe.py --config config4 --parts 1 2 4 8 --inflight 1 16 --frames 32 > $OUT/probe_config4.log 2>&1 || exit $?
