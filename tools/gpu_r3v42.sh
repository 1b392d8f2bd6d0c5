set -u
OUT=gpurun_out/r3v42
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
T0=$(date +%s)
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 --profile-out $OUT/prof3 > $OUT/bench.log 2>&1 || exit $?
echo "command: python3 bench.py --gpus 1 --steps 20 --warmup 5 --profile-out $OUT/prof3; wall $(( $(date +%s) - T0 )) s" > $OUT/driver_cmd_wall.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-profile --cpu-budget 0 > $OUT/bench_repeat.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --config config5 --no-js --cpu-budget 0 --profile-out $OUT/prof5 > $OUT/bench_config5.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --config config1 --no-js --cpu-budget 0 > $OUT/bench_config1.log 2>&1 || exit $?
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 200 python tools/pipeline_probe.py --config config3 --parts 1 2 4 8 --inflight 1 16 --frames 64 > $OUT/probe_config3.log 2>&1 || exit $?
