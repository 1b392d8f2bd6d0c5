set -u
OUT=gpurun_out/r5_v1
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config config3 --lights 2 --no-js --cpu-budget 0 --no-profile > $OUT/bench_config3_lights2.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --config config5 --lights 2 --no-js --cpu-budget 0 --no-profile > $OUT/bench_config5_lights2.log 2>&1 || exit $?
