set -u
OUT=gpurun_out/r5_v8
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_shadow_rays.py tests/test_host_stream.py tests/test_gpu_parity.py -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config config3 --lights 2 --no-js --cpu-budget 0 --steps 16 --profile-out $OUT/prof3l > $OUT/bench_config3_lights2.log 2>&1 || exit $?
timeout -k 10 480 python3 bench.py --config config5 --lights 2 --no-js --cpu-budget 0 --steps 8 --profile-out $OUT/prof5l > $OUT/bench_config5_lights2.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config config3 --no-js --cpu-budget 0 --steps 20 --no-profile > $OUT/bench_config3.log 2>&1 || exit $?
