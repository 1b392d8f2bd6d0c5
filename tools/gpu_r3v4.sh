set -u
mkdir -p gpurun_out/r3v4
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_multi_device.py -p no:cacheprovider > gpurun_out/r3v4/pytest_multi.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config config5 --no-js --cpu-budget 0 --profile-out gpurun_out/r3v4/prof5 > gpurun_out/r3v4/bench_config5.log 2>&1 || exit $?
timeout -k 10 400 python tools/pipeline_probe.py --config config4 --parts 1 2 4 8 --inflight 1 16 --frames 24 > gpurun_out/r3v4/pipeline_probe_config4.log 2>&1 || exit $?
