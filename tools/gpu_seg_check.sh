set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sweep.py --frames 10 base: noseg:RT_SEG=0 base2: > gpurun_out/sweep.log 2>&1 && cat gpurun_out/sweep.log
timeout -k 10 300 python tools/pipeline_probe.py --parts 1 8 --inflight 1 4 > gpurun_out/probe.log 2>&1 && cat gpurun_out/probe.log
