#!/bin/bash
# GPU-box check for the segmented continuation walks: gpu tests, a timing sweep over segments per
# ray, the frames-in-flight probe, and a kernel trace of the 8-part probe (one GPU's share of an
# 8-GPU frame).  Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sweep.py --frames 10 ${SWEEP:-base: noseg:RT_SEG=0} > gpurun_out/sweep.log 2>&1 && cat gpurun_out/sweep.log || exit 1
timeout -k 10 300 python tools/pipeline_probe.py --parts ${PARTS:-1 8} --inflight ${INFL:-1 4} > gpurun_out/probe.log 2>&1 && cat gpurun_out/probe.log || exit 1
if [ "${TRACE:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace8 -o run --output-format csv -- python3 tools/pipeline_probe.py --parts 8 --inflight 1 --frames 10 > gpurun_out/trace8.log 2>&1 || exit 1
fi
