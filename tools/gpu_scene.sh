#!/bin/bash
# GPU-box check for the resident scene: build, the GPU tests, scene build / upload / update timing.
set -u
mkdir -p gpurun_out
make -C raytracer.js_amd -j16 >/dev/null && make -C raytracer.js_amd/js >/dev/null && make -C oracle >/dev/null || exit 3
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ${TESTS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python tools/scene_timing.py > gpurun_out/scene_timing.log 2>&1
tail -20 gpurun_out/scene_timing.log
exit $rc
