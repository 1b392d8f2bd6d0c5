set -u
OUT=gpurun_out/r3v41
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
for i in 1 2; do
timeout -k 10 200 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_new$i.log 2>&1 || exit $?
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_contfull.so timeout -k 10 200 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_fullgrids$i.log 2>&1 || exit $?
done
