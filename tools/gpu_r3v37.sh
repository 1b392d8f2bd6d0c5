set -u
OUT=gpurun_out/r3v37
mkdir -p $OUT
export PYTHONUNBUFFERED=1
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_segshade.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_segshade.so timeout -k 10 200 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_fused.log 2>&1 || exit $?
timeout -k 10 200 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_noshade.log 2>&1 || exit $?
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_segshade.so timeout -k 10 200 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_fused2.log 2>&1 || exit $?
timeout -k 10 200 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_noshade2.log 2>&1 || exit $?
CONFIGS=config3 OUT=$OUT/ab_segshade CASES="fused=raytracer.js_amd/lib/librt_amd_segshade.so: noshade=:" timeout -k 10 300 bash tools/ab_lds.sh > $OUT/ab_segshade.txt 2>&1 || exit $?
