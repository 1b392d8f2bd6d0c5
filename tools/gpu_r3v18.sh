set -u
OUT=gpurun_out/r3v18
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
OUT=$OUT/ab_flat CASES="flat=: nested=raytracer.js_amd/lib/librt_amd_nested.so: flat2=: nested2=raytracer.js_amd/lib/librt_amd_nested.so:" timeout -k 10 700 bash tools/ab_lds.sh > $OUT/ab_flat.txt 2>&1 || exit $?
