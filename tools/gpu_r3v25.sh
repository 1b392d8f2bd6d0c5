set -u
OUT=gpurun_out/r3v25
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
OUT=$OUT/ab_box16 CASES="box16=: box32=raytracer.js_amd/lib/librt_amd_box32.so: box16b=: box32b=raytracer.js_amd/lib/librt_amd_box32.so:" timeout -k 10 700 bash tools/ab_lds.sh > $OUT/ab_box16.txt 2>&1 || exit $?
