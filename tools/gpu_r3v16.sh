set -u
OUT=gpurun_out/r3v16
mkdir -p $OUT
export PYTHONUNBUFFERED=1
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_rm2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_rm2.log 2>&1 || exit $?
OUT=$OUT/ab_rm CASES="base=: rm1=raytracer.js_amd/lib/librt_amd_rm1.so: rm2=raytracer.js_amd/lib/librt_amd_rm2.so:" timeout -k 10 600 bash tools/ab_lds.sh > $OUT/ab_rm.txt 2>&1 || exit $?
