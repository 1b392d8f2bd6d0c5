set -u
OUT=gpurun_out/r3v20
mkdir -p $OUT
export PYTHONUNBUFFERED=1
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_divfma.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_divfma.log 2>&1 || exit $?
OUT=$OUT/ab_div CASES="base=: divfma=raytracer.js_amd/lib/librt_amd_divfma.so: base2=: divfma2=raytracer.js_amd/lib/librt_amd_divfma.so:" timeout -k 10 700 bash tools/ab_lds.sh > $OUT/ab_div.txt 2>&1 || exit $?
