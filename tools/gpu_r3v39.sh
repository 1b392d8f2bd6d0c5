set -u
OUT=gpurun_out/r3v39
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
OUT=$OUT/ab CASES="new=: noshade=raytracer.js_amd/lib/librt_amd_noseg.so: new2=: noshade2=raytracer.js_amd/lib/librt_amd_noseg.so:" timeout -k 10 800 bash tools/ab_lds.sh > $OUT/ab.txt 2>&1 || exit $?
