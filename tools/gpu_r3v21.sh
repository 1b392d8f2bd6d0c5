set -u
OUT=gpurun_out/r3v21
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_wfcoop.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -p no:cacheprovider > $OUT/pytest_wfcoop.log 2>&1 || exit $?
OUT=$OUT/ab_coop CASES="coop=: nocoop=raytracer.js_amd/lib/librt_amd_nocoop.so: wfcoop=raytracer.js_amd/lib/librt_amd_wfcoop.so: coop2=: nocoop2=raytracer.js_amd/lib/librt_amd_nocoop.so: wfcoop2=raytracer.js_amd/lib/librt_amd_wfcoop.so:" timeout -k 10 800 bash tools/ab_lds.sh > $OUT/ab_coop.txt 2>&1 || exit $?
