set -u
OUT=gpurun_out/r3v14
mkdir -p $OUT
export PYTHONUNBUFFERED=1
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_wf.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -p no:cacheprovider > $OUT/pytest_wf.log 2>&1 || exit $?
OUT=$OUT/ab_wf CASES="base=: wf=raytracer.js_amd/lib/librt_amd_wf.so: base2=: wf2=raytracer.js_amd/lib/librt_amd_wf.so:" timeout -k 10 700 bash tools/ab_lds.sh > $OUT/ab_wf.txt 2>&1 || exit $?
timeout -k 10 400 python3 tools/sweep.py --config config5 --frames 3 base: sh4:RT_SHADE_OCC=4 sh5:RT_SHADE_OCC=5 > $OUT/sweep_shade_config5.log 2>&1 || exit $?
