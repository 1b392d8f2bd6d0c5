set -u
OUT=gpurun_out/r3v26
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
OUT=$OUT/ab_cube CASES="cube=: load=raytracer.js_amd/lib/librt_amd_cubeload.so: cube2=: load2=raytracer.js_amd/lib/librt_amd_cubeload.so:" timeout -k 10 700 bash tools/ab_lds.sh > $OUT/ab_cube.txt 2>&1 || exit $?
