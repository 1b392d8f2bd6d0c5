set -u
OUT=gpurun_out/r3v6
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 node tools/js_edit_time.js 1000000 256 > $OUT/js_edit_time.log 2>&1 || exit $?
OUT=$OUT/ab_lds timeout -k 10 900 bash tools/ab_lds.sh > $OUT/ab_lds.txt 2>&1 || exit $?
timeout -k 10 300 python tools/sweep.py --config config5 --frames 3 base: occ8:RT_OCC=8 > $OUT/sweep_occ_config5.log 2>&1 || exit $?
timeout -k 10 200 python tools/sweep.py --config config3 --frames 20 base: occ8:RT_OCC=8 base2: > $OUT/sweep_occ_config3.log 2>&1 || exit $?
OUT=$OUT/ab_head CASES="base=: head0=raytracer.js_amd/lib/librt_amd_head0.so: buf=raytracer.js_amd/lib/librt_amd_buf.so: fpipe=raytracer.js_amd/lib/librt_amd_fpipe.so:" timeout -k 10 600 bash tools/ab_lds.sh > $OUT/ab_head.txt 2>&1 || exit $?
