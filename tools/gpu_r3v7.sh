set -u
OUT=gpurun_out/r3v7
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 node tools/js_edit_time.js 1000000 256 > $OUT/js_edit_time.log 2>&1 || exit $?
OUT=$OUT/ab_lds timeout -k 10 900 bash tools/ab_lds.sh > $OUT/ab_lds.txt 2>&1 || exit $?
OUT=$OUT/ab_head CASES="base=: head0=raytracer.js_amd/lib/librt_amd_head0.so: buf=raytracer.js_amd/lib/librt_amd_buf.so: fpipe=raytracer.js_amd/lib/librt_amd_fpipe.so:" timeout -k 10 700 bash tools/ab_lds.sh > $OUT/ab_head.txt 2>&1 || exit $?
timeout -k 10 300 python tools/sweep.py --config config5 --frames 3 base: occ8:RT_OCC=8 > $OUT/sweep_occ_config5.log 2>&1 || exit $?
