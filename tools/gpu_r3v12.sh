set -u
OUT=gpurun_out/r3v13
mkdir -p $OUT
export PYTHONUNBUFFERED=1

OUT=$OUT/ab_refill CONFIGS=config5 CASES="refold=raytracer.js_amd/lib/librt_amd_refold.so: nofr=raytracer.js_amd/lib/librt_amd_nofr.so: fronly=raytracer.js_amd/lib/librt_amd_fr_only.so: base=: refold2=raytracer.js_amd/lib/librt_amd_refold.so:" timeout -k 10 500 bash tools/ab_lds.sh > $OUT/ab_refill.txt 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --config config5 --no-js --cpu-budget 0 --profile-out $OUT/prof5 > $OUT/bench_config5.log 2>&1 || exit $?
