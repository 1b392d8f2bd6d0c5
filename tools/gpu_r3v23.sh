set -u
OUT=gpurun_out/r3v23
mkdir -p $OUT
export PYTHONUNBUFFERED=1
CONFIGS=config3 OUT=$OUT/ab_reread CASES="reread=: keep=raytracer.js_amd/lib/librt_amd_keep.so: reread2=: keep2=raytracer.js_amd/lib/librt_amd_keep.so:" timeout -k 10 400 bash tools/ab_lds.sh > $OUT/ab_reread.txt 2>&1 || exit $?
for P in 4 8 16 24 32; do
  timeout -k 10 200 python3 bench.py --no-js --cpu-budget 0 --no-profile --inflight $P --steps 48 > $OUT/bench_inflight$P.log 2>&1 || exit $?
done
