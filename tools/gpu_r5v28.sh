# round 5: refill threshold (RT_REFILL idle lanes per claim) on config 5 with per-XCD refill heads
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v28
mkdir -p $OUT
timeout -k 10 800 python3 tools/sweep.py --config config5 --frames 4 base: r4:RT_REFILL=4 r8:RT_REFILL=8 r32:RT_REFILL=32 base2: r8b:RT_REFILL=8 > $OUT/sweep5.log 2>&1 || { tail $OUT/sweep5.log; exit 1; }
grep variant $OUT/sweep5.log | cut -c1-120
