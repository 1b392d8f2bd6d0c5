# round 5: k_walk occupancy (RT_OCC 3 / 4 / 5) on config 5's split level-0 walk, after the f32 screen
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v26
mkdir -p $OUT
timeout -k 10 600 python3 tools/sweep.py --config config5 --frames 4 base: o5:RT_OCC=5 o3:RT_OCC=3 base2: o5b:RT_OCC=5 > $OUT/sweep5.log 2>&1 || { tail $OUT/sweep5.log; exit 1; }
grep variant $OUT/sweep5.log | cut -c1-120
