# round 5: segments per bounce ray (RT_SEG base 4 / 8) for frames in flight (1 and 8 parts)
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v21
mkdir -p $OUT
for k in 8 4 2 8 4; do
RT_SEG=$k timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_seg$k.log 2>&1 || exit 1
grep '^{' $OUT/probe_seg$k.log | sed "s/^/seg=$k /" | cut -c1-110
done
