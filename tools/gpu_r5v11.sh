# round 5: segments per bounce ray (RT_SEG) at 1 and 8 parts, serial and in flight
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v11
mkdir -p $OUT
for k in 8 16 32 64 8; do
RT_SEG=$k timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_seg$k.log 2>&1 || exit 1
done
for k in 8 16 32; do
RT_SEG=$k timeout -k 10 300 python tools/pipeline_probe.py --config config5 --parts 1 --inflight 1 --frames 6 > $OUT/probe5_seg$k.log 2>&1 || exit 1
done
