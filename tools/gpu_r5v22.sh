# round 5: frames in flight and hardware queues at 8 parts (the driver's N = 8 per-GPU workload) and 1 part
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v22
mkdir -p $OUT
for q in 8 12 16 8; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 8 1 --inflight 4 6 8 12 16 --frames 96 > $OUT/probe_q$q.log 2>&1 || exit 1
grep '^{' $OUT/probe_q$q.log | sed "s/^/hwq=$q /" | cut -c1-100
done
