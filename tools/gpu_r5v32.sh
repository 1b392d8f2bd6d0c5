# round 5: level-0 trip cap between 128 and 192 (8 parts serial)
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v32
mkdir -p $OUT
for cap in 0 144 160 176 0 160; do
RT_L0_CAP=$cap timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 8 1 --inflight 1 --frames 64 > $OUT/probe_cap$cap.log 2>&1 || exit 1
grep '^{' $OUT/probe_cap$cap.log | sed "s/^/cap=$cap /" | cut -c1-100
done
