# round 5: segments per ray doubled for narrow levels (seg_k, RT_SEG_LANES): parity, then 8-part A/B
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v13
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "segmented or level_solo or refill or hinted" > $OUT/pytest_seg.log 2>&1 || { tail -30 $OUT/pytest_seg.log; exit 1; }
tail -2 $OUT/pytest_seg.log
for v in 0 65536 32768 0 65536; do
RT_SEG_LANES=$v timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_lanes$v.log 2>&1 || exit 1
grep '^{' $OUT/probe_lanes$v.log | sed "s/^/lanes=$v /"
done
