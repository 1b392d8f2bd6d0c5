# round 5: level-0 walk cap (RT_L0_CAP: long primary walks handed to the segmented level 1): parity,
# then the serial 8-part frame and full frames at several caps
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v30
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "level0_cap" > $OUT/pytest_cap.log 2>&1 || { tail -30 $OUT/pytest_cap.log; exit 1; }
tail -2 $OUT/pytest_cap.log
for cap in 0 128 192 256 384 0; do
RT_L0_CAP=$cap timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 8 1 --inflight 1 16 --frames 64 > $OUT/probe_cap$cap.log 2>&1 || exit 1
grep '^{' $OUT/probe_cap$cap.log | sed "s/^/cap=$cap /" | cut -c1-100
done
