# round 5: banded refill claims + level-0 refill walk: parity, then A/B on configs 5 and 3
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v12
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "refill or split_equals or hinted or level_solo" > $OUT/pytest_refill.log 2>&1 || { tail -30 $OUT/pytest_refill.log; exit 1; }
tail -3 $OUT/pytest_refill.log
timeout -k 10 300 python3 tools/sweep.py --config config5 --frames 4 base: l0r:RT_L0_REFILL=1 l0r32:RT_L0_REFILL=1,RT_REFILL=32 base2: > $OUT/sweep5.log 2>&1 || { tail $OUT/sweep5.log; exit 1; }
timeout -k 10 300 python3 tools/sweep.py --config config3 --frames 20 base: l0r:RT_L0_REFILL=1,RT_WF_LIST=-1 sep:RT_WF_LIST=-1 base2: > $OUT/sweep3.log 2>&1 || { tail $OUT/sweep3.log; exit 1; }
RT_L0_REFILL=1 RT_WF_LIST=-1 timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_l0r.log 2>&1 || exit 1
