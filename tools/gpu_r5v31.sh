# round 5: strided level-0 tile order (RT_L0_PERM) for small parts: parity, then 8 / 4 / 1 parts
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v31
mkdir -p $OUT
RT_L0_PERM=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_host_stream.py > $OUT/pytest_perm.log 2>&1 || { tail -30 $OUT/pytest_perm.log; exit 1; }
tail -2 $OUT/pytest_perm.log
for p in 0 1 0 1; do
RT_L0_PERM=$p timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 8 4 1 --inflight 1 16 --frames 64 > $OUT/probe_perm$p.log 2>&1 || exit 1
grep '^{' $OUT/probe_perm$p.log | sed "s/^/perm=$p /" | cut -c1-100
done
