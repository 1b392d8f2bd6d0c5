set -u
OUT=gpurun_out/r3v33
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
for K in 8 16 32; do
  RT_SEG=$K timeout -k 10 200 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_seg$K.log 2>&1 || exit $?
done
for G in 4 16; do
  RT_CONT_GROUP=$G timeout -k 10 200 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_group$G.log 2>&1 || exit $?
done
