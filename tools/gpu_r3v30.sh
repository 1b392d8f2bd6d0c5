set -u
OUT=gpurun_out/r3v30
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/pipeline_probe.py --config config3 --parts 1 2 4 8 --inflight 1 16 --frames 64 > $OUT/probe_submit.log 2>&1 || exit $?
