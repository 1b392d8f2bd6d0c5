set -u
OUT=gpurun_out/r3v27
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/pipeline_probe.py --config config3 --parts 1 2 4 8 --inflight 1 16 32 --frames 48 > $OUT/pipeline_probe_config3.log 2>&1 || exit $?
