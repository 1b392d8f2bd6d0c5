set -u
OUT=gpurun_out/r3v31
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt8 -o kt --output-format csv -- python3 tools/pipeline_probe.py --config config3 --parts 8 --inflight 16 --frames 64 > $OUT/probe8.log 2>&1 || exit $?
