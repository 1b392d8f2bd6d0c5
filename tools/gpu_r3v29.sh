set -u
OUT=gpurun_out/r3v29
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for B in 0 512 256 128; do
  RT_L0_BLOCKS=$B timeout -k 10 200 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 48 > $OUT/probe_l0_$B.log 2>&1 || exit $?
done
