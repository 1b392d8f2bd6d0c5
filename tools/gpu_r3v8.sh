set -u
OUT=gpurun_out/r3v8
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
T0=$(date +%s.%N)
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 --profile-out $OUT/prof3 > $OUT/bench.log 2>&1 || exit $?
echo "command: python3 bench.py --gpus 1 --steps 20 --warmup 5 --profile-out $OUT/prof3; wall $(echo "$(date +%s.%N) - $T0" | bc) s" > $OUT/driver_cmd_wall.txt
timeout -k 10 400 python3 bench.py --config config5 --no-js --cpu-budget 0 --profile-out $OUT/prof5 > $OUT/bench_config5.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/small_frame_probe.py --sizes 128 256 --frames 50 base: fused:RT_SPLIT=0 nohint:RT_HINTS=0 > $OUT/small_frame.log 2>&1 || exit $?
