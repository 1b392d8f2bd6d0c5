set -u
OUT=gpurun_out/r3v19
mkdir -p $OUT
export PYTHONUNBUFFERED=1
T0=$(date +%s)
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 --profile-out $OUT/prof3 > $OUT/bench.log 2>&1 || exit $?
echo "command: python3 bench.py --gpus 1 --steps 20 --warmup 5 --profile-out $OUT/prof3; wall $(( $(date +%s) - T0 )) s" > $OUT/driver_cmd_wall.txt
timeout -k 10 400 python3 bench.py --config config5 --no-js --cpu-budget 0 --profile-out $OUT/prof5 > $OUT/bench_config5.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/sweep.py --config config5 --frames 3 base: occ8:RT_OCC=8 occ4:RT_OCC=4 base2: > $OUT/sweep_occ_config5.log 2>&1 || exit $?
