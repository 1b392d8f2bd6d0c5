#!/bin/bash
# One GPU-box pass over the round's state: GPU tests, smoke, the driver's bench command (timed, with
# rocprofv3 roofline passes kept under $OUT/prof3), configs 5 and 1, and the config-3 / config-4 part
# probes, configs 5 and 3 with shadow rays (each bench with its rocprofv3 passes and a CPU baseline).  Every GPU step has its own time limit; the first failing step ends the pass.
#   gpurun -- 'OUT=gpurun_out/r4x bash tools/gpu_round.sh'
# PART=1 runs the tests, smoke and the headline bench only; PART=2 the rest (one gpurun call each fits
# the per-call limit).
set -u
OUT=${OUT:-gpurun_out/round}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
PART=${PART:-all}
if [ "$PART" != 2 ]; then
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
T0=$(date +%s)
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 --profile-out "$OUT/prof3" > "$OUT/bench.log" 2>&1 || exit $?
echo "command: python3 bench.py --gpus 1 --steps 20 --warmup 5 --profile-out $OUT/prof3; wall $(( $(date +%s) - T0 )) s" > "$OUT/driver_cmd_wall.txt"
fi
[ "${QUICK:-0}" = 1 ] || [ "$PART" = 1 ] && exit 0
timeout -k 10 480 python3 bench.py --config config5 --no-js --cpu-budget 10 --profile-out "$OUT/prof5" > "$OUT/bench_config5.log" 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config config1 --no-js --cpu-budget 10 --profile-out "$OUT/prof1" > "$OUT/bench_config1.log" 2>&1 || exit $?
timeout -k 10 200 python tools/pipeline_probe.py --config config3 --parts 1 2 4 8 --inflight 1 16 --frames 64 > "$OUT/probe_config3.log" 2>&1 || exit $?
timeout -k 10 200 python tools/pipeline_probe.py --config config4 --parts 1 8 --inflight 1 16 --frames 32 > "$OUT/probe_config4.log" 2>&1 || exit $?
# shadow rays (build extension): BASELINE config 5's "4 bounces + shadow rays", two point lights, with
# the rocprofv3 roofline passes and a CPU baseline like the headline; config 3 with the same lights
timeout -k 10 480 python3 bench.py --config config5 --lights 2 --no-js --cpu-budget 10 --profile-out "$OUT/prof5l" > "$OUT/bench_config5_lights2.log" 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config config3 --lights 2 --no-js --cpu-budget 10 --profile-out "$OUT/prof3l" > "$OUT/bench_config3_lights2.log" 2>&1 || exit $?
