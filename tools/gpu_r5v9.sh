set -u
OUT=gpurun_out/r5_v9
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for x in 0 1 0 1; do
RT_XCD=$x timeout -k 10 300 python3 bench.py --config config3 --no-js --cpu-budget 0 --steps 20 --no-profile > $OUT/bench_config3_xcd$x.log 2>&1 || exit $?
done
RT_XCD=1 timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_xcd1.log 2>&1 || exit $?
RT_XCD=0 timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_xcd0.log 2>&1 || exit $?
RT_XCD=1 timeout -k 10 400 python3 bench.py --config config5 --no-js --cpu-budget 0 --steps 8 --no-profile > $OUT/bench_config5_xcd1.log 2>&1 || exit $?
RT_XCD=0 timeout -k 10 400 python3 bench.py --config config5 --no-js --cpu-budget 0 --steps 8 --no-profile > $OUT/bench_config5_xcd0.log 2>&1 || exit $?
