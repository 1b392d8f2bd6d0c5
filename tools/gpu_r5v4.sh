set -u
OUT=gpurun_out/r5_v5
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_shadow_rays.py -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
for o in 4 5 6; do
RT_SHADOW_OCC=$o timeout -k 10 300 python3 bench.py --config config3 --lights 2 --no-js --cpu-budget 0 --no-profile --steps 16 > $OUT/bench_config3_lights2_o$o.log 2>&1 || exit $?
done
for g in 64 128; do
RT_SHADOW_GRID=$g timeout -k 10 400 python3 bench.py --config config5 --lights 2 --no-js --cpu-budget 0 --no-profile --steps 8 > $OUT/bench_config5_lights2_g$g.log 2>&1 || exit $?
done
timeout -k 10 300 python3 bench.py --config config3 --lights 2 --no-js --cpu-budget 0 --steps 16 --profile-out $OUT/prof3l > $OUT/bench_config3_lights2_prof.log 2>&1 || exit $?
