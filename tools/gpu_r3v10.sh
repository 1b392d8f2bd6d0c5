set -u
OUT=gpurun_out/r3v10
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "small_frames or top_levels" -p no:cacheprovider > $OUT/pytest_small.log 2>&1 || exit $?
timeout -k 10 240 python3 tools/small_frame_probe.py --scene config2 --sizes 128 256 512 --frames 30 split:RT_FUSE_MAX=0 fused:RT_FUSE_MAX=100000000,RT_FUSE_LIST=100000000 > $OUT/small_frame_config2.log 2>&1 || exit $?
timeout -k 10 240 python3 tools/small_frame_probe.py --scene small4 --sizes 128 256 512 --frames 30 split:RT_FUSE_MAX=0 fused:RT_FUSE_MAX=100000000,RT_FUSE_LIST=100000000 default: > $OUT/small_frame_small4.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/small_frame_probe.py --scene config1 --sizes 128 256 --frames 50 default: > $OUT/small_frame_config1_default.log 2>&1 || exit $?
T0=$(date +%s)
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 --profile-out $OUT/prof3 > $OUT/bench.log 2>&1 || exit $?
echo "command: python3 bench.py --gpus 1 --steps 20 --warmup 5 --profile-out $OUT/prof3; wall $(( $(date +%s) - T0 )) s" > $OUT/driver_cmd_wall.txt
timeout -k 10 400 python3 bench.py --config config5 --no-js --cpu-budget 0 --profile-out $OUT/prof5 > $OUT/bench_config5.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --config config1 --no-js --cpu-budget 0 > $OUT/bench_config1.log 2>&1 || exit $?
OUT=$OUT/ab_nobox CASES="base=: nobox=raytracer.js_amd/lib/librt_amd_nobox.so:" timeout -k 10 400 bash tools/ab_lds.sh > $OUT/ab_nobox.txt 2>&1 || exit $?
