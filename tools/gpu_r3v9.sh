set -u
OUT=gpurun_out/r3v9
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 240 python3 tools/small_frame_probe.py --sizes 128 256 384 512 --frames 40 split:RT_FUSE_MAX=0 fused:RT_FUSE_MAX=100000000 > $OUT/small_frame_config1.log 2>&1 || exit $?
timeout -k 10 240 python3 tools/small_frame_probe.py --scene config3 --sizes 128 256 384 512 --frames 30 split:RT_FUSE_MAX=0 fused:RT_FUSE_MAX=100000000 > $OUT/small_frame_config3.log 2>&1 || exit $?
timeout -k 10 240 python3 tools/sweep.py --config config3 --frames 20 leaf1:RT_BVH_LEAF=1 leaf2:RT_BVH_LEAF=2 leaf4:RT_BVH_LEAF=4 leaf1b:RT_BVH_LEAF=1 > $OUT/sweep_leaf_config3.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/sweep.py --config config5 --frames 3 leaf1:RT_BVH_LEAF=1 leaf2:RT_BVH_LEAF=2 leaf4:RT_BVH_LEAF=4 > $OUT/sweep_leaf_config5.log 2>&1 || exit $?
