# round 5: compiler scheduling strategies for the kernels (max-ilp, AMDGPU RP trackers, occupancy
# bias, memory clauses): kernel-trace A/B on config 3, then config 5 for any that helps
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v29
mkdir -p $OUT
L=raytracer.js_amd/lib
OUT=$OUT/ab3 SWEEP_ARGS="--config config3" FRAMES=20 LIBS="cur= ilp=$L/librt_amd_ilp.so trk=$L/librt_amd_trk.so bias=$L/librt_amd_bias.so mem=$L/librt_amd_mem.so cur2=" bash tools/ab_libs.sh > $OUT/ab3.txt 2>&1 || exit 1
OUT=$OUT/ab5 SWEEP_ARGS="--config config5" FRAMES=4 LIBS="cur= ilp=$L/librt_amd_ilp.so trk=$L/librt_amd_trk.so bias=$L/librt_amd_bias.so mem=$L/librt_amd_mem.so" bash tools/ab_libs.sh > $OUT/ab5.txt 2>&1 || exit 1
