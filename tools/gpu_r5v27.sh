# round 5: config 5's refill walk at 5 (default) / 6 / 8 waves per SIMD (spilling builds)
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v27
mkdir -p $OUT
OUT=$OUT/ab5 SWEEP_ARGS="--config config5" FRAMES=4 LIBS="cur= rf6=raytracer.js_amd/lib/librt_amd_rf6.so rf8=raytracer.js_amd/lib/librt_amd_rf8.so cur2=" bash tools/ab_libs.sh > $OUT/ab5.txt 2>&1 || exit 1
