# Same-box A/B of walk-loop builds: LIBS (name=path pairs, "cur=" the working tree) on config 3
# (20 frames) and config 5 (3 frames), then the walk-loop profile of the RT_WALK_PROF build.
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/wp
OUT=gpurun_out/ab_w3 LIBS="$LIBS" FRAMES=20 bash tools/ab_libs.sh > gpurun_out/ab_w3.txt 2>&1
OUT=gpurun_out/ab_w5 LIBS="$LIBS" FRAMES=3 SWEEP_ARGS="--config config5" bash tools/ab_libs.sh > gpurun_out/ab_w5.txt 2>&1
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_prof.so timeout -k 10 120 python tools/walk_profile.py --config config3 > gpurun_out/wp/c3_w.log 2>&1
