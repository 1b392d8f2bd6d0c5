# round 5: dynamic walk-loop profile of config 3 (RT_WALK_PROF build)
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v33
mkdir -p $OUT
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_prof.so timeout -k 10 300 python tools/walk_profile.py --config config3 > $OUT/walk_profile_config3.log 2>&1 || exit 1
tail -30 $OUT/walk_profile_config3.log
