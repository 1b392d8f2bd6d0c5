# round 5: nontemporal candidate lists A/B (config 5 and 3), and the 8-part serial timeline
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v10
mkdir -p $OUT
OUT=$OUT/ab5 SWEEP_ARGS="--config config5" FRAMES=4 LIBS="cur= nt1=raytracer.js_amd/lib/librt_amd_nt1.so nt2=raytracer.js_amd/lib/librt_amd_nt2.so cur2=" bash tools/ab_libs.sh > $OUT/ab5.txt 2>&1 || exit 1
OUT=$OUT/ab3 SWEEP_ARGS="--config config3" FRAMES=20 LIBS="cur= nt1=raytracer.js_amd/lib/librt_amd_nt1.so nt2=raytracer.js_amd/lib/librt_amd_nt2.so cur2=" bash tools/ab_libs.sh > $OUT/ab3.txt 2>&1 || exit 1
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_tl.so timeout -k 10 300 python3 tools/tl_probe.py --parts 8 1 --inflight 1 --frames 32 > $OUT/tl_serial.log 2>&1 || exit 1
