# round 5: k_walk_first at 3 / 4 / 5 waves per SIMD (RT_WF_WAVES builds), config 3 kernel trace A/B
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v14
mkdir -p $OUT
OUT=$OUT/ab3 SWEEP_ARGS="--config config3" FRAMES=20 LIBS="cur= wf5=raytracer.js_amd/lib/librt_amd_wf5.so wf3=raytracer.js_amd/lib/librt_amd_wf3.so cur2= wf5b=raytracer.js_amd/lib/librt_amd_wf5.so" bash tools/ab_libs.sh > $OUT/ab3.txt 2>&1 || exit 1
for L in wf5 wf3; do
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_$L.so timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_$L.log 2>&1 || exit 1
done
timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 1 8 --inflight 1 16 --frames 64 > $OUT/probe_cur.log 2>&1 || exit 1
