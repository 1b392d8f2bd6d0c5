# round 5: per-XCD band parity (RT_XCD 0 / 15 against the default); the cull-record prefetch (next
# record loaded with the current one, RT_BVH_PF): parity of the scans, then kernel-trace A/B
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v25
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $OUT/pytest_parity.log 2>&1 || { tail -30 $OUT/pytest_parity.log; exit 1; }
tail -2 $OUT/pytest_parity.log
OUT=$OUT/ab3 SWEEP_ARGS="--config config3" FRAMES=20 LIBS="cur= pf0=raytracer.js_amd/lib/librt_amd_pf0.so cur2= pf0b=raytracer.js_amd/lib/librt_amd_pf0.so" bash tools/ab_libs.sh > $OUT/ab3.txt 2>&1 || exit 1
OUT=$OUT/ab5 SWEEP_ARGS="--config config5" FRAMES=4 LIBS="cur= pf0=raytracer.js_amd/lib/librt_amd_pf0.so" bash tools/ab_libs.sh > $OUT/ab5.txt 2>&1 || exit 1
