# round 5: (a) the slot-exit screen on the RayBox's f32 reciprocals (Walker 6 VGPRs lighter); (b) lit
# matte ends deferred from the first-hit pass (no level-0 k_shade for them); (c) the grid's occupancy
# map in LDS for the shadow rays (RT_SHADOW_OCCMAP): parity, then A/B against the previous build (base)
# and a 5-wave k_walk_first build; level-0 grid caps at 8 parts in flight
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v15
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_shadow_rays.py tests/test_host_stream.py > $OUT/pytest_parity.log 2>&1 || { tail -30 $OUT/pytest_parity.log; exit 1; }
tail -2 $OUT/pytest_parity.log
bl() {  # tag config extra-env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 400 python3 bench.py --config $cfg --lights 2 --no-js --cpu-budget 0 --no-profile > $OUT/bench_${cfg}l_$tag.log 2>&1 || return 1
  grep '^{' $OUT/bench_${cfg}l_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $cfg+2 lights', d['value'], d['ms_per_step'])"
}
bl cur config3 && bl occ0 config3 RT_SHADOW_OCCMAP=0 && bl base config3 RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_base.so && bl cur2 config3 || exit 1
bl cur config5 && bl occ0 config5 RT_SHADOW_OCCMAP=0 && bl base config5 RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_base.so || exit 1
OUT=$OUT/ab3 SWEEP_ARGS="--config config3" FRAMES=20 LIBS="cur= base=raytracer.js_amd/lib/librt_amd_base.so wf5=raytracer.js_amd/lib/librt_amd_wf5.so cur2= base2=raytracer.js_amd/lib/librt_amd_base.so" bash tools/ab_libs.sh > $OUT/ab3.txt 2>&1 || exit 1
OUT=$OUT/ab5 SWEEP_ARGS="--config config5" FRAMES=4 LIBS="cur= base=raytracer.js_amd/lib/librt_amd_base.so" bash tools/ab_libs.sh > $OUT/ab5.txt 2>&1 || exit 1
for b in 0 1024 2048 0; do
RT_L0_BLOCKS=$b timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 8 --inflight 16 --frames 64 > $OUT/probe_l0b$b.log 2>&1 || exit 1
grep '^{' $OUT/probe_l0b$b.log | sed "s/^/l0_blocks=$b /"
done
