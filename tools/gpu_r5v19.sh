# round 5: config 1 (256^2, fused k_trace) regression hunt: per-XCD level-0 claims and the f32
# slot-exit screen
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v19
mkdir -p $OUT
b1() {  # tag extra-env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --config config1 --no-js --cpu-budget 0 --no-profile > $OUT/bench_config1_$tag.log 2>&1 || return 1
  grep '^{' $OUT/bench_config1_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag config1', d['value'], d['ms_per_step'], d['serial']['ms_per_frame'], d['host_frame']['ms_per_frame_median'])"
}
b1 cur && b1 xcd0 RT_XCD=0 && b1 base RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_base.so && b1 base_xcd0 RT_XCD=0 RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_base.so && b1 cur2 || exit 1
