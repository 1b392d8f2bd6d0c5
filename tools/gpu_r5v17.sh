# round 5: shadow grid resolution (RT_SHADOW_GRID) on the kept build (early matte deferral, f32
# slot-exit screen); the occupancy-map experiment is removed
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v17
mkdir -p $OUT
bl() {  # tag config extra-env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 400 python3 bench.py --config $cfg --lights 2 --no-js --cpu-budget 0 --no-profile > $OUT/bench_${cfg}l_$tag.log 2>&1 || return 1
  grep '^{' $OUT/bench_${cfg}l_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $cfg+2 lights', d['value'], d['ms_per_step'])"
}
bl cur config3 && bl g32 config3 RT_SHADOW_GRID=32 && bl g48 config3 RT_SHADOW_GRID=48 && bl cur2 config3 && bl g32b config3 RT_SHADOW_GRID=32 || exit 1
bl cur config5 && bl g64 config5 RT_SHADOW_GRID=64 && bl g96 config5 RT_SHADOW_GRID=96 || exit 1
