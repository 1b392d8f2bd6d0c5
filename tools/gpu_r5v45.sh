# round 5: light maps, the large-list cell limit (RT_LM_BIG 64 / 256 / 1024) and the map size on the
# lit benches (every primitive over more cells is tested by every search toward that light)
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v45
mkdir -p $OUT
bl() {  # tag config extra-env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 400 python3 bench.py --config $cfg --lights 2 --no-js --cpu-budget 0 --no-profile > $OUT/bench_${cfg}l_$tag.log 2>&1 || { grep -E "Error" $OUT/bench_${cfg}l_$tag.log | tail -2; return 1; }
  grep '^{' $OUT/bench_${cfg}l_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $cfg+2 lights', d['value'], d['ms_per_step'])"
}
bl b64 config3 && bl b256 config3 RT_LM_BIG=256 && bl b1024 config3 RT_LM_BIG=1024 && bl r512b256 config3 RT_LIGHT_MAP=512 RT_LM_BIG=256 && bl r128 config3 RT_LIGHT_MAP=128 RT_LM_BIG=256 || exit 1
bl b64 config5 && bl b256 config5 RT_LM_BIG=256 && bl b1024 config5 RT_LM_BIG=1024 || exit 1
