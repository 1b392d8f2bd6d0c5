# round 5: light maps, the large-list cell limit (RT_LM_BIG 4096 / 16384, smaller maps) and the map size on the
# lit benches (every primitive over more cells is tested by every search toward that light)
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v46
mkdir -p $OUT
bl() {  # tag config extra-env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 400 python3 bench.py --config $cfg --lights 2 --no-js --cpu-budget 0 --no-profile > $OUT/bench_${cfg}l_$tag.log 2>&1 || { grep -E "Error" $OUT/bench_${cfg}l_$tag.log | tail -2; return 1; }
  grep '^{' $OUT/bench_${cfg}l_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $cfg+2 lights', d['value'], d['ms_per_step'])"
}
bl b4096 config3 RT_LM_BIG=4096 && bl b16k config3 RT_LM_BIG=16384 && bl r128b4k config3 RT_LIGHT_MAP=128 RT_LM_BIG=4096 || exit 1
bl b4096 config5 RT_LM_BIG=4096 && bl b16k config5 RT_LM_BIG=16384 && bl r256b4k config5 RT_LIGHT_MAP=256 RT_LM_BIG=4096 || exit 1
