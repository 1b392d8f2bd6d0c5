# round 5: k_shadow_rays occupancy (RT_SHADOW_OCC 4 / 5 / 6) on lit configs 3 and 5
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v24
mkdir -p $OUT
bl() {  # tag config extra-env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 400 python3 bench.py --config $cfg --lights 2 --no-js --cpu-budget 0 --no-profile > $OUT/bench_${cfg}l_$tag.log 2>&1 || return 1
  grep '^{' $OUT/bench_${cfg}l_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $cfg+2 lights', d['value'], d['ms_per_step'])"
}
bl o5 config3 && bl o4 config3 RT_SHADOW_OCC=4 && bl o6 config3 RT_SHADOW_OCC=6 && bl o5b config3 && bl o4b config3 RT_SHADOW_OCC=4 || exit 1
bl o5 config5 && bl o4 config5 RT_SHADOW_OCC=4 || exit 1
