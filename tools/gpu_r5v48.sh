# round 5: light maps: the shadow kernel's waves per SIMD (RT_SHADOW_OCC 4 / 5 / 6) on the lit benches

set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v48
mkdir -p $OUT
bl() {  # tag config extra-env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 400 python3 bench.py --config $cfg --lights 2 --no-js --cpu-budget 0 --no-profile > $OUT/bench_${cfg}l_$tag.log 2>&1 || { grep -E "Error" $OUT/bench_${cfg}l_$tag.log | tail -2; return 1; }
  grep '^{' $OUT/bench_${cfg}l_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $cfg+2 lights', d['value'], d['ms_per_step'])"
}
bl o4 config3 RT_SHADOW_OCC=4 && bl o5 config3 RT_SHADOW_OCC=5 && bl o6 config3 RT_SHADOW_OCC=6 || exit 1
bl o4 config5 RT_SHADOW_OCC=4 && bl o5 config5 RT_SHADOW_OCC=5 && bl o6 config5 RT_SHADOW_OCC=6 || exit 1
