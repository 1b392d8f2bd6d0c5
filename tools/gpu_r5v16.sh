# round 5: shadow grid search stepping over empty blocks (LDS occupancy map, up to 16 cells a trip):
# shadow parity, then lit benches with the map on / off and other grid resolutions
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v16
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_shadow_rays.py > $OUT/pytest_shadow.log 2>&1 || { tail -30 $OUT/pytest_shadow.log; exit 1; }
tail -2 $OUT/pytest_shadow.log
bl() {  # tag config extra-env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 400 python3 bench.py --config $cfg --lights 2 --no-js --cpu-budget 0 --no-profile > $OUT/bench_${cfg}l_$tag.log 2>&1 || return 1
  grep '^{' $OUT/bench_${cfg}l_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $cfg+2 lights', d['value'], d['ms_per_step'])"
}
bl cur config3 && bl occ0 config3 RT_SHADOW_OCCMAP=0 && bl g32 config3 RT_SHADOW_GRID=32 && bl g128 config3 RT_SHADOW_GRID=128 && bl cur2 config3 || exit 1
bl cur config5 && bl occ0 config5 RT_SHADOW_OCCMAP=0 && bl g64 config5 RT_SHADOW_GRID=64 || exit 1
