# round 5: light maps with bounded fills (zeroed entries, per-cell and large-list caps): shadow and
# host-frame parity, the lit benches at the default map size, then the R=1024 config 5 case that faulted
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v41
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_shadow_rays.py tests/test_host_stream.py > $OUT/pytest_shadow.log 2>&1 || { tail -40 $OUT/pytest_shadow.log; exit 1; }
tail -2 $OUT/pytest_shadow.log
bl() {  # tag config extra-env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 400 python3 bench.py --config $cfg --lights 2 --no-js --cpu-budget 0 --no-profile > $OUT/bench_${cfg}l_$tag.log 2>&1 || { grep -E "Error" $OUT/bench_${cfg}l_$tag.log | tail -2; return 1; }
  grep '^{' $OUT/bench_${cfg}l_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $cfg+2 lights', d['value'], d['ms_per_step'])"
}
bl map config3 && bl grid config3 RT_LIGHT_MAP=-1 && bl map config5 && bl grid config5 RT_LIGHT_MAP=-1 || exit 1
bl m1024 config5 RT_LIGHT_MAP=1024 || exit 1
