# round 5: per-XCD bands only for k_walk_first by default (RT_XCD=1); bit 8 = the fused kernel, k_walk
# and the segmented levels (A/B 1 vs 9) on configs 1, 3 (1 and 8 parts) and 5
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v20
mkdir -p $OUT
bb() {  # tag config extra-env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 400 python3 bench.py --config $cfg --no-js --cpu-budget 0 --no-profile > $OUT/bench_${cfg}_$tag.log 2>&1 || return 1
  grep '^{' $OUT/bench_${cfg}_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $cfg', d['value'], d['ms_per_step'], d['serial']['ms_per_frame'], d['host_frame']['ms_per_frame_median'])"
}
bb x1 config1 && bb x9 config1 RT_XCD=9 && bb x0 config1 RT_XCD=0 || exit 1
bb x1 config3 && bb x9 config3 RT_XCD=9 && bb x1b config3 || exit 1
bb x1 config5 && bb x9 config5 RT_XCD=9 || exit 1
for x in 1 9 1 9; do
RT_XCD=$x timeout -k 10 300 python tools/pipeline_probe.py --config config3 --parts 8 --inflight 1 16 --frames 64 > $OUT/probe_x$x.log 2>&1 || exit 1
grep '^{' $OUT/probe_x$x.log | sed "s/^/xcd=$x /"
done
