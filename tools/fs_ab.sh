#!/bin/bash
# k_frame_start A/B on one box: the default library against variant builds
# (tools/build_variant.sh NAME -D...; VARIANTS="default fsptr ..."), two rounds each, kernel stats per run.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/${OUT:-gpurun_out/fsab}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for round in 1 2; do
  for v in ${VARIANTS:-default fsptr}; do
    lib=$R/raytracer.js_amd/lib/librt_amd.so
    [ $v != default ] && lib=$R/raytracer.js_amd/lib/librt_amd_$v.so
    RT_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/${v}_$round" -o run --output-format csv -- \
      python3 "$R/tools/frame_start_ab.py" --frames 40 > "$OUT/${v}_$round.log" 2>&1 || exit $?
  done
done
