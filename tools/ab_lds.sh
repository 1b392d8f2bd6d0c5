#!/bin/bash
# Same-box A/B of the LDS-staged upper octree levels: per case (name=lib:knobs),
# rocprofv3 --kernel-trace over tools/sweep.py with that build and the knobs (e.g. RT_TOP_LEVELS=3),
# printing each kernel's time per frame and the sweep's event-timed frame; configs 3 and 5.
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab_lds}
mkdir -p "$OUT"
CASES=${CASES:-"base=: top3=:RT_TOP_LEVELS=3 lds128=raytracer.js_amd/lib/librt_amd_lds128.so:RT_TOP_LEVELS=2 lds256=raytracer.js_amd/lib/librt_amd_lds256.so:RT_TOP_LEVELS=3"}
for CFG in ${CONFIGS:-config3 config5}; do
  FR=20; [ "$CFG" = config5 ] && FR=3
  for E in $CASES; do
    N=${E%%=*}; R=${E#*=}; P=${R%%:*}; K=${R#*:}
    if [ -n "$P" ]; then export RT_LIB=$PWD/$P; else unset RT_LIB; fi
    rm -rf "$OUT/$CFG/$N"; mkdir -p "$OUT/$CFG"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$CFG/$N" -o kt --output-format csv -- \
        python3 tools/sweep.py --config $CFG --frames $FR "$N:$K" > "$OUT/$CFG/$N.log" 2>&1 || { echo "$CFG $N failed"; tail -5 "$OUT/$CFG/$N.log"; exit 1; }
    python3 - "$OUT/$CFG/$N" $((FR + 3)) "$CFG $N" <<'PY'
import csv, glob, sys, re
d, frames, tag = sys.argv[1], int(sys.argv[2]), sys.argv[3]
tot = {}
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[a-z_]+?)(?:<|\(|$)", r["Kernel_Name"].split("::")[-1])
        k = m.group(1) if m else r["Kernel_Name"][:30]
        tot[k] = tot.get(k, 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
print(tag, " ".join("%s=%.3f" % (k, v / frames) for k, v in sorted(tot.items(), key=lambda kv: -kv[1]) if v / frames > 0.005))
PY
    grep variant "$OUT/$CFG/$N.log" | cut -c1-220
  done
done
