#!/bin/bash
# Per-kernel A/B over several builds of librt_amd.so on one box: rocprofv3 --kernel-trace over
# tools/sweep.py for each LIBS entry (name=path; "cur" = the working tree's build), printing each
# kernel's total time per split-path frame (sweep.py traces FRAMES + 2 of them, and one counting frame
# whose k_trace is listed apart; round 5 fixed a divisor of FRAMES + 3).  Each GPU step has its own time limit; stops at the first failure.
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=${OUT:-gpurun_out/abl}
FR=${FRAMES:-10}
mkdir -p "$OUT"
for E in ${LIBS:-cur=}; do
  L=${E%%=*}; P=${E#*=}
  if [ -n "$P" ]; then export RT_LIB=$PWD/$P; else unset RT_LIB; fi
  rm -rf "$OUT/$L"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$L" -o kt --output-format csv -- \
      python3 tools/sweep.py --frames $FR ${SWEEP_ARGS:-} ${SWEEP:-base:} > "$OUT/$L.log" 2>&1 || { echo "$L failed"; tail -5 "$OUT/$L.log"; exit 1; }
  python3 - "$OUT/$L" $((FR + 2)) $L <<'PY'
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
  grep variant "$OUT/$L.log" | cut -c1-150
done
