#!/bin/bash
# PMC passes over the split-path kernels (one counter group per rocprofv3 run; no tracing domains
# combined with --pmc).  Output: $OUT/pmcw/<pass>/..._counter_collection.csv
set -u
OUT=${OUT:-gpurun_out}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p "$OUT/pmcw"
run() {  # name counters...
  local name=$1; shift
  echo "== pmc $name: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/pmcw/$name" -o "$name" --output-format csv -- python3 tools/sweep.py --frames 2 split: > "$OUT/pmcw/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pmcw/$name.log"; exit $rc; fi
}
run inst SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE
run lat SQ_INST_LEVEL_VMEM SQ_INSTS_FLAT SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32
run mem TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
echo "== pmc done"
