#!/bin/bash
# PMC passes for k_trace on the bench workload (one counter group per rocprofv3 run; no tracing
# domains combined with --pmc).  Output: $OUT/pmc/<pass>/..._counter_collection.csv
set -u
OUT=${OUT:-gpurun_out}
ARGS=${PMC_BENCH_ARGS:---steps 2 --warmup 0 --cpu-budget 0 --no-traffic}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p "$OUT/pmc"
timeout -k 10 120 rocprofv3 -L > "$OUT/pmc/counters_list.txt" 2>&1 || true
run() {  # name counters...
  local name=$1; shift
  echo "== pmc $name: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/pmc/$name" -o "$name" --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc/$name.log"; exit $rc; fi
}
run valu SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run stall SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
echo "== pmc done"
