#!/bin/bash
# Same-box A/B of two library builds (lib/librt_amd_ref.so vs lib/librt_amd.so), alternating runs of
# tools/sweep.py; optional GPU tests first (TESTS=1).  Each GPU step has its own time limit.
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
      > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  for L in ref new; do
    if [ $L = ref ]; then export RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_ref.so; else unset RT_LIB; fi
    echo -n "$L "
    timeout -k 10 200 python tools/sweep.py --frames ${FRAMES:-30} ${SWEEP:-base:} 2>&1 | grep variant | cut -c1-110 || exit 1
  done
done
