set -u
OUT=gpurun_out/r3v6
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 node tools/js_edit_time.js 1000000 256 > $OUT/js_edit_time.log 2>&1 || exit $?
OUT=$OUT/ab_lds timeout -k 10 900 bash tools/ab_lds.sh > $OUT/ab_lds.txt 2>&1 || exit $?
