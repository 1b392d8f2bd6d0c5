set -u
OUT=gpurun_out/r3v11
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 tools/sweep.py --config config5 --frames 3 g16:RT_REFILL=16 g8:RT_REFILL=8 g24:RT_REFILL=24 g32:RT_REFILL=32 g16b:RT_REFILL=16 > $OUT/sweep_refill_config5.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/sweep.py --config config5 --frames 3 base: cap48:RT_CAND_CAP=48 cap96:RT_CAND_CAP=96 cg16:RT_CONT_GROUP=16 > $OUT/sweep_misc_config5.log 2>&1 || exit $?
