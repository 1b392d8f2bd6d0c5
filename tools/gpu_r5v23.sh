# round 5: device timeline of the serial 8-part frame after the claim-head and seg_k changes
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v23
mkdir -p $OUT
RT_LIB=$PWD/raytracer.js_amd/lib/librt_amd_tl.so timeout -k 10 300 python3 tools/tl_probe.py --parts 8 1 --inflight 1 --frames 32 > $OUT/tl_serial.log 2>&1 || exit 1
