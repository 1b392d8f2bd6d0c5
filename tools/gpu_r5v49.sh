# round 5: config 5 device frames unlit, then lit (two lights), under a kernel trace: the lit frame's
# extra k_shade time, level by level
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v49
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 tools/shade_lit_probe.py > $OUT/probe.log 2>&1
rc=$?
echo "rc=$rc"; tail -3 $OUT/probe.log
exit $rc
