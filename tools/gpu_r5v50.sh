# round 5: the deferred-record counter on its own cache line: shadow / host-frame parity, then config 5
# unlit and lit frames under a kernel trace (as r5_v49)
set -u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5_v50
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_shadow_rays.py tests/test_host_stream.py > $OUT/pytest_shadow.log 2>&1 || { tail -40 $OUT/pytest_shadow.log; exit 1; }
tail -2 $OUT/pytest_shadow.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 tools/shade_lit_probe.py > $OUT/probe.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
