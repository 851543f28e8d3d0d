# r05: the r03 segment capture of the split step over forced one-rank RCCL, with
# and without the r04 pipelined plan (tools/segment_capture_probe.py).  Stops at
# the first probe that fails (an abort ends the call).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/segment_probe
mkdir -p $OUT
timeout -k 10 120 python3 tools/segment_capture_probe.py nopipe > $OUT/nopipe.log 2>&1
rc=$?
echo "nopipe rc=$rc"; grep -E "seg=|bit for bit" $OUT/nopipe.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python3 tools/segment_capture_probe.py pipe > $OUT/pipe.log 2>&1
rc=$?
echo "pipe rc=$rc"; grep -E "seg=|bit for bit" $OUT/pipe.log
exit 0
