cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/nmf_fr; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_neumf.py > $OUT/pytest.log 2>&1; rc=$?
tail -25 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in 1 0; do
    ROWS_IN_LINE=$v timeout -k 10 200 python3 tools/neumf_rate.py > $OUT/rate_${v}_$r.log 2>&1 || { echo "rate $v failed"; tail -5 $OUT/rate_${v}_$r.log; exit 1; }
    echo "rows_in_line=$v round $r: $(grep 'rep 1' $OUT/rate_${v}_$r.log)"
  done
done
