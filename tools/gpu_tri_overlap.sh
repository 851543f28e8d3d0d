# r05: the overlapped triplet-centric step (riders: the fused triplets beside the
# combines) -- its parity tests, the segment-capture fix, then the configs[4]
# d = 64 / 128 lines with the overlap on and off, interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-tri_overlap}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "tri_overlap or hash_plan or hot_slots or fused_triplets" > $OUT/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/tests.log | tail -12
[ $rc -eq 0 ] || { echo "tests rc $rc: stopping"; exit $rc; }
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_config5.py > $OUT/config5.log 2>&1
rc=$?
tail -2 $OUT/config5.log
[ $rc -eq 0 ] || { echo "config5 rc $rc: stopping"; exit $rc; }
if [ -n "$WITH_SHARD" ]; then
  timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_distributed.py -k captured > $OUT/captured.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/captured.log | tail -4
  [ $rc -eq 0 ] || { echo "captured rc $rc: stopping"; exit $rc; }
fi
timeout -k 10 500 python3 tools/large_line.py ${LINES:-64 64:noovl 64 64:noovl 128 128:noovl} > $OUT/lines.json 2> $OUT/lines.err || { tail -20 $OUT/lines.err; exit 1; }
cut -c1-400 $OUT/lines.json
