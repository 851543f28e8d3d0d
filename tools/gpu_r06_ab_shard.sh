# r06: the split-step GPU tests, then a same-box A/B of the sharded lines (world 1):
# a chunk of steps in one plan (default) against one plan beside every step
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r06_ab_shard}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python3 -u -m pytest -x -v --timeout 200 --timeout-method thread \
    ${TESTS:-tests/test_gpu_distributed.py} -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for k in 1 2; do
  for v in chunk perstep; do
    F=""; [ "$v" = perstep ] && F="--per-step-plans"
    timeout -k 10 300 python3 tools/shard_profile.py 24 $F > $OUT/${v}_$k.json 2> $OUT/${v}_$k.err || { tail -20 $OUT/${v}_$k.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/${v}_$k.json').read().strip().splitlines()[-1])
print('$v round $k', {k: (v['ms_per_step'], v['step_errors'], v['launch']) for k, v in d.items()})"
  done
done
