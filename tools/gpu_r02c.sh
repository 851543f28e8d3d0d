# shard mode: full -m gpu suite (distributed tests first)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02c
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -v -x --timeout 200 --timeout-method thread tests/test_gpu_distributed.py > $OUT/dist.log 2>&1 || { echo "dist failed"; tail -40 $OUT/dist.log; exit 1; }
tail -3 $OUT/dist.log
timeout -k 10 900 python3 -u -m pytest -v --timeout 200 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || { echo "suite failed"; grep -E "FAILED|Error" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
