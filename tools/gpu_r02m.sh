# new GPU tests (config-5 exact shape, yelp-shaped NeuMF) then the full suite
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02m
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_config5.py tests/test_gpu_neumf.py -k "config5 or yelp" > $OUT/new.log 2>&1 || { echo "new tests failed"; grep -E "FAILED|Error|assert|Mismatch|Max" $OUT/new.log | head -30; tail -5 $OUT/new.log; exit 1; }
tail -3 $OUT/new.log
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || { echo "suite failed"; grep -E "FAILED|Error" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
