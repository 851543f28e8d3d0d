# final r02 pass: full GPU suite + smoke
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02t
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || { echo "suite failed"; grep -E "FAILED|Error" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log
