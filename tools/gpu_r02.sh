# Round-2 check: full -m gpu suite, smoke, default bench, driver-shaped 20-step bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -v --timeout 200 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || echo "pytest rc=$?" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err
cat $OUT/bench.json $OUT/bench20.json
