# closing pass: full GPU suite + smoke, bench lines, then rocprofv3 stats + PMC passes
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-closing}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || { echo "suite failed"; grep -E "FAILED|Error" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log
timeout -k 10 250 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
timeout -k 10 250 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_20.json 2> $OUT/bench_20.err
python3 -c "import json;[print(f, json.loads(open('$OUT/'+f).read().strip().splitlines()[-1])['value']) for f in ('bench_default.json','bench_20.json')]"
true
