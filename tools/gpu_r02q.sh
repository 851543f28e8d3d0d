# k_stream paired / compacted tasks (depth 3): parity + plan tests, then bench lines and kernel stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r02q}
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_plan.py -m gpu > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert|Mismatch" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python3 bench.py --no-sharded > $OUT/bench_default.json 2> $OUT/bench_default.err
cat $OUT/bench_default.json
timeout -k 10 200 python3 bench.py --no-sharded --steps 20 --warmup 5 > $OUT/bench_20.json 2> $OUT/bench_20.err
cat $OUT/bench_20.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --no-sharded > $OUT/prof.log 2>&1
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
head -8 $OUT/kernel_stats.csv
