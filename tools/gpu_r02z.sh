# LDS-only barriers in the plan kernels: plan/parity tests, plan diagnostics, short call, 20-step bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r02z}
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_plan.py tests/test_gpu_parity.py -m gpu > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert|Mismatch" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log

timeout -k 10 200 python3 tools/short_call.py --reps 30 > $OUT/sc.json 2> $OUT/sc.err
python3 -c "
import json,statistics as st
d=json.loads(open('$OUT/sc.json').read().strip().splitlines()[-1])
r=[x['region_us'] for x in d['reps']]; e=[x['enqueue_us'] for x in d['reps']]
print('region median',st.median(r),'min',min(r),'enqueue median',st.median(e))"
for k in 1 2 3; do timeout -k 10 200 python3 bench.py --no-sharded --no-neumf --no-cpu-baseline --steps 20 --warmup 5 > $OUT/b20_$k.json 2> $OUT/b20_$k.err; python3 -c "import json;d=json.loads(open('$OUT/b20_$k.json').read().strip().splitlines()[-1]);print('bench20',d['value'],d['ms_per_step'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/sc_trace -o sc -- python3 tools/short_call.py --reps 10 > $OUT/sc_traced.json 2> $OUT/sc_traced.err
find $OUT/sc_trace -name "*kernel_stats.csv" -exec cp {} $OUT/sc_kernel_stats.csv \;
grep -E "bplan|k_stream" $OUT/sc_kernel_stats.csv | cut -c1-120
