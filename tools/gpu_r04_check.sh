# r04: the GPU suite + smoke, then the driver-shaped 20-batch call (region
# medians, the 20-step bench line, a kernel trace of the region).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_check}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread ${TESTS:-tests} -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
for fs in 1 0; do
  timeout -k 10 200 python3 tools/short_call.py --reps 30 --failsafe $fs > $OUT/sc_fs$fs.json 2> $OUT/sc_fs$fs.err
  python3 -c "
import json,statistics as st
d=json.loads(open('$OUT/sc_fs$fs.json').read().strip().splitlines()[-1]); r=[x['region_us'] for x in d['reps']]; e=[x['enqueue_us'] for x in d['reps']]
print('failsafe $fs region median', st.median(r), 'min', min(r), 'enqueue median', st.median(e), 'empty', st.median(d['empty_region_us']), 'errors', d['step_errors'])"
done
timeout -k 10 200 python3 bench.py --no-sharded --no-neumf --no-large --no-cpu-baseline --no-eval --steps 20 --warmup 5 > $OUT/b20.json 2> $OUT/b20.err
python3 -c "import json; b=json.loads(open('$OUT/b20.json').read().strip().splitlines()[-1]); print('bench20', b['value'], b['ms_per_step'], b['step_errors'], b['stream_recoveries'])"
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/trace -o sc -- python3 tools/short_call.py --reps 10 > $OUT/trace.log 2>&1
python3 tools/trace_region.py $(find $OUT/trace -name '*kernel_trace.csv' | head -1) > $OUT/trace_region.json 2>&1 || true
python3 -c "
import json
d=json.load(open('$OUT/trace_region.json'))
for r in d[-3:]:
    print(r['span_us'], [(x['kernel'][:28], x['dur_us']) for x in r['timeline']])"
