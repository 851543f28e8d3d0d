# r04: same-box A/B of the streamed call's end: k_stream_flush launch (ACF_TAIL=0)
# against the in-launch tail with various flusher counts (ACF_TAIL_FLUSHERS)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-tail_ab}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "stream or give_up or pipeline or unverified or overlap" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in "1 128" "1 256" "1 64"; do
  set -- $v
  ACF_TAIL=$1 ACF_TAIL_FLUSHERS=$2 timeout -k 10 200 python3 tools/tail_diag.py
done
for v in ${VARIANTS:-"0 128" "1 128" "1 256" "0 128" "1 128" "1 256"}; do
  set -- $v
  ACF_TAIL=$1 ACF_TAIL_FLUSHERS=$2 timeout -k 10 200 python3 tools/short_call.py --reps 30 > $OUT/sc_$1_$2.json 2> $OUT/sc_$1_$2.err
  python3 -c "
import json,statistics as st
d=json.loads(open('$OUT/sc_$1_$2.json').read().strip().splitlines()[-1]); r=[x['region_us'] for x in d['reps']]; e=[x['enqueue_us'] for x in d['reps']]
print('tail $1 flushers $2 region median', st.median(r), 'min', min(r), 'enqueue', st.median(e), 'errors', d['step_errors'])"
done
for v in "0 128" "1 128"; do
  set -- $v
  ACF_TAIL=$1 ACF_TAIL_FLUSHERS=$2 timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/trace_$1 -o sc -- python3 tools/short_call.py --reps 10 > $OUT/trace_$1.log 2>&1
  python3 tools/trace_region.py $(find $OUT/trace_$1 -name '*kernel_trace.csv' | head -1) > $OUT/trace_region_$1.json 2>&1 || true
  python3 -c "
import json
d=json.load(open('$OUT/trace_region_$1.json'))
for r in d[-2:]:
    print('tail $1', r['span_us'], [(x['kernel'][:28], x['dur_us']) for x in r['timeline']])"
done
