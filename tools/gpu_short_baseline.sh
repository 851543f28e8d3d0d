# The driver-shaped 20-batch call on the current libraries: region / enqueue
# medians (verified and unverified streamed calls), the 20-step bench line and a
# kernel trace of the region (tools/trace_region.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-short_baseline}
mkdir -p $OUT
for fs in 1 0; do
  timeout -k 10 200 python3 tools/short_call.py --reps 30 --failsafe $fs > $OUT/sc_fs$fs.json 2> $OUT/sc_fs$fs.err
  python3 -c "
import json,statistics as st
d=json.loads(open('$OUT/sc_fs$fs.json').read().strip().splitlines()[-1]); r=[x['region_us'] for x in d['reps']]; e=[x['enqueue_us'] for x in d['reps']]
print('failsafe $fs region median', st.median(r), 'min', min(r), 'enqueue median', st.median(e), 'empty', st.median(d['empty_region_us']))"
done
timeout -k 10 200 python3 bench.py --no-sharded --no-neumf --no-large --no-cpu-baseline --no-eval --steps 20 --warmup 5 > $OUT/b20.json 2> $OUT/b20.err
python3 -c "import json; b=json.loads(open('$OUT/b20.json').read().strip().splitlines()[-1]); print('bench20', b['value'], b['ms_per_step'])"
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/trace -o sc -- python3 tools/short_call.py --reps 10 > $OUT/trace.log 2>&1
python3 tools/trace_region.py $(find $OUT/trace -name '*kernel_trace.csv' | head -1) > $OUT/trace_region.txt 2>&1 || true
tail -40 $OUT/trace_region.txt
