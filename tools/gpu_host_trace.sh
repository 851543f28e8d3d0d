# r04: where the driver-shaped call's wall time goes on the host: short_call
# (fast path: the same call repeated) under a HIP runtime-API + kernel trace
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-host_trace}
mkdir -p $OUT
for v in "--same" ""; do
  timeout -k 10 200 python3 tools/short_call.py --reps 30 $v > $OUT/sc$v.json 2> $OUT/sc$v.err
  python3 -c "
import json,statistics as st
d=json.loads(open('$OUT/sc$v.json').read().strip().splitlines()[-1]); r=[x['region_us'] for x in d['reps']]; e=[x['enqueue_us'] for x in d['reps']]
print('short_call $v region median', st.median(r), 'min', min(r), 'enqueue', st.median(e), 'empty', st.median(d['empty_region_us']))"
done
timeout -k 10 200 python3 bench.py --no-sharded --no-neumf --no-large --no-cpu-baseline --no-eval --steps 20 --warmup 5 > $OUT/b20.json 2> $OUT/b20.err
python3 -c "import json; b=json.loads(open('$OUT/b20.json').read().strip().splitlines()[-1]); print('bench20', b['value'], b['ms_per_step'], b['step_errors'], b['stream_recoveries'])"
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace -f csv -d $OUT/trace -o sc -- python3 tools/short_call.py --reps 8 --same > $OUT/trace.log 2>&1
ls $OUT/trace/*/ 2>/dev/null | head; find $OUT/trace -name '*.csv' | head
