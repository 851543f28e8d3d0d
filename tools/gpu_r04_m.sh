# r04: the host wait of a short call under each hipSetDeviceFlags schedule (same box)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_m}
mkdir -p $OUT
for v in auto spin yield blocking auto spin; do
  timeout -k 10 200 python3 tools/short_call.py --reps 40 --same --sched $v > $OUT/sc_$v.json 2> $OUT/sc_$v.err
  python3 -c "
import json,statistics as st
d=json.loads(open('$OUT/sc_$v.json').read().strip().splitlines()[-1]); r=[x['region_us'] for x in d['reps']][5:]; e=[x['enqueue_us'] for x in d['reps']][5:]
print('$v region median', st.median(r), 'min', min(r), 'enqueue', st.median(e), 'empty', st.median(d['empty_region_us'][5:]), 'err', d['step_errors'])"
  grep hipSetDeviceFlags $OUT/sc_$v.err || true
done
