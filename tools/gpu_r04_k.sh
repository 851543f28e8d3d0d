# r04: A/Bs of two untested knobs: steps on a high-priority stream beside the
# configs[4] plan stream; the batch plan's sort at 1,024 threads on the short call
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_k}
mkdir -p $OUT
n=0
for v in ACF_PIPE_STEP_PRIO=0 ACF_PIPE_STEP_PRIO=1 ACF_PIPE_STEP_PRIO=0 ACF_PIPE_STEP_PRIO=1; do
  n=$((n+1))
  env $v timeout -k 10 300 python3 tools/large_line.py 64 > $OUT/l$n.json 2> $OUT/l$n.err
  python3 -c "
import json; d=json.loads(open('$OUT/l$n.json').read().strip().splitlines()[-1])
print('$v', round(d['triplets_per_s']/1e6,1), d['step_frac'], d['step_errors'])"
done
for v in 0 1024 0 1024; do
  ACF_BPLAN_SORT=$v timeout -k 10 200 python3 tools/short_call.py --reps 40 --same > $OUT/sc$v.json 2> $OUT/sc$v.err
  python3 -c "
import json,statistics as st
d=json.loads(open('$OUT/sc$v.json').read().strip().splitlines()[-1]); r=[x['region_us'] for x in d['reps']][5:]
print('bplan sort $v region median', st.median(r), 'min', min(r))"
done
