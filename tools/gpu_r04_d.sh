# r04: configs[4] A/B of env knobs on one box (large_line.py at d = 64)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_d}
mkdir -p $OUT
n=0
for v in ${VARIANTS:-"ACF_PIPE_STEP_PRIO=0" "ACF_PIPE_STEP_PRIO=1" "ACF_PIPE_STEP_PRIO=0" "ACF_PIPE_STEP_PRIO=1"}; do
  n=$((n+1))
  env $v timeout -k 10 300 python3 tools/large_line.py 64 > $OUT/l$n.json 2> $OUT/l$n.err
  python3 -c "
import json; d=json.loads(open('$OUT/l$n.json').read().strip().splitlines()[-1])
print('$v', round(d['triplets_per_s']/1e6,1), d['step_frac'], d['avg_launch_us'], d['step_errors'])"
done
