# host enqueue cost of a 20-batch call after the lean PlanPipeline.run path
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-short_call}
mkdir -p $OUT
timeout -k 10 200 python3 tools/short_call.py --reps 30 > $OUT/sc.json 2> $OUT/sc.err
python3 -c "
import json,statistics as st
d=json.loads(open('$OUT/sc.json').read().strip().splitlines()[-1])
r=[x['region_us'] for x in d['reps']]; e=[x['enqueue_us'] for x in d['reps']]
print('region median',st.median(r),'min',min(r),'enqueue median',st.median(e),'empty',d['empty_region_us'][-3:])"
timeout -k 10 200 python3 bench.py --no-sharded --no-neumf --no-cpu-baseline --steps 20 --warmup 5 > $OUT/b20.json 2> $OUT/b20.err
python3 -c "import json;d=json.loads(open('$OUT/b20.json').read().strip().splitlines()[-1]);print('bench20',d['value'],d['ms_per_step'])"
