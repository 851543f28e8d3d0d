# sharded lines with full-size warm chunks
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02v
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-neumf > $OUT/bench.json 2> $OUT/bench.err
python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['value']);[print(k,v['value'],v['ms_per_step'],v.get('route_ms_rank0')) for k,v in d['sharded'].items()]"
