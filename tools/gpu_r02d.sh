# sharded lines of the bench (world 1)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02d
mkdir -p $OUT
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-neumf --no-large --steps 647 --warmup 647 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json; b=json.load(open('$OUT/bench.json'))
print('default', b['value'])
for k,v in b['sharded'].items(): print(k, json.dumps(v))"
