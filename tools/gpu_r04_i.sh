# r04: combine finish prefetched on wave 1 + pipelined shard plan inside the captured graph
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_i}
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_config5.py tests/test_gpu_distributed.py -m gpu -k "hash_plan or fused or hot_slots or config5 or shard or split or rehears or collective or route" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for n in 1 2 3 4; do
  v=ACF_HPLAN_PART=$([ $((n % 2)) -eq 1 ] && echo 768 || echo 384)
  env $v timeout -k 10 300 python3 tools/large_line.py 64 > $OUT/l$n.json 2> $OUT/l$n.err
  python3 -c "
import json; d=json.loads(open('$OUT/l$n.json').read().strip().splitlines()[-1])
print('$v large d64', round(d['triplets_per_s']/1e6,1), d['step_frac'], {k: round(v,2) for k,v in (d['per_kernel_avg_us'] or {}).items()})"
done
timeout -k 10 600 python3 bench.py --no-neumf --no-large --no-cpu-baseline --no-eval --steps 20 --warmup 5 > $OUT/b20s.json 2> $OUT/b20s.err
python3 -c "
import json; b=json.loads(open('$OUT/b20s.json').read().strip().splitlines()[-1]); print('bench20', b['value'])
for k,v in b.get('sharded', {}).items():
    if isinstance(v, dict): print('sharded', k, v.get('value'), v.get('ms_per_step'), v.get('config', {}).get('launch'))"
