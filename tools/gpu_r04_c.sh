# r04: the whole GPU suite + smoke, then eval, NeuMF, configs[4] kernel stats,
# the 20-step bench with its sharded lines
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_c}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo "smoke ok"
timeout -k 10 300 python3 -c "
import sys, json, importlib, torch
sys.path.insert(0, '.')
import bench
acf = importlib.import_module(bench.PKG)
print(json.dumps(bench.eval_bench(acf, torch.device('cuda', 0))))
" > $OUT/eval.json 2> $OUT/eval.err
python3 -c "
import json; d=json.load(open('$OUT/eval.json'))
for k,v in d.items(): print(k, v['ms_per_eval'], v['mfma_ms_per_eval'], v['valu_ms_per_eval'], v['positions_equal_valu'], v['roofline']['frac'])"
timeout -k 10 200 python3 tools/neumf_rate.py > $OUT/nmf.log 2>&1
echo "nmf default: $(tail -1 $OUT/nmf.log)"
OUT_TAG=${OUT_TAG:-r04_c}/prof bash tools/gpu_prof_large.sh 2>&1 | grep -E "hplan|triplets|tri_|rocprim|fill" | cut -c1-150
timeout -k 10 600 python3 bench.py --no-neumf --no-large --no-cpu-baseline --no-eval --steps 20 --warmup 5 > $OUT/b20s.json 2> $OUT/b20s.err
python3 -c "
import json; b=json.loads(open('$OUT/b20s.json').read().strip().splitlines()[-1]); print('bench20', b['value'])
sh=b.get('sharded', {})
for k,v in sh.items():
    if isinstance(v, dict): print('sharded', k, v.get('value'), v.get('ms_per_step'), v.get('config', {}).get('launch'))
    else: print('sharded', k, v)"
