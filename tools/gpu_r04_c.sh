# r04: eval parity + timing after the exclusion-span change; NeuMF defaults
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_c}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_reference.py tests/test_gpu_torch_ops.py tests/test_gpu_e2e_video.py tests/test_gpu_neumf.py tests/test_gpu_distributed.py -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_plan.py -m gpu > $OUT/pytest_plan.log 2>&1 || { tail -20 $OUT/pytest_plan.log; exit 1; }
echo "plan tests: $(tail -1 $OUT/pytest_plan.log)"
for v in radix count radix count; do
  ACF_BPLAN_SORT=$v timeout -k 10 200 python3 tools/short_call.py --reps 40 --same > $OUT/sc_sort$v.json 2> $OUT/sc_sort$v.err
  python3 -c "
import json,statistics as st
d=json.loads(open('$OUT/sc_sort$v.json').read().strip().splitlines()[-1]); r=[x['region_us'] for x in d['reps']][5:]
print('sort $v region median', st.median(r), 'min', min(r))"
done
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
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/large_prof -o lg -- python3 -c "
import sys, json, importlib, torch
sys.path.insert(0, '.')
import bench
acf = importlib.import_module(bench.PKG); ops = importlib.import_module(bench.PKG + '.ops')
dev = torch.device('cuda', 0)
big = acf.synthetic_large(device=dev)
r = bench.large_batch_roofline(acf, ops, dev, big, 64)
print('large d64', r['triplets_per_s'], r['step_bandwidth']['frac'])
" > $OUT/large_prof.log 2>&1
grep "large d64" $OUT/large_prof.log
python3 -c "
import csv,glob
f=glob.glob('$OUT/large_prof/**/*kernel_stats.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
for r in rows[:16]: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])"
timeout -k 10 600 python3 bench.py --no-neumf --no-large --no-cpu-baseline --no-eval --steps 20 --warmup 5 > $OUT/b20s.json 2> $OUT/b20s.err
python3 -c "
import json; b=json.loads(open('$OUT/b20s.json').read().strip().splitlines()[-1]); print('bench20', b['value'])
sh=b.get('sharded', {})
for k,v in sh.items():
    if isinstance(v, dict): print('sharded', k, v.get('value'), v.get('ms_per_step'), v.get('config', {}).get('launch'))
    else: print('sharded', k, v)"
