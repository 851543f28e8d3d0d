# r04: eval tests + the eval line (auto / MFMA / VALU) + a kernel trace of it,
# then the tail A/B of tools/gpu_tail_ab.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_eval}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_reference.py tests/test_gpu_torch_ops.py -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 -c "
import sys, json, importlib, torch
sys.path.insert(0, '.')
import bench
acf = importlib.import_module(bench.PKG)
print(json.dumps(bench.eval_bench(acf, torch.device('cuda', 0))))
" > $OUT/eval.json 2> $OUT/eval.err
cat $OUT/eval.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ev -- python3 -c "
import sys, json, importlib, torch
sys.path.insert(0, '.')
import bench
acf = importlib.import_module(bench.PKG)
bench.eval_bench(acf, torch.device('cuda', 0))
" > $OUT/prof.log 2>&1
head -12 $(find $OUT/prof -name '*kernel_stats.csv' | head -1)
for v in "8 96" "16 96" "16 64" "16 48" "8 96" "16 64"; do
  set -- $v
  ACF_NMF_LAZY_S=$1 ACF_NMF_CATCHUP_WG=$2 timeout -k 10 200 python3 tools/neumf_rate.py > $OUT/nmf_$1_$2.log 2>&1
  echo "nmf lazy_s $1 wg $2: $(tail -1 $OUT/nmf_$1_$2.log)"
done
timeout -k 10 400 python3 -c "
import sys, json, importlib, torch
sys.path.insert(0, '.')
import bench
acf = importlib.import_module(bench.PKG); ops = importlib.import_module(bench.PKG + '.ops')
dev = torch.device('cuda', 0)
big = acf.synthetic_large(device=dev)
print('large d64', json.dumps(bench.large_batch_roofline(acf, ops, dev, big, 64)))
" > $OUT/large.json 2> $OUT/large.err
python3 -c "
import json
for l in open('$OUT/large.json'):
    if l.startswith('large'):
        d = json.loads(l.split(' ', 2)[2]); print('large d64 value', d.get('value'), 'step frac', d.get('step_bandwidth', {}).get('frac'), d.get('roofline', {}).get('avg_launch_us'))"
