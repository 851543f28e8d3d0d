# r04: eval (auto/MFMA/VALU), the 20-step bench line x3, short_call --same, NeuMF period A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_b}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_reference.py tests/test_gpu_torch_ops.py -m gpu -k "eval or rank or reference or stream or give_up or pipeline or unverified" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
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
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-sharded --no-neumf --no-large --no-cpu-baseline --no-eval --steps 20 --warmup 5 > $OUT/b20_$r.json 2> $OUT/b20_$r.err
  python3 -c "import json; b=json.loads(open('$OUT/b20_$r.json').read().strip().splitlines()[-1]); print('bench20', b['value'], b['ms_per_step'], b['step_errors'], b['stream_recoveries'])"
done
timeout -k 10 200 python3 tools/short_call.py --reps 30 --same > $OUT/sc.json 2> $OUT/sc.err
python3 -c "
import json,statistics as st
d=json.loads(open('$OUT/sc.json').read().strip().splitlines()[-1]); r=[x['region_us'] for x in d['reps']]; e=[x['enqueue_us'] for x in d['reps']]
print('short_call --same region median', st.median(r), 'min', min(r), 'enqueue', st.median(e), 'first', r[:5])"
for v in "16 96" "24 96" "31 96" "16 128" "24 128"; do
  set -- $v
  ACF_NMF_LAZY_S=$1 ACF_NMF_CATCHUP_WG=$2 timeout -k 10 200 python3 tools/neumf_rate.py > $OUT/nmf_$1_$2.log 2>&1
  echo "nmf lazy_s $1 wg $2: $(tail -1 $OUT/nmf_$1_$2.log)"
done
