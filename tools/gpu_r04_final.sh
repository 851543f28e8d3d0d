# r04 closing pass, part 1: the GPU suite + smoke, the driver's default bench
# line and its --steps 20 form (outputs under gpurun_out/r04_final/)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_final}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo smoke ok
timeout -k 10 900 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
python3 -c "
import json; b=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1])
print('default', b['value'], b['ms_per_step'], b['roofline']['frac'], b.get('step_errors'))
for k in ('roofline_large_batch','roofline_large_batch_d64'):
    v=b.get(k) or {}; print(k, v.get('triplets_per_s'), (v.get('step_bandwidth') or {}).get('frac'), v.get('frac'))
print('neumf', (b.get('neumf') or {}).get('value')); print('eval', {k: v.get('ms_per_eval') for k, v in (b.get('eval_all_items') or {}).items()})
print('cpu', b.get('cpu_baseline', {}).get('value'))"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_steps20.json 2> $OUT/bench_steps20.err
python3 -c "
import json; b=json.loads(open('$OUT/bench_steps20.json').read().strip().splitlines()[-1])
print('steps20', b['value'], b['ms_per_step'])"
