# r06 check: the targeted GPU tests of a change, then the unaided `bench.py --gpus 2`
# rehearsal (bench.py starts torchrun itself; every rank on cuda:0 over gloo), then
# the driver's own bench command.  TESTS: the test files to run (default: all -m gpu).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r06_check}
mkdir -p $OUT
timeout -k 10 ${TEST_TIMEOUT:-600} python3 -u -m pytest -x -v --timeout 200 --timeout-method thread ${TESTS:-tests} -m gpu \
  > $OUT/pytest.log 2>&1
tail -3 $OUT/pytest.log
if [ -z "$NO_REHEARSE" ]; then
  timeout -k 10 400 python3 bench.py --gpus 2 --rehearse-one-gpu --no-large --no-neumf --no-eval --steps 20 --warmup 5 \
    --sharded-steps 4 > $OUT/bench_gpus2_unaided.json 2> $OUT/bench_gpus2_unaided.err
  python3 -c "
import json;d=json.loads(open('$OUT/bench_gpus2_unaided.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'world', d['world'], 'value', d['value'], 'step_errors', d['step_errors'])
for k, v in d.get('sharded', {}).items(): print(k, v.get('n_gpus'), v.get('value'), v.get('config', {}).get('parallelism'))"
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_steps20.json 2> $OUT/bench_steps20.err
  python3 -c "
import json;d=json.loads(open('$OUT/bench_steps20.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'], 'cpu', d.get('cpu_baseline', {}).get('value'))
for k in ('roofline_large_batch', 'roofline_large_batch_d64'): print(k, d[k].get('triplets_per_s'), d[k].get('frac'))
print('sharded', {k: v.get('ms_per_step') for k, v in d['sharded'].items()}); print('neumf', d['neumf']['value'])"
fi
