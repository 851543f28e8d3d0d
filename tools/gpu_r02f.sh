# Keras BPR tests, distributed tests, the full bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02f
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_keras_bpr.py tests/test_gpu_distributed.py > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; }
tail -3 $OUT/pytest.log
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; b=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('default', b['value'], b['roofline']['frac'])
for k in ('roofline_large_batch','roofline_large_batch_d64'): print(k, b[k]['triplets_per_s'], b[k]['frac'])
for k,v in b['sharded'].items(): print('sharded', k, v['value'], v['ms_per_step'], v.get('route_ms_rank0'))
print('cpu', b['cpu_baseline']['value'], 'neumf', b['neumf']['value'])"
timeout -k 10 200 python3 tools/short_call.py > $OUT/sc_plain.json 2> $OUT/sc_plain.err
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/sc_trace -o sc -- python3 tools/short_call.py > $OUT/sc_traced.json 2> $OUT/sc_traced.err
cat $OUT/sc_plain.json
