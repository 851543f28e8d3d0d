# triplet-centric list step: parity file, then the large lines of the bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02g
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -v -x --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_plan.py tests/test_gpu_torch_ops.py > $OUT/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert|Mismatch|Max" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 500 python3 bench.py --no-cpu-baseline --no-neumf --no-sharded --steps 200 --warmup 100 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; b=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('default', b['value'])
for k in ('roofline_large_batch','roofline_large_batch_d64'): print(k, b[k]['triplets_per_s'], b[k]['frac'], b[k]['per_kernel_avg_us'])"
