# hot fan-in: parity file (hot/large/fused), then large lines
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02l
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_keras_bpr.py > $OUT/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert|Mismatch|Max" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 500 python3 bench.py --no-cpu-baseline --no-neumf --no-sharded --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; b=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
for k in ('roofline_large_batch','roofline_large_batch_d64'): print(k, b[k]['triplets_per_s'], b[k]['frac'], b[k]['per_kernel_avg_us'])"
