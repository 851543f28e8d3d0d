# hot-slot split: parity file + default bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02b
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -v -x --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "hot or large or single_step or fused" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 500 python3 bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
python3 -c "
import json; b=json.load(open('$OUT/bench.json'))
for k in ('roofline_large_batch','roofline_large_batch_d64'):
    r=b[k]; print(k, r['triplets_per_s'], r['frac'], r['per_kernel_avg_us'])
print('default', b['value'])"
