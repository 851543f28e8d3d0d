# k_tri_adv with two triplet groups per wave: large-batch parity tests, then the large lines
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r02ab}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_config5.py tests/test_gpu_parity.py -m gpu > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert|Mismatch" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for k in 1 2; do timeout -k 10 300 python3 bench.py --no-sharded --no-neumf --no-cpu-baseline --steps 20 --warmup 5 > $OUT/b_$k.json 2> $OUT/b_$k.err; python3 -c "
import json;d=json.loads(open('$OUT/b_$k.json').read().strip().splitlines()[-1])
for k in ('roofline_large_batch','roofline_large_batch_d64'): x=d[k]; print(k, x['avg_launch_us'], x['frac'], x['triplets_per_s'], x['per_kernel_avg_us'])"; done
