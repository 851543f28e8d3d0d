# r04: the hash plan (k_hplan_*) and the counting-sort batch plan: parity first,
# then same-box A/Bs (configs[4] d = 64 line; the driver-shaped short call)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_e}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "hash_plan or fused or hot_slots" > $OUT/pytest_hash.log 2>&1 || { tail -40 $OUT/pytest_hash.log; exit 1; }
echo "hash tests: $(tail -1 $OUT/pytest_hash.log)"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_config5.py tests/test_gpu_plan.py -m gpu > $OUT/pytest_plan.log 2>&1 || { tail -40 $OUT/pytest_plan.log; exit 1; }
echo "config5 + plan tests: $(tail -1 $OUT/pytest_plan.log)"
n=0
for v in "ACF_HASH_PLAN=0" "ACF_HASH_PLAN=1" "ACF_HASH_PLAN=0" "ACF_HASH_PLAN=1"; do
  n=$((n+1))
  env $v timeout -k 10 300 python3 tools/large_line.py 64 > $OUT/l$n.json 2> $OUT/l$n.err
  python3 -c "
import json; d=json.loads(open('$OUT/l$n.json').read().strip().splitlines()[-1])
print('$v', round(d['triplets_per_s']/1e6,1), d['step_frac'], d['avg_launch_us'], d['step_errors'])"
done
for v in radix count radix count; do
  ACF_BPLAN_SORT=$v timeout -k 10 200 python3 tools/short_call.py --reps 40 --same > $OUT/sc_sort$v.json 2> $OUT/sc_sort$v.err
  python3 -c "
import json,statistics as st
d=json.loads(open('$OUT/sc_sort$v.json').read().strip().splitlines()[-1]); r=[x['region_us'] for x in d['reps']][5:]
print('sort $v region median', st.median(r), 'min', min(r))"
done
