# r04: hash plan parity, configs[4] A/B, kernel stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_g}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "hash_plan or fused or hot_slots" > $OUT/pytest_hash.log 2>&1 || { tail -40 $OUT/pytest_hash.log; exit 1; }
tail -1 $OUT/pytest_hash.log
n=0
for v in "ACF_HASH_PLAN=0" "ACF_HASH_PLAN=1"; do
  n=$((n+1))
  env $v timeout -k 10 300 python3 tools/large_line.py 64 > $OUT/l$n.json 2> $OUT/l$n.err
  python3 -c "
import json; d=json.loads(open('$OUT/l$n.json').read().strip().splitlines()[-1])
print('$v', round(d['triplets_per_s']/1e6,1), d['step_frac'], d['avg_launch_us'], d['step_errors'])"
done
OUT_TAG=r04_g/prof bash tools/gpu_prof_large.sh 2>&1 | grep -E "hplan|triplets|tri_|rocprim|fill" | cut -c1-150
