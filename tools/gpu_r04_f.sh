# r04: the hash plan: parity, then the configs[4] d = 64 A/B and kernel stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_f}
mkdir -p $OUT
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "hash_plan or fused or hot_slots" > $OUT/pytest_hash.log 2>&1 || { tail -40 $OUT/pytest_hash.log; exit 1; }
echo "hash tests: $(tail -1 $OUT/pytest_hash.log)"
n=0
for v in ${VARIANTS:-"ACF_HASH_PLAN=0" "ACF_HASH_PLAN=1"}; do
  n=$((n+1))
  env $v timeout -k 10 300 python3 tools/large_line.py 64 > $OUT/l$n.json 2> $OUT/l$n.err
  python3 -c "
import json; d=json.loads(open('$OUT/l$n.json').read().strip().splitlines()[-1])
print('$v', round(d['triplets_per_s']/1e6,1), d['step_frac'], d['avg_launch_us'], d['step_errors'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o lg -- python3 tools/large_line.py 64 > $OUT/prof.log 2>&1
python3 -c "
import csv,glob
f=glob.glob('$OUT/prof/**/*kernel_stats.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
for r in rows[:24]: print(r['Name'][:70], r['Calls'], r['AverageNs'], r['Percentage'])"
