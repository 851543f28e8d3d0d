# kernel stats (rocprofv3) of the configs[4] d = 64 line; env passes through
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-prof_large}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o lg -- python3 tools/large_line.py 64 > $OUT/prof.log 2>&1
grep triplets_per_s $OUT/prof.log | cut -c1-120
python3 -c "
import csv,glob
f=glob.glob('$OUT/prof/**/*kernel_stats.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
for r in rows[:26]: print(r['Name'][:70], r['Calls'], r['AverageNs'], r['Percentage'])"
