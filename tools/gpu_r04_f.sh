# r04: kernel stats of the configs[4] d = 64 line with the hash plan
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_f}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o lg -- python3 tools/large_line.py 64 > $OUT/prof.log 2>&1
python3 -c "
import csv,glob
f=glob.glob('$OUT/prof/**/*kernel_stats.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
for r in rows[:24]: print(r['Name'][:70], r['Calls'], r['AverageNs'], r['Percentage'])"
