# r06: rocprofv3 kernel stats of the split-step lines alone (world 1) and of the
# configs[4] d = 64 line, reduced on the box to the top kernels
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r06_shard_prof}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/sp -o sp -- python3 tools/shard_profile.py > $OUT/sp.log 2>&1
tail -c 1500 $OUT/sp.log
python3 -c "
import csv,glob
f=glob.glob('$OUT/sp/**/*kernel_stats.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
for r in rows[:40]: print(r['Name'][:90], r['Calls'], r['AverageNs'], r['Percentage'])" > $OUT/sp_top.txt
cp $(find $OUT/sp -name '*kernel_stats.csv' | head -1) $OUT/sp_kernel_stats.csv
rm -rf $OUT/sp
cat $OUT/sp_top.txt
