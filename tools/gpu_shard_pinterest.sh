# configs[2] split step at world 1: route vs replay times, then a kernel trace of it
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-sp}
mkdir -p $OUT
timeout -k 10 200 python3 tools/shard_pinterest.py > $OUT/times.json 2> $OUT/times.err || { tail -20 $OUT/times.err; exit 1; }
cat $OUT/times.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o pp -- python3 tools/shard_pinterest.py > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/kernel_stats.csv
rm -rf $OUT/prof
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$OUT/kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:30]:
    print(r["Calls"], round(float(r["AverageNs"])/1e3, 2), round(float(r["TotalDurationNs"])/1e6, 3), r["Name"][:90])
PY
ls -la $OUT
