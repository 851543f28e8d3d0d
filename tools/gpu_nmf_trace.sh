# NeuMF step kernel breakdown (rocprofv3 kernel trace of tools/neumf_only.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-nmf_trace}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o nmf -- python3 tools/neumf_only.py > $OUT/run.log 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:48].ljust(48), r["Calls"].rjust(6), "%9.2f us" % (float(r["AverageNs"]) / 1e3), r["Percentage"][:5])
PY
