# r06: instruction-fetch and wait counters of the short call's kernels (batch plan,
# k_stream): one --pmc pass over tools/short_call.py
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06_plan_pmc; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES -f csv -d $OUT/pmc -o pmc -- python3 tools/short_call.py --reps 3 > $OUT/pmc.log 2>&1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r06_plan_pmc/pmc/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:40]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    if "bplan" in k or "k_stream" in k:
        w = d.get("SQ_WAVE_CYCLES", 0) or 1
        print(k, {c: round(v) for c, v in d.items()}, "inst_wait_frac", round(d.get("SQ_WAIT_INST_ANY", 0) / w, 3), "any_wait_frac", round(d.get("SQ_WAIT_ANY", 0) / w, 3))
PY
