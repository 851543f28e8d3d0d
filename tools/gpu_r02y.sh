set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02y
mkdir -p $OUT
timeout -k 10 200 python3 tools/diag_plan.py > $OUT/diag_plan.json 2> $OUT/diag_plan.err || { tail -20 $OUT/diag_plan.err; exit 1; }
cat $OUT/diag_plan.json
