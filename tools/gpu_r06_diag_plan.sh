# r06: phase stamps of the B = 512 batch plan (k_bplan_sort + k_bplan_build) from
# the -DACF_DIAG build (tools/build_diag.sh, tools/diag_plan.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r06_diag_plan}; mkdir -p $OUT
timeout -k 10 200 python3 tools/diag_plan.py --lib tools/libacf_apr_diag.so > $OUT/plan.json 2> $OUT/plan.err || { tail -20 $OUT/plan.err; exit 1; }
cat $OUT/plan.json
