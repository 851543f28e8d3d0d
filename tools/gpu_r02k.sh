# flakiness check of the k_ovl plan-equivalence case
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02k
mkdir -p $OUT
for r in 1 2 3; do
timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_plan.py -k "test_batch_plan_matches_sort_plan and sparse" > $OUT/run$r.log 2>&1 || true
tail -2 $OUT/run$r.log
done
