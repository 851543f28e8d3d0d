set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g2
for v in 0 1 2 3 4; do
  ACF_BPLAN_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/g2/trace$v -o sc -- python3 tools/short_call.py > gpurun_out/g2/sc$v.json 2> gpurun_out/g2/sc$v.err
done
timeout -k 10 200 python3 tools/short_call.py > gpurun_out/g2/plain.json 2> gpurun_out/g2/plain.err
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_plan.py -k "ml1m or replan or concurrent or range" > gpurun_out/g2/plan.log 2>&1 || true
