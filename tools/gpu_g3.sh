set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g3
timeout -k 10 200 python3 tools/short_call.py > gpurun_out/g3/plain.json 2> gpurun_out/g3/plain.err
timeout -k 10 300 python3 tools/parity_diag.py 32 > gpurun_out/g3/diag.json 2> gpurun_out/g3/diag.err
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_plan.py > gpurun_out/g3/plan.log 2>&1 || true
