set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g4
timeout -k 10 400 python3 -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_plan.py tests/test_gpu_e2e_video.py tests/test_gpu_parity.py -k "headline or single_step or video" > gpurun_out/g4/pytest.log 2>&1 || true
