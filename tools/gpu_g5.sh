set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g5
timeout -k 10 400 python3 -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_torch_ops.py tests/test_gpu_parity.py -k "torch or random or apr_step or segment or decomposed or score_rank or apr_train or out_of_range" > gpurun_out/g5/pytest.log 2>&1 || true
