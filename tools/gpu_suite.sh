set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/suite
timeout -k 10 900 python3 -u -m pytest -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/suite/pytest.log 2>&1 || true
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite/smoke.log 2>&1
