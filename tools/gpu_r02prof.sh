# r02 profiles: full GPU suite + smoke, then rocprofv3 passes over the bench (tools/profile_bench.sh)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02p
timeout -k 10 900 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r02p/pytest.log 2>&1 || { echo "suite failed"; grep -E "FAILED|Error" gpurun_out/r02p/pytest.log | head -30; tail -5 gpurun_out/r02p/pytest.log; exit 1; }
tail -2 gpurun_out/r02p/pytest.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02p/smoke.log 2>&1 && tail -1 gpurun_out/r02p/smoke.log
bash tools/profile_bench.sh --no-sharded
