set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g1
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_plan.py > gpurun_out/g1/plan.log 2>&1 || true
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g1/smoke.log 2>&1
timeout -k 10 200 python3 tools/short_call.py > gpurun_out/g1/sc.json 2> gpurun_out/g1/sc.err
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/g1/trace -o sc -- python3 tools/short_call.py > gpurun_out/g1/sc_traced.json 2> gpurun_out/g1/sc_traced.err
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-neumf > gpurun_out/g1/bench20.json 2> gpurun_out/g1/bench20.err
