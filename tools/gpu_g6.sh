set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g6
timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_sampler.py > gpurun_out/g6/pytest.log 2>&1 || true
timeout -k 10 500 python3 bench.py > gpurun_out/g6/bench.json 2> gpurun_out/g6/bench.err
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/g6/bench20.json 2> gpurun_out/g6/bench20.err
