set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sc
timeout -k 10 200 python3 tools/short_call.py > gpurun_out/sc/plain.json 2> gpurun_out/sc/plain.err
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/sc/trace -o sc -- python3 tools/short_call.py > gpurun_out/sc/traced.json 2> gpurun_out/sc/traced.err
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-neumf > gpurun_out/sc/bench20.json 2> gpurun_out/sc/bench20.err
