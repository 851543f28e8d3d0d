# round-3 closing pass: GPU suite + smoke, default and 20-step bench lines, then the
# rocprofv3 kernel stats and PMC traffic of the bench (summaries kept, raw traces dropped:
# gpurun copies back at most 64 MiB)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/closing_r03
mkdir -p $OUT
OUT_TAG=closing_r03 bash tools/gpu_closing_pass.sh
bash tools/profile_bench.sh --no-sharded
python3 tools/pmc_traffic.py gpurun_out/prof $OUT/pmc_traffic.json 647 > /dev/null
cp gpurun_out/prof/trace/bench_kernel_stats.csv $OUT/rocprof_kernel_stats_bench.csv
cp gpurun_out/prof/trace.json $OUT/bench_under_rocprof.json
rm -rf gpurun_out/prof
ls -la $OUT
