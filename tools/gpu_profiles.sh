# closing pass, part 2: profiles -- bench rocprofv3 kernel stats + FETCH_SIZE /
# WRITE_SIZE passes (tools/profile_bench.sh) reduced on the box to
# pmc_traffic.json + the stats csv, the configs[4] d = 64 step timeline and the
# short-call trace breakdown; the raw traces are deleted (gpurun copies back <= 64 MiB)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-profiles}
mkdir -p $OUT
bash tools/profile_bench.sh > $OUT/profile_bench.log 2>&1
python3 tools/pmc_traffic.py gpurun_out/prof $OUT/pmc_traffic.json
cp $(find gpurun_out/prof/trace -name '*kernel_stats.csv' | head -1) $OUT/rocprof_kernel_stats_bench.csv
cp gpurun_out/prof/trace.json $OUT/bench_under_rocprof.json
rm -rf gpurun_out/prof
echo "profile_bench done"
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $OUT/lg_trace -o lg -- python3 tools/large_step_trace.py --d 64 > $OUT/lg_trace.log 2>&1
python3 tools/large_step_trace.py --analyze $(find $OUT/lg_trace -name '*kernel_trace.csv' | head -1) > $OUT/large_step_timeline_d64.json 2>&1 || true
rm -rf $OUT/lg_trace
echo "large trace done"
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/sc_trace -o sc -- python3 tools/short_call.py --reps 10 --same > $OUT/sc_trace.log 2>&1
python3 tools/trace_region.py $(find $OUT/sc_trace -name '*kernel_trace.csv' | head -1) > $OUT/short_call_trace_breakdown.json 2>&1 || true
rm -rf $OUT/sc_trace
echo "short call trace done"
