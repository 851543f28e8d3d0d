# closing pass, part 2: profiles (short-call trace, configs[4] d=64 step
# timeline, bench rocprofv3 stats + PMC passes)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-profiles}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/sc_trace -o sc -- python3 tools/short_call.py --reps 10 --same > $OUT/sc_trace.log 2>&1
python3 tools/trace_region.py $(find $OUT/sc_trace -name '*kernel_trace.csv' | head -1) > $OUT/short_call_trace_breakdown.json 2>&1 || true
echo "short call trace done"
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $OUT/lg_trace -o lg -- python3 tools/large_step_trace.py --d 64 > $OUT/lg_trace.log 2>&1
python3 tools/large_step_trace.py --analyze $(find $OUT/lg_trace -name '*kernel_trace.csv' | head -1) > $OUT/large_step_timeline_d64.json 2>&1 || true
echo "large trace done"
bash tools/profile_bench.sh > $OUT/profile_bench.log 2>&1
echo "profile_bench done"
