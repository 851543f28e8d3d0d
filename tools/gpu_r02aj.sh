set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02aj
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/t64 -o lt -- python3 tools/large_step_trace.py --d 64 > $OUT/run64.log 2>&1
f=$(find $OUT/t64 -name "*kernel_trace.csv" | head -1)
python3 tools/large_step_trace.py --analyze $f --batches 128 > $OUT/analysis64.json
cat $OUT/analysis64.json
