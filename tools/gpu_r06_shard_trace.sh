# r06: kernel timeline of the configs[4] split step at world 1 (tools/shard_trace.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r06_shard_trace}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $OUT/tr -o st -- python3 tools/shard_trace.py > $OUT/tr.log 2>&1
python3 tools/shard_trace.py --analyze $(find $OUT/tr -name '*kernel_trace.csv' | head -1) > $OUT/shard_step_timeline.json
rm -rf $OUT/tr
head -c 3000 $OUT/shard_step_timeline.json
