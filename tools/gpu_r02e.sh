# rocprof of the split-step lines (world 1)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02e
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o shard -- python3 tools/shard_profile.py 24 > $OUT/out.json 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
tail -2 $OUT/out.json
find $OUT -name "*.csv"
