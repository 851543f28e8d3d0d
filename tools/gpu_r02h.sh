# rocprof of the large-batch lines (triplet-centric step)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02h
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o large -- python3 bench.py --no-cpu-baseline --no-neumf --no-sharded --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
find $OUT -name "*stats.csv"
