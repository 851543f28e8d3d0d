#!/bin/bash
# rocprofv3 passes over bench.py (run on the GPU box from the repo root):
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes
# (guide: they do not fit one pass; no trace domains with --pmc), then the same
# two counters over tools/calib_fetch.py (known byte counts per access width).
# Every k_stream launch of these runs covers 647 batches (graph chunk = timing
# pass), so per-launch counters divide evenly into per-batch figures.
# Summaries are parsed by tools/pmc_traffic.py into profiles/.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="--no-cpu-baseline --steps 647 --warmup 647 --time-batches 647 $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o bench -- python3 bench.py $ARGS > $OUT/trace.json 2> $OUT/trace.err
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/fetch -o bench -- python3 bench.py $ARGS > $OUT/fetch.json 2> $OUT/fetch.err
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/write -o bench -- python3 bench.py $ARGS > $OUT/write.json 2> $OUT/write.err
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/calib_fetch -o calib -- python3 tools/calib_fetch.py > $OUT/calib_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/calib_write -o calib -- python3 tools/calib_fetch.py > $OUT/calib_write.log 2>&1
find $OUT -name "*.csv"
