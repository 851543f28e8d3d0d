#!/bin/bash
# rocprofv3 passes over bench.py (run on the GPU box from the repo root):
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes
# (guide: they do not fit one pass; no trace domains with --pmc).
# Summaries are parsed by tools/pmc_traffic.py into profiles/.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="--no-cpu-baseline --steps 647 --warmup 647 --time-batches 100 $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o bench -- python3 bench.py $ARGS > $OUT/trace.json 2> $OUT/trace.err
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/fetch -o bench -- python3 bench.py $ARGS > $OUT/fetch.json 2> $OUT/fetch.err
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/write -o bench -- python3 bench.py $ARGS > $OUT/write.json 2> $OUT/write.err
find $OUT -name "*.csv" | head -20
