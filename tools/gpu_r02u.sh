# final r02 profiles: default bench line, then rocprofv3 stats + PMC passes (tools/profile_bench.sh)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02u
mkdir -p $OUT
timeout -k 10 250 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
timeout -k 10 200 python3 bench.py --no-sharded --steps 20 --warmup 5 > $OUT/bench_20.json 2> $OUT/bench_20.err
bash tools/profile_bench.sh --no-sharded
