# split step with captured hipGraphs: GPU distributed tests, then the split-step bench lines
# (world 1).  A test failure still runs the lines; a fault,
# abort or time limit stops the script.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-shard_graph}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_distributed.py > $OUT/dist.log 2>&1
rc=$?
tail -3 $OUT/dist.log
[ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
timeout -k 10 300 python3 tools/shard_profile.py ${STEPS:-24} > $OUT/shard.json 2> $OUT/shard.err || { echo "shard lines failed"; tail -20 $OUT/shard.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/shard.json').read().strip().splitlines()[-1]);[print(k, v['ms_per_step'], v['value'], v.get('launch')) for k, v in d.items()]"
if [ -n "$WITH_PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o shard -- python3 tools/shard_profile.py ${STEPS:-24} > $OUT/shard_prof.json 2> $OUT/shard_prof.err || exit 1
fi
