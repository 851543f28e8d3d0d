set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06_route_g1; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_distributed.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for k in 1 2; do
timeout -k 10 300 python3 tools/shard_profile.py 24 > $OUT/new_$k.json 2> $OUT/new_$k.err || { tail -20 $OUT/new_$k.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/new_$k.json').read().strip().splitlines()[-1])
print('new round $k', {k: (v['ms_per_step'], v['step_errors']) for k, v in d.items()})"
done
