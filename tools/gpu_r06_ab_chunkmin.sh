# r06: split-step lines (world 1) with chunk plans for every local batch size
# (--chunk-min 0: configs[2]'s 512-triplet local batches on the hash plan too)
# against the default (chunk plans above 1,024 triplets), two interleaved rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r06_ab_chunkmin}; mkdir -p $OUT
for k in 1 2; do
  for v in c0 base; do
    F=""; [ "$v" = c0 ] && F="--chunk-min 0"
    timeout -k 10 300 python3 tools/shard_profile.py 24 $F > $OUT/${v}_$k.json 2> $OUT/${v}_$k.err || { tail -20 $OUT/${v}_$k.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/${v}_$k.json').read().strip().splitlines()[-1])
print('$v round $k', {k: (v['ms_per_step'], v['step_errors']) for k, v in d.items()})"
  done
done
