# large-batch lines only (A/B of k_tri_adv variants)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02i
mkdir -p $OUT
timeout -k 10 500 python3 bench.py --no-cpu-baseline --no-neumf --no-sharded --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; b=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
for k in ('roofline_large_batch','roofline_large_batch_d64'): print(k, b[k]['triplets_per_s'], b[k]['frac'], b[k]['per_kernel_avg_us'])"
