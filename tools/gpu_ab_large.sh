# same-box A/B of two builds of libacf_apr.so on the large-batch lines (tools/ab/base.so vs tools/ab/new.so)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-ab}
mkdir -p $OUT
LIB=adversarial-collaborative-filtering_amd/lib/libacf_apr.so
for v in ${VARIANTS:-base new base new}; do
  cp tools/ab/$v.so $LIB
  timeout -k 10 300 python3 bench.py --no-sharded --no-neumf --no-cpu-baseline --no-eval --steps 20 --warmup 5 > $OUT/b_$v.json 2> $OUT/b_$v.err
  python3 -c "
import json;d=json.loads(open('$OUT/b_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], *[(k[-3:], d[k]['avg_launch_us'], d[k]['frac'], d[k]['per_kernel_avg_us']['clean'], d[k]['per_kernel_avg_us']['hot'], round(d[k]['triplets_per_s']/1e6,1)) for k in ('roofline_large_batch','roofline_large_batch_d64')])"
done
