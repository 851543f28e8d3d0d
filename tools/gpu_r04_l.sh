# r04: NeuMF catch-up workgroups; tri-combine small-slot waves 8192 (same box)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_l}
mkdir -p $OUT
n=0
for v in "ACF_NMF_CATCHUP_WG=128" "ACF_NMF_CATCHUP_WG=192" "ACF_NMF_CATCHUP_WG=96" "ACF_NMF_CATCHUP_WG=256" "ACF_NMF_CATCHUP_WG=128" "ACF_NMF_CATCHUP_WG=192"; do
  n=$((n+1))
  env $v timeout -k 10 200 python3 tools/neumf_rate.py > $OUT/n$n.log 2>&1
  echo "$v: $(tail -1 $OUT/n$n.log)"
done
n=0
for v in ACF_TRI_COMB_WAVES=4096 ACF_TRI_COMB_WAVES=8192 ACF_TRI_COMB_WAVES=4096 ACF_TRI_COMB_WAVES=8192; do
  n=$((n+1))
  env $v timeout -k 10 300 python3 tools/large_line.py 64 > $OUT/l$n.json 2> $OUT/l$n.err
  python3 -c "
import json; d=json.loads(open('$OUT/l$n.json').read().strip().splitlines()[-1])
print('$v', round(d['triplets_per_s']/1e6,1), {k: round(v,2) for k,v in (d['per_kernel_avg_us'] or {}).items()})"
done
