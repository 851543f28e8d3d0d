# r04: NeuMF lazy-Adam knobs A/B (catch-up period, catch-up workgroups), same box
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_j}
mkdir -p $OUT
n=0
for v in "ACF_NMF_LAZY_S=16" "ACF_NMF_LAZY_S=24" "ACF_NMF_LAZY_S=31" "ACF_NMF_LAZY_S=24 ACF_NMF_CATCHUP_WG=64" "ACF_NMF_LAZY_S=16" "ACF_NMF_LAZY_S=24"; do
  n=$((n+1))
  env $v timeout -k 10 200 python3 tools/neumf_rate.py > $OUT/n$n.log 2>&1
  echo "$v: $(tail -1 $OUT/n$n.log)"
done
