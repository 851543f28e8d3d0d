# NeuMF epoch rate A/B (configs[3]): the lazy-Adam catch-up period and workgroups,
# interleaved so box drift hits every variant alike.  VARIANTS: "LAZY_S,WG" pairs.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-neumf_ab}
mkdir -p $OUT
for r in 1 2; do
  for v in ${VARIANTS:-16,192 31,192 31,96 24,128}; do
    s=${v%,*}; w=${v#*,}
    ACF_NMF_LAZY_S=$s ACF_NMF_CATCHUP_WG=$w timeout -k 10 200 python3 tools/neumf_rate.py > $OUT/nmf_${s}_${w}_$r.log 2>&1 || { echo "neumf $v failed"; tail -5 $OUT/nmf_${s}_${w}_$r.log; exit 1; }
    echo "lazy_s=$s wg=$w rep $r: $(grep 'rep 1' $OUT/nmf_${s}_${w}_$r.log)"
  done
done
