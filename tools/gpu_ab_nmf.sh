# r05 same-box A/B of libacf_neumf.so builds on the NeuMF rate (tools/neumf_rate.py):
# VARIANTS = names of tools/libacf_neumf_<name>.so ("base" = the package's library)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-abn}; mkdir -p $OUT
for r in 1 2; do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then L=""; else L=$PWD/tools/libacf_neumf_$v.so; fi
    ACF_NEUMF_LIB=$L timeout -k 10 200 python3 tools/neumf_rate.py > $OUT/nmf_${v}_$r.log 2>&1 || { echo "neumf $v failed"; tail -5 $OUT/nmf_${v}_$r.log; exit 1; }
    echo "$v round $r: $(grep 'rep 1' $OUT/nmf_${v}_$r.log)"
  done
done
