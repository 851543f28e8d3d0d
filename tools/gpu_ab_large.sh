# Same-box A/B of the large-batch (configs[4]) lines over libacf_apr.so builds:
# VARIANTS = names of tools/libacf_apr_<name>.so (an older commit's, tools/build_at.sh,
# or a -D variant); "base" = the package's library.  Two interleaved rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-ab_large}; mkdir -p $OUT
for k in 1 2; do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then L=""; else L=$PWD/tools/libacf_apr_$v.so; fi
    ACF_LARGE_LINE_LIB=$L timeout -k 10 300 python3 tools/large_line.py ${LINES:-64} > $OUT/${v}_$k.json 2> $OUT/${v}_$k.err || { tail -20 $OUT/${v}_$k.err; exit 1; }
    echo "$v round $k: $(cut -c1-160 $OUT/${v}_$k.json)"
  done
done
