# Same-box A/B of the large-batch (configs[4]) lines: this build against an older
# commit's library (tools/build_at.sh <rev> first; OLD=rev), interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-ab_large}; mkdir -p $OUT
OLD=${OLD:-82557ee}
for k in 1 2; do
  timeout -k 10 300 python3 tools/large_line.py ${LINES:-64 128} > $OUT/new$k.json 2> $OUT/new$k.err || { tail -20 $OUT/new$k.err; exit 1; }
  ACF_LARGE_LINE_LIB=$PWD/tools/libacf_apr_$OLD.so timeout -k 10 300 python3 tools/large_line.py ${LINES:-64 128} > $OUT/old$k.json 2> $OUT/old$k.err || { tail -20 $OUT/old$k.err; exit 1; }
done
cut -c1-300 $OUT/new1.json $OUT/old1.json $OUT/new2.json $OUT/old2.json
