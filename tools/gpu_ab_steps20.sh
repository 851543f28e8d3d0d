# same-box A/B of libacf_apr.so builds on the driver's --steps 20 line (tools/bench_alt.py):
# VARIANTS = names of tools/libacf_apr_<name>.so ("base" = the package's library)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-ab20}; mkdir -p $OUT
for r in 1 2 3; do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then L=""; else L=$PWD/tools/libacf_apr_$v.so; fi
    ACF_LARGE_LINE_LIB=$L timeout -k 10 200 python3 tools/bench_alt.py --steps 20 --warmup 5 --no-sharded --no-neumf --no-eval --no-large --no-cpu-baseline > $OUT/b20_${v}_$r.json 2> $OUT/b20_${v}_$r.err || { echo "$v failed"; tail -5 $OUT/b20_${v}_$r.err; exit 1; }
    echo "$v round $r: $(python3 -c "import json;d=json.loads(open('$OUT/b20_${v}_$r.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done
