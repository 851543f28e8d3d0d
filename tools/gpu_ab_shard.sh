# Same-box A/B of the split-step lines (tools/shard_profile.py) over libacf_apr.so
# builds: VARIANTS = names of tools/libacf_apr_<name>.so, "base" = the package's.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-ab_shard}; mkdir -p $OUT
for k in 1 2; do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then L=""; else L=$PWD/tools/libacf_apr_$v.so; fi
    ACF_LARGE_LINE_LIB=$L timeout -k 10 300 python3 tools/shard_profile.py ${STEPS:-24} > $OUT/${v}_$k.json 2> $OUT/${v}_$k.err || { tail -20 $OUT/${v}_$k.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/${v}_$k.json').read().strip().splitlines()[-1]);print('$v round $k', {x:v['ms_per_step'] for x,v in d.items()})"
  done
done
