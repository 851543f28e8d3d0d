# r06: a change to the large-batch step against tools/libacf_apr_$VAR.so (the
# same sources built with the change switched off): the large-batch GPU tests,
# a bit-compare of the two builds on one Zipf case (tools/bitcmp_lib.py), then
# the configs[4] A/B (tools/gpu_ab_large.sh, two interleaved rounds).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r06_variant}; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread \
  ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_config5.py tests/test_gpu_plan.py} -m gpu -k "${TESTK:-large or hot or config5 or fused or hash}" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python3 tools/bitcmp_lib.py 64 128 > $OUT/bitcmp_package.json 2> $OUT/bitcmp_package.err || { tail -20 $OUT/bitcmp_package.err; exit 1; }
ACF_ALT_LIB=$PWD/tools/libacf_apr_$VAR.so timeout -k 10 300 python3 tools/bitcmp_lib.py 64 128 > $OUT/bitcmp_$VAR.json 2> $OUT/bitcmp_$VAR.err || { tail -20 $OUT/bitcmp_$VAR.err; exit 1; }
cat $OUT/bitcmp_package.json $OUT/bitcmp_$VAR.json
OUT_TAG=${OUT_TAG:-r06_variant} VARIANTS="$VAR base" LINES="${LINES:-64 128}" bash tools/gpu_ab_large.sh
