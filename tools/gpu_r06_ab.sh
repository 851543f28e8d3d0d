# r06: the GPU tests of the large-batch (hash plan, triplet-centric) path, then a
# same-box A/B of the configs[4] lines: tools/libacf_apr_head.so (the build before
# the change) against the package's build, two interleaved rounds.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r06_ab}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python3 -u -m pytest -x -v --timeout 200 --timeout-method thread \
    ${TESTS:-tests/test_gpu_plan.py tests/test_gpu_config5.py tests/test_gpu_parity.py} -m gpu ${TESTK:+-k "$TESTK"} \
    > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
OUT_TAG=${OUT_TAG:-r06_ab} VARIANTS="${VARIANTS:-head base}" LINES="${LINES:-64 128}" bash tools/gpu_ab_large.sh
