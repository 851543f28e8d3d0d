set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG2:-r02af}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_config5.py tests/test_gpu_parity.py -m gpu > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert|Mismatch" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
OUT_TAG=${ABTAG:-ab3} VARIANTS="${VARIANTS:-cur v3 cur v3}" bash tools/gpu_ab_large.sh
cp tools/ab/${KEEP:-v3}.so adversarial-collaborative-filtering_amd/lib/libacf_apr.so
