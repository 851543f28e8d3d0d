# r06: GPU tests of the B = 512 streamed path (owner positions), then a same-box
# A/B of the headline line: tools/libacf_apr_${AV:-head}.so against the package's build,
# REPS interleaved rounds of the driver's `--steps 20` call and one default-length
# run each (tools/bench_lib.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r06_ab_short}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python3 -u -m pytest -x -v --timeout 200 --timeout-method thread \
    ${TESTS:-tests} -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
ARGS="--no-sharded --no-neumf --no-large --no-cpu-baseline --no-eval"
for k in $(seq 1 ${REPS:-3}); do
  for v in ${AV:-head} base; do
    if [ "$v" = base ]; then L=""; else L=$PWD/tools/libacf_apr_$v.so; fi
    ACF_ALT_LIB=$L timeout -k 10 200 python3 tools/bench_lib.py $ARGS --steps 20 --warmup 5 > $OUT/s20_${v}_$k.json 2> $OUT/s20_${v}_$k.err || { tail -20 $OUT/s20_${v}_$k.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/s20_${v}_$k.json').read().strip().splitlines()[-1])
print('$v s20 round $k', round(d['value']/1e6,2), 'M  k_stream/batch', d['roofline']['per_kernel_avg_us'].get('stream_per_batch'), 'errs', d['step_errors'], d['stream_recoveries'])"
  done
done
for v in ${AV:-head} base; do
  if [ "$v" = base ]; then L=""; else L=$PWD/tools/libacf_apr_$v.so; fi
  ACF_ALT_LIB=$L timeout -k 10 300 python3 tools/bench_lib.py $ARGS > $OUT/long_${v}.json 2> $OUT/long_${v}.err || { tail -20 $OUT/long_${v}.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/long_${v}.json').read().strip().splitlines()[-1])
print('$v long', round(d['value']/1e6,2), 'M  k_stream/batch', d['roofline']['per_kernel_avg_us'].get('stream_per_batch'), 'errs', d['step_errors'], d['stream_recoveries'])"
done
