# same-box A/B of two builds of libacf_apr.so on the driver-shaped 20-batch call
# (tools/ab/base.so vs tools/ab/new.so): parity file with new.so first, then
# tools/short_call.py (region / enqueue medians) and the 20-step bench line per variant
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-ab_short}
mkdir -p $OUT
LIB=adversarial-collaborative-filtering_amd/lib/libacf_apr.so
cp tools/ab/new.so $LIB
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_plan.py -m gpu > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
for v in ${VARIANTS:-base new base new}; do
  cp tools/ab/$v.so $LIB
  timeout -k 10 200 python3 tools/short_call.py --reps 30 > $OUT/sc_$v.json 2> $OUT/sc_$v.err
  timeout -k 10 200 python3 bench.py --no-sharded --no-neumf --no-large --no-cpu-baseline --steps 20 --warmup 5 > $OUT/b20_$v.json 2> $OUT/b20_$v.err
  python3 -c "
import json,statistics as st
d=json.loads(open('$OUT/sc_$v.json').read().strip().splitlines()[-1]); r=[x['region_us'] for x in d['reps']]
b=json.loads(open('$OUT/b20_$v.json').read().strip().splitlines()[-1])
print('$v region median', st.median(r), 'min', min(r), 'bench20', b['value'])"
done
cp tools/ab/new.so $LIB
