# r04: tri-combine layout (hot chain first) parity + A/B of its slot-wave count
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r04_h}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_config5.py -m gpu -k "hash_plan or fused or hot_slots or config5" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
n=0
for v in ${VARIANTS:-"ACF_TRI_COMB_WAVES=4096" "ACF_TRI_COMB_WAVES=512" "ACF_TRI_COMB_WAVES=1024" "ACF_TRI_COMB_WAVES=4096" "ACF_TRI_COMB_WAVES=512"}; do
  n=$((n+1))
  env $v timeout -k 10 300 python3 tools/large_line.py 64 > $OUT/l$n.json 2> $OUT/l$n.err
  python3 -c "
import json; d=json.loads(open('$OUT/l$n.json').read().strip().splitlines()[-1])
print('$v', round(d['triplets_per_s']/1e6,1), d['step_frac'], d['avg_launch_us'], {k: round(v,2) for k,v in (d['per_kernel_avg_us'] or {}).items()}, d['step_errors'])"
done
