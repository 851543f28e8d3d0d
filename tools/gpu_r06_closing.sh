# r06 closing pass, part 1: GPU suite + smoke, the default bench and the driver's
# --steps 20 bench line (results under gpurun_out/r06_closing)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-r06_closing}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || { echo "suite failed"; grep -E "FAILED|Error" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_steps20.json 2> $OUT/bench_steps20.err
python3 - <<'PY'
import json
for f in ("bench_default.json", "bench_steps20.json"):
    d = json.loads(open(f"gpurun_out/r06_closing/{f}").read().strip().splitlines()[-1])
    print(f, "value", round(d["value"] / 1e6, 2), "M frac", d["roofline"]["frac"], "cpu", d.get("cpu_baseline", {}).get("value"))
    for k in ("roofline_large_batch", "roofline_large_batch_d64"):
        print(" ", k, d[k].get("triplets_per_s_passes"), d[k].get("kernel"), d[k].get("frac"), d[k]["step_bandwidth"]["frac"])
    print("  sharded", {k: v.get("ms_per_step") for k, v in d["sharded"].items()}, "neumf", d["neumf"]["value"],
          d["neumf"]["roofline"]["avg_launch_us"], "eval", d["eval_all_items"]["ml-1m"]["ms_per_eval"])
PY
