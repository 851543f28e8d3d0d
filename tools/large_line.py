"""configs[4] line(s) alone (bench.large_batch_roofline) for same-box A/B runs:
python3 tools/large_line.py [d ...] -> one JSON line per d."""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

acf = importlib.import_module(bench.PKG)
ops = importlib.import_module(bench.PKG + ".ops")
dev = torch.device("cuda", 0)
big = acf.synthetic_large(device=dev)
for d in [int(x) for x in sys.argv[1:]] or [64]:
    r = bench.large_batch_roofline(acf, ops, dev, big, d)
    print(json.dumps({"d": d, "triplets_per_s": r["triplets_per_s"], "step_frac": r["step_bandwidth"]["frac"],
                      "avg_launch_us": r.get("avg_launch_us"), "per_kernel_avg_us": r.get("per_kernel_avg_us"),
                      "step_errors": r["step_errors"], "env": {k: v for k, v in os.environ.items()
                                                              if k.startswith("ACF_")}}), flush=True)
