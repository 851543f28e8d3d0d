"""configs[4] line(s) alone (bench.large_batch_roofline) for same-box A/B runs:
python3 tools/large_line.py [d[:noovl] ...] -> one JSON line per entry
(":noovl": the overlapped step off -- the fused triplets in the adversarial pass
instead of beside the combines, acf_apr_set_step_overlap 0)."""
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
for arg in sys.argv[1:] or ["64"]:
    d = int(arg.split(":")[0])
    ovl = not arg.endswith(":noovl")
    r = bench.large_batch_roofline(acf, ops, dev, big, d, step_overlap=ovl)
    print(json.dumps({"d": d, "step_overlap": ovl, "triplets_per_s": r["triplets_per_s"], "step_frac": r["step_bandwidth"]["frac"],
                      "avg_launch_us": r.get("avg_launch_us"), "per_kernel_avg_us": r.get("per_kernel_avg_us"),
                      "step_errors": r["step_errors"]}), flush=True)
