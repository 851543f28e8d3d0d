"""Per-launch HBM traffic of the step kernels from rocprofv3 PMC passes
(tools/profile_bench.sh), corrected as MI355X_MICROARCH.md §HBM prescribes:
FETCH_SIZE reports half the bytes of 16-B-per-lane coalesced reads on gfx950
(doubled here; the step kernels read rows as float4 per lane); WRITE_SIZE is
exact for 16-B-per-lane stores.  Both are in KiB per dispatch.

Usage: python tools/pmc_traffic.py gpurun_out/prof profiles/r01/pmc_traffic.json
Writes {kernel name: {launches, fetch_kib_median, write_kib_median,
traffic_bytes_per_launch, trace_avg_us}} for the step kernels."""
import csv
import json
import statistics
import sys
from collections import defaultdict


def counters(path, name):
    vals = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == name:
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def trace_avg(path):
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            out[row["Name"]] = (int(row["Calls"]), float(row["AverageNs"]) / 1e3)
    return out


def main(src, dst):
    fetch = counters(f"{src}/fetch/bench_counter_collection.csv", "FETCH_SIZE")
    write = counters(f"{src}/write/bench_counter_collection.csv", "WRITE_SIZE")
    stats = trace_avg(f"{src}/trace/bench_kernel_stats.csv")
    out = {"_note": "traffic_bytes_per_launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024, medians over "
                    "dispatches (MI355X_MICROARCH.md: FETCH_SIZE counts half of 16-B/lane reads on gfx950)"}
    for k in sorted(fetch):
        if not (k.startswith("void k_adv") or k.startswith("void k_clean") or k.startswith("k_flush")
                or k.startswith("void k_ovl")
                or k.startswith("void k_nmf") or k.startswith("k_nmf")):
            continue
        f, w = statistics.median(fetch[k]), statistics.median(write.get(k, [0.0]))
        calls, avg = stats.get(k, (0, None))
        name = k.replace("void ", "")
        out[name[: name.index("(")] if "(" in name else name] = {
            "launches": len(fetch[k]), "fetch_kib_median": round(f, 2), "write_kib_median": round(w, 2),
            "traffic_bytes_per_launch": int((2 * f + w) * 1024),
            "trace_avg_us": None if avg is None else round(avg, 3)}
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
