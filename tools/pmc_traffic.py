"""Per-launch HBM traffic of the step kernels from rocprofv3 PMC passes
(tools/profile_bench.sh), corrected as MI355X_MICROARCH.md §HBM prescribes and
by this repo's own calibration (tools/calib_fetch.hip, same passes):
  FETCH_SIZE reports half the bytes of coalesced 16-B/lane reads on gfx950 — and,
  calibrated here, of the 8-B/lane granule reads k_stream uses — so it is doubled;
  WRITE_SIZE is exact for 16-B/lane stores; for k_stream's 8-B granule stores the
  calibrated factor of the same store pattern divides it.
Both counters are in KiB per dispatch.

Usage: python tools/pmc_traffic.py gpurun_out/prof profiles/r01/pmc_traffic.json [batches_per_stream_launch]
Writes {kernel name: {launches, fetch_kib_median, write_kib_median,
traffic_bytes_per_launch, trace_avg_us}} for the step kernels, and for k_stream
(one launch = many batches) also traffic_bytes_per_batch.  Records of kernels the
passes did not run are kept from the existing file (from_earlier_pass)."""
import csv
import json
import statistics
import sys
from collections import defaultdict

CALIB_BYTES = 1 << 30  # tools/calib_fetch.py
CALIB_KERNELS = {"k_read16": "read16", "k_read_granules": "read_granule",
                 "k_write_granules": "write_granule_strided", "k_write_granules_cm": "write_granule_consecutive"}


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


def calibration(src):
    """counter KiB x 1024 / true bytes, per access pattern (None if the pass is absent)"""
    out = {}
    for sub, cname in (("calib_fetch", "FETCH_SIZE"), ("calib_write", "WRITE_SIZE")):
        try:
            vals = counters(f"{src}/{sub}/calib_counter_collection.csv", cname)
        except FileNotFoundError:
            continue
        for k, v in vals.items():
            base = k.split("(")[0].replace("void ", "")
            if base in CALIB_KERNELS:
                out[f"{cname}:{CALIB_KERNELS[base]}"] = round(statistics.median(v) * 1024 / CALIB_BYTES, 4)
    return out


def main(src, dst, stream_batches=647):
    fetch = counters(f"{src}/fetch/bench_counter_collection.csv", "FETCH_SIZE")
    write = counters(f"{src}/write/bench_counter_collection.csv", "WRITE_SIZE")
    stats = trace_avg(f"{src}/trace/bench_kernel_stats.csv")
    cal = calibration(src)
    if not cal:  # no calibration pass this time: the previous file's (same kernels, same chip)
        try:
            with open(dst) as fh:
                cal = dict(json.load(fh).get("_calibration", {}), from_earlier_pass=True)
        except (FileNotFoundError, ValueError):
            cal = {}
    granule_write = cal.get("WRITE_SIZE:write_granule_consecutive", 1.0)
    out = {"_note": "traffic_bytes_per_launch = (2 x FETCH_SIZE + WRITE_SIZE / w) x 1024, medians over "
                    "dispatches (MI355X_MICROARCH.md: FETCH_SIZE counts half of 16-B/lane reads on gfx950; "
                    "calibration shows the same for 8-B granule reads); w = 1, except k_stream: w = the "
                    "calibrated WRITE_SIZE factor of its 8-B granule stores",
           "_calibration": cal}
    for k in sorted(fetch):
        if not (k.startswith("void k_adv") or k.startswith("void k_clean") or k.startswith("k_flush")
                or k.startswith("void k_ovl") or k.startswith("void k_stream") or k.startswith("k_stream")
                or k.startswith("void k_nmf") or k.startswith("k_nmf") or k.startswith("void k_tri")
                or k.startswith("void k_hot")):
            continue
        f, w = statistics.median(fetch[k]), statistics.median(write.get(k, [0.0]))
        calls, avg = stats.get(k, (0, None))
        name = k.replace("void ", "")
        name = name[: name.index("(")] if "(" in name else name
        wf = granule_write if name.startswith("k_stream<") else 1.0
        rec = {"launches": len(fetch[k]), "fetch_kib_median": round(f, 2), "write_kib_median": round(w, 2),
               "traffic_bytes_per_launch": int((2 * f + w / wf) * 1024),
               "trace_avg_us": None if avg is None else round(avg, 3)}
        if name.startswith("k_stream<"):
            rec["batches_per_launch"] = stream_batches
            rec["traffic_bytes_per_batch"] = int(rec["traffic_bytes_per_launch"] / stream_batches)
            rec["write_factor"] = wf
        out[name] = rec
    try:  # kernels these passes did not run (e.g. the --large list kernels) keep their earlier records
        with open(dst) as fh:
            prev = json.load(fh)
        for k, v in prev.items():
            if not k.startswith("_") and k not in out:
                out[k] = dict(v, from_earlier_pass=True)
    except (FileNotFoundError, ValueError):
        pass
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(int(x) for x in sys.argv[3:4]))
