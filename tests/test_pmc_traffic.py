"""tools/pmc_traffic.py: the correction bench.py's roofline.traffic relies on
(FETCH_SIZE doubled, k_stream's granule stores divided by their calibrated
WRITE_SIZE factor, k_stream per batch), on synthetic rocprofv3 CSVs."""
import csv
import importlib.util
import json
import os

from conftest import REPO


def _load():
    spec = importlib.util.spec_from_file_location("pmc_traffic", os.path.join(REPO, "tools", "pmc_traffic.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _counters(path, name, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for k, v in rows:
            w.writerow({"Kernel_Name": k, "Counter_Name": name, "Counter_Value": v})


def test_corrections_and_per_batch_stream(tmp_path):
    src = tmp_path / "prof"
    gib_kib = (1 << 30) / 1024
    stream = "void k_stream<16, 1, 4>(StepArgs, int)"
    adam = "k_nmf_adam(float*)"
    _counters(str(src / "fetch" / "bench_counter_collection.csv"), "FETCH_SIZE",
              [(stream, 1000.0), (stream, 1000.0), (adam, 50.0)])
    _counters(str(src / "write" / "bench_counter_collection.csv"), "WRITE_SIZE",
              [(stream, 800.0), (stream, 800.0), (adam, 100.0)])
    _counters(str(src / "calib_fetch" / "calib_counter_collection.csv"), "FETCH_SIZE",
              [("k_read16(float4 const*, long, float*)", 0.5 * gib_kib),
               ("k_read_granules(unsigned long long const*, long, float*)", 0.5 * gib_kib)])
    _counters(str(src / "calib_write" / "calib_counter_collection.csv"), "WRITE_SIZE",
              [("k_write_granules(unsigned long long*, long)", 4.0 * gib_kib),
               ("k_write_granules_cm(unsigned long long*, long)", 2.0 * gib_kib)])
    os.makedirs(src / "trace")
    with open(src / "trace" / "bench_kernel_stats.csv", "w") as f:
        f.write('"Name","Calls","AverageNs"\n')
        f.write(f'"{stream}",2,8000.0\n"{adam}",1,30000.0\n')
    dst = tmp_path / "pmc.json"
    json.dump({"k_adv_list<16, 1>": {"traffic_bytes_per_launch": 7}}, open(dst, "w"))
    _load().main(str(src), str(dst), 10)
    out = json.load(open(dst))
    assert out["_calibration"]["FETCH_SIZE:read_granule"] == 0.5
    assert out["_calibration"]["WRITE_SIZE:write_granule_consecutive"] == 2.0
    rec = out["k_stream<16, 1, 4>"]
    # 2 x FETCH + WRITE / (calibrated factor 2), KiB -> bytes; per batch over 10 batches
    assert rec["traffic_bytes_per_launch"] == int((2 * 1000 + 800 / 2) * 1024)
    assert rec["traffic_bytes_per_batch"] == int(rec["traffic_bytes_per_launch"] / 10)
    assert rec["trace_avg_us"] == 8.0
    # kernels without granule stores: WRITE_SIZE taken as exact
    assert out["k_nmf_adam"]["traffic_bytes_per_launch"] == int((2 * 50 + 100) * 1024)
    # a record the passes did not cover is kept, marked
    assert out["k_adv_list<16, 1>"]["from_earlier_pass"] is True


def test_bench_scales_stream_record_to_its_launch():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    newest = sorted(d for d in os.listdir(os.path.join(REPO, "profiles"))
                    if os.path.isfile(os.path.join(REPO, "profiles", d, "pmc_traffic.json")))[-1]
    rec = json.load(open(os.path.join(REPO, "profiles", newest, "pmc_traffic.json")))["k_stream<16, 1, 4>"]
    got, source = bench.pmc_traffic("k_stream<16, 1, 4>", 400)
    assert got == int(rec["traffic_bytes_per_batch"] * 400)
    assert "per batch x 400" in source
