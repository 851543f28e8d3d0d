#!/usr/bin/env python
"""Timeline of the dispatches between marker kernels in a rocprofv3 kernel trace.

Reads a `*_kernel_trace.csv` and, for every region bracketed by two
`spin_kernel` dispatches (tools/short_call.py), prints each kernel's start
offset, duration and the idle gap before it, plus totals: device-busy time,
idle gaps, and the region span from the first dispatch's start to the last
one's end.
"""
from __future__ import annotations

import csv
import json
import sys


def regions(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [k for k, r in enumerate(rows) if "spin_kernel" in r[2]]
    for a, b in zip(marks[0::2], marks[1::2]):
        yield rows[a + 1:b]


def summarize(reg):
    t0 = reg[0][0]
    out, prev_end, busy, gaps = [], t0, 0, 0
    for s, e, n in reg:
        gap = max(0, s - prev_end)
        gaps += gap
        busy += e - s
        out.append({"kernel": n.split("(")[0][:60], "start_us": round((s - t0) / 1e3, 2),
                    "dur_us": round((e - s) / 1e3, 2), "gap_us": round(gap / 1e3, 2)})
        prev_end = max(prev_end, e)
    return {"span_us": round((prev_end - t0) / 1e3, 2), "busy_us": round(busy / 1e3, 2),
            "gaps_us": round(gaps / 1e3, 2), "dispatches": len(reg), "timeline": out}


def main():
    res = [summarize(r) for r in regions(sys.argv[1]) if r]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
