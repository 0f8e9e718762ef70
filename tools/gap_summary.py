#!/usr/bin/env python3
"""Median idle time before each kernel (start minus the previous dispatch's end on the same
queue) from a rocprofv3 --kernel-trace CSV, with the predecessor's name.
Usage: gap_summary.py <kernel_trace.csv> [name filter]"""
import csv
import statistics
import sys
from collections import defaultdict


def short(n):
    return n.split("(")[0].replace("void ", "").replace("mbls::", "")[:48]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gaps = defaultdict(list)
    durs = defaultdict(list)
    last_end = {}
    last_name = {}
    for r in rows:
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = short(r["Kernel_Name"])
        if q in last_end:
            gaps[(last_name[q], name)].append((s - last_end[q]) / 1e3)
        durs[name].append((e - s) / 1e3)
        last_end[q], last_name[q] = e, name
    print(f"{'predecessor':>34} -> {'kernel':<34} {'n':>4} {'gap_med_us':>10} {'dur_med_us':>10}")
    for (a, b), v in sorted(gaps.items(), key=lambda kv: -statistics.median(kv[1])):
        if filt and filt not in a + b:
            continue
        print(f"{a:>34} -> {b:<34} {len(v):4d} {statistics.median(v):10.2f} {statistics.median(durs[b]):10.2f}")


if __name__ == "__main__":
    main()
