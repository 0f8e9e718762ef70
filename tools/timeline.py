#!/usr/bin/env python3
"""Per-dispatch timeline of one MSM from a rocprofv3 --kernel-trace CSV: the dispatches from the
LAST k_digits / k_glv_split launch of the run up to the next non-MSM kernel, with start offset,
duration and queue, to read the critical path and the gaps between launches.
Usage: timeline.py <run_kernel_trace.csv> [which: index of the MSM counted from the end, default 1]"""
import csv
import sys


def short(n):
    n = n.split("(")[0].replace("void ", "").replace("mbls::", "")
    return n.replace("Fp<FqCfg>", "G1").replace("Fp<FrCfg>", "Fr")[:48]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    which = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if any(k in r["Kernel_Name"] for k in ("k_glv_split", "k_glv_prep", "k_psi_split", "k_psi_prep"))]
    if not starts:
        print("no MSM found")
        return
    i0 = starts[-which]
    i1 = starts[-which + 1] if which > 1 else len(rows)
    t0 = int(rows[i0]["Start_Timestamp"])
    for r in rows[i0:i1]:
        if "ntt" in r["Kernel_Name"] or "k_twiddles" in r["Kernel_Name"]:
            break
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>3}  {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
