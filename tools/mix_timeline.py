#!/usr/bin/env python3
"""Timeline of the last G2 MSM + NTT batch of tools/mix_probe.py from a rocprofv3 kernel trace:
every dispatch from the last G2 split kernel on, start / end offsets (us), queue, name; then the
span of each stream's work.  Usage: mix_timeline.py <run_kernel_trace.csv>"""
import csv
import sys


def short(n):
    n = n.split("(")[0].replace("void ", "").replace("mbls::", "")
    return n.replace("Fp<FqCfg>", "G1").replace("Fp<FrCfg>", "Fr").replace("PFq2", "G2")[:46]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_psi" in r["Kernel_Name"]]
i0 = starts[-1]
# include NTT kernels that started before the split on the other queue (enqueued together)
t_first = int(rows[i0]["Start_Timestamp"])
sel = [r for r in rows if int(r["End_Timestamp"]) >= t_first - 5_000_000]
t0 = min(int(r["Start_Timestamp"]) for r in sel if int(r["Start_Timestamp"]) >= t_first - 3_000_000)
span = {}
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0:
        continue
    q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
    span.setdefault(q, [s, e])
    span[q][0] = min(span[q][0], s)
    span[q][1] = max(span[q][1], e)
    print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  q{q}  {short(r['Kernel_Name'])}")
for q, (s, e) in span.items():
    print(f"queue {q}: {(s - t0) / 1e3:.1f} .. {(e - t0) / 1e3:.1f} us")
