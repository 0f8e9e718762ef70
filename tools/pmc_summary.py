#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel (average per dispatch).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide
(16 B/lane) reads, so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (counters are in KB).
Usage: pmc_summary.py <dir holding FETCH_SIZE/ and WRITE_SIZE/ rocprofv3 outputs>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    per = defaultdict(list)
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r.get("Kernel_Name", "?")
            per[name].append(float(r["Counter_Value"]))
    return per


def short(name):
    for key in ("k_accumulate", "k_ntt_pass<true, false, false>", "k_ntt_pass<false, false, false>",
                "k_ntt_pass<false, true, false>", "k_ntt_pass<false, true, true>",
                "k_scatter", "k_digits_tiled", "k_bucket_small", "k_reduce_level", "k_glv_table", "k_vecop"):
        if key.replace(" ", "") in name.replace(" ", ""):
            return key
    return name[:80]


def main():
    d = sys.argv[1]
    fetch, write = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    out = {}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        fa = sum(f) / len(f) if f else None
        wa = sum(w) / len(w) if w else None
        out[short(name)] = {
            "dispatches": max(len(f), len(w)),
            "fetch_kb_avg": fa, "write_kb_avg": wa,
            "hbm_bytes_per_launch": (2 * (fa or 0) + (wa or 0)) * 1024 if (fa is not None or wa is not None) else None,
        }
    print(json.dumps({"correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE halving)",
                      "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
