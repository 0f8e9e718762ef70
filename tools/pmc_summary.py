#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes per kernel (average per dispatch of every counter found).

Directory layout: <dir>/<pass name>/**/*counter_collection.csv (one rocprofv3 run per pass).
gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide
(16 B/lane) reads, so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (counters are in KB).  The
halving is measured for coalesced streaming reads; for the MSM's random 96-byte point gathers it
is unverified, so `hbm_bytes_per_launch_uncorrected` (FETCH_SIZE + WRITE_SIZE) is kept beside it.
VALU: SQ_INSTS_VALU / SQ_INSTS_VALU_INT64 count wave-level instructions (x 64 lanes for lane ops);
v_mad_u64_u32 is an INT64 instruction.
Usage: pmc_summary.py <dir>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# (substring, key): G1 / G2 instances of the templated MSM kernels kept apart
ALIASES = (("k_accumulate_r28p<mbls::Fq2", "k_accumulate<G2>"), ("k_accumulate_r28<mbls::Fp<mbls::FqCfg>", "k_accumulate<G1>"), ("k_accumulate<mbls::Fp<mbls::FqCfg>", "k_accumulate<G1>"), ("k_accumulate<mbls::Fq2", "k_accumulate<G2>"),
           ("k_bucket_small<mbls::Fp<mbls::FqCfg>", "k_bucket_small<G1>"), ("k_bucket_small<mbls::Fq2", "k_bucket_small<G2>"))
KEYS = ("k_accumulate", "k_ntt_pass<true, false, false>", "k_ntt_pass<false, false, false>",
        "k_ntt_pass<false, true, false>", "k_ntt_pass<false, true, true>", "k_scatter", "k_digits_tiled",
        "k_digits_part", "k_part_sort", "k_bucket_small", "k_reduce_scaled", "k_reduce_tree4", "k_glv_table", "k_glv_prep", "k_vecop", "k_final",
        "k_jac_to_icicle")


def short(name):
    for sub, key in ALIASES:
        if sub.replace(" ", "") in name.replace(" ", ""):
            return key
    for key in KEYS:
        if key.replace(" ", "") in name.replace(" ", ""):
            return key
    return name.split("(")[0][:80]


def main():
    d = sys.argv[1]
    # counter -> kernel -> dispatch -> summed value
    vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = short(r.get("Kernel_Name", "?"))
            vals[r["Counter_Name"]][name][(f, r.get("Dispatch_Id"))] += float(r["Counter_Value"])
    out = defaultdict(dict)
    for counter, per_k in vals.items():
        for k, disp in per_k.items():
            out[k][counter] = sum(disp.values()) / len(disp)
            out[k]["dispatches"] = max(out[k].get("dispatches", 0), len(disp))
    for k, row in out.items():
        fa, wa = row.get("FETCH_SIZE"), row.get("WRITE_SIZE")
        if fa is not None or wa is not None:
            row["hbm_bytes_per_launch"] = (2 * (fa or 0) + (wa or 0)) * 1024
            row["hbm_bytes_per_launch_uncorrected"] = ((fa or 0) + (wa or 0)) * 1024
    print(json.dumps({"correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE halving, "
                                    "measured for coalesced streaming reads)",
                      "kernels": {k: out[k] for k in sorted(out)}}, indent=1))


if __name__ == "__main__":
    main()
