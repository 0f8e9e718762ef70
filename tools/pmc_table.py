#!/usr/bin/env python3
"""Per-kernel averages of every rocprofv3 --pmc counter found under the given directories
(one directory per pass), as JSON: {kernel: {counter: avg per dispatch, "dispatches": n}}.
Derived, for the VALU passes (counter units per MI355X_MICROARCH.md: SQ_*_CYCLES / SQ_ACTIVE_INST_*
count quad-cycles; GRBM_GUI_ACTIVE counts GPU clocks; 256 CUs x 4 SIMDs):
  valu_busy  = 4 * SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE * 1024)   (fraction of SIMD cycles with a VALU issue)
  valu_ipc   = SQ_INSTS_VALU / (GRBM_GUI_ACTIVE * 1024)              (wave-instructions per SIMD-cycle)
Usage: pmc_table.py <label> <dir> [<dir> ...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KEEP = ("k_accumulate", "k_ntt_pass", "k_bucket_small", "k_reduce_scaled", "k_final", "k_jac_to_icicle",
        "k_digits_part", "k_part_sort", "k_glv_table", "k_vecop", "k_glv_split", "k_glv_prep")


def short(name):
    base = name.split("(")[0].replace("void ", "").replace("mbls::", "")
    return base.replace("Fp<FqCfg>", "G1").replace("Fp<FrCfg>", "Fr")


def main():
    label, dirs = sys.argv[1], sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "?")
                if not any(k in name for k in KEEP):
                    continue
                key = (short(name), r.get("Dispatch_Id"))
                vals[short(name)][r["Counter_Name"]].append((r.get("Dispatch_Id"), float(r["Counter_Value"])))
    out = {}
    for k, cs in sorted(vals.items()):
        row = {}
        for c, lst in cs.items():
            # rocprofv3 writes one row per dispatch per counter (already summed over instances)
            per = defaultdict(float)
            for did, v in lst:
                per[did] += v
            row[c] = sum(per.values()) / len(per)
            row["dispatches"] = len(per)
        g = row.get("GRBM_GUI_ACTIVE")
        if g:
            if "SQ_ACTIVE_INST_VALU" in row:
                row["valu_busy"] = 4 * row["SQ_ACTIVE_INST_VALU"] / (g * 1024)
            if "SQ_INSTS_VALU" in row:
                row["valu_ipc_per_simd"] = row["SQ_INSTS_VALU"] / (g * 1024)
        out[k] = row
    print(json.dumps({"label": label, "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
