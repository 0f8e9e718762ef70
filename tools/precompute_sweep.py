#!/usr/bin/env python3
"""G1 MSM wall ms per call (ICICLE entry, Montgomery scalars, device operands; 10 reps after 2
warmups) with plain bases (F = 1) and precompute tables F = 2 (prepared [P, phi P]), 4, 8, across
sizes; every result equal to the plain one.  Usage: precompute_sweep.py [--logs 14,16,18,20]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--logs", default="14,16,18,20")
    ap.add_argument("--group", default="g1")
    ap.add_argument("--fs", default="")
    ap.add_argument("--cs", default="0", help="window sizes passed through MSMConfig.c (0 = automatic)")
    a = ap.parse_args()
    import torch
    import bls12_381_amd as amd
    w = 12 if a.group == "g1" else 24
    fs = (1, 2, 4, 8) if a.group == "g1" else (1, 4, 8)
    if a.fs:
        fs = tuple(int(x) for x in a.fs.split(","))
    cs = [int(x) for x in a.cs.split(",")]
    for lg in [int(x) for x in a.logs.split(",")]:
        n = 1 << lg
        s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        b = torch.zeros((n, w), dtype=torch.int64, device="cuda")
        amd.gen_scalars(s, 0x5EED0003, montgomery=True)
        amd.gen_bases(a.group, b, 0x5EED0013)
        ref = torch.zeros((1, w * 3 // 2), dtype=torch.int64, device="cuda")
        out = torch.zeros_like(ref)
        row = {"log": lg}
        for F, c in [(F, c) for F in fs for c in (cs if F > 1 else [0])]:
            tab = b
            if F > 1:
                tab = torch.zeros((n * F, w), dtype=torch.int64, device="cuda")
                amd.precompute_bases(a.group, b, F, n, out=tab)
            torch.cuda.synchronize()

            def call():
                amd.msm(a.group, s, tab, icicle=True, scalars_mont=True, points_mont=(F == 1), precompute_factor=F, c=c,
                        out=out if F > 1 else ref, is_async=True, n=n)
            for _ in range(2):
                call()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                call()
            torch.cuda.synchronize()
            row[f"F{F}" + (f"c{c}" if c else "")] = round((time.perf_counter() - t0) / 10 * 1e3, 4)
            if F > 1:
                assert torch.equal(out, ref), (lg, F)
            del tab
        print(json.dumps(row), flush=True)
        del s, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
