#!/usr/bin/env python3
"""G1 / G2 MSM wall ms per call on skewed scalar distributions (prover-shaped: selector-like 0 / 1
columns, small scalars, one repeated value) against uniform random scalars, device operands,
standard-form scalars, ICICLE entry.  Usage: skew_probe.py [--log 20] [--group g1]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log", type=int, default=20)
    ap.add_argument("--group", default="g1")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cases", default="")
    ap.add_argument("--stages", action="store_true", help="also print the stage profiler's ms per stage")
    a = ap.parse_args()
    import torch
    import bls12_381_amd as amd
    n = 1 << a.log
    w = 12 if a.group == "g1" else 24
    b = torch.zeros((n, w), dtype=torch.int64, device="cuda")
    amd.gen_bases(a.group, b, 0x5EED0013)
    rnd = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(rnd, 0x5EED0003, montgomery=False)
    half = torch.arange(n, device="cuda") % 2 == 0
    one = torch.tensor([1, 0, 0, 0], dtype=torch.int64, device="cuda")

    def case(name):
        s = rnd.clone()
        if name == "ones":
            s[:] = one
        elif name == "half_zero":
            s[half] = 0
        elif name == "half_one":
            s[half] = one
        elif name == "bits8":
            s[:, 1:] = 0
            s[:, 0] &= 0xff
        elif name == "bits1_of_64":  # 64-bit scalars with one set bit each
            s[:, 1:] = 0
            s[:, 0] = torch.bitwise_left_shift(torch.ones(n, dtype=torch.int64, device="cuda"),
                                               torch.arange(n, device="cuda") % 63)
        elif name == "repeated":
            s[:] = rnd[7]
        return s

    cases = a.cases.split(",") if a.cases else ["random", "half_zero", "half_one", "bits8", "bits1_of_64", "ones",
                                                "repeated"]
    out = torch.zeros((1, w * 3 // 2), dtype=torch.int64, device="cuda")
    row = {"group": a.group, "log": a.log}
    for name in cases:
        s = case(name)
        torch.cuda.synchronize()

        def call():
            amd.msm(a.group, s, b, icicle=True, scalars_mont=False, points_mont=True, out=out, is_async=True, n=n)
        call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            call()
        torch.cuda.synchronize()
        row[name] = round((time.perf_counter() - t0) / a.reps * 1e3, 3)
        print(json.dumps(row), flush=True)
        if a.stages:
            amd.profile(True)
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            prof = amd.profile_read()
            amd.profile(False)
            print(json.dumps({"case": name, "stage_ms": {k: round(v[0] / v[1], 4) for k, v in sorted(prof.items()) if v[1]}}),
                  flush=True)


if __name__ == "__main__":
    main()
