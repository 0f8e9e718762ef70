#!/usr/bin/env python3
"""Window-size sweep of the G1 / G2 MSM (ICICLE entry, Montgomery scalars, device operands) across
sizes: wall ms per call (10 reps after 2 warmups) for each c passed through MSMConfig.c, against
the automatic choice (c = 0).  Usage: c_sweep.py [--group g1] [--logs 12,14,16,18] [--cs 0,10,11,12,13,16]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--group", default="g1")
    ap.add_argument("--logs", default="12,14,15,16,17,18,19")
    ap.add_argument("--cs", default="0,10,11,12,13,16")
    a = ap.parse_args()
    import torch
    import bls12_381_amd as amd
    dev = torch.device("cuda", 0)
    w = 12 if a.group == "g1" else 24
    logs = [int(x) for x in a.logs.split(",")]
    N = 1 << max(logs)
    s = torch.zeros((N, 4), dtype=torch.int64, device=dev)
    b = torch.zeros((N, w), dtype=torch.int64, device=dev)
    amd.gen_scalars(s, 0x5EED0003, montgomery=True)
    amd.gen_bases(a.group, b, 0x5EED0013)
    out = torch.zeros((1, w * 3 // 2), dtype=torch.int64, device=dev)
    ref = torch.zeros_like(out)
    torch.cuda.synchronize()
    for lg in logs:
        n = 1 << lg
        row = {"log": lg}
        for c in [int(x) for x in a.cs.split(",")]:
            def call():
                amd.msm(a.group, s, b, icicle=True, scalars_mont=True, c=c, out=out, is_async=True, n=n)
            for _ in range(2):
                call()
            torch.cuda.synchronize()
            if c == 0:
                ref.copy_(out)
            t0 = time.perf_counter()
            for _ in range(10):
                call()
            torch.cuda.synchronize()
            row[f"c{c}"] = round((time.perf_counter() - t0) / 10 * 1e3, 4)
            assert torch.equal(out, ref), (lg, c)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
