#!/usr/bin/env python3
"""rocprof workload: `--reps` G1 MSMs of 2^log through the ICICLE entry (Montgomery scalars,
(x, y, 1) result) and `--reps` through the raw entry (standard scalars, Jacobian result), bench
inputs, so the per-kernel trace shows what the production path adds."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--log", type=int, default=20)
    a = ap.parse_args()
    import torch
    import bls12_381_amd as amd
    n = 1 << a.log
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    s_std = torch.zeros_like(s)
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0003, montgomery=True)
    amd.gen_scalars(s_std, 0x5EED0003, montgomery=False)
    amd.gen_bases("g1", b, 0x5EED0013)
    out = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
    for _ in range(a.reps):
        amd.msm("g1", s, b, icicle=True, scalars_mont=True, out=out, is_async=True, n=n)
    torch.cuda.synchronize()
    for _ in range(a.reps):
        amd.msm("g1", s_std, b, icicle=False, out=out, is_async=True, n=n)
    torch.cuda.synchronize()
    print("paths probe done", flush=True)


if __name__ == "__main__":
    main()
