#!/usr/bin/env python3
"""rocprof workload: G2 MSMs of 2^20 (config #5's inputs, ICICLE entry), for a kernel timeline."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))


def main():
    import torch
    import bls12_381_amd as amd
    n = 1 << 20
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    b = torch.zeros((n, 24), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0005, montgomery=True)
    amd.gen_bases("g2", b, 0x5EED0015)
    out = torch.zeros((1, 36), dtype=torch.int64, device="cuda")
    for _ in range(3):
        amd.msm("g2", s, b, icicle=True, scalars_mont=True, out=out, is_async=True, n=n)
    torch.cuda.synchronize()
    print("g2 probe done", flush=True)


if __name__ == "__main__":
    main()
