#!/usr/bin/env python3
"""rocprof workload: the bench's batched G1 MSM (batch 8 x 2^20, shared device bases, ICICLE
entry, members pipelined on two streams), twice, for a kernel timeline of the pipelining."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))


def main():
    import torch
    import bls12_381_amd as amd
    n, B = 1 << 20, 8
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0013)
    sb = torch.zeros((B * n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(sb, 0x5EED0033, montgomery=True)
    rb = torch.zeros((B, 18), dtype=torch.int64, device="cuda")
    for _ in range(2):
        amd.msm("g1", sb, b, icicle=True, scalars_mont=True, batch=B, out=rb, is_async=True, n=n)
    torch.cuda.synchronize()
    print("batch probe done", flush=True)


if __name__ == "__main__":
    main()
