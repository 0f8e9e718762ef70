#!/usr/bin/env python3
"""vector add / mul 2^24 (and 2^16) GB/s, the bench's vecops leg alone (A/B of vecops builds)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))


def main():
    import torch
    import bls12_381_amd as amd
    row = {}
    for log_n in (16, 24):
        n = 1 << log_n
        a = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        b = torch.zeros_like(a)
        c = torch.zeros_like(a)
        amd.gen_scalars(a, 0x5EED0001, montgomery=True)
        amd.gen_scalars(b, 0x5EED0101, montgomery=True)
        for op in ("add", "mul"):
            reps = 200 if log_n == 16 else 50
            for _ in range(3):
                amd.vec_op(op, a, b, out=c, is_async=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                amd.vec_op(op, a, b, out=c, is_async=True)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / reps * 1e3
            row[f"{op}_2^{log_n}_gbs"] = round(96 * n / (ms * 1e-3) / 1e9, 1)
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
