#!/usr/bin/env python3
"""G2 MSM 2^20 wall time (config #5's inputs, ICICLE entry, device operands): median of --reps
timed calls after one warm-up, and the result digest (to compare settings).  A/B helper:
  for E in "" "MBLS_PSI_SERIAL=1"; do env $E python3 tools/g2_time.py; done"""
import argparse
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    import torch
    import bls12_381_amd as amd
    n = 1 << 20
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    b = torch.zeros((n, 24), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0005, montgomery=True)
    amd.gen_bases("g2", b, 0x5EED0015)
    out = torch.zeros((1, 36), dtype=torch.int64, device="cuda")
    amd.msm("g2", s, b, icicle=True, scalars_mont=True, out=out, is_async=True, n=n)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        amd.msm("g2", s, b, icicle=True, scalars_mont=True, out=out, is_async=True, n=n)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    dig = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"[{os.environ.get('MBLS_TAG', '')}] g2 2^20 median {ts[len(ts) // 2]:.3f} ms min {ts[0]:.3f} digest {dig}", flush=True)


if __name__ == "__main__":
    main()
