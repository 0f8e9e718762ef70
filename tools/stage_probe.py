#!/usr/bin/env python3
"""Per-stage MSM times (HIP-event stage profiler) for one group / size:
   python tools/stage_probe.py --group g2 --log 20 --reps 5"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--group", default="g1")
    ap.add_argument("--log", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import bls12_381_amd as amd
    dev = torch.device("cuda", 0)
    n = 1 << a.log
    width = 12 if a.group == "g1" else 24
    s = torch.zeros((n, 4), dtype=torch.int64, device=dev)
    b = torch.zeros((n, width), dtype=torch.int64, device=dev)
    amd.gen_scalars(s, 0x5EED0005, montgomery=True)
    amd.gen_bases(a.group, b, 0x5EED0015)
    out = torch.zeros((1, width * 3 // 2), dtype=torch.int64, device=dev)
    for _ in range(2):
        amd.msm(a.group, s, b, icicle=False, scalars_mont=True, out=out, is_async=True, n=n)
    torch.cuda.synchronize()
    amd.profile(True)
    for _ in range(a.reps):
        amd.msm(a.group, s, b, icicle=False, scalars_mont=True, out=out, is_async=True, n=n)
    torch.cuda.synchronize()
    prof = amd.profile_read()
    amd.profile(False)
    print(json.dumps({k: round(v[0] / v[1], 4) for k, v in sorted(prof.items()) if v[1]}))


if __name__ == "__main__":
    main()
