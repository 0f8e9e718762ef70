#!/usr/bin/env python3
"""Fixed workload for PMC passes (tools/gpu_pmc.sh): `--reps` G1 MSMs of 2^20 (bench.py's
headline inputs and call: ICICLE entry, Montgomery scalars, device bases and result) and
`--reps` forward Fr NTTs of 2^22, `--g2-reps` G2 MSMs of 2^20 (config #5 inputs), nothing else, so per-kernel counter averages are per launch
of exactly the benchmarked configurations."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--msm-log", type=int, default=20)
    ap.add_argument("--ntt-log", type=int, default=22)
    ap.add_argument("--g2-reps", type=int, default=2, help="G2 MSMs of 2^msm_log (config #5 inputs)")
    a = ap.parse_args()
    import torch
    import bls12_381_amd as amd
    dev = torch.device("cuda", 0)
    n = 1 << a.msm_log
    s = torch.zeros((n, 4), dtype=torch.int64, device=dev)
    b = torch.zeros((n, 12), dtype=torch.int64, device=dev)
    amd.gen_scalars(s, 0x5EED0003, montgomery=True)
    amd.gen_bases("g1", b, 0x5EED0013)
    out = torch.zeros((1, 18), dtype=torch.int64, device=dev)
    for _ in range(a.reps):
        amd.msm("g1", s, b, icicle=True, scalars_mont=True, out=out, is_async=True, n=n)
    torch.cuda.synchronize()
    if a.g2_reps:
        s2 = torch.zeros((n, 4), dtype=torch.int64, device=dev)
        b2 = torch.zeros((n, 24), dtype=torch.int64, device=dev)
        amd.gen_scalars(s2, 0x5EED0005, montgomery=True)
        amd.gen_bases("g2", b2, 0x5EED0015)
        o2 = torch.zeros((1, 36), dtype=torch.int64, device=dev)
        for _ in range(a.g2_reps):
            amd.msm("g2", s2, b2, icicle=True, scalars_mont=True, out=o2, is_async=True, n=n)
        torch.cuda.synchronize()
        del s2, b2
    amd.ntt_init_domain()
    x = torch.zeros((1 << a.ntt_log, 4), dtype=torch.int64, device=dev)
    y = torch.zeros_like(x)
    amd.gen_scalars(x, 0x5EED0025, montgomery=True)
    for _ in range(a.reps):
        amd.ntt(x, out=y, is_async=True)
    torch.cuda.synchronize()
    print("pmc probe done", flush=True)


if __name__ == "__main__":
    main()
