#!/usr/bin/env python3
"""Config #5 overlap probe: G2 MSM 2^20 (ICICLE entry) on a high-priority stream and a batch of 4
Fr NTTs 2^22 on a normal-priority stream, enqueued together, 3 times; run under
rocprofv3 --kernel-trace and read with tools/mix_timeline.py.  Usage: mix_probe.py [--equal]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))


def main():
    import torch
    import bls12_381_amd as amd
    equal = "--equal" in sys.argv
    dev = torch.device("cuda", 0)
    n, nn, B = 1 << 20, 1 << 22, 4
    s_a = torch.cuda.Stream(dev, priority=0 if equal else -1)
    s_b = torch.cuda.Stream(dev)
    sc = torch.zeros((n, 4), dtype=torch.int64, device=dev)
    bs = torch.zeros((n, 24), dtype=torch.int64, device=dev)
    amd.gen_scalars(sc, 0x5EED0005, montgomery=True)
    amd.gen_bases("g2", bs, 0x5EED0015)
    res = torch.zeros((1, 36), dtype=torch.int64, device=dev)
    xb = torch.zeros((B * nn, 4), dtype=torch.int64, device=dev)
    yb = torch.zeros_like(xb)
    amd.gen_scalars(xb, 0x5EED0025, montgomery=True)
    amd.ntt_init_domain()
    torch.cuda.synchronize()
    ev = amd.HipEvent()
    for _ in range(3):
        if not equal:
            amd.msm_accumulate_event(s_a, ev.handle)
        amd.msm("g2", sc, bs, icicle=True, scalars_mont=True, out=res, stream=s_a, is_async=True, n=n)
        if not equal:
            ev.wait(s_b)
        amd.ntt(xb, out=yb, batch=B, stream=s_b, is_async=True)
        torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
