#!/usr/bin/env python3
"""Host-staged 2^20 G1 MSM (ICICLE entry, Montgomery scalars on the host, device bases and result):
pinned vs pageable scalars, the device-scalar MSM beside them; wall ms per call (20 reps after 3
warmups), with whatever library MBLS_LIB names.  VERDICT r3 item 5."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))
import torch  # noqa: E402
import bls12_381_amd as amd  # noqa: E402


def main():
    n = 1 << 20
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    s = torch.zeros((n, 4), dtype=torch.int64, device=dev)
    b = torch.zeros((n, 12), dtype=torch.int64, device=dev)
    amd.gen_scalars(s, 0x5EED0003, montgomery=True, stream=st)
    amd.gen_bases("g1", b, 0x5EED0013, stream=st)
    res = torch.zeros((1, 18), dtype=torch.int64, device=dev)
    pinned = s.cpu().pin_memory()
    pageable = s.cpu().numpy().copy()
    torch.cuda.synchronize()

    def timed(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    out = {"lib": os.environ.get("MBLS_LIB", "default")}
    out["device_ms"] = timed(lambda: amd.msm("g1", s, b, scalars_mont=True, out=res, stream=st, is_async=True))
    out["pinned_ms"] = timed(lambda: amd.msm("g1", pinned, b, scalars_mont=True, out=res, stream=st, is_async=True))
    out["pageable_ms"] = timed(lambda: amd.msm("g1", pageable, b, scalars_mont=True, out=res, stream=st, is_async=True))
    out["pinned_h2d_ms"] = out["pinned_ms"] - out["device_ms"]
    out["pageable_h2d_ms"] = out["pageable_ms"] - out["device_ms"]
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
