"""NTT timing probe: forward / inverse 2^k transforms (device in / out, the prover's shape), stage
profiler per transform and per pass, wall time per call, and the exact round trip.
Usage: python tools/ntt_time.py [log_n=22] [reps=50]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "midnight-bls12-381-cuda_amd"))
import torch  # noqa: E402

import bls12_381_amd as amd  # noqa: E402


def main():
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    n = 1 << log_n
    x = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(x, 0x5EED7700, montgomery=True)
    y, z = torch.zeros_like(x), torch.zeros_like(x)
    amd.ntt_init_domain()
    st = torch.cuda.Stream()
    out = {"log_n": log_n, "reps": reps}
    for name, fn in (("forward", lambda: amd.ntt(x, out=y, stream=st, is_async=True)),
                     ("inverse", lambda: amd.ntt(y, inverse=True, out=z, stream=st, is_async=True))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps * 1e3
        amd.profile(True)
        for _ in range(reps):
            fn()
        prof = amd.profile_read()
        amd.profile(False)
        t, p = prof.get("ntt.transform", (0, 0)), prof.get("ntt.pass", (0, 0))
        out[name] = {"wall_ms": round(wall, 4), "per_sec": round(1e3 / wall, 1),
                     "transform_ms": round(t[0] / t[1], 4) if t[1] else None,
                     "pass_ms": round(p[0] / p[1], 4) if p[1] else None}
    torch.cuda.synchronize()
    out["roundtrip_exact"] = bool(torch.equal(z, x))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
