"""Diagnostic: time individual MSM calls (progress flushed line by line)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import helpers as H  # noqa: E402
import gpu_helpers as gh  # noqa: E402
from helpers import pyref as pr  # noqa: E402

amd = gh.amd
group = sys.argv[1] if len(sys.argv) > 1 else "g2"
g = H.load_golden(f"msm_{group}.json")
import torch  # noqa: E402

torch.cuda.init()
for case in g["cases"]:
    sc = [H.hx(s) for s in case["scalars"]]
    pts = [H.pt_from_json(b, group) for b in case["bases"]]
    n = len(sc)
    nl = 12 if group == "g1" else 24
    s_std = H.ints_to_limbs(sc, 4) if n else np.zeros((0, 4), dtype=np.uint64)
    b_mont = gh.affine_mont_array(group, pts) if n else np.zeros((0, nl), dtype=np.uint64)
    t = time.time()
    r = amd.msm(group, s_std, b_mont, icicle=True, n=n)
    dt = time.time() - t
    ok = gh.decode_icicle(group, r[0]) == H.pt_from_json(case["result"], group)
    print(f"{case['name']:40s} n={n:5d} {dt*1e3:9.1f} ms ok={ok}", flush=True)
