import sys, os
sys.path.insert(0, "/root/repo/midnight-bls12-381-cuda_amd"); sys.path.insert(0, "/root/repo/tests")
import numpy as np
import bls12_381_amd as amd
import helpers as H
from helpers import pyref as pr
amd.ntt_init_domain()
for log_n in (1, 2, 3, 4, 9, 11):
    n = 1 << log_n
    x = np.zeros((n, 4), dtype=np.uint64)
    x[1] = pr.int_to_limbs(pr.fr_to_mont(1), 4)
    got = [pr.fr_from_mont(v) for v in H.limbs_to_ints(amd.ntt(x))]
    w = pr.omega(log_n)
    exp = [pow(w, j, pr.R) for j in range(n)]
    bad = [j for j in range(n) if got[j] != exp[j]]
    print(log_n, "bad", len(bad), bad[:8], flush=True)
    if bad:
        j = bad[0]
        for s in range(1, log_n + 1):
            ws = pr.omega(s)
            print("  got[j] == w_s^k ?", s, [k for k in range(1 << s) if pow(ws, k, pr.R) == got[j]][:3])
