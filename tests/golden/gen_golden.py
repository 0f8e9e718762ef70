#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the pure-Python restatement
(oracle/pyref.py).  Deterministic: re-running reproduces the committed JSON byte for byte.

Values are stored as hex strings of the integer a byte layout holds:
  * scalars in MSM fixtures: standard-form integers in [0, r), except the
    ``noncanonical_scalars`` case ([r, 2^256): the result is (s mod r) P);
  * points: affine standard-form coordinates, ``null`` = identity
    (G2 coordinates are [c0, c1] pairs);
  * vecops / NTT fixtures: the raw 256-bit value of the limbs, i.e. the Montgomery-encoded
    value of the logical field element (vecops ``mul`` is the Montgomery product on raw
    limbs, reference ``vec_ops.cu:93-103`` / ``field.cuh:510-576``).

Reference-held known-answer values (constants, generators, 2^32 root) are *copied data*
from ``bls12-381/include/bls12_381_constants.h`` and ``tests/test_known_answer_vectors.cu``
and live in ``reference_kat.json`` (hand-transcribed, with file:line citations); this
script does not generate that file.

Usage:  python3 tests/golden/gen_golden.py
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pyref as pr  # noqa: E402


def h(x):
    if x is None:
        return None
    if isinstance(x, tuple):
        return [h(v) for v in x]
    return hex(x)


def pt_json(pt):
    if pt is None:
        return None
    return [h(pt[0]), h(pt[1])]


def dump(name, obj):
    path = os.path.join(HERE, name)
    with open(path, "w") as f:
        json.dump(obj, f, indent=0, sort_keys=True)
        f.write("\n")
    print("wrote", path)


# ----------------------------------------------------------------------------------------
def gen_vecops():
    g = pr.rng(0x5EED0001)
    edge = [0, 1, 2, pr.FR_R, pr.R - 1, pr.R - 2, (pr.R - 1) // 2, (pr.R + 1) // 2,
            (1 << 255) % pr.R, (1 << 64) - 1, (1 << 128) - 1, pr.FR_R2]
    a = edge + [pr.random_fr(g) for _ in range(116)]
    b = [pr.random_fr(g) for _ in range(len(edge))] + [pr.random_fr(g) for _ in range(116)]
    # make a few b equal to a or to -a to exercise the carry / zero paths
    b[20] = a[20]
    b[21] = (-a[21]) % pr.R
    b[22] = 0
    b[23] = pr.R - 1
    s = pr.random_fr(g)
    return {
        "n": len(a),
        "a": [h(x) for x in a],
        "b": [h(x) for x in b],
        "scalar": h(s),
        "add": [h((x + y) % pr.R) for x, y in zip(a, b)],
        "sub": [h((x - y) % pr.R) for x, y in zip(a, b)],
        "mul": [h(pr.fr_mont_mul(x, y)) for x, y in zip(a, b)],
        "scalar_mul": [h(pr.fr_mont_mul(s, y)) for y in b],
        "scalar_add": [h((s + y) % pr.R) for y in b],
    }


def gen_ntt():
    g = pr.rng(0x5EED0002)
    cases = []
    for log_n in range(0, 11):
        n = 1 << log_n
        x = [pr.random_fr(g) for _ in range(n)]
        cases.append({"name": f"random_2^{log_n}", "log_n": log_n, "input": [h(v) for v in x],
                      "forward": [h(v) for v in pr.ntt_forward(x)],
                      "inverse": [h(v) for v in pr.ntt_inverse(x)]})
    for log_n in (3, 6):
        n = 1 << log_n
        specials = {
            "zeros": [0] * n,
            "delta0": [1] + [0] * (n - 1),
            "delta1": [0, 1] + [0] * (n - 2),
            "constant": [pr.FR_R] * n,
            "r_minus_1": [pr.R - 1] * n,
        }
        for nm, x in specials.items():
            cases.append({"name": f"{nm}_2^{log_n}", "log_n": log_n, "input": [h(v) for v in x],
                          "forward": [h(v) for v in pr.ntt_forward(x)],
                          "inverse": [h(v) for v in pr.ntt_inverse(x)]})
    omegas = {str(k): h(pr.fr_to_mont(pr.omega(k))) for k in range(0, 33)}
    return {"cases": cases, "omega_mont": omegas,
            "root_of_unity_mont": h(pr.fr_to_mont(pr.ROOT_OF_UNITY))}


def _msm_cases(group: str, seed: int, rand_sizes):
    gen = pr.G1 if group == "g1" else pr.G2
    mul = pr.g1_mul if group == "g1" else pr.g2_mul
    neg = pr.g1_neg if group == "g1" else pr.g2_neg
    g = pr.rng(seed)
    cases = []

    def add_case(name, scalars, bases, result=None):
        if result is None:
            result = pr.msm_shared_doubling(scalars, bases, group)
        cases.append({"name": name, "n": len(scalars), "scalars": [h(s) for s in scalars],
                      "bases": [pt_json(b) for b in bases], "result": pt_json(result)})

    # Reference-derived relations (tests/test_msm_security.cu:908-940, core/msm.rs:1667-1694)
    add_case("empty", [], [], None)
    add_case("one_times_G", [1], [gen])
    add_case("zero_times_G", [0], [gen])
    add_case("five_times_G", [5], [gen])
    add_case("sum_i_times_G_64", list(range(1, 65)), [gen] * 64, mul(2080, gen))
    pow2 = [mul(1 << i, gen) for i in range(8)]
    add_case("ones_on_2^i_G", [1] * 8, pow2)
    add_case("all_zero_scalars", [0] * 16, [mul(pr.random_fr(g), gen) for _ in range(16)])
    P1 = mul(pr.random_fr(g), gen)
    add_case("P_plus_P", [1, 1], [P1, P1])
    add_case("P_plus_minus_P", [1, 1], [P1, neg(P1)])
    add_case("s_P_plus_s_minusP", [12345, 12345], [P1, neg(P1)])
    add_case("identity_bases", [7, 9, 11], [None, P1, None])
    add_case("r_minus_1", [pr.R - 1], [gen])
    add_case("r_minus_1_many", [pr.R - 1] * 5 + [1] * 5, [P1] * 10)
    add_case("max_digit_patterns",
             [(1 << 255) % pr.R, (1 << 254) + 1, 2 ** 16 - 1, 2 ** 15, 2 ** 15 + 1,
              (1 << 253) - 1, pr.R - 2 ** 15, 2 ** 32 - 1],
             [mul(pr.random_fr(g), gen) for _ in range(8)])
    for n in rand_sizes:
        sc = [pr.random_fr(g) for _ in range(n)]
        bs = [mul(pr.random_fr(g), gen) for _ in range(n)]
        add_case(f"random_{n}", sc, bs)
    # duplicated bases with random scalars: many equal points inside buckets
    sc = [pr.random_fr(g) for _ in range(40)]
    add_case("random_scalars_generator_bases_40", sc, [gen] * 40)
    sc = [g.randrange(1, 64) for _ in range(64)]
    add_case("small_scalars_same_base_64", sc, [P1] * 64)
    # standard-form scalars >= r: the reference's raw entry digitises all 256
    # bits (msm_kernels.cu:86-142, :648), i.e. s P = (s mod r) P; own generator, so the cases
    # above are unchanged
    g2 = pr.rng(seed ^ 0xB16)
    R = pr.R
    sc = [R, R + 1, 2 * R - 1, 2 * R, (1 << 255), (1 << 256) - 1, (1 << 256) - R, R + pr.GLV_LAMBDA,
          R + (pr.GLV_LAMBDA >> 1) + 1, R + pr.PSI_X ** 3] + [g2.randrange(R, 1 << 256) for _ in range(6)]
    bs = [mul(pr.random_fr(g2), gen) for _ in range(len(sc))]
    bs[1] = bs[0]
    add_case("noncanonical_scalars", sc, bs)
    return cases


def gen_msm_g1():
    return {"group": "g1", "cases": _msm_cases("g1", 0x5EED0013, [1, 2, 3, 5, 16, 100, 300])}


def gen_msm_g2():
    return {"group": "g2", "cases": _msm_cases("g2", 0x5EED0015, [1, 2, 3, 17, 64])}


def gen_points():
    """Point-arithmetic vectors: k*G for a handful of k (affine std), used to pin the C
    oracle's double/add/to-affine paths."""
    g = pr.rng(0x5EED0099)
    ks = [1, 2, 3, 4, 5, 7, 2080, pr.R - 1] + [pr.random_fr(g) for _ in range(8)]
    return {"k": [h(k) for k in ks],
            "g1": [pt_json(pr.g1_mul(k, pr.G1)) for k in ks],
            "g2": [pt_json(pr.g2_mul(k, pr.G2)) for k in ks]}


if __name__ == "__main__":
    dump("vecops.json", gen_vecops())
    dump("ntt.json", gen_ntt())
    dump("points.json", gen_points())
    dump("msm_g1.json", gen_msm_g1())
    dump("msm_g2.json", gen_msm_g2())
