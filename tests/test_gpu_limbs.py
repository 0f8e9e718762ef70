"""Unsaturated-limb arithmetic at its documented extremes (VERDICT r5 "what's weak" 1, item 3).

csrc/mbls_fq28.hpp (radix-2^28 Fq, the G1 accumulation) and csrc/mbls_fr29.hpp (radix-2^29 Fr,
the NTT products) accumulate product columns in one 64-bit register with no carry tracking; their
header bound tables say which limb sizes keep every column below 2^64.  Random canonical data never
drives a limb to those bounds, so the MSM / NTT parity tests cannot catch a column overflow at the
extremes.  Here every operation runs on limbs AT the maxima the formulas produce (all-MASK
normalised operands, neg<B512> of them, x4(x2(.)) operands, doubled accumulators at their
invariant bounds, 2^256 - 1 words), through tests/diag/liblimbs_diag.so (the same headers, one
operation per launch), and each result is checked against Python integers: congruence mod p / r
(Montgomery radix R' = 2^392 / 2^261) and the documented output bounds.

CPU tests (no GPU): the headers' constants (P limbs, bias tables K p with their limb minima, R'
one, -p^-1, the fold reciprocal, Fr limbs, the twiddle 2^5 factor) against Python integers."""
import ctypes
import os
import random
import re

import numpy as np
import pytest

import helpers as H
from helpers import pyref as pr

CSRC = os.path.join(H.ROOT, "midnight-bls12-381-cuda_amd", "csrc")
DIAG = os.path.join(H.ROOT, "tests", "diag", "liblimbs_diag.so")
P, R = pr.P, pr.R
M28, M29 = (1 << 28) - 1, (1 << 29) - 1
RP28 = 1 << 392  # R' of the radix-2^28 Fq
RP29 = 1 << 261  # R' of the radix-2^29 Fr


def _carray(src, name):
    m = re.search(r"\b" + name + r"\[[^\]]*\]\s*=\s*\{([^}]*)\}", src)
    assert m, name
    return [int(v.strip().rstrip("uU"), 16) for v in m.group(1).split(",") if v.strip()]


def _val(limbs, bits):
    return sum(int(v) << (bits * i) for i, v in enumerate(limbs))


def _limbs(x, bits, n):
    return [(x >> (bits * i)) & ((1 << bits) - 1) for i in range(n - 1)] + [x >> (bits * (n - 1))]


# ----------------------------------------------------------------------------- constants (CPU)
def test_fq28_constants():
    src = open(os.path.join(CSRC, "mbls_fq28.hpp")).read()
    assert _val(_carray(src, "P"), 28) == P
    assert _val(_carray(src, "ONE"), 28) == RP28 % P
    for name, lo in (("B16", M28), ("B32", 1 << 29), ("B512", 1 << 30)):
        b = _carray(src, name)
        assert _val(b, 28) % P == 0, name
        assert all(v >= lo for v in b[:-1]), name
    ninv = int(re.search(r"NINV = (0x[0-9a-f]+)u", src).group(1), 16)
    assert (P * ninv) % (1 << 28) == (1 << 28) - 1  # -p^-1 mod 2^28
    assert (P * 0xfd) % 256 == 255  # PINV8
    b512 = _carray(src, "B512")
    # the largest limb the formulas feed a product: neg<B512>(0) = B512 (< 2^30.32)
    assert max(b512).bit_length() <= 31 and max(b512) < int(2 ** 30.33)


def test_fr29_constants():
    src = open(os.path.join(CSRC, "mbls_fr29.hpp")).read()
    rl = _carray(src, "RL")
    assert _val(rl, 29) == R and rl[0] == 1 and all(v < (1 << 29) for v in rl)
    ntt = open(os.path.join(CSRC, "ntt.hip")).read()
    c32 = _val(_carray(ntt, "TW_C32"), 32)
    assert c32 == (32 << 256) % R  # 2^5 R mod r: x * C32 = x 2^5 in R-form products


# ----------------------------------------------------------------------------- the probes
# every bound test runs twice: through the limb-exact Python model (CPU: the bound table as an
# executable check, tests/limbs_model.py) and through the device code (GPU probe)
@pytest.fixture(scope="module", params=["model", pytest.param("device", marks=pytest.mark.gpu)])
def diag(request):
    if request.param == "model":
        import limbs_model
        src = open(os.path.join(CSRC, "mbls_fq28.hpp")).read()
        ninv = int(re.search(r"NINV = (0x[0-9a-f]+)u", src).group(1), 16)
        return limbs_model.Model(P, R, ninv, (1 << 40) // (0x1a011 + 1), *(_carray(src, n) for n in ("B16", "B32", "B512", "ONE")))
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    if not os.path.exists(DIAG):
        pytest.fail(f"{DIAG} not built (__graft_entry__.build())")
    L = ctypes.CDLL(DIAG)
    L.limbs_diag_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.limbs_diag_run.restype = ctypes.c_int
    iw, ow = L.limbs_diag_in_words(), L.limbs_diag_out_words()

    def run(op, cases):
        """cases: list of lists of operand limb lists (<= 5 operands of <= 16 words)"""
        a = np.zeros((len(cases), iw), dtype=np.uint32)
        for i, ops in enumerate(cases):
            for k, v in enumerate(ops):
                a[i, 16 * k:16 * k + len(v)] = v
        o = np.zeros((len(cases), ow), dtype=np.uint32)
        rc = L.limbs_diag_run(op, a.ctypes.data, o.ctypes.data, len(cases))
        assert rc == 0, rc
        return o
    return run


rng = random.Random(0x1F28)
FQ28 = open(os.path.join(CSRC, "mbls_fq28.hpp")).read()
B16, B32, B512, ONE28 = (_carray(FQ28, n) for n in ("B16", "B32", "B512", "ONE"))


def mm(a, b):  # radix-2^28 Montgomery product mod p
    return a * b * pow(RP28, -1, P) % P


def norm_max(top_bound):
    """normalised limbs at their maximum (all MASK) under a value bound: the top limb is the
    largest keeping the value < top_bound"""
    low = (1 << 364) - 1
    top = (top_bound - 1 - low) >> 364
    return [M28] * 13 + [top]


def unpack8(w):  # unpack_shift8 of canonical words w: w 2^8, normalised limbs
    return _limbs(w << 8, 28, 14)


def neg(bk, a):
    return [b - x for b, x in zip(bk, a)]


def x2(a):
    return [v << 1 for v in a]


def is_normalised(l):
    return all(v <= M28 for v in l[:-1])


def fq28_operand_pairs():
    """(a, b) limb pairs at the extremes the formulas produce (header: A + B <= 60.1)"""
    mx = [M28] * 14  # all-MASK normalised: value ~2^392
    q_hi = unpack8(P - 1)  # the largest unpacked base coordinate (< 256 p)
    y_neg0 = neg(B512, [0] * 14)  # neg<B512>(0): limbs = B512, up to 2^30.32
    y_negq = neg(B512, q_hi)
    z_max = x2(norm_max(4 * P))  # acc.z = x2(H), H folded: limbs < 2^29
    x4x2 = [v << 3 for v in norm_max(P)]  # dbl: x4(x2(B)) against B (limbs < 2^31)
    e3 = [3 * v for v in norm_max(P)]  # dbl: E = 3A (limbs < 3 2^28)
    pairs = [(mx, mx), (y_neg0, z_max), (y_negq, z_max), (y_neg0, mx), (x4x2, mx), (e3, e3), (q_hi, z_max),
             (mx, z_max)]
    for _ in range(24):  # random unpacked coordinates (< 256 p), negated
        a = unpack8(rng.randrange(P))
        pairs.append((neg(B512, a), z_max))
    return pairs


def test_fq28_products_at_limb_extremes(diag):
    pairs = fq28_operand_pairs()
    o = diag(0, [[a, b] for a, b in pairs])
    for i, (a, b) in enumerate(pairs):
        r = [int(v) for v in o[i, :14]]
        assert _val(r, 28) % P == mm(_val(a, 28), _val(b, 28)), ("mul", i)
        assert is_normalised(r), ("mul normalised", i)
    # squares: operands whose doubled cross terms are the largest the formulas square
    # (header: 7 doubled cross terms + the diagonal + 14 reduction terms < 2^64 for limbs < 2^30)
    sq = [[M28] * 14, x2(norm_max(4 * P)), [3 * v for v in norm_max(P)], [M28 + b for b in B16],
          x2(x2(norm_max(P))), [3 * M28] * 13 + [1 << 16]]
    assert all(max(a) < (1 << 30) for a in sq)
    o = diag(1, [[a] for a in sq])
    for i, a in enumerate(sq):
        r = [int(v) for v in o[i, :14]]
        assert _val(r, 28) % P == mm(_val(a, 28), _val(a, 28)), ("sqr", i)
        assert is_normalised(r)
    # mul2 (the lazy Y3): R2 (carried) x (V - X3 against B16) + neg<B32>(x2(y)) x J
    quads = []
    for _ in range(16):
        r2 = [rng.randrange(1 << 28) for _ in range(13)] + [rng.randrange(1 << 12)]
        v_x3 = [bv + rng.randrange(1 << 28) for bv in B16]
        ny = neg(B32, x2(norm_max(3 * P)))
        j = norm_max(2 * P)
        quads.append([r2, v_x3, ny, j])
    quads.append([[M28] * 13 + [1 << 14], [b + M28 for b in B16], neg(B32, x2([M28] * 13 + [0])), [M28] * 14])
    o = diag(2, quads)
    for i, (a, b, c, d) in enumerate(quads):
        r = [int(v) for v in o[i, :14]]
        exp = (_val(a, 28) * _val(b, 28) + _val(c, 28) * _val(d, 28)) * pow(RP28, -1, P) % P
        assert _val(r, 28) % P == exp, ("mul2", i)
        assert is_normalised(r)


def test_fq28_fold_and_words_at_limb_extremes(diag):
    """fold takes limbs < 2^32 (no uint32 wrap) and values < 2^391: the largest is mmadd's
    sub<B512>(neg<B512>(qy), acc.y) (limbs ~2^31.3); its output is normalised, < 3p"""
    cases = [neg(B512, [0] * 14), [a + b for a, b in zip(neg(B512, [0] * 14), B512)],
             [a + b - c for a, b, c in zip(neg(B512, [0] * 14), B512, norm_max(3 * P))]]
    cases += [[rng.randrange(1 << 31) for _ in range(13)] + [rng.randrange(1 << 14)] for _ in range(32)]
    for c in cases:
        assert max(c) < (1 << 32) and _val(c, 28) < (1 << 391)
    o = diag(3, [[c] for c in cases])
    for i, c in enumerate(cases):
        r = [int(v) for v in o[i, :14]]
        assert _val(r, 28) % P == _val(c, 28) % P, ("fold", i)
        assert is_normalised(r) and _val(r, 28) < 3 * P, ("fold bound", i, _val(r, 28) / P)
    o = diag(4, [[c] for c in cases])
    for i, c in enumerate(cases):
        w = _val([int(v) for v in o[i, :12]], 32)
        assert w == _val(c, 28) * pow(1 << 8, -1, P) % P, ("to_words", i)  # x R' -> canonical x R


def madd_ref(X, Y, Z, x2v, y2v):
    """r28::madd's field values (madd-2007-bl, lazy Y3, Z3 = 2 Z1 H), mod p; None: infinity"""
    if Z % P == 0 and Z == 0:
        return x2v % P, y2v % P, RP28 % P
    ZZ = mm(Z, Z)
    H = (mm(x2v, ZZ) - X) % P
    Rr = (mm(mm(y2v, Z), ZZ) - Y) % P
    if mm(H, H) == 0:
        if Rr == 0:
            A, B = mm(X, X), mm(Y, Y)
            E, D, C8 = 3 * A, mm(4 * X, B), mm(8 * B, B)
            X3 = (mm(E, E) - 2 * D) % P
            return X3, (mm(E, D - X3) - C8) % P, mm(2 * Y, Z)
        return None
    I = 4 * mm(H, H)
    J, V, R2 = mm(H, I), mm(X, I), 2 * Rr
    X3 = (mm(R2, R2) - J - 2 * V) % P
    Y3 = (R2 * (V - X3) - 2 * Y * J) * pow(RP28, -1, P) % P
    return X3, Y3, mm(2 * Z, H)


def test_fq28_madd_mmadd_at_bounds(diag):
    """the accumulation's mixed additions with the accumulator AT its invariant bounds (x, y
    normalised < 3p, z limbs < 2^29) and the base at the unpack / neg<B512> extremes, including
    the exceptional H = 0 branches (doubling, infinity)"""
    cases = []
    xs = [norm_max(3 * P), _limbs(3 * P - 1, 28, 14), _limbs(P, 28, 14)]
    zs = [x2(norm_max(4 * P)), _limbs(7 * P, 28, 14)]
    qxs = [unpack8(P - 1), unpack8(rng.randrange(P))]
    for X in xs:
        for Y in xs:
            for Z in zs:
                for qx in qxs:
                    for qy in (unpack8(P - 1), neg(B512, [0] * 14), neg(B512, unpack8(P - 1))):
                        cases.append([X, Y, Z, qx, qy])
    # H = 0: the accumulator holds the base (another representative): doubling, and its negation
    Z = x2(norm_max(4 * P))
    for qx, qy in ((unpack8(P - 1), unpack8(5)), (unpack8(12345), neg(B512, [0] * 14))):
        zv = _val(Z, 28)
        Xv = mm(_val(qx, 28), mm(zv, zv))
        Yv = mm(mm(_val(qy, 28), zv), mm(zv, zv))
        cases.append([_limbs(Xv + P, 28, 14), _limbs(Yv + 2 * P, 28, 14), Z, qx, qy])      # equal: doubling
        cases.append([_limbs(Xv, 28, 14), _limbs((P - Yv) % P, 28, 14), Z, qx, qy])      # opposite: infinity
    o = diag(7, cases)
    for i, (X, Y, Z, qx, qy) in enumerate(cases):
        exp = madd_ref(_val(X, 28), _val(Y, 28), _val(Z, 28), _val(qx, 28), _val(qy, 28))
        rx, ry, rz = ([int(v) for v in o[i, 14 * k:14 * k + 14]] for k in range(3))
        if exp is None:
            assert all(v == 0 for v in rz), ("madd infinity", i)
            continue
        assert (_val(rx, 28) % P, _val(ry, 28) % P, _val(rz, 28) % P) == exp, ("madd", i)
        assert is_normalised(rx) and is_normalised(ry) and _val(rx, 28) < 3 * P and _val(ry, 28) < 3 * P, i
        assert all(v < (1 << 29) for v in rz[:-1]) and _val(rz, 28) < 8 * P, ("z bound", i)
    # mmadd: the chunk's first point folded into acc (z = R'), the second point at the extremes
    mc = []
    for X in xs:
        for Y in xs:
            for qx in qxs:
                for qy in (unpack8(P - 1), neg(B512, [0] * 14), neg(B512, unpack8(P - 1))):
                    mc.append([X, Y, [0] * 14, qx, qy])
    mc.append([_limbs(_val(unpack8(77), 28) % P + P, 28, 14), xs[0], [0] * 14, unpack8(77), unpack8(9)])  # x1 = x2
    o = diag(8, mc)
    one = RP28 % P
    for i, (X, Y, _, qx, qy) in enumerate(mc):
        done = int(o[i, 42])
        exp = madd_ref(_val(X, 28), _val(Y, 28), one, _val(qx, 28), _val(qy, 28))
        if (_val(qx, 28) - _val(X, 28)) % P == 0:
            assert done == 0, ("mmadd must refuse x1 == x2", i)
            continue
        assert done == 1
        rx, ry, rz = ([int(v) for v in o[i, 14 * k:14 * k + 14]] for k in range(3))
        assert (_val(rx, 28) % P, _val(ry, 28) % P, _val(rz, 28) % P) == exp, ("mmadd", i)
        assert is_normalised(rx) and is_normalised(ry) and _val(rx, 28) < 3 * P and _val(ry, 28) < 3 * P, i
        assert all(v < (1 << 29) for v in rz[:-1]) and _val(rz, 28) < 8 * P, ("mmadd z bound", i)


# ----------------------------------------------------------------------------- radix 2^29 Fr
def mm29(a, b):
    return a * b * pow(RP29, -1, R) % R


def test_fr29_products_at_extremes(diag):
    """the NTT products: any 256-bit word operand (lazy values < 2r, and 2^256 - 1 as the column
    bound's worst case) against canonical twiddles up to r - 1; output normalised, < 2^256 and
    < 2r when the operand is < 2r (mbls_fr29.hpp bounds)"""
    words = [(1 << 256) - 1, 2 * R - 1, R, R - 1, 0, 1] + [rng.randrange(2 * R) for _ in range(40)]
    tw = [R - 1, R - 2, (1 << 254), 1] + [rng.randrange(R) for _ in range(40)]
    cases = [(x, w) for x in words[:6] for w in tw[:4]] + list(zip(words[6:], tw[4:]))
    # unpack / pack round trip
    o = diag(21, [[_limbs(x, 32, 8)] for x, _ in cases])
    for i, (x, _) in enumerate(cases):
        l = [int(v) for v in o[i, :9]]
        assert _val(l, 29) == x and all(v <= M29 for v in l[:-1]), ("unpack", i)
    o = diag(22, [[_limbs(x, 29, 9)] for x, _ in cases])
    for i, (x, _) in enumerate(cases):
        assert _val([int(v) for v in o[i, :8]], 32) == x, ("pack", i)
    # limb products
    o = diag(20, [[_limbs(x, 29, 9), _limbs(w, 29, 9)] for x, w in cases])
    for i, (x, w) in enumerate(cases):
        l = [int(v) for v in o[i, :9]]
        v = _val(l, 29)
        assert v % R == mm29(x, w), ("mul", i)
        assert all(t <= M29 for t in l[:-1]) and v < (1 << 256), ("mul bound", i)
        if x < 2 * R:
            assert v < 2 * R, ("lazy bound", i)
    # the butterflies' form: words in, words out
    o = diag(23, [[_limbs(x, 32, 8), _limbs(w, 29, 9)] for x, w in cases if x < 2 * R])
    for i, (x, w) in enumerate([c for c in cases if c[0] < 2 * R]):
        v = _val([int(t) for t in o[i, :8]], 32)
        assert v % R == mm29(x, w) and v < 2 * R, ("mul_words", i)


def test_model_detects_overflow():
    """negative control: the model's checks fire past the bounds (limbs beyond the table)"""
    import limbs_model
    F = limbs_model.Fq28(P, 0xffcfffd, (1 << 40) // (0x1a011 + 1))
    with pytest.raises(limbs_model.Overflow):
        F.mul([1 << 31] * 14, [1 << 31] * 14)  # A + B = 62 > 60.1
    with pytest.raises(limbs_model.Overflow):
        F.sqr([1 << 31] * 14)  # 2A + 1 > 60
    G = limbs_model.Fr29(R)
    with pytest.raises(limbs_model.Overflow):
        G.mul([(1 << 32) - 1] * 9, [(1 << 32) - 1] * 9)


# ----------------------------------------------------------------------------- pair-sliced Fq2 (G2)
def _fq2_ops():
    inv = pow(RP28, -1, P)

    def mm2(a, b):  # Fq2 Montgomery product (radix R' = 2^392), u^2 = -1
        return ((a[0] * b[0] - a[1] * b[1]) * inv % P, (a[0] * b[1] + a[1] * b[0]) * inv % P)

    def lin(*terms):  # sum of k * a over (k, a)
        return tuple(sum(k * a[j] for k, a in terms) % P for j in range(2))
    return mm2, lin


def madd2_ref(X, Y, Z, x2v, y2v):
    """jac_madd's Fq2 field values (madd-2007-bl, lazy Y3, Z3 = 2 Z1 H); None: H = 0"""
    mm2, lin = _fq2_ops()
    ZZ = mm2(Z, Z)
    H = lin((1, mm2(x2v, ZZ)), (-1, X))
    Rr = lin((1, mm2(mm2(y2v, Z), ZZ)), (-1, Y))
    if H == (0, 0):
        return None
    I = lin((4, mm2(H, H)))
    J, V, R2 = mm2(H, I), mm2(X, I), lin((2, Rr))
    X3 = lin((1, mm2(R2, R2)), (-1, J), (-2, V))
    Y3 = lin((1, mm2(R2, lin((1, V), (-1, X3)))), (-2, mm2(Y, J)))
    return X3, Y3, mm2(lin((2, Z)), H)


def _v2(a):
    return (_val(a[0], 28) % P, _val(a[1], 28) % P)


def fq2_madd_cases():
    """accumulators at their invariant bounds (x, y normalised < 3p, z normalised), bases at the
    unpack extremes with the negated y carried (the kernel's form), per component"""
    import limbs_model
    F = limbs_model.Fq28(P, 0xffcfffd, (1 << 40) // (0x1a011 + 1))
    xs = [norm_max(3 * P), _limbs(3 * P - 1, 28, 14), _limbs(P, 28, 14), _limbs(rng.randrange(3 * P), 28, 14)]
    zs = [norm_max(6 * P), _limbs(2 * P - 1, 28, 14), _limbs(rng.randrange(6 * P), 28, 14)]
    q = [unpack8(P - 1), unpack8(0), unpack8(rng.randrange(P))]
    cases = []
    for k in range(48):
        X = (xs[k % 4], xs[(k // 4) % 4])
        Y = (xs[(k + 1) % 4], xs[(k // 2) % 4])
        Z = (zs[k % 3], zs[(k // 3) % 3])
        qx = (q[k % 3], q[(k + 1) % 3])
        qy = (q[(k // 3) % 3], q[(k + 2) % 3])
        if k % 2:  # negative digit: y2 = carry(neg<B512>(qy)) per component
            qy = tuple(F.carry(F.neg(B512, c)) for c in qy)
        cases.append((X, Y, Z, qx, qy))
    return cases


def test_fq2_pair_madd_model():
    """the pair-sliced radix-2^28 G2 mixed additions (tests/limbs_model.py _fq2_formulas, what
    csrc/mbls_fq2_28.hpp computes): no column reaches 2^64, every coordinate equals jac_madd's
    field value, outputs keep the accumulator invariant"""
    import limbs_model
    src = open(os.path.join(CSRC, "mbls_fq28.hpp")).read()
    F = limbs_model.Fq28(P, 0xffcfffd, (1 << 40) // (0x1a011 + 1))
    madd, mmadd = limbs_model._fq2_formulas(F, B16, B32, B512, _carray(src, "ONE"))
    for i, (X, Y, Z, qx, qy) in enumerate(fq2_madd_cases()):
        r = madd((X, Y, Z), qx, qy)
        exp = madd2_ref(_v2(X), _v2(Y), _v2(Z), _v2(qx), _v2(qy))
        assert (r is None) == (exp is None), i
        if r is None:
            continue
        assert tuple(_v2(c) for c in r) == exp, ("g2 madd", i)
        for c in r[0] + r[1] + r[2]:
            assert is_normalised(c)
        assert all(_val(c, 28) < 3 * P for c in r[0] + r[1]) and all(_val(c, 28) < 6 * P for c in r[2])
        one = (RP28 % P, 0)
        r = mmadd((X, Y, None), qx, qy)
        exp = madd2_ref(_v2(X), _v2(Y), one, _v2(qx), _v2(qy))
        assert tuple(_v2(c) for c in r) == exp, ("g2 mmadd", i)
        for c in r[0] + r[1] + r[2]:
            assert is_normalised(c)
        assert all(_val(c, 28) < 3 * P for c in r[0] + r[1]) and all(_val(c, 28) < 6 * P for c in r[2])


@pytest.mark.gpu
def test_fq2_pair_madd_device(diag):
    """the device's pair-sliced G2 madd / mmadd (csrc/mbls_fq2_28.hpp) on the model's cases:
    every coordinate equals jac_madd's field value and the model's limbs, bit for bit"""
    import limbs_model
    if isinstance(diag, limbs_model.Model):
        pytest.skip("the model side of these formulas is test_fq2_pair_madd_model")
    src = open(os.path.join(CSRC, "mbls_fq28.hpp")).read()
    F = limbs_model.Fq28(P, 0xffcfffd, (1 << 40) // (0x1a011 + 1))
    madd, mmadd = limbs_model._fq2_formulas(F, B16, B32, B512, _carray(src, "ONE"))
    cases = fq2_madd_cases()
    # the exceptional H = 0 case: acc = q with another representative (the caller's word path)
    X, Y, Z, qx, qy = cases[0]
    cases.append(((unpack8(5), unpack8(7)), Y, ([int(v) for v in ONE28], [0] * 14), (unpack8(5), unpack8(7)), qy))
    for op, fn in ((30, madd), (31, mmadd)):
        rows = []
        for X, Y, Z, qx, qy in cases:
            for j in range(2):
                rows.append([X[j], Y[j], Z[j], qx[j], qy[j]])
        o = diag(op, rows)
        for i, (X, Y, Z, qx, qy) in enumerate(cases):
            exp = fn((X, Y, Z), qx, qy)
            done = int(o[2 * i, 42])
            assert done == int(o[2 * i + 1, 42]) == (0 if exp is None else 1), (op, i)
            if exp is None:
                continue
            for k in range(3):
                for j in range(2):
                    got = [int(v) for v in o[2 * i + j, 14 * k:14 * k + 14]]
                    assert got == exp[k][j], (op, i, k, j)


# ----------------------------------------------------------------------------- XYZZ (round 6)
def _aff_of_xyzz(X, Y, ZZ, ZZZ):
    """plain affine point of an XYZZ quadruple of R'-form values (R' cancels in X / ZZ, Y / ZZZ)"""
    if ZZ % P == 0:
        return None
    return (X * pow(ZZ, -1, P) % P, Y * pow(ZZZ, -1, P) % P)


def _aff_of_jac(X, Y, Z):
    """plain affine point of R'-form Jacobian values"""
    if Z % P == 0:
        return None
    zi = pow(Z, -1, P)
    # R'-form values: x = (X R'^-1) / (Z R'^-1)^2 = X R' / Z^2
    return (X * RP28 * zi * zi % P, Y * RP28 * RP28 * zi * zi * zi % P)


def _rp(v):  # a field value into R'-form
    return v * RP28 % P


def _xyzz_of(pt, z, bump=0):
    """pt (affine, plain) as XYZZ limbs with the implicit Z = z, R'-form, each coordinate lifted by
    `bump` multiples of p (inside the < 3p invariant)"""
    x, y = pt
    vals = (x * z * z % P, y * z * z * z % P, z * z % P, z * z * z % P)
    return [_limbs(_rp(v) + bump * P, 28, 14) for v in vals]


def _q_unpacked(pt, negate):
    """a base as the accumulation sees it: unpack_shift8 of its canonical Montgomery words
    (x R' < 256 p); a negative digit takes y through neg<B512>"""
    x, y = pt
    qx, qy = unpack8(x * (1 << 384) % P), unpack8(y * (1 << 384) % P)
    return qx, (neg(B512, qy) if negate else qy)


def xyzz_cases():
    """(acc, q, negate) on real G1 points: generic sums, the accumulator's coordinates lifted to their
    invariant bounds, equal points (doubling), opposite points (infinity), an infinite accumulator"""
    pts = [pr.g1_mul(k, pr.G1) for k in (1, 2, 3, 5, 1234567, 2 ** 200 + 7, pr.R - 1, 0xdeadbeef)]
    cases = []
    for i, a in enumerate(pts):
        for j, b in enumerate(pts):
            if i == j:
                continue
            z = rng.randrange(1, P)
            cases.append((_xyzz_of(a, z, bump=(i + j) % 3), b, (i * j) % 2 == 1))
    for k, a in enumerate(pts[:4]):
        z = rng.randrange(1, P)
        cases.append((_xyzz_of(a, z, bump=k % 3), a, False))   # equal: doubling
        cases.append((_xyzz_of(a, z, bump=2), a, True))         # -a: infinity
    cases.append(([list(ONE28), list(ONE28), [0] * 14, [0] * 14], pts[3], False))  # infinite accumulator
    return cases


def _check_xyzz_out(out, want, what):
    rx, ry, rzz, rzzz = ([int(v) for v in out[14 * k:14 * k + 14]] for k in range(4))
    got = _aff_of_xyzz(*(_val(c, 28) for c in (rx, ry, rzz, rzzz)))
    assert got == want, what
    if want is not None:
        for c in (rx, ry, rzz, rzzz):
            assert is_normalised(c) and _val(c, 28) < 3 * P, (what, "invariant")


def test_xyzz_madd_mmadd_on_curve(diag):
    """r28::xmadd / xmmadd (the G1 accumulation, round 6) on real points: the affine result equals
    pyref's group law, including doubling / infinity on the exceptional branch, and the outputs
    keep the accumulator invariant (normalised, < 3p); device and model alike"""
    cases = xyzz_cases()
    rows = []
    for acc, b, ng in cases:
        qx, qy = _q_unpacked(b, ng)
        rows.append(acc + [qx, qy])
    o = diag(9, rows)
    for i, (acc, b, ng) in enumerate(cases):
        a = _aff_of_xyzz(*(_val(c, 28) for c in acc))
        bb = pr.g1_neg(b) if ng else b
        _check_xyzz_out(o[i], bb if a is None else pr.g1_add(a, bb), ("xmadd", i))
    # mmadd: the chunk's first point folded into acc (zz = zzz = R'-one)
    mrows, mw = [], []
    for acc, b, ng in cases[:-1]:
        a = _aff_of_xyzz(*(_val(c, 28) for c in acc))
        if a is None:
            continue
        x1, y1 = _limbs(_rp(a[0]) + P, 28, 14), _limbs(_rp(a[1]) + 2 * P, 28, 14)  # folded: < 3p
        qx, qy = _q_unpacked(b, ng)
        mrows.append([x1, y1, [0] * 14, [0] * 14, qx, qy])
        mw.append((a, pr.g1_neg(b) if ng else b))
    o = diag(10, mrows)
    for i, (ap, bb) in enumerate(mw):
        if ap[0] == bb[0]:
            assert int(o[i, 56]) == 0, ("xmmadd must refuse x1 == x2", i)
            continue
        assert int(o[i, 56]) == 1
        _check_xyzz_out(o[i], pr.g1_add(ap, bb), ("xmmadd", i))


def test_xyzz_add_dbl_to_jac_on_curve(diag):
    """r28::xadd (bucket sums of XYZZ partials), xdbl and x_to_jac on real points against pyref"""
    pts = [pr.g1_mul(k, pr.G1) for k in (1, 2, 7, 99991, 2 ** 130 + 3, pr.R - 2)]
    rows, want = [], []
    for i, a in enumerate(pts):
        for j, b in enumerate(pts):
            za, zb = rng.randrange(1, P), rng.randrange(1, P)
            acc = _xyzz_of(a, za, bump=(i + j) % 3)
            # the partial as stored (canonical words) and unpacked: w 2^8 = v R'
            part = [unpack8(_val(c, 28) % P * pow(1 << 8, -1, P) % P) for c in _xyzz_of(b, zb)]
            rows.append(acc + part)
            want.append(pr.g1_add(a, b))
        za = rng.randrange(1, P)
        rows.append(_xyzz_of(a, za, bump=1) + [unpack8(_val(c, 28) % P * pow(1 << 8, -1, P) % P)
                                               for c in _xyzz_of(pr.g1_neg(a), rng.randrange(1, P))])
        want.append(None)  # a + (-a)
    o = diag(11, rows)
    for i, w in enumerate(want):
        _check_xyzz_out(o[i], w, ("xadd", i))
    drows = [_xyzz_of(a, rng.randrange(1, P), bump=k % 3) for k, a in enumerate(pts)]
    o = diag(12, drows)
    for i, a in enumerate(pts):
        _check_xyzz_out(o[i], pr.g1_add(a, a), ("xdbl", i))
    o = diag(13, drows)
    for i, a in enumerate(pts):
        rx, ry, rz = ([int(v) for v in o[i, 14 * k:14 * k + 14]] for k in range(3))
        assert _aff_of_jac(_val(rx, 28), _val(ry, 28), _val(rz, 28)) == a, ("x_to_jac", i)
        assert all(v < (1 << 29) for v in rz[:-1]) and _val(rz, 28) < 8 * P  # J28's z invariant


def xyzz_extreme_rows():
    """limbs at the maxima the XYZZ formulas take (not curve points): accumulators at the invariant
    bounds (all-MASK < 3p, 3p - 1, p), bases at the unpack / neg<B512> extremes"""
    xs = [norm_max(3 * P), _limbs(3 * P - 1, 28, 14), _limbs(P, 28, 14)]
    q = [unpack8(P - 1), unpack8(rng.randrange(P))]
    rows9, rows11 = [], []
    for k in range(27):
        acc = [xs[k % 3], xs[(k // 3) % 3], xs[(k // 9) % 3], xs[(k + 1) % 3]]
        qy = (unpack8(P - 1), neg(B512, [0] * 14), neg(B512, unpack8(P - 1)))[k % 3]
        rows9.append(acc + [q[k % 2], qy])
        rows11.append(acc + [unpack8(P - 1), q[k % 2], unpack8(P - 1), q[(k + 1) % 2]])
    return rows9, rows11


def test_xyzz_columns_at_limb_extremes(diag):
    """the XYZZ formulas on limbs at their maxima: the model raises if any column reaches 2^64;
    the device's limbs equal the model's bit for bit"""
    import limbs_model
    src = open(os.path.join(CSRC, "mbls_fq28.hpp")).read()
    ninv = int(re.search(r"NINV = (0x[0-9a-f]+)u", src).group(1), 16)
    M = limbs_model.Model(P, R, ninv, (1 << 40) // (0x1a011 + 1), B16, B32, B512, ONE28)
    rows9, rows11 = xyzz_extreme_rows()
    for op, rows in ((9, rows9), (10, rows9), (11, rows11), (12, rows9), (13, rows9)):
        exp = M(op, rows)  # raises limbs_model.Overflow past a bound
        got = diag(op, rows)
        assert np.array_equal(np.asarray(got, dtype=np.uint64)[:, :57], exp[:, :57]), op


# ----------------------------------------------------------------------------- pair-sliced XYZZ (G2)
def _f2_rp(v):
    return (v[0] * RP28 % P, v[1] * RP28 % P)


def _xyzz2_of(pt, z, bump=0):
    """G2 pt (affine, plain Fq2) as pair XYZZ limbs with the implicit Z = z: 4 tuples (c0, c1)"""
    x, y = pt
    z2 = pr.f2_mul(z, z)
    z3 = pr.f2_mul(z2, z)
    vals = (pr.f2_mul(x, z2), pr.f2_mul(y, z3), z2, z3)
    return [tuple(_limbs(c + bump * P, 28, 14) for c in _f2_rp(v)) for v in vals]


def _aff2(X, Y, ZZ, ZZZ):
    """plain affine of pair XYZZ component values (R' cancels)"""
    if ZZ[0] % P == 0 and ZZ[1] % P == 0:
        return None
    return (pr.f2_mul(X, pr.f2_inv(ZZ)), pr.f2_mul(Y, pr.f2_inv(ZZZ)))


def _v2l(c):  # a pair of component limb lists -> component values
    return (_val(c[0], 28), _val(c[1], 28))


def _q2_unpacked(pt, negate):
    """a G2 base as k_accumulate_r28p sees it: per component unpack_shift8 of the canonical
    words; a negative digit: carry(neg<B512>(.)) per component"""
    import limbs_model
    F = limbs_model.Fq28(P, 0xffcfffd, (1 << 40) // (0x1a011 + 1))
    x, y = pt
    qx = tuple(unpack8(c * (1 << 384) % P) for c in x)
    qy = tuple(unpack8(c * (1 << 384) % P) for c in y)
    if negate:
        qy = tuple(F.carry(F.neg(B512, c)) for c in qy)
    return qx, qy


def xyzz2_cases():
    rz = lambda: (rng.randrange(P), rng.randrange(P))  # noqa: E731
    pts = [pr.g2_mul(k, pr.G2) for k in (1, 2, 3, 77, 2 ** 100 + 9, pr.R - 1)]
    cases = []
    for i, a in enumerate(pts):
        for j, b in enumerate(pts):
            if i != j:
                cases.append((_xyzz2_of(a, rz(), bump=(i + j) % 3), b, (i + j) % 2 == 1))
    for k, a in enumerate(pts[:3]):
        z = rz()
        cases.append((_xyzz2_of(a, z, bump=k % 3), a, False))  # doubling
        cases.append((_xyzz2_of(a, z, bump=1), a, True))        # infinity
    return pts, cases


def _check_xyzz2(out_pair, want, what):
    """out_pair: (lane-0 limbs, lane-1 limbs) of the 4 coordinates"""
    cs = [(out_pair[0][k], out_pair[1][k]) for k in range(4)]
    got = _aff2(*(_v2l(c) for c in cs))
    assert got == want, what
    if want is not None:
        for c in cs:
            for comp in c:
                assert is_normalised(comp) and _val(comp, 28) < 3 * P, (what, "invariant")


def _pair_model():
    import limbs_model
    F = limbs_model.Fq28(P, 0xffcfffd, (1 << 40) // (0x1a011 + 1))
    return limbs_model._fq2_xyzz_formulas(F, B16, B32, B512, ONE28)


def _run_pair(diag, op, rows_per_case):
    """device pair op: each case is a list of operand pairs (c0, c1); returns per case the 4 (or 3)
    coordinates as (lane-0 list, lane-1 list) plus the flag"""
    rows = []
    for ops in rows_per_case:
        for j in range(2):
            rows.append([o[j] for o in ops])
    o = diag(op, rows)
    res = []
    for i in range(len(rows_per_case)):
        lanes = [[[int(v) for v in o[2 * i + j, 14 * k:14 * k + 14]] for k in range(4)] for j in range(2)]
        res.append((lanes, int(o[2 * i, 56]), int(o[2 * i + 1, 56])))
    return res


def test_xyzz2_pair_on_curve_model():
    """the pair-sliced XYZZ forms (tests/limbs_model.py _fq2_xyzz_formulas = csrc/mbls_fq2_28.hpp)
    on real G2 points: affine results equal pyref's group law; no column reaches 2^64"""
    xdbl, xmadd, xmmadd, xadd, x_to_jac = _pair_model()
    pts, cases = xyzz2_cases()
    for i, (acc, b, ng) in enumerate(cases):
        qx, qy = _q2_unpacked(b, ng)
        r = xmadd(tuple(acc), qx, qy)
        a = _aff2(*(_v2l(c) for c in acc))
        bb = pr.g2_neg(b) if ng else b
        want = pr.g2_add(a, bb)
        got = _aff2(*(_v2l(c) for c in r))
        assert got == want, ("g2 xmadd", i)
        if a is not None and a[0] != bb[0]:
            x1 = tuple(_limbs(c + P, 28, 14) for c in _f2_rp(a[0]))
            y1 = tuple(_limbs(c + 2 * P, 28, 14) for c in _f2_rp(a[1]))
            r = xmmadd((x1, y1, None, None), qx, qy)
            assert _aff2(*(_v2l(c) for c in r)) == want, ("g2 xmmadd", i)
    for i, a in enumerate(pts):
        for j, b in enumerate(pts):
            r = xadd(tuple(_xyzz2_of(a, (rng.randrange(P), 5), bump=1)), *_xyzz2_of(b, (3, rng.randrange(P))))
            assert _aff2(*(_v2l(c) for c in r)) == pr.g2_add(a, b), ("g2 xadd", i, j)
        acc = tuple(_xyzz2_of(a, (rng.randrange(P), rng.randrange(P)), bump=2))
        assert _aff2(*(_v2l(c) for c in xdbl(acc))) == pr.g2_add(a, a), ("g2 xdbl", i)
        X, Y, Z = (_v2l(c) for c in x_to_jac(acc))
        zi = pr.f2_inv(Z)
        zi2 = pr.f2_mul(zi, zi)
        # R'-form Jacobian: x = X R' / Z^2, y = Y R'^2 / Z^3
        xa = pr.f2_mul(pr.f2_mul(X, zi2), (RP28 % P, 0))
        ya = pr.f2_mul(pr.f2_mul(pr.f2_mul(Y, zi2), zi), (RP28 * RP28 % P, 0))
        assert (xa, ya) == a, ("g2 x_to_jac", i)


@pytest.mark.gpu
def test_xyzz2_pair_device(diag):
    """the device's pair-sliced XYZZ forms equal the model's limbs bit for bit, on G2 curve cases
    and on accumulators at their invariant bounds (limb extremes)"""
    import limbs_model
    if isinstance(diag, limbs_model.Model):
        pytest.skip("the model side is test_xyzz2_pair_on_curve_model")
    xdbl, xmadd, xmmadd, xadd, x_to_jac = _pair_model()
    pts, cases = xyzz2_cases()
    ext = [norm_max(3 * P), _limbs(3 * P - 1, 28, 14), _limbs(P, 28, 14)]
    rows9, exp9 = [], []
    for acc, b, ng in cases:
        qx, qy = _q2_unpacked(b, ng)
        rows9.append(list(acc) + [qx, qy])
    for k in range(9):  # extremes: every coordinate at an invariant bound, bases at the unpack maximum
        acc = [(ext[k % 3], ext[(k + 1) % 3]), (ext[(k // 3) % 3], ext[k % 3]), (ext[(k + 2) % 3], ext[k % 3]),
               (ext[(k // 3) % 3], ext[(k + 1) % 3])]
        qx, qy = (unpack8(P - 1), unpack8(P - 1)), (unpack8(P - 1), unpack8(rng.randrange(P)))
        rows9.append(acc + [qx, qy])
    for ops in rows9:
        exp9.append(xmadd(tuple(ops[:4]), ops[4], ops[5]))
    for i, (lanes, _, _) in enumerate(_run_pair(diag, 32, rows9)):
        for k in range(4):
            assert (lanes[0][k], lanes[1][k]) == tuple(exp9[i][k]), ("xmadd", i, k)
    rows11 = [list(_xyzz2_of(a, (rng.randrange(P), 7), bump=1)) + list(_xyzz2_of(b, (5, rng.randrange(P))))
              for a in pts for b in pts]
    for i, (lanes, _, _) in enumerate(_run_pair(diag, 34, rows11)):
        exp = xadd(tuple(rows11[i][:4]), *rows11[i][4:])
        for k in range(4):
            assert (lanes[0][k], lanes[1][k]) == tuple(exp[k]), ("xadd", i, k)
    rows12 = [list(_xyzz2_of(a, (rng.randrange(P), rng.randrange(P)), bump=k % 3)) for k, a in enumerate(pts)]
    for i, (lanes, _, _) in enumerate(_run_pair(diag, 35, rows12)):
        exp = xdbl(tuple(rows12[i]))
        for k in range(4):
            assert (lanes[0][k], lanes[1][k]) == tuple(exp[k]), ("xdbl", i, k)
    for i, (lanes, _, _) in enumerate(_run_pair(diag, 36, rows12)):
        exp = x_to_jac(tuple(rows12[i]))
        for k in range(3):
            assert (lanes[0][k], lanes[1][k]) == tuple(exp[k]), ("x_to_jac", i, k)
    # mmadd: acc = (x1, y1) folded, zz = zzz = one (set by the op)
    rows10 = []
    for acc, b, ng in cases:
        a = _aff2(*(_v2l(c) for c in acc))
        if a is None:
            continue
        x1 = tuple(_limbs(c + P, 28, 14) for c in _f2_rp(a[0]))
        y1 = tuple(_limbs(c + 2 * P, 28, 14) for c in _f2_rp(a[1]))
        qx, qy = _q2_unpacked(b, ng)
        rows10.append([x1, y1, ([0] * 14, [0] * 14), ([0] * 14, [0] * 14), qx, qy])
    for i, (lanes, f0, f1) in enumerate(_run_pair(diag, 33, rows10)):
        exp = xmmadd((rows10[i][0], rows10[i][1], None, None), rows10[i][4], rows10[i][5])
        assert f0 == f1 == (0 if exp is None else 1), ("xmmadd flag", i)
        if exp is None:
            continue
        for k in range(4):
            assert (lanes[0][k], lanes[1][k]) == tuple(exp[k]), ("xmmadd", i, k)
