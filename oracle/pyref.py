"""Pure-Python big-integer restatement of BLS12-381 (TEST INFRASTRUCTURE ONLY).

This module is part of the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may use anything under ``oracle/``; the product
path (``midnight-bls12-381-cuda_amd/``) never imports it.

It is an independent restatement of the *mathematics* the reference relies on, written
from the BLS12-381 specification, and is used for small cases and to generate the golden
fixtures under ``tests/golden/``.  Everything is plain Python ``int`` arithmetic:

* Fr / Fq constants -- reference ``bls12-381/include/bls12_381_constants.h:54-224``
  (the values there are pinned against this module by ``tests/test_oracle.py``).
* Montgomery encoding x -> x*R mod m, R = 2^256 (Fr) / 2^384 (Fq) --
  reference ``bls12-381/include/field.cuh:906-928``.
* Fq2 = Fq[u]/(u^2+1) -- reference ``bls12-381/include/point.cuh:81-225``.
* G1: y^2 = x^3 + 4, G2: y^2 = x^3 + 4(1+u), affine identity = (0, 0) in the byte layout --
  reference ``point.cuh:287-318`` and ``core/types.rs:89-108``.
* MSM = sum_i s_i * P_i (the unique group element every Pippenger variant must produce) --
  reference CPU path ``core/traits/cpu_impl.rs:117-165`` (BLST ``multi_exp``).
* NTT = DFT with omega_k = ROOT_OF_UNITY^(2^(32-k)), ROOT_OF_UNITY = 7^((r-1)/2^32);
  inverse scales by n^-1 -- reference ``core/ntt.rs:1488-1603`` (``best_fft``).
"""
from __future__ import annotations

import random

# --------------------------------------------------------------------------------------
# Field constants (BLS12-381 specification)
# --------------------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
FQ_BITS = 384
FR_BITS = 256
FQ_R = (1 << FQ_BITS) % P        # Montgomery one of Fq
FR_R = (1 << FR_BITS) % R        # Montgomery one of Fr
FQ_R2 = pow(1 << FQ_BITS, 2, P)
FR_R2 = pow(1 << FR_BITS, 2, R)
FQ_INV = (-pow(P, -1, 1 << 64)) % (1 << 64)
FR_INV = (-pow(R, -1, 1 << 64)) % (1 << 64)
FQ_RINV = pow(1 << FQ_BITS, -1, P)
FR_RINV = pow(1 << FR_BITS, -1, R)

TWO_ADICITY = 32
FR_GENERATOR = 7
ROOT_OF_UNITY = pow(FR_GENERATOR, (R - 1) >> TWO_ADICITY, R)   # primitive 2^32-th root

# Generators (affine, standard form)
G1_X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1_Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1
G2_X = (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E)
G2_Y = (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE)
G1_B = 4
G2_B = (4, 4)

G1 = (G1_X, G1_Y)
G2 = (G2_X, G2_Y)


# --------------------------------------------------------------------------------------
# Encodings
# --------------------------------------------------------------------------------------
def fq_to_mont(x: int) -> int:
    return (x * FQ_R) % P


def fq_from_mont(x: int) -> int:
    return (x * FQ_RINV) % P


def fr_to_mont(x: int) -> int:
    return (x * FR_R) % R


def fr_from_mont(x: int) -> int:
    return (x * FR_RINV) % R


def fr_mont_mul(a: int, b: int) -> int:
    """Montgomery product on raw (possibly Montgomery-encoded) values: a*b*R^-1 mod r.

    Reference ``field.cuh:510-576`` (CIOS); any correct implementation yields this
    canonical value."""
    return (a * b * FR_RINV) % R


def fq_mont_mul(a: int, b: int) -> int:
    return (a * b * FQ_RINV) % P


def int_to_limbs(x: int, n: int) -> list[int]:
    return [(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n)]


def limbs_to_int(limbs) -> int:
    v = 0
    for i, l in enumerate(limbs):
        v |= int(l) << (64 * i)
    return v


# --------------------------------------------------------------------------------------
# Fq2
# --------------------------------------------------------------------------------------
def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_inv(a):
    t = pow((a[0] * a[0] + a[1] * a[1]) % P, -1, P)
    return ((a[0] * t) % P, (-a[1] * t) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_eq(a, b):
    return a[0] % P == b[0] % P and a[1] % P == b[1] % P


# --------------------------------------------------------------------------------------
# Generic affine group law (None = point at infinity)
# --------------------------------------------------------------------------------------
class _Ops:
    def __init__(self, add, sub, mul, inv, neg, zero, b, eq, small):
        self.add, self.sub, self.mul, self.inv, self.neg = add, sub, mul, inv, neg
        self.zero, self.b, self.eq, self.small = zero, b, eq, small


_G1OPS = _Ops(lambda a, b: (a + b) % P, lambda a, b: (a - b) % P, lambda a, b: (a * b) % P,
              lambda a: pow(a, -1, P), lambda a: (-a) % P, 0, G1_B, lambda a, b: a % P == b % P,
              lambda k: k % P)
_G2OPS = _Ops(f2_add, f2_sub, f2_mul, f2_inv, f2_neg, (0, 0), G2_B, f2_eq, lambda k: (k % P, 0))


def _on_curve(o: _Ops, pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return o.eq(o.mul(y, y), o.add(o.mul(o.mul(x, x), x), o.b))


def _add(o: _Ops, p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if o.eq(x1, x2):
        if o.eq(y1, y2) and not o.eq(y1, o.zero):
            lam = o.mul(o.mul(o.small(3), o.mul(x1, x1)), o.inv(o.mul(o.small(2), y1)))
        else:
            return None
    else:
        lam = o.mul(o.sub(y2, y1), o.inv(o.sub(x2, x1)))
    x3 = o.sub(o.sub(o.mul(lam, lam), x1), x2)
    y3 = o.sub(o.mul(lam, o.sub(x1, x3)), y1)
    return (x3, y3)


def _neg(o: _Ops, pt):
    if pt is None:
        return None
    return (pt[0], o.neg(pt[1]))


def _mul(o: _Ops, k: int, pt):
    k %= R
    acc = None
    base = pt
    while k:
        if k & 1:
            acc = _add(o, acc, base)
        base = _add(o, base, base)
        k >>= 1
    return acc


def g1_add(a, b):
    return _add(_G1OPS, a, b)


def g1_neg(a):
    return _neg(_G1OPS, a)


def g1_mul(k, a):
    return _mul(_G1OPS, k, a)


def g1_on_curve(a):
    return _on_curve(_G1OPS, a)


def g2_add(a, b):
    return _add(_G2OPS, a, b)


def g2_neg(a):
    return _neg(_G2OPS, a)


def g2_mul(k, a):
    return _mul(_G2OPS, k, a)


def g2_on_curve(a):
    return _on_curve(_G2OPS, a)


def msm(scalars, points, group: str = "g1"):
    """Naive sum_i s_i * P_i; scalars are integers (standard form) reduced mod r."""
    add = g1_add if group == "g1" else g2_add
    mul = g1_mul if group == "g1" else g2_mul
    acc = None
    for s, pt in zip(scalars, points):
        acc = add(acc, mul(s, pt))
    return acc


def msm_shared_doubling(scalars, points, group: str = "g1"):
    """Same value as :func:`msm`, computed with one shared double-and-add chain
    (Straus over 1-bit windows) -- much cheaper for n in the hundreds."""
    add = g1_add if group == "g1" else g2_add
    acc = None
    pts = list(points)
    ks = [s % R for s in scalars]
    for bit in range(255, -1, -1):
        acc = add(acc, acc)
        for k, pt in zip(ks, pts):
            if (k >> bit) & 1:
                acc = add(acc, pt)
    return acc


# --------------------------------------------------------------------------------------
# Fr NTT (DFT semantics of best_fft)
# --------------------------------------------------------------------------------------
def omega(log_n: int) -> int:
    """omega_k = ROOT_OF_UNITY^(2^(32-k)) -- reference core/ntt.rs:1488-1494."""
    w = ROOT_OF_UNITY
    for _ in range(log_n, TWO_ADICITY):
        w = (w * w) % R
    return w


def _fft(vals, w):
    n = len(vals)
    if n == 1:
        return list(vals)
    even = _fft(vals[0::2], (w * w) % R)
    odd = _fft(vals[1::2], (w * w) % R)
    out = [0] * n
    t = 1
    for i in range(n // 2):
        u = even[i]
        v = (odd[i] * t) % R
        out[i] = (u + v) % R
        out[i + n // 2] = (u - v) % R
        t = (t * w) % R
    return out


def ntt_forward(vals):
    """out_j = sum_i vals_i * omega^(ij), values are field elements (any linear encoding)."""
    n = len(vals)
    if n == 0:
        return []
    log_n = n.bit_length() - 1
    assert 1 << log_n == n
    return _fft([v % R for v in vals], omega(log_n))


def ntt_inverse(vals):
    n = len(vals)
    if n == 0:
        return []
    log_n = n.bit_length() - 1
    w_inv = pow(omega(log_n), -1, R)
    n_inv = pow(n, -1, R)
    return [(v * n_inv) % R for v in _fft([v % R for v in vals], w_inv)]


def dft_naive(vals, w):
    n = len(vals)
    return [sum(vals[i] * pow(w, i * j, R) for i in range(n)) % R for j in range(n)]


# --------------------------------------------------------------------------------------
# Signed-digit window decomposition (reference msm_kernels.cu:86-142)
# --------------------------------------------------------------------------------------
def signed_digits(s: int, c: int, num_windows: int):
    """Returns (digits, final_carry); digits d_w in [-(2^(c-1)), 2^(c-1)] with
    s == sum d_w 2^(c w) + carry * 2^(c W)."""
    half = 1 << (c - 1)
    carry = 0
    out = []
    for w in range(num_windows):
        v = ((s >> (w * c)) & ((1 << c) - 1)) + carry
        carry = 0
        if v > half:
            v -= 1 << c
            carry = 1
        out.append(v)
    return out, carry


def precompute_shift(factor: int) -> int:
    """bits between consecutive multiples of a precomputed table [P, 2^s P, ...] (depends on
    the factor only; msm_common.hip precompute_shift)"""
    return -(-256 // factor) if factor > 1 else 0


def block_windows(c: int, factor: int):
    """(bit position, width) of every window of the precomputed-bases recoding
    (msm_common.hip window_span): factor blocks of s bits, ceil(s / c) windows per block,
    the last window of a block narrower when c does not divide s."""
    s = precompute_shift(factor)
    wg = -(-s // c)
    return [(s * f + c * l, min(c, s - c * l)) for f in range(factor) for l in range(wg)], wg


def signed_digits_blocks(x: int, c: int, factor: int):
    """signed digits over block_windows: the carry runs through all windows in order, a window
    narrower than c never carries (value + carry <= 2^(c-1)).  Returns (digits, final_carry)."""
    half = 1 << (c - 1)
    carry = 0
    out = []
    for pos, wid in block_windows(c, factor)[0]:
        v = ((x >> pos) & ((1 << wid) - 1)) + carry
        carry = 0
        if v > half:
            v -= 1 << c
            carry = 1
        out.append(v)
    return out, carry


def msm_precomputed(scalars, points, factor: int, c: int, group: str = "g1"):
    """sum s_i P_i evaluated the way the precomputed-bases MSM does: table entry (i, f) =
    2^(s f) P_i, digit (f, l) weighted 2^(c l) (small cases only)"""
    mul, add = (g1_mul, g1_add) if group == "g1" else (g2_mul, g2_add)
    s = precompute_shift(factor)
    wins, wg = block_windows(c, factor)
    acc = None
    for k, pt in zip(scalars, points):
        d, carry = signed_digits_blocks(k, c, factor)
        assert carry == 0
        for j, v in enumerate(d):
            f, l = divmod(j, wg)
            if v:
                acc = add(acc, mul(v % R, mul(1 << (s * f + c * l), pt)))
    return acc


# --------------------------------------------------------------------------------------
# GLV split used by the G1 MSM kernel (k_digits_glv).  Not a reference algorithm: the
# reference ships GLV constants only behind an experimental flag, off the MSM path
# (bls12-381/src/curve/point_ops.cu:103-145); the MSM result is unchanged by the split.
# r = lam^2 + lam + 1 exactly (lam = z^2 - 1), phi(x, y) = (beta x, y) = lam * P on G1.
# --------------------------------------------------------------------------------------
BLS_Z = -0xD201000000010000
GLV_LAMBDA = BLS_Z * BLS_Z - 1
GLV_BETA = 0x1A0111EA397FE699EC02408663D4DE85AA0D857D89759AD4897D29650FB85F9B409427EB4F49FFFD8BFD00000000AAAC


def glv_phi(pt):
    return None if pt is None else (GLV_BETA * pt[0] % P, pt[1])


def glv_decompose(s: int):
    """(m1, neg1, m2, neg2) with s == (+-m1) + (+-m2) * lam (mod r) and m1, m2 < 2^127,
    following the kernel step by step: q = floor(s / lam), balance k1 then k2."""
    lam = GLV_LAMBDA
    q, k1 = divmod(s, lam)
    half = lam >> 1
    m1, neg1, k2 = k1, False, q
    if k1 > half:
        m1, neg1, k2 = lam - k1, True, q + 1
    m2, neg2 = k2, False
    if k2 > half:
        m2, neg2 = lam + 1 - k2, True   # (k2 - lam - 1) * lam == k2 * lam + 1 (mod r)
        if neg1:
            m1 += 1
        elif m1 == 0:
            m1, neg1 = 1, True
        else:
            m1 -= 1
    return m1, neg1, m2, neg2


# --------------------------------------------------------------------------------------
# psi (untwist-Frobenius-twist) split used by the G2 MSM kernel (k_psi_split).  Not a
# reference algorithm (the reference G2 MSM runs 16 plain windows); the MSM result is unchanged.
# psi(x, y) = (conj(x) * PSI_CX, conj(y) * PSI_CY) with PSI_CX = (1+u)^-((p-1)/3),
# PSI_CY = (1+u)^-((p-1)/2); on G2 psi = [z] (z = BLS_Z), and r = x^4 - x^2 + 1 for x = |z|.
# --------------------------------------------------------------------------------------
PSI_X = -BLS_Z  # |z| = 0xd201000000010000


def _f2_pow(a, e):
    acc, b = (1, 0), a
    while e:
        if e & 1:
            acc = f2_mul(acc, b)
        b = f2_mul(b, b)
        e >>= 1
    return acc


PSI_CX = f2_inv(_f2_pow((1, 1), (P - 1) // 3))
PSI_CY = f2_inv(_f2_pow((1, 1), (P - 1) // 2))


def psi(pt):
    if pt is None:
        return None
    (x0, x1), (y0, y1) = pt
    return (f2_mul((x0, (-x1) % P), PSI_CX), f2_mul((y0, (-y1) % P), PSI_CY))


def psi_decompose(s: int):
    """[(mag_j, neg_j)] for j = 0..3 with s * Q == sum_j (-1)^neg_j mag_j psi^j(Q) on G2 and
    mag_j < 2^63, following the kernel step by step: balanced base-x digits d_j (|d_j| <= x/2),
    then the carry d_4 folded back with x^4 == x^2 - 1 (mod r); psi = [z] = [-x] flips the
    sign of the odd digits."""
    x = PSI_X
    t = s % R
    d = []
    for _ in range(4):
        t, rem = divmod(t, x)
        if rem > x // 2:
            rem -= x
            t += 1
        d.append(rem)
    d[2] += t
    d[0] -= t
    out = []
    for j, dj in enumerate(d):
        neg = (dj < 0) != (j % 2 == 1)
        out.append((abs(dj), neg))
    return out


def rng(seed: int) -> random.Random:
    return random.Random(seed)


def random_fr(r: random.Random) -> int:
    return r.randrange(R)


def random_fq(r: random.Random) -> int:
    return r.randrange(P)
