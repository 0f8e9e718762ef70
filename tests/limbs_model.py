"""Limb-exact Python model of csrc/mbls_fq28.hpp and csrc/mbls_fr29.hpp (test infrastructure).

Each function follows its header's algorithm step for step on raw limbs -- the same column order,
the same 64-bit accumulator, the same masks and shifts -- and ASSERTS the hardware limits the
header's bound table relies on: every column accumulator stays below 2^64 (v_mad_u64_u32 has no
carry-out into the next column), every uint32 limb stays below 2^32, fold's int64 stays in range.
tests/test_gpu_limbs.py runs its extreme-limb cases through this model on the CPU (the bounds as
an executable proof) and through the GPU probe (the device code itself), and checks both against
Python integers."""

U64 = 1 << 64
U32 = 1 << 32


class Overflow(AssertionError):
    pass


PEAK = {}  # largest column accumulator seen per operation (the bound tables' margins)


def _chk64(acc, what):
    if not 0 <= acc < U64:
        raise Overflow(f"{what}: column accumulator {acc:#x} >= 2^64")
    if acc > PEAK.get(what, 0):
        PEAK[what] = acc
    return acc


def _chk32(v, what):
    if not 0 <= v < U32:
        raise Overflow(f"{what}: limb {v:#x} outside uint32")
    return v


# ------------------------------------------------------------------ radix 2^28 Fq (mbls_fq28.hpp)
class Fq28:
    NL, MASK = 14, (1 << 28) - 1

    def __init__(self, P, ninv, fold_recip):
        self.P = [(P >> (28 * i)) & self.MASK for i in range(13)] + [P >> (28 * 13)]
        self.NINV, self.FOLD_RECIP = ninv, fold_recip

    def _reduce_col(self, acc, m, r, k, what):
        NL = self.NL
        lo = k - (NL - 1) if k > NL - 1 else 0
        for i in range(lo, min(k, NL)):
            acc = _chk64(acc + m[i] * self.P[k - i], what)
        if k < NL:
            m[k] = ((acc & 0xffffffff) * self.NINV) & self.MASK
            acc = _chk64(acc + m[k] * self.P[0], what)
        else:
            r[k - NL] = acc & self.MASK
        return acc >> 28

    def mul(self, a, b):
        return self.mul2(a, b, None, None)

    def mul2(self, a, b, c, d):
        NL = self.NL
        for x in (a, b) + ((c, d) if c is not None else ()):
            for v in x:
                _chk32(v, "operand")
        m, r, acc = [0] * NL, [0] * NL, 0
        for k in range(2 * NL - 1):
            lo, hi = (k - (NL - 1) if k > NL - 1 else 0), (k if k < NL - 1 else NL - 1)
            for i in range(lo, hi + 1):
                acc = _chk64(acc + a[i] * b[k - i], "mul")
            if c is not None:
                for i in range(lo, hi + 1):
                    acc = _chk64(acc + c[i] * d[k - i], "mul2")
            acc = self._reduce_col(acc, m, r, k, "mul reduction")
        r[NL - 1] = _chk32(acc, "mul top limb")
        return r

    def sqr(self, a):
        NL = self.NL
        d = [_chk32(v << 1, "sqr doubled operand") for v in a]
        m, r, acc = [0] * NL, [0] * NL, 0
        for k in range(2 * NL - 1):
            lo = k - (NL - 1) if k > NL - 1 else 0
            i = lo
            while 2 * i < k:
                acc = _chk64(acc + a[i] * d[k - i], "sqr")
                i += 1
            if k % 2 == 0:
                acc = _chk64(acc + a[k >> 1] * a[k >> 1], "sqr diagonal")
            acc = self._reduce_col(acc, m, r, k, "sqr reduction")
        r[NL - 1] = _chk32(acc, "sqr top limb")
        return r

    def add(self, a, b):
        return [_chk32(x + y, "add") for x, y in zip(a, b)]

    def sub(self, bk, a, b):
        return [_chk32(x + (k - y), "sub") for x, y, k in zip(a, b, bk)]

    def neg(self, bk, b):
        return [_chk32(k - y, "neg") for y, k in zip(b, bk)]

    def x2(self, a):
        return [_chk32(v << 1, "x2") for v in a]

    def x4(self, a):
        return [_chk32(v << 2, "x4") for v in a]

    def carry(self, a):
        r, c = [0] * self.NL, 0
        for i in range(self.NL - 1):
            t = _chk32(a[i] + c, "carry")
            r[i], c = t & self.MASK, t >> 28
        r[-1] = _chk32(a[-1] + c, "carry top")
        return r

    def fold(self, a):
        for v in a:
            _chk32(v, "fold input")
        top = (a[-1] + (a[-2] >> 28)) % U32
        nq = -(((top * self.FOLD_RECIP) % U64) >> 40)
        r, c = [0] * self.NL, 0
        for i in range(self.NL):
            t = nq * self.P[i] + c + a[i]
            if not -(1 << 63) <= t < (1 << 63):
                raise Overflow("fold int64")
            r[i], c = t & self.MASK, t >> 28
        r[-1] = (r[-1] + ((c << 28) % U32)) % U32
        return r


# ------------------------------------------------------------------ radix 2^29 Fr (mbls_fr29.hpp)
class Fr29:
    NL, MASK = 9, (1 << 29) - 1

    def __init__(self, R):
        self.RL = [(R >> (29 * i)) & self.MASK for i in range(8)] + [R >> (29 * 8)]

    def mul(self, a, b):
        NL = self.NL
        for x in (a, b):
            for v in x:
                _chk32(v, "operand")
        m, r, acc = [0] * NL, [0] * NL, 0
        for k in range(2 * NL - 1):
            lo, hi = (k - (NL - 1) if k > NL - 1 else 0), (k if k < NL - 1 else NL - 1)
            for i in range(lo, hi + 1):
                acc = _chk64(acc + a[i] * b[k - i], "fr mul")
            for i in range(lo, min(k, NL)):
                acc = _chk64(acc + m[i] * self.RL[k - i], "fr reduction")
            if k < NL:
                m[k] = (-(acc & 0xffffffff)) % U32 & self.MASK
                acc = _chk64(acc + m[k], "fr reduction")
            else:
                r[k - NL] = acc & self.MASK
            acc >>= 29
        r[NL - 1] = _chk32(acc, "fr top limb")
        return r


# ------------------------------------------------------------------ the accumulation's formulas
def _fq28_formulas(F, B16, B32, B512, ONE):
    """r28::is_zero_lt2p / is_zero_mod / dbl / madd / mmadd / to_words over the model F"""
    P = F.P

    def is_zero_lt2p(a):
        return all(v == 0 for v in a) or all(v == p for v, p in zip(a, P))

    def is_zero_mod(a):
        v = F.fold(a)
        p2, c = [], 0
        for p in P:
            t = (p << 1) + c
            c = t >> 28
            p2.append(t & F.MASK)
        return all(x == 0 for x in v) or v == P or v == p2

    def dbl(x, y, z):
        A, B = F.sqr(x), F.sqr(y)
        E = F.add(F.x2(A), A)
        D = F.mul(F.x4(x), B)
        C8 = F.mul(F.x4(F.x2(B)), B)
        X3 = F.fold(F.sub(B32, F.sqr(E), F.x2(D)))
        Y3 = F.fold(F.sub(B16, F.mul(E, F.sub(B16, D, X3)), C8))
        return X3, Y3, F.mul(F.x2(y), z)

    def madd(acc, x2_, y2_):
        x, y, z = acc
        if all(v == 0 for v in z):
            return F.fold(x2_), F.fold(y2_), list(ONE)
        Z1Z1 = F.sqr(z)
        H = F.sub(B16, F.mul(x2_, Z1Z1), x)
        Rr = F.sub(B16, F.mul(F.mul(y2_, z), Z1Z1), y)
        HH = F.sqr(H)
        if is_zero_lt2p(HH):
            return dbl(x, y, z) if is_zero_mod(Rr) else (list(ONE), list(ONE), [0] * 14)
        I = F.x4(HH)
        J = F.mul(H, I)
        Z3 = F.mul(F.x2(z), H)
        V = F.mul(x, I)
        R2 = F.carry(F.x2(Rr))
        X3 = F.fold(F.sub(B32, F.sub(B16, F.sqr(R2), J), F.x2(V)))
        Y3 = F.mul2(R2, F.sub(B16, V, X3), F.neg(B32, F.x2(y)), J)
        return X3, Y3, Z3

    def mmadd(acc, x2_, y2_):
        x, y, _ = acc
        H = F.fold(F.sub(B512, x2_, x))
        HH = F.sqr(H)
        if is_zero_lt2p(HH):
            return None
        I = F.x4(HH)
        J = F.mul(H, I)
        Z3 = F.x2(H)
        V = F.mul(x, I)
        R2 = F.x2(F.fold(F.sub(B512, y2_, y)))
        X3 = F.fold(F.sub(B32, F.sub(B16, F.sqr(R2), J), F.x2(V)))
        Y3 = F.mul2(R2, F.sub(B16, V, X3), F.neg(B32, F.x2(y)), J)
        return X3, Y3, Z3

    def to_words(a, Pint):
        v = F.fold(a)
        k = (v[0] * 0xfd) & 0xff
        c, t = 0, []
        for i in range(14):
            c += v[i] + k * P[i]
            t.append(c & F.MASK)
            c >>= 28
        if c:
            raise Overflow("to_words: (v + k p) >= 2^392")
        x = sum(x << (28 * i) for i, x in enumerate(t)) >> 8
        for _ in range(2):
            if x >= Pint:
                x -= Pint
        return [(x >> (32 * j)) & 0xffffffff for j in range(12)]

    return is_zero_mod, madd, mmadd, to_words


def _xyzz_formulas(F, B16, B32, B512, ONE):
    """r28::xdbl / xmadd / xmmadd / xadd / x_to_jac (XYZZ, mbls_fq28.hpp round 6) over the model F:
    the same operations in the same order, each column checked below 2^64"""
    is_zero_mod = _fq28_formulas(F, B16, B32, B512, ONE)[0]
    P = F.P
    ZERO = [0] * 14

    def is_zero_lt2p(a):
        return all(v == 0 for v in a) or all(v == p for v, p in zip(a, P))

    def is_inf(acc):
        return all(v == 0 for v in acc[2])

    def xdbl(acc):
        x, y, zz, zzz = acc
        U = F.x2(y)
        V = F.sqr(U)
        W = F.mul(U, V)
        S = F.mul(x, V)
        A = F.sqr(x)
        M = F.add(F.x2(A), A)
        X3 = F.fold(F.sub(B32, F.sqr(M), F.x2(S)))
        Y3 = F.mul2(M, F.sub(B16, S, X3), F.neg(B16, y), W)
        return X3, Y3, F.mul(V, zz), F.mul(W, zzz)

    def xmadd(acc, x2_, y2_):
        if is_inf(acc):
            return F.fold(x2_), F.fold(y2_), list(ONE), list(ONE)
        x, y, zz, zzz = acc
        U2 = F.mul(x2_, zz)
        S2 = F.mul(y2_, zzz)
        Pd = F.sub(B16, U2, x)
        Rr = F.carry(F.sub(B16, S2, y))
        PP = F.sqr(Pd)
        if is_zero_lt2p(PP):
            return xdbl(acc) if is_zero_mod(Rr) else (list(ONE), list(ONE), ZERO, ZERO)
        ZZ3 = F.mul(zz, PP)
        PPP = F.mul(Pd, PP)
        ZZZ3 = F.mul(zzz, PPP)
        Q = F.mul(x, PP)
        X3 = F.fold(F.sub(B32, F.sub(B16, F.sqr(Rr), PPP), F.x2(Q)))
        Y3 = F.mul2(Rr, F.sub(B16, Q, X3), F.neg(B16, y), PPP)
        return X3, Y3, ZZ3, ZZZ3

    def xmmadd(acc, x2_, y2_):
        x, y = acc[0], acc[1]
        Pd = F.fold(F.sub(B512, x2_, x))
        PP = F.sqr(Pd)
        if is_zero_lt2p(PP):
            return None
        Rr = F.fold(F.sub(B512, y2_, y))
        PPP = F.mul(Pd, PP)
        Q = F.mul(x, PP)
        X3 = F.fold(F.sub(B32, F.sub(B16, F.sqr(Rr), PPP), F.x2(Q)))
        Y3 = F.mul2(Rr, F.sub(B16, Q, X3), F.neg(B16, y), PPP)
        return X3, Y3, PP, PPP

    def xadd(acc, x2_, y2_, zz2, zzz2):
        if is_inf(acc):
            return F.fold(x2_), F.fold(y2_), F.fold(zz2), F.fold(zzz2)
        x, y, zz, zzz = acc
        U1 = F.mul(x, zz2)
        U2 = F.mul(x2_, zz)
        S1 = F.mul(y, zzz2)
        S2 = F.mul(y2_, zzz)
        Pd = F.sub(B16, U2, U1)
        Rr = F.carry(F.sub(B16, S2, S1))
        PP = F.sqr(Pd)
        if is_zero_lt2p(PP):
            return xdbl(acc) if is_zero_mod(Rr) else (list(ONE), list(ONE), ZERO, ZERO)
        PPP = F.mul(Pd, PP)
        Q = F.mul(U1, PP)
        ZZ3 = F.mul(F.mul(zz, zz2), PP)
        ZZZ3 = F.mul(F.mul(zzz, zzz2), PPP)
        X3 = F.fold(F.sub(B32, F.sub(B16, F.sqr(Rr), PPP), F.x2(Q)))
        Y3 = F.mul2(Rr, F.sub(B16, Q, X3), F.neg(B16, S1), PPP)
        return X3, Y3, ZZ3, ZZZ3

    def x_to_jac(acc):
        if is_inf(acc):
            return list(ONE), list(ONE), ZERO
        x, y, zz, zzz = acc
        return F.mul(x, F.sqr(zz)), F.mul(y, F.sqr(zzz)), list(zzz)

    return xdbl, xmadd, xmmadd, xadd, x_to_jac


class Model:
    """the GPU probe's interface (tests/diag/limbs_diag.hip op codes) over the limb model"""

    def __init__(self, P, R, ninv, fold_recip, B16, B32, B512, ONE):
        self.F, self.G, self.Pint = Fq28(P, ninv, fold_recip), Fr29(R), P
        self.ONE = ONE
        self.is_zero_mod, self.madd, self.mmadd, self.to_words = _fq28_formulas(self.F, B16, B32, B512, ONE)
        self.xdbl, self.xmadd, self.xmmadd, self.xadd, self.x_to_jac = _xyzz_formulas(self.F, B16, B32, B512, ONE)

    def __call__(self, op, cases):
        import numpy as np
        out = np.zeros((len(cases), 64), dtype=np.uint64)
        F, G = self.F, self.G
        for i, x in enumerate(cases):
            x = [list(v) for v in x] + [[0] * 16] * (8 - len(x))
            a, b, c, d, e = (v[:14] for v in x[:5])
            xs = [v[:14] for v in x]
            if op == 0:
                r = F.mul(a, b)
            elif op == 1:
                r = F.sqr(a)
            elif op == 2:
                r = F.mul2(a, b, c, d)
            elif op == 3:
                r = F.fold(a)
            elif op == 4:
                r = self.to_words(a, self.Pint)
            elif op == 5:
                r = F.carry(a)
            elif op == 6:
                r = [1 if self.is_zero_mod(a) else 0]
            elif op == 7:
                X, Y, Z = self.madd((a, b, c), d, e)
                r = X + Y + Z
            elif op == 8:
                res = self.mmadd((a, b, None), d, e)
                r = [0] * 42 + [0] if res is None else res[0] + res[1] + res[2] + [1]
                if res is None:  # acc untouched
                    r = a + b + list(self.ONE) + [0]
            elif op == 9:  # xmadd(acc = x0..x3; q = x4, x5)
                r = [v for c in self.xmadd(tuple(xs[:4]), xs[4], xs[5]) for v in c]
            elif op == 10:  # xmmadd(acc = x0, x1, one, one; q = x4, x5): 56 words + the flag
                res = self.xmmadd((xs[0], xs[1], None, None), xs[4], xs[5])
                r = (xs[0] + xs[1] + list(self.ONE) * 2 + [0]) if res is None else [v for c in res for v in c] + [1]
            elif op == 11:  # xadd(acc = x0..x3; partial = x4..x7)
                r = [v for c in self.xadd(tuple(xs[:4]), *xs[4:8]) for v in c]
            elif op == 12:  # xdbl(x0..x3)
                r = [v for c in self.xdbl(tuple(xs[:4])) for v in c]
            elif op == 13:  # x_to_jac(x0..x3): 42 words
                r = [v for c in self.x_to_jac(tuple(xs[:4])) for v in c]
            elif op in (30, 31):
                raise ValueError("pair ops: use run_pairs")
            elif op == 20:
                r = G.mul(x[0][:9], x[1][:9])
            elif op == 21:
                w = sum(int(v) << (32 * j) for j, v in enumerate(x[0][:8]))
                r = [(w >> (29 * j)) & G.MASK for j in range(8)] + [w >> 232]
            elif op == 22:
                v = sum(int(t) << (29 * j) for j, t in enumerate(x[0][:9]))
                r = [(v >> (32 * j)) & 0xffffffff for j in range(8)]
            elif op == 23:
                w = sum(int(v) << (32 * j) for j, v in enumerate(x[0][:8]))
                m = G.mul([(w >> (29 * j)) & G.MASK for j in range(8)] + [w >> 232], x[1][:9])
                v = sum(int(t) << (29 * j) for j, t in enumerate(m))
                if v >= 1 << 256:
                    raise Overflow("mul_words: product >= 2^256 does not pack")
                r = [(v >> (32 * j)) & 0xffffffff for j in range(8)]
            else:
                raise ValueError(op)
            out[i, :len(r)] = r
        return out


# ------------------------------------------------------------------ pair-sliced Fq2 (mbls_fq2_28.hpp)
class Fq2P28:
    """lane j of a pair holds component c_j (14 limbs); the partner's limbs arrive by DPP.  Every
    operation here is what ONE pair of lanes computes, lane 0 and lane 1 each with the model F."""

    def __init__(self, F, B16, B32, B512):
        self.F, self.B16, self.B32, self.B512 = F, B16, B32, B512

    def mul4(self, terms):
        """sum of up to 4 limb products with ONE reduction (a lane's share of an Fq2 product or
        product sum); the column bound covers all of them at once"""
        F = self.F
        NL = F.NL
        for a, b in terms:
            for v in a + b:
                _chk32(v, "operand")
        m, r, acc = [0] * NL, [0] * NL, 0
        for k in range(2 * NL - 1):
            lo, hi = (k - (NL - 1) if k > NL - 1 else 0), (k if k < NL - 1 else NL - 1)
            for a, b in terms:
                for i in range(lo, hi + 1):
                    acc = _chk64(acc + a[i] * b[k - i], "fq2 product")
            acc = F._reduce_col(acc, m, r, k, "fq2 reduction")
        r[NL - 1] = _chk32(acc, "fq2 top limb")
        return r

    def mul(self, a, b, bk):
        """a b: lane 0 a0 b0 + a1 (bk - b1), lane 1 a1 b0 + a0 b1; bk: the bias of the partner
        negation (limbs >= b1's)"""
        F = self.F
        return (self.mul4([(a[0], b[0]), (a[1], F.neg(bk, b[1]))]), self.mul4([(a[1], b[0]), (a[0], b[1])]))

    def mul2(self, a, b, c, d, bkb, bkd):
        F = self.F
        return (self.mul4([(a[0], b[0]), (a[1], F.neg(bkb, b[1])), (c[0], d[0]), (c[1], F.neg(bkd, d[1]))]),
                self.mul4([(a[1], b[0]), (a[0], b[1]), (c[1], d[0]), (c[0], d[1])]))

    def sqr(self, a, bk):
        """lane 0 (a0 + a1)(a0 - a1 + bk), lane 1 a1 (2 a0)"""
        F = self.F
        return (self.mul4([(F.add(a[0], a[1]), F.sub(bk, a[0], a[1]))]), self.mul4([(a[1], F.x2(a[0]))]))

    def each(self, f, *xs):
        return tuple(f(*(x[j] for x in xs)) for j in range(2))


def _fq2_formulas(F, B16, B32, B512, ONE):
    """the G2 accumulation's madd / mmadd over pair-sliced radix-2^28 Fq2, with the carries that
    keep every product's columns below 2^64 (csrc/mbls_fq2_28.hpp follows this step for step)"""
    Q = Fq2P28(F, B16, B32, B512)
    ONE2 = (list(ONE), [0] * 14)
    e = Q.each

    Pint = sum(v << (28 * i) for i, v in enumerate(F.P))

    def is_zero_lt2p(a):
        """0 mod p for components below 2p (the test reads 0 or p): asserts that precondition"""
        for c in a:
            if sum(v << (28 * i) for i, v in enumerate(c)) >= 2 * Pint:
                raise Overflow("is_zero_lt2p: component >= 2p")
        P = F.P
        return all(all(v == 0 for v in c) or c == P for c in a)

    def madd(acc, x2_, y2_):
        """acc (x, y normalised < 3p, z normalised); q = (x2_, y2_) normalised (the caller
        carries a negated y2).  None for the exceptional H = 0 (the kernel's word-form path).
        The partner negations take the bias whose limbs (top limb included) cover the operand:
        B16 for values < 16p, B32 < 32p, B512 beyond."""
        x, y, z = acc
        Z1Z1 = Q.sqr(z, B16)
        U2 = Q.mul(x2_, Z1Z1, B16)
        S2 = Q.mul(Q.mul(y2_, z, B16), Z1Z1, B16)
        H = e(F.carry, e(lambda a, b: F.sub(B16, a, b), U2, x))  # < 19p
        R = e(lambda a, b: F.sub(B16, a, b), S2, y)
        HH = Q.sqr(H, B32)
        if is_zero_lt2p(HH):
            return None
        I = e(F.x4, HH)
        J = Q.mul(H, I, B512)
        Z3 = Q.mul(e(F.x2, z), H, B32)
        V = Q.mul(x, I, B512)
        R2 = e(F.carry, e(F.x2, R))  # < 38p
        X3 = e(F.fold, e(lambda a, b: F.sub(B32, a, b), e(lambda a, b: F.sub(B16, a, b), Q.sqr(R2, B512), J),
                         e(F.x2, V)))
        VX = e(F.carry, e(lambda a, b: F.sub(B16, a, b), V, X3))  # < 19p
        NY = e(F.carry, e(lambda a: F.neg(B32, a), e(F.x2, y)))
        Y3 = Q.mul2(R2, VX, NY, J, B32, B16)
        return X3, Y3, Z3

    def mmadd(acc, x2_, y2_):
        x, y, _ = acc
        H = e(F.fold, e(lambda a, b: F.sub(B512, a, b), x2_, x))
        HH = Q.sqr(H, B16)
        if is_zero_lt2p(HH):
            return None
        I = e(F.x4, HH)
        J = Q.mul(H, I, B512)
        Z3 = e(F.carry, e(F.x2, H))
        V = Q.mul(x, I, B512)
        R2 = e(F.carry, e(F.x2, e(F.fold, e(lambda a, b: F.sub(B512, a, b), y2_, y))))
        X3 = e(F.fold, e(lambda a, b: F.sub(B32, a, b), e(lambda a, b: F.sub(B16, a, b), Q.sqr(R2, B16), J),
                         e(F.x2, V)))
        VX = e(F.carry, e(lambda a, b: F.sub(B16, a, b), V, X3))
        NY = e(F.carry, e(lambda a: F.neg(B32, a), e(F.x2, y)))
        Y3 = Q.mul2(R2, VX, NY, J, B32, B16)
        return X3, Y3, Z3

    return madd, mmadd


def _fq2_xyzz_formulas(F, B16, B32, B512, ONE):
    """the G2 accumulation's XYZZ forms over pair-sliced radix-2^28 Fq2 (csrc/mbls_fq2_28.hpp round
    6: xdbl / xmadd / xmmadd / xadd / x_to_jac), step for step with their carries and biases"""
    Q = Fq2P28(F, B16, B32, B512)
    ONE2 = (list(ONE), [0] * 14)
    ZERO2 = ([0] * 14, [0] * 14)
    e = Q.each
    Pint = sum(v << (28 * i) for i, v in enumerate(F.P))
    is_zero_mod1 = _fq28_formulas(F, B16, B32, B512, ONE)[0]

    def is_zero_lt2p(a):
        for c in a:
            if sum(v << (28 * i) for i, v in enumerate(c)) >= 2 * Pint:
                raise Overflow("is_zero_lt2p: component >= 2p")
        return all(all(v == 0 for v in c) or c == F.P for c in a)

    def is_inf(acc):
        return all(all(v == 0 for v in c) for c in acc[2])

    def sub(bk):
        return lambda a, b: F.sub(bk, a, b)

    def xdbl(acc):
        x, y, zz, zzz = acc
        U = e(F.carry, e(F.x2, y))
        V = Q.sqr(U, B16)
        W = Q.mul(U, V, B16)
        S = Q.mul(x, V, B16)
        A = Q.sqr(x, B16)
        M = e(F.carry, e(F.add, e(F.x2, A), A))
        X3 = e(F.fold, e(sub(B32), Q.sqr(M, B16), e(F.x2, S)))
        Y3 = Q.mul2(M, e(F.carry, e(sub(B16), S, X3)), e(F.carry, e(lambda a: F.neg(B16, a), y)), W, B32, B16)
        return X3, Y3, Q.mul(V, zz, B16), Q.mul(W, zzz, B16)

    def xmadd(acc, x2_, y2_):
        if is_inf(acc):
            return e(F.fold, x2_), e(F.fold, y2_), ONE2, ONE2
        x, y, zz, zzz = acc
        U2 = Q.mul(x2_, zz, B16)
        S2 = Q.mul(y2_, zzz, B16)
        Pd = e(F.carry, e(sub(B16), U2, x))
        Rr = e(F.carry, e(sub(B16), S2, y))
        PP = Q.sqr(Pd, B32)
        if is_zero_lt2p(PP):
            if all(is_zero_mod1(c) for c in Rr):
                return xdbl(acc)
            return ONE2, ONE2, ZERO2, ZERO2
        ZZ3 = Q.mul(zz, PP, B16)
        PPP = Q.mul(Pd, PP, B16)
        ZZZ3 = Q.mul(zzz, PPP, B16)
        Qv = Q.mul(x, PP, B16)
        X3 = e(F.fold, e(sub(B32), e(sub(B16), Q.sqr(Rr, B32), PPP), e(F.x2, Qv)))
        Y3 = Q.mul2(Rr, e(F.carry, e(sub(B16), Qv, X3)), e(F.carry, e(lambda a: F.neg(B16, a), y)), PPP, B32, B16)
        return X3, Y3, ZZ3, ZZZ3

    def xmmadd(acc, x2_, y2_):
        x, y = acc[0], acc[1]
        Pd = e(F.fold, e(sub(B512), x2_, x))
        PP = Q.sqr(Pd, B16)
        if is_zero_lt2p(PP):
            return None
        Rr = e(F.fold, e(sub(B512), y2_, y))
        PPP = Q.mul(Pd, PP, B16)
        Qv = Q.mul(x, PP, B16)
        X3 = e(F.fold, e(sub(B32), e(sub(B16), Q.sqr(Rr, B16), PPP), e(F.x2, Qv)))
        Y3 = Q.mul2(Rr, e(F.carry, e(sub(B16), Qv, X3)), e(F.carry, e(lambda a: F.neg(B16, a), y)), PPP, B32, B16)
        return X3, Y3, PP, PPP

    def xadd(acc, x2_, y2_, zz2, zzz2):
        if is_inf(acc):
            return x2_, y2_, zz2, zzz2
        x, y, zz, zzz = acc
        U1 = Q.mul(x, zz2, B16)
        U2 = Q.mul(x2_, zz, B16)
        S1 = Q.mul(y, zzz2, B16)
        S2 = Q.mul(y2_, zzz, B16)
        Pd = e(F.carry, e(sub(B16), U2, U1))
        Rr = e(F.carry, e(sub(B16), S2, S1))
        PP = Q.sqr(Pd, B32)
        if is_zero_lt2p(PP):
            if all(is_zero_mod1(c) for c in Rr):
                return xdbl(acc)
            return ONE2, ONE2, ZERO2, ZERO2
        PPP = Q.mul(Pd, PP, B16)
        Qv = Q.mul(U1, PP, B16)
        ZZ3 = Q.mul(Q.mul(zz, zz2, B16), PP, B16)
        ZZZ3 = Q.mul(Q.mul(zzz, zzz2, B16), PPP, B16)
        X3 = e(F.fold, e(sub(B32), e(sub(B16), Q.sqr(Rr, B32), PPP), e(F.x2, Qv)))
        Y3 = Q.mul2(Rr, e(F.carry, e(sub(B16), Qv, X3)), e(F.carry, e(lambda a: F.neg(B16, a), S1)), PPP, B32, B16)
        return X3, Y3, ZZ3, ZZZ3

    def x_to_jac(acc):
        if is_inf(acc):
            return ONE2, ONE2, ZERO2
        x, y, zz, zzz = acc
        return Q.mul(x, Q.sqr(zz, B16), B16), Q.mul(y, Q.sqr(zzz, B16), B16), zzz

    return xdbl, xmadd, xmmadd, xadd, x_to_jac
