// mbls_fq28.hpp -- BLS12-381 Fq in unsaturated radix 2^28 for the accumulation's lane arithmetic.
//
// Why: on gfx950 every wave64 VALU instruction issues over ~4 SIMD cycles, v_mad_u64_u32 as much as
// v_addc_co_u32 (tools/valu_ceiling.hip, profiles/r05/valu_ceiling.json).  The 32-bit product-
// scanning Montgomery product (mbls_fips.hpp) pays one v_addc for the column-overflow counter
// after EVERY v_mad_u64_u32: ~576 instructions per Fq product, half of them carries.  With 14
// limbs of 28 bits a partial product is < 2^60 and a column of <= 28 products plus <= 14
// reduction terms stays below 2^64, so a column is a plain v_mad_u64_u32 chain into one 64-bit
// accumulator with no carry tracking at all: 196 product + 196 reduction mads and ~70 other
// instructions (~460) -- 20% fewer instructions per product, ~17% per mixed addition.
//
// Representation.  A value v is 14 limbs l_i with v = sum l_i 2^(28 i); limbs may exceed 28 bits
// ("unsaturated") inside formulas.  Montgomery radix R' = 2^392 (14 x 28), so x is held as
// x R' mod p (up to a multiple of p).  Memory keeps the library's format, canonical x R mod p with
// R = 2^384 (blst / reference layout): `unpack_shift8` re-splits those 12 words 8 bits lower,
// giving x R 2^8 = x R' exactly with no arithmetic (< 256 p, normalised limbs), and `to_words`
// divides by 2^8 (one 8-bit Montgomery step) and reduces to the canonical 32-bit words.
//
// Bounds (at their maxima: tests/test_gpu_limbs.py, limb-exact model on the CPU and the device code
// through tests/diag/limbs_diag.hip; random chains bit-exact against the FIPS path: tools/fq28_bench):
//   * product inputs: limbs a_i < 2^A, b_j < 2^B with 14 * 2^(A+B) + 14 * 2^56 + carry < 2^64
//     (A + B <= 60.1; the squaring doubles one operand: A + B + 1 <= 60.1 for 7 cross terms);
//   * product outputs are normalised (limbs < 2^28) and < p (1 + a b / 2^392) for inputs a, b:
//     < 2p for every operand in the mixed addition below;
//   * a - b as a + (K p - b) with a bias K p whose limbs are >= every limb of b (B16: b
//     normalised and < 8p; B32: b limbs < 2^29 and < 16p; B512: b < 256p);
//   * `fold` carries and subtracts q p with q from the top limb: normalised, < 3p.
#pragma once
#include "mbls_field.hpp"
#include "mbls_madchain.hpp"

namespace mbls {
namespace r28 {

constexpr int NL = 14;
constexpr uint32_t MASK = (1u << 28) - 1;
constexpr uint32_t P[NL] = {0xfffaaabu, 0xfefffffu, 0x3ffffb9u, 0xfffeb15u, 0x6241eabu, 0xa0f6b0fu, 0xf6730d2u,
                            0xf38512bu, 0x4774b84u, 0x4bacd76u, 0xba7b643u, 0xe69a4b1u, 0x1ea397fu, 0x1a011u};
constexpr uint32_t NINV = 0xffcfffdu;  // -p^-1 mod 2^28
// K p with every limb below the top >= 2^28 - 1 (B16), >= 2^29 (B32), >= 2^30 (B512)
constexpr uint32_t B16[NL] = {0x1ffaaab0u, 0x1efffffeu, 0x1ffffb9eu, 0x1ffeb152u, 0x1241eabeu, 0x10f6b0f5u, 0x16730d29u,
                              0x138512beu, 0x1774b84eu, 0x1bacd763u, 0x1a7b6433u, 0x169a4b1au, 0x1ea397fdu, 0x1a0110u};
constexpr uint32_t B32[NL] = {0x2ff55560u, 0x2dfffffdu, 0x2ffff73du, 0x2ffd62a5u, 0x2483d57du, 0x21ed61eau, 0x2ce61a52u,
                              0x270a257cu, 0x2ee9709cu, 0x2759aec6u, 0x24f6c867u, 0x2d349635u, 0x2d472ffau, 0x340221u};
constexpr uint32_t B512[NL] = {0x4f555600u, 0x4ffffffbu, 0x4fff73f9u, 0x4fd62a7bu, 0x483d57fbu, 0x4ed61ec0u, 0x4e61a53du,
                               0x40a257e8u, 0x4e9709e3u, 0x459aec8au, 0x4f6c8693u, 0x43496370u, 0x4472ffc9u, 0x3402239u};
// R' mod p = 2^392 mod p (the Montgomery one of this representation)
constexpr uint32_t ONE[NL] = {0x347fcb8u, 0xd800000u, 0x2b119u,   0xcde6d2u,  0xc7212e0u, 0x83a2090u, 0x37669fu,
                              0xda0f73eu, 0x9b09b42u, 0x1297bb0u, 0x515d98fu, 0x12ca7cu,  0x659fcfau, 0x577au};
constexpr uint32_t PINV8 = 0xfdu;  // -p^-1 mod 2^8
// floor(2^40 / (floor(p / 2^364) + 1)): q = (top * FOLD_RECIP) >> 40 <= top / (p_top + 1) <= v / p
constexpr uint64_t FOLD_RECIP = (1ull << 40) / (0x1a011ull + 1);

struct F28 {
    uint32_t l[NL];
    MBLS_DEV static F28 one() {
        F28 r;
#pragma unroll
        for (int i = 0; i < NL; ++i) r.l[i] = ONE[i];
        return r;
    }
    MBLS_DEV static F28 zero() {
        F28 r;
#pragma unroll
        for (int i = 0; i < NL; ++i) r.l[i] = 0;
        return r;
    }
};

// ------------------------------------------------------------------------- products
// Montgomery product (a b + m p) / 2^392, product scanning; column k accumulates its
// a_i b_(k-i) and m_i p_(k-i) in ONE 64-bit register as one v_mad_u64_u32 chain (mbls_madchain.hpp:
// written as C++ additions LLVM gave every column a fresh chain plus a 64-bit merge add, ~39
// extra instructions per product).  Columns by compile-time recursion; SQ: the square's column
// (cross products against the doubled operand d, then the diagonal term); C2/D2: mul2's second
// product.
template <int K>
MBLS_DEV void reduce_col(uint64_t& acc, uint32_t (&m)[NL], F28& r) {
    constexpr int LO = K > NL - 1 ? K - (NL - 1) : 0;
    madc::col<K, LO, (K < NL ? K : NL) - 1, true>(acc, m, P);
    if constexpr (K < NL) {
        m[K] = ((uint32_t)acc * NINV) & MASK;
        madc::mad1<true>(acc, m[K], P[0]);  // the low 28 bits become zero
    } else {
        r.l[K - NL] = (uint32_t)acc & MASK;
    }
    acc >>= 28;
}
template <int K>
MBLS_DEV void mul_cols(uint64_t& acc, uint32_t (&m)[NL], F28& r, const F28& a, const F28& b) {
    if constexpr (K < 2 * NL - 1) {
        madc::col<K, (K > NL - 1 ? K - (NL - 1) : 0), (K < NL - 1 ? K : NL - 1), false>(acc, a.l, b.l);
        reduce_col<K>(acc, m, r);
        mul_cols<K + 1>(acc, m, r, a, b);
    }
}
template <int K>
MBLS_DEV void mul2_cols(uint64_t& acc, uint32_t (&m)[NL], F28& r, const F28& a, const F28& b, const F28& c,
                        const F28& d) {
    if constexpr (K < 2 * NL - 1) {
        constexpr int LO = K > NL - 1 ? K - (NL - 1) : 0, HI = K < NL - 1 ? K : NL - 1;
        madc::col<K, LO, HI, false>(acc, a.l, b.l);
        madc::col<K, LO, HI, false>(acc, c.l, d.l);
        reduce_col<K>(acc, m, r);
        mul2_cols<K + 1>(acc, m, r, a, b, c, d);
    }
}
// four products, one reduction: a lane's share of a pair-sliced Fq2 product sum (mbls_fq2_28.hpp)
template <int K>
MBLS_DEV void mul4_cols(uint64_t& acc, uint32_t (&m)[NL], F28& r, const F28 (&x)[8]) {
    if constexpr (K < 2 * NL - 1) {
        constexpr int LO = K > NL - 1 ? K - (NL - 1) : 0, HI = K < NL - 1 ? K : NL - 1;
        madc::col<K, LO, HI, false>(acc, x[0].l, x[1].l);
        madc::col<K, LO, HI, false>(acc, x[2].l, x[3].l);
        madc::col<K, LO, HI, false>(acc, x[4].l, x[5].l);
        madc::col<K, LO, HI, false>(acc, x[6].l, x[7].l);
        reduce_col<K>(acc, m, r);
        mul4_cols<K + 1>(acc, m, r, x);
    }
}
template <int K>
MBLS_DEV void sqr_cols(uint64_t& acc, uint32_t (&m)[NL], F28& r, const F28& a, const uint32_t (&d)[NL]) {
    if constexpr (K < 2 * NL - 1) {
        constexpr int LO = K > NL - 1 ? K - (NL - 1) : 0;
        madc::col<K, LO, (K + 1) / 2 - 1, false>(acc, a.l, d);  // i < k - i: a_i (2 a_(k-i)) (none at k = 0)
        if constexpr ((K & 1) == 0) madc::mad1<false>(acc, a.l[K >> 1], a.l[K >> 1]);
        reduce_col<K>(acc, m, r);
        sqr_cols<K + 1>(acc, m, r, a, d);
    }
}

MBLS_DEV F28 mul(const F28& a, const F28& b) {
    uint32_t m[NL];
    F28 r;
    uint64_t acc = 0;
    mul_cols<0>(acc, m, r, a, b);
    r.l[NL - 1] = (uint32_t)acc;
    return r;
}

// a b + c d with one reduction (lazy Y3 of the mixed addition)
MBLS_DEV F28 mul2(const F28& a, const F28& b, const F28& c, const F28& d) {
    uint32_t m[NL];
    F28 r;
    uint64_t acc = 0;
    mul2_cols<0>(acc, m, r, a, b, c, d);
    r.l[NL - 1] = (uint32_t)acc;
    return r;
}

// a b + c d + e f + g h with one reduction (column bound: 56 products + 14 reduction terms)
MBLS_DEV F28 mul4(const F28& a, const F28& b, const F28& c, const F28& d, const F28& e, const F28& f, const F28& g,
                  const F28& h) {
    uint32_t m[NL];
    F28 r;
    uint64_t acc = 0;
    const F28 x[8] = {a, b, c, d, e, f, g, h};
    mul4_cols<0>(acc, m, r, x);
    r.l[NL - 1] = (uint32_t)acc;
    return r;
}

// square: cross products once against the doubled operand (limb bound: a_i 2 a_j, see header)
MBLS_DEV F28 sqr(const F28& a) {
    uint32_t d[NL], m[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) d[i] = a.l[i] << 1;
    F28 r;
    uint64_t acc = 0;
    sqr_cols<0>(acc, m, r, a, d);
    r.l[NL - 1] = (uint32_t)acc;
    return r;
}

// ------------------------------------------------------------------------- additions
MBLS_DEV F28 add(const F28& a, const F28& b) {
    F28 r;
#pragma unroll
    for (int i = 0; i < NL; ++i) r.l[i] = a.l[i] + b.l[i];
    return r;
}
// a - b + K p (bias table BK: limbs >= b's limbs)
template <const uint32_t* BK>
MBLS_DEV F28 sub(const F28& a, const F28& b) {
    F28 r;
#pragma unroll
    for (int i = 0; i < NL; ++i) r.l[i] = a.l[i] + (BK[i] - b.l[i]);
    return r;
}
// K p - b
template <const uint32_t* BK>
MBLS_DEV F28 neg(const F28& b) {
    F28 r;
#pragma unroll
    for (int i = 0; i < NL; ++i) r.l[i] = BK[i] - b.l[i];
    return r;
}
MBLS_DEV F28 x2(const F28& a) {
    F28 r;
#pragma unroll
    for (int i = 0; i < NL; ++i) r.l[i] = a.l[i] << 1;
    return r;
}
MBLS_DEV F28 x4(const F28& a) {
    F28 r;
#pragma unroll
    for (int i = 0; i < NL; ++i) r.l[i] = a.l[i] << 2;
    return r;
}

// carry propagation: limbs < 2^28 except the top one (value unchanged)
MBLS_DEV F28 carry(const F28& a) {
    F28 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < NL - 1; ++i) {
        const uint32_t t = a.l[i] + c;
        r.l[i] = t & MASK;
        c = t >> 28;
    }
    r.l[NL - 1] = a.l[NL - 1] + c;
    return r;
}

// normalise and fold: limbs < 2^32 (no uint32 wrap; the sums work in int64), value < 2^391 ->
// normalised, congruent, < 3p.  With t = l_13 + (l_12 >> 28) the value is below (t + 1 + 2^-23)
// 2^364 (the rest of l_12 and every lower limb < 2^32 add < 2^364 + 2^341), and p >= P_13 2^364, so
// v / p - q < (t + 1.001) / P_13 - t / (P_13 + 1) + 1 = t / (P_13 (P_13 + 1)) + 1.001 / P_13 + 1
// < 1.02 for t < 2^27: q under-estimates floor(v / p) by <= 2 (mmadd's sub<B512>(y2, acc.y) with a
// negated y2 reaches limbs ~2^31.3; pinned by tests/test_gpu_limbs.py at the limb maxima).
MBLS_DEV F28 fold(const F28& a) {
    const uint32_t top = a.l[NL - 1] + (a.l[NL - 2] >> 28);
    const int32_t nq = -(int32_t)(uint32_t)(((uint64_t)top * FOLD_RECIP) >> 40);
    F28 r;
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        const int64_t t = (int64_t)nq * (int64_t)P[i] + c + (int64_t)a.l[i];
        r.l[i] = (uint32_t)t & MASK;
        c = t >> 28;
    }
    r.l[NL - 1] += (uint32_t)c << 28;  // the top limb keeps what is left (value < 3p: 0 here)
    return r;
}

// ------------------------------------------------------------------------- conversions
// canonical Montgomery words (x R mod p, R = 2^384, 12 x u32) -> x R' = x R 2^8 (< 256 p):
// limb i = bits [28 i - 8, 28 i + 20) of the 384-bit word string, no arithmetic
MBLS_DEV F28 unpack_shift8(const uint32_t (&w)[12]) {
    F28 r;
    r.l[0] = (w[0] << 8) & MASK;
#pragma unroll
    for (int i = 1; i < NL; ++i) {
        const int bit = 28 * i - 8, wi = bit >> 5, sh = bit & 31;
        const uint32_t lo = w[wi], hi = wi + 1 < 12 ? w[wi + 1] : 0u;
        r.l[i] = (sh ? __builtin_amdgcn_alignbit(hi, lo, sh) : lo) & MASK;
    }
    return r;
}

// x R' (normalised or not, < 2^391) -> canonical words x R mod p: fold, divide by 2^8 (one
// Montgomery step with an 8-bit multiplier), repack 28 -> 32-bit limbs, subtract p while >= p
MBLS_DEV void to_words(const F28& a, uint32_t (&w)[12]) {
    F28 v = fold(a);  // < 3p, normalised
    const uint32_t k = (v.l[0] * PINV8) & 0xffu;
    // (v + k p) / 2^8, carried in 28-bit limbs
    uint64_t c = 0;
    uint32_t t[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        c += (uint64_t)v.l[i] + (uint64_t)k * P[i];
        t[i] = (uint32_t)c & MASK;
        c >>= 28;
    }
    // value = sum t_i 2^(28 i) + c 2^392, divisible by 2^8; shift right by 8 into 32-bit words
    uint32_t x[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        // bits [32 j + 8, 32 j + 40) of the 28-bit-limb string
        const int bit = 32 * j + 8;
        const int li = bit / 28, sh = bit % 28;
        uint64_t s = (uint64_t)t[li] >> sh;
        if (li + 1 < NL) s |= (uint64_t)t[li + 1] << (28 - sh);
        if (li + 2 < NL) s |= (uint64_t)t[li + 2] << (56 - sh);
        x[j] = (uint32_t)s;
    }
    // < 3p after the division (v < 3p, k p / 2^8 < p): at most two subtractions
#pragma unroll
    for (int rep = 0; rep < 2; ++rep) {
        uint32_t d[12];
        unsigned br = 0;
#pragma unroll
        for (int j = 0; j < 12; ++j) d[j] = __builtin_subc(x[j], FqCfg::MOD[j], br, &br);
#pragma unroll
        for (int j = 0; j < 12; ++j) x[j] = br ? x[j] : d[j];
    }
#pragma unroll
    for (int j = 0; j < 12; ++j) w[j] = x[j];
}

// is the (normalised, < 2p) value 0 mod p, i.e. 0 or p
MBLS_DEV bool is_zero_lt2p(const F28& a) {
    uint32_t z = 0, e = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        z |= a.l[i];
        e |= a.l[i] ^ P[i];
    }
    return z == 0 || e == 0;
}
// any value (< 2^391): 0 mod p?  fold to < 3p, then compare with 0, p, 2p
MBLS_DEV bool is_zero_mod(const F28& a) {
    const F28 v = fold(a);
    uint32_t z = 0, e1 = 0, e2 = 0;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        const uint32_t p2 = (P[i] << 1) + c;  // 2p in normalised limbs
        c = p2 >> 28;
        z |= v.l[i];
        e1 |= v.l[i] ^ P[i];
        e2 |= v.l[i] ^ (p2 & MASK);
    }
    return z == 0 || e1 == 0 || e2 == 0;
}

// ------------------------------------------------------------------------- G1 points
// Jacobian accumulator of the lane accumulation.  Invariant between steps: x, y normalised and
// < 3p (they are subtrahends against B16); z < 8p with limbs < 2^29 (z only meets products).
struct J28 {
    F28 x, y, z;
    MBLS_DEV bool is_inf() const {
        uint32_t t = 0;
#pragma unroll
        for (int i = 0; i < NL; ++i) t |= z.l[i];
        return t == 0;  // the representation of infinity here is exactly z = 0 (set, never computed)
    }
    MBLS_DEV static J28 inf() { return {F28::one(), F28::one(), F28::zero()}; }
};

// dbl-2009-l (exceptional path only: P == Q inside a bucket)
MBLS_DEV J28 dbl(const J28& p) {
    const F28 A = sqr(p.x), B = sqr(p.y);
    const F28 E = add(x2(A), A);         // 3A: limbs < 3 2^28
    const F28 D = mul(x4(p.x), B);       // 4 X B
    const F28 C8 = mul(x4(x2(B)), B);    // 8 B^2 (x2 x4: limbs < 2^31, against B < 2^28)
    J28 r;
    r.x = fold(sub<B32>(sqr(E), x2(D)));
    r.y = fold(sub<B16>(mul(E, sub<B16>(D, r.x)), C8));
    r.z = mul(x2(p.y), p.z);
    return r;
}

// Register parking for the mixed addition: acc.x is needed again at V and acc.y at Y3, across
// the products in between.  ParkReg keeps them in registers; a kernel at its register bound can
// park them in memory it owns instead of letting the compiler spill to scratch (Park::put / get
// of slot 0 = x, 1 = y; a park that holds only some slots keeps the others in registers).
struct ParkReg {
    F28 v[2];
    MBLS_DEV void put(int s, const F28& a) { v[s] = a; }
    MBLS_DEV F28 get(int s) const { return v[s]; }
};

// acc + q, q = (x2, y2) affine from unpack_shift8 (< 256 p, normalised, not the identity; y2
// may instead be neg<B512> of one: < 512 p, limbs < 2^30.4 -- it only meets products and folds):
// madd-2007-bl with the lazy Y3, Z3 = 2 Z1 H (the same field values as mbls_curve.hpp's
// jac_madd, hence the same Jacobian representative)
template <class Park>
MBLS_DEV void madd(J28& acc, const F28& x2_, const F28& y2_, Park& pk) {
    if (acc.is_inf()) {
        acc = {fold(x2_), fold(y2_), F28::one()};
        return;
    }
    const F28 Z1Z1 = sqr(acc.z);
    const F28 H = sub<B16>(mul(x2_, Z1Z1), acc.x);
    pk.put(0, acc.x);
    const F28 R = sub<B16>(mul(mul(y2_, acc.z), Z1Z1), acc.y);
    pk.put(1, acc.y);
    const F28 HH = sqr(H);
    if (is_zero_lt2p(HH)) {  // H == 0 mod p: equal or opposite points
        acc.x = pk.get(0);
        acc.y = pk.get(1);
        acc = is_zero_mod(R) ? dbl(acc) : J28::inf();
        return;
    }
    // ordered for register pressure: z and H die at Z3, x and I at V
    const F28 I = x4(HH);
    const F28 J = mul(H, I);
    acc.z = mul(x2(acc.z), H);
    const F28 V = mul(pk.get(0), I);
    const F28 R2 = carry(x2(R));
    acc.x = fold(sub<B32>(sub<B16>(sqr(R2), J), x2(V)));
    acc.y = mul2(R2, sub<B16>(V, acc.x), neg<B32>(x2(pk.get(1))), J);
}
MBLS_DEV void madd(J28& acc, const F28& x2_, const F28& y2_) {
    ParkReg pk;
    madd(acc, x2_, y2_, pk);
}

// acc + q for a Jacobian q = (x2, y2, z2) from unpack_shift8 (each < 256 p, normalised; z2 != 0):
// add-2007-bl with the lazy Y3 and Z3 = 2 Z1 Z2 H (the field values of mbls_curve.hpp's jac_add,
// hence the same representative).  Bounds as in madd; Z2Z2 of an unpacked z2 is < 27 p.
MBLS_DEV void jadd(J28& acc, const F28& x2_, const F28& y2_, const F28& z2_) {
    if (acc.is_inf()) {
        acc = {fold(x2_), fold(y2_), fold(z2_)};
        return;
    }
    const F28 Z1Z1 = sqr(acc.z);
    const F28 Z2Z2 = sqr(z2_);
    const F28 U1 = mul(acc.x, Z2Z2);
    const F28 S1 = mul(mul(acc.y, z2_), Z2Z2);
    const F28 H = sub<B16>(mul(x2_, Z1Z1), U1);
    const F28 R = sub<B16>(mul(mul(y2_, acc.z), Z1Z1), S1);
    const F28 HH = sqr(H);
    if (is_zero_lt2p(HH)) {  // H == 0 mod p: equal or opposite points
        acc = is_zero_mod(R) ? dbl(acc) : J28::inf();
        return;
    }
    const F28 I = x4(HH);
    const F28 J = mul(H, I);
    acc.z = mul(mul(x2(acc.z), z2_), H);
    const F28 V = mul(U1, I);
    const F28 R2 = carry(x2(R));
    acc.x = fold(sub<B32>(sub<B16>(sqr(R2), J), x2(V)));
    acc.y = mul2(R2, sub<B16>(V, acc.x), neg<B32>(x2(S1)), J);
}

// acc fresh from the chunk's first point (z = R'-one, x, y folded): mmadd-2007-bl, Z3 = 2H.
// Returns false (acc untouched) when x1 == x2 mod p, left to madd's branches.
MBLS_DEV bool mmadd(J28& acc, const F28& x2_, const F28& y2_) {
    const F28 H = fold(sub<B512>(x2_, acc.x));
    const F28 HH = sqr(H);
    if (is_zero_lt2p(HH)) return false;
    const F28 I = x4(HH);
    const F28 J = mul(H, I);
    acc.z = x2(H);
    const F28 V = mul(acc.x, I);
    const F28 R2 = x2(fold(sub<B512>(y2_, acc.y)));
    acc.x = fold(sub<B32>(sub<B16>(sqr(R2), J), x2(V)));
    acc.y = mul2(R2, sub<B16>(V, acc.x), neg<B32>(x2(acc.y)), J);
    return true;
}

// ------------------------------------------------------------------------- XYZZ (round 6)
// Extended Jacobian "XYZZ" coordinates: x = X / ZZ, y = Y / ZZZ with ZZ^3 = ZZZ^2 (ZZ = Z^2,
// ZZZ = Z^3 for a Z that is never formed).  The accumulation's mixed addition (madd-2008-s) is
// 6M + 2S + one lazy mul2 against madd-2007-bl's 6M + 3S + mul2 -- one squaring (~370 of ~4700
// instructions) fewer per contribution -- and the full addition (add-2008-s) 10M + 2S + mul2
// against add-2007-bl's 10M + 4S + mul2.  The chunk's second point (mmadd: ZZ = PP, ZZZ = PPP) costs
// the same as the Jacobian one.  Partials leave the accumulation in XYZZ words (4 x 48 B); the
// bucket sums add them in XYZZ and convert each bucket sum once (x_to_jac) for the reduction.
// Invariant between steps: x, y folded (normalised, < 3p); zz, zzz normalised (< 3p).  The limb
// bounds of every step are restated in tests/limbs_model.py (_fq28_formulas) and pinned at their
// extremes by tests/test_gpu_limbs.py; largest column: mul2's R (carried) x (Q - X3 against B16)
// plus neg<B16>(y) x PPP, < 2^62.4.
struct X28 {
    F28 x, y, zz, zzz;
    MBLS_DEV bool is_inf() const {
        uint32_t t = 0;
#pragma unroll
        for (int i = 0; i < NL; ++i) t |= zz.l[i];
        return t == 0;  // infinity is exactly zz = 0 (set, never computed)
    }
    MBLS_DEV static X28 inf() { return {F28::one(), F28::one(), F28::zero(), F28::zero()}; }
};

// dbl-2008-s-1 (a = 0; exceptional path only: P == Q inside a bucket)
MBLS_DEV void xdbl(X28& a) {
    const F28 U = x2(a.y);  // limbs < 2^29
    const F28 V = sqr(U);
    const F28 W = mul(U, V);
    const F28 S = mul(a.x, V);
    const F28 A = sqr(a.x);
    const F28 M = add(x2(A), A);  // 3 X^2: limbs < 3 2^28
    const F28 X3 = fold(sub<B32>(sqr(M), x2(S)));
    a.y = mul2(M, sub<B16>(S, X3), neg<B16>(a.y), W);
    a.x = X3;
    a.zz = mul(V, a.zz);
    a.zzz = mul(W, a.zzz);
}

// acc + q, q = (x2, y2) affine from unpack_shift8 (< 256 p, normalised; y2 may be neg<B512> of one:
// < 512 p, limbs < 2^30.4), not the identity: madd-2008-s with the lazy Y3.  Park: as madd.
template <class Park>
MBLS_DEV void xmadd(X28& acc, const F28& x2_, const F28& y2_, Park& pk) {
    if (acc.is_inf()) {
        acc = {fold(x2_), fold(y2_), F28::one(), F28::one()};
        return;
    }
    const F28 U2 = mul(x2_, acc.zz);
    const F28 S2 = mul(y2_, acc.zzz);
    const F28 Pd = sub<B16>(U2, acc.x);          // limbs < 2^29.6
    const F28 R = carry(sub<B16>(S2, acc.y));    // normalised but the top limb
    pk.put(1, acc.y);
    const F28 PP = sqr(Pd);
    if (is_zero_lt2p(PP)) {  // U2 == X mod p: equal or opposite points
        acc.y = pk.get(1);
        if (is_zero_mod(R))
            xdbl(acc);
        else
            acc = X28::inf();
        return;
    }
    // ordered for register pressure: zz dies at ZZ3, P at PPP, zzz at ZZZ3, x and PP at Q
    acc.zz = mul(acc.zz, PP);
    const F28 PPP = mul(Pd, PP);
    acc.zzz = mul(acc.zzz, PPP);
    const F28 Q = mul(acc.x, PP);
    acc.x = fold(sub<B32>(sub<B16>(sqr(R), PPP), x2(Q)));
    acc.y = mul2(R, sub<B16>(Q, acc.x), neg<B16>(pk.get(1)), PPP);
}
MBLS_DEV void xmadd(X28& acc, const F28& x2_, const F28& y2_) {
    ParkReg pk;
    xmadd(acc, x2_, y2_, pk);
}

// acc fresh from the chunk's first point (zz = zzz = R'-one, x, y folded) + q: ZZ = PP, ZZZ = PPP.
// Returns false (acc untouched) when x1 == x2 mod p, left to xmadd's branches.
MBLS_DEV bool xmmadd(X28& acc, const F28& x2_, const F28& y2_) {
    const F28 Pd = fold(sub<B512>(x2_, acc.x));
    const F28 PP = sqr(Pd);
    if (is_zero_lt2p(PP)) return false;
    const F28 R = fold(sub<B512>(y2_, acc.y));  // limbs < 2^31.4 before the fold
    const F28 PPP = mul(Pd, PP);
    const F28 Q = mul(acc.x, PP);
    const F28 X3 = fold(sub<B32>(sub<B16>(sqr(R), PPP), x2(Q)));
    acc.y = mul2(R, sub<B16>(Q, X3), neg<B16>(acc.y), PPP);
    acc.x = X3;
    acc.zz = PP;
    acc.zzz = PPP;
    return true;
}

// acc + a partial (x2, y2, zz2, zzz2), each normalised and < 256 p (unpack_shift8 of words, or a
// stored accumulator's raw limbs: < 3p), zz2 != 0:
// add-2008-s with the lazy Y3
MBLS_DEV void xadd(X28& acc, const F28& x2_, const F28& y2_, const F28& zz2, const F28& zzz2) {
    if (acc.is_inf()) {
        acc = {fold(x2_), fold(y2_), fold(zz2), fold(zzz2)};
        return;
    }
    const F28 U1 = mul(acc.x, zz2);
    const F28 U2 = mul(x2_, acc.zz);
    const F28 S1 = mul(acc.y, zzz2);
    const F28 S2 = mul(y2_, acc.zzz);
    const F28 Pd = sub<B16>(U2, U1);
    const F28 R = carry(sub<B16>(S2, S1));
    const F28 PP = sqr(Pd);
    if (is_zero_lt2p(PP)) {  // equal or opposite points
        if (is_zero_mod(R))
            xdbl(acc);
        else
            acc = X28::inf();
        return;
    }
    const F28 PPP = mul(Pd, PP);
    const F28 Q = mul(U1, PP);
    acc.zz = mul(mul(acc.zz, zz2), PP);
    acc.zzz = mul(mul(acc.zzz, zzz2), PPP);
    acc.x = fold(sub<B32>(sub<B16>(sqr(R), PPP), x2(Q)));
    acc.y = mul2(R, sub<B16>(Q, acc.x), neg<B16>(S1), PPP);
}

// XYZZ -> Jacobian with Z = ZZZ: (X ZZ^2, Y ZZZ^2, ZZZ) (x = X ZZ^2 / ZZ^3, y = Y ZZZ^2 / ZZZ^3)
MBLS_DEV J28 x_to_jac(const X28& a) {
    if (a.is_inf()) return J28::inf();
    return {mul(a.x, sqr(a.zz)), mul(a.y, sqr(a.zzz)), a.zzz};
}

}  // namespace r28
}  // namespace mbls
