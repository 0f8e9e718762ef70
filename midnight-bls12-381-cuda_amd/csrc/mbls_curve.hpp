// mbls_curve.hpp -- G1 / G2 point arithmetic for CDNA4.
//
// Semantics follow the reference (bls12-381/include/point.cuh): short Weierstrass a = 0,
// G1: y^2 = x^3 + 4 over Fq, G2: y^2 = x^3 + 4(1+u) over Fq2; affine identity (0, 0)
// (point.cuh:287-318), Jacobian (X, Y, Z) with x = X/Z^2, y = Y/Z^3 and identity Z = 0
// (point.cuh:456-525).  Formulas: dbl-2009-l, add-2007-bl, madd-2007-bl (point.cuh:610-1250).
// Unlike the reference these are NOT constant-time: the exceptional cases (P == Q, P == -Q,
// identity) branch.  A sort-based Pippenger already leaks digit patterns through its memory
// schedule, so the constant-time formulas buy nothing on this path.
#pragma once
#include "mbls_field.hpp"
#include "mbls_pairfield.hpp"

namespace mbls {

template <class F>
struct Affine {
    F x, y;
    MBLS_DEV bool is_inf() const { return x.is_zero() && y.is_zero(); }
    MBLS_DEV static Affine inf() { return {F::zero(), F::zero()}; }
};

template <class F>
struct Jacobian {
    F x, y, z;
    MBLS_DEV bool is_inf() const { return z.is_zero(); }
    MBLS_DEV static Jacobian inf() { return {F::one(), F::one(), F::zero()}; }
    MBLS_DEV static Jacobian from_affine(const Affine<F>& a) {
        if (a.is_inf()) return inf();
        return {a.x, a.y, F::one()};
    }
};

// Where a square costs less than a product (the lane types: FIPS squaring computes each cross
// product once) the formulas trade products for squares plus additions; the row-sliced types
// square with a full product, so there the plain product saves the additions (mbls_rowfield.hpp
// specialises this to false).  Same values either way.
template <class F>
struct SqrCheaper {
    static constexpr bool value = true;
};
// x2_in / x4_in / x8_in are free-standing shifts (no reduction) and a square costs a full
// product: G1 rows (mbls_rowfield.hpp specialises this for RFq)
template <class F>
struct ShiftOperands {
    static constexpr bool value = false;
};

template <class F>
MBLS_DEV Jacobian<F> jac_dbl(const Jacobian<F>& p) {
    // dbl-2009-l: 2M + 5S
    if (p.is_inf()) return p;
    F A = sqr(p.x);
    F B = sqr(p.y);
    F E = add_in(x2_in(A), A);  // 3A: feeds the products E^2 and E (D - X3) only
    F Fv = sqr(E);
    Jacobian<F> r;
    if constexpr (SqrCheaper<F>::value) {
        F C = sqr(B);
        F D = dbl(sqr(add_in(p.x, B)) - A - C);  // 2((X + B)^2 - A - C) = 4 X B
        r.x = Fv - dbl(D);
        F C8 = dbl(dbl(dbl(C)));
        r.y = E * (D - r.x) - C8;
        r.z = dbl(p.y * p.z);
    } else {
        // row types: a square is a full product, and the constant factors ride on unreduced
        // operands (x4_in, x8_in, x2_in: shifts) instead of reduced doublings of the results
        F D = x4_in(p.x) * B;  // 4 X B
        F C8;                  // 8 C = 8 B^2
        if constexpr (ShiftOperands<F>::value)
            C8 = x8_in(B) * B;
        else
            C8 = dbl(dbl(dbl(sqr(B))));  // Fq2: a square is 2 Fq products, a product 3
        r.x = Fv - dbl(D);
        r.y = E * (D - r.x) - C8;
        r.z = x2_in(p.y) * p.z;  // 2 Y Z
    }
    return r;
}

// All point operations are inlined; kernels keep ONE call site per operation inside their
// loops (code size: one Fq product is ~1.3 K instructions), see msm_core.hpp.
template <class F>
MBLS_DEV Jacobian<F> jac_add(const Jacobian<F>& p, const Jacobian<F>& q) {
    // add-2007-bl: 11M + 5S
    if (p.is_inf()) return q;
    if (q.is_inf()) return p;
    F Z1Z1 = sqr(p.z);
    F Z2Z2 = sqr(q.z);
    F U1 = p.x * Z2Z2;
    F U2 = q.x * Z1Z1;
    F S1 = p.y * q.z * Z2Z2;
    F S2 = q.y * p.z * Z1Z1;
    F H = U2 - U1;
    F R = S2 - S1;
    if (H.is_zero()) {
        if (R.is_zero()) return jac_dbl(p);
        return Jacobian<F>::inf();
    }
    // 2H, 2R and Z1 + Z2 feed products only: unreduced operands (add_in, mbls_field.hpp)
    F I = sqr(x2_in(H));
    F J = H * I;
    R = x2_in(R);
    F V = U1 * I;
    Jacobian<F> r;
    r.x = sqr(R) - J - dbl(V);
    if constexpr (SqrCheaper<F>::value) {
        r.y = mul_sum(R, V - r.x, neg(dbl(S1)), J);
        r.z = (sqr(add_in(p.z, q.z)) - Z1Z1 - Z2Z2) * H;  // 2 Z1 Z2 H
    } else {
        r.y = R * (V - r.x) - x2_in(S1) * J;  // row types: one subtraction, 2 S1 as a shift
        r.z = x2_in(p.z * q.z) * H;
    }
    return r;
}

template <class F>
MBLS_DEV Jacobian<F> jac_madd(const Jacobian<F>& p, const Affine<F>& q) {
    // madd-2007-bl: 7M + 4S
    if (q.is_inf()) return p;
    if (p.is_inf()) return Jacobian<F>::from_affine(q);
    F Z1Z1 = sqr(p.z);
    F U2 = q.x * Z1Z1;
    F S2 = q.y * p.z * Z1Z1;
    F H = U2 - p.x;
    F R = S2 - p.y;
    if (H.is_zero()) {
        if (R.is_zero()) return jac_dbl(p);
        return Jacobian<F>::inf();
    }
    F HH = sqr(H);
    // 4HH, 2R and Z1 + H feed products only: unreduced operands (add_in, mbls_field.hpp)
    F I = x4_in(HH);
    F J = H * I;
    R = x2_in(R);
    F V = p.x * I;
    Jacobian<F> r;
    r.x = sqr(R) - J - dbl(V);
    r.y = mul_sum(R, V - r.x, neg(dbl(p.y)), J);
    r.z = sqr(add_in(p.z, H)) - Z1Z1 - HH;
    return r;
}

// affine + affine (p.z == 1): mmadd-2007-bl, 4M + 2S with Y3 as one lazy product sum -- the
// formula madd-2007-bl reduces to at Z1 = 1 (Z1Z1 = 1, U2 = X2, S2 = Y2, Z3 = (1 + H)^2 - 1 - HH
// = 2H), so the result is the same projective representative jac_madd returns.  The second
// point of every accumulation chunk meets an accumulator fresh from its first point.  Returns
// false (r untouched) when x1 == x2 (equal or opposite points), left to jac_madd's branches.
template <class F>
MBLS_DEV bool jac_mmadd(const Jacobian<F>& p, const Affine<F>& q, Jacobian<F>& r) {
    const F H = q.x - p.x;
    if (H.is_zero()) return false;
    const F HH = sqr(H);
    const F I = x4_in(HH);
    const F J = H * I;
    const F R = x2_in(q.y - p.y);
    const F V = p.x * I;
    r.x = sqr(R) - J - dbl(V);
    r.y = mul_sum(R, V - r.x, neg(dbl(p.y)), J);
    r.z = dbl(H);
    return true;
}

template <class F>
MBLS_DEV Affine<F> aff_neg(const Affine<F>& a) {
    if (a.is_inf()) return a;
    return {a.x, neg(a.y)};
}

template <class F>
MBLS_DEV Jacobian<F> jac_neg(const Jacobian<F>& a) {
    return {a.x, neg(a.y), a.z};
}

template <class F>
MBLS_DEV Affine<F> jac_to_affine(const Jacobian<F>& p) {
    if (p.is_inf()) return Affine<F>::inf();
    F zi = inv(p.z);
    F zi2 = sqr(zi);
    return {p.x * zi2, p.y * zi2 * zi};
}

// k * P, k a standard-form 256-bit scalar as 8 x u32 (LSB first); one add site
template <class F>
MBLS_DEV Jacobian<F> jac_mul_u32(const Jacobian<F>& p, const uint32_t (&k)[8]) {
    Jacobian<F> acc = Jacobian<F>::inf();
    for (int i = 255; i >= 0; --i) {
        acc = jac_dbl(acc);
        uint32_t word = 0;
#pragma unroll
        for (int w = 0; w < 8; ++w) word = (w == (i >> 5)) ? k[w] : word;
        if ((word >> (i & 31)) & 1) acc = jac_add(acc, p);
    }
    return acc;
}

// ------------------------------------------------------------------------------------
// memory helpers: F = Fq (48 B) or Fq2 (96 B)
// ------------------------------------------------------------------------------------
template <class F>
struct FieldIO;

template <>
struct FieldIO<Fq> {
    static constexpr int BYTES = 48;
    MBLS_DEV static Fq ld(const uint8_t* p) { return load<FqCfg>(p); }
    MBLS_DEV static void st(uint8_t* p, const Fq& v) { store<FqCfg>(p, v); }
};

template <>
struct FieldIO<Fq2> {
    static constexpr int BYTES = 96;
    MBLS_DEV static Fq2 ld(const uint8_t* p) { return {load<FqCfg>(p), load<FqCfg>(p + 48)}; }
    MBLS_DEV static void st(uint8_t* p, const Fq2& v) {
        store<FqCfg>(p, v.c0);
        store<FqCfg>(p + 48, v.c1);
    }
};

// pair-sliced Fq2: same 96-byte storage, lane j moves the 48 bytes of component j
template <>
struct FieldIO<PFq2> {
    static constexpr int BYTES = 96;
    MBLS_DEV static PFq2 ld(const uint8_t* p) { return {load<FqCfg>(p + (pairdpp::odd() ? 48 : 0))}; }
    MBLS_DEV static void st(uint8_t* p, const PFq2& v) { store<FqCfg>(p + (pairdpp::odd() ? 48 : 0), v.v); }
};

// element type of the one-chain-per-thread ("lane") kernels: G1 uses Fq in one lane, G2 the
// pair-sliced Fq2 in two lanes (mbls_pairfield.hpp)
template <class F>
struct LaneOf {
    using type = F;
    static constexpr uint32_t LANES = 1;
};
template <>
struct LaneOf<Fq2> {
    using type = PFq2;
    static constexpr uint32_t LANES = 2;
};

template <class F>
MBLS_DEV Affine<F> load_affine(const void* base, size_t idx) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(base) + idx * (2 * FieldIO<F>::BYTES);
    return {FieldIO<F>::ld(p), FieldIO<F>::ld(p + FieldIO<F>::BYTES)};
}

template <class F>
MBLS_DEV void store_affine(void* base, size_t idx, const Affine<F>& a) {
    uint8_t* p = reinterpret_cast<uint8_t*>(base) + idx * (2 * FieldIO<F>::BYTES);
    FieldIO<F>::st(p, a.x);
    FieldIO<F>::st(p + FieldIO<F>::BYTES, a.y);
}

template <class F>
MBLS_DEV Jacobian<F> load_jac(const void* base, size_t idx) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(base) + idx * (3 * FieldIO<F>::BYTES);
    return {FieldIO<F>::ld(p), FieldIO<F>::ld(p + FieldIO<F>::BYTES), FieldIO<F>::ld(p + 2 * FieldIO<F>::BYTES)};
}

template <class F>
MBLS_DEV void store_jac(void* base, size_t idx, const Jacobian<F>& a) {
    uint8_t* p = reinterpret_cast<uint8_t*>(base) + idx * (3 * FieldIO<F>::BYTES);
    FieldIO<F>::st(p, a.x);
    FieldIO<F>::st(p + FieldIO<F>::BYTES, a.y);
    FieldIO<F>::st(p + 2 * FieldIO<F>::BYTES, a.z);
}

// generators (Montgomery form) -- reference bls12_381_constants.h:147-224
MBLS_DEV Affine<Fq> g1_generator() {
    const uint32_t X[12] = {0xfd530c16u, 0x5cb38790u, 0x9976fff5u, 0x7817fc67u, 0x143ba1c1u, 0x154f95c7u,
                            0xf3d0e747u, 0xf0ae6acdu, 0x21dbf440u, 0xedce6eccu, 0x9e0bfb75u, 0x12017741u};
    const uint32_t Y[12] = {0x0ce72271u, 0xbaac93d5u, 0x7918fd8eu, 0x8c22631au, 0x570725ceu, 0xdd595f13u,
                            0x50405194u, 0x51ac5829u, 0xad0059c0u, 0x0e1c8c3fu, 0x5008a26au, 0x0bbc3efcu};
    Affine<Fq> g;
    for (int i = 0; i < 12; ++i) {
        g.x.v[i] = X[i];
        g.y.v[i] = Y[i];
    }
    return g;
}

MBLS_DEV Affine<Fq2> g2_generator() {
    const uint32_t X0[12] = {0x02940a10u, 0xf5f28fa2u, 0x87b4961au, 0xb3f5fb26u, 0x3e2ae580u, 0xa1a893b5u,
                             0x1a3caee9u, 0x9894999du, 0x1863366bu, 0x6f67b763u, 0x4350bcd7u, 0x05819192u};
    const uint32_t X1[12] = {0x9e23f606u, 0xa5a9c075u, 0xbccd60c3u, 0xaaa0c59du, 0xe2867806u, 0x3bb17e18u,
                             0x8541b367u, 0x1b1ab6ccu, 0xf2158547u, 0xc2b6ed0eu, 0x7360edf3u, 0x11922a09u};
    const uint32_t Y0[12] = {0x60494c4au, 0x4c730af8u, 0x5e369c5au, 0x597cfa1fu, 0xaa0a635au, 0xe7e6856cu,
                             0x6e0d495fu, 0xbbefb5e9u, 0xf0ef25a2u, 0x07d3a975u, 0x7e80dae5u, 0x0083fd8eu};
    const uint32_t Y1[12] = {0xdf64b05du, 0xadc0fc92u, 0x2b1461dcu, 0x18aa270au, 0x3be4eba0u, 0x86adac6au,
                             0xc93da33au, 0x79495c4eu, 0xa43ccaedu, 0xe7175850u, 0x63de1bf2u, 0x0b2bc2a1u};
    Affine<Fq2> g;
    for (int i = 0; i < 12; ++i) {
        g.x.c0.v[i] = X0[i];
        g.x.c1.v[i] = X1[i];
        g.y.c0.v[i] = Y0[i];
        g.y.c1.v[i] = Y1[i];
    }
    return g;
}

}  // namespace mbls
