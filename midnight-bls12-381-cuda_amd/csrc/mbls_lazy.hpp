// mbls_lazy.hpp -- "lazy" prime-field values in [0, 2m) for the bucket accumulation.
//
// k_accumulate runs at its VALU issue bound, so only fewer instructions per mixed
// addition help.  The canonical operators end every Montgomery product with a conditional
// subtraction of m (12 subtract-with-borrow + 12 selects); inside the accumulation chain the
// values only feed further products and additions, so they are kept in [0, 2m) instead:
//   * products:  a, b < 2m  =>  a b < 4 m^2 < m R  (4m < 2^384 for p), so the FIPS product
//     without its final subtraction returns (a b + q m) / R < 2m;
//   * product sums (mul2):  a b + c d < 8 m^2 < m R  (8p < 2^384), same bound;
//   * add / sub reduce against 2m instead of m (a + b < 4m < 2^384: no carry out);
//   * zero tests:  x == 0 (mod m)  <=>  x == 0 or x == m;
//   * the accumulator is made canonical (one conditional subtraction per coordinate) when it
//     is stored, so partials -- and everything downstream -- are bit-identical to the
//     canonical path.
// Only the prime field with 4m < 2^(32N) qualifies; Fq does (p < 2^381), the static_assert
// below checks the 8m bound for mul2 on the top word.
#pragma once
#include "mbls_curve.hpp"

namespace mbls {
namespace lz {

template <class C>
struct TwoM {
    uint32_t v[C::N];
    constexpr TwoM() : v() {
        for (int i = 0; i < C::N; ++i) v[i] = (C::MOD[i] << 1) | (i ? (C::MOD[i - 1] >> 31) : 0u);
    }
};
template <class C>
constexpr TwoM<C> TWO_M{};

static_assert(FqCfg::MOD[11] < (1u << 29), "8p < 2^384 (lazy product sums)");

template <class C>
MBLS_DEV Fp<C> mul(const Fp<C>& a, const Fp<C>& b) {
    return fips::mul<C, false>(a, b);
}
template <class C>
MBLS_DEV Fp<C> sqr(const Fp<C>& a) {
    return fips::sqr<C, false>(a);
}
template <class C>
MBLS_DEV Fp<C> mul2(const Fp<C>& a, const Fp<C>& b, const Fp<C>& c, const Fp<C>& d) {
    return fips::mul2<C, false>(a, b, c, d);
}

// (a + b) mod' 2m, a, b < 2m
template <class C>
MBLS_DEV Fp<C> add(const Fp<C>& a, const Fp<C>& b) {
    Fp<C> r, t;
    unsigned carry = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = __builtin_addc(a.v[i], b.v[i], carry, &carry);
    unsigned borrow = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) t.v[i] = __builtin_subc(r.v[i], TWO_M<C>.v[i], borrow, &borrow);
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = borrow ? r.v[i] : t.v[i];
    return r;
}

// (a - b) mod' 2m, a, b < 2m
template <class C>
MBLS_DEV Fp<C> sub(const Fp<C>& a, const Fp<C>& b) {
    Fp<C> r;
    unsigned borrow = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = __builtin_subc(a.v[i], b.v[i], borrow, &borrow);
    const uint32_t mask = 0u - borrow;
    unsigned carry = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = __builtin_addc(r.v[i], TWO_M<C>.v[i] & mask, carry, &carry);
    return r;
}

template <class C>
MBLS_DEV Fp<C> dbl(const Fp<C>& a) {
    return add(a, a);
}

// a == 0 (mod m) for a < 2m
template <class C>
MBLS_DEV bool is_zero(const Fp<C>& a) {
    uint32_t z = 0, e = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) {
        z |= a.v[i];
        e |= a.v[i] ^ C::MOD[i];
    }
    return z == 0 || e == 0;
}

template <class C>
MBLS_DEV Fp<C> canon(Fp<C> a) {
    reduce_once(a);
    return a;
}

template <class C>
MBLS_DEV Jacobian<Fp<C>> canon(const Jacobian<Fp<C>>& p) {
    return {canon(p.x), canon(p.y), canon(p.z)};
}

// madd-2007-bl (7M + 4S, Y3 as one lazy product sum) on lazy coordinates: p's coordinates in
// [0, 2m) with p.z == 0 exactly for the identity (Z3 = 2 Z1 H != 0 otherwise), q canonical
// affine.  Same branches as jac_madd; the doubling branch runs the canonical formula.
template <class C>
MBLS_DEV Jacobian<Fp<C>> madd(const Jacobian<Fp<C>>& p, const Affine<Fp<C>>& q) {
    using F = Fp<C>;
    if (q.is_inf()) return p;
    if (p.z.is_zero()) return Jacobian<F>::from_affine(q);
    const F Z1Z1 = lz::sqr(p.z);
    const F U2 = lz::mul(q.x, Z1Z1);
    const F S2 = lz::mul(lz::mul(q.y, p.z), Z1Z1);
    const F H = lz::sub(U2, p.x);
    F R = lz::sub(S2, p.y);
    if (lz::is_zero(H)) {
        if (lz::is_zero(R)) return jac_dbl(lz::canon(p));
        return Jacobian<F>::inf();
    }
    const F HH = lz::sqr(H);
    const F I = lz::dbl(lz::dbl(HH));
    const F J = lz::mul(H, I);
    R = lz::dbl(R);
    const F V = lz::mul(p.x, I);
    Jacobian<F> r;
    r.x = lz::sub(lz::sub(lz::sqr(R), J), lz::dbl(V));
    r.y = lz::mul2(R, lz::sub(V, r.x), lz::sub(F::zero(), lz::dbl(p.y)), J);
    r.z = lz::sub(lz::sub(lz::sqr(lz::add(p.z, H)), Z1Z1), HH);
    return r;
}

}  // namespace lz
}  // namespace mbls
