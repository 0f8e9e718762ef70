// mbls_field.hpp -- BLS12-381 Fr / Fq / Fq2 arithmetic for CDNA4 (gfx950).
//
// Storage layout in HBM is the reference's / blst's: little-endian u64 limbs, canonical
// Montgomery values (Fr 32 B, Fq 48 B, Fq2 = c0||c1 96 B) -- reference
// bls12-381/include/field.cuh:197-326, core/types.rs:89-108.
//
// In registers a value is N x u32 limbs (Fr N=8, Fq N=12): CDNA4 has no 64x64->128 multiply,
// but v_mad_u64_u32 (32x32 + 64 -> 64) and the 64-bit add v_lshl_add_u64, so Montgomery
// multiplication is a CIOS over 32-bit words where every step is one v_mad_u64_u32 plus one
// 64-bit add.  Both moduli leave the top bit of the top word clear (p < 2^381, r < 2^255), so
// the "no-carry" CIOS variant applies: the running value never needs an (N+1)-th word and the
// result is < 2m before one final conditional subtraction.  Outputs are canonical, i.e. the
// exact limbs blst / the reference produce (field.cuh:510-576 semantics).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MBLS_DEV __device__ __forceinline__
#define MBLS_HD __host__ __device__ __forceinline__

namespace mbls {

// ------------------------------------------------------------------------------------
// field configurations (32-bit little-endian words)
// ------------------------------------------------------------------------------------
struct FrCfg {
    static constexpr int N = 8;
    // r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    static constexpr uint32_t MOD[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                        0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
    static constexpr uint32_t NINV = 0xffffffffu;  // -r^-1 mod 2^32
    static constexpr uint32_t ONE[8] = {0xfffffffeu, 0x00000001u, 0x00034802u, 0x5884b7fau,
                                        0xecbc4ff5u, 0x998c4fefu, 0xacc5056fu, 0x1824b159u};
    static constexpr uint32_t R2[8] = {0xf3f29c6du, 0xc999e990u, 0x87925c23u, 0x2b6cedcbu,
                                       0x7254398fu, 0x05d31496u, 0x9f59ff11u, 0x0748d9d9u};
};

struct FqCfg {
    static constexpr int N = 12;
    static constexpr uint32_t MOD[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu,
                                         0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u,
                                         0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
    static constexpr uint32_t NINV = 0xfffcfffdu;  // -p^-1 mod 2^32
    static constexpr uint32_t ONE[12] = {0x0002fffdu, 0x76090000u, 0xc40c0002u, 0xebf4000bu,
                                         0x53c758bau, 0x5f489857u, 0x70525745u, 0x77ce5853u,
                                         0xa256ec6du, 0x5c071a97u, 0xfa80e493u, 0x15f65ec3u};
    static constexpr uint32_t R2[12] = {0x1c341746u, 0xf4df1f34u, 0x09d104f1u, 0x0a76e6a6u,
                                        0x4c95b6d5u, 0x8de5476cu, 0x939d83c0u, 0x67eb88a9u,
                                        0xb519952du, 0x9a793e85u, 0x92cae3aau, 0x11988fe5u};
};

// ------------------------------------------------------------------------------------
// generic prime-field element
// ------------------------------------------------------------------------------------
template <class C>
struct Fp {
    static constexpr int N = C::N;
    uint32_t v[N];

    MBLS_DEV static Fp zero() {
        Fp r;
#pragma unroll
        for (int i = 0; i < N; ++i) r.v[i] = 0;
        return r;
    }
    MBLS_DEV static Fp one() {
        Fp r;
#pragma unroll
        for (int i = 0; i < N; ++i) r.v[i] = C::ONE[i];
        return r;
    }
    MBLS_DEV static Fp r2() {
        Fp r;
#pragma unroll
        for (int i = 0; i < N; ++i) r.v[i] = C::R2[i];
        return r;
    }
    MBLS_DEV bool is_zero() const {
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < N; ++i) x |= v[i];
        return x == 0;
    }
    MBLS_DEV bool operator==(const Fp& o) const {
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < N; ++i) x |= v[i] ^ o.v[i];
        return x == 0;
    }
};

using Fr = Fp<FrCfg>;
using Fq = Fp<FqCfg>;

// raw forms for Fq (see add_in above): a, b canonical (or the stated bounds) -> no reduction
static_assert(FqCfg::MOD[11] < (1u << 29), "Fq raw operand bounds assume p < 2^381");
MBLS_DEV Fq add_in(const Fq& a, const Fq& b) {
    Fq r;
    unsigned carry = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) r.v[i] = __builtin_addc(a.v[i], b.v[i], carry, &carry);
    return r;
}
MBLS_DEV Fq x2_in(const Fq& a) {
    Fq r;
    r.v[0] = a.v[0] << 1;
#pragma unroll
    for (int i = 1; i < 12; ++i) r.v[i] = __builtin_amdgcn_alignbit(a.v[i], a.v[i - 1], 31);
    return r;
}
// p - a for canonical a: in (0, p], congruent to -a (an operand of a product only)
MBLS_DEV Fq neg_in(const Fq& a) {
    Fq r;
    unsigned borrow = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) r.v[i] = __builtin_subc(FqCfg::MOD[i], a.v[i], borrow, &borrow);
    return r;
}
MBLS_DEV Fq x4_in(const Fq& a) {
    Fq r;
    r.v[0] = a.v[0] << 2;
#pragma unroll
    for (int i = 1; i < 12; ++i) r.v[i] = __builtin_amdgcn_alignbit(a.v[i], a.v[i - 1], 30);
    return r;
}

// Carry chains use __builtin_addc / __builtin_subc, which lower to one v_add_co/v_addc
// (v_sub_co/v_subb) per word; the 64-bit C formulation produced ~3x the instructions
// (v_mov + v_lshl_add_u64 per word, measured on an Fq add: 148 vs 53 VALU instructions).

// (a - m) with borrow; returns 1 if a < m
template <class C>
MBLS_DEV uint32_t sub_mod_raw(uint32_t (&r)[C::N], const uint32_t (&a)[C::N]) {
    unsigned borrow = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) r[i] = __builtin_subc(a[i], C::MOD[i], borrow, &borrow);
    return borrow;
}

// conditional final subtraction: a in [0, 2m) -> [0, m)
template <class C>
MBLS_DEV void reduce_once(Fp<C>& a) {
    uint32_t t[C::N];
    uint32_t borrow = sub_mod_raw<C>(t, a.v);
#pragma unroll
    for (int i = 0; i < C::N; ++i) a.v[i] = borrow ? a.v[i] : t[i];
}

template <class C>
MBLS_DEV Fp<C> operator+(const Fp<C>& a, const Fp<C>& b) {
    Fp<C> r;
    unsigned carry = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = __builtin_addc(a.v[i], b.v[i], carry, &carry);
    // both moduli < 2^(32N-1): a+b < 2m fits in N words, carry == 0
    reduce_once(r);
    return r;
}

template <class C>
MBLS_DEV Fp<C> operator-(const Fp<C>& a, const Fp<C>& b) {
    Fp<C> r;
    unsigned borrow = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = __builtin_subc(a.v[i], b.v[i], borrow, &borrow);
    // add m back if negative (mask form keeps the wave convergent)
    const uint32_t mask = 0u - borrow;
    unsigned carry = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = __builtin_addc(r.v[i], C::MOD[i] & mask, carry, &carry);
    return r;
}

template <class C>
MBLS_DEV Fp<C> neg(const Fp<C>& a) {
    return Fp<C>::zero() - a;
}

template <class C>
MBLS_DEV Fp<C> dbl(const Fp<C>& a) {
    return a + a;
}

// Unreduced sums for operands that ONLY feed products (add_in, x2_in, x4_in).  A Montgomery
// product with a * b < m R returns < 2m and its conditional subtraction makes it canonical, and
// the squaring wants a < 2^(32N - 1) (mbls_fips.hpp).  For Fq (p < 0.82 * 2^381) an operand up
// to 4p with a canonical partner, or two operands up to 3p, stay inside both bounds, so these
// skip the conditional subtraction (or two) a reduced sum costs.  Other field types reduce.
template <class F>
MBLS_DEV F add_in(const F& a, const F& b) { return a + b; }
template <class F>
MBLS_DEV F x2_in(const F& a) { return dbl(a); }
template <class F>
MBLS_DEV F x4_in(const F& a) { return dbl(dbl(a)); }
template <class F>
MBLS_DEV F x8_in(const F& a) { return dbl(dbl(dbl(a))); }

// Montgomery product a*b*2^(-32N) mod m -- no-carry CIOS, every word step is
// v_mad_u64_u32 + one 64-bit add.  Reference implementation; the hot paths use the
// product-scanning form in mbls_fips.hpp (operator* below), 1.4-1.5x faster on gfx950.
template <class C>
MBLS_DEV Fp<C> mul_cios(const Fp<C>& a, const Fp<C>& b) {
    constexpr int N = C::N;
    uint32_t t[N];
#pragma unroll
    for (int i = 0; i < N; ++i) t[i] = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint32_t bi = b.v[i];
        uint64_t A = (uint64_t)a.v[0] * bi + t[0];
        const uint32_t t0 = (uint32_t)A;
        const uint32_t m = t0 * C::NINV;
        uint64_t Cc = (uint64_t)m * C::MOD[0] + t0;
#pragma unroll
        for (int j = 1; j < N; ++j) {
            A = (uint64_t)a.v[j] * bi + ((uint64_t)t[j] + (A >> 32));
            Cc = (uint64_t)m * C::MOD[j] + ((uint64_t)(uint32_t)A + (Cc >> 32));
            t[j - 1] = (uint32_t)Cc;
        }
        t[N - 1] = (uint32_t)(Cc >> 32) + (uint32_t)(A >> 32);
    }
    Fp<C> r;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = t[i];
    reduce_once(r);
    return r;
}

}  // namespace mbls
#include "mbls_fips.hpp"
#include "mbls_binv.hpp"
#include "mbls_binv_quad.hpp"
namespace mbls {

template <class C>
MBLS_DEV Fp<C> operator*(const Fp<C>& a, const Fp<C>& b) {
    return fips::mul(a, b);
}

template <class C>
MBLS_DEV Fp<C> sqr(const Fp<C>& a) {
    return fips::sqr(a);
}

#ifndef MBLS_LAZY
#define MBLS_LAZY 1
#endif
// a*b + c*d.  Generic form for the row-sliced / extension types; prime-field elements use one
// shared Montgomery reduction (fips::mul2).
template <class F>
MBLS_DEV F mul_sum(const F& a, const F& b, const F& c, const F& d) {
    return a * b + c * d;
}
template <class C>
MBLS_DEV Fp<C> mul_sum(const Fp<C>& a, const Fp<C>& b, const Fp<C>& c, const Fp<C>& d) {
#if MBLS_LAZY
    return fips::mul2(a, b, c, d);
#else
    return a * b + c * d;
#endif
}

template <class C>
MBLS_DEV Fp<C> to_mont(const Fp<C>& a) {
    return a * Fp<C>::r2();
}

template <class C>
MBLS_DEV Fp<C> from_mont(const Fp<C>& a) {
    Fp<C> one = Fp<C>::zero();
    one.v[0] = 1;
    return a * one;
}

// a^e for a compile-time-free exponent given as 32-bit words (square-and-multiply, MSB first)
template <class C, int EW>
MBLS_DEV Fp<C> pow_words(const Fp<C>& a, const uint32_t (&e)[EW]) {
    Fp<C> acc = Fp<C>::one();
    for (int w = EW - 1; w >= 0; --w) {
        for (int b = 31; b >= 0; --b) {
            acc = sqr(acc);
            if ((e[w] >> b) & 1) acc = acc * a;
        }
    }
    return acc;
}

// Fermat inversion a^(m-2); 0 -> 0 (reference field.cuh:750-900 semantics).  Kept for the
// row-sliced types and as the cross-check of inv() below.
template <class C>
MBLS_DEV Fp<C> inv_fermat(const Fp<C>& a) {
    uint32_t e[C::N];
#pragma unroll
    for (int i = 0; i < C::N; ++i) e[i] = C::MOD[i];
    // m - 2 with borrow: r's low word is 0x00000001
    uint32_t br = 2;
#pragma unroll
    for (int i = 0; i < C::N; ++i) {
        const uint32_t d = e[i] - br;
        br = e[i] < br ? 1u : 0u;
        e[i] = d;
    }
    return pow_words<C, C::N>(a, e);
}

// Inversion by the batched binary GCD (mbls_binv.hpp; variable time -- used only on public
// data: the MSM result normalisation and G2 norms; the Fr batch inversion, whose
// inputs may be witness-derived, keeps the fixed Fermat chain, vecops.hip): full-rate word
// operations plus ~100 small-factor word products per 30 steps, where the Fermat chain above
// is ~570 serial Montgomery products.  The input's Montgomery limbs are inverted as an
// integer, (aR)^-1, then one product with R^3 (= R2 * R2 in Montgomery form) gives a^-1 R.
// The input is reduced once first (a value in [0, 2m), e.g. the non-canonical zero m, is a
// valid input; the GCD needs 1 <= y < m).  0 -> 0 (field.cuh:750-900 semantics).
template <class C>
MBLS_DEV Fp<C> inv(const Fp<C>& a_in) {
    constexpr int N = C::N;
    Fp<C> a = a_in;
    reduce_once(a);
    if (a.is_zero()) return a;
    uint32_t m[N];
#pragma unroll
    for (int i = 0; i < N; ++i) m[i] = C::MOD[i];
    Fp<C> x;
    binv::inverse<N>(x.v, a.v, m, C::NINV);
    const Fp<C> r2 = Fp<C>::r2();
    return x * (r2 * r2);
}

// ------------------------------------------------------------------------------------
// HBM <-> register movement (u64 limbs in memory, u32 in registers: same bytes)
// ------------------------------------------------------------------------------------
template <class C>
MBLS_DEV Fp<C> load(const void* p) {
    static_assert(C::N % 4 == 0, "16-byte vector loads");
    Fp<C> r;
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int i = 0; i < C::N / 4; ++i) {
        uint4 x = q[i];
        r.v[4 * i + 0] = x.x;
        r.v[4 * i + 1] = x.y;
        r.v[4 * i + 2] = x.z;
        r.v[4 * i + 3] = x.w;
    }
    return r;
}

template <class C>
MBLS_DEV void store(void* p, const Fp<C>& a) {
    uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
    for (int i = 0; i < C::N / 4; ++i) q[i] = make_uint4(a.v[4 * i], a.v[4 * i + 1], a.v[4 * i + 2], a.v[4 * i + 3]);
}

// non-temporal streaming variants (data touched once)
template <class C>
MBLS_DEV Fp<C> load_nt(const void* p) {
    Fp<C> r;
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = __builtin_nontemporal_load(q + i);
    return r;
}

// ------------------------------------------------------------------------------------
// Fq2 = Fq[u] / (u^2 + 1)   (reference point.cuh:131-225)
// ------------------------------------------------------------------------------------
struct Fq2 {
    Fq c0, c1;
    MBLS_DEV static Fq2 zero() { return {Fq::zero(), Fq::zero()}; }
    MBLS_DEV static Fq2 one() { return {Fq::one(), Fq::zero()}; }
    MBLS_DEV bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
    MBLS_DEV bool operator==(const Fq2& o) const { return c0 == o.c0 && c1 == o.c1; }
};

MBLS_DEV Fq2 operator+(const Fq2& a, const Fq2& b) { return {a.c0 + b.c0, a.c1 + b.c1}; }
MBLS_DEV Fq2 operator-(const Fq2& a, const Fq2& b) { return {a.c0 - b.c0, a.c1 - b.c1}; }
MBLS_DEV Fq2 neg(const Fq2& a) { return {neg(a.c0), neg(a.c1)}; }
MBLS_DEV Fq2 dbl(const Fq2& a) { return {a.c0 + a.c0, a.c1 + a.c1}; }
// Karatsuba: 3 Fq products.  Out of line: a G2 point formula inlining ~16 of these (48 Fq
// products, ~60 K instructions) per call site made the G2 translation unit take ~25 min to
// compile; a call costs < 1% of the ~4 K instructions of the body.
__device__ __noinline__ Fq2 fq2_mul(const Fq2 a, const Fq2 b) {
    Fq t0 = a.c0 * b.c0;
    Fq t1 = a.c1 * b.c1;
    Fq t2 = (a.c0 + a.c1) * (b.c0 + b.c1);
    return {t0 - t1, (t2 - t0) - t1};
}
// (a0 + a1 u)^2 = (a0+a1)(a0-a1) + 2 a0 a1 u : 2 Fq products
__device__ __noinline__ Fq2 fq2_sqr(const Fq2 a) {
    Fq t = a.c0 * a.c1;
    return {(a.c0 + a.c1) * (a.c0 - a.c1), t + t};
}
MBLS_DEV Fq2 operator*(const Fq2& a, const Fq2& b) { return fq2_mul(a, b); }
MBLS_DEV Fq2 sqr(const Fq2& a) { return fq2_sqr(a); }
MBLS_DEV Fq2 inv(const Fq2& a) {
    Fq n = inv(sqr(a.c0) + sqr(a.c1));
    return {a.c0 * n, neg(a.c1 * n)};
}

// inv() on the four lanes of a DPP quad (all active, same input; mbls_binv_quad.hpp): the outer
// step's four 12-word updates run one per lane instead of one after the other
template <class C>
MBLS_DEV Fp<C> inv_quad(const Fp<C>& a_in) {
    constexpr int N = C::N;
    Fp<C> a = a_in;
    reduce_once(a);
    if (a.is_zero()) return a;
    uint32_t m[N];
#pragma unroll
    for (int i = 0; i < N; ++i) m[i] = C::MOD[i];
    Fp<C> x;
    binv::inverse_quad<N>(x.v, a.v, m, C::NINV);
    const Fp<C> r2 = Fp<C>::r2();
    return x * (r2 * r2);
}
MBLS_DEV Fq2 inv_quad(const Fq2& a) {
    Fq n = inv_quad(sqr(a.c0) + sqr(a.c1));
    return {a.c0 * n, neg(a.c1 * n)};
}

}  // namespace mbls
