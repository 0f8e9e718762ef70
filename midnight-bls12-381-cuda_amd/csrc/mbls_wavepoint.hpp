// mbls_wavepoint.hpp -- WAVE-parallel Jacobian formulas for the serial EC chains.
//
// The row-sliced types (mbls_rowfield.hpp) put one Fq element on a 16-lane row, so a wave holds
// 4 rows.  In the serial phases (bucket-reduction levels with few segments, the window Horner,
// the final fold over windows) a chain of dependent point operations is the critical path,
// and a row-sliced product (~1 K cycles of dependent DPP/mad steps) is its unit.  Here ONE
// point operation occupies a whole wave: every row holds the same point, and the independent
// products of each dependency level of the formula are spread one per row (the row selects
// its operands, computes one row product, and the 4 results are broadcast back to all rows by
// ds_bpermute).  Additions/subtractions run replicated on every row.
//   dbl-2009-l:  7 products in 3 levels      (row-serial: 7; D = 4 X B as a product)
//   add-2007-bl: 16 products in 5 levels     (row-serial: 16; Z3 = 2 (Z1 Z2) H)
// Fq2 (G2) products expand into 3 Fq products (2 for squares) and a level's Fq products are
// processed 4 at a time.  Results equal jac_dbl / jac_add exactly (same formulas, same
// branches); only the schedule differs.
#pragma once
#include <type_traits>

#include "mbls_curve.hpp"
#include "mbls_rowfield.hpp"

namespace mbls {
namespace wave {

MBLS_DEV uint32_t row() { return (__lane_id() >> 4) & 3u; }

// r[k] = a[k] * b[k] for k < K <= 4, one product per row, all rows receive all results
template <int K>
MBLS_DEV void mul4(RFq* r, const RFq* a, const RFq* b) {
    static_assert(K >= 1 && K <= 4, "one product per row");
    // row k takes operand k: v_cndmask with the constant lane mask of row k (inline asm -- a
    // select chain on row() was turned into a dynamically indexed stack array, i.e. a scratch
    // store + load on every product level of the latency-bound chains)
    uint32_t A = a[0].v, B = b[0].v;
#pragma unroll
    for (int k = 1; k < K; ++k) {
        const uint64_t rowk = 0xffffull << (16 * k);
        A = rowop::pick(rowk, A, a[k].v);
        B = rowop::pick(rowk, B, b[k].v);
    }
    const RFq p = RFq{A} * RFq{B};
    const int l16 = (int)rowdpp::lane16();
#pragma unroll
    for (int k = 0; k < K; ++k) r[k].v = (uint32_t)__shfl((int)p.v, l16 + 16 * k, 64);
}

// N Fq products in groups of 4 (compile-time recursion)
template <int N, int G = 0>
MBLS_DEV void muln(RFq* r, const RFq* a, const RFq* b) {
    if constexpr (G < N) {
        constexpr int K = (N - G) >= 4 ? 4 : (N - G);
        mul4<K>(r + G, a + G, b + G);
        muln<N, G + K>(r, a, b);
    }
}

// K independent products of the field type
template <int K>
MBLS_DEV void mul(RFq (&r)[K], const RFq (&a)[K], const RFq (&b)[K]) {
    muln<K>(r, a, b);
}

template <int K>
MBLS_DEV void mul(RFq2 (&r)[K], const RFq2 (&a)[K], const RFq2 (&b)[K]) {
    // Karatsuba: t0 = a0 b0, t1 = a1 b1, t2 = (a0 + a1)(b0 + b1)
    RFq A[3 * K], B[3 * K], P[3 * K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        A[3 * k] = a[k].c0;
        B[3 * k] = b[k].c0;
        A[3 * k + 1] = a[k].c1;
        B[3 * k + 1] = b[k].c1;
        A[3 * k + 2] = a[k].c0 + a[k].c1;
        B[3 * k + 2] = b[k].c0 + b[k].c1;
    }
    muln<3 * K>(P, A, B);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        r[k].c0 = P[3 * k] - P[3 * k + 1];
        r[k].c1 = (P[3 * k + 2] - P[3 * k]) - P[3 * k + 1];
    }
}

// squares: Fq -> one product; Fq2 -> (a0 + a1)(a0 - a1), a0 a1
template <int K>
MBLS_DEV void sqr(RFq (&r)[K], const RFq (&a)[K]) {
    muln<K>(r, a, a);
}

template <int K>
MBLS_DEV void sqr(RFq2 (&r)[K], const RFq2 (&a)[K]) {
    RFq A[2 * K], B[2 * K], P[2 * K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        A[2 * k] = a[k].c0 + a[k].c1;
        B[2 * k] = a[k].c0 - a[k].c1;
        A[2 * k + 1] = a[k].c0;
        B[2 * k + 1] = a[k].c1;
    }
    muln<2 * K>(P, A, B);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        r[k].c0 = P[2 * k];
        r[k].c1 = dbl(P[2 * k + 1]);
    }
}

// mixed level: squares of s[0..KS) and products a[k]*b[k], k < KM, in one batch
template <int KS, int KM>
MBLS_DEV void sqr_mul(RFq (&rs)[KS], RFq (&rm)[KM], const RFq (&s)[KS], const RFq (&a)[KM], const RFq (&b)[KM]) {
    RFq A[KS + KM], B[KS + KM], P[KS + KM];
#pragma unroll
    for (int k = 0; k < KS; ++k) A[k] = B[k] = s[k];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        A[KS + k] = a[k];
        B[KS + k] = b[k];
    }
    muln<KS + KM>(P, A, B);
#pragma unroll
    for (int k = 0; k < KS; ++k) rs[k] = P[k];
#pragma unroll
    for (int k = 0; k < KM; ++k) rm[k] = P[KS + k];
}

template <int KS, int KM>
MBLS_DEV void sqr_mul(RFq2 (&rs)[KS], RFq2 (&rm)[KM], const RFq2 (&s)[KS], const RFq2 (&a)[KM],
                      const RFq2 (&b)[KM]) {
    constexpr int N = 2 * KS + 3 * KM;
    RFq A[N], B[N], P[N];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
        A[2 * k] = s[k].c0 + s[k].c1;
        B[2 * k] = s[k].c0 - s[k].c1;
        A[2 * k + 1] = s[k].c0;
        B[2 * k + 1] = s[k].c1;
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        const int o = 2 * KS + 3 * k;
        A[o] = a[k].c0;
        B[o] = b[k].c0;
        A[o + 1] = a[k].c1;
        B[o + 1] = b[k].c1;
        A[o + 2] = a[k].c0 + a[k].c1;
        B[o + 2] = b[k].c0 + b[k].c1;
    }
    muln<N>(P, A, B);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
        rs[k].c0 = P[2 * k];
        rs[k].c1 = dbl(P[2 * k + 1]);
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        const int o = 2 * KS + 3 * k;
        rm[k].c0 = P[o] - P[o + 1];
        rm[k].c1 = (P[o + 2] - P[o]) - P[o + 1];
    }
}

// dbl-2009-l in 3 product levels (same result as jac_dbl).
// G1 rows (RFq): the constant factors ride on unreduced product operands (x2_in / x4_in /
// x8_in: row shifts, add_in: no conditional subtraction), and the spare row of level 2 computes
// 2D directly:
//   L1: E = X (3X), B = Y^2, Z3 = (2Y) Z
//   L2: F = E^2, D = (4X) B, 2D = (8X) B, 8C = (8B) B
//   X3 = F - 2D;  L3: E (D - X3);  Y3 = E (D - X3) - 8C
// -- 3 reduced subtractions on the chain instead of 12 additions / doublings / subtractions.
// G2 rows (RFq2): an Fq2 square is 2 Fq products against 3 for a product, so the square
// forms stay (levels of 7, 7 and 3 Fq products).
template <class RF>
MBLS_DEV Jacobian<RF> jdbl(const Jacobian<RF>& p) {
    if (p.is_inf()) return p;
    Jacobian<RF> r;
    if constexpr (std::is_same<RF, RFq>::value) {
        RF m1[3];
        mul<3>(m1, {p.x, p.y, x2_in(p.y)}, {add_in(x2_in(p.x), p.x), p.y, p.z});
        const RF E = m1[0], B = m1[1];
        RF m2[4];
        mul<4>(m2, {E, x4_in(p.x), x8_in(p.x), x8_in(B)}, {E, B, B, B});
        const RF D = m2[1];
        r.x = m2[0] - m2[2];
        RF m3[1];
        mul<1>(m3, {E}, {D - r.x});
        r.y = m3[0] - m2[3];
        r.z = m1[2];
    } else {
        // L1: A = X^2, B = Y^2 | YZ = Y*Z
        RF s1[2], m1[1];
        sqr_mul<2, 1>(s1, m1, {p.x, p.y}, {p.y}, {p.z});
        const RF A = s1[0], B = s1[1];
        const RF E = dbl(A) + A;
        // L2: C = B^2, Fv = E^2 | XB = X*B  (D = 4 X B)
        RF s2[2], m2[1];
        sqr_mul<2, 1>(s2, m2, {B, E}, {p.x}, {B});
        const RF C = s2[0];
        const RF D = dbl(dbl(m2[0]));
        r.x = s2[1] - dbl(D);
        // L3: E * (D - X3)
        RF m3[1];
        mul<1>(m3, {E}, {D - r.x});
        r.y = m3[0] - dbl(dbl(dbl(C)));
        r.z = dbl(m1[0]);
    }
    return r;
}

// add-2007-bl in 5 product levels (same result and branches as jac_add); for G1 rows 2H, 2R,
// 2 Z1Z2 and 2 S1 are unreduced shifts feeding products (reduced doublings for Fq2)
template <class RF>
MBLS_DEV Jacobian<RF> jadd(const Jacobian<RF>& p, const Jacobian<RF>& q) {
    if (p.is_inf()) return q;
    if (q.is_inf()) return p;
    // L1: Z1Z1, Z2Z2 | Z1Z2 (Z3 = 2 Z1 Z2 H instead of ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H)
    RF s1[2], m1[1];
    sqr_mul<2, 1>(s1, m1, {p.z, q.z}, {p.z}, {q.z});
    const RF Z1Z1 = s1[0], Z2Z2 = s1[1];
    // L2: U1 = X1 Z2Z2, U2 = X2 Z1Z1, Z2^3, Z1^3
    RF m2[4];
    mul<4>(m2, {p.x, q.x, q.z, p.z}, {Z2Z2, Z1Z1, Z2Z2, Z1Z1});
    const RF U1 = m2[0], U2 = m2[1];
    const RF H = U2 - U1;
    // L3: S1 = Y1 Z2^3, S2 = Y2 Z1^3 | I = (2H)^2
    const RF H2 = x2_in(H);
    RF s3[1], m3[2];
    sqr_mul<1, 2>(s3, m3, {H2}, {p.y, q.y}, {m2[2], m2[3]});
    const RF S1 = m3[0];
    const RF R = m3[1] - S1;
    if (H.is_zero()) {
        if (R.is_zero()) return jdbl(p);
        return Jacobian<RF>::inf();
    }
    const RF I = s3[0];
    const RF R2 = x2_in(R);
    // L4: RR = (2R)^2 | J = H I, V = U1 I, Z3 = (2 Z1Z2) H
    RF s4[1], m4[3];
    sqr_mul<1, 3>(s4, m4, {R2}, {H, U1, x2_in(m1[0])}, {I, I, H});
    const RF J = m4[0], V = m4[1];
    Jacobian<RF> r;
    r.x = s4[0] - J - dbl(V);
    r.z = m4[2];
    // L5: 2R (V - X3), (2 S1) J
    RF m5[2];
    mul<2>(m5, {R2, x2_in(S1)}, {V - r.x, J});
    r.y = m5[0] - m5[1];
    return r;
}

// stores from one row only (all rows hold the same value)
MBLS_DEV bool leader_row() { return row() == 0; }

}  // namespace wave
}  // namespace mbls
