// mbls_binv.hpp -- modular inversion by the batched binary GCD (Pornin, "Optimized Binary GCD
// for Modular Inversion", IACR ePrint 2020/972, algorithm 2; variable-time form).
//
// The hot-path products are quarter-rate v_mad_u64_u32 chains; a Fermat inversion a^(m-2) is
// ~570 of them in series (0.29 ms on one row-sliced wave for the one (x, y, 1) normalisation of
// an MSM result).  The binary GCD needs no products in its inner loop: 31 steps run on 64-bit
// approximations of (a, b) (exact low 31 bits, top 33 bits), recording the update matrix
// (f0 g0; f1 g1); the 12-word values are then updated once per 31 steps with word-by-word
// small-factor products.  ~26 outer steps for a 381-bit modulus.
//
// GPU form (the one-lane normalisation is latency-bound): K = 30 inner steps per outer step so the
// update factors satisfy |f|, |g| <= 2^30 and each pair (f, g) packs into ONE 64-bit word
// f + g 2^32 (exact in two's complement, unpacked by sign extension) -- the pair updates are one
// 64-bit subtract and one shift; the inner steps are unrolled and branch-free (the subtraction's
// borrow is the a < b test); the bit length is taken once, of a | b, without a branch chain.
//
// Invariants (integers a, b >= 0; u, v mod m; y the input): a = u*y, b = v*y (mod m).  Start
// a = y, b = m, u = 1, v = 0; each outer step maps (a, b) -> ((f0 a + g0 b) / 2^31, (f1 a + g1 b)
// / 2^31) and (u, v) the same way mod m (exact division for a, b; Montgomery division by 2^31
// for u, v).  The loop ends at a = 0 with b = gcd(y, m) = 1 and v = 1/y.
//
// Portable C++ (host-testable: tests/test_oracle.py builds tests/binv_host.cpp against it).
#pragma once
#include <stdint.h>

#ifndef MBLS_HD
#if defined(__HIPCC__)
#define MBLS_HD __host__ __device__ __forceinline__
#else
#define MBLS_HD inline
#endif
#endif

namespace mbls {
namespace binv {

static constexpr int K = 30;  // inner steps per outer step

template <int N>
MBLS_HD bool is_zero(const uint32_t (&a)[N]) {
    uint32_t t = 0;
    for (int i = 0; i < N; ++i) t |= a[i];
    return t == 0;
}

// bit length of a | b, i.e. max(bitlen(a), bitlen(b)), as a max over words (no branch chain)
template <int N>
MBLS_HD int bitlen_or(const uint32_t (&a)[N], const uint32_t (&b)[N]) {
    int n = 0;
    for (int i = 0; i < N; ++i) {
        const uint32_t w = a[i] | b[i];
        const int l = w ? 32 * i + 32 - __builtin_clz(w | 1u) : 0;
        n = l > n ? l : n;
    }
    return n;
}

// (a >> pos) & (2^33 - 1) for 0 <= pos, when a < 2^(pos + 33)
template <int N>
MBLS_HD uint64_t top33(const uint32_t (&a)[N], int pos) {
    const int wi = pos >> 5, sh = pos & 31;
    uint32_t w0 = 0, w1 = 0, w2 = 0;
    for (int i = 0; i < N; ++i) {  // selects, not dynamic register indexing
        w0 = i == wi ? a[i] : w0;
        w1 = i == wi + 1 ? a[i] : w1;
        w2 = i == wi + 2 ? a[i] : w2;
    }
    uint64_t x = ((uint64_t)w1 << 32) | w0;
    x >>= sh;
    if (sh) x |= (uint64_t)w2 << (64 - sh);
    return x & ((1ull << 33) - 1);
}

// r (N+1 words) = a * k
template <int N>
MBLS_HD void mul_small(uint32_t (&r)[N + 1], const uint32_t (&a)[N], uint32_t k) {
    uint64_t c = 0;
    for (int i = 0; i < N; ++i) {
        c += (uint64_t)a[i] * k;
        r[i] = (uint32_t)c;
        c >>= 32;
    }
    r[N] = (uint32_t)c;
}

// S = s_p * P + s_q * Q as sign + magnitude (M words, |S| < 2^(32 M - 1)); returns true if
// negative.  Branch-free (two's complement sum of the conditionally negated operands, then a
// conditional negation), so the callers' updates stay in one basic block the scheduler can
// interleave with the next inner loop.
template <int M>
MBLS_HD bool signed_sum(uint32_t (&S)[M], const uint32_t (&P)[M], bool np, const uint32_t (&Q)[M], bool nq) {
    const uint32_t mp = np ? ~0u : 0u, mq = nq ? ~0u : 0u;
    uint64_t c = (uint64_t)(np ? 1u : 0u) + (nq ? 1u : 0u);
    for (int i = 0; i < M; ++i) {
        c += (uint64_t)(P[i] ^ mp) + (Q[i] ^ mq);
        S[i] = (uint32_t)c;
        c >>= 32;
    }
    const uint32_t ms = (uint32_t)((int32_t)S[M - 1] >> 31);  // all ones when negative
    c = ms & 1u;
    for (int i = 0; i < M; ++i) {
        c += (uint64_t)(S[i] ^ ms);
        S[i] = (uint32_t)c;
        c >>= 32;
    }
    return ms != 0;
}

// r = |f a + g b| / 2^K (exact); returns true if f a + g b < 0.  |f|, |g| <= 2^K.
template <int N>
MBLS_HD bool lincomb_shift(uint32_t (&r)[N], const uint32_t (&a)[N], const uint32_t (&b)[N], int64_t f, int64_t g) {
    uint32_t P[N + 1], Q[N + 1], S[N + 1];
    mul_small<N>(P, a, (uint32_t)(f < 0 ? -f : f));
    mul_small<N>(Q, b, (uint32_t)(g < 0 ? -g : g));
    const bool neg = signed_sum<N + 1>(S, P, f < 0, Q, g < 0);
    uint32_t z = 0;
    for (int i = 0; i < N; ++i) {
        r[i] = (S[i] >> K) | (S[i + 1] << (32 - K));
        z |= r[i];
    }
    return neg && z != 0;
}

// r = (f u + g v) / 2^K mod m, u, v in [0, m); result in [0, m).  |f|, |g| <= 2^K.  Branch-free.
template <int N>
MBLS_HD void lincomb_mod(uint32_t (&r)[N], const uint32_t (&u)[N], const uint32_t (&v)[N], int64_t f, int64_t g,
                         const uint32_t (&m)[N], uint32_t ninv) {
    uint32_t P[N + 1], Q[N + 1], S[N + 1];
    mul_small<N>(P, u, (uint32_t)(f < 0 ? -f : f));
    mul_small<N>(Q, v, (uint32_t)(g < 0 ? -g : g));
    const bool neg = signed_sum<N + 1>(S, P, f < 0, Q, g < 0);
    {  // negative: |S| <= 2^(K+1) m, S <- 2^(K+1) m - |S| in [0, 2^(K+1) m]
        int64_t br = 0;
        for (int i = 0; i <= N; ++i) {
            const uint32_t lo = i == 0 ? 0u : m[i - 1] >> (31 - K);
            const uint32_t mw = (i < N ? m[i] << (K + 1) : 0u) | lo;
            int64_t d = (int64_t)mw - S[i] + br;
            br = d >> 32;
            S[i] = neg ? (uint32_t)d : S[i];
        }
    }
    // S + k m = 0 (mod 2^K), k = S * (-1/m) mod 2^K; S + k m < 3 * 2^K m < 2^(32(N+1))
    const uint32_t k = (S[0] * ninv) & ((1u << K) - 1);
    uint64_t c = 0;
    for (int i = 0; i <= N; ++i) {
        c += (uint64_t)S[i] + (i < N ? (uint64_t)m[i] * k : 0ull);
        S[i] = (uint32_t)c;
        c >>= 32;
    }
    // (S + k m) / 2^K < 3m: N + 1 words (3r > 2^256 for the 255-bit Fr modulus)
    uint32_t t[N + 1];
    for (int i = 0; i < N; ++i) t[i] = (S[i] >> K) | (S[i + 1] << (32 - K));
    t[N] = S[N] >> K;
    for (int q = 0; q < 2; ++q) {
        uint32_t d[N + 1];
        int64_t br = 0;
        for (int i = 0; i <= N; ++i) {
            int64_t x = (int64_t)t[i] - (i < N ? m[i] : 0u) + br;
            d[i] = (uint32_t)x;
            br = x >> 32;
        }
        for (int i = 0; i <= N; ++i) t[i] = br ? t[i] : d[i];
    }
    for (int i = 0; i < N; ++i) r[i] = t[i];
}

// One of the four updates of an outer step, as one branch-free body for the four-lane form
// (mbls_binv_quad.hpp: one role per lane of a DPP quad).  exact lanes (modl false): r = |f x + g y| / 2^K, neg = (f x + g y < 0, nonzero) -- lincomb_shift;
// mod lanes (modl true): r = (f x + g y) / 2^K mod m -- lincomb_mod.  |f|, |g| <= 2^K.
template <int N>
MBLS_HD void lincomb_role(uint32_t (&r)[N], bool& neg_out, const uint32_t (&x)[N], const uint32_t (&y)[N], int64_t f,
                          int64_t g, bool modl, const uint32_t (&m)[N], uint32_t ninv) {
    uint32_t P[N + 1], Q[N + 1], S[N + 1];
    mul_small<N>(P, x, (uint32_t)(f < 0 ? -f : f));
    mul_small<N>(Q, y, (uint32_t)(g < 0 ? -g : g));
    const bool neg = signed_sum<N + 1>(S, P, f < 0, Q, g < 0);
    {  // mod lanes, negative: |S| <= 2^(K+1) m, S <- 2^(K+1) m - |S|
        const bool fix = modl && neg;
        int64_t br = 0;
        for (int i = 0; i <= N; ++i) {
            const uint32_t lo = i == 0 ? 0u : m[i - 1] >> (31 - K);
            const uint32_t mw = (i < N ? m[i] << (K + 1) : 0u) | lo;
            int64_t d = (int64_t)mw - S[i] + br;
            br = d >> 32;
            S[i] = fix ? (uint32_t)d : S[i];
        }
    }
    // mod lanes: S + k m = 0 (mod 2^K); exact lanes: k = 0 (S is a multiple of 2^K already)
    const uint32_t k = modl ? (S[0] * ninv) & ((1u << K) - 1) : 0u;
    uint64_t c = 0;
    for (int i = 0; i <= N; ++i) {
        c += (uint64_t)S[i] + (i < N ? (uint64_t)m[i] * k : 0ull);
        S[i] = (uint32_t)c;
        c >>= 32;
    }
    uint32_t t[N + 1];
    for (int i = 0; i < N; ++i) t[i] = (S[i] >> K) | (S[i + 1] << (32 - K));
    t[N] = S[N] >> K;
    for (int q = 0; q < 2; ++q) {  // mod lanes: < 3m -> < m
        uint32_t d[N + 1];
        int64_t br = 0;
        for (int i = 0; i <= N; ++i) {
            int64_t xx = (int64_t)t[i] - (i < N ? m[i] : 0u) + br;
            d[i] = (uint32_t)xx;
            br = xx >> 32;
        }
        const bool keep = br || !modl;
        for (int i = 0; i <= N; ++i) t[i] = keep ? t[i] : d[i];
    }
    uint32_t z = 0;
    for (int i = 0; i < N; ++i) {
        r[i] = t[i];
        z |= t[i];
    }
    neg_out = neg && z != 0;
}

// out = 1 / y mod m (plain integers, y in [1, m), m odd, gcd(y, m) = 1).  Returns the number of
// outer steps (<= 2 * bitlen(m) / K + 2 for valid input; capped so a bad input still ends).
// The (u, v) update of outer step k is independent of the (a, b) work of step k + 1, so it runs
// one step late, in the same basic block as the next inner loop (software pipelining: the lone
// lane's dependency chains interleave instead of running back to back); the first step's pending
// update is the identity (f, g) = (2^K, 0), (0, 2^K).
template <int N>
MBLS_HD int inverse(uint32_t (&out)[N], const uint32_t (&y)[N], const uint32_t (&m)[N], uint32_t ninv) {
    uint32_t a[N], b[N], u[N], v[N];
    for (int i = 0; i < N; ++i) {
        a[i] = y[i];
        b[i] = m[i];
        u[i] = i == 0 ? 1u : 0u;
        v[i] = 0;
    }
    int64_t pf0 = (int64_t)1 << K, pg0 = 0, pf1 = 0, pg1 = (int64_t)1 << K;  // pending (u, v) update
    int steps = 0;
    const int cap = (64 * N) / K + 8;
    while (!is_zero<N>(a) && steps < cap) {
        ++steps;
        const int nl = bitlen_or<N>(a, b);
        const int n = nl > 64 ? nl : 64;
        uint64_t xa = (a[0] & 0x7fffffffu) | (top33<N>(a, n - 33) << 31);
        uint64_t xb = (b[0] & 0x7fffffffu) | (top33<N>(b, n - 33) << 31);
        // (f0, g0) and (f1, g1) packed as f + g 2^32 (two's complement, |f|, |g| <= 2^K)
        uint64_t F0 = 1, F1 = 1ull << 32;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const bool odd = (xa & 1) != 0;
            const bool lt = xa < xb;
            const bool sw = odd && lt;
            const uint64_t d = lt ? xb - xa : xa - xb;  // |xa - xb|: the new xa when odd
            const uint64_t G0 = sw ? F1 : F0, G1 = sw ? F0 : F1;
            xb = sw ? xa : xb;
            xa = (odd ? d : xa) >> 1;
            F0 = odd ? G0 - G1 : G0;
            F1 = G1 << 1;
        }
        // the previous step's (u, v) update, beside this step's inner loop
        uint32_t nu[N], nv[N];
        lincomb_mod<N>(nu, u, v, pf0, pg0, m, ninv);
        lincomb_mod<N>(nv, u, v, pf1, pg1, m, ninv);
        int64_t f0 = (int32_t)(uint32_t)F0, g0 = ((int64_t)F0 - f0) >> 32;
        int64_t f1 = (int32_t)(uint32_t)F1, g1 = ((int64_t)F1 - f1) >> 32;
        uint32_t na[N], nb[N];
        if (lincomb_shift<N>(na, a, b, f0, g0)) {
            f0 = -f0;
            g0 = -g0;
        }
        if (lincomb_shift<N>(nb, a, b, f1, g1)) {
            f1 = -f1;
            g1 = -g1;
        }
        for (int i = 0; i < N; ++i) {
            a[i] = na[i];
            b[i] = nb[i];
            u[i] = nu[i];
            v[i] = nv[i];
        }
        pf0 = f0;
        pg0 = g0;
        pf1 = f1;
        pg1 = g1;
    }
    uint32_t nv[N];
    lincomb_mod<N>(nv, u, v, pf1, pg1, m, ninv);  // the last step's update (only v is needed)
    for (int i = 0; i < N; ++i) out[i] = nv[i];
    return steps;
}

// The four-lane form (mbls_binv_quad.hpp::inverse_quad) with its four roles run one after the
// other: the same outer loop, role selection and exchange, for the host check of lincomb_role
// (tests/binv_host.cpp).  Returns the number of outer steps.
template <int N>
MBLS_HD int inverse_roles(uint32_t (&out)[N], const uint32_t (&y)[N], const uint32_t (&m)[N], uint32_t ninv) {
    uint32_t a[N], b[N], u[N], v[N];
    for (int i = 0; i < N; ++i) {
        a[i] = y[i];
        b[i] = m[i];
        u[i] = i == 0 ? 1u : 0u;
        v[i] = 0;
    }
    int64_t pf0 = (int64_t)1 << K, pg0 = 0, pf1 = 0, pg1 = (int64_t)1 << K;
    int steps = 0;
    const int cap = (64 * N) / K + 8;
    while (!is_zero<N>(a) && steps < cap) {
        ++steps;
        const int nl = bitlen_or<N>(a, b);
        const int n = nl > 64 ? nl : 64;
        uint64_t xa = (a[0] & 0x7fffffffu) | (top33<N>(a, n - 33) << 31);
        uint64_t xb = (b[0] & 0x7fffffffu) | (top33<N>(b, n - 33) << 31);
        uint64_t F0 = 1, F1 = 1ull << 32;
        for (int j = 0; j < K; ++j) {
            const bool odd = (xa & 1) != 0;
            const bool lt = xa < xb;
            const bool sw = odd && lt;
            const uint64_t d = lt ? xb - xa : xa - xb;
            const uint64_t G0 = sw ? F1 : F0, G1 = sw ? F0 : F1;
            xb = sw ? xa : xb;
            xa = (odd ? d : xa) >> 1;
            F0 = odd ? G0 - G1 : G0;
            F1 = G1 << 1;
        }
        int64_t f0 = (int32_t)(uint32_t)F0, g0 = ((int64_t)F0 - f0) >> 32;
        int64_t f1 = (int32_t)(uint32_t)F1, g1 = ((int64_t)F1 - f1) >> 32;
        uint32_t R[4][N];
        bool neg[4];
        for (int role = 0; role < 4; ++role) {
            const bool modl = role >= 2;
            const int64_t f = role == 0 ? f0 : role == 1 ? f1 : role == 2 ? pf0 : pf1;
            const int64_t g = role == 0 ? g0 : role == 1 ? g1 : role == 2 ? pg0 : pg1;
            lincomb_role<N>(R[role], neg[role], modl ? u : a, modl ? v : b, f, g, modl, m, ninv);
        }
        for (int i = 0; i < N; ++i) {
            a[i] = R[0][i];
            b[i] = R[1][i];
            u[i] = R[2][i];
            v[i] = R[3][i];
        }
        if (neg[0]) {
            f0 = -f0;
            g0 = -g0;
        }
        if (neg[1]) {
            f1 = -f1;
            g1 = -g1;
        }
        pf0 = f0;
        pg0 = g0;
        pf1 = f1;
        pg1 = g1;
    }
    uint32_t nv[N];
    lincomb_mod<N>(nv, u, v, pf1, pg1, m, ninv);
    for (int i = 0; i < N; ++i) out[i] = nv[i];
    return steps;
}

}  // namespace binv
}  // namespace mbls
