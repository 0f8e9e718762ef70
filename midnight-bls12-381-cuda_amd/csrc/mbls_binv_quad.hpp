// mbls_binv_quad.hpp -- the binary-GCD inversion of mbls_binv.hpp on a QUAD of lanes (device only).
//
// The one (x, y, 1) normalisation at the end of an MSM (k_final_icicle) runs on a single wave: its
// time is the instruction stream of one lane.  An outer step of binv::inverse is the 30-step inner
// loop plus FOUR independent 12-word updates -- (a, b) by lincomb_shift, (u, v) by lincomb_mod --
// issued one after the other.  Here the four lanes of a DPP quad run the same inner loop (same
// inputs, same result, no exchange) and then ONE update each:
//     lane 0: a' = (f0 a + g0 b) / 2^K     lane 1: b' = (f1 a + g1 b) / 2^K      (exact, signed)
//     lane 2: u' = (f0' u + g0' v) / 2^K   lane 3: v' = (f1' u + g1' v) / 2^K    (mod m, one step late)
// as one branch-free body (`lincomb_role`: the mod-m corrections are selects that the exact lanes
// turn off), followed by four DPP quad broadcasts per word.  Same values as binv::inverse, step for
// step (the same factors, the same software pipelining of the (u, v) update).
#pragma once
#include "mbls_binv.hpp"

namespace mbls {
namespace binv {

// word w of lane LANE of the quad, on every lane of the quad (DPP quad_perm [LANE x 4])
template <int LANE>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t w) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)w, LANE * 0x55, 0xf, 0xf, false);
}

// out = 1 / y mod m on the four lanes of a quad (all four active, same y); every lane returns it
template <int N>
__device__ __forceinline__ int inverse_quad(uint32_t (&out)[N], const uint32_t (&y)[N], const uint32_t (&m)[N],
                                            uint32_t ninv) {
    const int role = (int)(__lane_id() & 3u);
    const bool modl = role >= 2;
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
        uint64_t F0 = 1, F1 = 1ull << 32;
#pragma unroll
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
        // this lane's update
        uint32_t X[N], Y[N], R[N];
        for (int i = 0; i < N; ++i) {
            X[i] = modl ? u[i] : a[i];
            Y[i] = modl ? v[i] : b[i];
        }
        const int64_t f = role == 0 ? f0 : role == 1 ? f1 : role == 2 ? pf0 : pf1;
        const int64_t g = role == 0 ? g0 : role == 1 ? g1 : role == 2 ? pg0 : pg1;
        bool neg;
        lincomb_role<N>(R, neg, X, Y, f, g, modl, m, ninv);
        for (int i = 0; i < N; ++i) {
            a[i] = quad_bcast<0>(R[i]);
            b[i] = quad_bcast<1>(R[i]);
            u[i] = quad_bcast<2>(R[i]);
            v[i] = quad_bcast<3>(R[i]);
        }
        const uint32_t nf = neg ? 1u : 0u;
        if (quad_bcast<0>(nf)) {
            f0 = -f0;
            g0 = -g0;
        }
        if (quad_bcast<1>(nf)) {
            f1 = -f1;
            g1 = -g1;
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

}  // namespace binv
}  // namespace mbls
