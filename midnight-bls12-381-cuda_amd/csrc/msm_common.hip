// msm_common.hip -- group-independent MSM stages: plan, signed-digit decomposition, scans,
// counting-sort scatter, chunking, synthetic scalars.
//
// Reference: get_optimal_c (msm.cuh:115-133), compute_bucket_indices_kernel
// (msm_kernels.cu:69-143), histogram (:224-256), cub ExclusiveSum / SortPairs (:748-781).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <set>

#include "msm_core.hpp"

namespace mbls {

// window size: the reference's size classes (msm.cuh:115-133) except c = 15, where
// 17 * 15 = 255 leaves an 18th window holding only the final carry -- one bucket with about
// half of all points (measured: 1.3 s of serial bucket summation at 2^20).  c = 16 instead.
static int optimal_c(long long n) {
    if (n <= (1 << 8)) return 7;
    if (n <= (1 << 10)) return 8;
    if (n <= (1 << 12)) return 10;
    if (n <= (1 << 14)) return 12;
    if (n <= (1 << 16)) return 13;
    if (n <= (1 << 18)) return 14;
    return 16;
}

int precompute_shift(int F) { return F > 1 ? (256 + F - 1) / F : 0; }

// -DMBLS_PART_SORT=0 (variant builds) forces the tiled digits + scatter sort for every c; the
// shipped library uses it for c > 16 only
#ifndef MBLS_PART_SORT
#define MBLS_PART_SORT 1
#endif
#ifndef SLOT0_MIN_TABLE_BYTES
#define SLOT0_MIN_TABLE_BYTES (1ull << 30)  // G1 shift tables above run the GLV plan on slot 0 (shift_plan)
#endif
// -DMBLS_C=<c> (tools/ variant builds) overrides the automatic window size; the caller's
// MSMConfig.c always wins.  No run-time environment switch: a prover's environment cannot
// select an untested schedule.
#ifndef MBLS_C
#define MBLS_C 0
#endif
// Split plans (round 4, tools/c_sweep.py on MI355X, profiles/r04/c_sweep.txt): the digits are
// 128-bit (GLV) or 64-bit (psi) and the reference's classes assume 255-bit ones, so below 2^16
// they leave the top window nearly empty (its buckets collect most digits) or too many buckets
// for the latency-bound reduction.  Measured best windows (wall ms per call, ICICLE entry):
//   G1 GLV: 2^8 c 8 0.71 (auto 7: 0.84); 2^12 c 8 0.88 (10: 0.91); 2^13 c 8 1.04 (12: 1.21);
//           2^14 c 11 0.97 (1.19);
//           2^15 c 11 0.99 (13: 1.12); 2^16 c 16 1.21 (13: 1.39); >= 2^17 16
//   G2 psi: 2^8 c 11 1.29 (7: 1.41); 2^12 c 11 1.52 (10: 1.72); 2^13 c 13 1.59 (12: 2.14);
//           2^14 c 13 1.63 (12: 2.25);
//           2^16 c 16 2.24 (13: 2.43); >= 2^17 16
static int split_c(long long n, int split) {
    if (split == 2) return n <= (1 << 13) ? 8 : n <= (1 << 15) ? 11 : 16;
    return n <= (1 << 12) ? 11 : n <= (1 << 15) ? 13 : 16;
}
// Shift tables (precompute factor F > 1 run on its own blocks of sF = ceil(256 / F) bits, the
// shift plan): a window size that leaves a block's top window a few bits wide puts that window's
// digits into a handful of buckets (c = 14 against sF = 64: G1 2^18 F = 4 2.38 ms, c = 16 1.64),
// and small MSMs are bound by the sort's partitions and the reduction's buckets rather than the
// contributions.  Measured best windows (G1 / G2 wall ms per call, tools/precompute_sweep.py,
// profiles/r04/precompute_sweep.txt):
//   sF = 64 (F = 4):  2^8 c 8 0.58 (16: 1.52); 2^12 c 11 0.72 (16: 1.06); 2^13 c 13 0.82
//                     (16: 1.08); 2^15 c 13 0.98 (16: 1.09); >= 2^16 16
//   sF = 32 (F = 8):  2^10 c 11 0.53 (16: 0.86); 2^13 c 11 0.77 (16: 0.82); >= 2^14 16;
//                     G2 2^14 c 11 1.63 (16: 1.80)
//   sF = 16 (F = 16): 2^8 c 8 0.53 (16: 0.96); >= 2^10 16
static int shift_c(long long n, int F, int endo) {
    const int sF = precompute_shift(F);
    if (sF >= 64) return n <= (1 << 8) ? 8 : n <= (1 << 12) ? 11 : n <= (1 << 15) ? 13 : 16;
    if (sF >= 32) return n <= (endo == 4 ? (1 << 14) : (1 << 13)) ? 11 : 16;
    if (sF >= 16) return n <= (1 << 8) ? 8 : 16;
    return sF;
}
static int auto_c(long long n, int split, int F, int endo) {
    if (MBLS_C >= 2 && MBLS_C <= 20) return MBLS_C;
    if (split > 1) return split_c(n, split);
    if (F > 1) return shift_c(n, F, endo);
    return optimal_c(n);
}

// Which precompute factors run the shift plan.  Every contribution of a shift plan is one point
// of one window of one block, n F ceil(sF / c) of them; the split plans take 16 n (c = 16), so
// the shift plan gains only through its smaller bucket set (Wg windows of 2^(c-1) instead of 8),
// and only when c divides the block: F = 4, 8, 16 (G2: 8, 16; its F = 4 is the prepared psi
// table).  Factors 3, 5, 6, 7 lose at every size from 2^14 up (G1 2^18: 3.20 / 1.97 / 2.40 / 2.41
// ms against 1.73 plain), G2 F = 2 and 3 too (2^14: 3.27 / 2.93 against 1.62).  G1 tables above
// 1 GiB (F n 96 B > SLOT0_MIN_TABLE_BYTES) lose to the GLV plan's 201 MB working set: 2^20 F = 16
// (1.6 GB) 4.17 ms against 4.13, while the 805 MB F = 8 table still wins (3.92; 2^19 F = 16 2.37
// against 2.56).  Everything else runs the group's split plan
// on slot 0 of the table (plan.bstride = F): P_i is the table's entry i F, and the split kernel
// writes a compact per-call [P, phi P] / [P, psi P, psi^2 P, psi^3 P].
static bool shift_plan(long long n, int F, int endo) {
    if (!MBLS_PART_SORT) return true;  // variant builds: no slot-0 plan without the fused front
    if (endo == 2) return (F == 4 || F == 8 || F == 16) && (size_t)n * F * 96 <= SLOT0_MIN_TABLE_BYTES;
    return F == 8 || F == 16;
}

eIcicleError make_plan(long long n, const MSMConfig* cfg, MsmPlan& p, int endo) {
    int bits = cfg->bitsize > 0 ? cfg->bitsize : 255;
    if (bits > 256) return MBLS_INVALID_ARGUMENT;
    int F = cfg->precompute_factor > 0 ? cfg->precompute_factor : 1;
    if (F > MAX_PRECOMPUTE) return MBLS_INVALID_ARGUMENT;
    // a precomputed table of the group's endomorphism images (precompute_factor == the split:
    // G1 2 -> [P, phi P], G2 4 -> [P, psi P, psi^2 P, psi^3 P], precompute_call) always takes the
    // split, whatever the bit size: the per-call image table is not built (DESIGN.md "prepared
    // bases").  Shift tables run the shift plan or the split plan on slot 0 (shift_plan).
    p.prepared = endo > 1 && F == endo;
    const bool slot0 = F > 1 && !p.prepared && !shift_plan(n, F, endo);
    // Endomorphism split (no precomputed table, wide scalars):
    //   G1 GLV: two half-width digit streams, |m| < 2^127;
    //   G2 psi: four quarter-width streams, |m| < 2^63 (tiled digits only, c <= 16; worth it
    //   only for wide scalars: plain needs ceil((bits+1)/c) windows of n, psi 4 x ceil(64/c)).
    const bool wide = endo == 2 ? bits > 128 : bits > 192;
    const int split = endo > 1 && (p.prepared || slot0 || (F == 1 && wide)) ? endo : 1;
    int c = cfg->c > 0 ? cfg->c : auto_c(n, split, split > 1 ? 1 : F, endo);
    if (c < 2 || c > 20) return MBLS_INVALID_ARGUMENT;
    p.split = 1;
    p.fq2 = endo == 4;
    if (split == 2) p.split = 2;
    // the psi digits need c <= 16: a plain-bases MSM with a larger c stays unsplit, a table's
    // schedule (c only shapes it) runs with 16
    if (split == 4 && (c <= 16 || F > 1)) p.split = 4;
    if (p.split == 4 && c > 16) c = 16;
    p.bstride = slot0 ? F : 1;
    if (p.split > 1 && F > 1) F = 1;
    // The split halves / quarters are 128 / 64-bit digit streams.  A caller's large c (picked for
    // 255-bit scalars, e.g. MIDNIGHT_MSM_WINDOW=15) can leave the top window a few bits wide: all
    // of that window's 2^21 digits (G1 2^20) then fall into a handful of buckets -- one partition
    // of the sort and a few heavy buckets take the whole window (c = 15: sort 3.3 ms instead of
    // 0.16).  c only shapes the schedule, never the result, so c >= 14 whose top window would be
    // more than 2 bits short becomes 16, which divides both widths (c > 16 also leaves the
    // partitioned sort).
    if (p.split > 1 && c >= 14) {
        const int H = p.split == 2 ? 128 : 64;
        const int Wc = (H + c - 1) / c;
        if (H - c * (Wc - 1) < c - 2 || c > 16) c = 16;
    }
    // signed digits need one bit of headroom for the top carry
    int W = p.split == 2 ? (128 + c - 1) / c : p.split == 4 ? (64 + c - 1) / c : (bits + 1 + c - 1) / c;
    int Wg = W;
    p.sF = 0;
    if (F > 1) {
        // precomputed bases: the table's shift depends on F only (precompute_shift), so the
        // table serves every c and msm_size (core/msm.rs:441-454 precomputes with c = 0, the MSM
        // may run with MIDNIGHT_MSM_WINDOW); blocks of sF bits, Wg windows each, all 256 bits
        p.sF = precompute_shift(F);
        Wg = (p.sF + c - 1) / c;
        // automatic c: windows balanced inside the block when its top window would be nearly
        // empty (-DMBLS_PART_SORT=0 variant builds, where every factor runs the shift plan:
        // F = 3: sF = 86, c 16 -> 15; F = 5: 52, 16 -> 13; F = 7: 37, 16 -> 13)
        if (cfg->c <= 0 && p.sF - c * (Wg - 1) < c - 2) {
            c = (p.sF + Wg - 1) / Wg;
            Wg = (p.sF + c - 1) / c;
        }
        W = F * Wg;
    }
    p.c = c;
    p.W = W;
    p.F = F;
    p.Wg = Wg;
    p.B = 1u << (c - 1);
    p.TB = (uint32_t)Wg * p.B;
    p.chunk = CHUNK;  // msm_call replaces it with accumulate_chunk<F>(contributions)
    p.pts = (size_t)n * (p.split > 1 ? p.split : F);  // point indices (P_i, then the images)
    p.table = p.prepared ? p.split : p.bstride > 1 ? p.bstride : F;  // bases-buffer entries per point
    p.contributions = (size_t)n * W * p.split;
    if (p.pts >= (1u << 31)) return MBLS_INVALID_ARGUMENT;
    return plan_levels(p, Wg);
}

}  // namespace mbls

extern "C" eIcicleError mbls_msm_plan(int group, int msm_size, const MSMConfig* config, int32_t* out) {
    if (!config || !out) return MBLS_INVALID_POINTER;
    if ((group != 1 && group != 2) || msm_size < 0) return MBLS_INVALID_ARGUMENT;
    mbls::MsmPlan p;
    const eIcicleError er = mbls::make_plan(msm_size > 0 ? msm_size : 1, config, p, group == 1 ? 2 : 4);
    if (er != MBLS_SUCCESS) return er;
    const int32_t v[10] = {p.c, p.W, p.Wg, p.F, p.sF, p.split, p.prepared ? 1 : 0, p.bstride, (int32_t)p.TB, p.levels};
    for (int k = 0; k < 10; ++k) out[k] = v[k];
    return MBLS_SUCCESS;
}

namespace mbls {

// Reduction levels for launches over Wl windows: level 0 has B inputs, level l divides by
// 2^seg_log[l], the last has one output.  A level with many segments runs one per LANE, fewer
// one per 16-lane ROW, few one per WAVE with shorter segments.  The -DMBLS_ROW_SEG_LOG /
// MBLS_WSEG_LOG / MBLS_LANE_MIN ... macros (tools/ variant builds) override the row / wave segment
// lengths and the lane threshold; the shipped values are the measured defaults below.
#ifndef MBLS_ROW_SEG_LOG
#define MBLS_ROW_SEG_LOG SEG_LOG
#endif
// G2: row segments of 8 and rows from 4096 segments (wave layout below): G2 2^20 12.69 ->
// 12.57 ms against 16 / 8192 (G1: segments of 8 too since the 2-point tree rows, SEG_LOG)
#ifndef MBLS_ROW_SEG_LOG_G2
#define MBLS_ROW_SEG_LOG_G2 3
#endif
#ifndef MBLS_SEG0_LOG  // level 0, one segment per lane
#define MBLS_SEG0_LOG SEG0_LOG
#endif
// measured (G1 2^20): 2 -> reduction 1.04 ms, 4 -> 1.12 ms once the narrow levels' tree sums are
// batched; before that, short segments lost
#ifndef MBLS_WSEG_LOG
#define MBLS_WSEG_LOG 2
#endif
// level 0 one segment per lane only with >= lane_min chains (65536 at G1 2^20 with all 8
// windows in one launch; a window group has fewer and its chains are latency-bound)
#ifndef MBLS_LANE_MIN
#define MBLS_LANE_MIN 32768u
#endif
// levels [0, lane_levels) may run one segment per lane
#ifndef MBLS_LANE_LEVELS
#define MBLS_LANE_LEVELS 1
#endif
// segment log of the lane levels after level 0 (variant builds: short chains, many lanes)
#ifndef MBLS_SEGL_LOG
#define MBLS_SEGL_LOG MBLS_SEG0_LOG
#endif
// the same three for G2: two more lane levels of 2-input segments (the FIPS pair chain) from 8192
// chains instead of wave-layout levels -- G2 2^20 9.36 / 9.37 -> 9.23 / 9.16 ms
// (profiles/r06/ab/g2_lane_levels_ab.txt; G1 within 1%, lane_levels_ab.txt)
#ifndef MBLS_LANE_LEVELS_G2
#define MBLS_LANE_LEVELS_G2 3
#endif
#ifndef MBLS_SEGL_LOG_G2
#define MBLS_SEGL_LOG_G2 1
#endif
#ifndef MBLS_LANE_MIN_G2
#define MBLS_LANE_MIN_G2 8192u
#endif
eIcicleError plan_levels(MsmPlan& p, int Wl) {
    constexpr int row_log = MBLS_ROW_SEG_LOG, row_log_g2 = MBLS_ROW_SEG_LOG_G2, seg0_log = MBLS_SEG0_LOG,
                  wave_log = MBLS_WSEG_LOG, lane_levels = MBLS_LANE_LEVELS;
    constexpr uint32_t lane_min = MBLS_LANE_MIN;
    static_assert(row_log >= 1 && row_log <= 6 && row_log_g2 >= 1 && row_log_g2 <= 6 && seg0_log >= 1 &&
                      seg0_log <= 6 && wave_log >= 1 && wave_log <= 6 && lane_levels >= 1 && lane_levels <= 4,
                  "reduction plan macros out of range");
    p.levels = 0;
    uint32_t m = p.B;
    while (true) {
        if (p.levels >= MAX_LEVELS) return MBLS_INVALID_ARGUMENT;
        const int ll = p.levels == 0 ? seg0_log : p.fq2 ? MBLS_SEGL_LOG_G2 : MBLS_SEGL_LOG;
        int lg = ll, mode = MODE_LANE;
        const uint32_t lane_chains = ((m + (1u << ll) - 1) >> ll) * (uint32_t)Wl;
        const int lanes_to = p.fq2 ? MBLS_LANE_LEVELS_G2 : lane_levels;
        const uint32_t lmin = (p.levels > 0 && p.fq2) ? MBLS_LANE_MIN_G2 : lane_min;
        if (p.levels >= lanes_to || lane_chains < lmin) {
            const int rl = p.fq2 ? row_log_g2 : row_log;
            const uint32_t row_chains = ((m + (1u << rl) - 1) >> rl) * (uint32_t)Wl;
            mode = row_chains >= wave_min_chains(p.fq2) ? MODE_ROW : MODE_WAVE;
            lg = mode == MODE_ROW ? rl : wave_log;
        }
        p.seg_log[p.levels] = (uint8_t)lg;
        p.mode[p.levels] = (uint8_t)mode;
        p.level_m[p.levels++] = m;
        const uint32_t seg = p.seg(p.levels - 1);
        uint32_t mo = (m + seg - 1) / seg;
        if (mo <= 1) break;
        m = mo;
    }
    return MBLS_SUCCESS;
}

// one (key, value) contribution: the histogram atomic's return value is the contribution's
// rank inside its bucket, so the scatter needs no atomics (sorted[offsets[key] + rank]).
// A wave whose lanes all hit one bucket (adversarial inputs: equal scalars) takes one atomic.
MBLS_DEV void emit_digit(uint32_t key, uint32_t val, size_t o, uint32_t* __restrict__ keys,
                         uint32_t* __restrict__ vals, uint32_t* __restrict__ ranks,
                         uint32_t* __restrict__ counts) {
    keys[o] = key;
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(key);
    const uint64_t active = __ballot(1);
    uint32_t rank = 0;
    if (__ballot(key == k0) == active) {
        if (k0 == INVALID_KEY) return;
        const uint32_t leader = (uint32_t)__builtin_ctzll(active);
        uint32_t base = 0;
        if (__lane_id() == leader) base = atomicAdd(&counts[k0], (uint32_t)__popcll(active));
        base = __shfl(base, leader, 64);
        rank = base + (uint32_t)__popcll(active & ((1ull << __lane_id()) - 1));
    } else if (key != INVALID_KEY) {
        rank = atomicAdd(&counts[key], 1u);
    }
    if (key != INVALID_KEY) {
        vals[o] = val;
        ranks[o] = rank;
    }
}

// Window geometry.  sF == 0: uniform windows, window j = bits [c j, c j + c).  sF > 0
// (precomputed bases, factor F): the scalar is cut into F blocks of sF = ceil(256 / F) bits,
// block f multiplies table entry i*F + f = 2^(sF f) P_i, and holds Wg = ceil(sF / c) windows;
// window j = f Wg + l covers bits [sF f + c l, sF f + min(c (l + 1), sF)) -- the block's last
// window is narrower when c does not divide sF.  The signed-digit carry runs through all
// windows in order; a window of width < c never carries (its value + carry <= 2^(c-1) = B).
MBLS_DEV void window_span(int j, int c, int Wg, int sF, int& pos, int& wid) {
    if (sF == 0) {
        pos = j * c;
        wid = c;
        return;
    }
    const int f = j / Wg, l = j - f * Wg;
    pos = sF * f + c * l;
    wid = min(c, sF - c * l);
}

// ------------------------------------------------------------------------------------
// 0. scalars.  The reference's raw entry digitises all 256 bits of a standard-form scalar
//    (msm_kernels.cu:86-142, W = ceil(256 / c) at :648), so ANY 32-byte s gives s P; on the
//    order-r subgroup that is (s mod r) P.  The GLV / psi splits and the closed-form digits
//    assume s < r, so standard scalars are reduced first: 2^256 < 3r, two conditional
//    subtractions (tests/test_gpu_parity.py::test_msm_noncanonical_scalars).
//    Montgomery scalars need none: from_mont of any 256-bit word string is already < r.
// ------------------------------------------------------------------------------------
MBLS_DEV void reduce_scalar_words(uint32_t (&x)[8]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        uint32_t t[8];
        const uint32_t borrow = sub_mod_raw<FrCfg>(t, x);
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = borrow ? x[i] : t[i];
    }
}
template <bool MONT>
MBLS_DEV Fr load_scalar(const uint8_t* __restrict__ scalars, size_t i) {
    Fr s = load<FrCfg>(scalars + 32 * i);
    if (MONT)
        s = from_mont(s);
    else
        reduce_scalar_words(s.v);
    return s;
}

// ------------------------------------------------------------------------------------
// 1. digits: one thread per scalar
// ------------------------------------------------------------------------------------
template <bool MONT>
__global__ __launch_bounds__(256) void k_digits(const uint8_t* __restrict__ scalars, uint32_t n, int c, int W, int Wg, int sF, uint32_t F,
                                                uint32_t B, uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                uint32_t* __restrict__ ranks, uint32_t* __restrict__ counts) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr s = load_scalar<MONT>(scalars, i);
    uint32_t carry = 0;
    for (int w = 0; w < W; ++w) {
        int bit, wid;
        window_span(w, c, Wg, sF, bit, wid);
        const uint32_t mask = (1u << wid) - 1;
        const int word = bit >> 5, sh = bit & 31;
        // select words without dynamic register indexing (which would go to scratch)
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            lo = (k == word) ? s.v[k] : lo;
            hi = (k == word + 1) ? s.v[k] : hi;
        }
        uint64_t win = ((uint64_t)hi << 32) | lo;
        uint32_t v = ((uint32_t)(win >> sh) & mask) + carry;
        carry = 0;
        uint32_t sign = 0;
        if (v > B) {  // signed digit: v - 2^c, carry into the next window (msm_kernels.cu:111-117)
            v = (1u << c) - v;
            sign = 1;
            carry = 1;
        }
        const int f = w / Wg, wl = w % Wg;
        // precomputed bases are point-major: [P_i, 2^l P_i, ..., 2^((F-1) l) P_i] (core/msm.rs:164-165)
        emit_digit(v ? (uint32_t)wl * B + (v - 1) : INVALID_KEY, ((i * F + (uint32_t)f) << 1) | sign,
                   (size_t)w * n + i, keys, vals, ranks, counts);
    }
    // canonical scalars (< r < 2^255) never leave a final carry: W*c >= 256 (checked for
    // c = 7..16 in tests/test_oracle.py)
}

// ------------------------------------------------------------------------------------
// 1b. GLV digits (G1): s = +-m1 +- m2*lam (mod r), m1, m2 < 2^127 (oracle/pyref.py
//     glv_decompose), lam = z^2 - 1 and r = lam^2 + lam + 1.  Point index i carries the m1
//     digits, index n + i (the phi(P_i) table) the m2 digits; both halves share each window's
//     buckets, so the windows halve (255 -> 127 bits) at the same contribution count.
// ------------------------------------------------------------------------------------
__constant__ uint32_t GLV_LAM[4] = {0xffffffffu, 0x00000000u, 0x0001a402u, 0xac45a401u};
__constant__ uint32_t GLV_HALF[4] = {0x7fffffffu, 0x00000000u, 0x8000d201u, 0x5622d200u};
// floor(2^383 / lam)
__constant__ uint32_t GLV_G[8] = {0xc4b6396eu, 0xed2f27c6u, 0x9345fbd1u, 0x1c4fa4d3u,
                                  0x7b67f718u, 0xb1fb7291u, 0xf00fd56eu, 0xbe35f678u};

MBLS_DEV bool gt4(const uint32_t* a, const uint32_t* b) {  // a > b, 4 words
    bool gt = false, eq = true;
#pragma unroll
    for (int k = 3; k >= 0; --k) {
        gt = gt || (eq && a[k] > b[k]);
        eq = eq && a[k] == b[k];
    }
    return gt;
}
MBLS_DEV void sub4(uint32_t* d, const uint32_t* a, const uint32_t* b) {  // d = a - b
    uint64_t br = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint64_t t = (uint64_t)a[k] - b[k] - br;
        d[k] = (uint32_t)t;
        br = (t >> 63) & 1;
    }
}
MBLS_DEV void add4_u32(uint32_t* a, uint32_t x) {
    uint64_t c = x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint64_t t = (uint64_t)a[k] + c;
        a[k] = (uint32_t)t;
        c = t >> 32;
    }
}
MBLS_DEV void sub4_u32(uint32_t* a, uint32_t x) {
    uint64_t br = x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint64_t t = (uint64_t)a[k] - br;
        a[k] = (uint32_t)t;
        br = (t >> 63) & 1;
    }
}

MBLS_DEV void glv_split(const Fr& s, uint32_t (&m1)[4], bool& neg1, uint32_t (&m2)[4], bool& neg2) {
    // q_est = floor(s * G / 2^383) in {q - 1, q}
    uint32_t prod[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) prod[k] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint64_t t = (uint64_t)s.v[i] * GLV_G[j] + prod[i + j] + c;
            prod[i + j] = (uint32_t)t;
            c = t >> 32;
        }
        prod[i + 8] = (uint32_t)c;
    }
    uint32_t q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = (prod[11 + k] >> 31) | (prod[12 + k] << 1);
    // rem = s - q * lam  (< 2 lam < 2^129)
    uint32_t ql[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) ql[k] = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint64_t t = (uint64_t)q[i] * GLV_LAM[j] + ql[i + j] + c;
            ql[i + j] = (uint32_t)t;
            c = t >> 32;
        }
        ql[i + 4] = (uint32_t)c;
    }
    uint32_t rem[5];
    {
        uint64_t br = 0;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            uint64_t t = (uint64_t)s.v[k] - ql[k] - br;
            rem[k] = (uint32_t)t;
            br = (t >> 63) & 1;
        }
    }
    uint32_t k1[4] = {rem[0], rem[1], rem[2], rem[3]};
    if (rem[4] != 0 || !gt4(GLV_LAM, k1)) {  // rem >= lam
        sub4(k1, k1, GLV_LAM);
        add4_u32(q, 1);
    }
    // balance k1 into (-lam/2, lam/2]
    neg1 = gt4(k1, GLV_HALF);
    if (neg1) {
        sub4(m1, GLV_LAM, k1);
        add4_u32(q, 1);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) m1[k] = k1[k];
    }
    // balance k2: (k2 - lam - 1) * lam == k2 * lam + 1 (mod r), so k1 absorbs a -1
    neg2 = gt4(q, GLV_HALF);
    if (neg2) {
        sub4(m2, GLV_LAM, q);
        add4_u32(m2, 1);
        if (neg1) {
            add4_u32(m1, 1);
        } else if ((m1[0] | m1[1] | m1[2] | m1[3]) == 0) {
            m1[0] = 1;
            neg1 = true;
        } else {
            sub4_u32(m1, 1);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) m2[k] = q[k];
    }
}

template <bool MONT>
__global__ __launch_bounds__(256) void k_digits_glv(const uint8_t* __restrict__ scalars, uint32_t n, int c, int W,
                                                    uint32_t B, uint32_t* __restrict__ keys,
                                                    uint32_t* __restrict__ vals, uint32_t* __restrict__ ranks,
                                                    uint32_t* __restrict__ counts, SplitLayout lay) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr s = load_scalar<MONT>(scalars, i);
    uint32_t m[2][4];
    bool neg[2];
    glv_split(s, m[0], neg[0], m[1], neg[1]);
    const uint32_t mask = (1u << c) - 1;
    const size_t stride = 2 * (size_t)n;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint32_t carry = 0;
        for (int w = 0; w < W; ++w) {
            const int bit = w * c;
            const int word = bit >> 5, sh = bit & 31;
            uint32_t lo = 0, hi = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                lo = (k == word) ? m[h][k] : lo;
                hi = (k == word + 1) ? m[h][k] : hi;
            }
            uint64_t win = ((uint64_t)hi << 32) | lo;
            uint32_t v = ((uint32_t)(win >> sh) & mask) + carry;
            carry = 0;
            uint32_t sign = neg[h] ? 1u : 0u;
            if (v > B) {
                v = (1u << c) - v;
                sign ^= 1u;
                carry = 1;
            }
            const uint32_t idx = lay.at(h, i);
            emit_digit(v ? (uint32_t)w * B + (v - 1) : INVALID_KEY, (idx << 1) | sign, (size_t)w * stride + idx, keys,
                       vals, ranks, counts);
        }
    }
}

// phi table: phi[i] = (beta x_i, y_i) (Montgomery); identity (0, 0) maps to itself.
// beta: the cube root of unity in Fq with phi(G) = lam G (oracle/pyref.py GLV_BETA)
__constant__ uint32_t GLV_BETA_MONT[12] = {0x8671f071u, 0xcd03c9e4u, 0x1fcda5d2u, 0x5dab2246u,
                                           0xd3851b95u, 0x587042afu, 0x01bacb9eu, 0x8eb60ebeu,
                                           0x83d050d2u, 0x03f97d6eu, 0x54638741u, 0x18f02065u};
__global__ void k_glv_table(const uint8_t* __restrict__ bases, uint8_t* __restrict__ phi, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fq beta;
#pragma unroll
    for (int k = 0; k < 12; ++k) beta.v[k] = GLV_BETA_MONT[k];
    Affine<Fq> p = load_affine<Fq>(bases, i);
    p.x = p.x * beta;
    store_affine<Fq>(phi, i, p);
}

// Host operands of an MSM (core/msm.rs:665,773 pass a HostSlice).  Page-locked host memory is
// read by a kernel through its device alias (PCIe reads by every CU, 4 x 16 B in flight per
// lane); hipMemcpyAsync from pinned memory ran at ~28 GB/s for the 32 MiB of a 2^20 MSM's scalars
// (VERDICT r3), below HIP's own staged copy of PAGEABLE memory (~40 GB/s).  Pageable memory and
// other devices' memory (multi-device shards) keep hipMemcpyAsync.
__global__ __launch_bounds__(256) void k_copy_pinned(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

#ifndef MBLS_PINNED_KERNEL
#define MBLS_PINNED_KERNEL 1  // variant builds: 0 = hipMemcpyAsync for pinned memory too
#endif
eIcicleError stage_to_device(void* dst, const void* src, size_t bytes, hipStream_t st) {
    const void* alias = (MBLS_PINNED_KERNEL && bytes % 16 == 0 && ((uintptr_t)src & 15) == 0)
                            ? pinned_host_device_pointer(src)
                            : nullptr;
    if (alias) {
        const size_t n16 = bytes / 16;
        size_t blocks = (n16 + 4 * 256 - 1) / (4 * 256);
        if (blocks > 2048) blocks = 2048;
        if (blocks == 0) return MBLS_SUCCESS;
        hipLaunchKernelGGL(k_copy_pinned, dim3((unsigned)blocks), dim3(256), 0, st, static_cast<uint4*>(dst),
                           static_cast<const uint4*>(alias), n16);
        MBLS_TRY(hipGetLastError());
        return MBLS_SUCCESS;
    }
    MBLS_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, st));
    return MBLS_SUCCESS;
}

eIcicleError launch_glv_table(const uint8_t* bases, uint8_t* phi, uint32_t n, hipStream_t st) {
    hipLaunchKernelGGL(k_glv_table, dim3((n + 255) / 256), dim3(256), 0, st, bases, phi, n);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// ------------------------------------------------------------------------------------
// 1b'. psi split (G2): s == sum_j (-1)^neg_j m_j psi^j(Q) on G2, m_j < 2^63
//      (oracle/pyref.py psi_decompose).  psi = [z] on G2 and r = x^4 - x^2 + 1 for x = |z|,
//      so balanced base-x digits d_j (|d_j| <= x/2) plus the carry d_4 folded back with
//      x^4 == x^2 - 1 give s == sum_j d_j x^j == sum_j (-1)^j d_j z^j.
//      Point index j*n + i carries psi^j(P_i) (k_psi_table); the digit source per index is
//      one uint4 in the GLV format (magnitude words 0-1, bit 127 = sign).
// ------------------------------------------------------------------------------------
static constexpr uint64_t PSI_X = 0xd201000000010000ull;  // |z| = PSI_XP << 16
static constexpr uint64_t PSI_XP = 0xd20100000001ull;

// t <- t div |z|, returns t mod |z|  (t: 8 little-endian u32 words).  |z| = 2^16 x' with a
// 48-bit x', so the division is a 16-bit-digit long division of t >> 16 by x' (every partial
// remainder * 2^16 + digit fits 64 bits).
MBLS_DEV uint64_t divmod_x(uint32_t (&t)[8]) {
    const uint32_t low16 = t[0] & 0xffffu;
    uint64_t r = 0;
    uint32_t q[8];
#pragma unroll
    for (int w = 7; w >= 0; --w) {
        const uint32_t uw = (t[w] >> 16) | (w < 7 ? (t[w + 1] << 16) : 0u);  // word w of t >> 16
        uint64_t cur = (r << 16) | (uw >> 16);
        const uint64_t qh = cur / PSI_XP;
        r = cur - qh * PSI_XP;
        cur = (r << 16) | (uw & 0xffffu);
        const uint64_t ql = cur / PSI_XP;
        r = cur - ql * PSI_XP;
        q[w] = (uint32_t)((qh << 16) | ql);
    }
#pragma unroll
    for (int w = 0; w < 8; ++w) t[w] = q[w];
    return (r << 16) | low16;
}

template <bool MONT>
MBLS_DEV void psi_split_one(const uint8_t* __restrict__ scalars, uint32_t n, uint4* __restrict__ out, uint32_t i,
                            SplitLayout lay) {
    Fr s = load_scalar<MONT>(scalars, i);
    uint32_t t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = s.v[k];
    int64_t d[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t rem = divmod_x(t);
        if (rem > (PSI_X >> 1)) {  // balance: rem - x, carry one into the quotient
            d[j] = -(int64_t)(PSI_X - rem);
            unsigned c = 1;
#pragma unroll
            for (int k = 0; k < 8; ++k) t[k] = __builtin_addc(t[k], 0u, c, &c);
        } else {
            d[j] = (int64_t)rem;
        }
    }
    const int64_t d4 = (int64_t)t[0];  // s < r < x^4: the fifth digit is 0 or 1
    d[2] += d4;
    d[0] -= d4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool neg = (d[j] < 0) != ((j & 1) != 0);  // psi^j = [z^j] = [(-x)^j]
        const uint64_t m = (uint64_t)(d[j] < 0 ? -d[j] : d[j]);
        out[lay.at(j, i)] = make_uint4((uint32_t)m, (uint32_t)(m >> 32), 0u, neg ? 0x80000000u : 0u);
    }
}

template <bool MONT>
__global__ __launch_bounds__(256) void k_psi_split(const uint8_t* __restrict__ scalars, uint32_t n,
                                                   uint4* __restrict__ out, ZeroList z, SplitLayout lay) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    z.run(i, gridDim.x * blockDim.x);
    if (i >= n) return;
    psi_split_one<MONT>(scalars, n, out, i, lay);
}

// psi(x, y) = (conj(x) * CX, conj(y) * CY), CX = (0, CX1) (oracle/pyref.py PSI_CX / PSI_CY),
// Montgomery limbs; the table holds psi^1..3(P_i) at (j-1)*n + i
// psi^2 x-multiplier C2 = 0x1a0111ea...00000000aaac (an Fq cube root of unity), Montgomery form
__constant__ uint32_t PSI2_CX_MONT[12] = {0x8671f071u, 0xcd03c9e4u, 0x1fcda5d2u, 0x5dab2246u, 0xd3851b95u, 0x587042afu,
                                          0x01bacb9eu, 0x8eb60ebeu, 0x83d050d2u, 0x03f97d6eu, 0x54638741u, 0x18f02065u};
__constant__ uint32_t PSI_CX1_MONT[12] = {0x867545c3u, 0x890dc9e4u, 0x3285a5d5u, 0x2af32253u, 0x309b7e2cu, 0x50880866u,
                                          0x7e881024u, 0xa20d1b8cu, 0xe2db9068u, 0x14e4f04fu, 0x1564853au, 0x14e56d3fu};
__constant__ uint32_t PSI_CY0_MONT[12] = {0xa55c9ad1u, 0x3e2f585du, 0x86c18183u, 0x4294213du, 0x8b623732u, 0x382844c8u,
                                          0x19103e18u, 0x92ad2afdu, 0xac7cf0b9u, 0x1d794e4fu, 0x7d825ec8u, 0x0bd592fcu};
__constant__ uint32_t PSI_CY1_MONT[12] = {0x5aa30fdau, 0x7bcfa7a2u, 0x2a927e7cu, 0xdc17dec1u, 0x6b4ebef1u, 0x2f088dd8u,
                                          0xda74d4a7u, 0xd1ca2087u, 0x96cebc1du, 0x2da25966u, 0xbbfd87d2u, 0x0e2b7eedu};

// Table rows staged in LDS and written out as whole lines: a lane's 96 / 192-byte row stored
// straight from registers is 24 / 48 dword stores at a 96 / 192-byte lane stride, partial-line
// writes that cost 1.6 GB of HBM traffic per 2^20-point psi table (2x its 0.6 GB of rows).
// All threads of the block call it (barriers); rows = valid rows of this block.
template <int ROW>
MBLS_DEV void block_rows_out(uint8_t* __restrict__ dst, const uint4* __restrict__ stage, uint32_t rows) {
    __syncthreads();
    const uint32_t cnt = rows * (ROW / 16);
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (uint32_t k = threadIdx.x; k < cnt; k += blockDim.x) d[k] = stage[k];
    __syncthreads();  // the stage is reused by the next table
}

// psi(P), psi^2(P), psi^3(P) of one G2 point, Montgomery
MBLS_DEV void psi_images(const Affine<Fq2>& p, Affine<Fq2>& q1, Affine<Fq2>& q2, Affine<Fq2>& q3) {
    Fq cx1;
    Fq2 cy;
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        cx1.v[k] = PSI_CX1_MONT[k];
        cy.c0.v[k] = PSI_CY0_MONT[k];
        cy.c1.v[k] = PSI_CY1_MONT[k];
    }
    // psi(P): conj(x) * (CX1 u) = x1 CX1 + x0 CX1 u, conj(y) * CY (5 Fq products); identity
    // (0, 0) maps to itself
    q1.x.c0 = p.x.c1 * cx1;
    q1.x.c1 = p.x.c0 * cx1;
    {  // conj(y) * CY, Karatsuba in line (fq2_mul is out of line: a call frame in scratch)
        const Fq a0 = p.y.c0, a1 = neg(p.y.c1);
        const Fq t0 = a0 * cy.c0, t1 = a1 * cy.c1, t2 = (a0 + a1) * (cy.c0 + cy.c1);
        q1.y = Fq2{t0 - t1, (t2 - t0) - t1};
    }
    // psi^2 = (x, y) -> (C2 x, -y) with C2 in Fq (oracle/pyref.py psi, checked numerically),
    // so psi^2(P) and psi^3(P) = psi^2(psi(P)) take 2 Fq products each (15 -> 9 per point)
    Fq c2;
#pragma unroll
    for (int k = 0; k < 12; ++k) c2.v[k] = PSI2_CX_MONT[k];
    q2 = Affine<Fq2>{Fq2{p.x.c0 * c2, p.x.c1 * c2}, neg(p.y)};
    q3 = Affine<Fq2>{Fq2{q1.x.c0 * c2, q1.x.c1 * c2}, neg(q1.y)};
}

// the block's rows of the three psi tables (table j at (j - 1) n), through one 48 KB stage.
// bstride > 1: the bases are slot 0 of a precomputed table with bstride entries per point
// (plan.bstride); the compact copy of the points goes first, [P, psi P, psi^2 P, psi^3 P] (4n rows)
MBLS_DEV void psi_block(const uint8_t* __restrict__ bases, uint8_t* __restrict__ phi, uint32_t n,
                        uint32_t bstride = 1) {
    __shared__ uint4 stage[256 * 12];
    const uint32_t b0 = blockIdx.x * blockDim.x, i = b0 + threadIdx.x;
    const uint32_t rows = min(blockDim.x, n - b0);
    Affine<Fq2> q[3];
    if (bstride > 1) {  // uniform branch
        Affine<Fq2> p;
        if (i < n) {
            p = load_affine<Fq2>(bases, (size_t)i * bstride);
            store_affine<Fq2>(stage, threadIdx.x, p);
            psi_images(p, q[0], q[1], q[2]);
        }
        block_rows_out<192>(phi + (size_t)b0 * 192, stage, rows);
        phi += (size_t)n * 192;
    } else if (i < n) {
        psi_images(load_affine<Fq2>(bases, i), q[0], q[1], q[2]);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        if (i < n) store_affine<Fq2>(stage, threadIdx.x, q[j]);
        block_rows_out<192>(phi + ((size_t)j * n + b0) * 192, stage, rows);
    }
}

__global__ __launch_bounds__(256) void k_psi_table(const uint8_t* __restrict__ bases, uint8_t* __restrict__ phi, uint32_t n) {
    psi_block(bases, phi, n);
}

// G2 front in one launch (the psi counterpart of k_glv_prep): thread i splits scalar i and
// writes psi(P_i), psi^2(P_i), psi^3(P_i) -- the table on a side stream ran beside the split and
// digit kernels and slowed both (VALU contention) more than its own time
template <bool MONT>
__global__ __launch_bounds__(256) void k_psi_prep(const uint8_t* __restrict__ scalars, uint32_t n,
                                                  uint4* __restrict__ out, ZeroList z,
                                                  const uint8_t* __restrict__ bases, uint8_t* __restrict__ phi,
                                                  uint32_t bstride) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    z.run(i, gridDim.x * blockDim.x);
    psi_block(bases, phi, n, bstride);  // every thread (block barriers)
    if (i >= n) return;
    psi_split_one<MONT>(scalars, n, out, i, SplitLayout{n, 1});
}

// Prepared bases (precompute_call with precompute_factor == the split): the point-major image
// table out[S i + j] = endo^j(P_i) -- G1 S = 2: [P, phi P]; G2 S = 4: [P, psi P, psi^2 P, psi^3 P]
// -- built once per base set (core/msm.rs:308-332 uploads the bases once per proof), so the
// MSM's front only splits scalars.  Rows through an LDS stage, written as whole lines.
__global__ __launch_bounds__(256) void k_endo_table_g1(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                        uint32_t n) {
    __shared__ uint4 stage[256 * 12];
    const uint32_t b0 = blockIdx.x * blockDim.x, i = b0 + threadIdx.x;
    if (i < n) {
        Affine<Fq> p = load_affine<Fq>(in, i);
        store_affine<Fq>(stage, 2 * threadIdx.x, p);
        Fq beta;
#pragma unroll
        for (int k = 0; k < 12; ++k) beta.v[k] = GLV_BETA_MONT[k];
        p.x = p.x * beta;
        store_affine<Fq>(stage, 2 * threadIdx.x + 1, p);
    }
    block_rows_out<192>(out + (size_t)b0 * 192, stage, min(blockDim.x, n - b0));
}

__global__ __launch_bounds__(128) void k_endo_table_g2(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                        uint32_t n) {
    __shared__ uint4 stage[128 * 48];
    const uint32_t b0 = blockIdx.x * blockDim.x, i = b0 + threadIdx.x;
    if (i < n) {
        const Affine<Fq2> p = load_affine<Fq2>(in, i);
        Affine<Fq2> q1, q2, q3;
        psi_images(p, q1, q2, q3);
        store_affine<Fq2>(stage, 4 * threadIdx.x, p);
        store_affine<Fq2>(stage, 4 * threadIdx.x + 1, q1);
        store_affine<Fq2>(stage, 4 * threadIdx.x + 2, q2);
        store_affine<Fq2>(stage, 4 * threadIdx.x + 3, q3);
    }
    block_rows_out<768>(out + (size_t)b0 * 768, stage, min(blockDim.x, n - b0));
}

eIcicleError launch_endo_table(const uint8_t* in, uint8_t* out, uint32_t n, int split, hipStream_t st) {
    if (split == 2)
        hipLaunchKernelGGL(k_endo_table_g1, dim3((n + 255) / 256), dim3(256), 0, st, in, out, n);
    else if (split == 4)
        hipLaunchKernelGGL(k_endo_table_g2, dim3((n + 127) / 128), dim3(128), 0, st, in, out, n);
    else
        return MBLS_INVALID_ARGUMENT;
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

eIcicleError launch_psi_table(const uint8_t* bases, uint8_t* phi, uint32_t n, hipStream_t st) {
    hipLaunchKernelGGL(k_psi_table, dim3((n + 255) / 256), dim3(256), 0, st, bases, phi, n);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// ------------------------------------------------------------------------------------
// 1c. tiled digits (c <= 16): workgroup (tile, window) histograms its tile's digits in LDS
//     (local rank = LDS atomic return), then flushes the histogram with ONE coalesced
//     returning global add per bucket (base of this tile in the bucket).  Random-address
//     global atomics run ~17x below the coalesced rate on CDNA4 (MI355X_MICROARCH.md, global
//     atomics: "64 lanes in 64 different rows"); this is what k_digits paid per digit.
//     Digit sources: NW words per index (GLV halves: 4 words, bit 127 = sign; plain: 8 words).
// ------------------------------------------------------------------------------------
static constexpr int DT_THREADS = 1024;
#ifndef MBLS_DT_PER
#define MBLS_DT_PER 16
#endif
static constexpr int DT_PER = MBLS_DT_PER;  // indices per thread
static constexpr uint32_t DT_TILE = DT_THREADS * DT_PER;
// gfx950 workgroup LDS limit (160 KiB per workgroup, the whole CU; MI355X_MICROARCH.md): the
// digit pass stages a whole tile (DT_TILE words) beside its 256-word part histogram
static constexpr size_t LDS_LIMIT_BYTES = 160 * 1024;
static_assert(DT_TILE * 4 + (256 + 1) * 4 <= LDS_LIMIT_BYTES, "MBLS_DT_PER too large: k_digits_part's LDS stage overflows");
static constexpr uint32_t DT_MAX_B = 1u << 15;

template <bool MONT>
__global__ __launch_bounds__(256) void k_glv_split(const uint8_t* __restrict__ scalars, uint32_t n,
                                                   uint4* __restrict__ out, ZeroList z, SplitLayout lay) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    z.run(i, gridDim.x * blockDim.x);
    if (i >= n) return;
    Fr s = load_scalar<MONT>(scalars, i);
    uint32_t m1[4], m2[4];
    bool n1, n2;
    glv_split(s, m1, n1, m2, n2);
    out[lay.at(0, i)] = make_uint4(m1[0], m1[1], m1[2], m1[3] | (n1 ? 0x80000000u : 0u));
    out[lay.at(1, i)] = make_uint4(m2[0], m2[1], m2[2], m2[3] | (n2 ? 0x80000000u : 0u));
}

// G1 front in one launch: thread i splits scalar i (k_glv_split) AND writes phi(P_i) (k_glv_table)
// -- the table no longer runs on a side stream beside the digit / sort front (its fork / join
// event waits and its contention with k_glv_split cost more than its own time)
template <bool MONT>
// bstride > 1: the bases are slot 0 of a precomputed table with bstride entries per point
// (plan.bstride, make_plan); the kernel then writes the compact [P_0..P_(n-1), phi(P_0)..] into
// `phi` (2n rows) so the accumulation reads a 2n-point table instead of the whole precomputed one
__global__ __launch_bounds__(256) void k_glv_prep(const uint8_t* __restrict__ scalars, uint32_t n,
                                                  uint4* __restrict__ out, ZeroList z,
                                                  const uint8_t* __restrict__ bases, uint8_t* __restrict__ phi,
                                                  uint32_t bstride) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    z.run(i, gridDim.x * blockDim.x);
    {  // phi rows through a 24 KB stage, written as whole lines (block_rows_out)
        __shared__ uint4 stage[256 * 6];
        const uint32_t b0 = blockIdx.x * blockDim.x;
        const uint32_t rows = min(blockDim.x, n - b0);
        Affine<Fq> p;
        if (i < n) p = load_affine<Fq>(bases, (size_t)i * bstride);
        uint8_t* phi_rows = phi;
        if (bstride > 1) {  // the compact copy of the points first (uniform branch)
            if (i < n) store_affine<Fq>(stage, threadIdx.x, p);
            block_rows_out<96>(phi + (size_t)b0 * 96, stage, rows);
            phi_rows = phi + (size_t)n * 96;
        }
        if (i < n) {
            Fq beta;
#pragma unroll
            for (int k = 0; k < 12; ++k) beta.v[k] = GLV_BETA_MONT[k];
            p.x = p.x * beta;
            store_affine<Fq>(stage, threadIdx.x, p);
        }
        block_rows_out<96>(phi_rows + (size_t)b0 * 96, stage, rows);
    }
    if (i >= n) return;
    Fr s = load_scalar<MONT>(scalars, i);
    uint32_t m1[4], m2[4];
    bool n1, n2;
    glv_split(s, m1, n1, m2, n2);
    out[i] = make_uint4(m1[0], m1[1], m1[2], m1[3] | (n1 ? 0x80000000u : 0u));
    out[n + i] = make_uint4(m2[0], m2[1], m2[2], m2[3] | (n2 ? 0x80000000u : 0u));
}

__global__ void k_scalars_std(const uint8_t* __restrict__ scalars, uint32_t n, uint8_t* __restrict__ out, ZeroList z) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    z.run(i, gridDim.x * blockDim.x);
    if (i >= n) return;
    store<FrCfg>(out + 32 * (size_t)i, from_mont(load<FrCfg>(scalars + 32 * (size_t)i)));
}

// signed digit of window w (carry chain from window 0), magnitude in v, sign in bit 31
template <int NW>
MBLS_DEV uint32_t digit_at(const uint32_t (&x)[NW], int w, int c, uint32_t B, int Wg, int sF) {
    uint32_t carry = 0, v = 0;
    for (int j = 0; j <= w; ++j) {
        int bit, wid;
        window_span(j, c, Wg, sF, bit, wid);
        const int word = bit >> 5, sh = bit & 31;
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            lo = (k == word) ? x[k] : lo;
            hi = (k == word + 1) ? x[k] : hi;
        }
        v = ((uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & ((1u << wid) - 1)) + carry;
        carry = v > B ? 1u : 0u;
    }
    return carry ? (((1u << c) - v) | 0x80000000u) : v;
}

// GLV: indices [0, 2n) over the split halves, vals (idx << 1 | sign), key w*B + v - 1.
// plain: indices [0, n) over scalars, vals ((i*F + w/Wg) << 1 | sign), key (w%Wg)*B + v - 1.
template <bool GLV>
__global__ __launch_bounds__(DT_THREADS) void k_digits_tiled(const uint32_t* __restrict__ src, uint32_t nidx, int c,
                                                             int Wg, int sF, uint32_t F, uint32_t B,
                                                             uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                             uint32_t* __restrict__ ranks, uint32_t* __restrict__ counts) {
    __shared__ uint32_t hist[DT_MAX_B];
    constexpr int NW = GLV ? 4 : 8;
    const uint32_t tiles = (nidx + DT_TILE - 1) / DT_TILE;
    const uint32_t tile = blockIdx.x % tiles;
    const int w = (int)(blockIdx.x / tiles);
    const uint32_t wl = GLV ? (uint32_t)w : (uint32_t)(w % Wg), f = GLV ? 0u : (uint32_t)(w / Wg);
    for (uint32_t j = threadIdx.x; j < B; j += DT_THREADS) hist[j] = 0;
    __syncthreads();
    uint32_t dig[DT_PER], lr[DT_PER];
#pragma unroll
    for (int k = 0; k < DT_PER; ++k) {
        const uint32_t idx = tile * DT_TILE + k * DT_THREADS + threadIdx.x;
        dig[k] = 0;
        lr[k] = 0;
        if (idx < nidx) {
            uint32_t x[NW];
            const uint4* p = reinterpret_cast<const uint4*>(src) + (size_t)idx * (NW / 4);
#pragma unroll
            for (int q = 0; q < NW / 4; ++q) {
                const uint4 u = p[q];
                x[4 * q] = u.x;
                x[4 * q + 1] = u.y;
                x[4 * q + 2] = u.z;
                x[4 * q + 3] = u.w;
            }
            uint32_t negh = 0;
            if constexpr (GLV) {
                negh = x[3] >> 31;
                x[3] &= 0x7fffffffu;
            } else {
                reduce_scalar_words(x);  // standard scalars read in place (section 0)
            }
            const uint32_t d = digit_at<NW>(x, w, c, B, Wg, sF) ^ (negh << 31);
            dig[k] = d;
            if (d & 0x7fffffffu) lr[k] = atomicAdd(&hist[(d & 0x7fffffffu) - 1], 1u);
        }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < B; j += DT_THREADS) {
        const uint32_t h = hist[j];
        hist[j] = h ? atomicAdd(&counts[wl * B + j], h) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < DT_PER; ++k) {
        const uint32_t idx = tile * DT_TILE + k * DT_THREADS + threadIdx.x;
        if (idx >= nidx) continue;
        const size_t o = (size_t)w * nidx + idx;
        const uint32_t v = dig[k] & 0x7fffffffu, sign = dig[k] >> 31;
        if (v == 0) {
            keys[o] = INVALID_KEY;
            continue;
        }
        keys[o] = wl * B + v - 1;
        vals[o] = ((GLV ? idx : idx * F + f) << 1) | sign;
        ranks[o] = hist[v - 1] + lr[k];
    }
}

// digit sources per scalar: GLV 2 x 16 B, psi 4 x 16 B, plain standard scalars 32 B
size_t digits_src_bytes(uint32_t n, int split) { return (size_t)n * (split == 4 ? 64 : 32); }

// the tiled digit kernels' sources: split halves / quarters (sign-magnitude uint4s) or
// standard-form scalars; nidx = digit-source entries
__global__ void k_zero_list(ZeroList z) { z.run(blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x); }

// the MSM's first kernel also clears the words later kernels accumulate into (ZeroList): a
// separate hipMemsetAsync is a fill kernel of its own, ~9-18 us on the critical path each
static eIcicleError digit_sources(const uint8_t* scalars, bool mont, uint32_t n, const MsmPlan& P, uint8_t* dsrc,
                                  const ZeroList& z, hipStream_t st, const uint32_t*& src, uint32_t& nidx,
                                  const uint8_t* bases = nullptr, uint8_t* phi = nullptr) {
    dim3 g((n + 255) / 256);
    // digit-source (= point) index of stream j of scalar i: j n + i against the per-call image
    // table, i S + j against a prepared point-major table [P, phi P] / [P, psi P, psi^2 P, psi^3 P]
    const SplitLayout lay = P.prepared ? SplitLayout{1u, (uint32_t)P.split} : SplitLayout{n, 1u};
    if (P.split == 2 && phi) {  // split + phi table fused (k_glv_prep)
        if (mont)
            hipLaunchKernelGGL(k_glv_prep<true>, g, dim3(256), 0, st, scalars, n, (uint4*)dsrc, z, bases, phi,
                               (uint32_t)P.bstride);
        else
            hipLaunchKernelGGL(k_glv_prep<false>, g, dim3(256), 0, st, scalars, n, (uint4*)dsrc, z, bases, phi,
                               (uint32_t)P.bstride);
        src = (const uint32_t*)dsrc;
        nidx = 2 * n;
    } else if (P.split == 2) {
        if (mont)
            hipLaunchKernelGGL(k_glv_split<true>, g, dim3(256), 0, st, scalars, n, (uint4*)dsrc, z, lay);
        else
            hipLaunchKernelGGL(k_glv_split<false>, g, dim3(256), 0, st, scalars, n, (uint4*)dsrc, z, lay);
        src = (const uint32_t*)dsrc;
        nidx = 2 * n;
    } else if (P.split == 4 && phi) {  // split + psi table fused (k_psi_prep)
        if (mont)
            hipLaunchKernelGGL(k_psi_prep<true>, g, dim3(256), 0, st, scalars, n, (uint4*)dsrc, z, bases, phi,
                               (uint32_t)P.bstride);
        else
            hipLaunchKernelGGL(k_psi_prep<false>, g, dim3(256), 0, st, scalars, n, (uint4*)dsrc, z, bases, phi,
                               (uint32_t)P.bstride);
        src = (const uint32_t*)dsrc;
        nidx = 4 * n;
    } else if (P.split == 4) {
        if (mont)
            hipLaunchKernelGGL(k_psi_split<true>, g, dim3(256), 0, st, scalars, n, (uint4*)dsrc, z, lay);
        else
            hipLaunchKernelGGL(k_psi_split<false>, g, dim3(256), 0, st, scalars, n, (uint4*)dsrc, z, lay);
        src = (const uint32_t*)dsrc;
        nidx = 4 * n;
    } else {
        if (mont)
            hipLaunchKernelGGL(k_scalars_std, g, dim3(256), 0, st, scalars, n, dsrc, z);
        else
            hipLaunchKernelGGL(k_zero_list, dim3(8), dim3(256), 0, st, z);
        src = (const uint32_t*)(mont ? dsrc : scalars);
        nidx = n;
    }
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

eIcicleError launch_digits(const uint8_t* scalars, bool mont, uint32_t n, const MsmPlan& P, uint32_t* keys,
                           uint32_t* vals, uint32_t* ranks, uint32_t* counts, uint8_t* dsrc, hipStream_t st) {
    dim3 g((n + 255) / 256);
    if (P.B <= DT_MAX_B) {
        const uint32_t* src;
        uint32_t nidx;
        eIcicleError er = digit_sources(scalars, mont, n, P, dsrc, ZeroList{}, st, src, nidx);
        if (er != MBLS_SUCCESS) return er;
        const uint32_t tiles = (nidx + DT_TILE - 1) / DT_TILE;
        dim3 gt(tiles * (uint32_t)P.W);
        if (P.split > 1)  // GLV / psi sources share the sign-magnitude uint4 format
            hipLaunchKernelGGL(k_digits_tiled<true>, gt, dim3(DT_THREADS), 0, st, src, nidx, P.c, P.Wg, P.sF, (uint32_t)P.F,
                               P.B, keys, vals, ranks, counts);
        else
            hipLaunchKernelGGL(k_digits_tiled<false>, gt, dim3(DT_THREADS), 0, st, src, nidx, P.c, P.Wg, P.sF,
                               (uint32_t)P.F, P.B, keys, vals, ranks, counts);
        MBLS_TRY(hipGetLastError());
        return MBLS_SUCCESS;
    }
    if (P.split == 4) return MBLS_INVALID_ARGUMENT;  // make_plan keeps psi to c <= 16
    if (P.split == 2) {
        const SplitLayout lay = P.prepared ? SplitLayout{1u, 2u} : SplitLayout{n, 1u};
        if (mont)
            hipLaunchKernelGGL(k_digits_glv<true>, g, dim3(256), 0, st, scalars, n, P.c, P.W, P.B, keys, vals, ranks, counts,
                               lay);
        else
            hipLaunchKernelGGL(k_digits_glv<false>, g, dim3(256), 0, st, scalars, n, P.c, P.W, P.B, keys, vals, ranks,
                               counts, lay);
    } else if (mont)
        hipLaunchKernelGGL(k_digits<true>, g, dim3(256), 0, st, scalars, n, P.c, P.W, P.Wg, P.sF, (uint32_t)P.F, P.B, keys,
                           vals, ranks, counts);
    else
        hipLaunchKernelGGL(k_digits<false>, g, dim3(256), 0, st, scalars, n, P.c, P.W, P.Wg, P.sF, (uint32_t)P.F, P.B, keys,
                           vals, ranks, counts);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// ------------------------------------------------------------------------------------
// 2. exclusive scan: three phases, 1024 elements per block, wave64 shuffles
// ------------------------------------------------------------------------------------
// (wave_incl_scan: msm_core.hpp)

__device__ __forceinline__ void block_scan_1024(uint32_t (&x)[4], uint32_t* sh_wave, uint32_t& total) {
    uint32_t s0 = x[0], s1 = s0 + x[1], s2 = s1 + x[2], s3 = s2 + x[3];
    uint32_t incl = wave_incl_scan(s3);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 63) sh_wave[wid] = incl;
    __syncthreads();
    uint32_t wave_off = 0;
    for (int k = 0; k < wid; ++k) wave_off += sh_wave[k];
    total = sh_wave[0] + sh_wave[1] + sh_wave[2] + sh_wave[3];
    uint32_t excl = wave_off + incl - s3;
    x[0] = excl;
    x[1] = excl + s0;
    x[2] = excl + s1;
    x[3] = excl + s2;
}

__global__ __launch_bounds__(256) void k_scan_local(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                    uint32_t* __restrict__ block_sums, uint32_t m) {
    __shared__ uint32_t sh[4];
    uint32_t base = blockIdx.x * SCAN_BLOCK + threadIdx.x * 4;
    uint32_t x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = (base + k < m) ? in[base + k] : 0u;
    uint32_t total;
    block_scan_1024(x, sh, total);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + k < m) out[base + k] = x[k];
    if (threadIdx.x == 0) block_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_scan_blocks(uint32_t* __restrict__ sums, uint32_t nb, uint32_t* __restrict__ grand) {
    __shared__ uint32_t sh[4];
    uint32_t carry = 0;
    for (uint32_t off = 0; off < nb; off += SCAN_BLOCK) {
        uint32_t base = off + threadIdx.x * 4;
        uint32_t x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = (base + k < nb) ? sums[base + k] : 0u;
        uint32_t total;
        block_scan_1024(x, sh, total);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (base + k < nb) sums[base + k] = x[k] + carry;
        carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) *grand = carry;
}

__global__ __launch_bounds__(256) void k_scan_add(uint32_t* __restrict__ out, const uint32_t* __restrict__ sums, uint32_t m,
                                                  const uint32_t* __restrict__ grand) {
    uint32_t base = blockIdx.x * SCAN_BLOCK + threadIdx.x * 4;
    uint32_t add = sums[blockIdx.x];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + k < m) out[base + k] += add;
    if (blockIdx.x == 0 && threadIdx.x == 0) out[m] = *grand;
}

size_t scan_tmp_words(uint32_t m) { return (m + SCAN_BLOCK - 1) / SCAN_BLOCK + 8; }

eIcicleError scan_exclusive(const uint32_t* in, uint32_t* out, uint32_t m, uint32_t* tmp, hipStream_t st) {
    uint32_t nb = (m + SCAN_BLOCK - 1) / SCAN_BLOCK;
    hipLaunchKernelGGL(k_scan_local, dim3(nb), dim3(256), 0, st, in, out, tmp, m);
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(256), 0, st, tmp, nb, tmp + nb);
    hipLaunchKernelGGL(k_scan_add, dim3(nb), dim3(256), 0, st, out, tmp, m, tmp + nb);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// ------------------------------------------------------------------------------------
// 2b. partitioned counting sort (c <= 16), replacing keys / vals / ranks + the random scatter.
//   pass A (k_digits_part): workgroup (tile, window) = one SEGMENT buckets its tile's digits
//     into NP <= 256 coarse PARTS (the top bits of bucket - 1) in LDS and writes them
//     part-contiguously into its own DT_TILE-entry slice of `ent`, each entry carrying the FB
//     fine bits; per-part totals go to part_tot with NP coalesced atomics per workgroup.
//   pass B (k_part_sort): workgroup (window group, part) gathers that part from every segment
//     of its windows, counts its 2^FB fine buckets in LDS, writes their counts / offsets and
//     places the entries into the part's span of `sorted`.
//   Every global write lands in a region one workgroup owns (its slice of ent, its part's span
//   of sorted), so L2 assembles whole lines instead of 4-byte random writes reaching HBM.
//   Entry: packed (val | fine << (32 - FB)) when val < 2^(32 - FB), else uint2 {fine, val}.
// ------------------------------------------------------------------------------------
static int part_fine_bits(uint32_t B) {
    const int lb = 31 - __builtin_clz(B);
    return lb > 8 ? lb - 8 : 0;
}

bool partition_sort(const MsmPlan& P) { return MBLS_PART_SORT && P.B <= DT_MAX_B; }

PartSortSizes part_sort_sizes(const MsmPlan& P) {
    PartSortSizes s;
    const size_t nidx = P.split > 1 ? P.pts : P.pts / P.F;
    s.FB = part_fine_bits(P.B);
    s.NP = P.B >> s.FB;
    s.tiles = (uint32_t)((nidx + DT_TILE - 1) / DT_TILE);
    s.segments = s.tiles * (uint32_t)P.W;
    s.pack = (uint64_t)P.pts <= (1ull << (31 - s.FB));
    s.ent = (size_t)s.segments * DT_TILE * (s.pack ? 4 : 8);
    s.segtab = (size_t)s.segments * s.NP * 4;
    s.parts = ((size_t)P.Wg * s.NP + 1) * 4;
    return s;
}

// Signed digits in closed form: with C = sum (B - 1) 2^pos_w over the full-width windows w, the
// bits e_w of s + C at window w's span (window_span) give d_w = e_w - (B - 1) in [1 - B, B] for a
// full window -- the unique signed representation with that digit range, so exactly digit_at's
// carry-chain digits, without its loop over the lower windows (O(w) per digit) -- and d_w = e_w
// for the narrower top window of a shift-table block (sF not a multiple of c), which never
// carries in the chain.  The two representations differ only where a narrow window's digits and
// carry add up to 2^wid (the chain's digit 2^wid, here 0 and one more in the next block); both
// sum to s, and the result is the same point.  s + C < 2^(c W) (uniform windows) or 2^256 (shift
// tables: s < 2^255 and C's top term is below 2^255) for the plans make_plan picks; NW + 1 words
// hold it.
struct DigitOffset {
    uint32_t w[9];
};
static DigitOffset digit_offset(int c, int W, uint32_t B, int Wg, int sF) {
    DigitOffset o{};
    for (int j = 0; j < W; ++j) {
        int pos = c * j, wid = c;
        if (sF) {
            const int f = j / Wg, l = j - f * Wg;
            pos = sF * f + c * l;
            wid = std::min(c, sF - c * l);
        }
        if (wid != c) continue;
        const uint64_t v = (uint64_t)(B - 1) << (pos & 31);
        const int k = pos >> 5;
        if (k < 9) o.w[k] += (uint32_t)v;  // windows do not overlap: no carries between terms
        if (k + 1 < 9) o.w[k + 1] += (uint32_t)(v >> 32);
    }
    return o;
}
template <int NW>
MBLS_DEV uint32_t digit_closed(const uint32_t (&x)[NW], const DigitOffset& C, int w, int c, uint32_t B, int Wg,
                               int sF) {
    uint32_t y[NW + 1];
    unsigned carry = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) y[k] = __builtin_addc(x[k], C.w[k], carry, &carry);
    y[NW] = C.w[NW] + carry;
    int bit, wid;
    window_span(w, c, Wg, sF, bit, wid);
    const int word = bit >> 5, sh = bit & 31;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int k = 0; k <= NW; ++k) {
        lo = (k == word) ? y[k] : lo;
        hi = (k == word + 1) ? y[k] : hi;
    }
    const uint32_t e = (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & ((1u << wid) - 1);
    if (wid != c) return e;  // a block's narrow top window
    // d = e - (B - 1): positive (e >= B - 1) or -(B - 1 - e), as magnitude | sign bit
    return e >= B - 1 ? e - (B - 1) : ((B - 1 - e) | 0x80000000u);
}

template <bool SPLIT, bool PACK>
__global__ __launch_bounds__(DT_THREADS) void k_digits_part(const uint32_t* __restrict__ src, uint32_t nidx, int c,
                                                            int Wg, int sF, uint32_t F, uint32_t B, int FB, uint32_t NP,
                                                            uint32_t* __restrict__ ent, uint32_t* __restrict__ seg_off,
                                                            uint32_t* __restrict__ seg_cnt,
                                                            uint32_t* __restrict__ part_tot, DigitOffset C) {
    __shared__ uint32_t hist[256], tile_n;
    // packed entries: the tile's slice of `ent` is assembled in LDS and written out in order
    // (whole lines) instead of one random 4-byte store per contribution
    __shared__ uint32_t stage[PACK ? DT_TILE : 1];
    constexpr int NW = SPLIT ? 4 : 8;
    const uint32_t tiles = (nidx + DT_TILE - 1) / DT_TILE;
    const uint32_t seg = blockIdx.x;  // w * tiles + tile
    const uint32_t tile = seg % tiles;
    const int w = (int)(seg / tiles);
    const uint32_t wl = SPLIT ? (uint32_t)w : (uint32_t)(w % Wg), f = SPLIT ? 0u : (uint32_t)(w / Wg);
    if (threadIdx.x < 256) hist[threadIdx.x] = 0;
    __syncthreads();
    uint32_t dig[DT_PER], lr[DT_PER];
#pragma unroll
    for (int k = 0; k < DT_PER; ++k) {
        const uint32_t idx = tile * DT_TILE + k * DT_THREADS + threadIdx.x;
        dig[k] = 0;
        lr[k] = 0;
        if (idx < nidx) {
            uint32_t x[NW];
            const uint4* p = reinterpret_cast<const uint4*>(src) + (size_t)idx * (NW / 4);
#pragma unroll
            for (int q = 0; q < NW / 4; ++q) {
                const uint4 u = p[q];
                x[4 * q] = u.x;
                x[4 * q + 1] = u.y;
                x[4 * q + 2] = u.z;
                x[4 * q + 3] = u.w;
            }
            uint32_t negh = 0;
            if constexpr (SPLIT) {
                negh = x[3] >> 31;
                x[3] &= 0x7fffffffu;
            } else {
                reduce_scalar_words(x);  // standard scalars read in place (section 0)
            }
            const uint32_t d = digit_closed<NW>(x, C, w, c, B, Wg, sF) ^ (negh << 31);
            dig[k] = d;
            if (d & 0x7fffffffu) lr[k] = atomicAdd(&hist[((d & 0x7fffffffu) - 1) >> FB], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // wave 0: exclusive scan of the NP part sizes, 4 per lane
        const uint32_t l = threadIdx.x;
        uint32_t h[4], s = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            h[k] = 4 * l + k < NP ? hist[4 * l + k] : 0u;
            s += h[k];
        }
        uint32_t run = wave_incl_scan(s) - s;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t j = 4 * l + k;
            if (j < NP) {
                hist[j] = run;
                seg_off[seg * NP + j] = run;
                seg_cnt[seg * NP + j] = h[k];
                if (h[k]) atomicAdd(&part_tot[wl * NP + j], h[k]);
            }
            run += h[k];
        }
        if (l == 63) tile_n = run;  // entries of this tile
    }
    __syncthreads();
    const uint32_t fmask = (1u << FB) - 1;
#pragma unroll
    for (int k = 0; k < DT_PER; ++k) {
        const uint32_t idx = tile * DT_TILE + k * DT_THREADS + threadIdx.x;
        const uint32_t v = dig[k] & 0x7fffffffu, sign = dig[k] >> 31;
        if (idx >= nidx || v == 0) continue;
        const uint32_t part = (v - 1) >> FB, fine = (v - 1) & fmask;
        const uint32_t val = ((SPLIT ? idx : idx * F + f) << 1) | sign;
        if (PACK)
            stage[hist[part] + lr[k]] = FB ? (val | (fine << (32 - FB))) : val;
        else
            reinterpret_cast<uint2*>(ent)[(size_t)seg * DT_TILE + hist[part] + lr[k]] = make_uint2(fine, val);
    }
    if constexpr (PACK) {
        __syncthreads();
        const uint32_t nt = tile_n;
        uint32_t* dst = ent + (size_t)seg * DT_TILE;
        for (uint32_t i = threadIdx.x; i < nt; i += DT_THREADS) dst[i] = stage[i];
    }
}

// order-histogram index of (block, bin): group-major, then bin (heaviest first: the longest
// bucket sums start first), then block inside the group; bpg = blocks of 256 buckets per group
MBLS_DEV uint32_t order_index(uint32_t blk, uint32_t bin, uint32_t bpg) {
    return (blk / bpg) * (ORDER_BINS * bpg) + (SMALL_MAX - bin) * bpg + blk % bpg;
}

template <bool PACK>
__device__ __forceinline__ void part_entry(const uint32_t* __restrict__ ent, size_t o, int FB, uint32_t& fine,
                                           uint32_t& val) {
    if (PACK) {
        const uint32_t e = ent[o];
        fine = FB ? e >> (32 - FB) : 0u;
        val = FB ? e & ((1u << (32 - FB)) - 1) : e;
    } else {
        const uint2 e = reinterpret_cast<const uint2*>(ent)[o];
        fine = e.x;
        val = e.y;
    }
}

// teams of PS_TEAM lanes walk the segments of the workgroup's windows (64 B contiguous per
// team and load when packed)
#ifndef MBLS_PS_TEAM
#define MBLS_PS_TEAM 16
#endif
static constexpr uint32_t PS_TEAM = MBLS_PS_TEAM;
// LDS stage of one part's span of `sorted`: 2^21 x 8 contributions over 8 x 256 parts average
// 8192 entries per part at G1 2^20; 9216 words (36 KB) leave four workgroups per CU
#ifndef MBLS_PS_STAGE
#define MBLS_PS_STAGE 9216
#endif
static constexpr uint32_t PS_STAGE = MBLS_PS_STAGE;
static_assert(PS_STAGE * 4 + (2 * 128 + 1) * 4 <= LDS_LIMIT_BYTES, "MBLS_PS_STAGE too large for the workgroup LDS");

// register-kept entries of the partition sort (k_part_sort): segments per team, entries per lane
// and segment; MBLS_PS_KEEP=0 builds without it (A/B)
static constexpr uint32_t PS_RS = 8, PS_RK = 6;
#ifndef MBLS_PS_KEEP
#define MBLS_PS_KEEP 1
#endif
static constexpr bool PS_KEEP = MBLS_PS_KEEP != 0;

// rank of this lane's entry in LDS counter cnt[key]: the lanes sharing the key of the first
// remaining lane take one atomic together (up to PEEL such keys per call), the rest one atomic
// per lane.  Skewed scalars put most of a heavy part's entries into one fine bucket.  Ranks
// inside a bucket follow lane order, which only permutes the bucket's summands.  PEEL = 1 / 2 /
// 4 measured equal within noise on the skewed distributions of tools/skew_probe.py (1 best:
// half ones 3.53 / 3.63 / 3.65 ms): the heavy part's lone workgroup is not bound by its atomics.
#ifndef MBLS_PS_PEEL
#define MBLS_PS_PEEL 1
#endif
template <int PEEL>
MBLS_DEV uint32_t lds_rank(uint32_t* cnt, uint32_t key) {
    const uint32_t lane = __lane_id();
    const uint64_t below = (1ull << lane) - 1;
    uint64_t rem = __ballot(1);
    // the first group: its leader is the first active lane, so its key and the atomic's result
    // broadcast with v_readfirstlane (no LDS round trip besides the atomic itself)
    {
        const uint32_t k = __builtin_amdgcn_readfirstlane(key);
        const uint64_t m = __ballot(key == k);
        uint32_t base = 0;
        if (lane == (uint32_t)__builtin_ctzll(rem)) base = atomicAdd(&cnt[k], (uint32_t)__popcll(m));
        base = __builtin_amdgcn_readfirstlane(base);
        if ((m >> lane) & 1) return base + (uint32_t)__popcll(m & below);
        rem &= ~m;
    }
    for (int p = 1; p < PEEL && rem; ++p) {
        const uint32_t src = (uint32_t)__builtin_ctzll(rem);
        const uint32_t k = __shfl(key, (int)src, 64);
        const uint64_t m = __ballot(key == k) & rem;
        uint32_t base = 0;
        if (lane == src) base = atomicAdd(&cnt[k], (uint32_t)__popcll(m));
        base = __shfl(base, (int)src, 64);
        if ((m >> lane) & 1) return base + (uint32_t)__popcll(m & below);
        rem &= ~m;
    }
    return atomicAdd(&cnt[key], 1u);
}

// the counting pass's form of lds_rank: no ranks, so no atomic waits for its result
MBLS_DEV void lds_count(uint32_t* cnt, uint32_t key) {
    const uint32_t k = __builtin_amdgcn_readfirstlane(key);
    const uint64_t m = __ballot(key == k);
    if (key != k)
        atomicAdd(&cnt[key], 1u);
    else if (__lane_id() == (uint32_t)__builtin_ctzll(__ballot(1)))
        atomicAdd(&cnt[k], (uint32_t)__popcll(m));
}

// the entries of one segment's part (k of them from ent[o]), PS_U loads in flight per lane (a
// heavy part's workgroup walks up to 2^20 entries: one load latency per entry was its bound)
#ifndef MBLS_PS_U
#define MBLS_PS_U 16  // G1 2^20 all-1 scalars: 1.55 / 1.49 / 1.46 ms with 4 / 8 / 16; random unchanged
#endif
static constexpr uint32_t PS_U = MBLS_PS_U;
template <bool PACK, uint32_t TEAM = PS_TEAM, class Fn>
MBLS_DEV void part_walk(const uint32_t* __restrict__ ent, size_t o, uint32_t k, uint32_t tl, int FB, Fn&& fn) {
    for (uint32_t i = tl; i < k; i += PS_U * TEAM) {
        uint32_t fine[PS_U], val[PS_U];
        // unconditional loads (a clamped index past the segment's end): straight-line code keeps
        // all PS_U loads in flight together
#pragma unroll
        for (uint32_t u = 0; u < PS_U; ++u)
            part_entry<PACK>(ent, o + min(i + u * TEAM, k - 1), FB, fine[u], val[u]);
#pragma unroll
        for (uint32_t u = 0; u < PS_U; ++u)
            if (i + u * TEAM < k) fn(fine[u], val[u]);
    }
}

// workgroup size of k_part_sort: a heavy part (skewed scalars) is walked by one workgroup, whose
// dependent LDS ranks are latency-bound at four waves.  1024 threads (G1 2^20, tools/skew_probe.py):
// every scalar 1 3.57 -> 1.78 ms, 8-bit scalars 2.38 -> 1.71, half ones 4.36 -> 3.55; random
// scalars unchanged (4.26-4.37 / 4.28-4.30)
#ifndef MBLS_PS_THREADS
#define MBLS_PS_THREADS 1024
#endif
static constexpr uint32_t PS_THREADS = MBLS_PS_THREADS;
static_assert(PS_THREADS % 64 == 0 && PS_THREADS <= 1024 && PS_THREADS >= 256, "MBLS_PS_THREADS");

// ---- heavy parts (skewed scalars, round 5) ----
// A part holding far more entries than the average (one repeated scalar: 2^20 entries in one or
// two parts of every window at G1 2^20) was walked twice by its lone workgroup: sort 0.55 ms
// against 0.13 for random scalars.  k_part_heavy_count plans helpers for such parts from
// part_tot (every workgroup derives the same plan, part_plan): a part above max(PH_MIN, 4 x the
// average) entries is heavy and gets ceil(tot / Q) helpers, Q = max(PH_QMIN, heavy entries /
// (PH_HELPERS - heavy parts)), so at most PH_HELPERS in all; helper i of H takes the part's
// segments [S i / H, S (i + 1) / H) and counts their fine keys into hh[helper].  k_part_sort then
// takes a heavy part's fine counts as the sum of its helpers' (its own workgroup: offsets, counts,
// chunk counts, no walk), and its PH_HELPERS extra workgroups place their ranges: part base +
// fine prefix + the earlier helpers' counts of the key + LDS rank.  Without a heavy part (random
// scalars) every helper exits after the plan.  MBLS_PS_HELP=0 builds without them (A/B).
#ifndef MBLS_PS_HELP
#define MBLS_PS_HELP 1
#endif
static constexpr uint32_t PH_MIN = 32768, PH_QMIN = 8192;

// fn(p, first, H) for every part p < M in order per thread (H = 0: light); all PS_THREADS threads
template <class Fn>
MBLS_DEV void part_plan(const uint32_t* __restrict__ part_tot, uint32_t M, Fn&& fn) {
    constexpr uint32_t NWV = PS_THREADS / 64;
    __shared__ uint32_t red[4][NWV];
    const uint32_t per = (M + PS_THREADS - 1) / PS_THREADS;
    const uint32_t p0 = min(threadIdx.x * per, M), p1 = min(p0 + per, M), wv = threadIdx.x >> 6;
    auto bsum = [&](uint32_t v, uint32_t* r) {
        for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
        if ((threadIdx.x & 63) == 0) r[wv] = v;
        __syncthreads();
        uint32_t t = 0;
#pragma unroll
        for (uint32_t k = 0; k < NWV; ++k) t += r[k];
        return t;
    };
    uint32_t a = 0;
    for (uint32_t p = p0; p < p1; ++p) a += part_tot[p];
    const uint32_t total = bsum(a, red[0]);
    const uint32_t thr = max(PH_MIN, (uint32_t)(4ull * total / M));
    uint32_t nh = 0, hs = 0;
    for (uint32_t p = p0; p < p1; ++p) {
        const uint32_t t = part_tot[p];
        if (t > thr) ++nh, hs += t;
    }
    nh = bsum(nh, red[1]);
    hs = bsum(hs, red[2]);
    // many heavy parts already spread over many workgroups: no helpers
    const bool on = nh > 0 && nh <= PH_HELPERS / 2;
    const uint32_t Q = on ? max(PH_QMIN, (uint32_t)(((uint64_t)hs + (PH_HELPERS - nh) - 1) / (PH_HELPERS - nh))) : 1u;
    auto helpers = [&](uint32_t t) { return on && t > thr ? (t + Q - 1) / Q : 0u; };
    uint32_t hc = 0;
    for (uint32_t p = p0; p < p1; ++p) hc += helpers(part_tot[p]);
    const uint32_t incl = wave_incl_scan(hc);
    if ((threadIdx.x & 63) == 63) red[3][wv] = incl;
    __syncthreads();
    uint32_t first = incl - hc;
    for (uint32_t k = 0; k < wv; ++k) first += red[3][k];
    for (uint32_t p = p0; p < p1; ++p) {
        const uint32_t H = helpers(part_tot[p]);
        fn(p, first, H);
        first += H;
    }
}

// helper i of H's segment range of a part with S segments
MBLS_DEV void helper_range(uint32_t S, uint32_t i, uint32_t H, uint32_t& s0, uint32_t& s1) {
    s0 = (uint32_t)((uint64_t)S * i / H);
    s1 = (uint32_t)((uint64_t)S * (i + 1) / H);
}

// grid PH_HELPERS: the plan (help, hpart) and the helpers' fine counts (hh)
template <bool PACK>
__global__ __launch_bounds__(PS_THREADS) void k_part_heavy_count(const uint32_t* __restrict__ ent,
                                                          const uint32_t* __restrict__ seg_off,
                                                          const uint32_t* __restrict__ seg_cnt,
                                                          const uint32_t* __restrict__ part_tot, uint32_t tiles, int W,
                                                          int Wg, int FB, uint32_t NP, PartHelp hp) {
    __shared__ uint32_t cnt[128], mine[3];
    const uint32_t M = (uint32_t)Wg * NP, g = blockIdx.x;
    if (threadIdx.x < 128) cnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) mine[0] = ~0u, mine[1] = mine[2] = 0;
    __syncthreads();
    part_plan(part_tot, M, [&](uint32_t p, uint32_t first, uint32_t H) {
        if (p % PH_HELPERS == g) hp.help[p] = H ? (first << 16) | H : 0u;  // each part by one workgroup
        if (H && g >= first && g < first + H) mine[0] = p, mine[1] = g - first, mine[2] = H;
    });
    __syncthreads();
    const uint32_t p = mine[0], i = mine[1], H = mine[2];
    if (threadIdx.x == 0) hp.hpart[g] = p;
    if (p == ~0u) return;  // workgroup-uniform
    const uint32_t wl = p / NP, part = p % NP;
    const uint32_t S = ((uint32_t)(W - 1 - (int)wl) / (uint32_t)Wg + 1) * tiles;
    uint32_t s0, s1;
    helper_range(S, i, H, s0, s1);
    // a helper's range is a few segments: the whole workgroup walks each (teams per segment
    // would leave most lanes idle)
    for (uint32_t s = s0; s < s1; ++s) {
        const uint32_t seg = (wl + (s / tiles) * (uint32_t)Wg) * tiles + s % tiles;
        const uint32_t k = seg_cnt[seg * NP + part];
        const size_t o = (size_t)seg * DT_TILE + seg_off[seg * NP + part];
        part_walk<PACK, PS_THREADS>(ent, o, k, threadIdx.x, FB, [&](uint32_t fine, uint32_t) { lds_count(cnt, fine); });
    }
    __syncthreads();
    if (threadIdx.x < 128) hp.hh[(size_t)g * 128 + threadIdx.x] = threadIdx.x < (1u << FB) ? cnt[threadIdx.x] : 0u;
}

// helper workgroup g of k_part_sort (blockIdx >= Wg NP): place its segment range of part p
template <bool PACK>
MBLS_DEV void part_help_place(const uint32_t* __restrict__ ent, const uint32_t* __restrict__ seg_off,
                              const uint32_t* __restrict__ seg_cnt, const uint32_t* __restrict__ part_tot,
                              uint32_t tiles, int W, int Wg, int FB, uint32_t NP, uint32_t* __restrict__ sorted,
                              const PartHelp& hp, uint32_t* cnt, uint32_t* pre, uint32_t* wsum) {
    const uint32_t g = blockIdx.x - (uint32_t)Wg * NP;
    const uint32_t p = hp.hpart[g];
    if (p == ~0u) return;  // workgroup-uniform
    const uint32_t h = hp.help[p], first = h >> 16, H = h & 0xffffu, i = g - first;
    const uint32_t wl = p / NP, part = p % NP, FBN = 1u << FB;
    // part base: the entries of the parts before p (the scan order of k_part_sort)
    uint32_t a = 0;
    for (uint32_t k = threadIdx.x; k < p; k += PS_THREADS) a += part_tot[k];
    for (int d = 32; d > 0; d >>= 1) a += __shfl_xor(a, d, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = a;
    if (threadIdx.x < FBN) {  // the part's fine counts, and those of the helpers before this one
        uint32_t t = 0, before = 0;
        for (uint32_t k = 0; k < H; ++k) {
            const uint32_t v = hp.hh[(size_t)(first + k) * 128 + threadIdx.x];
            t += v;
            before += k < i ? v : 0u;
        }
        cnt[threadIdx.x] = t;
        pre[threadIdx.x] = before;
    }
    __syncthreads();
    uint32_t base = 0;
#pragma unroll
    for (uint32_t k = 0; k < PS_THREADS / 64; ++k) base += wsum[k];
    if (threadIdx.x < 64) {  // pre[f] += exclusive prefix of the fine counts
        const uint32_t l = threadIdx.x;
        const uint32_t h0 = 2 * l < FBN ? cnt[2 * l] : 0u, h1 = 2 * l + 1 < FBN ? cnt[2 * l + 1] : 0u;
        const uint32_t run = wave_incl_scan(h0 + h1) - (h0 + h1);
        if (2 * l < FBN) pre[2 * l] += run;
        if (2 * l + 1 < FBN) pre[2 * l + 1] += run + h0;
    }
    __syncthreads();
    if (threadIdx.x < FBN) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t S = ((uint32_t)(W - 1 - (int)wl) / (uint32_t)Wg + 1) * tiles;
    uint32_t s0, s1;
    helper_range(S, i, H, s0, s1);
    for (uint32_t s = s0; s < s1; ++s) {
        const uint32_t seg = (wl + (s / tiles) * (uint32_t)Wg) * tiles + s % tiles;
        const uint32_t k = seg_cnt[seg * NP + part];
        const size_t o = (size_t)seg * DT_TILE + seg_off[seg * NP + part];
        part_walk<PACK, PS_THREADS>(ent, o, k, threadIdx.x, FB, [&](uint32_t fine, uint32_t val) {
            sorted[base + pre[fine] + lds_rank<MBLS_PS_PEEL>(cnt, fine)] = val;
        });
    }
}

template <bool PACK>
__global__ __launch_bounds__(PS_THREADS) void k_part_sort(const uint32_t* __restrict__ ent, const uint32_t* __restrict__ seg_off,
                                                   const uint32_t* __restrict__ seg_cnt,
                                                   const uint32_t* __restrict__ part_tot, uint32_t tiles, int W,
                                                   int Wg, uint32_t B, int FB, uint32_t NP,
                                                   uint32_t* __restrict__ counts, uint32_t* __restrict__ offsets,
                                                   uint32_t* __restrict__ sorted, ChunkCountOut cc, PartHelp hp) {
    __shared__ uint32_t cnt[128], pre[128], span_sh, chist[ORDER_BINS];
    __shared__ uint32_t ps_stage[PS_STAGE > 0 ? PS_STAGE : 1];
    constexpr uint32_t NWV = PS_THREADS / 64, PJ = 2048 / PS_THREADS;
    __shared__ uint32_t wsum[NWV];
    const uint32_t FBN = 1u << FB;
    if (blockIdx.x >= (uint32_t)Wg * NP) {  // a heavy part's helper (grid Wg NP + PH_HELPERS)
        if (threadIdx.x < FBN) cnt[threadIdx.x] = 0;
        part_help_place<PACK>(ent, seg_off, seg_cnt, part_tot, tiles, W, Wg, FB, NP, sorted, hp, cnt, pre, wsum);
        return;
    }
    // a heavy part (k_part_heavy_count): its fine counts are its helpers', which also place it
    const uint32_t help = hp.help ? hp.help[blockIdx.x] : 0u;
    const uint32_t wl = blockIdx.x / NP, part = blockIdx.x % NP;
    // windows of group wl: wl, wl + Wg, ... < W (precompute factor F > 1), `tiles` segments each
    const uint32_t S = ((uint32_t)(W - 1 - (int)wl) / (uint32_t)Wg + 1) * tiles;
    const uint32_t team = threadIdx.x / PS_TEAM, tl = threadIdx.x % PS_TEAM, nteams = PS_THREADS / PS_TEAM;
    if (threadIdx.x < FBN) cnt[threadIdx.x] = 0;
    if (threadIdx.x < ORDER_BINS) chist[threadIdx.x] = 0;
    __syncthreads();
    // a team owning <= PS_RS segments of <= PS_RK * PS_TEAM entries each (G1 2^20: 8 of ~64) keeps
    // its lanes' packed entries in registers between the passes, so the placement pass reads no
    // global memory (MBLS_PS_KEEP=0: both passes walk `ent`); the decision is per team
    const uint32_t nseg = team < S ? (S - team + nteams - 1) / nteams : 0u;
    uint32_t sk[PS_RS], so[PS_RS], e[PS_RS * PS_RK];
    bool keep = !help && PACK && PS_KEEP && nseg <= PS_RS;
    if (keep) {
#pragma unroll
        for (uint32_t j = 0; j < PS_RS; ++j) {
            sk[j] = so[j] = 0;
            if (j < nseg) {
                const uint32_t sj = team + j * nteams;
                const uint32_t seg = (wl + (sj / tiles) * (uint32_t)Wg) * tiles + sj % tiles;
                sk[j] = seg_cnt[seg * NP + part];
                so[j] = seg * DT_TILE + seg_off[seg * NP + part];  // nseg <= PS_RS: few tiles, < 2^32
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < PS_RS; ++j) keep = keep && sk[j] <= PS_RK * PS_TEAM;
    }
    if (keep) {
#pragma unroll
        for (uint32_t j = 0; j < PS_RS; ++j)
#pragma unroll
            for (uint32_t q = 0; q < PS_RK; ++q) {
                const uint32_t i = tl + q * PS_TEAM;
                e[j * PS_RK + q] = i < sk[j] ? ent[so[j] + i] : 0u;
            }
#pragma unroll
        for (uint32_t j = 0; j < PS_RS; ++j)
#pragma unroll
            for (uint32_t q = 0; q < PS_RK; ++q)
                if (tl + q * PS_TEAM < sk[j]) atomicAdd(&cnt[FB ? e[j * PS_RK + q] >> (32 - FB) : 0u], 1u);
    } else if (help) {
        if (threadIdx.x < FBN) {
            const uint32_t first = help >> 16, H = help & 0xffffu;
            uint32_t t = 0;
            for (uint32_t k = 0; k < H; ++k) t += hp.hh[(size_t)(first + k) * 128 + threadIdx.x];
            cnt[threadIdx.x] = t;
        }
    } else {
        for (uint32_t s = team; s < S; s += nteams) {
            const uint32_t seg = (wl + (s / tiles) * (uint32_t)Wg) * tiles + s % tiles;
            const uint32_t k = seg_cnt[seg * NP + part];
            const size_t o = (size_t)seg * DT_TILE + seg_off[seg * NP + part];
            part_walk<PACK>(ent, o, k, tl, FB, [&](uint32_t fine, uint32_t) { lds_count(cnt, fine); });
        }
    }
    // this part's base: the sum of the part totals before it (blockIdx = wl * NP + part, the
    // scan order); block 0 sums them all for offsets[Wg B].  <= Wg * NP = 2048 words: cheaper
    // than the three launches of a separate scan
    {
        const uint32_t lim = blockIdx.x == 0 ? (uint32_t)Wg * NP : blockIdx.x;
        uint32_t a = 0;
        if (lim <= PJ * PS_THREADS) {  // independent loads (the strided loop waited one latency per step)
#pragma unroll
            for (uint32_t j = 0; j < PJ; ++j) {
                const uint32_t k = threadIdx.x + PS_THREADS * j;
                a += k < lim ? part_tot[k] : 0u;
            }
        } else {
            for (uint32_t k = threadIdx.x; k < lim; k += blockDim.x) a += part_tot[k];
        }
        for (int d = 32; d > 0; d >>= 1) a += __shfl_xor(a, d, 64);
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = a;
    }
    __syncthreads();
    uint32_t psum = 0;
#pragma unroll
    for (uint32_t k = 0; k < NWV; ++k) psum += wsum[k];
    const uint32_t base = blockIdx.x == 0 ? 0u : psum;
    if (threadIdx.x < 64) {  // wave 0: exclusive scan of the FBN <= 128 fine counts, 2 per lane
        const uint32_t l = threadIdx.x;
        const uint32_t h0 = 2 * l < FBN ? cnt[2 * l] : 0u, h1 = 2 * l + 1 < FBN ? cnt[2 * l + 1] : 0u;
        const uint32_t incl = wave_incl_scan(h0 + h1), run = incl - (h0 + h1);
        if (l == 63) span_sh = incl;  // this part's entry count
        const size_t key = (size_t)wl * B + part * FBN + 2 * l;
        if (cc.nchunks) {
            // fused k_chunk_counts (FBN == 128: the part is one 128-bucket block of the chunk-count
            // scan): chunk counts of the L-aligned chunks, their prefix inside the block (over
            // `counts`), the block total, the order histogram and the running maximum
            const uint32_t o0 = base + run, o1 = o0 + h0;
            const uint32_t c0 = h0 ? (o0 + h0 - 1) / cc.L - o0 / cc.L + 1 : 0u;
            const uint32_t c1 = h1 ? (o1 + h1 - 1) / cc.L - o1 / cc.L + 1 : 0u;
            pre[2 * l] = run;
            pre[2 * l + 1] = run + h0;
            offsets[key] = o0;
            offsets[key + 1] = o1;
            cc.nchunks[key] = c0;
            cc.nchunks[key + 1] = c1;
            const uint32_t cin = wave_incl_scan(c0 + c1);
            counts[key] = cin - (c0 + c1);
            counts[key + 1] = cin - c1;
            if (l == 63) cc.blk_tot[key >> CHUNK_FUSED_SHIFT] = cin;
            if (c0 <= SMALL_MAX) atomicAdd(&chist[c0], 1u);
            if (c1 <= SMALL_MAX) atomicAdd(&chist[c1], 1u);
            uint32_t cm = max(c0, c1);
            for (int d = 32; d > 0; d >>= 1) cm = max(cm, (uint32_t)__shfl_xor(cm, d, 64));
            if (l == 0 && cm > 1 && cm > __atomic_load_n(&cc.nchunks[cc.m], __ATOMIC_RELAXED))
                atomicMax(&cc.nchunks[cc.m], cm);
        } else {
            if (2 * l < FBN) {
                pre[2 * l] = run;
                counts[key] = h0;
                offsets[key] = base + run;
            }
            if (2 * l + 1 < FBN) {
                pre[2 * l + 1] = run + h0;
                counts[key + 1] = h1;
                offsets[key + 1] = base + run + h0;
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 64) offsets[(size_t)Wg * B] = psum;
    __syncthreads();
    if (threadIdx.x < FBN) cnt[threadIdx.x] = 0;
    if (cc.nchunks && threadIdx.x < ORDER_BINS && chist[threadIdx.x]) {
        const uint32_t blk = (uint32_t)(((size_t)wl * B + part * FBN) >> 8), bpg = (cc.m + 255) / 256;
        atomicAdd(&cc.binhist[order_index(blk, threadIdx.x, bpg)], chist[threadIdx.x]);
    }
    if (help) return;  // workgroup-uniform: the helpers place the entries
    __syncthreads();
    // the part's span of `sorted` is assembled in LDS and written out in order (whole lines),
    // instead of one random 4-byte store per entry; a span larger than the stage (adversarial
    // bucket skew) takes the direct stores
    const uint32_t span = span_sh;
    const bool staged = span <= PS_STAGE;
    // register-kept parts are light (<= PS_RK * PS_TEAM entries per segment): plain atomics
    auto put = [&](uint32_t pos, uint32_t val) {
        if (staged)
            ps_stage[pos] = val;
        else
            sorted[base + pos] = val;
    };
    auto place = [&](uint32_t fine, uint32_t val) { put(pre[fine] + lds_rank<MBLS_PS_PEEL>(cnt, fine), val); };
    auto place_light = [&](uint32_t fine, uint32_t val) { put(pre[fine] + atomicAdd(&cnt[fine], 1u), val); };
    if (keep) {
        const uint32_t vmask = FB ? (1u << (32 - FB)) - 1 : ~0u;
#pragma unroll
        for (uint32_t j = 0; j < PS_RS; ++j)
#pragma unroll
            for (uint32_t q = 0; q < PS_RK; ++q)
                if (tl + q * PS_TEAM < sk[j]) {
                    const uint32_t x = e[j * PS_RK + q];
                    place_light(FB ? x >> (32 - FB) : 0u, x & vmask);
                }
    } else {
        for (uint32_t s = team; s < S; s += nteams) {
            const uint32_t seg = (wl + (s / tiles) * (uint32_t)Wg) * tiles + s % tiles;
            const uint32_t k = seg_cnt[seg * NP + part];
            const size_t o = (size_t)seg * DT_TILE + seg_off[seg * NP + part];
            part_walk<PACK>(ent, o, k, tl, FB, place);
        }
    }
    if (staged) {  // workgroup-uniform
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < span; i += blockDim.x) sorted[base + i] = ps_stage[i];
    }
}

eIcicleError launch_digits_part(const uint8_t* scalars, bool mont, uint32_t n, const MsmPlan& P, uint32_t* ent,
                                uint32_t* seg_off, uint32_t* seg_cnt, uint32_t* part_tot, uint8_t* dsrc,
                                uint32_t* zero_word, hipStream_t st, const uint8_t* bases, uint8_t* phi,
                                uint32_t* zero2, uint32_t nzero2) {
    if (P.B > DT_MAX_B) return MBLS_INVALID_ARGUMENT;
    const PartSortSizes z = part_sort_sizes(P);
    const uint32_t* src;
    uint32_t nidx;
    ZeroList zl;
    zl.p[0] = part_tot;  // k_digits_part's per-part totals (atomics)
    zl.n[0] = (uint32_t)P.Wg * z.NP;
    zl.p[1] = zero_word;  // the chunk-count maximum (k_chunk_counts' atomicMax), HeavyTab counters
    zl.n[1] = zero_word ? 3u : 0u;
    zl.p[2] = zero2;  // the fused chunk-count order histograms (k_part_sort atomics)
    zl.n[2] = zero2 ? nzero2 : 0u;
    eIcicleError er = digit_sources(scalars, mont, n, P, dsrc, zl, st, src, nidx, bases, phi);
    if (er != MBLS_SUCCESS) return er;
    dim3 g(z.segments), b(DT_THREADS);
    const uint32_t F = (uint32_t)P.F;
    const DigitOffset C = digit_offset(P.c, P.W, P.B, P.Wg, P.sF);
#define MBLS_DP(S_, P_)                                                                                           \
    hipLaunchKernelGGL((k_digits_part<S_, P_>), g, b, 0, st, src, nidx, P.c, P.Wg, P.sF, F, P.B, z.FB, z.NP, ent, seg_off, \
                       seg_cnt, part_tot, C)
    if (P.split > 1) {
        if (z.pack)
            MBLS_DP(true, true);
        else
            MBLS_DP(true, false);
    } else if (z.pack)
        MBLS_DP(false, true);
    else
        MBLS_DP(false, false);
#undef MBLS_DP
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

bool part_sort_fuses_chunks(const MsmPlan& P) { return part_fine_bits(P.B) == CHUNK_FUSED_SHIFT; }

eIcicleError launch_part_sort(const MsmPlan& P, const uint32_t* ent, const uint32_t* seg_off, const uint32_t* seg_cnt,
                              const uint32_t* part_tot, uint32_t* counts, uint32_t* offsets, uint32_t* sorted,
                              const ChunkCountOut& cc, hipStream_t st, const PartHelp& hp_in) {
    const PartSortSizes z = part_sort_sizes(P);
    if (cc.nchunks && z.FB != CHUNK_FUSED_SHIFT) return MBLS_INVALID_ARGUMENT;
    if (z.FB > 7) return MBLS_INVALID_ARGUMENT;  // 128 fine counters per part (cnt, pre, hh rows)
    const bool help = MBLS_PS_HELP && hp_in.help && hp_in.hh && hp_in.hpart;
    const PartHelp hp = help ? hp_in : PartHelp();
    const uint32_t M = (uint32_t)P.Wg * z.NP;
    dim3 g(M + (help ? PH_HELPERS : 0u)), b(PS_THREADS);
    if (help) {
        if (z.pack)
            hipLaunchKernelGGL(k_part_heavy_count<true>, dim3(PH_HELPERS), b, 0, st, ent, seg_off, seg_cnt, part_tot,
                               z.tiles, P.W, P.Wg, z.FB, z.NP, hp);
        else
            hipLaunchKernelGGL(k_part_heavy_count<false>, dim3(PH_HELPERS), b, 0, st, ent, seg_off, seg_cnt, part_tot,
                               z.tiles, P.W, P.Wg, z.FB, z.NP, hp);
        MBLS_TRY(hipGetLastError());
    }
    if (z.pack)
        hipLaunchKernelGGL(k_part_sort<true>, g, b, 0, st, ent, seg_off, seg_cnt, part_tot, z.tiles, P.W, P.Wg, P.B,
                           z.FB, z.NP, counts, offsets, sorted, cc, hp);
    else
        hipLaunchKernelGGL(k_part_sort<false>, g, b, 0, st, ent, seg_off, seg_cnt, part_tot, z.tiles, P.W, P.Wg, P.B,
                           z.FB, z.NP, counts, offsets, sorted, cc, hp);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// Chunks are L-ALIGNED in the sorted array (chunk t = positions [L t, L t + L)), so every
// accumulation thread does exactly L additions; a chunk crossing bucket boundaries yields one
// partial ("segment") per bucket it touches.  Segments of bucket b: the aligned chunks that
// overlap [off_b, off_b + cnt_b).  nchunks[m] receives the maximum (heavy-bucket passes).

// also the first half of the chunk_off scan: cloc[b] = exclusive prefix of the chunk counts
// inside b's block of 256 buckets, blk_tot[block] = the block's total (k_scan_small scans the
// totals, k_chunk_owner adds the prefixes: no separate 3-kernel scan).  cloc may alias counts
// (each thread reads its count before writing its prefix).
__global__ __launch_bounds__(256) void k_chunk_counts(const uint32_t* counts, const uint32_t* __restrict__ offsets,
                                                      uint32_t* __restrict__ nchunks, uint32_t m, uint32_t L,
                                                      uint32_t* __restrict__ binhist, uint32_t bpg, uint32_t* cloc,
                                                      uint32_t* __restrict__ blk_tot) {
    __shared__ uint32_t hist[ORDER_BINS];
    __shared__ uint32_t wsum[4];
    if (threadIdx.x < ORDER_BINS) hist[threadIdx.x] = 0;
    __syncthreads();
    uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t c = 0;
    if (b < m) {
        const uint32_t cnt = counts[b], o = offsets[b];
        c = cnt ? (o + cnt - 1) / L - o / L + 1 : 0u;
        nchunks[b] = c;
        if (c <= SMALL_MAX) atomicAdd(&hist[c], 1u);
    }
    {
        const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        uint32_t incl = c;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t t = __shfl_up(incl, d, 64);
            if (lane >= (uint32_t)d) incl += t;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t base = 0;
        for (uint32_t k = 0; k < w; ++k) base += wsum[k];
        if (b < m) cloc[b] = base + incl - c;
        if (threadIdx.x == 0) blk_tot[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    }
    // block max, then at most one atomic per block and only when it raises the running max
    // (4096 same-address atomics cost 46 us at 2^20; the filtered read is monotone-safe)
    for (int d = 32; d > 0; d >>= 1) c = max(c, (uint32_t)__shfl_xor(c, d, 64));
    __shared__ uint32_t wmax[4];
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        c = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        if (c > 1 && c > __atomic_load_n(&nchunks[m], __ATOMIC_RELAXED)) atomicMax(&nchunks[m], c);
    }
    // per-block histogram of the light buckets' chunk counts (k_bucket_order)
    if (threadIdx.x < ORDER_BINS) binhist[order_index(blockIdx.x, threadIdx.x, bpg)] = hist[threadIdx.x];
}

// perm (k_chunk_owner) = the light buckets (<= SMALL_MAX chunks) grouped by window group, then
// by chunk count (heaviest first), so the waves of k_bucket_small run uniform trip counts (bucket
// order alone gave ~4 +- 1.5 chunks per lane and a wave ran its maximum).  binbase = exclusive
// scan of k_chunk_counts' histograms (order_index layout).

eIcicleError launch_chunk_counts(const uint32_t* counts, const uint32_t* offsets, uint32_t* nchunks, uint32_t m,
                                 uint32_t L, uint32_t* binhist, uint32_t groups, bool zeroed, uint32_t* cloc,
                                 uint32_t* blk_tot, hipStream_t st) {
    if (!zeroed) MBLS_TRY(hipMemsetAsync(nchunks + m, 0, 12, st));  // maximum + HeavyTab counters
    const uint32_t nblk = (m + 255) / 256;
    hipLaunchKernelGGL(k_chunk_counts, dim3(nblk), dim3(256), 0, st, counts, offsets, nchunks, m, L, binhist,
                       nblk / groups, cloc, blk_tot);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

uint32_t order_words(uint32_t m) { return ORDER_BINS * ((m + 255) / 256); }

// exclusive scan of a short array in ONE workgroup of 1024 threads; out[m] = total
MBLS_DEV void scan_wg(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint32_t m, uint32_t* wtot) {
    const uint32_t per = (m + 1023) / 1024;
    const uint32_t b0 = min(threadIdx.x * per, m), b1 = min(b0 + per, m);
    // up to SCAN_REG words per thread are loaded into registers by independent loads (a runtime
    // bounded loop issued them one latency at a time: 17 words per thread at G1 2^20, ~20 us)
    constexpr uint32_t SCAN_REG = 24;
    uint32_t v[SCAN_REG];
    uint32_t a = 0;
    if (per <= SCAN_REG) {
#pragma unroll
        for (uint32_t j = 0; j < SCAN_REG; ++j) {
            v[j] = b0 + j < b1 ? in[b0 + j] : 0u;
            a += v[j];
        }
    } else {
        for (uint32_t k = b0; k < b1; ++k) a += in[k];
    }
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t incl = a;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += t;
    }
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    uint32_t wbase = 0;
    for (uint32_t k = 0; k < w; ++k) wbase += wtot[k];
    uint32_t run = wbase + incl - a;
    if (per <= SCAN_REG) {
#pragma unroll
        for (uint32_t j = 0; j < SCAN_REG; ++j) {
            if (b0 + j < b1) out[b0 + j] = run;
            run += v[j];
        }
    } else {
        for (uint32_t k = b0; k < b1; ++k) {
            const uint32_t x = in[k];
            out[k] = run;
            run += x;
        }
    }
    if (threadIdx.x == 1023) out[m] = run;
    __syncthreads();  // wtot is reused by the next scan
}

// the order histograms (~17 K words) and the chunk-count block totals (k_chunk_counts), one
// workgroup for both
__global__ __launch_bounds__(1024) void k_scan_small(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                     uint32_t m, const uint32_t* __restrict__ in2,
                                                     uint32_t* __restrict__ out2, uint32_t m2) {
    __shared__ uint32_t wtot[16];
    scan_wg(in, out, m, wtot);
    scan_wg(in2, out2, m2, wtot);
}

eIcicleError launch_order_scan(const uint32_t* binhist, uint32_t* binbase, uint32_t m, const uint32_t* blk_tot,
                               uint32_t* blk_pre, uint32_t nblk, hipStream_t st) {
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(1024), 0, st, binhist, binbase, order_words(m), blk_tot, blk_pre,
                       nblk);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// ------------------------------------------------------------------------------------
// 3. scatter (counting sort)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_scatter(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                 const uint32_t* __restrict__ ranks, size_t total,
                                                 const uint32_t* __restrict__ offsets, uint32_t* __restrict__ sorted) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= total) return;
    const uint32_t k = keys[i];
    if (k == INVALID_KEY) return;
    sorted[offsets[k] + ranks[i]] = vals[i];
}

eIcicleError launch_scatter(const uint32_t* keys, const uint32_t* vals, const uint32_t* ranks, size_t total,
                            const uint32_t* offsets, uint32_t* sorted, hipStream_t st) {
    hipLaunchKernelGGL(k_scatter, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, keys, vals, ranks, total,
                       offsets, sorted);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// chunk_off[b] = cloc[b] + blk_pre[b >> cs] (the scan begun in k_chunk_counts or k_part_sort; chunk_off[m] =
// the total); owner[segment] = bucket; first[t] = the bucket holding position L t (the start of
// chunk t); and the bucket order of k_bucket_order (same grid: one thread per bucket)
__global__ __launch_bounds__(256) void k_chunk_owner(const uint32_t* __restrict__ cloc, const uint32_t* __restrict__ blk_pre,
                                                     int cs, uint32_t* __restrict__ chunk_off, const uint32_t* __restrict__ offsets,
                                                     uint32_t m, uint32_t L, uint32_t* __restrict__ owner,
                                                     uint32_t* __restrict__ first, const uint32_t* __restrict__ nchunks,
                                                     const uint32_t* __restrict__ binbase, uint32_t* __restrict__ perm,
                                                     HeavyTab H) {
    __shared__ uint32_t cur[ORDER_BINS];
    // long owner / first ranges (heavy buckets: skewed scalars put up to 2^16 chunks in one
    // bucket, whose lone thread took 2.75 ms to write them at G1 2^20) are queued and written by
    // the whole workgroup
    __shared__ uint32_t qn, qk0[256], qk1[256], qt0[256], qt1[256], qb[256];
    if (threadIdx.x < ORDER_BINS) cur[threadIdx.x] = binbase[order_index(blockIdx.x, threadIdx.x, gridDim.x)];
    if (threadIdx.x == 0) qn = 0;
    __syncthreads();
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < m) {
        const uint32_t k0 = cloc[b] + blk_pre[b >> cs];
        const uint32_t k1 = b + 1 < m ? cloc[b + 1] + blk_pre[(b + 1) >> cs] : blk_pre[(m + (1u << cs) - 1) >> cs];
        chunk_off[b] = k0;
        if (b + 1 == m) chunk_off[m] = k1;
        const uint32_t o = offsets[b], e = offsets[b + 1];
        const uint32_t t0 = (o + L - 1) / L, t1 = (e + L - 1) / L;
        if (k1 - k0 > 32 || t1 > t0 + 32) {
            const uint32_t q = atomicAdd(&qn, 1u);
            qk0[q] = k0, qk1[q] = k1, qt0[q] = t0, qt1[q] = t1, qb[q] = b;
        } else {
            for (uint32_t k = k0; k < k1; ++k) owner[k] = b;
            for (uint32_t t = t0; t < t1; ++t) first[t] = b;
        }
    }
    __syncthreads();
    for (uint32_t q = 0; q < qn; ++q) {
        const uint32_t qv = qb[q];
        for (uint32_t k = qk0[q] + threadIdx.x; k < qk1[q]; k += blockDim.x) owner[k] = qv;
        for (uint32_t t = qt0[q] + threadIdx.x; t < qt1[q]; t += blockDim.x) first[t] = qv;
    }
    if (blockIdx.x == 0)  // the planned slices' group counters (heavy_slices)
        for (uint32_t i = threadIdx.x; i < HEAVY_GDONE; i += blockDim.x) H.gdone[i] = 0;
    if (b >= m) return;
    const uint32_t c = nchunks[b];
    if (c <= SMALL_MAX) {
        perm[atomicAdd(&cur[c], 1u)] = b;
    } else {  // heavy bucket (adversarial inputs only): list it with its slices for k_bucket_small
        const uint32_t ns = (c + HEAVY_SLICE - 1) / HEAVY_SLICE;
        const uint32_t ent = atomicAdd(&H.cnt[0], 1u);
        const uint32_t f0 = atomicAdd(&H.cnt[1], ns);
        H.bucket[ent] = b;
        H.first[ent] = f0;
        H.nslices[ent] = ns;
        H.done[ent] = 0;
        for (uint32_t k = 0; k < ns; ++k) H.owner[f0 + k] = ent;
    }
}

eIcicleError launch_chunk_owner(const uint32_t* cloc, const uint32_t* blk_pre, int cs, uint32_t* chunk_off,
                                const uint32_t* offsets, uint32_t m, uint32_t L, uint32_t* owner, uint32_t* first,
                                const uint32_t* nchunks, const uint32_t* binbase, uint32_t* perm, HeavyTab H,
                                hipStream_t st) {
    const uint32_t nblk = (m + 255) / 256;
    hipLaunchKernelGGL(k_chunk_owner, dim3(nblk), dim3(256), 0, st, cloc, blk_pre, cs, chunk_off, offsets, m, L, owner,
                       first, nchunks, binbase, perm, H);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// ------------------------------------------------------------------------------------
// scalars
// ------------------------------------------------------------------------------------
__global__ void k_scalars_from_mont(uint8_t* s, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    store<FrCfg>(s + 32 * i, from_mont(load<FrCfg>(s + 32 * i)));
}

eIcicleError launch_scalars_from_mont(uint8_t* s, size_t n, hipStream_t st) {
    hipLaunchKernelGGL(k_scalars_from_mont, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, s, n);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

__global__ void k_gen_scalars(uint8_t* out, uint64_t seed, size_t start, size_t n, int mont) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr s = gen_scalar(seed, start + i);
    if (mont) s = to_mont(s);
    store<FrCfg>(out + 32 * i, s);
}

}  // namespace mbls

using namespace mbls;

extern "C" eIcicleError mbls_gen_scalars_range(mbls_fr_t* out_device, uint64_t seed, size_t start, size_t n,
                                               bool montgomery, void* stream) {
    if (!out_device) return MBLS_INVALID_POINTER;
    if (n == 0) return MBLS_SUCCESS;
    hipLaunchKernelGGL(k_gen_scalars, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (uint8_t*)out_device, seed, start, n, montgomery ? 1 : 0);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}
extern "C" eIcicleError mbls_gen_scalars(mbls_fr_t* out_device, uint64_t seed, size_t n, bool montgomery, void* stream) {
    return mbls_gen_scalars_range(out_device, seed, 0, n, montgomery, stream);
}

namespace mbls {

// per-device resources of mbls_g*_msm_multi_device (msm_core.hpp msm_multi_device): one
// non-blocking stream, one event per shard, the shards' partial slots and the first device's
// gather slots; created on first use, kept for the process (like the scratch pool)
std::mutex& multi_device_mutex() {
    static std::mutex* m = new std::mutex();
    return *m;
}

MultiDevRes*& multi_device_last() {
    static MultiDevRes* last = nullptr;
    return last;
}

// Peer access between the first device and a shard's device, enabled once per ordered pair
// (under the multi-device lock): the shard's scalar staging copy reads the first device's
// memory and the exchange copies the shard's partial back.  Without it hipMemcpyPeerAsync /
// hipMemcpyDefault between devices may be staged through host memory.  Pairs the hardware
// cannot map are left to the runtime's staged copy (still correct).
eIcicleError enable_peer(int from, int to) {
    static std::set<std::pair<int, int>>* done = new std::set<std::pair<int, int>>();
    if (from == to || done->count({from, to})) return MBLS_SUCCESS;
    int can = 0;
    MBLS_TRY(hipDeviceCanAccessPeer(&can, from, to));
    if (can) {
        int cur = 0;
        MBLS_TRY(hipGetDevice(&cur));
        MBLS_TRY(hipSetDevice(from));
        hipError_t e = hipDeviceEnablePeerAccess(to, 0);
        (void)hipSetDevice(cur);
        if (e == hipErrorPeerAccessAlreadyEnabled) {
            (void)hipGetLastError();
        } else if (e != hipSuccess) {
            return map_hip_error(e, "hipDeviceEnablePeerAccess");
        }
    }
    done->insert({from, to});
    return MBLS_SUCCESS;
}

eIcicleError multi_device_res(int dev, MultiDevRes*& out) {
    static std::map<int, MultiDevRes>* tab = new std::map<int, MultiDevRes>();
    auto it = tab->find(dev);
    if (it != tab->end()) {
        out = &it->second;
        return MBLS_SUCCESS;
    }
    int cur = 0;
    MBLS_TRY(hipGetDevice(&cur));
    MBLS_TRY(hipSetDevice(dev));
    MultiDevRes r;
    constexpr size_t JAC = GroupTraits<Fq2>::JAC;  // the larger point
    hipError_t e = hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking);
    for (int k = 0; k < MAX_SHARDS && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&r.ev[k], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&r.done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipMalloc(&r.partials, MAX_SHARDS * JAC);
    if (e == hipSuccess) e = hipMalloc(&r.gather, (MAX_SHARDS + 1) * JAC);
    (void)hipSetDevice(cur);
    if (e != hipSuccess) return map_hip_error(e, "multi-device resources");
    out = &(*tab)[dev];
    *out = r;
    return MBLS_SUCCESS;
}

}  // namespace mbls
