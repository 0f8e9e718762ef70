// msm_core.hpp -- Pippenger multi-scalar multiplication over G1 / G2 for CDNA4 (templates).
//
// Reference: orchestration msm::msm_cuda (bls12-381/src/curve/msm_kernels.cu:603-903),
// digits compute_bucket_indices_kernel (:69-143), histogram (:224-256), cub scan+sort
// (:748-781), accumulation (:269-366), bucket reduction (:376-513), final (:529-596);
// boundary msm_cuda_impl / msm_g2_cuda_impl (icicle_curve_api.cu:243-618).
//
// Pipeline (all on the caller's stream, scratch from the per-stream arena):
//   1. k_digits       (msm_common.hip) one thread per scalar: Montgomery -> standard if
//                     flagged, signed c-bit digits, (key, index|sign) pairs window-major,
//                     bucket histogram by atomics.
//   2. scans          bucket offsets; buckets are split in chunks of <= CHUNK points so one
//                     heavy bucket (e.g. all-equal scalars) cannot serialise a thread.
//   3. k_scatter      counting-sort scatter (keys < TB: no radix sort needed).
//      c <= 16 (default): steps 1-3 are the partitioned counting sort instead
//                     (k_digits_part + k_part_sort, msm_common.hip 2b).
//   4. k_accumulate   one thread per chunk: sum of +-P_i by mixed additions -> partial.
//   5. k_bucket_sum   one thread per bucket: sum of its chunk partials.
//   6. bucket reduction sum_d d*B_d per window as a recursive running sum (k_reduce_scaled):
//                     level l splits its inputs in segments of 2^s; each segment's chain walks
//                     R += V_t, S += R, S += U_t and outputs U' = S and V' = 2^s R, so every level's
//                     outputs carry weight 1 and the last level's output IS the window sum (no
//                     scalar multiplications, no per-level tree sums, no window Horner).
//   7. k_final*       fold over windows: sum_w 2^(c w) G_w (+ ICICLE normalisation).
// Precompute factor F (bases table = F blocks of n bases, block f = 2^(c*Wg*f) * P) folds
// the W windows into Wg = ceil(W/F) groups so the final fold shrinks to (Wg-1)*c doublings.
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <vector>

#include "mbls_common.hpp"
#include "mbls_curve.hpp"
#include "mbls_fq28.hpp"
#include "mbls_fq2_28.hpp"
#include "mbls_rowfield.hpp"
#include "mbls_wavepoint.hpp"

namespace mbls {

static constexpr uint32_t INVALID_KEY = 0xffffffffu;

// Wave priority of the latency-bound tail kernels (bucket sums, reduction, folds).  With window
// groups they run beside the next group's VALU-saturating accumulation, and the VALU issue
// arbiter picks by priority, then age (MI355X_MICROARCH.md): raised, their chains keep issuing.
#ifndef MBLS_SETPRIO
#define MBLS_SETPRIO 3
#endif
#define MBLS_TAIL_PRIO() __builtin_amdgcn_s_setprio(MBLS_SETPRIO)
#ifndef MBLS_LIGHT_PRIO
#define MBLS_LIGHT_PRIO 2
#endif
#ifndef MBLS_CHUNK
#define MBLS_CHUNK 16
#endif
static constexpr int CHUNK = MBLS_CHUNK;  // max points per accumulation thread
static constexpr int SEG_LOG = 3;   // row segment length 8, levels >= 1 (reduction 0.96 -> 0.92 ms against 16 at G1 2^20)
static constexpr int SEG0_LOG = 2;  // level 0 (one segment per lane): short chains, many lanes
static constexpr int MAX_MSM_LOG = 26;
static constexpr int SCAN_BLOCK = 1024;
static constexpr int MAX_LEVELS = 16;

static constexpr int MAX_PRECOMPUTE = 64;
static constexpr int SMALL_MAX = 16;  // buckets of <= SMALL_MAX chunks: one thread (k_bucket_small)
static constexpr int ORDER_BINS = SMALL_MAX + 1;  // k_bucket_order bins: chunk counts 0..SMALL_MAX

// words a kernel clears in passing (grid-stride), instead of a hipMemsetAsync fill launch
struct ZeroList {
    uint32_t* p[3] = {nullptr, nullptr, nullptr};
    uint32_t n[3] = {0, 0, 0};
    MBLS_DEV void run(uint32_t gid, uint32_t stride) const {
        for (int k = 0; k < 3; ++k)
            for (uint32_t i = gid; i < n[k]; i += stride) p[k][i] = 0;
    }
};

// digit-source index of stream j of point i: j * sj + i * si (blocked: sj = n, si = 1; prepared
// point-major table: sj = 1, si = split)
struct SplitLayout {
    uint32_t sj, si;
    MBLS_DEV uint32_t at(uint32_t j, uint32_t i) const { return j * sj + i * si; }
};

struct MsmPlan {
    int c, W, Wg, F;
    int sF;                     // precomputed-table block shift in bits (0: F == 1), see window_span
    int split;                  // endomorphism split: 1 none, 2 G1 GLV (phi), 4 G2 psi
    bool prepared;              // the bases buffer is the point-major image table (no per-call table)
    int table;                  // bases-buffer entries per point (F, or split when prepared)
    int bstride;                // > 1: GLV plan on slot 0 of an F-entry shift table (make_plan)
    bool fq2;                   // G2 (Fq2 coordinates)
    uint32_t B, TB;
    uint32_t chunk;             // contributions per accumulation thread (accumulate_chunk)
    size_t pts;                 // distinct point indices (n, n*F, or split*n)
    size_t contributions;
    int levels;                 // bucket-reduction levels
    uint32_t level_m[MAX_LEVELS];  // inputs per window at each level
    uint8_t seg_log[MAX_LEVELS];   // log2 segment length per level
    uint8_t mode[MAX_LEVELS];      // MODE_LANE / MODE_ROW / MODE_WAVE per level
    uint32_t seg(int l) const { return 1u << seg_log[l]; }
};

// endo: the split the group offers (1 none, 2 G1 GLV, 4 G2 psi); make_plan decides whether to use it
eIcicleError make_plan(long long n, const MSMConfig* cfg, MsmPlan& p, int endo = 1);
eIcicleError plan_levels(MsmPlan& p, int Wl);
// bits between consecutive multiples in a precomputed table: [P, 2^s P, 2^(2s) P, ...], s = ceil(256 / F)
int precompute_shift(int F);

// ---- non-templated launchers (msm_common.hip) ----------------------------------------
eIcicleError launch_digits(const uint8_t* scalars, bool mont, uint32_t n, const MsmPlan& P, uint32_t* keys,
                           uint32_t* vals, uint32_t* ranks, uint32_t* counts, uint8_t* dsrc, hipStream_t st);
size_t digits_src_bytes(uint32_t n, int split);
eIcicleError scan_exclusive(const uint32_t* in, uint32_t* out, uint32_t m, uint32_t* tmp, hipStream_t st);
eIcicleError launch_chunk_counts(const uint32_t* counts, const uint32_t* offsets, uint32_t* nchunks, uint32_t m,
                                 uint32_t L, uint32_t* binhist, uint32_t groups, bool zeroed, uint32_t* cloc,
                                 uint32_t* blk_tot, hipStream_t st);
// blk_tot: the chunk-count block totals (nblk of them), scanned into blk_pre
eIcicleError launch_order_scan(const uint32_t* binhist, uint32_t* binbase, uint32_t m, const uint32_t* blk_tot,
                               uint32_t* blk_pre, uint32_t nblk, hipStream_t st);
uint32_t order_words(uint32_t m);
eIcicleError launch_scatter(const uint32_t* keys, const uint32_t* vals, const uint32_t* ranks, size_t total,
                            const uint32_t* offsets, uint32_t* sorted, hipStream_t st);
// heavy buckets (> SMALL_MAX chunk partials), listed by k_chunk_owner for k_bucket_small's slice
// workgroups.  cnt[0] = heavy buckets, cnt[1] = slices: words TB + 1, TB + 2 of the chunk-count
// array, zeroed by the digit pass with the chunk-count maximum at TB.
struct HeavyTab {
    uint32_t* cnt;
    uint32_t* bucket;   // entry e -> its bucket
    uint32_t* first;    // entry e -> its first slice
    uint32_t* nslices;  // entry e -> its slice count
    uint32_t* done;     // entry e -> slices finished (last-block-done counter)
    uint32_t* owner;    // slice g -> its entry
    uint8_t* res;       // slice g -> its sum (Jacobian)
    uint32_t* gdone;    // planned slices: group of HEAVY_GROUP slices led by g -> slices finished
};
static constexpr uint32_t HEAVY_GDONE = 2048;  // gdone words (zeroed by k_chunk_owner)
// cloc / blk_pre: the chunk-count prefixes inside blocks of 2^cs buckets and the blocks' scan
eIcicleError launch_chunk_owner(const uint32_t* cloc, const uint32_t* blk_pre, int cs, uint32_t* chunk_off,
                                const uint32_t* offsets, uint32_t m, uint32_t L, uint32_t* owner, uint32_t* first,
                                const uint32_t* nchunks, const uint32_t* binbase, uint32_t* perm, HeavyTab H,
                                hipStream_t st);
eIcicleError launch_scalars_from_mont(uint8_t* s, size_t n, hipStream_t st);
eIcicleError launch_glv_table(const uint8_t* bases, uint8_t* phi, uint32_t n, hipStream_t st);
// host (pinned: a PCIe-reading copy kernel; pageable: hipMemcpyAsync) or peer memory -> device
eIcicleError stage_to_device(void* dst, const void* src, size_t bytes, hipStream_t st);
eIcicleError launch_psi_table(const uint8_t* bases, uint8_t* phi, uint32_t n, hipStream_t st);
// point-major endomorphism image table (prepared bases): out[S i + j] = endo^j(P_i), S = 2 (G1) / 4 (G2)
eIcicleError launch_endo_table(const uint8_t* in, uint8_t* out, uint32_t n, int split, hipStream_t st);
size_t scan_tmp_words(uint32_t m);

// partitioned counting sort (msm_common.hip 2b): pass A digits -> per-segment coarse parts,
// pass B per-part LDS counting sort.  Replaces keys / vals / ranks + k_scatter for c <= 16.
struct PartSortSizes {
    uint32_t NP = 0, tiles = 0, segments = 0;
    int FB = 0;
    bool pack = false;
    size_t ent = 0, segtab = 0, parts = 0;  // bytes
};
bool partition_sort(const MsmPlan& P);
PartSortSizes part_sort_sizes(const MsmPlan& P);
// bases / phi: the endomorphism table is written by the split kernel itself (k_glv_prep, k_psi_prep)
// chunk counts computed by the partition sort itself (k_part_sort, parts of 128 fine buckets):
// k_chunk_counts' outputs with the prefixes in blocks of 128 buckets (CHUNK_FUSED_SHIFT)
struct ChunkCountOut {
    uint32_t* nchunks = nullptr;  // null: not fused (k_part_sort writes the bucket counts)
    uint32_t* binhist = nullptr;  // order histograms (accumulated: zeroed by the digit pass)
    uint32_t* blk_tot = nullptr;  // per 128-bucket block: the chunk-count total
    uint32_t L = 0, m = 0;        // chunk length, bucket count
};
static constexpr int CHUNK_FUSED_SHIFT = 7;
bool part_sort_fuses_chunks(const MsmPlan& P);
// helpers of heavy parts (skewed scalars; msm_common.hip k_part_heavy_count): help[M] per part
// (first helper << 16 | helpers, 0: light), hh[PH_HELPERS][128] the helpers' fine counts,
// hpart[PH_HELPERS] each helper's part (~0: idle)
static constexpr uint32_t PH_HELPERS = 512;
struct PartHelp {
    uint32_t* help = nullptr;
    uint32_t* hh = nullptr;
    uint32_t* hpart = nullptr;
};
// zero2 / nzero2: words the digit pass clears besides its own (the fused order histograms)
eIcicleError launch_digits_part(const uint8_t* scalars, bool mont, uint32_t n, const MsmPlan& P, uint32_t* ent,
                                uint32_t* seg_off, uint32_t* seg_cnt, uint32_t* part_tot, uint8_t* dsrc,
                                uint32_t* zero_word, hipStream_t st, const uint8_t* bases = nullptr,
                                uint8_t* phi = nullptr, uint32_t* zero2 = nullptr, uint32_t nzero2 = 0);
// counts: the bucket counts, or with cc.nchunks the chunk-count prefixes (cloc)
eIcicleError launch_part_sort(const MsmPlan& P, const uint32_t* ent, const uint32_t* seg_off, const uint32_t* seg_cnt,
                              const uint32_t* part_tot, uint32_t* counts, uint32_t* offsets, uint32_t* sorted,
                              const ChunkCountOut& cc, hipStream_t st, const PartHelp& hp = PartHelp());

// ------------------------------------------------------------------------------------
// 4. accumulation: thread t sums the L contributions at sorted positions [L t, L t + L),
//    one partial per bucket segment it touches (see k_chunk_counts): no idle lanes on the
//    short last chunk of each bucket.  L = accumulate_chunk: max(16, contributions per bucket
//    / 8) -- 16 at 2^20 (one 64-byte line of sorted indices per thread, ~5 partials per
//    bucket), growing with the buckets at 2^22+ so they stay off the heavy-bucket passes
//    (MBLS_ACC_CHUNK=auto: one round of resident waves, measured slower at 2^20).
// ------------------------------------------------------------------------------------
#ifndef MBLS_ACC_MMADD
#define MBLS_ACC_MMADD 1
#endif
#ifndef MBLS_ACC_LDS
#define MBLS_ACC_LDS 1  // G1: next point prefetched into LDS (LDS-DMA) instead of VGPRs
#endif
template <class F, int MINW>
__global__ __launch_bounds__(256, MINW) void k_accumulate(const uint32_t* __restrict__ sorted, const uint32_t* __restrict__ offsets,
                                                    const uint32_t* __restrict__ chunk_off,
                                                    const uint32_t* __restrict__ first, uint32_t b0, uint32_t b1,
                                                    const uint8_t* __restrict__ bases, const uint8_t* __restrict__ phi,
                                                    uint32_t nsplit, uint32_t chunk, uint8_t* __restrict__ partials) {
    using L = typename LaneOf<F>::type;
    // buckets [b0, b1) only (one window group): sorted positions [offsets[b0], offsets[b1]); a
    // chunk straddling the group boundary is shared, each side summing its own positions
    const uint32_t gb = offsets[b0], ge = offsets[b1];
    const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) / LaneOf<F>::LANES + gb / chunk;  // chunk index
    uint32_t beg = t * chunk;
    const uint32_t end = min(beg + chunk, ge);
    beg = max(beg, gb);
    if (beg >= end) return;
    uint32_t b = first[t];
    while (offsets[b + 1] <= beg) ++b;  // straddling chunk: the group's first non-empty bucket
    uint32_t seg = chunk_off[b] + (t - offsets[b] / chunk);
    uint32_t bend = offsets[b + 1];
    Jacobian<L> acc = Jacobian<L>::inf();
    // endomorphism split: indices >= nsplit address the image table (phi(P) / psi^j(P))
    auto fetch = [&](uint32_t v) {
        uint32_t idx = v >> 1;
        const uint8_t* src = idx >= nsplit ? phi : bases;
        idx = idx >= nsplit ? idx - nsplit : idx;
        return load_affine<L>(src, idx);
    };
    // second point of the chunk (the same step for every lane of the wave): the accumulator is
    // still the first point, Z = 1, so the affine + affine formula applies (~55% of a mixed
    // addition); a bucket boundary at this step left it at the identity instead
    auto step = [&](uint32_t e, const Affine<L>& q) {
        if (e == bend) {  // bucket boundary inside the chunk: flush, move to the next bucket
            store_jac<L>(partials, seg, acc);
            acc = Jacobian<L>::inf();
            do {
                ++b;
            } while (offsets[b + 1] == e);  // skip empty buckets
            seg = chunk_off[b];
            bend = offsets[b + 1];
        }
        bool done = false;
        if (MBLS_ACC_MMADD && e == beg + 1 && !acc.is_inf() && !q.is_inf()) done = jac_mmadd(acc, q, acc);
        if (!done) acc = jac_madd(acc, q);
    };
    uint32_t v = sorted[beg];
    if constexpr (std::is_same<L, Fq>::value && MBLS_ACC_LDS) {
        // G1: the next point is prefetched into LDS by LDS-DMA (global_load_lds_dwordx4: six
        // 16-byte pieces per lane, no VGPR destination), double-buffered per wave, instead of
        // into 24 VGPRs held across the mixed addition: the accumulation fits its 168-VGPR /
        // 3-waves-per-SIMD bound without spills.  Stage: [slot][wave][piece][lane] x 16 B.
        __shared__ uint4 stage[2][256 / 64][6][64];
        const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
        auto issue = [&](uint32_t vv, uint32_t slot) {
            uint32_t idx = vv >> 1;
            const uint8_t* src = idx >= nsplit ? phi : bases;
            idx = idx >= nsplit ? idx - nsplit : idx;
            const uint8_t* g = src + (size_t)idx * 96;
#pragma unroll
            for (int k = 0; k < 6; ++k)
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const void*)(g + 16 * k),
                                                 (__attribute__((address_space(3))) void*)&stage[slot][wv][k][0], 16, 0, 0);
        };
        issue(v, 0);
        uint32_t vn = beg + 1 < end ? sorted[beg + 1] : v;
        for (uint32_t e = beg; e < end; ++e) {
            const uint32_t slot = (e - beg) & 1;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this point's pieces have landed
            Affine<Fq> p;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint4 xa = stage[slot][wv][k][ln], ya = stage[slot][wv][3 + k][ln];
                p.x.v[4 * k] = xa.x, p.x.v[4 * k + 1] = xa.y, p.x.v[4 * k + 2] = xa.z, p.x.v[4 * k + 3] = xa.w;
                p.y.v[4 * k] = ya.x, p.y.v[4 * k + 1] = ya.y, p.y.v[4 * k + 2] = ya.z, p.y.v[4 * k + 3] = ya.w;
            }
            // the other slot was read one full addition ago: safe to overwrite
            if (e + 1 < end) issue(vn, slot ^ 1u);
            const uint32_t vnn = e + 2 < end ? sorted[e + 2] : vn;
            step(e, (v & 1) ? aff_neg(p) : p);
            v = vn;
            vn = vnn;
        }
    } else {
        // one point ahead: the next random 96/192-byte fetch overlaps this mixed addition
        Affine<L> p = fetch(v);
        for (uint32_t e = beg; e < end; ++e) {
            const uint32_t vn = e + 1 < end ? sorted[e + 1] : v;
            const Affine<L> pn = fetch(vn);
            step(e, (v & 1) ? aff_neg(p) : p);
            v = vn;
            p = pn;
        }
    }
    store_jac<L>(partials, seg, acc);
}

// ------------------------------------------------------------------------------------
// 4'. G1 accumulation in unsaturated radix 2^28 (mbls_fq28.hpp; round 5).  Same schedule as
//     k_accumulate's LDS-DMA path -- chunks, bucket boundaries, the free first point and the
//     mmadd second point, the next point staged in LDS -- with the lane arithmetic on 14 x 28-bit
//     limbs: a column of a product is one v_mad_u64_u32 chain with no carry tracking (the 32-bit
//     FIPS product pays a v_addc per mad, and on gfx950 every VALU instruction costs the same
//     ~4 cycles: tools/valu_ceiling.hip).  Points are unpacked 8 bits low (x R 2^8 = x R',
//     free), partials are written back in the library's canonical Montgomery words, so every
//     other kernel is unchanged.  Same field values as jac_madd / jac_mmadd / jac_dbl, hence the
//     same Jacobian partials, bit for bit (tools/fq28_bench.hip; the GPU parity suite).
// ------------------------------------------------------------------------------------
#ifndef MBLS_ACC_R28
#define MBLS_ACC_R28 1
#endif
#ifndef MBLS_BS_R28
#define MBLS_BS_R28 1  // light bucket sums (k_bucket_small, G1) in radix 2^28 too
#endif
#ifndef MBLS_ACC_XYZZ
#define MBLS_ACC_XYZZ 1  // G1 accumulation and light / slice-chain bucket sums in XYZZ (r28::X28)
#endif
// a chunk partial's bytes: G1 partials are the accumulator's raw radix-2^28 XYZZ limbs when the
// accumulation runs in XYZZ (4 x 14 words: no to_words conversion at the flush, which is divergent
// -- a bucket boundary falls inside ~25% of the chunks, at a different step in every lane -- and no
// unpack_shift8 when the bucket sums read them), Jacobian words otherwise
template <class F>
struct PartialBytes {
    static constexpr size_t value = 3 * sizeof(F);  // Jacobian
};
template <>
struct PartialBytes<Fq> {
    static constexpr size_t value = (MBLS_ACC_XYZZ && MBLS_ACC_R28 && MBLS_ACC_LDS && MBLS_BS_R28) ? 224 : 144;
};
#ifndef MBLS_ACC_G2_R28
#define MBLS_ACC_G2_R28 1
#endif
#ifndef MBLS_ACC_G2_XYZZ
#define MBLS_ACC_G2_XYZZ 1  // G2 accumulation and bucket sums in pair-sliced XYZZ (r28p::X28p), raw partials
#endif
#define MBLS_G2_XYZZ_PARTIALS (MBLS_ACC_G2_XYZZ && MBLS_ACC_G2_R28)
template <>
struct PartialBytes<Fq2> {
    static constexpr size_t value = MBLS_G2_XYZZ_PARTIALS ? 448 : 288;
};
static_assert(!MBLS_ACC_XYZZ || (MBLS_ACC_R28 && MBLS_ACC_LDS && MBLS_BS_R28),
              "XYZZ partials need the radix-2^28 accumulation and bucket sums");
#ifndef MBLS_RED_R28
#define MBLS_RED_R28 1  // G1's lane-mode reduction levels in radix 2^28 (k_reduce_scaled_r28)
#endif
#ifndef MBLS_BUCKETS_XYZZ
#define MBLS_BUCKETS_XYZZ 1  // G1: the bucket sums stay raw XYZZ (224 B) for a lane-mode level 0
#endif
#ifndef MBLS_BUCKETS_XYZZ_G2
#define MBLS_BUCKETS_XYZZ_G2 1  // G2: the same, pair-sliced (448 B)
#endif
// G1 with a lane-mode level 0 (every large MSM): k_bucket_small stores the bucket sums as raw XYZZ
// limbs (store_xyzz28) and level 0 adds them in XYZZ (k_reduce_scaled_r28x): no x_to_jac per
// bucket, add-2008-s instead of add-2007-bl in the level's chains, no unpack_shift8 on its loads
template <class F>
constexpr bool buckets_xyzz_ok() {
    return (std::is_same<F, Fq>::value && MBLS_ACC_XYZZ && MBLS_RED_R28 && MBLS_BUCKETS_XYZZ) ||
           (std::is_same<F, Fq2>::value && MBLS_G2_XYZZ_PARTIALS && MBLS_BUCKETS_XYZZ_G2);
}
template <class F>
constexpr size_t xyzz_bucket_bytes() {
    return std::is_same<F, Fq>::value ? 224 : 448;
}
MBLS_DEV void store_xyzz28(uint8_t* __restrict__ partials, uint32_t seg, const r28::X28& acc) {
    // x, y folded (normalised, < 3p), zz, zzz normalised: valid xadd operands as they are; the
    // identity is stored as zz = 0 (the reader's test)
    uint4* q = reinterpret_cast<uint4*>(partials + (size_t)seg * 224);
    uint32_t w[56];
#pragma unroll
    for (int i = 0; i < 14; ++i) {
        w[i] = acc.x.l[i];
        w[14 + i] = acc.y.l[i];
        w[28 + i] = acc.zz.l[i];
        w[42 + i] = acc.zzz.l[i];
    }
#pragma unroll
    for (int j = 0; j < 14; ++j) q[j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
}
MBLS_DEV void store_jac28(uint8_t* __restrict__ partials, uint32_t seg, const r28::J28& acc) {
    Jacobian<Fq> out;
    if (acc.is_inf()) {
        out = Jacobian<Fq>::inf();
    } else {
        r28::to_words(acc.x, out.x.v);
        r28::to_words(acc.y, out.y.v);
        r28::to_words(acc.z, out.z.v);
    }
    store_jac<Fq>(partials, seg, out);
}

#ifndef MBLS_ACC_R28_PARK
#define MBLS_ACC_R28_PARK 1
#endif
#ifndef MBLS_ACC_R28_MINW
#define MBLS_ACC_R28_MINW 3  // waves per SIMD the register budget is sized for (variant builds: 2)
#endif
template <class F>  // F = Fq only (a template so only msm_g1.hip instantiates it)
__global__ __launch_bounds__(256, MBLS_ACC_R28_MINW) void k_accumulate_r28(const uint32_t* __restrict__ sorted,
                                                           const uint32_t* __restrict__ offsets,
                                                           const uint32_t* __restrict__ chunk_off,
                                                           const uint32_t* __restrict__ first, uint32_t b0, uint32_t b1,
                                                           const uint8_t* __restrict__ bases,
                                                           const uint8_t* __restrict__ phi, uint32_t nsplit,
                                                           uint32_t chunk, uint8_t* __restrict__ partials) {
    const uint32_t gb = offsets[b0], ge = offsets[b1];
    const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) + gb / chunk;  // chunk index
    uint32_t beg = t * chunk;
    const uint32_t end = min(beg + chunk, ge);
    beg = max(beg, gb);
    if (beg >= end) return;
    uint32_t b = first[t];
    while (offsets[b + 1] <= beg) ++b;
    uint32_t seg = chunk_off[b] + (t - offsets[b] / chunk);
    uint32_t bend = offsets[b + 1];
#if MBLS_ACC_XYZZ
    using Acc = r28::X28;
#else
    using Acc = r28::J28;
#endif
    Acc acc = Acc::inf();
    auto flush = [&](uint32_t sg) __attribute__((always_inline)) {
#if MBLS_ACC_XYZZ
        store_xyzz28(partials, sg, acc);
#else
        store_jac28(partials, sg, acc);
#endif
    };
    __shared__ uint4 stage[2][256 / 64][6][64];
#if MBLS_ACC_R28_PARK
    // acc.y parked in the lane's half of the stage that the current point was just read from
    // (free until the next step's DMA), across the mixed addition's middle: 14 VGPRs fewer at
    // the register bound, where the compiler otherwise spilled ~30 VGPRs to scratch
    struct ParkStage {
        uint4* q;  // this lane's 6 pieces of the free slot: stage[slot][wv][k][ln], stride 64
        r28::F28 x;
        MBLS_DEV void put(int s, const r28::F28& a) {
            if (s == 0) {
                x = a;
                return;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                q[64 * k] = make_uint4(a.l[4 * k], a.l[4 * k + 1], k < 3 ? a.l[4 * k + 2] : 0u, k < 3 ? a.l[4 * k + 3] : 0u);
            asm volatile("" ::: "memory");  // the register copy is dead: reload from LDS
        }
        MBLS_DEV r28::F28 get(int s) const {
            if (s == 0) return x;
            asm volatile("" ::: "memory");
            r28::F28 r;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 u = q[64 * k];
                r.l[4 * k] = u.x;
                r.l[4 * k + 1] = u.y;
                if (k < 3) {
                    r.l[4 * k + 2] = u.z;
                    r.l[4 * k + 3] = u.w;
                }
            }
            return r;
        }
    };
#endif
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    auto issue = [&](uint32_t vv, uint32_t slot) {
        uint32_t idx = vv >> 1;
        const uint8_t* src = idx >= nsplit ? phi : bases;
        idx = idx >= nsplit ? idx - nsplit : idx;
        const uint8_t* g = src + (size_t)idx * 96;
#pragma unroll
        for (int k = 0; k < 6; ++k)
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const void*)(g + 16 * k),
                                             (__attribute__((address_space(3))) void*)&stage[slot][wv][k][0], 16, 0, 0);
    };
    uint32_t v = sorted[beg];
    issue(v, 0);
    uint32_t vn = beg + 1 < end ? sorted[beg + 1] : v;
    for (uint32_t e = beg; e < end; ++e) {
        const uint32_t slot = (e - beg) & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this point's pieces have landed
        uint32_t xw[12], yw[12], any = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint4 xa = stage[slot][wv][k][ln], ya = stage[slot][wv][3 + k][ln];
            xw[4 * k] = xa.x, xw[4 * k + 1] = xa.y, xw[4 * k + 2] = xa.z, xw[4 * k + 3] = xa.w;
            yw[4 * k] = ya.x, yw[4 * k + 1] = ya.y, yw[4 * k + 2] = ya.z, yw[4 * k + 3] = ya.w;
            any |= xa.x | xa.y | xa.z | xa.w | ya.x | ya.y | ya.z | ya.w;
        }
        if (e + 1 < end) issue(vn, slot ^ 1u);  // the other slot was read one addition ago
        const uint32_t vnn = e + 2 < end ? sorted[e + 2] : vn;
        if (e == bend) {  // bucket boundary inside the chunk: flush, move to the next bucket
            flush(seg);
            acc = Acc::inf();
            do {
                ++b;
            } while (offsets[b + 1] == e);
            seg = chunk_off[b];
            bend = offsets[b + 1];
        }
        if (any) {  // the affine identity (0, 0) adds nothing
            const r28::F28 qx = r28::unpack_shift8(xw);
            r28::F28 qy = r28::unpack_shift8(yw);
            if (v & 1) qy = r28::neg<r28::B512>(qy);  // -P: < 512 p, limbs < 2^30.4 (mbls_fq28.hpp)
            bool done = false;
#if MBLS_ACC_R28_PARK
            ParkStage pk{&stage[slot][wv][0][ln]};
#else
            r28::ParkReg pk;
#endif
#if MBLS_ACC_XYZZ
            if (MBLS_ACC_MMADD && e == beg + 1 && !acc.is_inf()) done = r28::xmmadd(acc, qx, qy);
            if (!done) r28::xmadd(acc, qx, qy, pk);
#else
            if (MBLS_ACC_MMADD && e == beg + 1 && !acc.is_inf()) done = r28::mmadd(acc, qx, qy);
            if (!done) r28::madd(acc, qx, qy, pk);
#endif
        }
        v = vn;
        vn = vnn;
    }
    flush(seg);
}

// ------------------------------------------------------------------------------------
// 4''. G2 accumulation in pair-sliced radix 2^28 (mbls_fq2_28.hpp; round 6).  k_accumulate's
//     schedule over PAIRS of lanes (lane j: component j of every Fq2 value), with the next point
//     prefetched into registers one addition ahead, the chunk's first point free and its second
//     by mmadd; each lane's Fq2 product is one radix-2^28 product sum (no carry tracking).  The
//     rare exceptional step (H = 0: equal or opposite points) converts the accumulator to words
//     and takes jac_madd over PFq2.  Partials are stored in the library's canonical words: every
//     other kernel is unchanged, and the partials equal k_accumulate<Fq2>'s bit for bit.
// ------------------------------------------------------------------------------------
#ifndef MBLS_ACC_G2_R28
#define MBLS_ACC_G2_R28 1
#endif
#ifndef MBLS_ACC_G2_MINW
#define MBLS_ACC_G2_MINW 2  // waves per SIMD the register budget is sized for
#endif
#ifndef MBLS_ACC_G2_LDS
#define MBLS_ACC_G2_LDS 0  // 1: next point prefetched into LDS (LDS-DMA) instead of VGPRs
#endif
#ifndef MBLS_ACC_G2_XYZZ
#define MBLS_ACC_G2_XYZZ 1  // G2 accumulation and bucket sums in pair-sliced XYZZ (r28p::X28p), raw partials
#endif
// G2 XYZZ partial k: lane j (component j) holds its 4 x 14 raw limbs at k * 448 + j * 224
MBLS_DEV void store_xyzz28p(uint8_t* __restrict__ partials, uint32_t seg, const r28p::X28p& acc) {
    uint4* q = reinterpret_cast<uint4*>(partials + (size_t)seg * 448 + (pairdpp::odd() ? 224 : 0));
    uint32_t w[56];
#pragma unroll
    for (int i = 0; i < 14; ++i) {
        w[i] = acc.x.l[i];
        w[14 + i] = acc.y.l[i];
        w[28 + i] = acc.zz.l[i];
        w[42 + i] = acc.zzz.l[i];
    }
#pragma unroll
    for (int j = 0; j < 14; ++j) q[j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
}
MBLS_DEV void r28p_add_partial(r28p::X28p& acc, const uint8_t* __restrict__ partials, uint32_t k) {
    const uint4* q = reinterpret_cast<const uint4*>(partials + (size_t)k * 448 + (pairdpp::odd() ? 224 : 0));
    uint32_t w[56];
#pragma unroll
    for (int j = 0; j < 14; ++j) {
        const uint4 u = q[j];
        w[4 * j] = u.x, w[4 * j + 1] = u.y, w[4 * j + 2] = u.z, w[4 * j + 3] = u.w;
    }
    r28::F28 x, y, zz, zzz;
    uint32_t zany = 0;
#pragma unroll
    for (int i = 0; i < 14; ++i) {
        x.l[i] = w[i];
        y.l[i] = w[14 + i];
        zz.l[i] = w[28 + i];
        zzz.l[i] = w[42 + i];
        zany |= w[28 + i];
    }
    // the identity is zz = 0 on both lanes (pair-uniform predicate)
    if (!r28p::both(zany == 0)) r28p::xadd(acc, x, y, zz, zzz);
}
MBLS_DEV void xadd_raw(r28p::X28p& acc, const uint32_t (&w)[56]) {
    r28::F28 x, y, zz, zzz;
    uint32_t zany = 0;
#pragma unroll
    for (int i = 0; i < 14; ++i) {
        x.l[i] = w[i];
        y.l[i] = w[14 + i];
        zz.l[i] = w[28 + i];
        zzz.l[i] = w[42 + i];
        zany |= w[28 + i];
    }
    if (!r28p::both(zany == 0)) r28p::xadd(acc, x, y, zz, zzz);
}
// pair XYZZ sum -> the library's Jacobian words of this lane's component
MBLS_DEV Jacobian<PFq2> xyzz28p_to_words(const r28p::X28p& acc) {
    const r28p::J28p j = r28p::x_to_jac(acc);
    if (j.is_inf()) return Jacobian<PFq2>::inf();
    return {r28p::to_pf(j.x), r28p::to_pf(j.y), r28p::to_pf(j.z)};
}
MBLS_DEV void store_jac28p(uint8_t* __restrict__ partials, uint32_t seg, const r28p::J28p& acc) {
    Jacobian<PFq2> out;
    if (acc.is_inf())
        out = Jacobian<PFq2>::inf();
    else
        out = {r28p::to_pf(acc.x), r28p::to_pf(acc.y), r28p::to_pf(acc.z)};
    store_jac<PFq2>(partials, seg, out);
}

template <class F>  // F = Fq2 only (a template so only msm_g2.hip instantiates it)
__global__ __launch_bounds__(256, MBLS_ACC_G2_MINW) void k_accumulate_r28p(const uint32_t* __restrict__ sorted,
                                                            const uint32_t* __restrict__ offsets,
                                                            const uint32_t* __restrict__ chunk_off,
                                                            const uint32_t* __restrict__ first, uint32_t b0,
                                                            uint32_t b1, const uint8_t* __restrict__ bases,
                                                            const uint8_t* __restrict__ phi, uint32_t nsplit,
                                                            uint32_t chunk, uint8_t* __restrict__ partials) {
    const uint32_t gb = offsets[b0], ge = offsets[b1];
    const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) / 2 + gb / chunk;  // chunk index (pair)
    uint32_t beg = t * chunk;
    const uint32_t end = min(beg + chunk, ge);
    beg = max(beg, gb);
    if (beg >= end) return;  // pair-uniform: both lanes share t
    uint32_t b = first[t];
    while (offsets[b + 1] <= beg) ++b;
    uint32_t seg = chunk_off[b] + (t - offsets[b] / chunk);
    uint32_t bend = offsets[b + 1];
#if MBLS_ACC_G2_XYZZ
    using Acc = r28p::X28p;
#else
    using Acc = r28p::J28p;
#endif
    Acc acc = Acc::inf();
    auto flush = [&](uint32_t sg) __attribute__((always_inline)) {
#if MBLS_ACC_G2_XYZZ
        store_xyzz28p(partials, sg, acc);
#else
        store_jac28p(partials, sg, acc);
#endif
    };
#if MBLS_ACC_G2_LDS
    // the next point's component (x: 3 x 16 B, y: 3 x 16 B per lane) prefetched into LDS by
    // LDS-DMA, double-buffered per wave (the G1 kernel's stage): no 24 VGPRs held across the
    // addition.  Stage: [slot][wave][piece][lane] x 16 B = 48 KiB per workgroup.
    __shared__ uint4 stage[2][256 / 64][6][64];
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const uint32_t half = pairdpp::odd() ? 48u : 0u;
    auto issue = [&](uint32_t vv, uint32_t slot) {
        uint32_t idx = vv >> 1;
        const uint8_t* src = idx >= nsplit ? phi : bases;
        idx = idx >= nsplit ? idx - nsplit : idx;
        const uint8_t* g = src + (size_t)idx * 192 + half;
#pragma unroll
        for (int k = 0; k < 6; ++k)
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const void*)(g + (k < 3 ? 16 * k : 96 + 16 * (k - 3))),
                                             (__attribute__((address_space(3))) void*)&stage[slot][wv][k][0], 16, 0, 0);
    };
    uint32_t v = sorted[beg];
    issue(v, 0);
    uint32_t vn = beg + 1 < end ? sorted[beg + 1] : v;
    for (uint32_t e = beg; e < end; ++e) {
        const uint32_t slot = (e - beg) & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this point's pieces have landed
        Affine<PFq2> p;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint4 xa = stage[slot][wv][k][ln], ya = stage[slot][wv][3 + k][ln];
            p.x.v.v[4 * k] = xa.x, p.x.v.v[4 * k + 1] = xa.y, p.x.v.v[4 * k + 2] = xa.z, p.x.v.v[4 * k + 3] = xa.w;
            p.y.v.v[4 * k] = ya.x, p.y.v.v[4 * k + 1] = ya.y, p.y.v.v[4 * k + 2] = ya.z, p.y.v.v[4 * k + 3] = ya.w;
        }
        if (e + 1 < end) issue(vn, slot ^ 1u);  // the other slot was read one addition ago
        const uint32_t vnn = e + 2 < end ? sorted[e + 2] : vn;
#else
    auto fetch = [&](uint32_t vv) {
        uint32_t idx = vv >> 1;
        const uint8_t* src = idx >= nsplit ? phi : bases;
        idx = idx >= nsplit ? idx - nsplit : idx;
        return load_affine<PFq2>(src, idx);  // this lane's component of x and y
    };
    uint32_t v = sorted[beg];
    Affine<PFq2> p = fetch(v);
    for (uint32_t e = beg; e < end; ++e) {
        const uint32_t vn = e + 1 < end ? sorted[e + 1] : v;
        const Affine<PFq2> pn = fetch(vn);  // one point ahead: the gather overlaps this addition
#endif
        if (e == bend) {  // bucket boundary inside the chunk: flush, move to the next bucket
            flush(seg);
            acc = Acc::inf();
            do {
                ++b;
            } while (offsets[b + 1] == e);
            seg = chunk_off[b];
            bend = offsets[b + 1];
        }
        if (!p.is_inf()) {  // the affine identity (0, 0) adds nothing (pair-uniform predicate)
            const r28::F28 qx = r28::unpack_shift8(p.x.v.v);
            r28::F28 qy = r28::unpack_shift8(p.y.v.v);
            if (v & 1) qy = r28::carry(r28::neg<r28::B512>(qy));  // -P, normalised (mbls_fq2_28.hpp)
#if MBLS_ACC_G2_XYZZ
            bool done = false;
            if (MBLS_ACC_MMADD && e == beg + 1 && !acc.is_inf()) done = r28p::xmmadd(acc, qx, qy);
            if (!done) r28p::xmadd(acc, qx, qy);  // equal / opposite points: xdbl / identity inside
#else
            if (acc.is_inf()) {
                acc = {r28::fold(qx), r28::fold(qy), r28p::one()};
            } else {
                bool done = false;
                if (MBLS_ACC_MMADD && e == beg + 1) done = r28p::mmadd(acc, qx, qy);
                if (!done) done = r28p::madd(acc, qx, qy);
                if (!done) {  // H = 0: doubling or the identity, in words (rare)
                    const Jacobian<PFq2> aw = jac_madd(
                        Jacobian<PFq2>{r28p::to_pf(acc.x), r28p::to_pf(acc.y), r28p::to_pf(acc.z)},
                        (v & 1) ? aff_neg(p) : p);
                    if (aw.is_inf())
                        acc = r28p::J28p::inf();
                    else
                        acc = {r28::fold(r28p::from_pf(aw.x)), r28::fold(r28p::from_pf(aw.y)),
                               r28::fold(r28p::from_pf(aw.z))};
                }
            }
#endif
        }
#if MBLS_ACC_G2_LDS
        v = vn;
        vn = vnn;
#else
        v = vn;
        p = pn;
#endif
    }
    flush(seg);
}

// ------------------------------------------------------------------------------------
// Serial phases run on ROW-SLICED arithmetic (mbls_rowfield.hpp): one logical thread =
// one 16-lane row holding a field element limb-per-lane, so a serial chain of additions
// costs ~150 instead of ~1.3 K dependent instructions per product.  `rid` = row index.
// ------------------------------------------------------------------------------------
template <class F>
using RJac = Jacobian<typename RowOf<F>::type>;

template <class F>
MBLS_DEV RJac<F> rload_jac(const uint8_t* base, size_t idx) {
    using RO = RowOf<F>;
    const size_t q = idx * 3 * RO::FQS;
    return {RO::ld(base, q), RO::ld(base, q + RO::FQS), RO::ld(base, q + 2 * RO::FQS)};
}
template <class F>
MBLS_DEV void rstore_jac(uint8_t* base, size_t idx, const RJac<F>& a) {
    using RO = RowOf<F>;
    const size_t q = idx * 3 * RO::FQS;
    RO::st(base, q, a.x);
    RO::st(base, q + RO::FQS, a.y);
    RO::st(base, q + 2 * RO::FQS, a.z);
}
MBLS_DEV uint32_t row_id() { return (blockIdx.x * blockDim.x + threadIdx.x) >> 4; }

// ------------------------------------------------------------------------------------
// 6. one level of the recursive running-sum reduction.
//   in:  V[w * m_in + k], k < m_in, weight (k + off)
//   out: T[w * m_out + q], R[w * m_out + q], m_out = ceil(m_in / seg)
// Level 0 has plenty of segments and runs one segment per LANE (scalar arithmetic, short
// segments); the later, narrower levels run one segment per ROW (row-sliced arithmetic).
// Single jac_add call site: the loop alternates the R and S updates.
// ------------------------------------------------------------------------------------
// execution modes of the serial phases: one point chain per LANE (scalar arithmetic), per
// 16-lane ROW (row-sliced), or per WAVE (row-sliced, independent products spread over rows)
enum : int { MODE_LANE = 0, MODE_ROW = 1, MODE_WAVE = 2 };

template <class F, int MODE>
struct RedIO;
template <class F>
struct RedIO<F, MODE_LANE> {
    using L = typename LaneOf<F>::type;
    using J = Jacobian<L>;
    MBLS_DEV static uint32_t id() { return (blockIdx.x * blockDim.x + threadIdx.x) / LaneOf<F>::LANES; }
    MBLS_DEV static J ld(const uint8_t* b, size_t i) { return load_jac<L>(b, i); }
    MBLS_DEV static void st(uint8_t* b, size_t i, const J& v) { store_jac<L>(b, i, v); }
    MBLS_DEV static J add(const J& a, const J& b) { return jac_add(a, b); }
    MBLS_DEV static J dbl(const J& a) { return jac_dbl(a); }
};
template <class F>
struct RedIO<F, MODE_ROW> {
    using J = RJac<F>;
    MBLS_DEV static uint32_t id() { return row_id(); }
    MBLS_DEV static J ld(const uint8_t* b, size_t i) { return rload_jac<F>(b, i); }
    MBLS_DEV static void st(uint8_t* b, size_t i, const J& v) { rstore_jac<F>(b, i, v); }
    MBLS_DEV static J add(const J& a, const J& b) { return jac_add(a, b); }
    MBLS_DEV static J dbl(const J& a) { return jac_dbl(a); }
};
template <class F>
struct RedIO<F, MODE_WAVE> {
    using J = RJac<F>;
    MBLS_DEV static uint32_t id() { return (blockIdx.x * blockDim.x + threadIdx.x) >> 6; }
    MBLS_DEV static J ld(const uint8_t* b, size_t i) { return rload_jac<F>(b, i); }
    MBLS_DEV static void st(uint8_t* b, size_t i, const J& v) {
        if (wave::leader_row()) rstore_jac<F>(b, i, v);
    }
    MBLS_DEV static J add(const J& a, const J& b) { return wave::jadd(a, b); }
    MBLS_DEV static J dbl(const J& a) { return wave::jdbl(a); }
};
template <int MODE>
constexpr uint32_t lanes_per_chain() { return MODE == MODE_LANE ? 1u : MODE == MODE_ROW ? 16u : 64u; }

// ------------------------------------------------------------------------------------
// 5. bucket sums from chunk partials.  Light buckets (<= SMALL_MAX partials -- every bucket of
//    random inputs): one thread each.  Heavy buckets (equal scalars, adversarial inputs): cut into
//    slices (heavy_slices' plan, or HEAVY_SLICE partials listed by k_chunk_owner); one workgroup per slice
//    sums its slice (strided chains + an LDS tree), and the workgroup that finishes a bucket's
//    last slice (a counter per bucket: last-block-done) sums the bucket's slice sums.  The slice
//    workgroups ride in the same launch as the light buckets (HEAVY_BLOCKS extra workgroups that
//    exit at once when there is no heavy bucket): no extra launch, no side stream, no event.
// ------------------------------------------------------------------------------------
#ifndef MBLS_HEAVY_SLICE
#define MBLS_HEAVY_SLICE 2048
#endif
static constexpr uint32_t HEAVY_SLICE = MBLS_HEAVY_SLICE;  // chunk partials per heavy slice (one workgroup)
static constexpr uint32_t HEAVY_BLOCKS = 512;  // workgroups appended to k_bucket_small (two per CU)

// Heavy buckets: a slice workgroup's lanes sum strided chains of its partials (lane arithmetic:
// throughput), then its 16 rows sum the chain results ROW-SLICED (RedIO<MODE_ROW>: one 16-lane
// row per chain, ~5 us per Jacobian addition against ~25 us for a lone lane at one wave per SIMD)
// and a 4-level row tree through LDS finishes; the slice sums of a bucket are added the same way
// by the workgroup that finishes its last slice.  The former 8-level lane tree per slice took
// 0.58 ms for one bucket of 2^16 partials (G1 2^20, every scalar 1) and 1.44 ms for 16.
template <class F>
MBLS_DEV RJac<F> row_tree(RJac<F> acc, uint8_t* sh, uint32_t r) {
    using IO = RedIO<F, MODE_ROW>;
    constexpr uint32_t ROWS = 256 / 16;
    IO::st(sh, r, acc);
    __syncthreads();
    for (uint32_t s = ROWS / 2; s > 0; s >>= 1) {
        if (r < s) {
            acc = IO::add(acc, IO::ld(sh, r + s));
            IO::st(sh, r, acc);
        }
        __syncthreads();
    }
    return acc;
}

// sum of n <= 16 Jacobian points ld(k) by the workgroup's 4 waves in the wave layout (a wave
// addition spreads its independent products over the 4 rows: ~1/3 of a row addition's latency):
// wave w adds points w, w + 4, ... (<= 3 additions), wave 0 adds the 3 other wave sums through
// sh slots 1..3 (a wave writes only its own slot, read by no other wave before the barrier).
// Result valid in wave 0.  6 dependent additions against the row tree's 4 x ~3.
template <class F, class Ld>
MBLS_DEV RJac<F> wave_sum16(uint8_t* sh, uint32_t n, Ld&& ld) {
    using W = RedIO<F, MODE_WAVE>;
    const uint32_t wv = threadIdx.x >> 6;
    RJac<F> acc = wv < n ? ld(wv) : RJac<F>::inf();
    for (uint32_t k = wv + 4; k < n; k += 4) acc = W::add(acc, ld(k));
    W::st(sh, wv, acc);
    __syncthreads();
    if (wv == 0)
        for (uint32_t k = 1; k < 4 && k < n; ++k) acc = W::add(acc, W::ld(sh, k));
    __syncthreads();  // sh is reused by the caller
    return acc;
}

// sum of the CHAINS Jacobian points in sh (lane layout), by rows; result in row 0
template <class F>
MBLS_DEV RJac<F> rows_sum_chains(uint8_t* sh, uint32_t chains) {
    using IO = RedIO<F, MODE_ROW>;
    constexpr uint32_t ROWS = 256 / 16;
    const uint32_t r = threadIdx.x >> 4;
    RJac<F> acc = r < chains ? IO::ld(sh, r) : RJac<F>::inf();  // no addition to the identity first
    for (uint32_t k = r + ROWS; k < chains; k += ROWS) acc = IO::add(acc, IO::ld(sh, k));
    // row r has read its slots (k = r, r + 16, ...); row_tree overwrites only slot r < 16
    return row_tree<F>(acc, sh, r);
}

// inclusive wave64 scan (shuffles)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

MBLS_DEV bool load_j28(const uint8_t* __restrict__ base, size_t i, r28::F28& x, r28::F28& y, r28::F28& z) {
    const uint4* q = reinterpret_cast<const uint4*>(base + i * 144);
    uint32_t w[3][12], zany = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint4 u = q[3 * c + j];
            w[c][4 * j] = u.x, w[c][4 * j + 1] = u.y, w[c][4 * j + 2] = u.z, w[c][4 * j + 3] = u.w;
        }
#pragma unroll
    for (int j = 0; j < 12; ++j) zany |= w[2][j];
    if (!zany) return false;  // the identity
    x = r28::unpack_shift8(w[0]);
    y = r28::unpack_shift8(w[1]);
    z = r28::unpack_shift8(w[2]);
    return true;
}
// r28 XYZZ addition of chunk partial k (G1 with MBLS_ACC_XYZZ: the light path's and the slice
// chains' form; raw limbs, store_xyzz28); the identity (zz = 0) adds nothing
// the 56 raw words of XYZZ record k (224 B; `half` selects the odd lane's half of a 448-B pair record)
MBLS_DEV void load_raw56(const uint8_t* __restrict__ recs, size_t off, uint32_t (&w)[56]) {
    const uint4* q = reinterpret_cast<const uint4*>(recs + off);
#pragma unroll
    for (int j = 0; j < 14; ++j) {
        const uint4 u = q[j];
        w[4 * j] = u.x, w[4 * j + 1] = u.y, w[4 * j + 2] = u.z, w[4 * j + 3] = u.w;
    }
}
MBLS_DEV void xadd_raw(r28::X28& acc, const uint32_t (&w)[56]) {
    r28::F28 x, y, zz, zzz;
    uint32_t zany = 0;
#pragma unroll
    for (int i = 0; i < 14; ++i) {
        x.l[i] = w[i];
        y.l[i] = w[14 + i];
        zz.l[i] = w[28 + i];
        zzz.l[i] = w[42 + i];
        zany |= w[28 + i];
    }
    if (zany) r28::xadd(acc, x, y, zz, zzz);
}
MBLS_DEV void r28_add_partial(r28::X28& acc, const uint8_t* __restrict__ partials, uint32_t k) {
    uint32_t w[56];
    load_raw56(partials, (size_t)k * 224, w);
    xadd_raw(acc, w);
}
// r28 lane addition of Jacobian chunk partial k (G1 without MBLS_ACC_XYZZ)
MBLS_DEV void r28_add_partial(r28::J28& acc, const uint8_t* __restrict__ partials, uint32_t k) {
    const uint4* q = reinterpret_cast<const uint4*>(partials + (size_t)k * 144);
    uint32_t w[3][12], zany = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint4 u = q[3 * c + j];
            w[c][4 * j] = u.x, w[c][4 * j + 1] = u.y, w[c][4 * j + 2] = u.z, w[c][4 * j + 3] = u.w;
        }
#pragma unroll
    for (int j = 0; j < 12; ++j) zany |= w[2][j];
    if (zany) r28::jadd(acc, r28::unpack_shift8(w[0]), r28::unpack_shift8(w[1]), r28::unpack_shift8(w[2]));
}

// Slice plan (round 5): the slice length S adapts to the heavy partials T of the call, S =
// clamp(pow2 >= T / (slice workgroups), HEAVY_SLICE_MIN, HEAVY_SLICE), so that few heavy buckets
// (half the scalars 1: one bucket of 2^15 partials at G1 2^20) spread over many workgroups
// instead of 16 slices of 8-deep lane chains, while many (one repeated scalar: 16 buckets of 2^16)
// keep 2048-partial slices, one round of workgroups.  Every slice workgroup derives the plan from
// the heavy-bucket list (their chunk counts, a prefix of slices per bucket in LDS); more than
// HEAVY_LDS heavy buckets take k_chunk_owner's fixed HEAVY_SLICE plan (H.owner / first / nslices).
// Planned slices finish in groups of HEAVY_GROUP: the workgroup finishing a group's last slice
// sums the group (one row each, a 4-level row tree), the one finishing a bucket's last group sums
// the group sums -- with 64-partial slices a bucket of 2^15 partials takes 3 + 4, 4 and 2 + 4
// dependent row additions instead of 16 + 4 and 32 + 4 in one level.
#ifndef MBLS_HEAVY_SLICE_MIN
#define MBLS_HEAVY_SLICE_MIN 256
#endif
#ifndef MBLS_HEAVY_TRACE
#define MBLS_HEAVY_TRACE 0
#endif
static constexpr uint32_t HEAVY_SLICE_MIN = MBLS_HEAVY_SLICE_MIN, HEAVY_LDS = 1024, HEAVY_GROUP = 16;

// a bucket's row-layout sum (limb j on lane j of row 0 -- wave layout's leader row, or the row
// tree's row 0) into `buckets`: Jacobian words (rstore_jac), or with xb the raw XYZZ limbs of
// (X, Y, Z^2, Z^3) the lane-mode level 0 reads (k_reduce_scaled_r28x).  Wave 0, all 64 lanes.
template <class F>
MBLS_DEV void store_bucket_row(uint8_t* __restrict__ buckets, uint32_t b, const RJac<F>& p, bool xb) {
    if constexpr (std::is_same<F, Fq>::value && buckets_xyzz_ok<F>()) {
        if (xb) {
            uint32_t w[3][12], zany = 0;
#pragma unroll
            for (int i = 0; i < 12; ++i) {
                w[0][i] = (uint32_t)__shfl((int)p.x.v, i, 64);
                w[1][i] = (uint32_t)__shfl((int)p.y.v, i, 64);
                w[2][i] = (uint32_t)__shfl((int)p.z.v, i, 64);
                zany |= w[2][i];
            }
            if (threadIdx.x != 0) return;
            r28::X28 a = r28::X28::inf();
            if (zany) {
                const r28::F28 z = r28::unpack_shift8(w[2]);
                a.x = r28::fold(r28::unpack_shift8(w[0]));
                a.y = r28::fold(r28::unpack_shift8(w[1]));
                a.zz = r28::sqr(z);
                a.zzz = r28::mul(a.zz, z);
            }
            store_xyzz28(buckets, b, a);
            return;
        }
    }
    if constexpr (std::is_same<F, Fq2>::value && buckets_xyzz_ok<F>()) {
        if (xb) {  // every lane of wave 0 forms its pair component (c0 on even lanes, c1 on odd)
            const bool odd = pairdpp::odd();
            uint32_t w[3][12], zany = 0;
#pragma unroll
            for (int i = 0; i < 12; ++i) {
                const uint32_t x0 = (uint32_t)__shfl((int)p.x.c0.v, i, 64), x1 = (uint32_t)__shfl((int)p.x.c1.v, i, 64);
                const uint32_t y0 = (uint32_t)__shfl((int)p.y.c0.v, i, 64), y1 = (uint32_t)__shfl((int)p.y.c1.v, i, 64);
                const uint32_t z0 = (uint32_t)__shfl((int)p.z.c0.v, i, 64), z1 = (uint32_t)__shfl((int)p.z.c1.v, i, 64);
                w[0][i] = odd ? x1 : x0;
                w[1][i] = odd ? y1 : y0;
                w[2][i] = odd ? z1 : z0;
                zany |= z0 | z1;
            }
            r28p::X28p a = r28p::X28p::inf();
            if (zany) {  // wave-uniform
                const r28::F28 z = r28::fold(r28::unpack_shift8(w[2]));
                a.x = r28::fold(r28::unpack_shift8(w[0]));
                a.y = r28::fold(r28::unpack_shift8(w[1]));
                a.zz = r28p::sqr<r28::B16>(z);
                a.zzz = r28p::mul<r28::B16>(a.zz, z);
            }
            if (threadIdx.x < 2) store_xyzz28p(buckets, b, a);
            return;
        }
    }
    if (wave::leader_row()) rstore_jac<F>(buckets, b, p);
}

template <class F>
MBLS_DEV void heavy_slices(const uint32_t* __restrict__ chunk_off, const uint8_t* __restrict__ partials,
                           uint8_t* __restrict__ buckets, const HeavyTab& H, uint32_t hb, uint32_t nhb, bool xb) {
    using L = typename LaneOf<F>::type;
    using IO = RedIO<F, MODE_ROW>;
    constexpr uint32_t LN = LaneOf<F>::LANES;
    constexpr uint32_t CHAINS = 256 / LN;
    __shared__ __attribute__((aligned(16))) uint8_t sh[CHAINS * 3 * sizeof(F)];
    __shared__ uint32_t last, hfirst[HEAVY_LDS + 1], wred[4];
    const uint32_t nh = H.cnt[0];
    if (nh == 0) return;  // workgroup-uniform (random scalars: every slice workgroup leaves here)
#if MBLS_HEAVY_TRACE  // diagnostic builds only: per-workgroup wall-clock stamps
    const uint64_t tr0 = wall_clock64();
    uint64_t trs = 0, trg = 0;
#endif
    const bool planned = nh <= HEAVY_LDS;
    uint32_t S = HEAVY_SLICE, nsl = H.cnt[1];
    if (planned) {
        const uint32_t per = (nh + 255) / 256, e0 = min(threadIdx.x * per, nh), e1 = min(e0 + per, nh);
        uint32_t t = 0;
        for (uint32_t e = e0; e < e1; ++e) {
            const uint32_t b = H.bucket[e];
            t += chunk_off[b + 1] - chunk_off[b];
        }
        uint32_t r = t;
        for (int d = 32; d > 0; d >>= 1) r += __shfl_xor(r, d, 64);
        if ((threadIdx.x & 63) == 0) wred[threadIdx.x >> 6] = r;
        __syncthreads();
        const uint32_t T = wred[0] + wred[1] + wred[2] + wred[3];
        const uint32_t want = (T + nhb - 1) / nhb;
        S = HEAVY_SLICE_MIN;
        while (S < want && S < HEAVY_SLICE) S <<= 1;
        uint32_t c = 0;
        for (uint32_t e = e0; e < e1; ++e) {
            const uint32_t b = H.bucket[e];
            c += (chunk_off[b + 1] - chunk_off[b] + S - 1) / S;
        }
        const uint32_t incl = wave_incl_scan(c);
        __syncthreads();  // wred is reused
        if ((threadIdx.x & 63) == 63) wred[threadIdx.x >> 6] = incl;
        __syncthreads();
        uint32_t f = incl - c;
        for (uint32_t k = 0; k < (threadIdx.x >> 6); ++k) f += wred[k];
        for (uint32_t e = e0; e < e1; ++e) {
            const uint32_t b = H.bucket[e];
            hfirst[e] = f;
            f += (chunk_off[b + 1] - chunk_off[b] + S - 1) / S;
        }
        if (e1 == nh && e0 < e1) hfirst[nh] = f;
        __syncthreads();
        nsl = hfirst[nh];
    }
    // slices <= nhb + nh with S >= T / nhb: within HEAVY_GDONE for nh <= HEAVY_LDS (checked anyway)
    const bool grouped = planned && nsl <= HEAVY_GDONE;
    const uint32_t j = threadIdx.x / LN;
    for (uint32_t g = hb; g < nsl; g += nhb) {
        uint32_t e, f0, ns;
        if (planned) {  // the bucket whose slices hold g: last e with hfirst[e] <= g
            uint32_t lo = 0, hi = nh;  // hfirst[lo] <= g < hfirst[hi]
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (hfirst[mid] <= g)
                    lo = mid;
                else
                    hi = mid;
            }
            e = lo, f0 = hfirst[lo], ns = hfirst[lo + 1] - f0;
        } else {
            e = H.owner[g], f0 = H.first[e], ns = H.nslices[e];
        }
        const uint32_t b = H.bucket[e];
        const uint32_t c0 = chunk_off[b] + (g - f0) * S;
        const uint32_t c1 = min(c0 + S, chunk_off[b + 1]);
        // chains, then a lane tree down to 16 chain sums (log depth: a lane addition is ~1.3x a
        // row addition's latency, but 16 rows summing 256 chains took 15 of them in series), then
        // the rows
        uint32_t live = min(CHAINS, c1 - c0);
        if constexpr (std::is_same<L, Fq>::value && MBLS_BS_R28) {
#if MBLS_ACC_XYZZ
            r28::X28 xacc = r28::X28::inf();
            for (uint32_t k = c0 + j; k < c1; k += CHAINS) r28_add_partial(xacc, partials, k);
            r28::J28 acc = r28::x_to_jac(xacc);  // the lane tree below adds Jacobian chain sums
#else
            r28::J28 acc = r28::J28::inf();
            for (uint32_t k = c0 + j; k < c1; k += CHAINS) r28_add_partial(acc, partials, k);
#endif
            store_jac28(sh, j, acc);
            __syncthreads();
            for (; live > 16; live = (live + 1) / 2) {
                const uint32_t h = (live + 1) / 2;  // chain j < live - h takes chain j + h
                if (j < live - h) {
                    r28::F28 x, y, z;
                    if (load_j28(sh, j + h, x, y, z)) r28::jadd(acc, x, y, z);
                }
                __syncthreads();
                if (j < live - h) store_jac28(sh, j, acc);
                __syncthreads();
            }
        } else {
            Jacobian<L> acc = Jacobian<L>::inf();
            if constexpr (std::is_same<F, Fq2>::value && MBLS_G2_XYZZ_PARTIALS) {
                r28p::X28p xacc = r28p::X28p::inf();
                for (uint32_t k = c0 + j; k < c1; k += CHAINS) r28p_add_partial(xacc, partials, k);
                acc = xyzz28p_to_words(xacc);  // the lane tree below adds Jacobian chain sums
            } else {
                for (uint32_t k = c0 + j; k < c1; k += CHAINS) acc = jac_add(acc, load_jac<L>(partials, k));
            }
            store_jac<L>(sh, j, acc);
            __syncthreads();
            for (; live > 16; live = (live + 1) / 2) {
                const uint32_t h = (live + 1) / 2;
                if (j < live - h) acc = jac_add(acc, load_jac<L>(sh, j + h));
                __syncthreads();
                if (j < live - h) store_jac<L>(sh, j, acc);
                __syncthreads();
            }
        }
        using WIO = RedIO<F, MODE_WAVE>;
        const RJac<F> ssum = wave_sum16<F>(sh, live, [&](uint32_t k) { return WIO::ld(sh, k); });
#if MBLS_HEAVY_TRACE
        trs = wall_clock64();
#endif
        if (threadIdx.x < 64) WIO::st(H.res, g, ssum);
        __threadfence();
        __syncthreads();
        const uint32_t r = threadIdx.x >> 4;
        // the sums to combine at the bucket level: slice sums (one level), or the group sums at
        // f0, f0 + HEAVY_GROUP, ... (grouped)
        uint32_t nsum = ns, step = 1;
        if (grouped) {
            const uint32_t gl = f0 + (g - f0) / HEAVY_GROUP * HEAVY_GROUP;  // the group's first slice
            const uint32_t gs = min(HEAVY_GROUP, f0 + ns - gl);
            if (threadIdx.x == 0) last = atomicAdd(&H.gdone[gl], 1u) + 1 == gs ? 1u : 0u;
            __syncthreads();
            if (!last) continue;  // workgroup-uniform; sh and `last` are rewritten after barriers
            __threadfence();
            const RJac<F> gsum = wave_sum16<F>(sh, gs, [&](uint32_t k) { return WIO::ld(H.res, gl + k); });
            if (threadIdx.x < 64) WIO::st(H.res, gl, gsum);
#if MBLS_HEAVY_TRACE
            trg = wall_clock64();
#endif
            __threadfence();
            __syncthreads();
            nsum = (ns + HEAVY_GROUP - 1) / HEAVY_GROUP, step = HEAVY_GROUP;
        }
        if (threadIdx.x == 0) last = atomicAdd(&H.done[e], 1u) + 1 == nsum ? 1u : 0u;
        __syncthreads();
        if (last) {  // this workgroup finished bucket b's last slice (group): sum the sums
#if MBLS_HEAVY_TRACE
            const uint64_t trf0 = wall_clock64();
#endif
            __threadfence();
#if MBLS_HEAVY_TRACE
            const uint64_t trf1 = wall_clock64();
#endif
            if (nsum <= 16) {  // workgroup-uniform
                const RJac<F> tot = wave_sum16<F>(sh, nsum, [&](uint32_t k) { return WIO::ld(H.res, f0 + k * step); });
                if (threadIdx.x < 64) store_bucket_row<F>(buckets, b, tot, xb);
            } else {
                RJac<F> tot = r < nsum ? IO::ld(H.res, f0 + r * step) : RJac<F>::inf();
                for (uint32_t k = r + 16; k < nsum; k += 16) tot = IO::add(tot, IO::ld(H.res, f0 + k * step));
                tot = row_tree<F>(tot, sh, r);
                if (threadIdx.x < 64) store_bucket_row<F>(buckets, b, tot, xb);
            }
#if MBLS_HEAVY_TRACE
            const uint64_t trb = wall_clock64();
            if (threadIdx.x == 0)
                printf("HB g=%u e=%u t0=%llu ts=%llu tg=%llu tf0=%llu tf1=%llu tb=%llu\n", g, e, tr0, trs, trg, trf0, trf1, trb);
#endif
        }
#if MBLS_HEAVY_TRACE
        else if (threadIdx.x == 0) printf("HS g=%u e=%u t0=%llu ts=%llu tg=%llu\n", g, e, tr0, trs, trg);
#endif
        __syncthreads();  // sh and `last` are reused by the next slice
    }
}

// light buckets: one thread per bucket (<= SMALL_MAX chunks) sums its chunk partials; thread t
// takes perm[start + t] (k_chunk_owner: buckets grouped by chunk count, heaviest first, so a
// wave's lanes run the same number of additions).  The first HEAVY_BLOCKS workgroups take the
// heavy slices, the light buckets' `light_blocks` follow.
template <class F>
// 2 waves per SIMD: G1 fits anyway (181 VGPRs); G2's pair-sliced sums took 260 VGPRs + 4 AGPRs,
// i.e. one latency-bound wave per SIMD -- capped at 256 (4 spilled) its bucket sums take 0.93
// instead of 1.17 ms at 2^20 (A/B x2 on one box, profiles/r04/bs_minw_ab.txt)
#ifndef MBLS_BS_MINW
#define MBLS_BS_MINW 2
#endif
__global__ __launch_bounds__(256, MBLS_BS_MINW) void k_bucket_small(const uint32_t* __restrict__ chunk_off,
                                                      const uint32_t* __restrict__ perm, const uint32_t* __restrict__ binbase,
                                                      uint32_t gwords, const uint8_t* __restrict__ partials,
                                                      uint8_t* __restrict__ buckets, uint32_t light_blocks, HeavyTab H,
                                                      int xb) {
    MBLS_TAIL_PRIO();
    using L = typename LaneOf<F>::type;
    // the slice workgroups come first: dispatched at once, the heavy buckets' chains overlap the
    // light buckets (they used to start behind them: G1 2^20 half ones ~0.1 ms)
    if (blockIdx.x < HEAVY_BLOCKS) {
        heavy_slices<F>(chunk_off, partials, buckets, H, blockIdx.x, HEAVY_BLOCKS, xb != 0);
        return;
    }
    // light workgroups one wave-priority step below the slice workgroups: the heavy buckets'
    // dependent row chains share CUs with them (G1 2^20 half ones: a bucket-level row tree took
    // 130-220 us beside light sums instead of ~45)
    __builtin_amdgcn_s_setprio(MBLS_LIGHT_PRIO);
    const uint32_t start = binbase[0], stop = binbase[gwords];
    const uint32_t t = start + ((blockIdx.x - HEAVY_BLOCKS) * blockDim.x + threadIdx.x) / LaneOf<F>::LANES;
    if (t >= stop) return;
    const uint32_t b = perm[t];
    const uint32_t k0 = chunk_off[b], k1 = chunk_off[b + 1];
    if constexpr (std::is_same<L, Fq>::value && MBLS_BS_R28) {
        // radix 2^28: XYZZ sums of XYZZ partials (add-2008-s), one conversion per bucket (round 6);
        // Jacobian jadd otherwise (round 5)
#if MBLS_ACC_XYZZ
        r28::X28 acc = r28::X28::inf();
        for (uint32_t k = k0; k < k1; ++k) r28_add_partial(acc, partials, k);
        if (xb)
            store_xyzz28(buckets, b, acc);
        else
            store_jac28(buckets, b, r28::x_to_jac(acc));
#else
        r28::J28 acc = r28::J28::inf();
        for (uint32_t k = k0; k < k1; ++k) r28_add_partial(acc, partials, k);
        store_jac28(buckets, b, acc);
#endif
        return;
    }
    if constexpr (std::is_same<F, Fq2>::value && MBLS_G2_XYZZ_PARTIALS) {
        // pair-sliced radix-2^28 XYZZ sums of the raw XYZZ partials (round 6), one conversion
        r28p::X28p acc = r28p::X28p::inf();
        for (uint32_t k = k0; k < k1; ++k) r28p_add_partial(acc, partials, k);
        if (xb)
            store_xyzz28p(buckets, b, acc);
        else
            store_jac<L>(buckets, b, xyzz28p_to_words(acc));
        return;
    }
    Jacobian<L> acc = Jacobian<L>::inf();
    if (k1 > k0) acc = load_jac<L>(partials, k0);
    for (uint32_t k = k0 + 1; k < k1; ++k) acc = jac_add(acc, load_jac<L>(partials, k));
    store_jac<L>(buckets, b, acc);
}

// Scaled running-sum level: every level's outputs carry weight 1, so
// the last level's single output per window IS the window sum -- no per-level T tree sums on side
// streams and no window Horner.  Level l sees inputs with
//   G_w = sum_k ((k + off) V_k + U_k)            (level 0: V = buckets, off = 1, no U)
// and segment q = [k0, k1) of 2^s inputs produces
//   U'_q = sum_t (t - k0 + off) V_t + sum_t U_t   (running sum: R += V_t; S += R; S += U_t)
//   V'_q = 2^s sum_t V_t                           (s doublings of R)
// so that G_w = sum_q (q V'_q + U'_q): the same form with off = 0.  One add call site (the three
// steps of a t alternate), one doubling call site.
template <class F, int MODE>
__global__ __launch_bounds__(256) void k_reduce_scaled(const uint8_t* __restrict__ V, const uint8_t* __restrict__ U,
                                                       uint32_t m_in, uint32_t seg_log, int Wg, int off,
                                                       uint8_t* __restrict__ Vout, uint8_t* __restrict__ Uout) {
    MBLS_TAIL_PRIO();
    using IO = RedIO<F, MODE>;
    using J = typename IO::J;
    const uint32_t seg = 1u << seg_log;
    const uint32_t m_out = (m_in + seg - 1) >> seg_log;
    const uint32_t tid = IO::id();
    if (tid >= m_out * (uint32_t)Wg) return;
    const uint32_t w = tid / m_out, q = tid % m_out;
    const uint32_t k0 = q << seg_log;
    const uint32_t k1 = min(k0 + seg, m_in);  // exclusive
    const size_t base = (size_t)w * m_in;
    J R = J::inf(), S = J::inf();
    uint32_t t = k1 - 1;
    int ph = 0;  // 0: R += V_t, 1: S += R, 2: S += U_t
    while (true) {
        const bool skip = (ph == 1 && (t - k0) + off == 0) || (ph == 2 && !U);
        if (!skip) {
            const J x = ph == 0 ? R : S;
            const J y = ph == 0 ? IO::ld(V, base + t) : ph == 1 ? R : IO::ld(U, base + t);
            const J z = IO::add(x, y);
            if (ph == 0)
                R = z;
            else
                S = z;
        }
        if (ph == 2) {
            if (t == k0) break;
            --t;
            ph = 0;
        } else {
            ++ph;
        }
    }
    if (Vout) {
        for (uint32_t k = 0; k < seg_log; ++k) R = IO::dbl(R);
        IO::st(Vout, tid, R);
    }
    IO::st(Uout, tid, S);
}

// G1's lane-mode level in radix 2^28 (round 5: the same outputs as k_reduce_scaled<Fq,
// MODE_LANE> -- jadd / dbl compute the field values of jac_add / jac_dbl -- with ~20% fewer
// instructions per addition on a chain that runs one wave per SIMD)
template <class F>  // F = Fq only
__global__ __launch_bounds__(256) void k_reduce_scaled_r28(const uint8_t* __restrict__ V, const uint8_t* __restrict__ U,
                                                           uint32_t m_in, uint32_t seg_log, int Wg, int off,
                                                           uint8_t* __restrict__ Vout, uint8_t* __restrict__ Uout) {
    MBLS_TAIL_PRIO();
    const uint32_t seg = 1u << seg_log;
    const uint32_t m_out = (m_in + seg - 1) >> seg_log;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= m_out * (uint32_t)Wg) return;
    const uint32_t w = tid / m_out, q = tid % m_out;
    const uint32_t k0 = q << seg_log;
    const uint32_t k1 = min(k0 + seg, m_in);  // exclusive
    const size_t base = (size_t)w * m_in;
    r28::J28 R = r28::J28::inf(), S = r28::J28::inf();
    r28::F28 x, y, z;
    for (uint32_t t = k1; t-- > k0;) {
        if (load_j28(V, base + t, x, y, z)) r28::jadd(R, x, y, z);  // R += V_t
        if ((t - k0) + off != 0 && !R.is_inf()) r28::jadd(S, R.x, R.y, r28::carry(R.z));  // S += R
        if (U && load_j28(U, base + t, x, y, z)) r28::jadd(S, x, y, z);  // S += U_t
    }
    if (Vout) {
        for (uint32_t k = 0; k < seg_log; ++k) R = r28::dbl(R);
        store_jac28(Vout, tid, R);
    }
    store_jac28(Uout, tid, S);
}

#ifndef MBLS_RED0_PREFETCH
#define MBLS_RED0_PREFETCH 1  // level 0 loads bucket t - 1 before adding bucket t
#endif
// level 0 over raw XYZZ buckets (buckets_xyzz_ok, no U): the chain of k_reduce_scaled_r28 with
// add-2008-s (r28::xadd, 12M + 2S) for its two additions per step, the outputs converted once
template <class F>  // F = Fq only
__global__ __launch_bounds__(256) void k_reduce_scaled_r28x(const uint8_t* __restrict__ V, uint32_t m_in,
                                                            uint32_t seg_log, int Wg, int off,
                                                            uint8_t* __restrict__ Vout, uint8_t* __restrict__ Uout) {
    MBLS_TAIL_PRIO();
    const uint32_t seg = 1u << seg_log;
    const uint32_t m_out = (m_in + seg - 1) >> seg_log;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= m_out * (uint32_t)Wg) return;
    const uint32_t w = tid / m_out, q = tid % m_out;
    const uint32_t k0 = q << seg_log;
    const uint32_t k1 = min(k0 + seg, m_in);  // exclusive
    const uint32_t base = w * m_in;
    r28::X28 R = r28::X28::inf(), S = r28::X28::inf();
    uint32_t nw[56];  // bucket t - 1, loaded while bucket t is added (one wave per SIMD: nothing else hides it)
    load_raw56(V, (size_t)(base + k1 - 1) * 224, nw);
    for (uint32_t t = k1; t-- > k0;) {
        uint32_t cw[56];
#pragma unroll
        for (int i = 0; i < 56; ++i) cw[i] = nw[i];
        if (MBLS_RED0_PREFETCH && t > k0) load_raw56(V, (size_t)(base + t - 1) * 224, nw);
        xadd_raw(R, cw);                                                                   // R += V_t
        if ((t - k0) + off != 0 && !R.is_inf()) r28::xadd(S, R.x, R.y, R.zz, R.zzz);  // S += R
        if (!MBLS_RED0_PREFETCH && t > k0) load_raw56(V, (size_t)(base + t - 1) * 224, nw);
    }
    if (Vout) {
        if (!R.is_inf())
            for (uint32_t k = 0; k < seg_log; ++k) r28::xdbl(R);
        store_jac28(Vout, tid, r28::x_to_jac(R));
    }
    store_jac28(Uout, tid, r28::x_to_jac(S));
}

// the same over raw pair-sliced XYZZ records (G2): one chain per lane pair; a lane level after
// level 0 adds U_t too (raw, from the previous lane level).  Outputs raw when the next level is a
// lane level too (raw_out), else Jacobian words (store_jac<PFq2>, the form a row / wave level reads)
template <class F>  // F = Fq2 only
__global__ __launch_bounds__(256) void k_reduce_scaled_r28px(const uint8_t* __restrict__ V, const uint8_t* __restrict__ U,
                                                             uint32_t m_in, uint32_t seg_log, int Wg, int off,
                                                             uint8_t* __restrict__ Vout, uint8_t* __restrict__ Uout,
                                                             int raw_out) {
    MBLS_TAIL_PRIO();
    const uint32_t seg = 1u << seg_log;
    const uint32_t m_out = (m_in + seg - 1) >> seg_log;
    const uint32_t tid = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;  // pair-uniform
    if (tid >= m_out * (uint32_t)Wg) return;
    const uint32_t w = tid / m_out, q = tid % m_out;
    const uint32_t k0 = q << seg_log;
    const uint32_t k1 = min(k0 + seg, m_in);  // exclusive
    const uint32_t base = w * m_in;
    r28p::X28p R = r28p::X28p::inf(), S = r28p::X28p::inf();
    const size_t half = pairdpp::odd() ? 224 : 0;
    uint32_t nw[56];
    load_raw56(V, (size_t)(base + k1 - 1) * 448 + half, nw);
    for (uint32_t t = k1; t-- > k0;) {
        uint32_t cw[56];
#pragma unroll
        for (int i = 0; i < 56; ++i) cw[i] = nw[i];
        if (MBLS_RED0_PREFETCH && t > k0) load_raw56(V, (size_t)(base + t - 1) * 448 + half, nw);
        xadd_raw(R, cw);                                                                    // R += V_t
        if ((t - k0) + off != 0 && !R.is_inf()) r28p::xadd(S, R.x, R.y, R.zz, R.zzz);  // S += R
        if (!MBLS_RED0_PREFETCH && t > k0) load_raw56(V, (size_t)(base + t - 1) * 448 + half, nw);
        if (U) {  // S += U_t
            load_raw56(U, (size_t)(base + t) * 448 + half, cw);
            xadd_raw(S, cw);
        }
    }
    if (Vout) {
        // the identity stays exactly zz = 0: a pair product by zz = 0 is only 0 mod p (the partner's
        // negation is a bias multiple of p), which a raw record would carry on as a point
        if (!R.is_inf())
            for (uint32_t k = 0; k < seg_log; ++k) r28p::xdbl(R);
        if (raw_out)
            store_xyzz28p(Vout, tid, R);
        else
            store_jac<PFq2>(Vout, tid, xyzz28p_to_words(R));
    }
    if (raw_out)
        store_xyzz28p(Uout, tid, S);
    else
        store_jac<PFq2>(Uout, tid, xyzz28p_to_words(S));
}

// A narrow level (few segments: the GPU is idle but for one wave per chain) as a tree: one
// workgroup of 4 waves per segment of 4 inputs (off = 0), each wave one wave-layout point op per
// step, intermediate points through LDS.  The same outputs as k_reduce_scaled's chain
//   U' = V1 + 2 V2 + 3 V3 + U0 + U1 + U2 + U3,   V' = 4 (V0 + V1 + V2 + V3)
// in 4 dependent steps instead of 12:
//   1: a = V2 + V3 | b = U0 + U1 | c = U2 + U3 | d = V0 + V1
//   2: e = a + V3  | k = a + V1  | f = b + c   | g = d + a
//   3: W = k + e                               | 2g
//   4: U' = W + f                              | V' = 4g
// (inputs past the level's end are the identity; the additions are exact point additions, so
// the association does not change the resulting point -- only its Jacobian representative,
// which the final (x, y, 1) normalisation removes)
template <class F>
struct TreeLds {
    using J = RJac<F>;
    static constexpr int FQS = RowOf<F>::FQS;  // Fq words-of-12 per coordinate
    static constexpr int WORDS = 3 * FQS * 12;
    MBLS_DEV static void put1(uint32_t* s, const RFq& a) {
        if (wave::row() == 0 && rowdpp::lane16() < 12) s[rowdpp::lane16()] = a.v;
    }
    MBLS_DEV static RFq get1(const uint32_t* s) {
        const uint32_t j = rowdpp::lane16();
        return {j < 12 ? s[j] : 0u};
    }
    MBLS_DEV static void put1(uint32_t* s, const RFq2& a) {
        put1(s, a.c0);
        put1(s + 12, a.c1);
    }
    MBLS_DEV static void get1(const uint32_t* s, RFq2& a) {
        a.c0 = get1(s);
        a.c1 = get1(s + 12);
    }
    MBLS_DEV static void get1(const uint32_t* s, RFq& a) { a = get1(s); }
    MBLS_DEV static void put(uint32_t* s, const J& p) {
        put1(s, p.x);
        put1(s + 12 * FQS, p.y);
        put1(s + 24 * FQS, p.z);
    }
    MBLS_DEV static J get(const uint32_t* s) {
        J p;
        get1(s, p.x);
        get1(s + 12 * FQS, p.y);
        get1(s + 24 * FQS, p.z);
        return p;
    }
};

template <class F>
__global__ __launch_bounds__(256) void k_reduce_tree4(const uint8_t* __restrict__ V, const uint8_t* __restrict__ U,
                                                      uint32_t m_in, uint8_t* __restrict__ Vout,
                                                      uint8_t* __restrict__ Uout) {
    MBLS_TAIL_PRIO();
    using IO = RedIO<F, MODE_WAVE>;
    using J = RJac<F>;
    using T = TreeLds<F>;
    __shared__ uint32_t slot[8][T::WORDS];
    const uint32_t m_out = (m_in + 3) >> 2;
    const uint32_t seg = blockIdx.x;  // grid = m_out * windows exactly
    const uint32_t w = seg / m_out, q = seg % m_out;
    const uint32_t k0 = q << 2, cnt = min(4u, m_in - k0);
    const size_t base = (size_t)w * m_in + k0;
    const int wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    auto ldV = [&](uint32_t t) { return t < cnt ? IO::ld(V, base + t) : J::inf(); };
    auto ldU = [&](uint32_t t) { return (U && t < cnt) ? IO::ld(U, base + t) : J::inf(); };
    J r = J::inf();
    // steps 1..3 of the additions share one call site (wave-uniform operand selection)
    for (int step = 0; step < 3; ++step) {
        const bool active = step < 2 || wv == 0;
        J x = J::inf(), y = J::inf();
        if (step == 0) {
            x = wv == 0 ? ldV(2) : wv == 1 ? ldU(0) : wv == 2 ? ldU(2) : ldV(0);
            y = wv == 0 ? ldV(3) : wv == 1 ? ldU(1) : wv == 2 ? ldU(3) : ldV(1);
        } else if (step == 1) {
            x = wv == 2 ? T::get(slot[1]) : wv == 3 ? T::get(slot[3]) : T::get(slot[0]);
            y = wv == 0 ? ldV(3) : wv == 1 ? ldV(1) : wv == 2 ? T::get(slot[2]) : T::get(slot[0]);
        } else if (active) {
            x = T::get(slot[5]);  // k
            y = r;                // e
        }
        if (active) r = IO::add(x, y);
        if (step < 2) {
            T::put(slot[4 * step + wv], r);
            __syncthreads();
        }
    }
    if (wv == 0) {
        IO::st(Uout, seg, IO::add(r, T::get(slot[6])));  // U' = W + f
    } else if (wv == 3 && Vout) {
        for (int k = 0; k < 2; ++k) r = IO::dbl(r);  // V' = 4 g
        IO::st(Vout, seg, r);
    }
}

#ifndef MBLS_FINAL_QUAD
#define MBLS_FINAL_QUAD 1  // k_final_icicle's inversion on a lane quad (icicle_point_quad)
#endif
// final fold over window groups: sum_w 2^(c w) G_w  (one chain)
template <class F, int MODE>
MBLS_DEV auto final_fold(const uint8_t* __restrict__ windows, int Wg, int c) {
    using IO = RedIO<F, MODE>;
    auto acc = IO::ld(windows, Wg - 1);
    for (int w = Wg - 2; w >= 0; --w) {
        for (int k = 0; k < c; ++k) acc = IO::dbl(acc);
        acc = IO::add(acc, IO::ld(windows, w));
    }
    return acc;
}
template <class F, int MODE>
__global__ void k_final(const uint8_t* __restrict__ windows, int Wg, int c, uint8_t* __restrict__ result) {
    MBLS_TAIL_PRIO();
    using IO = RedIO<F, MODE>;
    if (IO::id() != 0) return;
    IO::st(result, 0, final_fold<F, MODE>(windows, Wg, c));
}

template <class F>
__global__ void k_store_inf(uint8_t* result, int count) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) store_jac<F>(result, i, Jacobian<F>::inf());
}

// ------------------------------------------------------------------------------------
// conversions / utilities
// ------------------------------------------------------------------------------------
MBLS_DEV Fq to_mont_f(const Fq& a) { return to_mont(a); }
MBLS_DEV Fq2 to_mont_f(const Fq2& a) { return {to_mont(a.c0), to_mont(a.c1)}; }
MBLS_DEV Fq from_mont_f(const Fq& a) { return from_mont(a); }
MBLS_DEV Fq2 from_mont_f(const Fq2& a) { return {from_mont(a.c0), from_mont(a.c1)}; }
template <class F>
MBLS_DEV F one_std();
template <>
MBLS_DEV Fq one_std<Fq>() {
    Fq r = Fq::zero();
    r.v[0] = 1;
    return r;
}
template <>
MBLS_DEV Fq2 one_std<Fq2>() {
    Fq2 r = Fq2::zero();
    r.c0.v[0] = 1;
    return r;
}

template <class F>
__global__ void k_points_to_mont(uint8_t* pts, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Affine<F> p = load_affine<F>(pts, i);
    p.x = to_mont_f(p.x);
    p.y = to_mont_f(p.y);
    store_affine<F>(pts, i, p);
}

// Jacobian Montgomery -> ICICLE standard projective (x, y, 1); identity (0, 1, 0)
// (reference icicle_curve_api.cu:134-229)
MBLS_DEV RFq from_mont_f(const RFq& a) { return from_mont(a); }
MBLS_DEV RFq2 from_mont_f(const RFq2& a) { return {from_mont(a.c0), from_mont(a.c1)}; }
template <>
MBLS_DEV RFq one_std<RFq>() {
    return {rowdpp::lane16() == 0 ? 1u : 0u};
}
template <>
MBLS_DEV RFq2 one_std<RFq2>() {
    return {one_std<RFq>(), RFq::zero()};
}

// one lane per point: the inversion is the binary extended Euclid of mbls_field.hpp (word
// shifts and adds at the full VALU rate; the row-sliced Fermat chain it replaces took 0.29 ms)
// (launched with 64 threads: the bound lets the inversion keep its words in VGPRs -- at the
// default 1024-thread bound it spilled 204 B (G1) / 912 B (G2) to scratch)
template <class F>
MBLS_DEV void icicle_point(const Jacobian<F>& p, uint8_t* out, size_t i) {
    Jacobian<F> o;
    if (p.is_inf()) {
        o.x = F::zero();
        o.y = one_std<F>();
        o.z = F::zero();
    } else {
        Affine<F> a = jac_to_affine(p);
        o.x = from_mont_f(a.x);
        o.y = from_mont_f(a.y);
        o.z = one_std<F>();
    }
    store_jac<F>(out, i, o);
}

// icicle_point on the four lanes of a DPP quad (all active, same p): the inversion runs as
// inv_quad (mbls_binv_quad.hpp); lane 0 of the quad stores
template <class F>
MBLS_DEV void icicle_point_quad(const Jacobian<F>& p, uint8_t* out, size_t i) {
    Jacobian<F> o;
    if (p.is_inf()) {
        o.x = F::zero();
        o.y = one_std<F>();
        o.z = F::zero();
    } else {
        const F zi = inv_quad(p.z);
        const F zi2 = sqr(zi);
        o.x = from_mont_f(p.x * zi2);
        o.y = from_mont_f(p.y * zi2 * zi);
        o.z = one_std<F>();
    }
    if ((__lane_id() & 3u) == 0) store_jac<F>(out, i, o);
}

// in and out may alias (in place)
template <class F>
__global__ __launch_bounds__(64) void k_jac_to_icicle(const uint8_t* in, uint8_t* out, int count) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= count) return;
    icicle_point<F>(load_jac<F>(in, i), out, i);
}

// a row-sliced value (limb j on lane j of every row) gathered into one lane's limbs
MBLS_DEV Fq row_to_lane(const RFq& a) {
    Fq r;
#pragma unroll
    for (int i = 0; i < 12; ++i) r.v[i] = (uint32_t)__shfl((int)a.v, i, 64);
    return r;
}
MBLS_DEV Fq2 row_to_lane(const RFq2& a) { return {row_to_lane(a.c0), row_to_lane(a.c1)}; }

// k_final + k_jac_to_icicle in one launch (single ICICLE MSM, result on device): the wave's
// folded point is gathered into lane 0, which normalises it and writes ICICLE's (x, y, 1)
// straight into the caller's buffer (one launch gap and the result copy fewer)
template <class F>
__global__ __launch_bounds__(64) void k_final_icicle(const uint8_t* __restrict__ windows, int Wg, int c,
                                                     uint8_t* __restrict__ out) {
    MBLS_TAIL_PRIO();
#if MBLS_HEAVY_TRACE
    const uint64_t t0 = wall_clock64();
#endif
    const RJac<F> acc = final_fold<F, MODE_WAVE>(windows, Wg, c);
    Jacobian<F> p;
    p.x = row_to_lane(acc.x);
    p.y = row_to_lane(acc.y);
    p.z = row_to_lane(acc.z);
#if MBLS_HEAVY_TRACE
    const uint64_t t1 = wall_clock64();
#endif
#if MBLS_FINAL_QUAD
    if (threadIdx.x < 4) icicle_point_quad<F>(p, out, 0);
#else
    if (threadIdx.x == 0) icicle_point<F>(p, out, 0);
#endif
#if MBLS_HEAVY_TRACE
    if (threadIdx.x == 0) printf("FIN fold=%llu inv=%llu\n", t1 - t0, wall_clock64() - t1);
#endif
}

template <class F>
__global__ void k_sum_jac(const uint8_t* pts, int count, uint8_t* out) {
    using IO = RedIO<F, MODE_WAVE>;
    if (IO::id() != 0) return;
    auto acc = RJac<F>::inf();
    for (int i = 0; i < count; ++i) acc = IO::add(acc, IO::ld(pts, i));
    IO::st(out, 0, acc);
}

template <class F>
MBLS_DEV Affine<F> generator();
template <>
MBLS_DEV Affine<Fq> generator<Fq>() { return g1_generator(); }
template <>
MBLS_DEV Affine<Fq2> generator<Fq2>() { return g2_generator(); }

MBLS_DEV uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}

// scalar i of stream `seed` (same as the oracle's gen_scalar): 4 splitmix64 words, masked to
// 255 bits, minus r once if >= r
MBLS_DEV Fr gen_scalar(uint64_t seed, uint64_t i) {
    uint64_t base = splitmix64(seed) ^ (i * 0xd1342543de82ef95ULL);
    Fr s;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint64_t l = splitmix64(base + (uint64_t)j * 0x632be59bd9b4e019ULL);
        if (j == 3) l &= 0x7fffffffffffffffULL;
        s.v[2 * j] = (uint32_t)l;
        s.v[2 * j + 1] = (uint32_t)(l >> 32);
    }
    reduce_once(s);
    return s;
}

// P_i = k_i * G (input generation only; not on the measured path)
template <class F>
__global__ void k_gen_bases(uint8_t* out, uint64_t seed, size_t start, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr k = gen_scalar(seed, start + i);
    Jacobian<F> g = Jacobian<F>::from_affine(generator<F>());
    store_affine<F>(out, i, jac_to_affine(jac_mul_u32(g, k.v)));
}

// precomputed bases, point-major as ICICLE / core/msm.rs:164-165 document:
// out[i*factor + f] = 2^(shift*f) * P_i (Montgomery affine)
template <class F>
__global__ __launch_bounds__(128) void k_precompute(const uint8_t* in, uint8_t* out, size_t n, int factor, int shift) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Affine<F> a = load_affine<F>(in, i);
    store_affine<F>(out, i * factor, a);
    Jacobian<F> p = Jacobian<F>::from_affine(a);
    for (int f = 1; f < factor; ++f) {
        for (int k = 0; k < shift; ++k) p = jac_dbl(p);
        store_affine<F>(out, i * factor + f, jac_to_affine(p));
    }
}

// ------------------------------------------------------------------------------------
// host orchestration
// ------------------------------------------------------------------------------------
template <class F>
struct GroupTraits;
template <>
struct GroupTraits<Fq> {
    static constexpr size_t AFF = 96, JAC = 144;
};
template <>
struct GroupTraits<Fq2> {
    static constexpr size_t AFF = 192, JAC = 288;
};

struct MsmScratchSizes {
    size_t dsrc, keys, vals, ranks, sorted, words, tmp, owner, first, partials, buckets, levelT, levelR, windows, phi;
    size_t ent, segtab, parts;  // partitioned sort (keys / vals / ranks are 0 then)
    size_t order, perm;         // k_bucket_order: bin histograms / their scan, bucket permutation
    size_t heavy, hslices, hres;  // HeavyTab: per-entry words (x4), per-slice owner words, slice sums
    size_t phelp;                 // PartHelp: hh + hpart (help shares the second `parts` array)
    size_t gdone = align_up(HEAVY_GDONE * 4);
    size_t total() const {
        return dsrc + keys + vals + ranks + sorted + 4 * words + tmp + owner + first + partials + buckets + levelT + levelR +
               windows + phi + ent + 2 * segtab + 2 * parts + 2 * order + perm + 4 * heavy + hslices + hres + phelp + gdone;
    }
};

// reduction levels with fewer segments than this run one segment per wave (-DMBLS_WAVE_MIN tunes;
// G2: MBLS_WAVE_MIN_G2).  An Fq2 row-sliced addition is three row products per Fq2 product in
// series, so G2 switches to the wave layout (the three spread over rows) at more segments
// (8192, with G2 row segments of 8: msm_common.hip plan_levels; 4096 measured 1.75 ms of G2
// reduction at 2^20, 8192 and 16384 1.64 ms).
// Tuning knobs in this file are compile-time macros for tools/ variant builds (never run-time
// environment reads: a prover's environment must not select untested kernels).
#ifndef MBLS_WAVE_MIN
#define MBLS_WAVE_MIN 2048u
#endif
#ifndef MBLS_WAVE_MIN_G2
#define MBLS_WAVE_MIN_G2 8192u
#endif
inline uint32_t wave_min_chains(bool fq2 = false) { return fq2 ? MBLS_WAVE_MIN_G2 : MBLS_WAVE_MIN; }

// raw XYZZ buckets for this plan (buckets_xyzz_ok, level 0 in lanes)
template <class F>
inline bool buckets_xyzz(const MsmPlan& P) {
    return buckets_xyzz_ok<F>() && P.levels > 0 && P.mode[0] == MODE_LANE;
}
#ifndef MBLS_RED_RAW_G2
#define MBLS_RED_RAW_G2 1  // G2 lane levels after level 0 take raw pair XYZZ records from the level before
#endif
// a level output record's bytes: raw pair XYZZ (448) when G2 chains lane levels, else Jacobian
template <class F>
inline size_t level_bytes(const MsmPlan& P, size_t jac) {
    return (std::is_same<F, Fq2>::value && MBLS_RED_RAW_G2 && buckets_xyzz<F>(P) && P.levels > 1 &&
            P.mode[1] == MODE_LANE)
               ? xyzz_bucket_bytes<F>()
               : jac;
}
// bkt: a bucket sum's bytes (jac, or 224 for raw XYZZ buckets)
inline MsmScratchSizes msm_scratch_sizes(const MsmPlan& P, size_t jac, size_t aff, uint32_t max_chunks, size_t part,
                                         size_t bkt, size_t lvl) {
    MsmScratchSizes z;
    // the per-call image table; with bstride > 1 also the compact copy of the points (2n rows)
    z.phi = P.split > 1 && !P.prepared ? align_up(P.pts / P.split * (P.split - 1 + (P.bstride > 1 ? 1 : 0)) * aff) : 0;
    const size_t NC = P.contributions;
    if (partition_sort(P)) {
        const PartSortSizes s = part_sort_sizes(P);
        z.keys = z.vals = z.ranks = 0;
        z.ent = align_up(s.ent);
        z.segtab = align_up(s.segtab);
        z.parts = align_up(s.parts);
        z.phelp = align_up((size_t)PH_HELPERS * 129 * 4);
    } else {
        z.phelp = 0;
        z.keys = align_up(NC * 4);
        z.vals = align_up(NC * 4);
        z.ranks = align_up(NC * 4);
        z.ent = z.segtab = z.parts = 0;
    }
    z.dsrc = align_up(digits_src_bytes((uint32_t)(P.split > 1 ? P.pts / P.split : P.pts / P.F), P.split));
    z.sorted = align_up(NC * 4);
    z.words = align_up(((size_t)P.TB + 4) * 4);  // + the maximum and the HeavyTab counters
    // heavy buckets have > SMALL_MAX partials: at most max_chunks / (SMALL_MAX + 1) of them, and
    // at most max_chunks / HEAVY_SLICE + (heavy buckets) slices
    const size_t max_heavy = std::min<size_t>(P.TB, max_chunks / (SMALL_MAX + 1) + 1);
    const size_t max_slices = max_chunks / HEAVY_SLICE + max_heavy + 1;
    z.heavy = align_up(max_heavy * 4);
    z.hslices = align_up(max_slices * 4);
    // slice sums: the planned slices (>= HEAVY_SLICE_MIN partials, <= HEAVY_LDS buckets) or the
    // fixed plan's
    z.hres = align_up(std::max(max_slices, max_chunks / HEAVY_SLICE_MIN + std::min<size_t>(max_heavy, HEAVY_LDS) + 1) * jac);
    z.order = align_up(((size_t)order_words(P.TB) + 1) * 4);
    z.perm = align_up((size_t)P.TB * 4);
    // + the chunk-count block totals and their prefixes (k_chunk_counts / k_scan_small)
    z.tmp = align_up((scan_tmp_words(std::max(std::max(max_chunks, P.TB), order_words(P.TB))) +
                      2 * ((size_t)P.TB / 128 + 2)) *
                     4);
    z.owner = align_up((size_t)max_chunks * 4);
    z.first = align_up((NC / P.chunk + 2) * 4);
    z.partials = align_up((size_t)max_chunks * part);  // part: a chunk partial's bytes (PartialBytes)
    z.buckets = align_up((size_t)P.TB * bkt);
    // V / U ping-pong halves sized for the widest level's outputs (k_reduce_scaled)
    const size_t mo0 = P.levels ? (P.level_m[0] + P.seg(0) - 1) / P.seg(0) : 1;
    z.levelT = align_up(2 * mo0 * P.Wg * lvl);  // lvl: a level record's bytes (level_bytes)
    z.levelR = align_up(2 * mo0 * P.Wg * lvl);
    z.windows = align_up((size_t)P.Wg * jac);
    return z;
}

inline bool debug_enabled() {
    static const bool v = [] {
        const char* e = getenv("MBLS_DEBUG");
        return e && atoi(e) != 0;
    }();
    return v;
}

// the accumulation kernel instance: G1 at <= 168 VGPRs (3 waves per SIMD; -DMBLS_ACC_W3=0: 1)
#ifndef MBLS_ACC_W3
#define MBLS_ACC_W3 1
#endif
using AccKernel = void (*)(const uint32_t*, const uint32_t*, const uint32_t*, const uint32_t*, uint32_t, uint32_t,
                           const uint8_t*, const uint8_t*, uint32_t, uint32_t, uint8_t*);
template <class F>
inline AccKernel accumulate_kernel() {
    if constexpr (std::is_same<F, Fq>::value && MBLS_ACC_R28 && MBLS_ACC_LDS) return k_accumulate_r28<F>;
    else if constexpr (std::is_same<F, Fq2>::value && MBLS_ACC_G2_R28) return k_accumulate_r28p<F>;
    else if constexpr (std::is_same<F, Fq>::value && MBLS_ACC_W3) return k_accumulate<F, 3>;
    else return k_accumulate<F, 1>;
}

// contributions per accumulation thread: CHUNK (16), or an eighth of the average bucket when
// buckets are bigger (2^24 points: 1024 contributions per bucket, chunk 128), so a bucket keeps
// <= ~9 partials and its sum stays on the one-thread-per-bucket path (k_bucket_small) -- with
// 16-point chunks every bucket at 2^24 had 64 partials, took the heavy-bucket tree passes and
// the bucket sums cost 93.5 ms against 50.6 ms of accumulation.  Short chunks pay off below
// that: a chunk's first addition is free when the whole wave starts a chunk together (acc = P,
// counter-checked: SQ_INSTS_VALU +5.2% at 86 instead of 16 at 2^20), and spreading NC over one
// round of resident waves (MBLS_ACC_CHUNK=auto, 86 at G1 2^20) cut the bucket sums 0.61 ->
// 0.19 ms but cost 3.25 -> 3.66 ms in the accumulation.
// -DMBLS_ACC_CHUNK=<n> fixes it (variant builds).
#ifndef MBLS_ACC_CHUNK
#define MBLS_ACC_CHUNK 0
#endif
template <class F>
inline uint32_t accumulate_chunk(const MsmPlan& P) {
    if (MBLS_ACC_CHUNK > 0) return (uint32_t)MBLS_ACC_CHUNK;
    const size_t per_bucket = P.contributions / std::max<uint32_t>(P.TB, 1u);
    return (uint32_t)std::max<size_t>(CHUNK, per_bucket / 8);
}

// batch_size > 1: member b's reduction and final fold on a side stream beside member b + 1's
// front and accumulation (TailPipe); 2: member b + 1's front on a second side stream beside member
// b's accumulation as well; 0: every member on the caller's stream (-DMBLS_BATCH_PIPE)
#ifndef MBLS_BATCH_PIPE
#define MBLS_BATCH_PIPE 2
#endif
inline int batch_pipe() { return MBLS_BATCH_PIPE; }

// wave-layout levels of 4-input segments with at most this many segments run as trees of 4
// waves (k_reduce_tree4; -DMBLS_TREE_MAX tunes, 0 disables)
#ifndef MBLS_TREE_MAX
#define MBLS_TREE_MAX 512u
#endif
inline uint32_t tree_max_chains() { return MBLS_TREE_MAX; }

// one reduction level over Wl windows (weights t + off; off = 1 at level 0: bucket t holds digit t + 1)
template <class F>
inline void launch_reduce_scaled(int mode, const uint8_t* V, const uint8_t* U, uint32_t m_in, uint32_t seg_log, int Wl,
                                 int off, uint8_t* Vo, uint8_t* Uo, uint32_t chains, hipStream_t s) {
    constexpr uint32_t LN = LaneOf<F>::LANES;
    if (mode == MODE_WAVE && seg_log == 2 && off == 0 && chains <= tree_max_chains()) {
        hipLaunchKernelGGL(k_reduce_tree4<F>, dim3(chains), dim3(256), 0, s, V, U, m_in, Vo, Uo);
        return;
    }
    if (mode == MODE_LANE && std::is_same<F, Fq>::value && MBLS_RED_R28)
        hipLaunchKernelGGL((k_reduce_scaled_r28<F>), dim3((chains + 255) / 256), dim3(256), 0, s, V, U, m_in, seg_log, Wl,
                           off, Vo, Uo);
    else if (mode == MODE_LANE)
        hipLaunchKernelGGL((k_reduce_scaled<F, MODE_LANE>), dim3((chains * LN + 255) / 256), dim3(256), 0, s, V, U, m_in,
                           seg_log, Wl, off, Vo, Uo);
    else if (mode == MODE_ROW)
        hipLaunchKernelGGL((k_reduce_scaled<F, MODE_ROW>), dim3((chains * 16 + 255) / 256), dim3(256), 0, s, V, U, m_in,
                           seg_log, Wl, off, Vo, Uo);
    else
        hipLaunchKernelGGL((k_reduce_scaled<F, MODE_WAVE>), dim3((chains * 64 + 255) / 256), dim3(256), 0, s, V, U, m_in,
                           seg_log, Wl, off, Vo, Uo);
}

// Batch tail pipeline (msm_call, batch_size > 1): member b's reduction levels and final fold --
// latency-bound chains that leave most of the GPU idle -- run on a side stream while member
// b + 1's front and accumulation run on the caller's stream.  The tail reads only the bucket
// sums, the level buffers and the window sums of its member's scratch region (two regions,
// alternating), so the main stream waits for member b - 2's tail (`reuse`) only before it
// writes that region's bucket sums again.
// The front (digits, sort, chunk tables) of member b likewise runs on a second side stream
// beside member b - 1's accumulation: it writes only its own region's front buffers, which member
// b - 2's accumulation and bucket sums read (`front_wait`: that member's bucket_done, or for the
// first two members the fork from the caller's stream).
struct TailPipe {
    hipStream_t side = nullptr;        // the tails run here
    hipEvent_t bucket_done = nullptr;  // recorded on the main stream after the bucket sums
    hipEvent_t reuse = nullptr;        // non-null: the region's previous tail; waited before the bucket sums
    hipStream_t front = nullptr;       // non-null: the front runs here
    hipEvent_t front_wait = nullptr;   // waited on `front` before the member's front
    hipEvent_t front_done = nullptr;   // recorded on `front` after it; the main stream waits on it
};

// Core MSM on device operands: scalars (standard or Montgomery), bases Montgomery affine
// (F*n entries when precomputed); result: one Jacobian Montgomery point on device, or, with
// icicle_out, ICICLE's normalised (x, y, 1) written there by the final fold's launch.
// Everything is enqueued on `st`; side streams of the leased context are forked from it and
// joined back, so the caller sees one stream-ordered operation -- except with `pipe`, where the
// reduction and the final fold are left on pipe->side for the caller to join.
template <class F>
eIcicleError msm_device(const uint8_t* scalars, bool scalars_mont, const uint8_t* bases, uint32_t n,
                        const MsmPlan& P, uint8_t* result, StreamCtx& ctx, hipStream_t st,
                        uint8_t* icicle_out = nullptr, const TailPipe* pipe = nullptr,
                        hipEvent_t acc_event = nullptr) {
    Arena& arena = ctx.arena;
    constexpr size_t JAC = GroupTraits<F>::JAC, AFF = GroupTraits<F>::AFF;
    constexpr uint32_t LN = LaneOf<F>::LANES;  // lanes per chain in the lane-mode kernels
    // mbls_msm_accumulate_event: recorded after the accumulation launch below, or wherever this
    // function returns before it (an empty MSM, an error)
    AccEventGuard acc_ev(acc_event, st);
    if (n == 0) {
        hipLaunchKernelGGL(k_store_inf<F>, dim3(1), dim3(64), 0, st, result, 1);
        if (icicle_out) hipLaunchKernelGGL(k_jac_to_icicle<F>, dim3(1), dim3(64), 0, st, result, icicle_out, 1);
        MBLS_TRY(hipGetLastError());
        return MBLS_SUCCESS;
    }
    const uint32_t TB = P.TB;
    const size_t NC = P.contributions;
    const uint32_t max_chunks = (uint32_t)(NC / P.chunk + TB + 1);
    const bool xb = buckets_xyzz<F>(P);
    MsmScratchSizes z =
        msm_scratch_sizes(P, JAC, AFF, max_chunks, PartialBytes<F>::value, xb ? xyzz_bucket_bytes<F>() : JAC,
                          level_bytes<F>(P, JAC));
    uint32_t* keys = (uint32_t*)arena.take(z.keys);
    uint32_t* vals = (uint32_t*)arena.take(z.vals);
    uint32_t* ranks = (uint32_t*)arena.take(z.ranks);
    uint8_t* dsrc = (uint8_t*)arena.take(z.dsrc);
    uint32_t* sorted = (uint32_t*)arena.take(z.sorted);
    uint32_t* counts = (uint32_t*)arena.take(z.words);
    uint32_t* offsets = (uint32_t*)arena.take(z.words);
    uint32_t* nchunks = (uint32_t*)arena.take(z.words);
    uint32_t* chunk_off = (uint32_t*)arena.take(z.words);
    uint32_t* tmp = (uint32_t*)arena.take(z.tmp);
    uint32_t* owner = (uint32_t*)arena.take(z.owner);
    uint32_t* first = (uint32_t*)arena.take(z.first);
    uint8_t* partials = (uint8_t*)arena.take(z.partials);
    uint8_t* buckets = (uint8_t*)arena.take(z.buckets);
    uint8_t* levelT = (uint8_t*)arena.take(z.levelT);
    uint8_t* levelR = (uint8_t*)arena.take(z.levelR);
    uint8_t* windows = (uint8_t*)arena.take(z.windows);
    const bool img_table = P.split > 1 && !P.prepared;  // the images are built per call
    uint8_t* phi = img_table ? (uint8_t*)arena.take(z.phi) : nullptr;
    const bool psort = partition_sort(P);
    uint32_t* ent = (uint32_t*)arena.take(z.ent);
    uint32_t* seg_off = (uint32_t*)arena.take(z.segtab);
    uint32_t* seg_cnt = (uint32_t*)arena.take(z.segtab);
    uint32_t* part_tot = (uint32_t*)arena.take(z.parts);
    PartHelp ph;
    ph.help = (uint32_t*)arena.take(z.parts);
    ph.hh = (uint32_t*)arena.take(z.phelp);
    ph.hpart = ph.hh ? ph.hh + (size_t)PH_HELPERS * 128 : nullptr;
    uint32_t* binhist = (uint32_t*)arena.take(z.order);
    uint32_t* binbase = (uint32_t*)arena.take(z.order);
    uint32_t* perm = (uint32_t*)arena.take(z.perm);
    HeavyTab H;
    H.bucket = (uint32_t*)arena.take(z.heavy);
    H.first = (uint32_t*)arena.take(z.heavy);
    H.nslices = (uint32_t*)arena.take(z.heavy);
    H.done = (uint32_t*)arena.take(z.heavy);
    H.owner = (uint32_t*)arena.take(z.hslices);
    H.res = (uint8_t*)arena.take(z.hres);
    H.gdone = (uint32_t*)arena.take(z.gdone);
    H.cnt = nchunks + TB + 1;
    if (!H.gdone || !H.res || !windows || (img_table && !phi) || (psort && !ph.hh)) return MBLS_ALLOCATION_FAILED;

    ProfScope prof_all("msm.total", st);
    eIcicleError er;
    // the front's stream: the caller's, or the batch pipeline's front stream
    const hipStream_t main_st = st;
    if (pipe && pipe->front) {
        if (pipe->front_wait) MBLS_TRY(hipStreamWaitEvent(pipe->front, pipe->front_wait, 0));
        st = pipe->front;
    }
    // side stream: the endomorphism table overlaps the digit / sort front (fork ev[0], join ev[1])
    if ((er = ctx.ensure_side(2, 1)) != MBLS_SUCCESS) return er;
    hipStream_t side = ctx.sides[0];
    hipEvent_t* ev = ctx.events.data();
    // with the partitioned sort the endomorphism table is written by the split kernel
    // (k_glv_prep / k_psi_prep); the tiled sort (c > 16) builds it on the side stream
    const bool fused_table = img_table && psort;
    if (img_table && !fused_table) {  // endomorphism images of the bases: phi(P) (G1) or psi^1..3(P) (G2)
        ctx.forked = true;
        MBLS_TRY(hipEventRecord(ev[0], st));
        MBLS_TRY(hipStreamWaitEvent(side, ev[0], 0));
        er = P.split == 2 ? launch_glv_table(bases, phi, n, side) : launch_psi_table(bases, phi, n, side);
        if (er != MBLS_SUCCESS) return er;
        MBLS_TRY(hipEventRecord(ev[1], side));
    }
    // the partition sort of 128-bucket parts also computes the chunk counts (k_chunk_counts'
    // outputs, prefixes in 128-bucket blocks): one launch fewer
    const bool fused_cc = psort && part_sort_fuses_chunks(P);
    const int cs = fused_cc ? CHUNK_FUSED_SHIFT : 8;
    {
        ProfScope ps("msm.digits", st);
        if (psort) {
            er = launch_digits_part(scalars, scalars_mont, n, P, ent, seg_off, seg_cnt, part_tot, dsrc, nchunks + TB, st,
                                    fused_table ? bases : nullptr, fused_table ? phi : nullptr,
                                    fused_cc ? binhist : nullptr, fused_cc ? order_words(TB) : 0u);
        } else {
            MBLS_TRY(hipMemsetAsync(counts, 0, (size_t)TB * 4, st));
            er = launch_digits(scalars, scalars_mont, n, P, keys, vals, ranks, counts, dsrc, st);
        }
        if (er != MBLS_SUCCESS) return er;
    }
    {
        ProfScope ps("msm.sort", st);
        // chunk_off = exclusive scan of the chunk counts, spread over the kernels below: block
        // prefixes in k_chunk_counts or k_part_sort (written over `counts`, no longer needed), the
        // block totals scanned beside the order histograms, the sum in k_chunk_owner
        uint32_t* cloc = counts;
        const uint32_t nblk = (TB + (1u << cs) - 1) >> cs;
        uint32_t* blk_tot = tmp;
        uint32_t* blk_pre = tmp + (nblk + 2);
        if (psort) {  // writes counts (or with fused_cc the chunk counts), offsets (incl. offsets[TB]) and sorted
            ChunkCountOut cc;
            if (fused_cc) {
                cc.nchunks = nchunks;
                cc.binhist = binhist;
                cc.blk_tot = blk_tot;
                cc.L = P.chunk;
                cc.m = TB;
            }
            er = launch_part_sort(P, ent, seg_off, seg_cnt, part_tot, counts, offsets, sorted, cc, st, ph);
            if (er != MBLS_SUCCESS) return er;
        } else if ((er = scan_exclusive(counts, offsets, TB, tmp, st)) != MBLS_SUCCESS) {
            return er;
        }
        if (!fused_cc &&
            (er = launch_chunk_counts(counts, offsets, nchunks, TB, P.chunk, binhist, 1u, psort, cloc, blk_tot, st)) !=
                MBLS_SUCCESS)
            return er;
        if ((er = launch_order_scan(binhist, binbase, TB, blk_tot, blk_pre, nblk, st)) != MBLS_SUCCESS) return er;
        if (!psort && (er = launch_scatter(keys, vals, ranks, NC, offsets, sorted, st)) != MBLS_SUCCESS) return er;
        if ((er = launch_chunk_owner(cloc, blk_pre, cs, chunk_off, offsets, TB, P.chunk, owner, first, nchunks, binbase,
                                     perm, H, st)) != MBLS_SUCCESS)
            return er;
    }
    if (st != main_st) {  // join: the accumulation waits for the front
        MBLS_TRY(hipEventRecord(pipe->front_done, st));
        st = main_st;
        MBLS_TRY(hipStreamWaitEvent(st, pipe->front_done, 0));
    }
    const uint32_t nsplit = img_table ? n : 0xffffffffu;
    {
        // the chunk count is data dependent: launch the bound, extra threads exit
        ProfScope ps("msm.accumulate", st);
        if (img_table && !fused_table) MBLS_TRY(hipStreamWaitEvent(st, ev[1], 0));
        const uint32_t threads = (uint32_t)((NC + P.chunk - 1) / P.chunk) * LN;
        // bstride > 1: the split kernel wrote [P; phi P] into `phi` (compact slot-0 copy)
        const uint8_t* acc_b = P.bstride > 1 ? phi : bases;
        const uint8_t* acc_phi = P.bstride > 1 ? phi + (size_t)n * AFF : phi;
        hipLaunchKernelGGL(accumulate_kernel<F>(), dim3((threads + 255) / 256), dim3(256), 0, st, sorted, offsets,
                           chunk_off, first, 0u, TB, acc_b, acc_phi, nsplit, P.chunk, partials);
    }
    // mbls_msm_accumulate_event: the tail starts here (the caller passes it to the last member)
    if (hipEvent_t e = acc_ev.release()) MBLS_TRY(hipEventRecord(e, st));
    {
        ProfScope ps("msm.bucket_sum", st);
        // light buckets one thread each, heavy buckets by slice workgroups in the same launch
        // (k_bucket_small); forked heavy passes on a side stream cost ~20 us per event wait,
        // in-line empty passes ~6 us per launch (round 3 timelines)
        const uint32_t light_blocks = (TB * LN + 255) / 256;
        if (pipe && pipe->reuse) MBLS_TRY(hipStreamWaitEvent(st, pipe->reuse, 0));
        hipLaunchKernelGGL(k_bucket_small<F>, dim3(light_blocks + HEAVY_BLOCKS), dim3(256), 0, st, chunk_off, perm, binbase,
                           order_words(TB), partials, buckets, light_blocks, H, xb ? 1 : 0);
    }
    if (pipe) {  // the tail moves to the side stream
        MBLS_TRY(hipEventRecord(pipe->bucket_done, st));
        MBLS_TRY(hipStreamWaitEvent(pipe->side, pipe->bucket_done, 0));
        st = pipe->side;
    }
    {
        ProfScope ps_red("msm.reduce", st);  // the levels only (k_final has its own scope)
        // scaled running-sum levels (k_reduce_scaled): V / U ping-pong in levelR / levelT, the
        // last level writes the window sums straight into `windows`
        const size_t half = ((P.level_m[0] + P.seg(0) - 1) / P.seg(0)) * (size_t)P.Wg * level_bytes<F>(P, JAC);
        uint8_t* vb[2] = {levelR, levelR + half};
        uint8_t* ub[2] = {levelT, levelT + half};
        const uint8_t* V = buckets;
        const uint8_t* U = nullptr;
        bool raw_in = xb;  // level l's inputs are raw XYZZ records
        for (int l = 0; l < P.levels; ++l) {
            const uint32_t m_in = P.level_m[l];
            const uint32_t m_out = (m_in + P.seg(l) - 1) / P.seg(l);
            const bool last = l == P.levels - 1;
            uint8_t* Vo = last ? nullptr : vb[l & 1];
            uint8_t* Uo = last ? windows : ub[l & 1];
            bool done = false;
            if constexpr (buckets_xyzz_ok<F>()) {
                if (raw_in) {  // a lane level (level 0, or G2's lane levels after it)
                    const uint32_t chains = m_out * (uint32_t)P.Wg;
                    if constexpr (std::is_same<F, Fq>::value) {
                        hipLaunchKernelGGL((k_reduce_scaled_r28x<F>), dim3((chains + 255) / 256), dim3(256), 0, st, V,
                                           m_in, P.seg_log[0], P.Wg, 1, Vo, Uo);
                        raw_in = false;
                    } else {
                        const bool raw_out = MBLS_RED_RAW_G2 && !last && P.mode[l + 1] == MODE_LANE;
                        hipLaunchKernelGGL((k_reduce_scaled_r28px<F>), dim3((2 * chains + 255) / 256), dim3(256), 0, st,
                                           V, U, m_in, P.seg_log[l], P.Wg, l == 0 ? 1 : 0, Vo, Uo, raw_out ? 1 : 0);
                        raw_in = raw_out;
                    }
                    done = true;
                }
            }
            if (!done)
                launch_reduce_scaled<F>(P.mode[l], V, U, m_in, P.seg_log[l], P.Wg, l == 0 ? 1 : 0, Vo, Uo,
                                        m_out * (uint32_t)P.Wg, st);
            V = Vo;
            U = Uo;
        }
    }
    {
        ProfScope ps("msm.final", st);
        if (icicle_out)
            hipLaunchKernelGGL(k_final_icicle<F>, dim3(1), dim3(64), 0, st, windows, P.Wg, P.c, icicle_out);
        else
            hipLaunchKernelGGL((k_final<F, MODE_WAVE>), dim3(1), dim3(64), 0, st, windows, P.Wg, P.c, result);
    }
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// ------------------------------------------------------------------------------------
// boundary wrappers (placement flags, Montgomery flags, batch, ICICLE result format)
// ------------------------------------------------------------------------------------
// entry-point semantics: RAW = the reference's bls12_381_g*_msm_cuda (standard scalars,
// Montgomery bases, flags for placement only, Jacobian Montgomery result, one MSM); ICICLE =
// msm_cuda_impl (Montgomery flags honoured, batch, (x, y, 1) standard result); JACOBIAN = ICICLE
// inputs with the Jacobian Montgomery result left unnormalised (the per-rank step of the
// sharded multi-GPU MSM: partials are summed before the one normalisation)
enum MsmEntry : int { MSM_RAW = 0, MSM_ICICLE = 1, MSM_JACOBIAN = 2 };

#ifndef MBLS_PINNED_ZERO_COPY
#define MBLS_PINNED_ZERO_COPY 1  // variant builds: 0 = always stage host scalars
#endif
template <class F>
eIcicleError msm_call(const void* scalars, const void* bases, int msm_size, const MSMConfig* cfg, void* results,
                      int entry) {
    const bool icicle_semantics = entry != MSM_RAW;
    constexpr size_t AFF = GroupTraits<F>::AFF, JAC = GroupTraits<F>::JAC;
    if (!cfg || !results) return MBLS_INVALID_POINTER;
    hipStream_t st = static_cast<hipStream_t>(cfg->stream);
    // a pending mbls_msm_accumulate_event belongs to this call whatever happens below: the last
    // member's accumulation records it (msm_device), any earlier return records it here
    AccEventGuard acc_ev(take_accumulate_event(st), st);
    if (msm_size < 0 || msm_size > (1 << MAX_MSM_LOG)) return MBLS_INVALID_ARGUMENT;
    if (msm_size > 0 && (!scalars || !bases)) return MBLS_INVALID_POINTER;
    const int batch = icicle_semantics ? (cfg->batch_size > 0 ? cfg->batch_size : 1) : 1;
    // The reference's plain device-bases MSMs (core/msm.rs:897-913, 1025-1040, 1097-1110) set
    // cfg.precompute_factor = MIDNIGHT_GPU_PRECOMPUTE on a buffer of n plain bases; its backend
    // never reads the factor.  A device allocation too short for n x F table entries cannot be a
    // precompute_bases table: it runs as factor 1, the reference's result (the
    // binding should pass PrecomputedBases::factor()).
    // Strict mode (mbls_msm_precompute_strict(1), for a binding that cannot pass the table's own
    // factor): only a table precompute_bases wrote (registered, same factor, covering the call)
    // runs as a table; anything else is plain bases -- exact for sub-allocated buffers too.
    MSMConfig cfg_plain;
    if (cfg->precompute_factor > 1 && cfg->are_points_on_device && bases && msm_size > 0) {
        const bool sh = cfg->are_points_shared_in_batch || batch == 1;
        const size_t want = (size_t)msm_size * (size_t)cfg->precompute_factor * (sh ? 1 : (size_t)batch) *
                            GroupTraits<F>::AFF;
        if (precompute_strict() ? !precompute_is_table(bases, cfg->precompute_factor, want)
                                : device_bytes_from(bases) < want) {
            cfg_plain = *cfg;
            cfg_plain.precompute_factor = 1;
            cfg = &cfg_plain;
        }
    }
    MsmPlan P;
    eIcicleError er = make_plan(msm_size > 0 ? msm_size : 1, cfg, P, std::is_same<F, Fq>::value ? 2 : 4);
    if (er != MBLS_SUCCESS) return er;
    const bool scal_mont = icicle_semantics ? cfg->are_scalars_montgomery_form : false;
    // a precomputed table (F > 1) is precompute_call output, Montgomery whatever the flag says:
    // core/msm.rs:641-643 passes are_bases_montgomery_form = !is_precomputed() = false with it
    const bool pts_mont = icicle_semantics && P.table == 1 ? cfg->are_points_montgomery_form : true;
    const bool shared = cfg->are_points_shared_in_batch || batch == 1;
    const size_t n = (size_t)msm_size;
    const size_t nbases_per = n * (size_t)P.table;
    const size_t nbases = shared ? nbases_per : nbases_per * batch;

    CtxLease lease(st);
    if (!lease) return lease.error();
    StreamCtx& ctx = *lease;
    Arena& A = ctx.arena;
    size_t st_s = (!cfg->are_scalars_on_device) ? align_up(n * 32 * batch) : 0;
    size_t st_b = (!cfg->are_points_on_device || !pts_mont) ? align_up(nbases * AFF) : 0;
    size_t st_r = align_up(JAC * (size_t)batch);
    P.chunk = accumulate_chunk<F>(P);
    if (debug_enabled())
        fprintf(stderr, "[mbls] msm n=%d c=%d W=%d Wg=%d split=%d TB=%u contributions=%zu chunk=%u levels=%d\n", msm_size,
                P.c, P.W, P.Wg, P.split, P.TB, P.contributions, P.chunk, P.levels);
    uint32_t max_chunks = (uint32_t)(P.contributions / P.chunk + P.TB + 1);
    size_t scratch =
        msm_scratch_sizes(P, JAC, AFF, max_chunks, PartialBytes<F>::value,
                          buckets_xyzz<F>(P) ? xyzz_bucket_bytes<F>() : JAC, level_bytes<F>(P, JAC))
            .total();
    const bool piped = batch > 1 && batch_pipe() > 0;
    er = lease.reserve(st_s + st_b + st_r + scratch * (piped ? 2 : 1) + 4096);
    if (er != MBLS_SUCCESS) return er;

    const uint8_t* d_s = static_cast<const uint8_t*>(scalars);
    const uint8_t* d_b = static_cast<const uint8_t*>(bases);
    if (st_s) {
        // host scalars (core/msm.rs:665,773 pass a HostSlice): stream-ordered; a pageable buffer is
        // out of the caller's memory when hipMemcpyAsync returns, a pinned one is the caller's to
        // keep alive until the stream completes (as in ICICLE).
        // Pinned memory whose first kernel reads each scalar exactly once (the GLV / psi split, or
        // the Montgomery -> standard conversion) is read in place over PCIe through its device
        // alias: the front kernel overlaps the transfer with its own work and no 32 MiB staging
        // copy is written and re-read.  Otherwise: a PCIe copy kernel (pinned)
        // or hipMemcpyAsync (pageable, or another device's memory for multi-device shards).
        const bool read_once = P.split > 1 || scal_mont;
        const void* alias = read_once && MBLS_PINNED_ZERO_COPY ? pinned_host_device_pointer(scalars) : nullptr;
        if (alias) {
            d_s = static_cast<const uint8_t*>(alias);
        } else {
            void* t = A.take(n * 32 * batch);
            if ((er = stage_to_device(t, scalars, n * 32 * batch, st)) != MBLS_SUCCESS) return er;
            d_s = static_cast<const uint8_t*>(t);
        }
    }
    if (st_b) {
        void* t = A.take(nbases * AFF);
        if (cfg->are_points_on_device) {
            MBLS_TRY(hipMemcpyAsync(t, bases, nbases * AFF, hipMemcpyDefault, st));
        } else if ((er = stage_to_device(t, bases, nbases * AFF, st)) != MBLS_SUCCESS) {
            return er;
        }
        if (!pts_mont) {
            hipLaunchKernelGGL(k_points_to_mont<F>, dim3((unsigned)((nbases + 255) / 256)), dim3(256), 0, st,
                               (uint8_t*)t, nbases);
            MBLS_TRY(hipGetLastError());
        }
        d_b = static_cast<const uint8_t*>(t);
    }
    uint8_t* d_r = static_cast<uint8_t*>(A.take(JAC * (size_t)batch));
    // one ICICLE MSM with its result on the device: the final fold writes the normalised
    // (x, y, 1) straight into `results` (k_final_icicle; 16-byte stores, so aligned buffers only)
    uint8_t* direct = (entry == MSM_ICICLE && batch == 1 && cfg->are_results_on_device &&
                       ((uintptr_t)results & 15) == 0)
                          ? (uint8_t*)results
                          : nullptr;
    const size_t mark = A.mark();
    // events: 2-3 bucket_done, 4-5 tail done, 6-7 front done, 8 the fork (per region where paired)
    if (piped && (er = ctx.ensure_side(9, 3)) != MBLS_SUCCESS) return er;
    if (piped) {
        ctx.forked = true;
        MBLS_TRY(hipEventRecord(ctx.events[8], st));
    }
    for (int b = 0; b < batch; ++b) {
        // scratch reused across the batch (stream-ordered); piped: two regions, alternating
        A.rewind(mark);
        TailPipe pipe;
        if (piped) {
            if ((b & 1) && !A.take(scratch)) return MBLS_ALLOCATION_FAILED;
            pipe.side = ctx.sides[1];
            pipe.bucket_done = ctx.events[2 + (b & 1)];
            pipe.reuse = b >= 2 ? ctx.events[4 + (b & 1)] : nullptr;
            pipe.front = batch_pipe() > 1 ? ctx.sides[2] : nullptr;
            pipe.front_wait = b >= 2 ? ctx.events[2 + (b & 1)] : ctx.events[8];
            pipe.front_done = ctx.events[6 + (b & 1)];
        }
        const uint8_t* sb = d_s + (size_t)b * n * 32;
        const uint8_t* bb = d_b + (shared ? 0 : (size_t)b * nbases_per * AFF);
        // piped ICICLE members are normalised inside their tails (hidden but for the last one)
        uint8_t* icicle_b = direct ? direct : (piped && entry == MSM_ICICLE ? d_r + (size_t)b * JAC : nullptr);
        er = msm_device<F>(sb, scal_mont, bb, (uint32_t)n, P, d_r + (size_t)b * JAC, ctx, st, icicle_b,
                           piped ? &pipe : nullptr, b == batch - 1 ? acc_ev.release() : nullptr);
        if (er != MBLS_SUCCESS) return er;
        if (piped) MBLS_TRY(hipEventRecord(ctx.events[4 + (b & 1)], pipe.side));
    }
    // the side stream runs the tails in member order: its last event covers them all
    if (piped) MBLS_TRY(hipStreamWaitEvent(st, ctx.events[4 + ((batch - 1) & 1)], 0));
    // every side stream is joined into `st` by now (the table's ev[1] before the accumulation,
    // the fronts' front_done, the tails' last event above): only an early error return leaves
    // the lease's fallback join to do
    ctx.forked = false;
    if (!direct) {
        if (entry == MSM_ICICLE && !piped) {
            hipLaunchKernelGGL(k_jac_to_icicle<F>, dim3((batch + 63) / 64), dim3(64), 0, st, d_r, d_r, batch);
            MBLS_TRY(hipGetLastError());
        }
        MBLS_TRY(hipMemcpyAsync(results, d_r, JAC * (size_t)batch,
                                cfg->are_results_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, st));
    }
    MBLS_TRY(hipGetLastError());
    // is_async is honoured whatever the input placement (staged inputs live in the leased
    // context, which later calls only reuse after this call's `done` event); a host result needs
    // the wait
    if (!cfg->is_async || !cfg->are_results_on_device) MBLS_TRY(hipStreamSynchronize(st));
    return MBLS_SUCCESS;
}

// ------------------------------------------------------------------------------------
// multi-device MSM for a single-process caller (mbls_g*_msm_multi_device): SURVEY.md 8e's
// shard -> partial -> exchange -> EC sum -> one normalisation, with the exchange as peer copies
// of the 144 / 288-byte Jacobian partials to the first device (RCCL's reduce ops cannot add
// curve points; the torch.distributed path of bench.py / sharded_msm.py all-gathers them).
// ------------------------------------------------------------------------------------
static constexpr int MAX_SHARDS = 64;
struct MultiDevRes {  // per device, created once, used under the multi-device lock
    hipStream_t stream = nullptr;
    hipEvent_t ev[MAX_SHARDS] = {};
    uint8_t* partials = nullptr;  // MAX_SHARDS Jacobian partials (G2 size)
    uint8_t* gather = nullptr;    // (first device) MAX_SHARDS gathered partials + the sum
    hipEvent_t done = nullptr;    // (first device) recorded on the call's first stream at its end
};
std::mutex& multi_device_mutex();
// the first device's resources of the last call (its `done` orders the next call's reuse of the
// partial / gather slots, whatever streams the two calls use); under the multi-device lock
MultiDevRes*& multi_device_last();
eIcicleError multi_device_res(int dev, MultiDevRes*& out);
eIcicleError enable_peer(int from, int to);

template <class F>
eIcicleError msm_multi_device(const void* scalars, const void* const* bases_per_dev, const int* devs, int ndev,
                              int msm_size, const MSMConfig* cfg, void* result) {
    constexpr size_t JAC = GroupTraits<F>::JAC;
    if (!cfg || !result || !devs || !bases_per_dev) return MBLS_INVALID_POINTER;
    if (ndev < 1 || ndev > MAX_SHARDS || msm_size < 0 || msm_size > (1 << MAX_MSM_LOG)) return MBLS_INVALID_ARGUMENT;
    if (cfg->batch_size > 1 || cfg->precompute_factor > 1) return MBLS_INVALID_ARGUMENT;
    if (msm_size > 0 && !scalars) return MBLS_INVALID_POINTER;
    int count = 0;
    MBLS_TRY(hipGetDeviceCount(&count));
    for (int k = 0; k < ndev; ++k) {
        if (devs[k] < 0 || devs[k] >= count) return MBLS_INVALID_DEVICE;
        if (msm_size > 0 && !bases_per_dev[k]) return MBLS_INVALID_POINTER;
    }
    int cur = 0;
    MBLS_TRY(hipGetDevice(&cur));
    std::lock_guard<std::mutex> lk(multi_device_mutex());
    struct Restore {
        int d;
        ~Restore() { (void)hipSetDevice(d); }
    } restore{cur};
    const int d0 = devs[0];
    MultiDevRes* r0 = nullptr;
    eIcicleError er = multi_device_res(d0, r0);
    if (er != MBLS_SUCCESS) return er;
    for (int k = 1; k < ndev; ++k) {  // both directions: scalars d0 -> d, the partial d -> d0
        if ((er = enable_peer(d0, devs[k])) != MBLS_SUCCESS) return er;
        if ((er = enable_peer(devs[k], d0)) != MBLS_SUCCESS) return er;
    }
    hipStream_t st0 = cfg->stream ? static_cast<hipStream_t>(cfg->stream) : r0->stream;
    // shard streams are forked from the caller's stream: the caller's earlier work on its
    // inputs (a device scalar upload, say) is ordered before every shard
    MBLS_TRY(hipSetDevice(d0));
    // a pending mbls_msm_accumulate_event of the caller's stream: taken here (so the first shard's
    // msm_call on st0 does not), recorded on st0 when this call returns
    AccEventGuard acc_ev(take_accumulate_event(st0), st0);
    // the previous call may still read or write the partial / gather slots on its own streams
    // (is_async with a caller stream): this call's fork -- and so every shard -- waits for its end
    if (MultiDevRes* last = multi_device_last()) MBLS_TRY(hipStreamWaitEvent(st0, last->done, 0));
    MBLS_TRY(hipEventRecord(r0->ev[MAX_SHARDS - 1], st0));
    const size_t n = (size_t)msm_size;
    for (int k = 0; k < ndev; ++k) {
        const int d = devs[k];
        MultiDevRes* r = nullptr;
        if ((er = multi_device_res(d, r)) != MBLS_SUCCESS) return er;
        MBLS_TRY(hipSetDevice(d));
        hipStream_t sk = (d == d0) ? st0 : r->stream;
        if (sk != st0) MBLS_TRY(hipStreamWaitEvent(sk, r0->ev[MAX_SHARDS - 1], 0));
        const size_t lo = n * (size_t)k / ndev, hi = n * (size_t)(k + 1) / ndev;
        MSMConfig c = *cfg;
        c.stream = sk;
        c.batch_size = 1;
        c.are_results_on_device = true;
        c.is_async = true;
        // scalars on another device than the shard's: staged (a peer copy, hipMemcpyDefault)
        c.are_scalars_on_device = cfg->are_scalars_on_device && d == d0;
        const uint8_t* sp = static_cast<const uint8_t*>(scalars) + lo * 32;
        er = msm_call<F>(hi > lo ? sp : nullptr, bases_per_dev[k], (int)(hi - lo), &c, r->partials + (size_t)k * JAC,
                         MSM_JACOBIAN);
        if (er != MBLS_SUCCESS) return er;
        MBLS_TRY(hipEventRecord(r->ev[k], sk));
    }
    // exchange: the partials to the first device, then one EC sum and one normalisation
    MBLS_TRY(hipSetDevice(d0));
    for (int k = 0; k < ndev; ++k) {
        MultiDevRes* r = nullptr;
        if ((er = multi_device_res(devs[k], r)) != MBLS_SUCCESS) return er;
        if (devs[k] != d0) MBLS_TRY(hipStreamWaitEvent(st0, r->ev[k], 0));
        MBLS_TRY(hipMemcpyPeerAsync(r0->gather + (size_t)k * JAC, d0, r->partials + (size_t)k * JAC, devs[k], JAC, st0));
    }
    uint8_t* sum = r0->gather + (size_t)MAX_SHARDS * JAC;
    hipLaunchKernelGGL(k_sum_jac<F>, dim3(1), dim3(64), 0, st0, r0->gather, ndev, sum);
    hipLaunchKernelGGL(k_jac_to_icicle<F>, dim3(1), dim3(64), 0, st0, sum, sum, 1);
    MBLS_TRY(hipGetLastError());
    MBLS_TRY(hipMemcpyAsync(result, sum, JAC, cfg->are_results_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                            st0));
    // the library's per-device resources are reused by the next call: it waits for `done`
    MBLS_TRY(hipEventRecord(r0->done, st0));
    multi_device_last() = r0;
    if (!cfg->is_async || !cfg->are_results_on_device || !cfg->stream) MBLS_TRY(hipStreamSynchronize(st0));
    return MBLS_SUCCESS;
}

// ICICLE precompute_bases (registered MsmPreComputeImpl, icicle_backend_api.cuh:188-193; the
// reference's icicle_curve_api.cu:415-440 is a plain byte copy, so its factor > 1 is wrong).
// out[i*F + f] = 2^(s f) P_i, s = precompute_shift(F) = ceil(256 / F): the shift depends on the
// factor only, so one table serves an MSM of any c (MIDNIGHT_MSM_WINDOW or auto) and any
// msm_size <= bases_size, as core/msm.rs:441-454 -> :630-650 uses it.  The output is always
// Montgomery affine; standard-form input (are_points_montgomery_form = false) is converted.
template <class F>
eIcicleError precompute_call(const void* in, int n, const MSMConfig* cfg, void* out) {
    constexpr size_t AFF = GroupTraits<F>::AFF;
    if (!cfg || !in || !out) return MBLS_INVALID_POINTER;
    if (n < 0) return MBLS_INVALID_ARGUMENT;
    const int factor = cfg->precompute_factor > 0 ? cfg->precompute_factor : 1;
    if (factor > MAX_PRECOMPUTE) return MBLS_INVALID_ARGUMENT;
    if (n == 0) return MBLS_SUCCESS;
    hipStream_t st = static_cast<hipStream_t>(cfg->stream);
    CtxLease lease(st);
    if (!lease) return lease.error();
    Arena& A = lease->arena;
    size_t in_b = (size_t)n * AFF, out_b = in_b * factor;
    eIcicleError er = lease.reserve(align_up(in_b) + align_up(out_b));
    if (er != MBLS_SUCCESS) return er;
    uint8_t* din = (uint8_t*)A.take(in_b);
    uint8_t* dout = (uint8_t*)A.take(out_b);
    MBLS_TRY(hipMemcpyAsync(din, in, in_b, cfg->are_points_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
    if (!cfg->are_points_montgomery_form)
        hipLaunchKernelGGL(k_points_to_mont<F>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, din, (size_t)n);
    // the factor equal to the group's endomorphism split prepares the image table instead
    // (make_plan: an MSM with that factor splits its scalars against it)
    constexpr int endo = std::is_same<F, Fq>::value ? 2 : 4;
    if (factor == endo) {
        if ((er = launch_endo_table(din, dout, (uint32_t)n, endo, st)) != MBLS_SUCCESS) return er;
    } else {
        hipLaunchKernelGGL(k_precompute<F>, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, st, din, dout, (size_t)n,
                           factor, precompute_shift(factor));
    }
    MBLS_TRY(hipGetLastError());
    MBLS_TRY(hipMemcpyAsync(out, dout, out_b, cfg->are_results_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, st));
    MBLS_TRY(hipStreamSynchronize(st));
    if (cfg->are_results_on_device) precompute_register(out, out_b, factor);  // strict mode's table list
    return MBLS_SUCCESS;
}

}  // namespace mbls
