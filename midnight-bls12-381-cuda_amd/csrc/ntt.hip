// ntt.hip -- radix-2 Fr NTT for CDNA4 (natural-order core; orderings / columns_batch by permutation).
//
// Semantics = the CPU path the prover uses (core/ntt.rs:1488-1603, midnight_curves best_fft):
//   forward  X_j = sum_i x_i w^(ij),  inverse  x_i = n^-1 sum_j X_j w^(-ij),
//   w = ROOT_OF_UNITY^(2^(32-k)) for n = 2^k, ROOT_OF_UNITY = 7^((r-1)/2^32).
// The reference GPU NTT (ntt_kernels.cu:710-958) derives its twiddles from whatever root the
// caller passes assuming order 2^24 (ntt_kernels.cu:1614,1644) and does not match best_fft
// (SURVEY.md finding 2); we do not reproduce that.
//
// Data layout in HBM: n contiguous 32-byte Fr values per polynomial, batch polynomials
// back to back (other layouts are permuted in and out).  Twiddles: per-stage tables
// concatenated, stage s (m = 2^s) holding w_(2^s)^i, i < 2^(s-1), at offset 2^(s-1) - 1
// (2^L - 1 entries for stages 1..L), so adjacent columns of a tile read adjacent twiddles.
// Each entry is w R' mod r in radix-2^29 limbs (mbls_fr29.hpp: the butterflies' products run in
// that form), stored as three planes -- limbs 0-3 (16 B), limbs 4-7 (16 B), limb 8 (4 B) -- so
// every twiddle is three aligned loads (36 B per entry).
// (A single w_(2^K)^i table read at stride 2^(K-s) put every lane on its own cache line:
// measured 3.5x the data bytes fetched by the later passes, profiles/r01.)
//
// Kernel structure: ceil(k / 10) passes, each a LDS-resident tile of T = 1024 elements
// (32 KiB) doing up to 10 radix-2 DIT stages between __syncthreads.  Pass 1 fuses the
// bit-reversal permutation into its gather: it reads C adjacent columns of the input viewed
// as a 2^L x 2^(k-L) matrix (coalesced C*32-byte rows) and writes contiguous DIT blocks.
// Later passes read/write tiles of 2^L strided rows x C adjacent columns in place.  The
// inverse's n^-1 scaling is fused into the last pass's store.
// Algorithmic traffic: 64 B per element per transform (one read + one write of 32 B);
// actual traffic = passes * 64 B + twiddle reads.  Arithmetic: (n/2) log n Montgomery
// products -- the kernel is VALU-bound on gfx950.
#include <hip/hip_runtime.h>
#include <string.h>

#include <memory>
#include <mutex>
#include <optional>
#include <vector>

#include "mbls_common.hpp"
#include "mbls_field.hpp"
#include "mbls_fr29.hpp"

namespace mbls {

#ifndef MBLS_NTT_TILE_LOG
#define MBLS_NTT_TILE_LOG 10
#endif
#ifndef MBLS_NTT_PASS_STAGES
#define MBLS_NTT_PASS_STAGES 8
#endif
#ifndef MBLS_NTT_THREADS
#define MBLS_NTT_THREADS 256
#endif
#ifndef MBLS_NTT_DIRECT
#define MBLS_NTT_DIRECT 1  // the pass's last stage group stores straight from registers (k_ntt_pass)
#endif
#ifndef MBLS_NTT_XCD
#define MBLS_NTT_XCD 0  // 1: tiles of adjacent columns on the same XCD (shared L2 lines)
#endif
// diagnostic variant builds only (results WRONG, never shipped): 1 = no twiddle loads (a
// register value instead), 2 = no barrier between stage pairs, 3 = no tile load from HBM (the
// LDS tile is used as found), 4 = no tile store to HBM -- to price those costs
#ifndef MBLS_NTT_EXP
#define MBLS_NTT_EXP 0
#endif
static constexpr int NTT_TILE_LOG = MBLS_NTT_TILE_LOG;
static constexpr int NTT_TILE = 1 << NTT_TILE_LOG;  // elements per workgroup tile
static constexpr int NTT_THREADS = MBLS_NTT_THREADS;
static constexpr int NTT_PASS_STAGES = MBLS_NTT_PASS_STAGES;

// canonical 2^32-th root of unity, Montgomery (bls12_381_constants.h:127-130)
static const uint64_t ROOT_2_32_MONT[4] = {0xb9b58d8c5f0e466aULL, 0x5b1b4c801819d7ecULL, 0x0af53ae352a31e64ULL,
                                           0x5bf3adda19e9b27bULL};

// Twiddle tables of one domain build.  Callers take a shared_ptr snapshot under the lock and
// enqueue their kernels with it; a table superseded by an extension or a release is freed only
// when the last snapshot is dropped, and then only after a device synchronisation -- no queued
// transform ever reads freed memory (concurrent callers on rayon threads, SURVEY.md 8b
// "Threading").  Release / extension happen once per domain size, so the synchronisation is
// rare; an event recorded after every transform instead (round 3) cost ~5 us of dispatch delay
// per transform (an event marker holds the next dispatch: profiles/r04/gapbench_markers.txt).
struct DomainTables {
    int max_log = 0;            // stage tables built for stages 1..max_log
    uint32_t count = 0;         // entries per table (2^max_log - 1): the limb planes' stride
    int device = 0;             // device the tables live on
    uint8_t* tw = nullptr;      // per-stage w_(2^s)^i tables (see header)
    uint8_t* tw_inv = nullptr;  // per-stage w_(2^s)^-i
    ~DomainTables() {
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (cur != device) (void)hipSetDevice(device);
        (void)hipDeviceSynchronize();  // every transform that read the tables has finished
        if (tw) (void)hipFree(tw);
        if (tw_inv) (void)hipFree(tw_inv);
        if (cur != device) (void)hipSetDevice(cur);
    }
};

struct Domain {
    int order_log = 32;  // 2^order_log: order of the initialised root (size bound)
    std::shared_ptr<DomainTables> tables;
};

static constexpr int MAX_DOMAIN_DEVICES = 64;
static std::mutex g_domain_mu;
// never destroyed: freeing device memory during runtime teardown at exit is unsafe
static Domain* g_domains[MAX_DOMAIN_DEVICES];

// the current device's domain (created on first use); caller holds g_domain_mu
static Domain* current_domain(int* dev_out = nullptr) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DOMAIN_DEVICES) return nullptr;
    if (!g_domains[dev]) g_domains[dev] = new Domain();
    if (dev_out) *dev_out = dev;
    return g_domains[dev];
}

__device__ __forceinline__ uint32_t bitrev(uint32_t x, int bits) {
    return bits == 0 ? 0u : (__builtin_bitreverse32(x) >> (32 - bits));
}

// per-stage tables: entry g (stage s = floor(log2(g+1)) + 1, i = g + 1 - 2^(s-1)) holds
// w_(2^L)^(i * 2^(L-s)) = w_(2^s)^i, one exponentiation per entry (init only), times 2^5 (the
// Montgomery form R = 2^256 -> R' = 2^261 of mbls_fr29.hpp), canonical, in the three limb planes
struct TwPlanes {
    uint4* a;     // limbs 0-3
    uint4* b;     // limbs 4-7
    uint32_t* c;  // limb 8
};
MBLS_DEV TwPlanes tw_planes(uint8_t* base, uint32_t count) {
    uint4* a = reinterpret_cast<uint4*>(base);
    return TwPlanes{a, a + count, reinterpret_cast<uint32_t*>(a + 2 * (size_t)count)};
}
static constexpr size_t TW_ENTRY_BYTES = 36;
// 2^5 R mod r (Montgomery form of 32): x * C32 = x 2^5 (R-form products)
static constexpr uint32_t TW_C32[8] = {0xffffffbau, 0x00000045u, 0x0072d846u, 0x1a25272eu,
                                       0x5dbeee8bu, 0xfe2eedcdu, 0x9eefbe41u, 0x4d043f42u};

__global__ void k_twiddles(uint8_t* table, Fr w, int L, uint32_t count) {
    uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= count) return;
    const int s = 32 - __builtin_clz(g + 1);  // floor(log2(g+1)) + 1
    const uint32_t i = g + 1 - (1u << (s - 1));
    Fr acc = Fr::one();
    Fr b = w;
    uint64_t e = (uint64_t)i << (L - s);
    while (e) {
        if (e & 1) acc = acc * b;
        b = sqr(b);
        e >>= 1;
    }
    Fr c32;
#pragma unroll
    for (int k = 0; k < 8; ++k) c32.v[k] = TW_C32[k];
    const r29::F29 t = r29::unpack(acc * c32);  // w R' mod r, canonical
    const TwPlanes P = tw_planes(table, count);
    P.a[g] = make_uint4(t.l[0], t.l[1], t.l[2], t.l[3]);
    P.b[g] = make_uint4(t.l[4], t.l[5], t.l[6], t.l[7]);
    P.c[g] = t.l[8];
}

// Lazy butterflies: between the first load and the last store of a transform, values live in
// [0, 2r) (2r < 2^256).  b*w with b < 2r and a canonical twiddle w < r is < r*R, so the
// Montgomery product needs no final subtraction (fips::mul<C, false>); a + t and a - t are
// brought back into [0, 2r) with one conditional 2r correction each (same cost as the
// canonical add / sub).  The last pass stores canonical values.
static constexpr uint32_t NTT_TWO_R[8] = {0x00000002u, 0xfffffffeu, 0xfffcb7fdu, 0xa77b4805u,
                                          0x1343b00au, 0x6673b010u, 0x533afa90u, 0xe7db4ea6u};  // literals
MBLS_DEV Fr add_2r(const Fr& a, const Fr& b) {
    Fr s, d;
    unsigned c = 0, br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
#pragma unroll
    for (int i = 0; i < 8; ++i) d.v[i] = __builtin_subc(s.v[i], NTT_TWO_R[i], br, &br);
    const bool keep = !c && br;  // a + b < 2r
#pragma unroll
    for (int i = 0; i < 8; ++i) s.v[i] = keep ? s.v[i] : d.v[i];
    return s;
}
MBLS_DEV Fr sub_2r(const Fr& a, const Fr& b) {
    Fr d;
    unsigned br = 0, c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
    const uint32_t mask = 0u - br;  // a < b: add 2r (mod 2^256)
#pragma unroll
    for (int i = 0; i < 8; ++i) d.v[i] = __builtin_addc(d.v[i], NTT_TWO_R[i] & mask, c, &c);
    return d;
}

// an Fr element as two 16-byte words (LDS tile, global data, twiddle tables): element e at
// [2e], [2e + 1] -- 32-bit element indices (transforms <= 2^30, ntt_call) and b128 accesses
MBLS_DEV Fr ld2(const uint4* p, uint32_t e) {
    const uint4 a = p[2 * e], b = p[2 * e + 1];
    return Fr{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
}
MBLS_DEV void st2(uint4* p, uint32_t e, const Fr& v) {
    p[2 * e] = make_uint4(v.v[0], v.v[1], v.v[2], v.v[3]);
    p[2 * e + 1] = make_uint4(v.v[4], v.v[5], v.v[6], v.v[7]);
}
// twiddle entry g of the limb planes
MBLS_DEV r29::F29 ldtw(const uint4* a, const uint4* b, const uint32_t* c, uint32_t g) {
    const uint4 x = a[g], y = b[g];
    return r29::F29{{x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, c[g]}};
}

// One pass of up to NTT_TILE_LOG DIT stages.
//   FIRST: stages 1..L with the bit-reversal gather from `in`; else stages s0+1..s0+L in place.
//   LAST:  store canonical values; SCALE (inverse, implies LAST): multiply them by n^-1.
// One tile per workgroup, grid = tiles.  Persistent workgroups walking several tiles lost in every
// form measured in round 6 (profiles/r06/README.md): reload after the stores (11% slower: vmcnt
// counts loads and stores in one in-order counter, so the next tile's first wait also waits for
// this tile's stores), the next tile prefetched into 32 VGPRs during the stage pairs (spills at 4
// workgroups per CU, occupancy at 3: +6-11%), and the next tile LDS-DMA'd behind this tile's
// stores (+7-13%), although a no-store pricing variant shows the stores at ~13% of the pass.
// Index arithmetic is 32-bit (element indices inside a polynomial and the twiddle tables stay
// below 2^31 for transforms <= 2^30), the tile is a uint4 LDS array (every access one b128),
// and the 2r constants are literals (the pass is VALU-issue bound, profiles/r05/ntt_diag.txt).
template <bool FIRST, bool LAST, bool SCALE>
__global__ __launch_bounds__(NTT_THREADS, 5) void k_ntt_pass(uint8_t* __restrict__ out_,
                                                                         const uint8_t* __restrict__ in_,
                                                                         const uint8_t* __restrict__ tw_,
                                                                         uint32_t tw_count, int log_n, int s0, int L,
                                                                         int logC, Fr scale, uint32_t ntiles) {
    __shared__ uint4 lds[NTT_TILE * 2];
    const uint32_t C = 1u << logC;
    const uint32_t rows = 1u << L;
    const uint32_t T = rows * C;  // active tile elements (== NTT_TILE except for tiny transforms)
    const size_t n = (size_t)1 << log_n;
    const uint32_t tiles_per_poly = (uint32_t)(n >> (L + logC));
    // twiddle limb planes (k_twiddles)
    const uint4* twa = reinterpret_cast<const uint4*>(tw_);
    const uint4* twb = twa + tw_count;
    const uint32_t* twc = reinterpret_cast<const uint32_t*>(twa + 2 * (size_t)tw_count);
    // FIRST: element (row tr, column c0 + c) at (tr << colbits) + c0 + c; else element (t, c) at
    // hi_base + (t << s0) + lo0 + c
    const uint32_t colbits = (uint32_t)(log_n - L);
    const uint32_t lo_tiles = FIRST ? 1u : (1u << s0) >> logC;
    struct Tile {
        size_t poly;  // element offset of the tile's polynomial
        uint32_t lo0, hi_base;
    };
    auto tile_of = [&](uint32_t id) {
        const uint32_t poly = id / tiles_per_poly, tile = id % tiles_per_poly;
        return Tile{(size_t)poly * n, FIRST ? tile * C : (tile % lo_tiles) * C,
                    FIRST ? 0u : (tile / lo_tiles) << (s0 + L)};
    };
    // element e of the tile ([row t][col c] in LDS order): its index in the polynomial
    auto src_of = [&](const Tile& g, uint32_t e) {
        const uint32_t c = e & (C - 1), t = e >> logC;
        return FIRST ? (t << colbits) + g.lo0 + c : g.hi_base + (t << s0) + g.lo0 + c;
    };
    const uint4* in = reinterpret_cast<const uint4*>(FIRST ? in_ : out_);
    uint4* out = reinterpret_cast<uint4*>(out_);

    const uint32_t id = blockIdx.x;  // one tile per workgroup
    if (id >= ntiles) return;
    const Tile g = tile_of(id);
    {
        // ---- the tile into LDS as [row t][col c] (FIRST: rows at their bit-reversed DIT
        // position; not vectorised: the loop vectoriser split the b128 LDS stores into b32)
#pragma clang loop vectorize(disable) interleave(disable)
        for (uint32_t e = threadIdx.x; e < T; e += NTT_THREADS) {
            const uint32_t c = e & (C - 1), t = e >> logC;
            if (MBLS_NTT_EXP == 3) {
                if (e == 0xffffffffu) st2(lds, e, ld2(in, e));  // never: keeps the loop's shape
            } else {
                st2(lds, FIRST ? bitrev(t, L) * C + c : e, ld2(in + 2 * g.poly, src_of(g, e)));
            }
        }
        __syncthreads();
        // ---- L DIT stages: pairs of stages as radix-4 (2 x 2) butterflies in registers (one LDS
        // round trip and one barrier per pair), an odd last stage as radix-2
        const uint32_t lo_base = FIRST ? 0u : g.lo0;
        uint4* o = out + 2 * g.poly;
        // the last stage group (MBLS_NTT_DIRECT) stores its outputs straight to HBM from registers:
        // no LDS round trip, barrier or separate store loop; (row, c) of the tile -> its position
        auto put = [&](uint32_t row, uint32_t c, Fr v) {
            if (SCALE) v = v * scale;  // v < 2r, scale < r: the reduced product is canonical
            else if (LAST) reduce_once(v);
            st2(o, FIRST ? (bitrev(g.lo0 + c, colbits) << L) + row : g.hi_base + (row << s0) + g.lo0 + c, v);
        };
        int l = 1;
        for (; l + 1 <= L; l += 2) {
            const bool fin = MBLS_NTT_DIRECT && l + 2 > L;  // the last pair, no radix-2 stage after it
            const uint32_t h = 1u << (l - 1);  // stage l pairs rows (t, t + h), stage l + 1 rows (t, t + 2h)
            const int s = s0 + l;              // global stage of the first of the pair
            const uint32_t t1 = (1u << (s - 1)) - 1, t2 = (1u << s) - 1;  // stage tables s, s + 1
            const uint32_t stride = h * C;
            for (uint32_t u = threadIdx.x; u < T / 4; u += NTT_THREADS) {
                const uint32_t c = u & (C - 1);
                const uint32_t r = u >> logC;
                const uint32_t j = r & (h - 1);
                const uint32_t q = ((r >> (l - 1)) << (l + 1)) + j;
                const uint32_t e0 = q * C + c;
                const uint32_t lo = FIRST ? 0u : lo_base + c;
                const bool triv = FIRST && l == 1;  // first pair of the first pass: j = 0, twiddles 1
                // twiddles first: their loads do not depend on the tile
                r29::F29 w1, w2, w3;
                const uint32_t jl = (j << s0) + lo;
                if (!triv) {
                    w1 = ldtw(twa, twb, twc, t1 + jl);
                    w2 = ldtw(twa, twb, twc, t2 + jl);
                }
                w3 = ldtw(twa, twb, twc, t2 + jl + (h << s0));
                Fr x0 = ld2(lds, e0), x1 = ld2(lds, e0 + stride), x2 = ld2(lds, e0 + 2 * stride),
                   x3 = ld2(lds, e0 + 3 * stride);
                if (MBLS_NTT_EXP == 1) w1 = w2 = w3 = r29::unpack(x0);
                // stage l: (x0, x1), (x2, x3) share twiddle w_(2^s)^j
                if (!triv) {
                    x1 = r29::mul_words(x1, w1);
                    x3 = r29::mul_words(x3, w1);
                }
                Fr y0 = add_2r(x0, x1), y1 = sub_2r(x0, x1), y2 = add_2r(x2, x3), y3 = sub_2r(x2, x3);
                // stage l + 1: (y0, y2) with w_(2^(s+1))^j, (y1, y3) with w_(2^(s+1))^(j + h)
                if (!triv) y2 = r29::mul_words(y2, w2);
                y3 = r29::mul_words(y3, w3);
                if (fin) {
                    put(q, c, add_2r(y0, y2));
                    put(q + 2 * h, c, sub_2r(y0, y2));
                    put(q + h, c, add_2r(y1, y3));
                    put(q + 3 * h, c, sub_2r(y1, y3));
                } else {
                    st2(lds, e0, add_2r(y0, y2));
                    st2(lds, e0 + 2 * stride, sub_2r(y0, y2));
                    st2(lds, e0 + stride, add_2r(y1, y3));
                    st2(lds, e0 + 3 * stride, sub_2r(y1, y3));
                }
            }
            if (fin) return;
            if (MBLS_NTT_EXP != 2) __syncthreads();
        }
        if (l == L) {  // odd stage count: one radix-2 stage
            const uint32_t half = 1u << (l - 1);
            const int s = s0 + l;                     // global stage, m = 2^s
            const uint32_t ts = (1u << (s - 1)) - 1;  // stage table s
            for (uint32_t u = threadIdx.x; u < T / 2; u += NTT_THREADS) {
                const uint32_t c = u & (C - 1);
                const uint32_t r = u >> logC;
                const uint32_t gg = r >> (l - 1);
                const uint32_t j = r & (half - 1);
                const uint32_t t0 = (gg << l) + j, t1 = t0 + half;
                r29::F29 w;
                if (l > 1 || !FIRST) w = ldtw(twa, twb, twc, ts + (j << s0) + (FIRST ? 0u : lo_base + c));
                const Fr a = ld2(lds, t0 * C + c);
                Fr b = ld2(lds, t1 * C + c);
                if (l > 1 || !FIRST) b = r29::mul_words(b, w);
                if (MBLS_NTT_DIRECT) {
                    put(t0, c, add_2r(a, b));
                    put(t1, c, sub_2r(a, b));
                } else {
                    st2(lds, t0 * C + c, add_2r(a, b));
                    st2(lds, t1 * C + c, sub_2r(a, b));
                }
            }
            if (MBLS_NTT_DIRECT) return;
            __syncthreads();
        }

        // ---- store (L = 0 only, or MBLS_NTT_DIRECT = 0)
        for (uint32_t e = threadIdx.x; e < T; e += NTT_THREADS) {
            Fr v;
            uint32_t dst;
            if (FIRST) {
                // write block by block: consecutive threads -> consecutive positions of one block
                const uint32_t p = e & (rows - 1), c = e >> L;
                v = ld2(lds, p * C + c);
                dst = (bitrev(g.lo0 + c, colbits) << L) + p;
            } else {
                v = ld2(lds, e);
                dst = src_of(g, e);
            }
            if (SCALE) v = v * scale;  // v < 2r, scale < r: the reduced product is canonical
            else if (LAST) reduce_once(v);
            if (MBLS_NTT_EXP == 4 && (v.v[0] ^ v.v[7]) != 0x12345u) continue;  // (almost) never stores
            st2(o, dst, v);
        }
    }
}

__global__ void k_copy_scale(uint8_t* out, const uint8_t* in, size_t count, Fr scale, int do_scale) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= count) return;
    Fr v = load<FrCfg>(in + 32 * i);
    if (do_scale) v = v * scale;
    store<FrCfg>(out + 32 * i, v);
}

// ---- host-side field helpers (tiny, init-time only) ----------------------------------
typedef unsigned __int128 u128;
static const uint64_t HFR_P[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                                  0x73eda753299d7d48ULL};
static const uint64_t HFR_ONE[4] = {0x00000001fffffffeULL, 0x5884b7fa00034802ULL, 0x998c4fefecbc4ff5ULL,
                                    0x1824b159acc5056fULL};
static const uint64_t HFR_R2[4] = {0xc999e990f3f29c6dULL, 0x2b6cedcb87925c23ULL, 0x05d314967254398fULL,
                                   0x0748d9d99f59ff11ULL};

static void hfr_mul(uint64_t* r, const uint64_t* a, const uint64_t* b) {
    uint64_t t[6] = {0};
    for (int i = 0; i < 4; ++i) {
        uint64_t c = 0;
        for (int j = 0; j < 4; ++j) {
            u128 s = (u128)a[j] * b[i] + t[j] + c;
            t[j] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
        u128 s = (u128)t[4] + c;
        t[4] = (uint64_t)s;
        t[5] = (uint64_t)(s >> 64);
        uint64_t q = t[0] * 0xfffffffeffffffffULL;
        s = (u128)q * HFR_P[0] + t[0];
        c = (uint64_t)(s >> 64);
        for (int j = 1; j < 4; ++j) {
            s = (u128)q * HFR_P[j] + t[j] + c;
            t[j - 1] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
        s = (u128)t[4] + c;
        t[3] = (uint64_t)s;
        t[4] = t[5] + (uint64_t)(s >> 64);
    }
    bool ge = t[4] != 0;
    if (!ge) {
        ge = true;
        for (int i = 3; i >= 0; --i)
            if (t[i] != HFR_P[i]) {
                ge = t[i] > HFR_P[i];
                break;
            }
    }
    if (ge) {
        uint64_t br = 0;
        for (int i = 0; i < 4; ++i) {
            u128 d = (u128)t[i] - HFR_P[i] - br;
            t[i] = (uint64_t)d;
            br = (uint64_t)(d >> 64) & 1;
        }
    }
    memcpy(r, t, 32);
}

static bool hfr_eq(const uint64_t* a, const uint64_t* b) { return memcmp(a, b, 32) == 0; }

static void hfr_pow(uint64_t* r, const uint64_t* a, const uint64_t* e) {
    uint64_t acc[4];
    memcpy(acc, HFR_ONE, 32);
    for (int i = 255; i >= 0; --i) {
        hfr_mul(acc, acc, acc);
        if ((e[i / 64] >> (i % 64)) & 1) hfr_mul(acc, acc, a);
    }
    memcpy(r, acc, 32);
}

static void hfr_inv(uint64_t* r, const uint64_t* a) {
    uint64_t e[4];
    memcpy(e, HFR_P, 32);
    e[0] -= 2;
    hfr_pow(r, a, e);
}

// order of `w` (Montgomery) as a power of two, or -1
static int hfr_log_order(const uint64_t* w) {
    uint64_t x[4];
    memcpy(x, w, 32);
    for (int k = 0; k <= 32; ++k) {
        if (hfr_eq(x, HFR_ONE)) return k;
        hfr_mul(x, x, x);
    }
    return -1;
}

static void canonical_omega(uint64_t* w, int log_n) {
    memcpy(w, ROOT_2_32_MONT, 32);
    for (int k = log_n; k < 32; ++k) hfr_mul(w, w, w);
}

static Fr to_dev(const uint64_t* h) {
    Fr r;
    memcpy(r.v, h, 32);
    return r;
}

// (re)build the stage tables of `dom` (the current device's) up to 2^max_log; caller holds
// g_domain_mu.  A superseded table stays alive while any snapshot of it does (DomainTables);
// the domain's own reference moves to *old, which the caller drops AFTER releasing the lock
// (the destructor's device synchronisation must not run under g_domain_mu: ADVICE r4)
static eIcicleError build_domain(Domain& dom, int max_log, hipStream_t st, std::shared_ptr<DomainTables>& old) {
    if (dom.tables && dom.tables->max_log >= max_log) return MBLS_SUCCESS;
    const int order = dom.order_log;
    if (max_log > order) return MBLS_INVALID_ARGUMENT;
    size_t count = ((size_t)1 << max_log) - 1;
    if (count == 0) count = 1;
    auto t = std::make_shared<DomainTables>();
    MBLS_TRY(hipGetDevice(&t->device));
    MBLS_TRY(hipMalloc(&t->tw, TW_ENTRY_BYTES * count));
    MBLS_TRY(hipMalloc(&t->tw_inv, TW_ENTRY_BYTES * count));
    t->count = (uint32_t)count;
    uint64_t w[4], wi[4];
    canonical_omega(w, max_log);
    hfr_inv(wi, w);
    int blocks = (int)((count + 255) / 256);
    hipLaunchKernelGGL(k_twiddles, dim3(blocks), dim3(256), 0, st, t->tw, to_dev(w), max_log, (uint32_t)count);
    hipLaunchKernelGGL(k_twiddles, dim3(blocks), dim3(256), 0, st, t->tw_inv, to_dev(wi), max_log, (uint32_t)count);
    MBLS_TRY(hipGetLastError());
    MBLS_TRY(hipStreamSynchronize(st));
    t->max_log = max_log;
    old = std::move(dom.tables);
    dom.tables = std::move(t);
    return MBLS_SUCCESS;
}

// enqueue forward/inverse NTT of `batch` polynomials of 2^log_n on device buffers
// (D: the caller's snapshot of the domain tables, kept alive across the enqueue)
eIcicleError ntt_device(uint8_t* out, const uint8_t* in, int log_n, bool inverse, int batch, const DomainTables& D,
                        hipStream_t st) {
    if (!D.tw || log_n > D.max_log) return MBLS_INVALID_ARGUMENT;
    const size_t n = (size_t)1 << log_n;
    const uint8_t* tw = inverse ? D.tw_inv : D.tw;
    uint64_t ninv_h[4] = {0, 0, 0, 0};
    if (inverse) {
        uint64_t nm[4] = {n, 0, 0, 0};
        hfr_mul(nm, nm, HFR_R2);  // n in Montgomery form
        hfr_inv(ninv_h, nm);
    }
    Fr scale = to_dev(inverse ? ninv_h : HFR_ONE);
    if (log_n == 0) {
        size_t cnt = (size_t)batch;
        hipLaunchKernelGGL(k_copy_scale, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, out, in, cnt, scale, 0);
        MBLS_TRY(hipGetLastError());
        return MBLS_SUCCESS;
    }
    // split the k stages into passes of <= NTT_PASS_STAGES stages (tile rows), so that a tile
    // keeps >= 4 adjacent columns (>= 128-byte contiguous row segments in HBM)
    int npass = (log_n + NTT_PASS_STAGES - 1) / NTT_PASS_STAGES;
    int s0 = 0;
    ProfScope prof_t("ntt.transform", st);
    for (int p = 0; p < npass; ++p) {
        ProfScope prof_p("ntt.pass", st);
        int remaining = log_n - s0;
        int L = (remaining + (npass - p) - 1) / (npass - p);
        bool first = (p == 0);
        bool last = (p == npass - 1);
        // columns per tile: limited by the tile size and by the available column count
        int colspace = first ? (log_n - L) : s0;
        int logC = NTT_TILE_LOG - L;
        if (logC > colspace) logC = colspace;
        size_t tiles = (n >> (L + logC)) * (size_t)batch;
        if (tiles > 0x7fffffff) return MBLS_INVALID_ARGUMENT;
        const uint32_t nt = (uint32_t)tiles;
        dim3 grid(nt), blk(NTT_THREADS);
        if (first && last && inverse)
            hipLaunchKernelGGL((k_ntt_pass<true, true, true>), grid, blk, 0, st, out, in, tw, D.count, log_n, s0, L, logC, scale, nt);
        else if (first && last)
            hipLaunchKernelGGL((k_ntt_pass<true, true, false>), grid, blk, 0, st, out, in, tw, D.count, log_n, s0, L, logC, scale, nt);
        else if (first)
            hipLaunchKernelGGL((k_ntt_pass<true, false, false>), grid, blk, 0, st, out, in, tw, D.count, log_n, s0, L, logC, scale, nt);
        else if (last && inverse)
            hipLaunchKernelGGL((k_ntt_pass<false, true, true>), grid, blk, 0, st, out, in, tw, D.count, log_n, s0, L, logC, scale, nt);
        else if (last)
            hipLaunchKernelGGL((k_ntt_pass<false, true, false>), grid, blk, 0, st, out, in, tw, D.count, log_n, s0, L, logC, scale, nt);
        else
            hipLaunchKernelGGL((k_ntt_pass<false, false, false>), grid, blk, 0, st, out, in, tw, D.count, log_n, s0, L, logC, scale, nt);
        MBLS_TRY(hipGetLastError());
        s0 += L;
    }
    return MBLS_SUCCESS;
}

static int log2_exact(long long n) {
    if (n <= 0 || (n & (n - 1))) return -1;
    int k = 0;
    while ((1LL << k) < n) ++k;
    return k;
}

eIcicleError ntt_init_domain(const mbls_fr_t* root, const NTTInitDomainConfig* cfg) {
    if (!root) return MBLS_INVALID_POINTER;
    hipStream_t st = cfg ? static_cast<hipStream_t>(cfg->stream) : nullptr;
    // The root only sizes the domain: its order 2^K (read as Montgomery, else as standard
    // form).  Twiddles are always the canonical best_fft roots (see file header).
    int K = hfr_log_order(root->limbs);
    if (K < 0) {
        uint64_t m[4];
        hfr_mul(m, root->limbs, HFR_R2);
        K = hfr_log_order(m);
    }
    if (K < 0) return MBLS_INVALID_ARGUMENT;
    std::shared_ptr<DomainTables> old;  // dropped after the lock (declared before it)
    std::lock_guard<std::mutex> lk(g_domain_mu);
    Domain* dom = current_domain();
    if (!dom) return MBLS_INVALID_DEVICE;
    // the tables are canonical (independent of the root): a smaller order only bounds sizes
    dom->order_log = K;
    // stage tables up to 2^22 now (2 x 128 MiB); larger sizes extend them on first use
    return build_domain(*dom, K < 22 ? K : 22, st, old);
}

eIcicleError ntt_release_domain() {
    std::shared_ptr<DomainTables> old;
    {
        std::lock_guard<std::mutex> lk(g_domain_mu);
        Domain* dom = current_domain();
        if (!dom) return MBLS_INVALID_DEVICE;
        old = std::move(dom->tables);
        dom->tables.reset();
        dom->order_log = 32;
    }
    return MBLS_SUCCESS;  // `old` frees the tables here unless a transform still holds them
}

// coset scaling x_i *= g^(+-i) within each polynomial (device, in place)
__global__ void k_coset_scale(uint8_t* data, Fr g, size_t n, size_t total) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= total) return;
    size_t e = i & (n - 1);
    Fr acc = Fr::one(), b = g;
    while (e) {
        if (e & 1) acc = acc * b;
        b = sqr(b);
        e >>= 1;
    }
    Fr v = load<FrCfg>(data + 32 * i);
    store<FrCfg>(data + 32 * i, v * acc);
}

// Layout permutation (gather): out position q of layout (out_cols, out_rev) takes the element
// of layout (in_cols, in_rev) holding the same (member b, natural index e).  *_cols: column-
// major batch (element e of member b at e*batch + b); *_rev: bit-reversed element order.
__global__ void k_perm(uint8_t* __restrict__ out, const uint8_t* __restrict__ in, int log_n, uint32_t batch,
                       int out_cols, int out_rev, int in_cols, int in_rev) {
    const size_t n = (size_t)1 << log_n;
    const size_t total = n * batch;
    for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < total; q += (size_t)gridDim.x * blockDim.x) {
        const size_t b = out_cols ? q % batch : q >> log_n;
        const size_t i = out_cols ? q / batch : q & (n - 1);
        const size_t e = out_rev ? bitrev((uint32_t)i, log_n) : i;
        const size_t pi = in_rev ? bitrev((uint32_t)e, log_n) : e;
        const size_t src = in_cols ? pi * batch + b : (b << log_n) + pi;
        store<FrCfg>(out + 32 * q, load<FrCfg>(in + 32 * src));
    }
}

static eIcicleError launch_perm(uint8_t* out, const uint8_t* in, int log_n, int batch, bool out_cols, bool out_rev,
                                bool in_cols, bool in_rev, hipStream_t st) {
    const size_t total = ((size_t)1 << log_n) * (size_t)batch;
    size_t blocks = (total + 255) / 256;
    if (blocks > 256 * 16) blocks = 256 * 16;
    hipLaunchKernelGGL(k_perm, dim3((unsigned)blocks), dim3(256), 0, st, out, in, log_n, (uint32_t)batch,
                       out_cols ? 1 : 0, out_rev ? 1 : 0, in_cols ? 1 : 0, in_rev ? 1 : 0);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// Full ICICLE-semantics NTT call: staging, batch (row or columns_batch layout), coset,
// orderings.  R = bit-reversed order; M ("mixed", implementation-defined in ICICLE) is
// bit-reversed here too, so kNM -> kMN round-trips.  Non-natural layouts are permuted to
// natural row-major around the natural-order transform (one extra HBM pass each).
eIcicleError ntt_call(const mbls_fr_t* input, int size, NTTDir dir, const NTTConfig* cfg, mbls_fr_t* output,
                      const mbls_fr_t* coset_gen) {
    if (!input || !output || !cfg) return MBLS_INVALID_POINTER;
    int log_n = log2_exact(size);
    if (log_n < 0) return MBLS_INVALID_ARGUMENT;
    const int ord = (int)cfg->ordering;
    if (ord < MBLS_ORDERING_NN || ord > MBLS_ORDERING_MN) return MBLS_INVALID_ARGUMENT;
    const bool in_rev = ord == MBLS_ORDERING_RN || ord == MBLS_ORDERING_RR || ord == MBLS_ORDERING_MN;
    const bool out_rev = ord == MBLS_ORDERING_NR || ord == MBLS_ORDERING_RR || ord == MBLS_ORDERING_NM;
    const bool cols = cfg->columns_batch;
    int batch = cfg->batch_size > 0 ? cfg->batch_size : 1;
    hipStream_t st = static_cast<hipStream_t>(cfg->stream);
    std::shared_ptr<DomainTables> tables;  // snapshot: valid for the whole enqueue below
    std::shared_ptr<DomainTables> superseded;  // an extension's old tables, dropped outside the lock
    {
        std::lock_guard<std::mutex> lk(g_domain_mu);
        Domain* dom = current_domain();
        if (!dom) return MBLS_INVALID_DEVICE;
        if (log_n > dom->order_log) return MBLS_INVALID_ARGUMENT;  // beyond the initialised root
        if (!dom->tables || dom->tables->max_log < log_n) {
            // lazily build / extend this device's stage tables (init_domain builds up to 2^22)
            int want = log_n < 20 ? 20 : log_n;
            if (want > dom->order_log) want = dom->order_log;
            eIcicleError er = build_domain(*dom, want, st, superseded);
            if (er != MBLS_SUCCESS) return er;
        }
        tables = dom->tables;
    }
    const size_t bytes = (size_t)size * 32 * (size_t)batch;
    const size_t total = (size_t)size * batch;
    const bool inverse = (dir == MBLS_NTT_INVERSE);
    // coset: forward evaluates on g*H (pre-scale by g^i); inverse post-scales by g^-i
    bool coset = false;
    uint64_t g[4];
    if (coset_gen) {
        memcpy(g, coset_gen->limbs, 32);
        coset = !hfr_eq(g, HFR_ONE);
    }
    const bool perm_in = (in_rev || cols) && log_n > 0;
    const bool perm_out = (out_rev || cols) && log_n > 0;
    const bool in_dev = cfg->are_inputs_on_device, out_dev = cfg->are_outputs_on_device;
    // the transform's source must be natural row-major, writable when coset-scaled, and
    // distinct from its destination (the first pass gathers bit-reversed)
    const bool same = in_dev && out_dev && input == output;
    const bool work_in_tmp = perm_in || (coset && !inverse) || (same && !perm_out);

    size_t need = 0;
    if (!in_dev) need += align_up(bytes);
    if (!out_dev) need += align_up(bytes);
    if (work_in_tmp) need += align_up(bytes);
    if (perm_out) need += align_up(bytes);
    // a transform that needs no staging (device in / out, natural order, distinct buffers: the
    // prover's shape) takes no scratch context, so it records no `done` event: an event marker
    // holds the next dispatch ~5 us, 1% of a 2^22 transform
    std::optional<CtxLease> lease;
    Arena* arena = nullptr;
    eIcicleError er = MBLS_SUCCESS;
    if (need) {
        lease.emplace(st);
        if (!*lease) return lease->error();
        if ((er = lease->reserve(need)) != MBLS_SUCCESS) return er;
        arena = &(**lease).arena;
    }
    const uint8_t* src = reinterpret_cast<const uint8_t*>(input);
    uint8_t* dst = reinterpret_cast<uint8_t*>(output);
    if (!in_dev) {
        void* t = arena->take(bytes);
        MBLS_TRY(hipMemcpyAsync(t, input, bytes, hipMemcpyHostToDevice, st));
        src = static_cast<const uint8_t*>(t);
    }
    if (!out_dev) dst = static_cast<uint8_t*>(arena->take(bytes));
    uint8_t* wout = perm_out ? static_cast<uint8_t*>(arena->take(bytes)) : dst;
    const uint8_t* win = src;
    if (work_in_tmp) {
        uint8_t* t = static_cast<uint8_t*>(arena->take(bytes));
        if (perm_in) {
            if ((er = launch_perm(t, src, log_n, batch, false, false, cols, in_rev, st)) != MBLS_SUCCESS) return er;
        } else {
            MBLS_TRY(hipMemcpyAsync(t, src, bytes, hipMemcpyDeviceToDevice, st));
        }
        if (coset && !inverse) {
            hipLaunchKernelGGL(k_coset_scale, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, t, to_dev(g),
                               (size_t)size, total);
            MBLS_TRY(hipGetLastError());
        }
        win = t;
    }
    er = ntt_device(wout, win, log_n, inverse, batch, *tables, st);
    if (er != MBLS_SUCCESS) return er;
    if (coset && inverse) {
        uint64_t gi[4];
        hfr_inv(gi, g);
        hipLaunchKernelGGL(k_coset_scale, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, wout, to_dev(gi),
                           (size_t)size, total);
        MBLS_TRY(hipGetLastError());
    }
    if (perm_out && (er = launch_perm(dst, wout, log_n, batch, cols, out_rev, false, false, st)) != MBLS_SUCCESS)
        return er;
    if (!out_dev) MBLS_TRY(hipMemcpyAsync(output, dst, bytes, hipMemcpyDeviceToHost, st));
    // a staged host input is out of the caller's memory once hipMemcpyAsync returns (pageable)
    // or is the caller's to keep alive (pinned): only a host result forces the wait
    if (!cfg->is_async || !out_dev) MBLS_TRY(hipStreamSynchronize(st));
    return MBLS_SUCCESS;
}

}  // namespace mbls

using namespace mbls;

extern "C" {

eIcicleError bls12_381_ntt_init_domain_cuda(const mbls_fr_t* root_of_unity, const NTTInitDomainConfig* config) {
    return ntt_init_domain(root_of_unity, config);
}
eIcicleError bls12_381_ntt_release_domain_cuda(void) { return ntt_release_domain(); }
eIcicleError bls12_381_ntt_cuda(const mbls_fr_t* input, int size, NTTDir dir, const NTTConfig* config,
                                mbls_fr_t* output) {
    return ntt_call(input, size, dir, config, output, config ? &config->coset_gen : nullptr);
}
eIcicleError bls12_381_coset_ntt_cuda(const mbls_fr_t* input, int size, NTTDir dir, const mbls_fr_t* coset_gen,
                                      const NTTConfig* config, mbls_fr_t* output) {
    return ntt_call(input, size, dir, config, output, coset_gen);
}
eIcicleError bls12_381_field_ntt_cuda(const mbls_fr_t* input, int size, NTTDir dir, const NTTConfig* config,
                                      mbls_fr_t* output) {
    return ntt_call(input, size, dir, config, output, config ? &config->coset_gen : nullptr);
}
eIcicleError bls12_381_field_ntt_init_domain_cuda(const mbls_fr_t* root_of_unity, const NTTInitDomainConfig* config) {
    return ntt_init_domain(root_of_unity, config);
}
eIcicleError bls12_381_field_ntt_release_domain_cuda(void) { return ntt_release_domain(); }

// ICICLE get_root_of_unity_from_domain (registered as NttGetRouFromDomainImpl,
// icicle_backend_api.cuh:135-138): w_(2^logn) of the initialised domain, Montgomery form
eIcicleError bls12_381_ntt_get_rou_from_domain(uint64_t logn, mbls_fr_t* rou) {
    if (!rou) return MBLS_INVALID_POINTER;
    std::lock_guard<std::mutex> lk(g_domain_mu);
    Domain* dom = current_domain();
    if (!dom) return MBLS_INVALID_DEVICE;
    if (!dom->tables || logn > (uint64_t)dom->order_log) return MBLS_INVALID_ARGUMENT;
    canonical_omega(rou->limbs, (int)logn);
    return MBLS_SUCCESS;
}

}  // extern "C"
