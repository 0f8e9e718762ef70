// mbls_madchain.hpp -- one column of an unsaturated-radix product as ONE v_mad_u64_u32 chain.
//
// The radix-2^28 Fq (mbls_fq28.hpp) and radix-2^29 Fr (mbls_fr29.hpp) products accumulate each
// column in a single 64-bit register.  Written as C++ additions, LLVM reassociates every column
// into its own fresh chain (first product with a zero addend) and merges the previous column's
// carry with an extra 64-bit add at the end: one v_lshl_add_u64 per column (~27 per Fq product,
// ~17 per Fr product, 6-8% of the instructions; tools/isa counts in DESIGN.md).  The mads here are
// inline asm, up to 8 per statement, each accumulating into the operand the previous one wrote:
// asm statements are opaque to the reassociation, so the column stays the chain the formula is.
// The statements write a dummy SGPR pair (the carry-out v_mad_u64_u32 must name on gfx9) that is
// never read.  The compiler schedules and allocates around them as usual.
#pragma once
#include "mbls_common.hpp"

namespace mbls {
namespace madc {

#define MBLS_MADC_STEP(A, B) "v_mad_u64_u32 %0, %1, " A ", " B ", %0\n\t"
#define MBLS_MADC_1 MBLS_MADC_STEP("%2", "%3")
#define MBLS_MADC_2 MBLS_MADC_1 MBLS_MADC_STEP("%4", "%5")
#define MBLS_MADC_4 MBLS_MADC_2 MBLS_MADC_STEP("%6", "%7") MBLS_MADC_STEP("%8", "%9")
#define MBLS_MADC_8                                                                                                  \
    MBLS_MADC_4 MBLS_MADC_STEP("%10", "%11") MBLS_MADC_STEP("%12", "%13") MBLS_MADC_STEP("%14", "%15") \
        MBLS_MADC_STEP("%16", "%17")

// acc += sum a_k b_k over N = 1, 2, 4, 8 pairs; S: the b operands are wave-uniform constants (SGPRs)
template <bool S>
MBLS_DEV void mad1(uint64_t& acc, uint32_t a0, uint32_t b0) {
    uint64_t c;
    if constexpr (S)
        asm(MBLS_MADC_1 : "+v"(acc), "=&s"(c) : "v"(a0), "s"(b0));
    else
        asm(MBLS_MADC_1 : "+v"(acc), "=&s"(c) : "v"(a0), "v"(b0));
}
template <bool S>
MBLS_DEV void mad2(uint64_t& acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1) {
    uint64_t c;
    if constexpr (S)
        asm(MBLS_MADC_2 : "+v"(acc), "=&s"(c) : "v"(a0), "s"(b0), "v"(a1), "s"(b1));
    else
        asm(MBLS_MADC_2 : "+v"(acc), "=&s"(c) : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
}
template <bool S>
MBLS_DEV void mad4(uint64_t& acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2,
                   uint32_t a3, uint32_t b3) {
    uint64_t c;
    if constexpr (S)
        asm(MBLS_MADC_4 : "+v"(acc), "=&s"(c) : "v"(a0), "s"(b0), "v"(a1), "s"(b1), "v"(a2), "s"(b2), "v"(a3), "s"(b3));
    else
        asm(MBLS_MADC_4 : "+v"(acc), "=&s"(c) : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3));
}
template <bool S>
MBLS_DEV void mad8(uint64_t& acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2,
                   uint32_t a3, uint32_t b3, uint32_t a4, uint32_t b4, uint32_t a5, uint32_t b5, uint32_t a6,
                   uint32_t b6, uint32_t a7, uint32_t b7) {
    uint64_t c;
    if constexpr (S)
        asm(MBLS_MADC_8
            : "+v"(acc), "=&s"(c)
            : "v"(a0), "s"(b0), "v"(a1), "s"(b1), "v"(a2), "s"(b2), "v"(a3), "s"(b3), "v"(a4), "s"(b4), "v"(a5),
              "s"(b5), "v"(a6), "s"(b6), "v"(a7), "s"(b7));
    else
        asm(MBLS_MADC_8
            : "+v"(acc), "=&s"(c)
            : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3), "v"(a4), "v"(b4), "v"(a5),
              "v"(b5), "v"(a6), "v"(b6), "v"(a7), "v"(b7));
}
#undef MBLS_MADC_8
#undef MBLS_MADC_4
#undef MBLS_MADC_2
#undef MBLS_MADC_1
#undef MBLS_MADC_STEP

// acc += sum_{i = I..HI} x[i] y[K - i] (S: y holds compile-time constants -> SGPR operands)
template <int K, int I, int HI, bool S, class X, class Y>
MBLS_DEV void col(uint64_t& acc, const X& x, const Y& y) {
    if constexpr (I <= HI) {
        constexpr int R = HI - I + 1;
        if constexpr (R >= 8) {
            mad8<S>(acc, x[I], y[K - I], x[I + 1], y[K - I - 1], x[I + 2], y[K - I - 2], x[I + 3], y[K - I - 3], x[I + 4],
                    y[K - I - 4], x[I + 5], y[K - I - 5], x[I + 6], y[K - I - 6], x[I + 7], y[K - I - 7]);
            col<K, I + 8, HI, S>(acc, x, y);
        } else if constexpr (R >= 4) {
            mad4<S>(acc, x[I], y[K - I], x[I + 1], y[K - I - 1], x[I + 2], y[K - I - 2], x[I + 3], y[K - I - 3]);
            col<K, I + 4, HI, S>(acc, x, y);
        } else if constexpr (R >= 2) {
            mad2<S>(acc, x[I], y[K - I], x[I + 1], y[K - I - 1]);
            col<K, I + 2, HI, S>(acc, x, y);
        } else {
            mad1<S>(acc, x[I], y[K - I]);
        }
    }
}

// Two independent columns (A, B) interleaved inside one statement: A0 B0 A1 B1 ... -- each chain's
// dependent mads are two instructions apart, so a wave waits half as long on the 64-bit mad
// latency (round 6: two products of a butterfly / an addition that do not depend on each other)
#define MBLS_MADX_STEP(ACC, A, B) "v_mad_u64_u32 " ACC ", %2, " A ", " B ", " ACC "\n\t"
template <bool S>
MBLS_DEV void madx1(uint64_t& p, uint64_t& q, uint32_t a0, uint32_t b0, uint32_t c0, uint32_t d0) {
    uint64_t c;
    if constexpr (S)
        asm(MBLS_MADX_STEP("%0", "%3", "%4") MBLS_MADX_STEP("%1", "%5", "%6")
            : "+v"(p), "+v"(q), "=&s"(c) : "v"(a0), "s"(b0), "v"(c0), "s"(d0));
    else
        asm(MBLS_MADX_STEP("%0", "%3", "%4") MBLS_MADX_STEP("%1", "%5", "%6")
            : "+v"(p), "+v"(q), "=&s"(c) : "v"(a0), "v"(b0), "v"(c0), "v"(d0));
}
template <bool S>
MBLS_DEV void madx4(uint64_t& p, uint64_t& q, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2,
                    uint32_t b2, uint32_t a3, uint32_t b3, uint32_t c0, uint32_t d0, uint32_t c1, uint32_t d1,
                    uint32_t c2, uint32_t d2, uint32_t c3, uint32_t d3) {
    uint64_t c;
#define MBLS_MADX_4                                                                                                \
    MBLS_MADX_STEP("%0", "%3", "%4") MBLS_MADX_STEP("%1", "%11", "%12") MBLS_MADX_STEP("%0", "%5", "%6")             \
        MBLS_MADX_STEP("%1", "%13", "%14") MBLS_MADX_STEP("%0", "%7", "%8") MBLS_MADX_STEP("%1", "%15", "%16")       \
            MBLS_MADX_STEP("%0", "%9", "%10") MBLS_MADX_STEP("%1", "%17", "%18")
    if constexpr (S)
        asm(MBLS_MADX_4
            : "+v"(p), "+v"(q), "=&s"(c)
            : "v"(a0), "s"(b0), "v"(a1), "s"(b1), "v"(a2), "s"(b2), "v"(a3), "s"(b3), "v"(c0), "s"(d0), "v"(c1),
              "s"(d1), "v"(c2), "s"(d2), "v"(c3), "s"(d3));
    else
        asm(MBLS_MADX_4
            : "+v"(p), "+v"(q), "=&s"(c)
            : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3), "v"(c0), "v"(d0), "v"(c1),
              "v"(d1), "v"(c2), "v"(d2), "v"(c3), "v"(d3));
#undef MBLS_MADX_4
}
#undef MBLS_MADX_STEP

// p += sum_{i = I..HI} x[i] y[K - i], q += the same over (u, v): one interleaved chain pair
template <int K, int I, int HI, bool S, class X, class Y>
MBLS_DEV void col2(uint64_t& p, const X& x, const Y& y, uint64_t& q, const X& u, const Y& v) {
    if constexpr (I <= HI) {
        constexpr int R = HI - I + 1;
        if constexpr (R >= 4) {
            madx4<S>(p, q, x[I], y[K - I], x[I + 1], y[K - I - 1], x[I + 2], y[K - I - 2], x[I + 3], y[K - I - 3], u[I],
                     v[K - I], u[I + 1], v[K - I - 1], u[I + 2], v[K - I - 2], u[I + 3], v[K - I - 3]);
            col2<K, I + 4, HI, S>(p, x, y, q, u, v);
        } else {
            madx1<S>(p, q, x[I], y[K - I], u[I], v[K - I]);
            col2<K, I + 1, HI, S>(p, x, y, q, u, v);
        }
    }
}

}  // namespace madc
}  // namespace mbls
