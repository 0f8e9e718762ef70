// tests/diag/limbs_diag.hip -- test probe for the unsaturated-limb arithmetic (test infrastructure).
//
// Runs ONE operation of csrc/mbls_fq28.hpp (radix-2^28 Fq) or csrc/mbls_fr29.hpp (radix-2^29 Fr)
// on caller-chosen raw limbs -- including limbs at the maxima the headers' bound tables allow,
// which random canonical data never produces -- and returns the raw output limbs, so that
// tests/test_gpu_limbs.py can check every result against Python integers (congruence mod p / r
// and the documented output bounds).  The library code is compiled from the same headers the
// kernels use; nothing here is part of the product.
// Built by __graft_entry__.build(): hipcc -shared -fPIC ... -> tests/diag/liblimbs_diag.so
#include <hip/hip_runtime.h>

#include "mbls_fq28.hpp"
#include "mbls_fq2_28.hpp"
#include "mbls_fr29.hpp"

using namespace mbls;

static constexpr int IN_W = 8 * 16;  // words per case: 8 operands of up to 16 words
static constexpr int OUT_W = 64;     // words per case

MBLS_DEV r28::F28 f28(const uint32_t* p) {
    r28::F28 r;
#pragma unroll
    for (int i = 0; i < r28::NL; ++i) r.l[i] = p[i];
    return r;
}
MBLS_DEV void put28(uint32_t* o, const r28::F28& a) {
#pragma unroll
    for (int i = 0; i < r28::NL; ++i) o[i] = a.l[i];
}
MBLS_DEV r29::F29 f29(const uint32_t* p) {
    r29::F29 r;
#pragma unroll
    for (int i = 0; i < r29::NL; ++i) r.l[i] = p[i];
    return r;
}

// op codes (tests/test_gpu_limbs.py): operands are 16-word slots x0..x4 of the case
//   r28:  0 mul(x0, x1)   1 sqr(x0)   2 mul2(x0, x1, x2, x3)   3 fold(x0)   4 to_words(x0) (12 words)
//         5 carry(x0)   6 is_zero_mod(x0) (1 word)   7 madd(acc = x0, x1, x2; q = x3, x4): 42 words
//         8 mmadd(acc = x0, x1, one; q = x3, x4): 42 words + the flag
//   XYZZ: 9 xmadd(acc = x0..x3; q = x4, x5): 56 words   10 xmmadd(acc = x0, x1, one, one; q = x4, x5):
//         56 words + the flag   11 xadd(acc = x0..x3; partial x4..x7)   12 xdbl(x0..x3)
//         13 x_to_jac(x0..x3): 42 words   32-36: the pair-sliced forms of 9-13 (rows as 30 / 31)
//  r29: 20 mul(x0, x1)   21 unpack(words x0)   22 pack(x0) (8 words)   23 mul_words(words x0, x1)
//  pair-sliced Fq2 (mbls_fq2_28.hpp): rows 2i, 2i + 1 are the two lanes of case i (component 0, 1):
//       30 madd(acc = x0, x1, x2; q = x3, x4): 42 words + the flag   31 mmadd(acc = x0, x1; q = x3, x4)
__global__ void k_limbs(int op, const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t* x = in + (size_t)t * IN_W;
    uint32_t* o = out + (size_t)t * OUT_W;
    switch (op) {
        case 0: put28(o, r28::mul(f28(x), f28(x + 16))); break;
        case 1: put28(o, r28::sqr(f28(x))); break;
        case 2: put28(o, r28::mul2(f28(x), f28(x + 16), f28(x + 32), f28(x + 48))); break;
        case 3: put28(o, r28::fold(f28(x))); break;
        case 4: {
            uint32_t w[12];
            r28::to_words(f28(x), w);
            for (int i = 0; i < 12; ++i) o[i] = w[i];
            break;
        }
        case 5: put28(o, r28::carry(f28(x))); break;
        case 6: o[0] = r28::is_zero_mod(f28(x)) ? 1u : 0u; break;
        case 7: {
            r28::J28 acc{f28(x), f28(x + 16), f28(x + 32)};
            r28::madd(acc, f28(x + 48), f28(x + 64));
            put28(o, acc.x);
            put28(o + 14, acc.y);
            put28(o + 28, acc.z);
            break;
        }
        case 8: {
            r28::J28 acc{f28(x), f28(x + 16), r28::F28::one()};
            const bool done = r28::mmadd(acc, f28(x + 48), f28(x + 64));
            put28(o, acc.x);
            put28(o + 14, acc.y);
            put28(o + 28, acc.z);
            o[42] = done ? 1u : 0u;
            break;
        }
        case 9:
        case 10:
        case 11:
        case 12:
        case 13: {
            r28::X28 acc{f28(x), f28(x + 16), op == 10 ? r28::F28::one() : f28(x + 32),
                         op == 10 ? r28::F28::one() : f28(x + 48)};
            bool done = true;
            if (op == 9) r28::xmadd(acc, f28(x + 64), f28(x + 80));
            if (op == 10) done = r28::xmmadd(acc, f28(x + 64), f28(x + 80));
            if (op == 11) r28::xadd(acc, f28(x + 64), f28(x + 80), f28(x + 96), f28(x + 112));
            if (op == 12) r28::xdbl(acc);
            if (op == 13) {
                const r28::J28 j = r28::x_to_jac(acc);
                put28(o, j.x);
                put28(o + 14, j.y);
                put28(o + 28, j.z);
                break;
            }
            put28(o, acc.x);
            put28(o + 14, acc.y);
            put28(o + 28, acc.zz);
            put28(o + 42, acc.zzz);
            if (op == 10) o[56] = done ? 1u : 0u;
            break;
        }
        case 20: {
            const r29::F29 r = r29::mul(f29(x), f29(x + 16));
            for (int i = 0; i < r29::NL; ++i) o[i] = r.l[i];
            break;
        }
        case 21: {
            Fr a;
            for (int i = 0; i < 8; ++i) a.v[i] = x[i];
            const r29::F29 r = r29::unpack(a);
            for (int i = 0; i < r29::NL; ++i) o[i] = r.l[i];
            break;
        }
        case 22: {
            const Fr r = r29::pack(f29(x));
            for (int i = 0; i < 8; ++i) o[i] = r.v[i];
            break;
        }
        case 23: {
            Fr a;
            for (int i = 0; i < 8; ++i) a.v[i] = x[i];
            const Fr r = r29::mul_words(a, f29(x + 16));
            for (int i = 0; i < 8; ++i) o[i] = r.v[i];
            break;
        }
        case 30:
        case 31: {
            r28p::J28p acc{f28(x), f28(x + 16), op == 30 ? f28(x + 32) : r28p::one()};
            const bool done = op == 30 ? r28p::madd(acc, f28(x + 48), f28(x + 64)) : r28p::mmadd(acc, f28(x + 48), f28(x + 64));
            put28(o, acc.x);
            put28(o + 14, acc.y);
            put28(o + 28, acc.z);
            o[42] = done ? 1u : 0u;
            break;
        }
        case 32:
        case 33:
        case 34:
        case 35:
        case 36: {  // pair-sliced XYZZ (G2): as 9 / 10 / 11 / 12 / 13, rows 2i, 2i + 1 = the pair's lanes
            r28p::X28p acc{f28(x), f28(x + 16), op == 33 ? r28p::one() : f28(x + 32), op == 33 ? r28p::one() : f28(x + 48)};
            bool done = true;
            if (op == 32) r28p::xmadd(acc, f28(x + 64), f28(x + 80));
            if (op == 33) done = r28p::xmmadd(acc, f28(x + 64), f28(x + 80));
            if (op == 34) r28p::xadd(acc, f28(x + 64), f28(x + 80), f28(x + 96), f28(x + 112));
            if (op == 35) r28p::xdbl(acc);
            if (op == 36) {
                const r28p::J28p j = r28p::x_to_jac(acc);
                put28(o, j.x);
                put28(o + 14, j.y);
                put28(o + 28, j.z);
                break;
            }
            put28(o, acc.x);
            put28(o + 14, acc.y);
            put28(o + 28, acc.zz);
            put28(o + 42, acc.zzz);
            if (op == 33) o[56] = done ? 1u : 0u;
            break;
        }
        default: o[0] = 0xdeadbeefu; break;
    }
}

extern "C" {
// n cases of IN_W input words -> n cases of OUT_W output words (host arrays); 0 on success
int limbs_diag_run(int op, const uint32_t* in, uint32_t* out, int n) {
    if (n <= 0 || !in || !out) return -1;
    uint32_t *d_in = nullptr, *d_out = nullptr;
    const size_t bi = (size_t)n * IN_W * 4, bo = (size_t)n * OUT_W * 4;
    if (hipMalloc(&d_in, bi) != hipSuccess) return -2;
    if (hipMalloc(&d_out, bo) != hipSuccess) {
        (void)hipFree(d_in);
        return -2;
    }
    int rc = 0;
    if (hipMemcpy(d_in, in, bi, hipMemcpyHostToDevice) != hipSuccess || hipMemset(d_out, 0, bo) != hipSuccess) rc = -3;
    if (!rc) {
        hipLaunchKernelGGL(k_limbs, dim3((n + 127) / 128), dim3(128), 0, 0, op, d_in, d_out, n);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = -4;
    }
    if (!rc && hipMemcpy(out, d_out, bo, hipMemcpyDeviceToHost) != hipSuccess) rc = -5;
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return rc;
}
int limbs_diag_in_words(void) { return IN_W; }
int limbs_diag_out_words(void) { return OUT_W; }
}
