// vecops.hip -- element-wise Fr vector operations (HBM-streaming kernels).
//
// Reference: kernels bls12-381/src/field/vec_ops.cu:63-118,335-345, boundary wrappers
// icicle_field_api.cu:133-334 (run_vec_op, scalar_*_vec_cuda_impl) and the exported C entry
// points vec_ops.cu:393-476 (vec_*_cuda) and :693-840 (bls12_381_vector_*).
//
// Algorithmic traffic: add/sub/mul 96 B per element (2 x 32 B read, 32 B write), scalar ops
// 64 B per element.  One thread per element, 32-byte coalesced loads as 2 x dwordx4,
// grid-stride over a grid sized to keep every CU busy.  add/sub are HBM-bound; mul is one
// Montgomery product (Fr, 8 x u32 words) per 96 B -- VALU-bound below ~16 Fr-mul/B... see
// DESIGN.md for the measured rates.
#include <hip/hip_runtime.h>

#include <optional>

#include <algorithm>

#include "mbls_common.hpp"
#include "mbls_field.hpp"

namespace mbls {

enum class VecOp { Add, Sub, Mul, ScalarMul, ScalarAdd };

// VEC_U elements per thread per step, from a workgroup tile of VEC_U x 256 contiguous elements,
// all loads issued before the arithmetic.  Measured (tools/vec_probe.py, add / mul 2^24, one box):
// tiles of 2 5.53 / 5.46-5.48 TB/s, 1 5.41-5.44 / 5.34-5.36, 4 5.45-5.47 / 5.44-5.45; 4 elements
// strided by the grid (not contiguous) fell to 3.98 TB/s for add.
#ifndef MBLS_VEC_U
#define MBLS_VEC_U 2
#endif
static constexpr int VEC_U = MBLS_VEC_U;
template <VecOp OP>
MBLS_DEV Fr vec_apply(const Fr& x, const Fr& y, const Fr& s) {
    if constexpr (OP == VecOp::Add) return x + y;
    if constexpr (OP == VecOp::Sub) return x - y;
    if constexpr (OP == VecOp::Mul) return x * y;
    if constexpr (OP == VecOp::ScalarMul) return s * y;
    return s + y;
}
template <VecOp OP>
__global__ __launch_bounds__(256) void k_vecop(uint8_t* __restrict__ out, const uint8_t* __restrict__ a,
                                               const uint8_t* __restrict__ b, Fr s, size_t n) {
    constexpr bool TWO = OP == VecOp::Add || OP == VecOp::Sub || OP == VecOp::Mul;
    // workgroup tiles of VEC_U x 256 contiguous elements (element u of a tile at u * 256 + lane)
    const size_t tile = (size_t)VEC_U * blockDim.x;
    size_t t0 = blockIdx.x * tile;
    for (; t0 + tile <= n; t0 += (size_t)gridDim.x * tile) {
        Fr x[VEC_U], y[VEC_U];
#pragma unroll
        for (int u = 0; u < VEC_U; ++u) {
            const size_t e = t0 + u * blockDim.x + threadIdx.x;
            y[u] = load<FrCfg>(b + 32 * e);
            if constexpr (TWO) x[u] = load<FrCfg>(a + 32 * e);
        }
#pragma unroll
        for (int u = 0; u < VEC_U; ++u)
            store<FrCfg>(out + 32 * (t0 + u * blockDim.x + threadIdx.x), vec_apply<OP>(x[u], y[u], s));
    }
    // the last, partial tile (one workgroup): element by element
    if (t0 >= n) return;
    size_t i = t0 + threadIdx.x;
    for (; i < n; i += blockDim.x) {
        const Fr y = load<FrCfg>(b + 32 * i);
        Fr x;
        if constexpr (TWO) x = load<FrCfg>(a + 32 * i);
        store<FrCfg>(out + 32 * i, vec_apply<OP>(x, y, s));
    }
}

// batched scalar ops: scalar k of `sv` (device) applies to batch member k; member of element
// i is i / size (row layout) or i % batch (columns_batch: element j of member k at j*batch+k)
template <VecOp OP>
__global__ __launch_bounds__(256) void k_scalar_batch(uint8_t* __restrict__ out, const uint8_t* __restrict__ sv,
                                                      const uint8_t* __restrict__ b, size_t size, uint32_t batch,
                                                      int cols, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        const size_t k = cols ? i % batch : i / size;
        const Fr s = load<FrCfg>(sv + 32 * k);
        const Fr y = load<FrCfg>(b + 32 * i);
        store<FrCfg>(out + 32 * i, OP == VecOp::ScalarMul ? s * y : s + y);
    }
}

// ---- sum reduction (vec_ops.cu:350-382, 479-524): per-block LDS tree, then one block
__global__ __launch_bounds__(256) void k_sum_partial(uint8_t* __restrict__ out, const uint8_t* __restrict__ in,
                                                     size_t n) {
    __shared__ __attribute__((aligned(16))) uint8_t sh[256 * 32];
    Fr acc = Fr::zero();
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc = acc + load<FrCfg>(in + 32 * i);
    store<FrCfg>(sh + 32 * threadIdx.x, acc);
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            acc = acc + load<FrCfg>(sh + 32 * (threadIdx.x + s));
            store<FrCfg>(sh + 32 * threadIdx.x, acc);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) store<FrCfg>(out + 32 * blockIdx.x, acc);
}

// ---- batch inversion (vec_ops.cu:606-673 batch_inv_cuda): Montgomery's trick per thread
// over a contiguous chunk, one inversion per chunk; zero inputs map to zero (field_inv
// semantics, field.cuh:750-900).  `out` holds the prefix products between the two sweeps.
// The inputs can be witness-derived scalars, so this path keeps the reference's constant-time
// shape: the chunk inversion is the fixed Fermat chain a^(r-2) (field.cuh:735-900; not the
// variable-time binary GCD of inv()), and zero inputs are handled by selects, not branches.
static constexpr int INV_CHUNK = 64;
// c ? a : b with a full-word mask (no data-dependent branch, whatever the compiler
// would make of a ternary); the zero test is an OR-reduction, not an early-exit compare
MBLS_DEV uint32_t zero_mask(const Fr& x) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) o |= x.v[i];
    return 0u - (uint32_t)(o == 0u);  // all ones iff x == 0
}
MBLS_DEV Fr fr_select(uint32_t mask, const Fr& a, const Fr& b) {
    Fr r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = (a.v[i] & mask) | (b.v[i] & ~mask);
    return r;
}
__global__ __launch_bounds__(256) void k_batch_inv(uint8_t* __restrict__ out, const uint8_t* __restrict__ in,
                                                   size_t n) {
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t s = t * INV_CHUNK;
    if (s >= n) return;
    const size_t e = s + INV_CHUNK < n ? s + INV_CHUNK : n;
    Fr acc = Fr::one();
    for (size_t i = s; i < e; ++i) {
        const Fr x = load<FrCfg>(in + 32 * i);
        store<FrCfg>(out + 32 * i, acc);
        acc = fr_select(zero_mask(x), acc, acc * x);
    }
    Fr inv_acc = inv_fermat(acc);
    for (size_t i = e; i-- > s;) {
        const Fr x = load<FrCfg>(in + 32 * i);
        const uint32_t z = zero_mask(x);
        store<FrCfg>(out + 32 * i, fr_select(z, Fr::zero(), inv_acc * load<FrCfg>(out + 32 * i)));
        inv_acc = fr_select(z, inv_acc, inv_acc * x);
    }
}

static int vec_grid(size_t n) {
    size_t blocks = (n + 255) / 256;
    const size_t cap = 256 * 16;  // 16 workgroups per CU, grid-stride beyond
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    return (int)blocks;
}

template <VecOp OP>
static eIcicleError launch(uint8_t* out, const uint8_t* a, const uint8_t* b, const Fr& s, size_t n, hipStream_t st) {
    if (n == 0) return MBLS_SUCCESS;
    hipLaunchKernelGGL(k_vecop<OP>, dim3(vec_grid(n)), dim3(256), 0, st, out, a, b, s, n);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

static Fr fr_from_host(const mbls_fr_t* p) {
    Fr s;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p->limbs);
    for (int i = 0; i < 8; ++i) s.v[i] = w[i];
    return s;
}

// Staged wrapper with the reference run_vec_op placement semantics
// (icicle_field_api.cu:133-192): host operands are copied in, host results copied out,
// synchronise unless is_async.  Scratch comes from the stream arena (no per-call hipMalloc).
template <VecOp OP>
static eIcicleError run_vec_op(const mbls_fr_t* a, const mbls_fr_t* b, size_t size, const VecOpsConfig* cfg,
                               mbls_fr_t* output) {
    if (!cfg || !b || !output || (!a && OP != VecOp::ScalarMul && OP != VecOp::ScalarAdd))
        return MBLS_INVALID_POINTER;
    constexpr bool scalar_op = (OP == VecOp::ScalarMul || OP == VecOp::ScalarAdd);
    if (scalar_op && !a) return MBLS_INVALID_POINTER;
    hipStream_t st = static_cast<hipStream_t>(cfg->stream);
    int batch = cfg->batch_size > 0 ? cfg->batch_size : 1;
    size_t total = size * (size_t)batch;
    if (total == 0) return MBLS_SUCCESS;
    const size_t bytes = total * 32;

    size_t need = 0;
    if (!scalar_op && !cfg->is_a_on_device) need += align_up(bytes);
    if (!cfg->is_b_on_device) need += align_up(bytes);
    if (!cfg->is_result_on_device) need += align_up(bytes);
    if (scalar_op && !cfg->is_a_on_device) need += align_up(32 * (size_t)batch);
    // device operands need no scratch: no context lease, hence no `done` event (an event marker
    // holds the next dispatch ~5 us)
    std::optional<CtxLease> lease;
    Arena* arena = nullptr;
    eIcicleError er = MBLS_SUCCESS;
    if (need) {
        lease.emplace(st);
        if (!*lease) return lease->error();
        if ((er = lease->reserve(need)) != MBLS_SUCCESS) return er;
        arena = &(**lease).arena;
    }

    const uint8_t* da = reinterpret_cast<const uint8_t*>(a);
    const uint8_t* db = reinterpret_cast<const uint8_t*>(b);
    uint8_t* dout = reinterpret_cast<uint8_t*>(output);
    if (!scalar_op && !cfg->is_a_on_device) {
        void* t = arena->take(bytes);
        MBLS_TRY(hipMemcpyAsync(t, a, bytes, hipMemcpyHostToDevice, st));
        da = static_cast<const uint8_t*>(t);
    }
    if (!cfg->is_b_on_device) {
        void* t = arena->take(bytes);
        MBLS_TRY(hipMemcpyAsync(t, b, bytes, hipMemcpyHostToDevice, st));
        db = static_cast<const uint8_t*>(t);
    }
    if (!cfg->is_result_on_device) dout = static_cast<uint8_t*>(arena->take(bytes));

    if (scalar_op) {
        // one scalar per batch entry (ICICLE v4 batched scalar ops), read on device
        const uint8_t* sv = reinterpret_cast<const uint8_t*>(a);
        if (!cfg->is_a_on_device) {
            void* t = arena->take(32 * (size_t)batch);
            MBLS_TRY(hipMemcpyAsync(t, a, 32 * (size_t)batch, hipMemcpyHostToDevice, st));
            sv = static_cast<const uint8_t*>(t);
        }
        hipLaunchKernelGGL(k_scalar_batch<OP>, dim3(vec_grid(total)), dim3(256), 0, st, dout, sv, db, size,
                           (uint32_t)batch, cfg->columns_batch ? 1 : 0, total);
        MBLS_TRY(hipGetLastError());
    } else {
        er = launch<OP>(dout, da, db, Fr{}, total, st);
        if (er != MBLS_SUCCESS) return er;
    }
    if (!cfg->is_result_on_device) MBLS_TRY(hipMemcpyAsync(output, dout, bytes, hipMemcpyDeviceToHost, st));
    // staged host inputs are copied out of the caller's memory before hipMemcpyAsync returns
    // (pageable) or are the caller's to keep alive (pinned, as in ICICLE): only a host result
    // forces the wait
    if (!cfg->is_async || !cfg->is_result_on_device) MBLS_TRY(hipStreamSynchronize(st));
    return MBLS_SUCCESS;
}

// sums of `batch` row-major members of `size` elements each -> output[0 .. batch) (device
// or host per is_result_on_device); input on the host or the device per is_a_on_device
static eIcicleError vec_sum(mbls_fr_t* output, const mbls_fr_t* input, size_t size, int batch, const VecOpsConfig* cfg) {
    if (!output || !input || !cfg) return MBLS_INVALID_POINTER;
    if (batch < 1) batch = 1;
    hipStream_t st = static_cast<hipStream_t>(cfg->stream);
    CtxLease lease(st);
    if (!lease) return lease.error();
    StreamCtx& ctx = *lease;
    const int blocks = size > 0 ? std::min(vec_grid(size), 1024) : 1;
    const size_t in_bytes = 32 * size * (size_t)batch;
    const bool stage = !cfg->is_a_on_device && in_bytes;
    eIcicleError er = lease.reserve(align_up(32 * (size_t)blocks) + align_up(32 * (size_t)batch) +
                                    (stage ? align_up(in_bytes) : 0));
    if (er != MBLS_SUCCESS) return er;
    uint8_t* part = static_cast<uint8_t*>(ctx.arena.take(32 * (size_t)blocks));
    uint8_t* res = static_cast<uint8_t*>(ctx.arena.take(32 * (size_t)batch));
    const uint8_t* src = reinterpret_cast<const uint8_t*>(input);
    if (stage) {
        void* t = ctx.arena.take(in_bytes);
        MBLS_TRY(hipMemcpyAsync(t, input, in_bytes, hipMemcpyHostToDevice, st));
        src = static_cast<const uint8_t*>(t);
    }
    for (int k = 0; k < batch; ++k) {
        hipLaunchKernelGGL(k_sum_partial, dim3(blocks), dim3(256), 0, st, part, src + 32 * size * (size_t)k, size);
        hipLaunchKernelGGL(k_sum_partial, dim3(1), dim3(256), 0, st, res + 32 * (size_t)k, part, (size_t)blocks);
    }
    MBLS_TRY(hipGetLastError());
    MBLS_TRY(hipMemcpyAsync(output, res, 32 * (size_t)batch,
                            cfg->is_result_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, st));
    if (!cfg->is_async || !cfg->is_result_on_device) MBLS_TRY(hipStreamSynchronize(st));
    return MBLS_SUCCESS;
}

// element-wise inverses of `size` device elements into device `output` (in place allowed:
// the inputs are then copied aside, since `output` holds the prefix products)
static eIcicleError batch_inv(mbls_fr_t* output, const mbls_fr_t* input, int size, const VecOpsConfig* cfg) {
    if (!output || !input) return MBLS_INVALID_POINTER;
    if (size < 0) return MBLS_INVALID_ARGUMENT;
    if (size == 0) return MBLS_SUCCESS;
    hipStream_t st = cfg ? static_cast<hipStream_t>(cfg->stream) : nullptr;
    const uint8_t* in = reinterpret_cast<const uint8_t*>(input);
    uint8_t* out = reinterpret_cast<uint8_t*>(output);
    CtxLease lease(st);
    if (!lease) return lease.error();
    StreamCtx& ctx = *lease;
    if (in == out) {  // in place: keep a copy of the inputs for the backward sweep
        eIcicleError er = lease.reserve(align_up(32 * (size_t)size));
        if (er != MBLS_SUCCESS) return er;
        uint8_t* t = static_cast<uint8_t*>(ctx.arena.take(32 * (size_t)size));
        MBLS_TRY(hipMemcpyAsync(t, in, 32 * (size_t)size, hipMemcpyDeviceToDevice, st));
        in = t;
    }
    const size_t threads = ((size_t)size + INV_CHUNK - 1) / INV_CHUNK;
    hipLaunchKernelGGL(k_batch_inv, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, out, in, (size_t)size);
    MBLS_TRY(hipGetLastError());
    if (!cfg || !cfg->is_async) MBLS_TRY(hipStreamSynchronize(st));
    return MBLS_SUCCESS;
}

// device-pointer entry points (vec_ops.cu:393-476): no staging, enqueue only
template <VecOp OP>
static eIcicleError raw_vec_op(mbls_fr_t* output, const mbls_fr_t* a, const mbls_fr_t* b, int size,
                               const VecOpsConfig* cfg) {
    if (!output || !a || !b) return MBLS_INVALID_POINTER;
    if (size < 0) return MBLS_INVALID_ARGUMENT;
    hipStream_t st = cfg ? static_cast<hipStream_t>(cfg->stream) : nullptr;
    constexpr bool scalar_op = (OP == VecOp::ScalarMul || OP == VecOp::ScalarAdd);
    Fr s{};
    if (scalar_op) s = fr_from_host(a);
    eIcicleError er = launch<OP>(reinterpret_cast<uint8_t*>(output), scalar_op ? nullptr : reinterpret_cast<const uint8_t*>(a),
                                 reinterpret_cast<const uint8_t*>(b), s, (size_t)size, st);
    if (er != MBLS_SUCCESS) return er;
    if (cfg && !cfg->is_async) MBLS_TRY(hipStreamSynchronize(st));
    return MBLS_SUCCESS;
}

}  // namespace mbls

using namespace mbls;

extern "C" {

eIcicleError bls12_381_vector_add(const mbls_fr_t* a, const mbls_fr_t* b, size_t size, const VecOpsConfig* config,
                                  mbls_fr_t* output) {
    return run_vec_op<VecOp::Add>(a, b, size, config, output);
}
eIcicleError bls12_381_vector_sub(const mbls_fr_t* a, const mbls_fr_t* b, size_t size, const VecOpsConfig* config,
                                  mbls_fr_t* output) {
    return run_vec_op<VecOp::Sub>(a, b, size, config, output);
}
eIcicleError bls12_381_vector_mul(const mbls_fr_t* a, const mbls_fr_t* b, size_t size, const VecOpsConfig* config,
                                  mbls_fr_t* output) {
    return run_vec_op<VecOp::Mul>(a, b, size, config, output);
}
eIcicleError bls12_381_scalar_mul_vec(const mbls_fr_t* scalar, const mbls_fr_t* vec, size_t size,
                                      const VecOpsConfig* config, mbls_fr_t* output) {
    return run_vec_op<VecOp::ScalarMul>(scalar, vec, size, config, output);
}
eIcicleError bls12_381_scalar_add_vec(const mbls_fr_t* scalar, const mbls_fr_t* vec, size_t size,
                                      const VecOpsConfig* config, mbls_fr_t* output) {
    return run_vec_op<VecOp::ScalarAdd>(scalar, vec, size, config, output);
}

eIcicleError vec_add_cuda(mbls_fr_t* output, const mbls_fr_t* a, const mbls_fr_t* b, int size, const VecOpsConfig* config) {
    return raw_vec_op<VecOp::Add>(output, a, b, size, config);
}
eIcicleError vec_sub_cuda(mbls_fr_t* output, const mbls_fr_t* a, const mbls_fr_t* b, int size, const VecOpsConfig* config) {
    return raw_vec_op<VecOp::Sub>(output, a, b, size, config);
}
eIcicleError vec_mul_cuda(mbls_fr_t* output, const mbls_fr_t* a, const mbls_fr_t* b, int size, const VecOpsConfig* config) {
    return raw_vec_op<VecOp::Mul>(output, a, b, size, config);
}
eIcicleError scalar_mul_vec_cuda(mbls_fr_t* output, const mbls_fr_t* scalar, const mbls_fr_t* vec, int size,
                                 const VecOpsConfig* config) {
    return raw_vec_op<VecOp::ScalarMul>(output, scalar, vec, size, config);
}
eIcicleError scalar_add_vec_cuda(mbls_fr_t* output, const mbls_fr_t* scalar, const mbls_fr_t* vec, int size,
                                 const VecOpsConfig* config) {
    return raw_vec_op<VecOp::ScalarAdd>(output, scalar, vec, size, config);
}
eIcicleError vec_sum_cuda(mbls_fr_t* output, const mbls_fr_t* input, int size, const VecOpsConfig* config) {
    if (size < 0) return MBLS_INVALID_ARGUMENT;
    if (!config) return MBLS_INVALID_POINTER;
    VecOpsConfig c = *config;
    c.is_a_on_device = true;  // the device-pointer entry point (vec_ops.cu:479-524)
    return vec_sum(output, input, (size_t)size, 1, &c);
}
eIcicleError bls12_381_vector_sum(const mbls_fr_t* a, size_t size, const VecOpsConfig* config, mbls_fr_t* output) {
    if (!config) return MBLS_INVALID_POINTER;
    if (config->columns_batch) return MBLS_API_NOT_IMPLEMENTED;
    return vec_sum(output, a, size, config->batch_size > 0 ? config->batch_size : 1, config);
}
eIcicleError bls12_381_batch_inv_cuda(mbls_fr_t* output, const mbls_fr_t* input, int size, const VecOpsConfig* config) {
    return batch_inv(output, input, size, config);
}

}  // extern "C"
