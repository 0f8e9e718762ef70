// h2dbench.hip -- host -> device staging of an MSM's scalars (32 MiB at 2^20):
// hipMemcpyAsync from pinned and from pageable memory against copy kernels that read the pinned
// buffer through its device alias, with several grid sizes / loads in flight.  hipEvent timing,
// median of 9 after 2 warmups.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

template <int U>
__global__ __launch_bounds__(256) void k_copy(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = src[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) dst[i + u * stride] = v[u];
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

template <class F>
static float med_ms(hipStream_t st, F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 2; ++i) f();
    std::vector<float> v;
    for (int r = 0; r < 9; ++r) {
        CK(hipEventRecord(a, st));
        f();
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[4];
}

int main() {
    const size_t bytes = 32u << 20;
    const size_t n16 = bytes / 16;
    void *pinned, *dev;
    CK(hipHostMalloc(&pinned, bytes, hipHostMallocDefault));
    void* pageable = malloc(bytes);
    memset(pinned, 1, bytes);
    memset(pageable, 1, bytes);
    CK(hipMalloc(&dev, bytes));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipPointerAttribute_t at;
    CK(hipPointerGetAttributes(&at, pinned));
    const uint4* alias = (const uint4*)at.devicePointer;
    printf("pinned host %p device alias %p type %d\n", pinned, (void*)alias, (int)at.type);
    auto gbs = [&](float ms) { return bytes / (ms * 1e-3) / 1e9; };
    float t;
    t = med_ms(st, [&] { CK(hipMemcpyAsync(dev, pinned, bytes, hipMemcpyHostToDevice, st)); });
    printf("hipMemcpyAsync pinned H2D        %.3f ms  %.1f GB/s\n", t, gbs(t));
    t = med_ms(st, [&] { CK(hipMemcpyAsync(dev, pinned, bytes, hipMemcpyDefault, st)); });
    printf("hipMemcpyAsync pinned Default    %.3f ms  %.1f GB/s\n", t, gbs(t));
    t = med_ms(st, [&] { CK(hipMemcpyAsync(dev, pageable, bytes, hipMemcpyHostToDevice, st)); });
    printf("hipMemcpyAsync pageable H2D      %.3f ms  %.1f GB/s\n", t, gbs(t));
    for (int blocks : {256, 512, 1024, 2048, 4096, 8192}) {
        t = med_ms(st, [&] { hipLaunchKernelGGL(k_copy<4>, dim3(blocks), dim3(256), 0, st, (uint4*)dev, alias, n16); });
        printf("k_copy<4> %5d blocks            %.3f ms  %.1f GB/s\n", blocks, t, gbs(t));
    }
    for (int blocks : {1024, 2048, 4096}) {
        t = med_ms(st, [&] { hipLaunchKernelGGL(k_copy<1>, dim3(blocks), dim3(256), 0, st, (uint4*)dev, alias, n16); });
        printf("k_copy<1> %5d blocks            %.3f ms  %.1f GB/s\n", blocks, t, gbs(t));
        t = med_ms(st, [&] { hipLaunchKernelGGL(k_copy<8>, dim3(blocks), dim3(256), 0, st, (uint4*)dev, alias, n16); });
        printf("k_copy<8> %5d blocks            %.3f ms  %.1f GB/s\n", blocks, t, gbs(t));
    }
    // chunked async copies (4 x 8 MiB)
    t = med_ms(st, [&] {
        for (int k = 0; k < 4; ++k)
            CK(hipMemcpyAsync((char*)dev + k * (bytes / 4), (char*)pinned + k * (bytes / 4), bytes / 4,
                              hipMemcpyHostToDevice, st));
    });
    printf("hipMemcpyAsync pinned 4 chunks   %.3f ms  %.1f GB/s\n", t, gbs(t));
    CK(hipStreamSynchronize(st));
    printf("h2dbench done\n");
    return 0;
}
