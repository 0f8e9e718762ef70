// common.cpp -- error mapping, scratch arenas, configs, version.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "mbls_common.hpp"

namespace mbls {

bool trace_enabled() {
    static int v = -1;
    if (v < 0) {
        const char* s = getenv("MBLS_TRACE");
        v = (s && *s && *s != '0') ? 1 : 0;
    }
    return v == 1;
}

eIcicleError map_hip_error(hipError_t e, const char* what) {
    if (trace_enabled()) fprintf(stderr, "[mbls] HIP error %s in %s\n", hipGetErrorString(e), what);
    switch (e) {
        case hipErrorOutOfMemory: return MBLS_OUT_OF_MEMORY;
        case hipErrorInvalidDevice:
        case hipErrorNoDevice: return MBLS_INVALID_DEVICE;
        case hipErrorInvalidValue: return MBLS_INVALID_ARGUMENT;
        case hipErrorInvalidDevicePointer: return MBLS_INVALID_POINTER;
        default: return MBLS_UNKNOWN_ERROR;
    }
}

Arena::~Arena() {
    // Arenas live for the process; freeing at exit races with runtime teardown, so leak.
}

eIcicleError Arena::reserve(size_t bytes) {
    bytes = align_up(bytes);
    if (bytes <= cap_) return MBLS_SUCCESS;
    size_t ncap = bytes + bytes / 4;
    void* p = nullptr;
    if (base_) {
        // older work on this stream may still read the old block: free it in stream order
        hipError_t e = hipStreamSynchronize(stream_);
        if (e != hipSuccess) return map_hip_error(e, "arena sync");
        (void)hipFree(base_);
        base_ = nullptr;
        cap_ = 0;
    }
    hipError_t e = hipMalloc(&p, ncap);
    if (e != hipSuccess) return map_hip_error(e, "arena hipMalloc");
    base_ = p;
    cap_ = ncap;
    used_ = 0;
    return MBLS_SUCCESS;
}

void* Arena::take(size_t bytes) {
    bytes = align_up(bytes);
    if (used_ + bytes > cap_) return nullptr;
    void* p = static_cast<char*>(base_) + used_;
    used_ += bytes;
    return p;
}

StreamCtx& stream_ctx(hipStream_t s) {
    static std::mutex g;
    static std::map<std::pair<int, hipStream_t>, std::unique_ptr<StreamCtx>> tab;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g);
    auto key = std::make_pair(dev, s);
    auto it = tab.find(key);
    if (it == tab.end()) it = tab.emplace(key, std::unique_ptr<StreamCtx>(new StreamCtx(s))).first;
    return *it->second;
}

static bool side_priority() {
    static const bool v = [] {
        const char* e = getenv("MBLS_SIDE_PRIO");
        return e ? atoi(e) != 0 : true;
    }();
    return v;
}

eIcicleError StreamCtx::ensure_side(size_t nevents, size_t nsides) {
    while (sides.size() < nsides) {
        hipStream_t s;
        // highest priority: the side streams carry the latency-bound tails that must not queue
        // behind the main stream's accumulation workgroups
        int least = 0, greatest = 0;
        MBLS_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        MBLS_TRY(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, side_priority() ? greatest : least));
        sides.push_back(s);
    }
    while (events.size() < nevents) {
        hipEvent_t e;
        MBLS_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        events.push_back(e);
    }
    return MBLS_SUCCESS;
}

eIcicleError StreamCtx::ensure_pipe() {
    for (int k = 0; k < 2; ++k)
        if (!pipe[k]) MBLS_TRY(hipStreamCreateWithFlags(&pipe[k], hipStreamNonBlocking));
    for (int k = 0; k < 3; ++k)
        if (!pipe_ev[k]) MBLS_TRY(hipEventCreateWithFlags(&pipe_ev[k], hipEventDisableTiming));
    for (int k = 0; k < 2; ++k)
        if (!acc_ev[k]) MBLS_TRY(hipEventCreateWithFlags(&acc_ev[k], hipEventDisableTiming));
    return MBLS_SUCCESS;
}

bool is_device_pointer(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

static std::mutex g_prof_mu;
static int g_prof_on = -1;
struct ProfEntry {
    std::string name;
    hipEvent_t a, b;
};
static std::vector<ProfEntry> g_prof_pending;
static std::map<std::string, std::pair<double, long>> g_prof_sum;

bool profile_enabled() {
    if (g_prof_on < 0) {
        const char* s = getenv("MBLS_PROFILE");
        g_prof_on = (s && *s && *s != '0') ? 1 : 0;
    }
    return g_prof_on == 1;
}

void profile_record(const char* name, hipEvent_t a, hipEvent_t b) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_pending.push_back({name, a, b});
}

static void profile_drain() {
    for (auto& e : g_prof_pending) {
        float ms = 0.f;
        (void)hipEventSynchronize(e.b);
        (void)hipEventElapsedTime(&ms, e.a, e.b);
        auto& s = g_prof_sum[e.name];
        s.first += ms;
        s.second += 1;
        (void)hipEventDestroy(e.a);
        (void)hipEventDestroy(e.b);
    }
    g_prof_pending.clear();
}

}  // namespace mbls

extern "C" {

void mbls_profile_enable(int on) {
    std::lock_guard<std::mutex> lk(mbls::g_prof_mu);
    mbls::g_prof_on = on ? 1 : 0;
}

void mbls_profile_reset(void) {
    std::lock_guard<std::mutex> lk(mbls::g_prof_mu);
    mbls::profile_drain();
    mbls::g_prof_sum.clear();
}

/* Fills up to `max` entries: names (static until the next reset), total ms, call counts.
 * Returns the number of stages recorded. */
int mbls_profile_read(const char** names, double* total_ms, long* counts, int max) {
    std::lock_guard<std::mutex> lk(mbls::g_prof_mu);
    mbls::profile_drain();
    int i = 0;
    for (auto& kv : mbls::g_prof_sum) {
        if (i >= max) break;
        names[i] = kv.first.c_str();
        total_ms[i] = kv.second.first;
        counts[i] = kv.second.second;
        ++i;
    }
    return (int)mbls::g_prof_sum.size();
}

const char* mbls_version(void) { return "bls12_381_mi355x 0.1 (gfx950)"; }

const char* mbls_error_string(eIcicleError e) {
    static const char* names[] = {"SUCCESS", "INVALID_DEVICE", "OUT_OF_MEMORY", "INVALID_POINTER",
                                  "ALLOCATION_FAILED", "DEALLOCATION_FAILED", "COPY_FAILED",
                                  "SYNCHRONIZATION_FAILED", "STREAM_CREATION_FAILED",
                                  "STREAM_DESTRUCTION_FAILED", "API_NOT_IMPLEMENTED", "INVALID_ARGUMENT",
                                  "BACKEND_LOAD_FAILED", "LICENSE_CHECK_ERROR", "UNKNOWN_ERROR"};
    int i = (int)e;
    if (i < 0 || i > 14) return "UNKNOWN_ERROR";
    return names[i];
}

MSMConfig mbls_default_msm_config(void) {
    MSMConfig c;
    memset(&c, 0, sizeof c);
    c.precompute_factor = 1;
    c.batch_size = 1;
    c.are_points_shared_in_batch = true;
    return c;
}

NTTConfig mbls_default_ntt_config(void) {
    NTTConfig c;
    memset(&c, 0, sizeof c);
    // coset_gen = one (Montgomery form of 1 in Fr)
    c.coset_gen.limbs[0] = 0x00000001fffffffeULL;
    c.coset_gen.limbs[1] = 0x5884b7fa00034802ULL;
    c.coset_gen.limbs[2] = 0x998c4fefecbc4ff5ULL;
    c.coset_gen.limbs[3] = 0x1824b159acc5056fULL;
    c.batch_size = 1;
    c.ordering = MBLS_ORDERING_NN;
    return c;
}

VecOpsConfig mbls_default_vec_ops_config(void) {
    VecOpsConfig c;
    memset(&c, 0, sizeof c);
    c.batch_size = 1;
    return c;
}

}  // extern "C"
