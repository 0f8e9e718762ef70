// common.cpp -- error mapping, the scratch-context pool, configs, version.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <condition_variable>
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

static std::atomic<uint64_t> g_scratch_mallocs{0}, g_scratch_frees{0}, g_scratch_bytes{0};
void count_scratch_alloc(size_t bytes) {
    g_scratch_mallocs.fetch_add(1);
    g_scratch_bytes.fetch_add(bytes);
}
void count_scratch_free(size_t bytes) {
    g_scratch_frees.fetch_add(1);
    g_scratch_bytes.fetch_sub(bytes);
}

Arena::~Arena() {
    // pool contexts live for the process; freeing at exit races with runtime teardown, so leak
    // (mbls_release_scratch frees idle arenas explicitly)
}

eIcicleError Arena::reserve(size_t bytes, hipEvent_t idle) {
    bytes = align_up(bytes);
    if (bytes <= cap_) return MBLS_SUCCESS;
    size_t ncap = bytes + bytes / 4;
    if (base_) {
        // earlier calls of this context may still read the old block: wait for them
        if (idle) {
            hipError_t e = hipEventSynchronize(idle);
            if (e != hipSuccess) return map_hip_error(e, "arena idle sync");
        }
        release();
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, ncap);
    if (e != hipSuccess) return map_hip_error(e, "arena hipMalloc");
    count_scratch_alloc(ncap);
    base_ = p;
    cap_ = ncap;
    used_ = 0;
    return MBLS_SUCCESS;
}

void Arena::release() {
    if (base_) {
        (void)hipFree(base_);
        count_scratch_free(cap_);
    }
    base_ = nullptr;
    cap_ = 0;
    used_ = 0;
}

void* Arena::take(size_t bytes) {
    bytes = align_up(bytes);
    if (used_ + bytes > cap_) return nullptr;
    void* p = static_cast<char*>(base_) + used_;
    used_ += bytes;
    return p;
}

// ---- per-device pool of scratch contexts ------------------------------------------------
// Lease policy (CtxLease): among the free contexts of the current device take, in order,
//   1. one whose last call was on this same stream (preferred: stream order usually serialises it);
//   2. an idle one (its `done` event complete, or never used), the largest arena first;
//   3. a new context while the pool holds fewer than MBLS_SCRATCH_CONTEXTS (default 4);
//   4. the least recently used one.
// Whenever the picked context was used and its `done` is not known complete, the caller's stream
// waits for `done` -- also in case 1: a handle equal to the last one may be a recycled stream (a
// destroyed ICICLE / torch stream whose address came back) or the default stream after
// mbls_release_stream, and a wait on an event recorded on the same queue costs HIP nothing.
// If every context is leased by another thread and the pool is full, wait for a release.
struct Pool {
    std::mutex mu;
    std::condition_variable cv;
    std::map<int, std::vector<std::unique_ptr<StreamCtx>>> by_dev;
    uint64_t clock = 0;
};
static Pool& pool() {
    static Pool* p = new Pool();  // never destroyed (see Arena::~Arena)
    return *p;
}
static size_t pool_limit() {
    static const size_t v = [] {
        const char* e = getenv("MBLS_SCRATCH_CONTEXTS");
        const long k = e ? atol(e) : 4;
        return (size_t)(k > 0 ? k : 1);
    }();
    return v;
}

CtxLease::CtxLease(hipStream_t st) : st_(st) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    Pool& P = pool();
    std::unique_lock<std::mutex> lk(P.mu);
    auto& v = P.by_dev[dev];
    StreamCtx* pick = nullptr;
    bool wait = false;
    while (!pick) {
        StreamCtx* idle = nullptr;
        StreamCtx* lru = nullptr;
        for (auto& c : v) {
            if (c->busy) continue;
            if (c->last_valid && c->last == st && c->used) {
                pick = c.get();
                wait = true;
                break;
            }
            const bool is_idle = !c->used || hipEventQuery(c->done) == hipSuccess;
            if (is_idle && (!idle || c->arena.capacity() > idle->arena.capacity())) idle = c.get();
            if (!lru || c->stamp < lru->stamp) lru = c.get();
        }
        if (pick) break;
        if (idle) {
            pick = idle;
        } else if (v.size() < pool_limit()) {
            std::unique_ptr<StreamCtx> c(new StreamCtx());
            c->device = dev;
            if (hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) {
                err_ = MBLS_UNKNOWN_ERROR;
                return;
            }
            pick = c.get();
            v.push_back(std::move(c));
        } else if (lru) {
            pick = lru;
            wait = lru->used;
        } else {
            P.cv.wait(lk);  // all leased by other threads
        }
    }
    pick->busy = true;
    pick->stamp = ++P.clock;
    lk.unlock();
    if (wait && hipStreamWaitEvent(st, pick->done, 0) != hipSuccess) {
        err_ = MBLS_UNKNOWN_ERROR;
        std::lock_guard<std::mutex> g(P.mu);
        pick->busy = false;
        P.cv.notify_one();
        return;
    }
    ctx_ = pick;
}

CtxLease::~CtxLease() {
    if (!ctx_) return;
    // everything the call enqueued is ordered before `done`.  A call that forked work to the
    // side streams joins them back before it returns; an early error return may not have, so
    // the side streams' tails are joined here whenever the call forked (a join event each)
    if (ctx_->forked) {
        for (size_t i = 0; i < ctx_->sides.size() && i < ctx_->join_events.size(); ++i)
            if (hipEventRecord(ctx_->join_events[i], ctx_->sides[i]) == hipSuccess)
                (void)hipStreamWaitEvent(st_, ctx_->join_events[i], 0);
        ctx_->forked = false;
    }
    const bool rec = hipEventRecord(ctx_->done, st_) == hipSuccess;
    Pool& P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    if (rec) ctx_->used = true;
    ctx_->last = st_;
    ctx_->last_valid = true;
    ctx_->busy = false;
    P.cv.notify_one();
}

#ifndef MBLS_SIDE_PRIO
#define MBLS_SIDE_PRIO 1  // variant builds: 0 = side streams at the lowest priority
#endif

eIcicleError StreamCtx::ensure_side(size_t nevents, size_t nsides) {
    while (sides.size() < nsides) {
        hipStream_t s;
        // highest priority: the side streams carry the latency-bound tails that must not queue
        // behind the main stream's accumulation workgroups
        int least = 0, greatest = 0;
        MBLS_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        MBLS_TRY(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, MBLS_SIDE_PRIO ? greatest : least));
        sides.push_back(s);
        hipEvent_t j;
        MBLS_TRY(hipEventCreateWithFlags(&j, hipEventDisableTiming));
        join_events.push_back(j);
    }
    while (events.size() < nevents) {
        hipEvent_t e;
        MBLS_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        events.push_back(e);
    }
    return MBLS_SUCCESS;
}

const void* pinned_host_device_pointer(const void* p) {
    hipPointerAttribute_t a;
    if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
    // only the alias of the calling device: whether a registered / non-portable allocation's
    // alias is valid on another device is not something the multi-device shards rely on (they
    // stage instead)
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || a.device != cur) {
        (void)hipGetLastError();
        return nullptr;
    }
    // the attribute describes the allocation: offset the device alias like the host pointer
    const char* hbase = static_cast<const char*>(a.hostPointer ? a.hostPointer : p);
    return static_cast<const char*>(a.devicePointer) + (static_cast<const char*>(p) - hbase);
}

size_t device_bytes_from(const void* p) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (!p || hipMemGetAddressRange(&base, &size, const_cast<void*>(p)) != hipSuccess || !base) {
        (void)hipGetLastError();
        return SIZE_MAX;
    }
    const char* b = static_cast<const char*>(base);
    const char* q = static_cast<const char*>(p);
    return q >= b && q <= b + size ? (size_t)(b + size - q) : SIZE_MAX;
}

// ---- precompute_bases tables (ADVICE / VERDICT r5: the plain-bases guard) ------------------
// precompute_call registers every table it writes; with strict mode on, an MSM takes
// precompute_factor > 1 only for a registered table whose factor matches and whose entries cover
// the call, and runs anything else as plain bases (factor 1).  Bounded: the oldest of
// PRECOMP_SLOTS registrations is forgotten first (re-running precompute_bases registers again).
namespace {
struct PrecompEntry {
    const void* p = nullptr;
    size_t bytes = 0;
    int factor = 0, device = -1;
};
constexpr int PRECOMP_SLOTS = 256;
std::mutex g_precomp_mu;
PrecompEntry g_precomp[PRECOMP_SLOTS];
int g_precomp_next = 0;
std::atomic<int> g_precomp_strict{0};
}  // namespace

void precompute_register(const void* table, size_t bytes, int factor) {
    int dev = -1;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_precomp_mu);
    for (auto& e : g_precomp)
        if (e.p == table && e.device == dev) {  // the same buffer rewritten: replace
            e = {table, bytes, factor, dev};
            return;
        }
    g_precomp[g_precomp_next] = {table, bytes, factor, dev};
    g_precomp_next = (g_precomp_next + 1) % PRECOMP_SLOTS;
}

bool precompute_strict() { return g_precomp_strict.load(std::memory_order_relaxed) != 0; }
void precompute_set_strict(bool on) { g_precomp_strict.store(on ? 1 : 0, std::memory_order_relaxed); }

bool precompute_is_table(const void* bases, int factor, size_t want_bytes) {
    int dev = -1;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_precomp_mu);
    for (const auto& e : g_precomp)
        if (e.p && e.p == bases && e.device == dev && e.factor == factor && want_bytes <= e.bytes) return true;
    return false;
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

// mbls_msm_accumulate_event: one pending event per stream, taken by the next MSM on it
namespace mbls {
static std::mutex g_acc_ev_mu;
static std::map<hipStream_t, hipEvent_t>* g_acc_ev = new std::map<hipStream_t, hipEvent_t>();
static std::atomic<int> g_acc_ev_n{0};
hipEvent_t take_accumulate_event(hipStream_t st) {
    if (g_acc_ev_n.load(std::memory_order_relaxed) == 0) return nullptr;  // the hot path: nothing pending
    std::lock_guard<std::mutex> g(g_acc_ev_mu);
    auto it = g_acc_ev->find(st);
    if (it == g_acc_ev->end()) return nullptr;
    hipEvent_t e = it->second;
    g_acc_ev->erase(it);
    g_acc_ev_n.fetch_sub(1, std::memory_order_relaxed);
    return e;
}
}  // namespace mbls

extern "C" {
eIcicleError mbls_msm_precompute_strict(int on) {
    mbls::precompute_set_strict(on != 0);
    return MBLS_SUCCESS;
}

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

/* scratch pool (include/bls12_381_mi355x.h) */

eIcicleError mbls_msm_accumulate_event(void* stream, void* event) {
    std::lock_guard<std::mutex> g(mbls::g_acc_ev_mu);
    const hipStream_t st = static_cast<hipStream_t>(stream);
    auto it = mbls::g_acc_ev->find(st);
    if (it != mbls::g_acc_ev->end()) {
        mbls::g_acc_ev->erase(it);
        mbls::g_acc_ev_n.fetch_sub(1, std::memory_order_relaxed);
    }
    if (event) {
        (*mbls::g_acc_ev)[st] = static_cast<hipEvent_t>(event);
        mbls::g_acc_ev_n.fetch_add(1, std::memory_order_relaxed);
    }
    return MBLS_SUCCESS;
}

eIcicleError mbls_msm_accumulate_event_drop(void* event) {
    if (!event) return MBLS_SUCCESS;
    std::lock_guard<std::mutex> g(mbls::g_acc_ev_mu);
    for (auto it = mbls::g_acc_ev->begin(); it != mbls::g_acc_ev->end();) {
        if (it->second == static_cast<hipEvent_t>(event)) {
            it = mbls::g_acc_ev->erase(it);
            mbls::g_acc_ev_n.fetch_sub(1, std::memory_order_relaxed);
        } else {
            ++it;
        }
    }
    return MBLS_SUCCESS;
}

eIcicleError mbls_release_stream(void* stream) {
    mbls::Pool& P = mbls::pool();
    std::lock_guard<std::mutex> g(P.mu);
    for (auto& kv : P.by_dev)
        for (auto& c : kv.second)
            if (c->last == static_cast<hipStream_t>(stream)) c->last_valid = false;
    return MBLS_SUCCESS;
}

eIcicleError mbls_release_scratch(void) {
    mbls::Pool& P = mbls::pool();
    std::lock_guard<std::mutex> g(P.mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    eIcicleError r = MBLS_SUCCESS;
    for (auto& kv : P.by_dev)
        for (auto& c : kv.second) {
            if (c->busy || !c->arena.capacity()) continue;
            if (hipSetDevice(c->device) != hipSuccess) {
                r = MBLS_INVALID_DEVICE;
                continue;
            }
            if (c->used && hipEventSynchronize(c->done) != hipSuccess) {
                r = MBLS_SYNCHRONIZATION_FAILED;
                continue;
            }
            c->arena.release();
        }
    (void)hipSetDevice(cur);
    return r;
}

void mbls_scratch_stats(uint64_t* mallocs, uint64_t* frees, uint64_t* bytes, int* contexts) {
    if (mallocs) *mallocs = mbls::g_scratch_mallocs.load();
    if (frees) *frees = mbls::g_scratch_frees.load();
    if (bytes) *bytes = mbls::g_scratch_bytes.load();
    if (contexts) {
        mbls::Pool& P = mbls::pool();
        std::lock_guard<std::mutex> g(P.mu);
        int k = 0;
        for (auto& kv : P.by_dev) k += (int)kv.second.size();
        *contexts = k;
    }
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
