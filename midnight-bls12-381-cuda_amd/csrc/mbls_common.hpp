// mbls_common.hpp -- host-side plumbing shared by the HIP translation units:
// error mapping, the per-device pool of scratch contexts (no per-call hipMalloc on the hot path,
// unlike the reference's 7 cudaMallocs per MSM, msm_kernels.cu:705-719), stage profiler.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <mutex>
#include <unordered_map>
#include <vector>

#include "bls12_381_mi355x.h"

namespace mbls {

#define MBLS_TRY(expr)                                                     \
    do {                                                                   \
        hipError_t _e = (expr);                                            \
        if (_e != hipSuccess) return ::mbls::map_hip_error(_e, #expr);     \
    } while (0)

eIcicleError map_hip_error(hipError_t e, const char* what);
bool trace_enabled();

// Device scratch arena.  Grows (never shrinks, unless trimmed) to the high-water mark of its
// calls; it belongs to a ScratchCtx of the per-device pool, never to a caller's stream.
class Arena {
  public:
    Arena() = default;
    ~Arena();
    // returns a device pointer to >= bytes, 256-B aligned; valid until the next reset()
    void* take(size_t bytes);
    void reset() { used_ = 0; }
    size_t mark() const { return used_; }
    void rewind(size_t m) { used_ = m; }
    size_t capacity() const { return cap_; }
    // grow to >= bytes; `idle` is an event after which no earlier work reads the block (null:
    // never used), synchronised before the old block is freed
    eIcicleError reserve(size_t bytes, hipEvent_t idle);
    // free the block (caller guarantees no queued work reads it)
    void release();

  private:
    void* base_ = nullptr;
    size_t cap_ = 0;
    size_t used_ = 0;
};

// Scratch context: an arena plus the side streams / events an MSM forks from the caller's
// stream.  Contexts live in a per-device pool and are LEASED for one call (CtxLease), not
// keyed by the caller's hipStream_t: the reference's callers create and destroy a stream per
// async MSM (core/msm.rs:742 -> stream.rs:189), which must neither leak an arena per stream
// nor hipMalloc a fresh one on the hot path.  At the end of a call the lease records `done` on
// the caller's stream; the next lease on another stream either finds the context idle (event
// complete), or makes its stream wait for `done`.
struct StreamCtx {
    int device = 0;
    Arena arena;
    // side streams for latency-bound work that overlaps the main chain (MSM tree sums, the
    // endomorphism table); forked from / joined back into the caller's stream with events, so
    // callers see one stream-ordered operation
    std::vector<hipStream_t> sides;
    std::vector<hipEvent_t> events;
    hipEvent_t done = nullptr;  // recorded on the caller's stream when a call's enqueue ends
    bool used = false;          // `done` has been recorded at least once
    hipStream_t last = nullptr; // caller stream of the last call
    bool last_valid = false;    // `last` names a live stream (false after mbls_release_stream)
    // the call forked work to `sides` (set at each fork): the lease joins them into the caller's
    // stream before recording `done`, covering early error returns
    bool forked = false;
    std::vector<hipEvent_t> join_events;  // one per side stream
    bool busy = false;          // leased by a thread right now
    uint64_t stamp = 0;         // LRU order
    eIcicleError ensure_side(size_t nevents, size_t nsides = 1);
};

// RAII lease of a pool context for one call on stream `st` (current device).
class CtxLease {
  public:
    explicit CtxLease(hipStream_t st);
    ~CtxLease();
    CtxLease(const CtxLease&) = delete;
    CtxLease& operator=(const CtxLease&) = delete;
    explicit operator bool() const { return ctx_ != nullptr; }
    eIcicleError error() const { return err_; }
    StreamCtx& operator*() const { return *ctx_; }
    StreamCtx* operator->() const { return ctx_; }
    // grow the context's arena (safe against its previous calls) and reset it
    eIcicleError reserve(size_t bytes) {
        ctx_->arena.reset();
        return ctx_->arena.reserve(bytes, ctx_->used ? ctx_->done : nullptr);
    }

  private:
    StreamCtx* ctx_ = nullptr;
    hipStream_t st_;
    eIcicleError err_ = MBLS_SUCCESS;
};

// library-side hipMalloc / hipFree counters of the scratch pool (tests: no allocation on the
// hot path after the first call)
void count_scratch_alloc(size_t bytes);
void count_scratch_free(size_t bytes);

// Reserve-then-take helper: computes the total of a list of sizes first, so the arena
// reallocates at most once per call (before any kernel of this call is enqueued).
inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// is `p` a device (or managed) pointer?  Used only for defensive validation.
bool is_device_pointer(const void* p);
// device-visible alias of page-locked (pinned / registered) host memory, or nullptr for pageable
// host memory and device memory
const void* pinned_host_device_pointer(const void* p);
// bytes from `p` to the end of the device allocation holding it (hipMemGetAddressRange), or
// SIZE_MAX when the runtime cannot tell (host memory, foreign allocators)
size_t device_bytes_from(const void* p);
// precompute_bases tables written by this library (common.cpp): registration, strict mode, lookup
void precompute_register(const void* table, size_t bytes, int factor);
bool precompute_strict();
void precompute_set_strict(bool on);
bool precompute_is_table(const void* bases, int factor, size_t want_bytes);
// the event mbls_msm_accumulate_event left pending for `st` (taken: nullptr afterwards), or nullptr
hipEvent_t take_accumulate_event(hipStream_t st);
// a taken accumulate event: recorded on `st` when the guard dies unless release()d first (the
// MSM paths that never reach an accumulation -- empty MSMs, errors -- still record it, so it
// cannot linger for an unrelated later MSM: ADVICE r5)
struct AccEventGuard {
    hipEvent_t ev;
    hipStream_t st;
    AccEventGuard(hipEvent_t e, hipStream_t s) : ev(e), st(s) {}
    AccEventGuard(const AccEventGuard&) = delete;
    AccEventGuard& operator=(const AccEventGuard&) = delete;
    hipEvent_t release() {
        hipEvent_t e = ev;
        ev = nullptr;
        return e;
    }
    ~AccEventGuard() {
        if (ev) (void)hipEventRecord(ev, st);
    }
};

// Stage profiler: when enabled (mbls_profile_enable / MBLS_PROFILE=1) a ProfScope records a
// hipEvent pair on the stream around the enclosed launches; mbls_profile_read() sums the
// elapsed times per stage name.  Disabled: one branch, no events.
bool profile_enabled();
void profile_record(const char* name, hipEvent_t a, hipEvent_t b);
struct ProfScope {
    const char* name;
    hipStream_t st;
    hipEvent_t a = nullptr, b = nullptr;
    ProfScope(const char* n, hipStream_t s) : name(n), st(s) {
        if (profile_enabled()) {
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            (void)hipEventRecord(a, st);
        }
    }
    ~ProfScope() {
        if (a) {
            (void)hipEventRecord(b, st);
            profile_record(name, a, b);
        }
    }
};

}  // namespace mbls
