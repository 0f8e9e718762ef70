// mbls_common.hpp -- host-side plumbing shared by the HIP translation units:
// error mapping, per-stream scratch arenas (no per-call hipMalloc on the hot path, unlike the
// reference's 7 cudaMallocs per MSM, msm_kernels.cu:705-719), staging of host/device operands.
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

// Device scratch arena bound to one stream.  Grows (never shrinks) to the high-water mark;
// reuse is safe because every user enqueues its work on the same stream.
class Arena {
  public:
    explicit Arena(hipStream_t s) : stream_(s) {}
    ~Arena();
    // returns a device pointer to >= bytes, 256-B aligned; valid until the next reset()
    void* take(size_t bytes);
    void reset() { used_ = 0; }
    size_t mark() const { return used_; }
    void rewind(size_t m) { used_ = m; }
    eIcicleError reserve(size_t bytes);

  private:
    hipStream_t stream_;
    void* base_ = nullptr;
    size_t cap_ = 0;
    size_t used_ = 0;
    std::vector<void*> retired_;
};

// One arena per (device, stream); the lock is held for the whole enqueue of a call so two
// host threads on the same stream serialise, different streams run concurrently.
struct StreamCtx {
    std::mutex mu;
    Arena arena;
    // side stream for latency-bound work that overlaps the main chain (MSM tree sums);
    // forked from / joined back into the caller's stream with events, so callers see one
    // stream-ordered operation
    std::vector<hipStream_t> sides;
    std::vector<hipEvent_t> events;
    // batch pipeline: two private streams (each with its own StreamCtx / arena) that run
    // alternate batch members, so one member's latency-bound tail overlaps the next member's
    // accumulation; pipe_ev[0] forks them from this stream, pipe_ev[1..2] join them back
    hipStream_t pipe[2] = {nullptr, nullptr};
    hipEvent_t pipe_ev[3] = {nullptr, nullptr, nullptr};
    // acc_ev[b & 1]: member b's accumulation done; member b + 1 (other stream) waits for it, so
    // the two streams run staggered (b+1 accumulates while b runs its tail) instead of lockstep
    hipEvent_t acc_ev[2] = {nullptr, nullptr};
    explicit StreamCtx(hipStream_t s) : arena(s) {}
    eIcicleError ensure_side(size_t nevents, size_t nsides = 1);
    eIcicleError ensure_pipe();
};
StreamCtx& stream_ctx(hipStream_t s);

// Reserve-then-take helper: computes the total of a list of sizes first, so the arena
// reallocates at most once per call (before any kernel of this call is enqueued).
inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// is `p` a device (or managed) pointer?  Used only for defensive validation.
bool is_device_pointer(const void* p);

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
