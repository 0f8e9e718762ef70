/*
 * bls12_381_mi355x.h -- C ABI of the MI355X (gfx950) BLS12-381 prover hot path.
 *
 * This is the drop-in boundary.  Every entry point below replaces one exported by the
 * reference backend (riusricardo/midnight-bls12-381-cuda, bls12-381/src/...) with the same
 * name, argument meaning and error behaviour; the citation on each declaration is the
 * reference definition it replaces.  Plain C: pointers, sizes, POD config structs, no C++ or
 * torch types.  Streams are hipStream_t passed as void* (NULL = the default stream).
 *
 * Byte layouts (identical to blst / the reference, little-endian u64 limbs):
 *   Fr          32 B   canonical, Montgomery (R = 2^256) unless a flag says standard
 *   Fq          48 B   canonical, Montgomery (R = 2^384)
 *   G1 affine   96 B   x || y;             identity = all zero
 *   G2 affine  192 B   x.c0||x.c1||y.c0||y.c1; identity = all zero
 *   G1 proj.   144 B   X || Y || Z          (meaning depends on the entry point, see below)
 *   G2 proj.   288 B
 */
#ifndef BLS12_381_MI355X_H
#define BLS12_381_MI355X_H

#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------------------ */
/* errors: ICICLE v4 numbering (reference include/icicle/errors.h:37-52).  The reference's
 * own icicle_types.cuh:47-63 renumbers UNKNOWN_ERROR to 999; we follow real ICICLE.       */
/* ------------------------------------------------------------------------------------ */
typedef enum {
    MBLS_SUCCESS = 0,
    MBLS_INVALID_DEVICE = 1,
    MBLS_OUT_OF_MEMORY = 2,
    MBLS_INVALID_POINTER = 3,
    MBLS_ALLOCATION_FAILED = 4,
    MBLS_DEALLOCATION_FAILED = 5,
    MBLS_COPY_FAILED = 6,
    MBLS_SYNCHRONIZATION_FAILED = 7,
    MBLS_STREAM_CREATION_FAILED = 8,
    MBLS_STREAM_DESTRUCTION_FAILED = 9,
    MBLS_API_NOT_IMPLEMENTED = 10,
    MBLS_INVALID_ARGUMENT = 11,
    MBLS_BACKEND_LOAD_FAILED = 12,
    MBLS_LICENSE_CHECK_ERROR = 13,
    MBLS_UNKNOWN_ERROR = 14
} eIcicleError;

/* ------------------------------------------------------------------------------------ */
/* element types (opaque byte containers with the layouts above)                         */
/* ------------------------------------------------------------------------------------ */
typedef struct { uint64_t limbs[4]; } mbls_fr_t;
typedef struct { uint64_t limbs[6]; } mbls_fq_t;
typedef struct { mbls_fq_t c0, c1; } mbls_fq2_t;
typedef struct { mbls_fq_t x, y; } mbls_g1_affine_t;
typedef struct { mbls_fq_t x, y, z; } mbls_g1_projective_t;
typedef struct { mbls_fq2_t x, y; } mbls_g2_affine_t;
typedef struct { mbls_fq2_t x, y, z; } mbls_g2_projective_t;

/* ------------------------------------------------------------------------------------ */
/* configs: byte-compatible with ICICLE v4 (reference icicle_types.cuh:102-201)           */
/* ------------------------------------------------------------------------------------ */
typedef enum { MBLS_NTT_FORWARD = 0, MBLS_NTT_INVERSE = 1 } NTTDir;   /* icicle_types.cuh:83-86 */
typedef enum {                                                      /* icicle_types.cuh:88-95 */
    MBLS_ORDERING_NN = 0, MBLS_ORDERING_NR = 1, MBLS_ORDERING_RN = 2,
    MBLS_ORDERING_RR = 3, MBLS_ORDERING_NM = 4, MBLS_ORDERING_MN = 5
} Ordering;

/* MSMConfig -- icicle_types.cuh:155-169 */
typedef struct {
    void* stream;
    int precompute_factor;
    int c;                            /* window bits, 0 = auto                         */
    int bitsize;                      /* scalar bits, 0 = 255                          */
    int batch_size;                   /* number of MSMs (scalars/results are batched)   */
    bool are_points_shared_in_batch;
    bool are_scalars_on_device;
    bool are_scalars_montgomery_form;
    bool are_points_on_device;
    bool are_points_montgomery_form;
    bool are_results_on_device;
    bool is_async;
    void* ext;
} MSMConfig;

/* NTTConfig<Fr> -- icicle_types.cuh:102-113 (coset_gen is a 32-byte Fr) */
typedef struct {
    void* stream;
    mbls_fr_t coset_gen;
    int batch_size;
    bool columns_batch;
    Ordering ordering;
    bool are_inputs_on_device;
    bool are_outputs_on_device;
    bool is_async;
    void* ext;
} NTTConfig;

/* NTTInitDomainConfig -- icicle_types.cuh:136-140 */
typedef struct {
    void* stream;
    bool is_async;
    void* ext;
} NTTInitDomainConfig;

/* VecOpsConfig -- ICICLE v4 layout (icicle_types.cuh:194-201 plus v4's batch fields,
 * which core/vecops.rs:346 sets) */
typedef struct {
    void* stream;
    bool is_a_on_device;
    bool is_b_on_device;
    bool is_result_on_device;
    bool is_async;
    int batch_size;
    bool columns_batch;
    void* ext;
} VecOpsConfig;

MSMConfig mbls_default_msm_config(void);
NTTConfig mbls_default_ntt_config(void);
VecOpsConfig mbls_default_vec_ops_config(void);

/* ------------------------------------------------------------------------------------ */
/* MSM                                                                                    */
/* ------------------------------------------------------------------------------------ */
/* Raw kernel-level MSM, reference icicle_curve_api.cu:679-705 (bls12_381_g1_msm_cuda /
 * bls12_381_g2_msm_cuda -> msm::msm_cuda, msm_kernels.cu:603-903):
 *   scalars STANDARD form, bases Montgomery affine, result = Jacobian Montgomery point
 *   (identity: Z = 0).  Host/device placement from config->are_*_on_device.           */
eIcicleError bls12_381_g1_msm_cuda(const mbls_fr_t* scalars, const mbls_g1_affine_t* bases, int msm_size,
                                   const MSMConfig* config, mbls_g1_projective_t* result);
eIcicleError bls12_381_g2_msm_cuda(const mbls_fr_t* scalars, const mbls_g2_affine_t* bases, int msm_size,
                                   const MSMConfig* config, mbls_g2_projective_t* result);

/* ICICLE-registered MSM semantics, reference icicle_curve_api.cu:243-407 (msm_cuda_impl) and
 * :454-618 (msm_g2_cuda_impl): honours are_scalars_montgomery_form /
 * are_points_montgomery_form, returns ICICLE standard-form projective (x, y, 1) with
 * identity (0, 1, 0).  batch_size > 1 computes batch_size MSMs (the reference silently
 * computes only the first, SURVEY.md finding 3): scalars are batch_size*msm_size, bases are
 * msm_size (shared) or batch_size*msm_size, results batch_size.                          */
eIcicleError bls12_381_icicle_g1_msm(const mbls_fr_t* scalars, const mbls_g1_affine_t* bases, int msm_size,
                                     const MSMConfig* config, mbls_g1_projective_t* results);
eIcicleError bls12_381_icicle_g2_msm(const mbls_fr_t* scalars, const mbls_g2_affine_t* bases, int msm_size,
                                     const MSMConfig* config, mbls_g2_projective_t* results);

/* precompute_bases, reference icicle_curve_api.cu:415-440 (there a plain byte copy, so its
 * factor > 1 gives wrong MSMs).  Here factor F = config->precompute_factor in 1..64 writes the
 * point-major table out[i*F + f] = 2^(s*f) * P_i with s = ceil(256 / F) (core/msm.rs:164-165):
 * the shift depends on F only, so ONE table serves MSMs of any c (config->c is ignored here)
 * and any msm_size <= bases_size.  Output: Montgomery affine; standard-form input
 * (are_points_montgomery_form = false) is converted first.  An MSM with precompute_factor
 * F > 1 reads such a table (n*F entries, the full buffer may be passed) and treats it as
 * Montgomery whatever are_points_montgomery_form says -- core/msm.rs:641-643 passes false
 * with a precomputed table.                                                               */
eIcicleError bls12_381_icicle_g1_msm_precompute_bases(const mbls_g1_affine_t* input_bases, int bases_size,
                                                      const MSMConfig* config, mbls_g1_affine_t* output_bases);
eIcicleError bls12_381_icicle_g2_msm_precompute_bases(const mbls_g2_affine_t* input_bases, int bases_size,
                                                      const MSMConfig* config, mbls_g2_affine_t* output_bases);

/* ------------------------------------------------------------------------------------ */
/* NTT (reference ntt_kernels.cu:1907-1943, icicle_field_api.cu:363-383)                  */
/* Semantics follow the CPU path (core/ntt.rs:1488-1603, best_fft): forward
 * out_j = sum_i in_i w^(ij), inverse = n^-1 sum_j in_j w^(-ij), w = ROOT_OF_UNITY^(2^(32-k))
 * for size 2^k, natural order in and out (kNN).                                          */
/* ------------------------------------------------------------------------------------ */
eIcicleError bls12_381_ntt_init_domain_cuda(const mbls_fr_t* root_of_unity, const NTTInitDomainConfig* config);
eIcicleError bls12_381_ntt_release_domain_cuda(void);
eIcicleError bls12_381_ntt_cuda(const mbls_fr_t* input, int size, NTTDir dir, const NTTConfig* config,
                                mbls_fr_t* output);
eIcicleError bls12_381_coset_ntt_cuda(const mbls_fr_t* input, int size, NTTDir dir, const mbls_fr_t* coset_gen,
                                      const NTTConfig* config, mbls_fr_t* output);
eIcicleError bls12_381_field_ntt_cuda(const mbls_fr_t* input, int size, NTTDir dir, const NTTConfig* config,
                                      mbls_fr_t* output);
eIcicleError bls12_381_field_ntt_init_domain_cuda(const mbls_fr_t* root_of_unity, const NTTInitDomainConfig* config);
eIcicleError bls12_381_field_ntt_release_domain_cuda(void);
/* w_(2^logn) of the initialised domain (Montgomery); INVALID_ARGUMENT without a domain or past
 * its order.  Backs ICICLE's NttGetRouFromDomainImpl (icicle_backend_api.cuh:135-138). */
eIcicleError bls12_381_ntt_get_rou_from_domain(uint64_t logn, mbls_fr_t* rou);

/* ------------------------------------------------------------------------------------ */
/* vecops (reference vec_ops.cu:393-524 and :693-840; icicle_field_api.cu:194-334)        */
/* raw-limb semantics: add/sub representation-agnostic, mul = Montgomery product.         */
/* ------------------------------------------------------------------------------------ */
eIcicleError bls12_381_vector_add(const mbls_fr_t* a, const mbls_fr_t* b, size_t size, const VecOpsConfig* config,
                                  mbls_fr_t* output);
eIcicleError bls12_381_vector_sub(const mbls_fr_t* a, const mbls_fr_t* b, size_t size, const VecOpsConfig* config,
                                  mbls_fr_t* output);
eIcicleError bls12_381_vector_mul(const mbls_fr_t* a, const mbls_fr_t* b, size_t size, const VecOpsConfig* config,
                                  mbls_fr_t* output);
/* scalar_{mul,add}_vec: `scalar` is ONE element on the host unless config->is_a_on_device
 * (icicle_field_api.cu:227-334). */
eIcicleError bls12_381_scalar_mul_vec(const mbls_fr_t* scalar, const mbls_fr_t* vec, size_t size,
                                      const VecOpsConfig* config, mbls_fr_t* output);
eIcicleError bls12_381_scalar_add_vec(const mbls_fr_t* scalar, const mbls_fr_t* vec, size_t size,
                                      const VecOpsConfig* config, mbls_fr_t* output);
/* device-pointer kernel entry points, vec_ops.cu:393-476 (output first, device pointers;
 * `scalar` is a HOST pointer to one element as in the reference). */
eIcicleError vec_add_cuda(mbls_fr_t* output, const mbls_fr_t* a, const mbls_fr_t* b, int size, const VecOpsConfig* config);
eIcicleError vec_sub_cuda(mbls_fr_t* output, const mbls_fr_t* a, const mbls_fr_t* b, int size, const VecOpsConfig* config);
eIcicleError vec_mul_cuda(mbls_fr_t* output, const mbls_fr_t* a, const mbls_fr_t* b, int size, const VecOpsConfig* config);
eIcicleError scalar_mul_vec_cuda(mbls_fr_t* output, const mbls_fr_t* scalar, const mbls_fr_t* vec, int size,
                                 const VecOpsConfig* config);
eIcicleError scalar_add_vec_cuda(mbls_fr_t* output, const mbls_fr_t* scalar, const mbls_fr_t* vec, int size,
                                 const VecOpsConfig* config);
/* sum of `size` device elements; output on device or host per config->is_result_on_device.
 * Replaces vec_sum_cuda (vec_ops.cu:479-524; the reference takes `const VecOpsConfig&`). */
eIcicleError vec_sum_cuda(mbls_fr_t* output, const mbls_fr_t* input, int size, const VecOpsConfig* config);
/* element-wise inverses (0 -> 0), device pointers, in place allowed.  Replaces the C++
 * template vec_ops::batch_inv_cuda<Fr> (vec_ops.cu:606-673); a C symbol here. */
eIcicleError bls12_381_batch_inv_cuda(mbls_fr_t* output, const mbls_fr_t* input, int size, const VecOpsConfig* config);

/* ------------------------------------------------------------------------------------ */
/* batch point-form conversions, reference point_ops.cu:759 / :844 / :924 (exported there as
 * extern "C").  Montgomery in, Montgomery out; Jacobian projective (x = X/Z^2, y = Y/Z^3).
 * affine_to_projective: (x, y) -> (x, y, 1), identity (0, 0) -> (0, 1, 0).
 * projective_to_affine: Z = 0 -> (0, 0).  Input placement config->is_a_on_device, output
 * config->is_result_on_device; a host output is synchronous.  size in 1..2^26, null pointers
 * or other sizes give INVALID_ARGUMENT (as the reference).  Input and output must not overlap. */
/* ------------------------------------------------------------------------------------ */
eIcicleError bls12_381_g1_affine_to_projective(const mbls_g1_affine_t* input, int size, const VecOpsConfig* config,
                                               mbls_g1_projective_t* output);
eIcicleError bls12_381_g1_projective_to_affine(const mbls_g1_projective_t* input, int size, const VecOpsConfig* config,
                                               mbls_g1_affine_t* output);
eIcicleError bls12_381_g2_projective_to_affine(const mbls_g2_projective_t* input, int size, const VecOpsConfig* config,
                                               mbls_g2_affine_t* output);

/* ------------------------------------------------------------------------------------ */
/* library utilities (no reference counterpart; used by the host API, tests and bench)   */
/* ------------------------------------------------------------------------------------ */
const char* mbls_version(void);
const char* mbls_error_string(eIcicleError e);
/* Fill `out` (device) with n synthetic scalars of stream `seed` (standard form if
 * montgomery == false).  Same stream as the oracle's orc_gen_scalars. */
eIcicleError mbls_gen_scalars(mbls_fr_t* out_device, uint64_t seed, size_t n, bool montgomery, void* stream);
/* Fill `out` (device) with P_i = k_i * G, k_i = scalar stream `seed` (affine Montgomery). */
eIcicleError mbls_gen_g1_bases(mbls_g1_affine_t* out_device, uint64_t seed, size_t n, void* stream);
eIcicleError mbls_gen_g2_bases(mbls_g2_affine_t* out_device, uint64_t seed, size_t n, void* stream);
/* The same streams from element `start` on (out[j] = element start + j): one rank of a sharded
 * run generates exactly its slice of the global inputs. */
eIcicleError mbls_gen_scalars_range(mbls_fr_t* out_device, uint64_t seed, size_t start, size_t n, bool montgomery,
                                    void* stream);
eIcicleError mbls_gen_g1_bases_range(mbls_g1_affine_t* out_device, uint64_t seed, size_t start, size_t n, void* stream);
eIcicleError mbls_gen_g2_bases_range(mbls_g2_affine_t* out_device, uint64_t seed, size_t start, size_t n, void* stream);
/* One rank's step of the sharded multi-GPU MSM (the reference has no
 * multi-GPU path): the inputs and flags of bls12_381_icicle_g*_msm, but the result is left
 * as the Jacobian Montgomery partial sum (no (x, y, 1) normalisation), so the partials of all
 * ranks can be all-gathered, added with mbls_g*_sum_jacobian and normalised once with
 * mbls_g*_jacobian_to_icicle. */
eIcicleError mbls_g1_msm_jacobian(const mbls_fr_t* scalars, const mbls_g1_affine_t* bases, int msm_size,
                                  const MSMConfig* config, mbls_g1_projective_t* results);
eIcicleError mbls_g2_msm_jacobian(const mbls_fr_t* scalars, const mbls_g2_affine_t* bases, int msm_size,
                                  const MSMConfig* config, mbls_g2_projective_t* results);
/* Sum `count` Jacobian-Montgomery points on device (the EC reduction after the multi-GPU
 * all-gather of partial MSM results). result: device pointer, Jacobian Montgomery. */
eIcicleError mbls_g1_sum_jacobian(const mbls_g1_projective_t* points_device, int count,
                                  mbls_g1_projective_t* result_device, void* stream);
eIcicleError mbls_g2_sum_jacobian(const mbls_g2_projective_t* points_device, int count,
                                  mbls_g2_projective_t* result_device, void* stream);
/* Jacobian Montgomery -> ICICLE standard projective (x, y, 1) / (0, 1, 0), in place on
 * device (reference icicle_curve_api.cu:134-229). */
eIcicleError mbls_g1_jacobian_to_icicle(mbls_g1_projective_t* points_device, int count, void* stream);
eIcicleError mbls_g2_jacobian_to_icicle(mbls_g2_projective_t* points_device, int count, void* stream);

/* Scratch ownership.  Device scratch comes from a small per-device pool of contexts (arena +
 * side streams) LEASED per call, never keyed by the caller's stream: the reference's async
 * MSM creates a stream per call and destroys it afterwards (core/msm.rs:742, stream.rs:189),
 * and the reference itself allocates and frees scratch inside every call
 * (msm_kernels.cu:705-719, :872-902).  Here a context's arena grows to the high-water mark and
 * is reused by later calls on any stream; no hipMalloc happens once it is large enough.
 *   mbls_release_stream: the stream is about to be destroyed (ICICLE DeviceAPI
 *     destroy_stream calls it): forget it as a context's last stream, so a new stream that
 *     reuses the handle value is never taken to be ordered after the old one's work.
 *   mbls_release_scratch: free the arenas of all idle contexts (after their last work).
 *   mbls_scratch_stats: library hipMalloc / hipFree counts of scratch arenas, bytes held,
 *     number of pool contexts (any pointer may be NULL). */
eIcicleError mbls_release_stream(void* stream);
eIcicleError mbls_release_scratch(void);
void mbls_scratch_stats(uint64_t* mallocs, uint64_t* frees, uint64_t* bytes, int* contexts);

/* Multi-device G1 MSM for a single-process caller (SURVEY.md section 8e in one process; the
 * reference's Rust core binds one device per process, core/config.rs:529-531, core/msm.rs:284).
 * Shard k = points [k*n/ndev, (k+1)*n/ndev) runs on device devs[k] against bases_per_dev[k]
 * (that shard's bases, resident on devs[k]; flags as config->are_points_*); `scalars` holds all
 * n scalars, on the host or on device devs[0] per config->are_scalars_on_device.  Each shard
 * leaves its Jacobian partial sum on its device, the partials (144 B each) are copied peer to
 * peer to devs[0], summed there and normalised once to ICICLE's (x, y, 1).  devs may repeat a
 * device (shards then run one after another on it).  `result`: host or device (devs[0]) per
 * config->are_results_on_device.  config->stream, if set, is a stream of devs[0]; the other
 * shards use library streams forked from it.  batch_size must be 1 and precompute_factor 1.
 * Concurrent multi-device calls from several host threads serialise (one library lock). */
eIcicleError mbls_g1_msm_multi_device(const mbls_fr_t* scalars, const mbls_g1_affine_t* const* bases_per_dev,
                                      const int* devs, int ndev, int msm_size, const MSMConfig* config,
                                      mbls_g1_projective_t* result);
/* the same for G2 (288-byte partials) */
eIcicleError mbls_g2_msm_multi_device(const mbls_fr_t* scalars, const mbls_g2_affine_t* const* bases_per_dev,
                                      const int* devs, int ndev, int msm_size, const MSMConfig* config,
                                      mbls_g2_projective_t* result);

/* ICICLE vector_sum with the staged semantics of the other vecops (host or device input,
 * batch_size sums of `size` elements, row-major batches; result host or device). */
eIcicleError bls12_381_vector_sum(const mbls_fr_t* a, size_t size, const VecOpsConfig* config, mbls_fr_t* output);

/* The MSM schedule the library picks for msm_size points under `config` (make_plan; host
 * only, no device work): out[0..9] = window bits c, windows W, windows per table block Wg, the
 * plan's precompute factor F (1 once a split plan takes the table), block shift sF (0: none),
 * split (1 none, 2 G1 GLV, 4 G2 psi), prepared endomorphism table (0 / 1), slot-0 stride (1:
 * none; F: the split plan on entry i F of a shift table), buckets, reduction levels.
 * group: 1 = G1, 2 = G2.  Diagnostics (tests/test_plan.py, tools/). */
eIcicleError mbls_msm_plan(int group, int msm_size, const MSMConfig* config, int32_t* out);

/* Stage profiler (tracing): hipEvent pairs recorded on the caller's
 * stream around each pipeline stage ("msm.accumulate", "ntt.pass", ...) when enabled
 * (or MBLS_PROFILE=1).  read() synchronises the recorded events and returns, per stage,
 * the total milliseconds and the number of recorded launches. */
void mbls_profile_enable(int on);
void mbls_profile_reset(void);
int mbls_profile_read(const char** names, double* total_ms, long* counts, int max);

/* Scheduling extension (no reference counterpart): the NEXT MSM call on `stream` takes `event`
 * and records it on that stream once its (last member's) bucket accumulation has been enqueued,
 * i.e. the event completes when the MSM enters its latency-bound tail (bucket sums, reduction
 * levels, final fold: ~2.5 ms of few-wave chains for G2 2^20).  Work made to wait on it from
 * another stream -- a batch of NTTs, say -- then fills the SIMDs the tail leaves idle instead of
 * time-slicing them with the VALU-bound accumulation (config #5, bench.py mix leg; give the MSM's
 * stream the higher priority).  Every MSM call that gets past its argument checks takes the
 * pending event: a batch records it after the LAST member's accumulation; an empty MSM, a
 * multi-device call (at its end, on the caller's stream) and a call that fails after taking it
 * record it where they stop, so it never lingers for an unrelated later MSM.  One pending event
 * per stream; a later call replaces it; mbls_msm_accumulate_event(stream, NULL) clears it.  The
 * event is the caller's: mbls_msm_accumulate_event_drop(event) removes every pending
 * registration of it (call it before destroying an event that may still be pending). */
eIcicleError mbls_msm_accumulate_event(void* stream, void* event);
eIcicleError mbls_msm_accumulate_event_drop(void* event);

/* precompute_factor guard (no reference counterpart).  The reference's plain
 * device-bases MSMs pass MIDNIGHT_GPU_PRECOMPUTE as precompute_factor with n PLAIN bases
 * (core/msm.rs:897-913).  Default: a device allocation too short for n x F entries runs as plain
 * bases (a sub-allocated buffer of a larger pool is not caught).  Strict (on != 0, process-wide):
 * precompute_factor > 1 is honoured only for a table this library's precompute_bases wrote to
 * device memory (same pointer, same factor, entries covering the call) and every other buffer
 * runs as plain bases -- exact for pooled buffers; a table assembled elsewhere (copied or
 * concatenated) then needs precompute_factor = 1 semantics or its own precompute_bases call. */
eIcicleError mbls_msm_precompute_strict(int on);

#ifdef __cplusplus
}
#endif
#endif /* BLS12_381_MI355X_H */
