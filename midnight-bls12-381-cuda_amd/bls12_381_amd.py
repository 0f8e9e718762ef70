"""ctypes binding of libbls12_381_mi355x.so (the C ABI in include/bls12_381_mi355x.h).

Thin: config structs, error mapping, and numpy/torch conveniences for tests and bench.
There is no CPU fallback -- if the HIP library is missing or fails to load this module raises.
Device buffers are torch tensors (torch is plumbing here: allocation + streams)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MBLS_LIB: an alternative in-tree build of the same library (A/B tuning runs only)
LIB_PATH = os.environ.get("MBLS_LIB") or os.path.join(HERE, "lib", "libbls12_381_mi355x.so")

ERRORS = ["SUCCESS", "INVALID_DEVICE", "OUT_OF_MEMORY", "INVALID_POINTER", "ALLOCATION_FAILED",
          "DEALLOCATION_FAILED", "COPY_FAILED", "SYNCHRONIZATION_FAILED", "STREAM_CREATION_FAILED",
          "STREAM_DESTRUCTION_FAILED", "API_NOT_IMPLEMENTED", "INVALID_ARGUMENT", "BACKEND_LOAD_FAILED",
          "LICENSE_CHECK_ERROR", "UNKNOWN_ERROR"]
SUCCESS, INVALID_POINTER, API_NOT_IMPLEMENTED, INVALID_ARGUMENT = 0, 3, 10, 11


class IcicleError(RuntimeError):
    def __init__(self, code, what):
        name = ERRORS[code] if 0 <= code < len(ERRORS) else str(code)
        super().__init__(f"{what} failed: {name} ({code})")
        self.code = code


class MSMConfig(ctypes.Structure):
    _fields_ = [("stream", ctypes.c_void_p), ("precompute_factor", ctypes.c_int), ("c", ctypes.c_int),
                ("bitsize", ctypes.c_int), ("batch_size", ctypes.c_int),
                ("are_points_shared_in_batch", ctypes.c_bool), ("are_scalars_on_device", ctypes.c_bool),
                ("are_scalars_montgomery_form", ctypes.c_bool), ("are_points_on_device", ctypes.c_bool),
                ("are_points_montgomery_form", ctypes.c_bool), ("are_results_on_device", ctypes.c_bool),
                ("is_async", ctypes.c_bool), ("ext", ctypes.c_void_p)]


class FrC(ctypes.Structure):
    _fields_ = [("limbs", ctypes.c_uint64 * 4)]


class NTTConfig(ctypes.Structure):
    _fields_ = [("stream", ctypes.c_void_p), ("coset_gen", FrC), ("batch_size", ctypes.c_int),
                ("columns_batch", ctypes.c_bool), ("ordering", ctypes.c_int),
                ("are_inputs_on_device", ctypes.c_bool), ("are_outputs_on_device", ctypes.c_bool),
                ("is_async", ctypes.c_bool), ("ext", ctypes.c_void_p)]


class NTTInitDomainConfig(ctypes.Structure):
    _fields_ = [("stream", ctypes.c_void_p), ("is_async", ctypes.c_bool), ("ext", ctypes.c_void_p)]


class VecOpsConfig(ctypes.Structure):
    _fields_ = [("stream", ctypes.c_void_p), ("is_a_on_device", ctypes.c_bool), ("is_b_on_device", ctypes.c_bool),
                ("is_result_on_device", ctypes.c_bool), ("is_async", ctypes.c_bool), ("batch_size", ctypes.c_int),
                ("columns_batch", ctypes.c_bool), ("ext", ctypes.c_void_p)]


# every symbol include/bls12_381_mi355x.h declares (checked by tests/test_abi.py)
EXPORTED = [
    "mbls_default_msm_config", "mbls_default_ntt_config", "mbls_default_vec_ops_config",
    "bls12_381_g1_msm_cuda", "bls12_381_g2_msm_cuda", "bls12_381_icicle_g1_msm", "bls12_381_icicle_g2_msm",
    "bls12_381_icicle_g1_msm_precompute_bases", "bls12_381_icicle_g2_msm_precompute_bases",
    "bls12_381_ntt_init_domain_cuda", "bls12_381_ntt_release_domain_cuda", "bls12_381_ntt_cuda",
    "bls12_381_coset_ntt_cuda", "bls12_381_field_ntt_cuda", "bls12_381_field_ntt_init_domain_cuda",
    "bls12_381_field_ntt_release_domain_cuda", "bls12_381_ntt_get_rou_from_domain",
    "bls12_381_vector_add", "bls12_381_vector_sub", "bls12_381_vector_mul", "bls12_381_scalar_mul_vec",
    "bls12_381_scalar_add_vec", "vec_add_cuda", "vec_sub_cuda", "vec_mul_cuda", "scalar_mul_vec_cuda",
    "scalar_add_vec_cuda", "vec_sum_cuda", "bls12_381_batch_inv_cuda",
    "mbls_version", "mbls_error_string", "mbls_gen_scalars", "mbls_gen_g1_bases", "mbls_gen_g2_bases",
    "mbls_gen_scalars_range", "mbls_gen_g1_bases_range", "mbls_gen_g2_bases_range",
    "mbls_g1_msm_jacobian", "mbls_g2_msm_jacobian",
    "mbls_g1_sum_jacobian", "mbls_g2_sum_jacobian", "mbls_g1_jacobian_to_icicle", "mbls_g2_jacobian_to_icicle",
    "mbls_profile_enable", "mbls_profile_reset", "mbls_profile_read",
    "mbls_release_stream", "mbls_release_scratch", "mbls_scratch_stats",
    "mbls_g1_msm_multi_device", "mbls_g2_msm_multi_device", "bls12_381_vector_sum",
    "bls12_381_g1_affine_to_projective", "bls12_381_g1_projective_to_affine", "bls12_381_g2_projective_to_affine",
    "mbls_msm_plan", "mbls_msm_accumulate_event", "mbls_msm_accumulate_event_drop", "mbls_msm_precompute_strict",
]

_LIB = None


def lib():
    """Load the HIP library (raises if it is missing: there is no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"HIP library not built: {LIB_PATH} (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    P, E = ctypes.c_void_p, ctypes.c_int
    sz, i32, u64, b = ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64, ctypes.c_bool
    sig = {
        "bls12_381_g1_msm_cuda": [P, P, i32, P, P], "bls12_381_g2_msm_cuda": [P, P, i32, P, P],
        "bls12_381_icicle_g1_msm": [P, P, i32, P, P], "bls12_381_icicle_g2_msm": [P, P, i32, P, P],
        "bls12_381_icicle_g1_msm_precompute_bases": [P, i32, P, P],
        "bls12_381_icicle_g2_msm_precompute_bases": [P, i32, P, P],
        "bls12_381_ntt_init_domain_cuda": [P, P], "bls12_381_ntt_release_domain_cuda": [],
        "bls12_381_ntt_cuda": [P, i32, i32, P, P], "bls12_381_coset_ntt_cuda": [P, i32, i32, P, P, P],
        "bls12_381_field_ntt_cuda": [P, i32, i32, P, P], "bls12_381_field_ntt_init_domain_cuda": [P, P],
        "bls12_381_field_ntt_release_domain_cuda": [], "bls12_381_ntt_get_rou_from_domain": [u64, P],
        "bls12_381_vector_add": [P, P, sz, P, P], "bls12_381_vector_sub": [P, P, sz, P, P],
        "bls12_381_vector_mul": [P, P, sz, P, P], "bls12_381_scalar_mul_vec": [P, P, sz, P, P],
        "bls12_381_scalar_add_vec": [P, P, sz, P, P],
        "vec_add_cuda": [P, P, P, i32, P], "vec_sub_cuda": [P, P, P, i32, P], "vec_mul_cuda": [P, P, P, i32, P],
        "scalar_mul_vec_cuda": [P, P, P, i32, P], "scalar_add_vec_cuda": [P, P, P, i32, P],
        "vec_sum_cuda": [P, P, i32, P], "bls12_381_batch_inv_cuda": [P, P, i32, P],
        "mbls_gen_scalars": [P, u64, sz, b, P], "mbls_gen_g1_bases": [P, u64, sz, P],
        "mbls_gen_g2_bases": [P, u64, sz, P], "mbls_g1_sum_jacobian": [P, i32, P, P],
        "mbls_gen_scalars_range": [P, u64, sz, sz, b, P], "mbls_gen_g1_bases_range": [P, u64, sz, sz, P],
        "mbls_gen_g2_bases_range": [P, u64, sz, sz, P],
        "mbls_g1_msm_jacobian": [P, P, i32, P, P], "mbls_g2_msm_jacobian": [P, P, i32, P, P],
        "mbls_g2_sum_jacobian": [P, i32, P, P], "mbls_g1_jacobian_to_icicle": [P, i32, P],
        "mbls_g2_jacobian_to_icicle": [P, i32, P],
        "mbls_release_stream": [P], "mbls_release_scratch": [],
        "mbls_g1_msm_multi_device": [P, P, P, i32, i32, P, P], "mbls_g2_msm_multi_device": [P, P, P, i32, i32, P, P],
        "bls12_381_vector_sum": [P, sz, P, P],
        "bls12_381_g1_affine_to_projective": [P, i32, P, P], "bls12_381_g1_projective_to_affine": [P, i32, P, P],
        "bls12_381_g2_projective_to_affine": [P, i32, P, P],
        "mbls_msm_plan": [i32, i32, P, P],
        "mbls_msm_accumulate_event": [P, P], "mbls_msm_accumulate_event_drop": [P],
        "mbls_msm_precompute_strict": [i32],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = E
    L.mbls_version.restype = ctypes.c_char_p
    L.mbls_error_string.restype = ctypes.c_char_p
    L.mbls_error_string.argtypes = [E]
    L.mbls_default_msm_config.restype = MSMConfig
    L.mbls_default_ntt_config.restype = NTTConfig
    L.mbls_default_vec_ops_config.restype = VecOpsConfig
    L.mbls_profile_enable.argtypes = [ctypes.c_int]
    L.mbls_profile_enable.restype = None
    L.mbls_profile_reset.argtypes = []
    L.mbls_profile_reset.restype = None
    L.mbls_profile_read.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                    ctypes.POINTER(ctypes.c_long), ctypes.c_int]
    L.mbls_profile_read.restype = ctypes.c_int
    L.mbls_scratch_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 3 + [ctypes.POINTER(ctypes.c_int)]
    L.mbls_scratch_stats.restype = None
    _LIB = L
    return L


def profile(enable=True):
    lib().mbls_profile_enable(1 if enable else 0)
    lib().mbls_profile_reset()


def profile_read():
    """{stage: (total_ms, launches)} since the last profile()/reset"""
    n = 64
    names = (ctypes.c_char_p * n)()
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_long * n)()
    k = lib().mbls_profile_read(names, ms, cnt, n)
    return {names[i].decode(): (ms[i], cnt[i]) for i in range(min(k, n))}


def check(code, what):
    if code != SUCCESS:
        raise IcicleError(code, what)


def _p(x):
    """pointer of a numpy array or torch tensor"""
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        assert x.flags["C_CONTIGUOUS"]
        return ctypes.c_void_p(x.ctypes.data)
    return ctypes.c_void_p(x.data_ptr())


def _is_dev(x):
    """device operand: a torch tensor on the GPU (numpy arrays and CPU / pinned torch tensors
    are host memory)"""
    return x is not None and not isinstance(x, np.ndarray) and bool(getattr(x, "is_cuda", True))


def _stream_handle(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)


# ----------------------------------------------------------------------------- configs
def msm_config(**kw):
    c = lib().mbls_default_msm_config()
    for k, v in kw.items():
        if k == "stream":
            c.stream = _stream_handle(v)
        else:
            setattr(c, k, v)
    return c


PLAN_FIELDS = ("c", "W", "Wg", "F", "sF", "split", "prepared", "bstride", "buckets", "levels")


def msm_plan(group, n, **cfg):
    """the MSM schedule the library picks (mbls_msm_plan; host only): dict of PLAN_FIELDS"""
    out = (ctypes.c_int32 * len(PLAN_FIELDS))()
    c = msm_config(**cfg)
    check(lib().mbls_msm_plan(1 if group == "g1" else 2, n, ctypes.byref(c), out), "msm_plan")
    return dict(zip(PLAN_FIELDS, list(out)))


def ntt_config(**kw):
    c = lib().mbls_default_ntt_config()
    for k, v in kw.items():
        if k == "stream":
            c.stream = _stream_handle(v)
        elif k == "coset_gen":
            for i in range(4):
                c.coset_gen.limbs[i] = int(v[i])
        else:
            setattr(c, k, v)
    return c


def vec_config(**kw):
    c = lib().mbls_default_vec_ops_config()
    for k, v in kw.items():
        if k == "stream":
            c.stream = _stream_handle(v)
        else:
            setattr(c, k, v)
    return c


# ----------------------------------------------------------------------------- vecops
_VEC = {"add": "bls12_381_vector_add", "sub": "bls12_381_vector_sub", "mul": "bls12_381_vector_mul",
        "scalar_mul": "bls12_381_scalar_mul_vec", "scalar_add": "bls12_381_scalar_add_vec"}


def vec_op(op, a, b, out=None, stream=None, is_async=False, batch=1, columns_batch=False):
    """a, b: (batch*n,4) uint64 numpy (host) or torch (device) arrays; for scalar ops `a`
    holds one element per batch member (host numpy unless it is a device tensor)."""
    total = b.shape[0]
    if out is None:
        out = np.zeros((total, 4), dtype=np.uint64)
    cfg = vec_config(is_a_on_device=_is_dev(a), is_b_on_device=_is_dev(b), is_result_on_device=_is_dev(out),
                     is_async=is_async, stream=stream, batch_size=batch, columns_batch=columns_batch)
    check(getattr(lib(), _VEC[op])(_p(a), _p(b), total // batch, ctypes.byref(cfg), _p(out)), _VEC[op])
    return out


# ----------------------------------------------------------------------------- point forms
_CONV = {("g1", "to_projective"): ("bls12_381_g1_affine_to_projective", 18),
         ("g1", "to_affine"): ("bls12_381_g1_projective_to_affine", 12),
         ("g2", "to_affine"): ("bls12_381_g2_projective_to_affine", 24)}


def convert_points(group, direction, pts, out=None, stream=None, is_async=False):
    """Batch point-form conversion (reference point_ops.cu:759,844,924): `pts` is (n, k) uint64
    (numpy host or torch device), Montgomery; returns (n, k') in the other form."""
    name, words = _CONV[(group, direction)]
    n = pts.shape[0]
    if out is None:
        out = np.zeros((n, words), dtype=np.uint64)
    cfg = vec_config(is_a_on_device=_is_dev(pts), is_result_on_device=_is_dev(out), stream=stream, is_async=is_async)
    check(getattr(lib(), name)(_p(pts), n, ctypes.byref(cfg), _p(out)), name)
    return out


def vec_sum(x, out=None, stream=None):
    """sum of the device tensor x (n,4) -> (1,4) numpy (host) unless `out` is a device tensor"""
    if out is None:
        out = np.zeros((1, 4), dtype=np.uint64)
    cfg = vec_config(is_a_on_device=True, is_b_on_device=True, is_result_on_device=_is_dev(out), stream=stream)
    check(lib().vec_sum_cuda(_p(out), _p(x), x.shape[0], ctypes.byref(cfg)), "vec_sum_cuda")
    return out


def vector_sum(a, batch=1, out=None, stream=None, is_async=False):
    """ICICLE vector_sum (bls12_381_vector_sum): `batch` row-major sums of a (batch*n, 4), host
    numpy or device torch -> (batch, 4) numpy unless `out` is a device tensor"""
    if out is None:
        out = np.zeros((batch, 4), dtype=np.uint64)
    cfg = vec_config(is_a_on_device=_is_dev(a), is_b_on_device=True, is_result_on_device=_is_dev(out),
                     stream=stream, batch_size=batch, is_async=is_async)
    check(lib().bls12_381_vector_sum(_p(a), a.shape[0] // batch, ctypes.byref(cfg), _p(out)), "bls12_381_vector_sum")
    return out


def batch_inv(x, out, stream=None):
    """element-wise inverses of device tensor x into device tensor out (may be x)"""
    cfg = vec_config(stream=stream)
    check(lib().bls12_381_batch_inv_cuda(_p(out), _p(x), x.shape[0], ctypes.byref(cfg)), "bls12_381_batch_inv_cuda")
    return out


# ----------------------------------------------------------------------------- NTT
def ntt_init_domain(root_mont=None):
    if root_mont is None:  # canonical 2^32-th root, Montgomery form
        root_mont = np.array([0xb9b58d8c5f0e466a, 0x5b1b4c801819d7ec, 0x0af53ae352a31e64, 0x5bf3adda19e9b27b],
                             dtype=np.uint64)
    cfg = NTTInitDomainConfig()
    check(lib().bls12_381_ntt_init_domain_cuda(_p(np.ascontiguousarray(root_mont, dtype=np.uint64)),
                                               ctypes.byref(cfg)), "ntt_init_domain")


ORDERINGS = {"NN": 0, "NR": 1, "RN": 2, "RR": 3, "NM": 4, "MN": 5}


def ntt(x, inverse=False, out=None, batch=1, stream=None, is_async=False, coset_gen=None, ordering="NN",
        columns_batch=False):
    """x: (batch*n, 4) uint64 numpy (host) or torch (device)."""
    total = x.shape[0]
    n = total // batch
    if out is None:
        out = np.zeros((total, 4), dtype=np.uint64) if isinstance(x, np.ndarray) else None
    kw = dict(batch_size=batch, are_inputs_on_device=_is_dev(x), are_outputs_on_device=_is_dev(out),
              is_async=is_async, stream=stream, ordering=ORDERINGS[ordering], columns_batch=columns_batch)
    if coset_gen is not None:
        kw["coset_gen"] = coset_gen
    cfg = ntt_config(**kw)
    check(lib().bls12_381_ntt_cuda(_p(x), n, 1 if inverse else 0, ctypes.byref(cfg), _p(out)), "ntt")
    return out


# ----------------------------------------------------------------------------- MSM
def msm(group, scalars, bases, *, icicle=True, scalars_mont=False, points_mont=True, c=0, bitsize=0,
        precompute_factor=1, batch=1, shared_bases=True, out=None, stream=None, is_async=False, n=None):
    """scalars (batch*n, 4) u64, bases (n*F[*batch], 12|24) u64; host numpy or device torch.
    icicle=True -> ICICLE semantics (standard (x, y, 1)); False -> the reference's raw entry
    (standard scalars, Jacobian Montgomery); "jacobian" -> ICICLE inputs, Jacobian Montgomery
    result (one rank's step of the sharded MSM)."""
    nl = 18 if group == "g1" else 36
    if n is None:
        n = scalars.shape[0] // batch
    if out is None:
        out = np.zeros((batch, nl), dtype=np.uint64)
    cfg = msm_config(c=c, bitsize=bitsize, precompute_factor=precompute_factor, batch_size=batch,
                     are_points_shared_in_batch=shared_bases, are_scalars_on_device=_is_dev(scalars),
                     are_scalars_montgomery_form=scalars_mont, are_points_on_device=_is_dev(bases),
                     are_points_montgomery_form=points_mont, are_results_on_device=_is_dev(out),
                     is_async=is_async, stream=stream)
    if icicle == "jacobian":
        fn = lib().mbls_g1_msm_jacobian if group == "g1" else lib().mbls_g2_msm_jacobian
    elif icicle:
        fn = lib().bls12_381_icicle_g1_msm if group == "g1" else lib().bls12_381_icicle_g2_msm
    else:
        fn = lib().bls12_381_g1_msm_cuda if group == "g1" else lib().bls12_381_g2_msm_cuda
    check(fn(_p(scalars), _p(bases), n, ctypes.byref(cfg), _p(out)), f"{group} msm")
    return out


def precompute_bases(group, bases, factor, n, c=0, out=None, points_mont=True):
    """ICICLE precompute_bases: out[i*factor + f] = 2^(s f) P_i, s = ceil(256 / factor) (the
    shift depends on the factor only, so c is irrelevant); output Montgomery affine."""
    nl = 12 if group == "g1" else 24
    if out is None:
        out = np.zeros((n * factor, nl), dtype=np.uint64)
    cfg = msm_config(precompute_factor=factor, c=c, are_points_on_device=_is_dev(bases),
                     are_points_montgomery_form=points_mont, are_results_on_device=_is_dev(out))
    fn = (lib().bls12_381_icicle_g1_msm_precompute_bases if group == "g1"
          else lib().bls12_381_icicle_g2_msm_precompute_bases)
    check(fn(_p(bases), n, ctypes.byref(cfg), _p(out)), "precompute_bases")
    return out


# ----------------------------------------------------------------------------- utilities
def gen_scalars(out_dev, seed, montgomery=False, stream=None, start=0):
    """elements start .. start + len(out_dev) - 1 of scalar stream `seed`"""
    check(lib().mbls_gen_scalars_range(_p(out_dev), seed, start, out_dev.shape[0], montgomery,
                                       _stream_handle(stream)), "gen_scalars")


def gen_bases(group, out_dev, seed, stream=None, start=0):
    fn = lib().mbls_gen_g1_bases_range if group == "g1" else lib().mbls_gen_g2_bases_range
    check(fn(_p(out_dev), seed, start, out_dev.shape[0], _stream_handle(stream)), "gen_bases")


def msm_multi_device(group, scalars, bases_per_dev, devs, n, *, scalars_mont=True, points_mont=True, out=None,
                     stream=None, is_async=False):
    """mbls_g*_msm_multi_device: shard k of n points runs on devs[k] with bases_per_dev[k] (that
    shard's bases, device tensors); scalars host numpy or device torch (devs[0]); ICICLE (x, y, 1)
    result (host numpy unless `out` is a device tensor on devs[0])"""
    nl = 18 if group == "g1" else 36
    if out is None:
        out = np.zeros((1, nl), dtype=np.uint64)
    k = len(devs)
    ptrs = (ctypes.c_void_p * k)(*[b.data_ptr() for b in bases_per_dev])
    dv = (ctypes.c_int * k)(*devs)
    cfg = msm_config(are_scalars_on_device=_is_dev(scalars), are_scalars_montgomery_form=scalars_mont,
                     are_points_on_device=True, are_points_montgomery_form=points_mont,
                     are_results_on_device=_is_dev(out), is_async=is_async, stream=stream)
    fn = lib().mbls_g1_msm_multi_device if group == "g1" else lib().mbls_g2_msm_multi_device
    check(fn(_p(scalars), ptrs, dv, k, n, ctypes.byref(cfg), _p(out)), f"{group} msm_multi_device")
    return out


def msm_accumulate_event(stream, event):
    """mbls_msm_accumulate_event: the next single MSM on `stream` records the raw hipEvent_t
    `event` (an int handle, or None to clear) when its accumulation is enqueued (its tail starts)"""
    check(lib().mbls_msm_accumulate_event(_stream_handle(stream), ctypes.c_void_p(event) if event else None),
          "mbls_msm_accumulate_event")


class HipEvent:
    """a raw hipEvent_t (timing disabled) that another stream can wait on (hipStreamWaitEvent)"""

    def __init__(self):
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        self.hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
        self.hip.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        self.ev = ctypes.c_void_p()
        if self.hip.hipEventCreateWithFlags(ctypes.byref(self.ev), 2) != 0:  # hipEventDisableTiming
            raise RuntimeError("hipEventCreateWithFlags failed")

    @property
    def handle(self):
        return self.ev.value

    def wait(self, stream):
        """make `stream` (torch stream) wait for the event"""
        if self.hip.hipStreamWaitEvent(_stream_handle(stream), self.ev, 0) != 0:
            raise RuntimeError("hipStreamWaitEvent failed")

    def query(self):
        """True when the event has completed (or was never recorded), False while pending"""
        self.hip.hipEventQuery.argtypes = [ctypes.c_void_p]
        r = self.hip.hipEventQuery(self.ev)
        if r not in (0, 600):  # hipSuccess, hipErrorNotReady
            raise RuntimeError(f"hipEventQuery failed ({r})")
        return r == 0

    def __del__(self):
        try:
            # a registration still pending for this event must not outlive it
            lib().mbls_msm_accumulate_event_drop(self.ev)
            self.hip.hipEventDestroy(self.ev)
        except Exception:
            pass


def scratch_stats():
    """(library scratch hipMallocs, hipFrees, bytes held, pool contexts)"""
    m, f, b = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    c = ctypes.c_int()
    lib().mbls_scratch_stats(ctypes.byref(m), ctypes.byref(f), ctypes.byref(b), ctypes.byref(c))
    return m.value, f.value, b.value, c.value


def release_stream(stream):
    check(lib().mbls_release_stream(_stream_handle(stream)), "mbls_release_stream")


def release_scratch():
    check(lib().mbls_release_scratch(), "mbls_release_scratch")


def sum_jacobian(group, pts_dev, out_dev, stream=None):
    fn = lib().mbls_g1_sum_jacobian if group == "g1" else lib().mbls_g2_sum_jacobian
    check(fn(_p(pts_dev), pts_dev.shape[0], _p(out_dev), _stream_handle(stream)), "sum_jacobian")


def jacobian_to_icicle(group, pts_dev, stream=None):
    fn = lib().mbls_g1_jacobian_to_icicle if group == "g1" else lib().mbls_g2_jacobian_to_icicle
    check(fn(_p(pts_dev), pts_dev.shape[0], _stream_handle(stream)), "jacobian_to_icicle")


def torch_u64(shape_or_array, device="cuda"):
    """uint64 limb storage on the device (int64 dtype: torch is only the allocator)."""
    import torch
    if isinstance(shape_or_array, np.ndarray):
        return torch.from_numpy(shape_or_array.view(np.int64)).to(device)
    return torch.zeros(shape_or_array, dtype=torch.int64, device=device)


def to_numpy_u64(t):
    return t.detach().cpu().numpy().view(np.uint64)


def msm_precompute_strict(on=True):
    """mbls_msm_precompute_strict: precompute_factor > 1 only for tables precompute_bases wrote
    (include/bls12_381_mi355x.h); process-wide"""
    check(lib().mbls_msm_precompute_strict(1 if on else 0), "mbls_msm_precompute_strict")
