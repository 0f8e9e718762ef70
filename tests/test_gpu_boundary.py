"""Boundary behaviour of the HIP library under the reference's real call shapes (SURVEY.md 8b
"Ownership" / "Threading" / "Callers"), through the C ABI, bit-exact against the oracle:

* core/msm.rs:742 -> msm() -> stream.rs:189: a fresh stream per async MSM with PAGEABLE host
  Montgomery scalars (HostSlice, core/msm.rs:665,773), device bases, the result copied back to
  the host, the stream destroyed -- 200 times: no library hipMalloc after the first call and a
  flat hipMemGetInfo (scratch is pooled per device, not per stream handle);
* two host threads on two streams running MSM and NTT at once (rayon callers);
* the single-process multi-device MSM entry (mbls_g1_msm_multi_device);
* ICICLE vector_sum with staged host input (no per-call hipMalloc in the shim)."""
import ctypes
import threading

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu
ORACLE_THREADS = 16


@pytest.fixture(scope="module")
def amd():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import gpu_helpers
    gpu_helpers.amd.lib()
    return gpu_helpers.amd


@pytest.fixture(scope="module")
def gh():
    import gpu_helpers
    return gpu_helpers


@pytest.fixture(scope="module")
def hip():
    L = ctypes.CDLL("libamdhip64.so")
    L.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    L.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    L.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    L.hipMemGetInfo.argtypes = [ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
    return L


def _std_scalars(seed, n, start=0):
    s = np.zeros((start + n, 4), dtype=np.uint64)
    H.oracle().orc_gen_scalars(H.ptr(s), seed, start + n)
    return np.ascontiguousarray(s[start:])


def _free_bytes(hip):
    free, total = ctypes.c_size_t(), ctypes.c_size_t()
    assert hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) == 0
    return free.value


def test_msm_per_op_stream_create_destroy_200x(amd, gh, hip):
    """core/msm.rs:742 (ManagedStream::create) -> msm(HostSlice scalars, device bases, is_async,
    device result) -> copy_to_host -> stream.rs:189 (destroy), 200 times at 2^16: every result
    equals the oracle, the library makes no scratch hipMalloc after the first call, and the free
    device memory stays flat (a per-stream arena would leak ~0.1 GB per call or hipMalloc it)"""
    import torch
    n, nsets = 1 << 16, 4
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0B01)
    bn = amd.to_numpy_u64(b)
    sets, refs = [], []
    for k in range(nsets):
        d = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        amd.gen_scalars(d, 0x5EED0B10 + k, montgomery=True)
        sets.append(np.ascontiguousarray(amd.to_numpy_u64(d)))  # pageable host Montgomery scalars
        refs.append(H.g1_from_affine_mont(H.oracle_msm("g1", _std_scalars(0x5EED0B10 + k, n), bn,
                                                       threads=ORACLE_THREADS)))
    torch.cuda.synchronize()
    dres = torch.zeros((1, 18), dtype=torch.int64, device="cuda")  # DeviceVec::device_malloc(1)
    m0 = f0 = None
    for it in range(200):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0  # hipStreamNonBlocking
        amd.msm("g1", sets[it % nsets], b, scalars_mont=True, out=dres, stream=s.value, is_async=True, n=n)
        assert hip.hipStreamSynchronize(s) == 0  # copy_to_host is ordered after the MSM
        host = amd.to_numpy_u64(dres)
        amd.release_stream(s.value)  # what HipDeviceAPI::destroy_stream does first
        assert hip.hipStreamDestroy(s) == 0
        assert gh.decode_icicle("g1", host[0]) == refs[it % nsets], it
        if it == 0:
            torch.cuda.synchronize()
            m0, f0 = amd.scratch_stats()[0], _free_bytes(hip)
    mallocs, frees, held, ctxs = amd.scratch_stats()
    assert mallocs == m0, (m0, mallocs)
    assert abs(_free_bytes(hip) - f0) < (64 << 20)
    assert ctxs <= 4


def test_two_threads_msm_and_ntt_concurrent(amd, gh):
    """two host threads, each on its own stream: one runs G1 MSMs with host scalars, the other
    forward NTTs of device data; both interleave and both stay bit-exact (SURVEY.md 8b
    "Threading": rayon callers with a stream per op)"""
    import torch
    amd.ntt_init_domain()
    n, log_n, reps = 1 << 15, 16, 6
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0B21)
    d = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(d, 0x5EED0B22, montgomery=True)
    x = torch.zeros((1 << log_n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(x, 0x5EED0B23, montgomery=True)
    torch.cuda.synchronize()
    hs = np.ascontiguousarray(amd.to_numpy_u64(d))
    ref_msm = H.g1_from_affine_mont(H.oracle_msm("g1", _std_scalars(0x5EED0B22, n), amd.to_numpy_u64(b),
                                                 threads=ORACLE_THREADS))
    ref_ntt = H.oracle_ntt(amd.to_numpy_u64(x), log_n, False, threads=ORACLE_THREADS)
    errors, got_msm, got_ntt = [], [], []
    ys = [torch.zeros_like(x) for _ in range(reps)]  # allocated (and zero-filled) before the threads
    torch.cuda.synchronize()

    def msm_worker():
        try:
            st = torch.cuda.Stream()
            for _ in range(reps):
                got_msm.append(gh.decode_icicle("g1", amd.msm("g1", hs, b, scalars_mont=True, stream=st, n=n)[0]))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def ntt_worker():
        try:
            st = torch.cuda.Stream()
            for k in range(reps):
                amd.ntt(x, out=ys[k], stream=st)  # synchronous on st (is_async false)
                got_ntt.append(amd.to_numpy_u64(ys[k]))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=msm_worker), threading.Thread(target=ntt_worker)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors
    assert len(got_msm) == reps and len(got_ntt) == reps
    assert all(g == ref_msm for g in got_msm)
    assert all(np.array_equal(g, ref_ntt) for g in got_ntt)


@pytest.mark.parametrize("group,ndev", [("g1", 1), ("g1", 3), ("g2", 1), ("g2", 3)])
def test_msm_multi_device_entry(amd, gh, group, ndev):
    """mbls_g*_msm_multi_device (the single-process form of SURVEY.md 8e): shards of an uneven
    split, each with its own bases buffer, on device 0 (one GPU here: the shards run in turn),
    host and device scalars, host and device result -- equal to the oracle"""
    import torch
    n = (1 << 18) + 5 if group == "g1" else (1 << 14) + 5
    w, nl = (12, 18) if group == "g1" else (24, 36)
    dec = H.g1_from_affine_mont if group == "g1" else H.g2_from_affine_mont
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0B31, montgomery=True)
    b = torch.zeros((n, w), dtype=torch.int64, device="cuda")
    amd.gen_bases(group, b, 0x5EED0B32)
    torch.cuda.synchronize()
    ref = dec(H.oracle_msm(group, _std_scalars(0x5EED0B31, n), amd.to_numpy_u64(b), threads=ORACLE_THREADS))
    shards = [b[n * k // ndev:n * (k + 1) // ndev].clone() for k in range(ndev)]
    torch.cuda.synchronize()
    r = amd.msm_multi_device(group, s, shards, [0] * ndev, n)
    assert gh.decode_icicle(group, r[0]) == ref
    out = torch.zeros((1, nl), dtype=torch.int64, device="cuda")
    amd.msm_multi_device(group, np.ascontiguousarray(amd.to_numpy_u64(s)), shards, [0] * ndev, n, out=out)
    torch.cuda.synchronize()
    assert gh.decode_icicle(group, amd.to_numpy_u64(out)[0]) == ref
    with pytest.raises(amd.IcicleError):
        amd.msm_multi_device(group, s, shards, [99] * ndev, n)


def test_vector_sum_staged_batch(amd):
    """ICICLE vector_sum (bls12_381_vector_sum): host input staged in the pooled scratch, batch of
    3 row-major sums, against the oracle's sums"""
    import torch
    n, batch = 5000, 3
    x = torch.zeros((n * batch, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(x, 0x5EED0B41, montgomery=True)
    torch.cuda.synchronize()
    xn = np.ascontiguousarray(amd.to_numpy_u64(x))
    m0 = amd.scratch_stats()[0]
    got_host = amd.vector_sum(xn, batch=batch)
    got_dev = amd.vector_sum(x, batch=batch)
    for k in range(batch):
        acc = np.zeros((1, 4), dtype=np.uint64)
        tmp = np.zeros((1, 4), dtype=np.uint64)
        for row in xn[k * n:(k + 1) * n]:
            H.oracle().orc_vec_add(H.ptr(tmp), H.ptr(acc), H.ptr(np.ascontiguousarray(row.reshape(1, 4))), 1)
            acc[:] = tmp
        assert np.array_equal(got_host[k], acc[0]), k
        assert np.array_equal(got_dev[k], acc[0]), k
    assert amd.scratch_stats()[0] - m0 <= 1  # at most one arena growth, never per call


class _RawDev:
    """a bare hipMalloc'd buffer (the Rust DeviceVec::device_malloc shape) for the binding"""
    is_cuda = True

    def __init__(self, hip, nbytes):
        self.hip, self.p = hip, ctypes.c_void_p()
        hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        hip.hipFree.argtypes = [ctypes.c_void_p]
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        assert hip.hipMalloc(ctypes.byref(self.p), nbytes) == 0

    def data_ptr(self):
        return self.p.value

    def upload(self, arr):
        assert self.hip.hipMemcpy(self.p, arr.ctypes.data, arr.nbytes, 1) == 0  # hipMemcpyHostToDevice

    def free(self):
        self.hip.hipFree(self.p)


@pytest.mark.parametrize("group", ["g1", "g2"])
def test_precompute_factor_on_plain_device_bases(amd, gh, hip, group):
    """core/msm.rs:897-913 / 1025-1040 / 1097-1110 pass n plain device bases with
    cfg.precompute_factor = MIDNIGHT_GPU_PRECOMPUTE (4 recommended); the reference backend
    ignores the factor.  A device allocation too short for an n x F table runs as factor 1
    (INTEGRATION.md "precompute_factor on plain device bases")"""
    import torch
    n, w = 3000, (12 if group == "g1" else 24)
    b = torch.zeros((n, w), dtype=torch.int64, device="cuda")
    amd.gen_bases(group, b, 0x5EED0B01)
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0B02, montgomery=True)
    torch.cuda.synchronize()
    bn, sn = amd.to_numpy_u64(b), amd.to_numpy_u64(s)
    raw = _RawDev(hip, bn.nbytes)
    try:
        raw.upload(np.ascontiguousarray(bn))
        ref = amd.msm(group, sn, b, scalars_mont=True, n=n)
        dec = H.g1_from_affine_mont if group == "g1" else H.g2_from_affine_mont
        std = np.zeros((n, 4), dtype=np.uint64)
        H.oracle().orc_gen_scalars(H.ptr(std), 0x5EED0B02, n)
        assert gh.decode_icicle(group, ref[0]) == dec(H.oracle_msm(group, std, bn, threads=ORACLE_THREADS))
        for F in (2, 4, 8):
            r = amd.msm(group, sn, raw, scalars_mont=True, precompute_factor=F, n=n)
            assert np.array_equal(r, ref), F
    finally:
        raw.free()


@pytest.mark.parametrize("group", ["g1", "g2"])
def test_precompute_factor_pooled_plain_bases(amd, gh, group):
    """n plain bases in a sub-buffer of a larger pooled allocation (a caching
    allocator's segment) with precompute_factor 4.  Default mode: the allocation heuristic cannot
    tell them from a table -- pinned here as the KNOWN limitation (the result is not the plain
    MSM).  Strict mode (mbls_msm_precompute_strict): only tables precompute_bases wrote run as
    tables, so the pooled plain bases give the plain result, while a registered table still
    gives the table result."""
    import torch
    n, w, F = 2048, (12 if group == "g1" else 24), 4
    pool = torch.zeros((6 * n, w), dtype=torch.int64, device="cuda")  # one segment, several buffers
    plain = pool[n:2 * n]
    amd.gen_bases(group, plain, 0x5EED0B71)
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0B72, montgomery=True)
    torch.cuda.synchronize()
    ref = amd.msm(group, s, plain, scalars_mont=True, n=n)
    table = torch.zeros((n * F, w), dtype=torch.int64, device="cuda")
    amd.precompute_bases(group, plain, F, n, out=table)
    try:
        r = amd.msm(group, s, plain, scalars_mont=True, precompute_factor=F, n=n)
        assert not np.array_equal(r, ref), "default mode: pooled plain bases read as a table (known)"
        amd.msm_precompute_strict(True)
        r = amd.msm(group, s, plain, scalars_mont=True, precompute_factor=F, n=n)
        assert np.array_equal(r, ref), "strict mode: pooled plain bases run as plain"
        r = amd.msm(group, s, table, scalars_mont=True, points_mont=False, precompute_factor=F, n=n)
        assert np.array_equal(r, ref), "strict mode: a registered table still runs as a table"
        r = amd.msm(group, s, table[n:], scalars_mont=True, precompute_factor=F, n=n // 2)
        assert gh.decode_icicle(group, r[0]) is not None  # an unregistered pointer: plain, no fault
    finally:
        amd.msm_precompute_strict(False)


def test_msm_accumulate_event_orders_a_second_stream(amd, gh):
    """mbls_msm_accumulate_event (config #5's overlap): the next MSM on the stream records the
    event once its accumulation is enqueued; an NTT on another stream waits on it.  Both results
    equal their isolated runs (MSM against the oracle), the pending event is taken by exactly one
    MSM, and clearing it (NULL) leaves the next MSM without one."""
    import torch
    n, nn = (1 << 12) + 3, 1 << 14
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0B41, montgomery=True)
    b = torch.zeros((n, 24), dtype=torch.int64, device="cuda")
    amd.gen_bases("g2", b, 0x5EED0B42)
    x = torch.zeros((nn, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(x, 0x5EED0B43, montgomery=True)
    amd.ntt_init_domain()
    torch.cuda.synchronize()
    ref_ntt = amd.to_numpy_u64(amd.ntt(x, out=torch.zeros_like(x)))
    ref = H.g2_from_affine_mont(H.oracle_msm("g2", _std_scalars(0x5EED0B41, n), amd.to_numpy_u64(b),
                                             threads=ORACLE_THREADS))
    s_a, s_b = torch.cuda.Stream(priority=-1), torch.cuda.Stream()
    ev = amd.HipEvent()
    for rep in range(3):
        out = torch.zeros((1, 36), dtype=torch.int64, device="cuda")
        y = torch.zeros_like(x)
        amd.msm_accumulate_event(s_a, ev.handle)
        amd.msm("g2", s, b, scalars_mont=True, out=out, stream=s_a, is_async=True, n=n)
        ev.wait(s_b)
        amd.ntt(x, out=y, stream=s_b, is_async=True)
        torch.cuda.synchronize()
        assert gh.decode_icicle("g2", amd.to_numpy_u64(out)[0]) == ref, rep
        assert np.array_equal(amd.to_numpy_u64(y), ref_ntt), rep
    amd.msm_accumulate_event(s_a, ev.handle)
    amd.msm_accumulate_event(s_a, None)  # cleared: the next MSM records nothing
    r = amd.msm("g2", s, b, scalars_mont=True, stream=s_a, n=n)
    assert gh.decode_icicle("g2", r[0]) == ref


def test_msm_accumulate_event_taken_by_every_msm(amd, gh):
    """the pending event is taken by the next MSM call on the stream whatever its
    shape -- an empty MSM records it where it stops, a batch after its LAST member's accumulation --
    and a later single MSM finds nothing pending.  Observed with hipEventQuery right after the
    enqueue, behind a ~2 ms NTT batch on the same stream: a recorded event is still pending then,
    an unrecorded (or already completed) one reads complete."""
    import torch
    n, nn, nb = 1 << 12, 1 << 22, 4
    s = torch.zeros((2 * n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0B51, montgomery=True)
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0B52)
    x = torch.zeros((nb * nn, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(x, 0x5EED0B53, montgomery=True)
    y = torch.zeros_like(x)
    amd.ntt_init_domain()
    torch.cuda.synchronize()
    s_a = torch.cuda.Stream()

    def busy():  # a few ms of NTT work queued ahead on s_a
        amd.ntt(x, out=y, stream=s_a, is_async=True, batch=nb)

    single = amd.msm("g1", s[:n], b, scalars_mont=True, n=n)
    out = torch.zeros((2, 18), dtype=torch.int64, device="cuda")

    def call(shape):
        if shape == "empty":
            amd.msm("g1", s[:0], b[:0], scalars_mont=True, out=out[:1], stream=s_a, is_async=True, n=0)
        else:
            amd.msm("g1", s, b, scalars_mont=True, out=out, stream=s_a, is_async=True, n=n, batch=2)

    for shape in ("empty", "batch"):  # warm the stream's scratch: no allocation (and its sync) below
        busy()
        call(shape)
    torch.cuda.synchronize()
    for shape in ("empty", "batch"):
        ev = amd.HipEvent()
        torch.cuda.synchronize()
        amd.msm_accumulate_event(s_a, ev.handle)
        busy()
        call(shape)
        assert not ev.query(), f"{shape}: the MSM did not record the pending event"
        torch.cuda.synchronize()
        assert ev.query()
        if shape == "batch":
            assert np.array_equal(amd.to_numpy_u64(out)[0], single[0])
        # nothing pending now: a single MSM behind busy work does not record the event again
        busy()
        r = amd.msm("g1", s[:n], b, scalars_mont=True, out=torch.zeros((1, 18), dtype=torch.int64, device="cuda"),
                    stream=s_a, is_async=True, n=n)
        assert ev.query(), f"{shape}: the event stayed pending for a later MSM"
        torch.cuda.synchronize()
        assert np.array_equal(amd.to_numpy_u64(r), single)
        del ev  # __del__ drops any registration before destroying the event
