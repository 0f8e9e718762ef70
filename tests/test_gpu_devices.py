"""Per-device state and the multi-GPU exchange paths on hardware (SURVEY.md 8b "Threading",
8e), through the C ABI, against the oracle:

* the NTT domain is per device (ntt.hip current_domain): init / release / get_rou act on the
  current device; a device without a domain builds its own tables on first use;
* a world-size-1 "nccl" (RCCL) process group runs bench.py's sharded step with the RCCL
  all_gather_into_tensor branch of sharded_msm.gather_partials (one GPU is enough for that);
* >= 2 visible GPUs (skipped on the one-GPU box, ready for the 8-GPU node): NTT replicas on two
  devices and mbls_g1_msm_multi_device over distinct devices (peer copies, cross-device events);
* the scratch lease and the multi-device resources under stream reuse: a released busy stream
  followed by a call on the default stream, and two async multi-device calls on two streams."""
import ctypes
import os
import subprocess
import sys

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


def _ndev():
    import torch
    return torch.cuda.device_count()


def _std_scalars(seed, n):
    s = np.zeros((n, 4), dtype=np.uint64)
    H.oracle().orc_gen_scalars(H.ptr(s), seed, n)
    return s


def _rou(amd, logn):
    r = np.zeros(4, dtype=np.uint64)
    code = amd.lib().bls12_381_ntt_get_rou_from_domain(logn, amd._p(r))
    return code, r


def test_ntt_domain_release_and_lazy_rebuild(amd):
    """release drops this device's domain (get_rou then fails), a transform rebuilds canonical
    tables on first use, init_domain with a 2^12 root bounds the sizes of this device only"""
    import torch
    amd.ntt_init_domain()
    code, w20 = _rou(amd, 20)
    assert code == amd.SUCCESS
    assert H.pyref.fr_from_mont(H.pyref.limbs_to_int([int(v) for v in w20])) == H.pyref.omega(20)
    assert amd.lib().bls12_381_ntt_release_domain_cuda() == amd.SUCCESS
    assert _rou(amd, 20)[0] == 11  # INVALID_ARGUMENT: no domain on this device
    n = 1 << 14
    x = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(x, 0x5EED0D01, montgomery=True)
    y = amd.ntt(x, out=torch.zeros_like(x))  # lazily rebuilt tables
    torch.cuda.synchronize()
    assert np.array_equal(amd.to_numpy_u64(y), H.oracle_ntt(amd.to_numpy_u64(x), 14, False))
    # a root of order 2^12 (Montgomery): sizes above 2^12 are refused on this device
    w12 = np.array(H.pyref.int_to_limbs(H.pyref.fr_to_mont(H.pyref.omega(12)), 4), dtype=np.uint64)
    amd.ntt_init_domain(w12)
    with pytest.raises(amd.IcicleError):
        amd.ntt(x, out=torch.zeros_like(x))
    x12 = x[: 1 << 12]
    y12 = amd.ntt(x12, out=torch.zeros_like(x12))
    torch.cuda.synchronize()
    assert np.array_equal(amd.to_numpy_u64(y12), H.oracle_ntt(amd.to_numpy_u64(x12), 12, False))
    amd.ntt_init_domain()  # restore the full domain for the other tests


def test_release_busy_stream_then_default_stream(amd, gh):
    """a stream released while its MSM is still queued, then an MSM on the default
    stream (the same handle value the old 'released' marker used): the second call must wait for
    the first's scratch -- both results equal the oracle"""
    import torch
    n = (1 << 16) + 3
    s = torch.zeros((2, n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s[0], 0x5EED0D11, montgomery=True)
    amd.gen_scalars(s[1], 0x5EED0D12, montgomery=True)
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0D13)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    out0 = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
    out1 = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
    amd.msm("g1", s[0], b, icicle=True, scalars_mont=True, out=out0, stream=side, is_async=True)
    amd.release_stream(side)  # still busy
    amd.msm("g1", s[1], b, icicle=True, scalars_mont=True, out=out1, stream=None, is_async=True)
    torch.cuda.synchronize()
    bn = amd.to_numpy_u64(b)
    for k, out in enumerate((out0, out1)):
        ref = H.g1_from_affine_mont(H.oracle_msm("g1", _std_scalars(0x5EED0D11 + k, n), bn, threads=ORACLE_THREADS))
        assert gh.decode_icicle("g1", amd.to_numpy_u64(out)[0]) == ref, k


def test_multi_device_async_two_streams(amd, gh):
    """two async multi-device calls on two different caller streams, results on the
    device: the second call's shards must not overwrite the partial / gather slots the first is
    still reading (msm_multi_device orders itself behind the previous call's `done`)"""
    import torch
    n = (1 << 17) + 11
    ndev = 3
    s = torch.zeros((2, n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s[0], 0x5EED0D21, montgomery=True)
    amd.gen_scalars(s[1], 0x5EED0D22, montgomery=True)
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0D23)
    torch.cuda.synchronize()
    shards = [b[n * k // ndev:n * (k + 1) // ndev].clone() for k in range(ndev)]
    torch.cuda.synchronize()
    st = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.zeros((1, 18), dtype=torch.int64, device="cuda") for _ in range(2)]
    for rep in range(3):
        for k in range(2):
            amd.msm_multi_device("g1", s[k], shards, [0] * ndev, n, out=outs[k], stream=st[k], is_async=True)
        torch.cuda.synchronize()
        bn = amd.to_numpy_u64(b)
        for k in range(2):
            ref = H.g1_from_affine_mont(H.oracle_msm("g1", _std_scalars(0x5EED0D21 + k, n), bn,
                                                     threads=ORACLE_THREADS))
            assert gh.decode_icicle("g1", amd.to_numpy_u64(outs[k])[0]) == ref, (rep, k)


NCCL_SCRIPT = r"""
import os, sys, json
sys.path.insert(0, os.path.join(os.environ["MBLS_ROOT"], "midnight-bls12-381-cuda_amd"))
import torch, torch.distributed as dist
import bls12_381_amd as amd, sharded_msm
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
n = int(sys.argv[1])
stream = torch.cuda.current_stream(dev)
s = torch.zeros((n, 4), dtype=torch.int64, device=dev)
b = torch.zeros((n, 12), dtype=torch.int64, device=dev)
amd.gen_scalars(s, 0x5EED0D31, montgomery=True, stream=stream)
amd.gen_bases("g1", b, 0x5EED0D32, stream=stream)
partial = torch.zeros((1, 18), dtype=torch.int64, device=dev)
gathered = torch.zeros((1, 18), dtype=torch.int64, device=dev)
result = torch.zeros((1, 18), dtype=torch.int64, device=dev)
# bench.py sharded_step's N > 1 sequence; with a live process group gather_partials takes the
# RCCL all_gather_into_tensor branch even for one rank
amd.msm("g1", s, b, icicle="jacobian", scalars_mont=True, out=partial, stream=stream, is_async=True)
g = sharded_msm.gather_partials(partial, dist.get_world_size(), dist, out=gathered)
assert g.data_ptr() == gathered.data_ptr()
amd.sum_jacobian("g1", gathered, result, stream=stream)
amd.jacobian_to_icicle("g1", result, stream=stream)
torch.cuda.synchronize(dev)
print(json.dumps({"result": [int(v) for v in result.cpu().numpy().view("uint64")[0]],
                  "partial_equal": bool(torch.equal(gathered[0], partial[0]))}))
dist.destroy_process_group()
"""


def test_rccl_world1_gather_branch(amd, gh, tmp_path):
    """bench.py's N > 1 sharded step (Jacobian partial -> RCCL all_gather_into_tensor -> EC sum
    -> one normalisation) through a real "nccl" process group of one rank on the GPU, against the
    oracle"""
    n = (1 << 16) + 7
    script = tmp_path / "nccl_world1.py"
    script.write_text(NCCL_SCRIPT)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29531", RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", MBLS_ROOT=H.ROOT)
    out = subprocess.run([sys.executable, str(script), str(n)], env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-3000:]
    import json
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["partial_equal"]
    b = np.zeros((n, 12), dtype=np.uint64)
    H.oracle().orc_gen_g1_bases(H.ptr(b), 0x5EED0D32, n, ORACLE_THREADS)
    ref = H.g1_from_affine_mont(H.oracle_msm("g1", _std_scalars(0x5EED0D31, n), b, threads=ORACLE_THREADS))
    assert gh.decode_icicle("g1", np.array(rec["result"], dtype=np.uint64)) == ref


@pytest.mark.skipif("_ndev() < 2")
def test_ntt_replicas_on_two_devices(amd):
    """NTT replicas: the domain initialised on device 0 only; device 1 builds its
    own tables on first use -- both transforms equal the oracle"""
    import torch
    n = 1 << 18
    amd.ntt_init_domain()
    xs, ys = [], []
    for d in (0, 1):
        with torch.cuda.device(d):
            x = torch.zeros((n, 4), dtype=torch.int64, device=f"cuda:{d}")
            amd.gen_scalars(x, 0x5EED0D41 + d, montgomery=True)
            y = amd.ntt(x, out=torch.zeros_like(x))
            xs.append(x)
            ys.append(y)
    for d in (0, 1):
        torch.cuda.synchronize(d)
        ref = H.oracle_ntt(amd.to_numpy_u64(xs[d]), 18, False, threads=ORACLE_THREADS)
        assert np.array_equal(amd.to_numpy_u64(ys[d]), ref), d


@pytest.mark.skipif("_ndev() < 2")
@pytest.mark.parametrize("group", ["g1", "g2"])
@pytest.mark.parametrize("scalars_on", ["device", "host", "pinned"])
def test_msm_multi_device_distinct_devices(amd, gh, group, scalars_on):
    """mbls_g*_msm_multi_device over devices [0, 1, ...]: scalars on device 0 (staged to the other
    shards by peer copies, peer access enabled by the library), on the host, or in page-locked
    host memory (read in place only by the device whose alias it is; staged elsewhere), each
    shard's bases on its own device, partials peer-copied to device 0 -- equal to the oracle"""
    import torch
    ndev = min(_ndev(), 8)
    n = (1 << 18) + 13 if group == "g1" else (1 << 15) + 13
    w = 12 if group == "g1" else 24
    dec = H.g1_from_affine_mont if group == "g1" else H.g2_from_affine_mont
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda:0")
    amd.gen_scalars(s, 0x5EED0D51, montgomery=True)
    b0 = torch.zeros((n, w), dtype=torch.int64, device="cuda:0")
    amd.gen_bases(group, b0, 0x5EED0D52)
    torch.cuda.synchronize(0)
    shards = []
    for k in range(ndev):
        lo, hi = n * k // ndev, n * (k + 1) // ndev
        shards.append(b0[lo:hi].to(f"cuda:{k}"))
    for k in range(ndev):
        torch.cuda.synchronize(k)
    if scalars_on == "device":
        sc = s
    elif scalars_on == "host":
        sc = np.ascontiguousarray(amd.to_numpy_u64(s))
    else:
        sc = s.cpu().pin_memory()
    r = amd.msm_multi_device(group, sc, shards, list(range(ndev)), n)
    ref = dec(H.oracle_msm(group, _std_scalars(0x5EED0D51, n), amd.to_numpy_u64(b0), threads=ORACLE_THREADS))
    assert gh.decode_icicle(group, r[0]) == ref


@pytest.mark.parametrize("offset", [0, 3])
def test_msm_pinned_host_operands(amd, gh, offset):
    """host operands in page-locked memory are staged by the PCIe copy kernel (stage_to_device):
    pinned scalars and pinned bases, also at an offset into the pinned allocation, equal to the
    device-operand MSM and to the oracle"""
    import torch
    n = (1 << 15) + 9
    s = torch.zeros((n + offset, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0D61, montgomery=True)
    b = torch.zeros((n + offset, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0D62)
    torch.cuda.synchronize()
    s_pin = s.cpu().pin_memory()[offset:]
    b_pin = b.cpu().pin_memory()[offset:]
    dev_out = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
    amd.msm("g1", s[offset:], b[offset:], icicle=True, scalars_mont=True, out=dev_out)
    r1 = amd.msm("g1", s_pin, b[offset:], icicle=True, scalars_mont=True)
    r2 = amd.msm("g1", s_pin, b_pin, icicle=True, scalars_mont=True)
    torch.cuda.synchronize()
    ref_dev = amd.to_numpy_u64(dev_out)[0]
    assert np.array_equal(np.asarray(r1)[0], ref_dev) and np.array_equal(np.asarray(r2)[0], ref_dev)
    full = _std_scalars(0x5EED0D61, n + offset)[offset:]
    ref = H.g1_from_affine_mont(H.oracle_msm("g1", np.ascontiguousarray(full), amd.to_numpy_u64(b)[offset:].copy(),
                                             threads=ORACLE_THREADS))
    assert gh.decode_icicle("g1", ref_dev) == ref
    # the reference's raw entry (standard scalars, Jacobian result) with pinned standard scalars:
    # read in place by the GLV split; standard scalars with bitsize 128 (no split: the digit pass
    # reads them once per window) are staged instead
    s_std = torch.from_numpy(np.ascontiguousarray(full).view(np.int64)).pin_memory()
    r3 = amd.msm("g1", s_std, b[offset:], icicle=False)
    assert gh.decode_jacobian_mont("g1", np.asarray(r3)[0]) == ref
    small = np.ascontiguousarray(full.copy())
    small[:, 2:] = 0  # < 2^128
    ref_small = H.g1_from_affine_mont(H.oracle_msm("g1", small, amd.to_numpy_u64(b)[offset:].copy(),
                                                   threads=ORACLE_THREADS))
    r4 = amd.msm("g1", torch.from_numpy(small.view(np.int64)).pin_memory(), b[offset:], icicle=False, bitsize=128)
    assert gh.decode_jacobian_mont("g1", np.asarray(r4)[0]) == ref_small


def test_g2_msm_pinned_host_scalars(amd, gh):
    """G2 (psi split) with pinned Montgomery scalars read in place, equal to the oracle"""
    import torch
    n = (1 << 12) + 5
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0D71, montgomery=True)
    b = torch.zeros((n, 24), dtype=torch.int64, device="cuda")
    amd.gen_bases("g2", b, 0x5EED0D72)
    torch.cuda.synchronize()
    r = amd.msm("g2", s.cpu().pin_memory(), b, icicle=True, scalars_mont=True)
    ref = H.g2_from_affine_mont(H.oracle_msm("g2", _std_scalars(0x5EED0D71, n), amd.to_numpy_u64(b),
                                             threads=ORACLE_THREADS))
    assert gh.decode_icicle("g2", np.asarray(r)[0]) == ref
