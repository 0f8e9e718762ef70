"""world_size-2 gloo test of the sharded-MSM logic (CPU): each rank computes its contiguous
shard with the oracle, partials are all_gathered, the EC sum equals the unsharded MSM."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import helpers as H

sys.path.insert(0, os.path.join(H.ROOT, "midnight-bls12-381-cuda_amd"))
import sharded_msm  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = H.oracle()
    scal = np.zeros((n, 4), dtype=np.uint64)
    lib.orc_gen_scalars(H.ptr(scal), 0x5EED0004, n)
    bases = np.zeros((n, 12), dtype=np.uint64)
    lib.orc_gen_g1_bases(H.ptr(bases), 0x5EED0014, n, 1)
    lo, hi = sharded_msm.shard_range(n, world, rank)

    def msm_fn(s, b):
        aff = H.oracle_msm("g1", np.ascontiguousarray(s), np.ascontiguousarray(b), threads=1)
        return torch.from_numpy(aff.view(np.int64).copy()).reshape(1, -1)

    def sum_fn(g):
        acc = np.zeros(12, dtype=np.uint64)
        for row in g.numpy().view(np.uint64):
            out = np.zeros(12, dtype=np.uint64)
            lib.orc_g1_add_affine(H.ptr(out), H.ptr(acc), H.ptr(np.ascontiguousarray(row)))
            acc = out
        return acc

    total = sharded_msm.sharded_msm("g1", scal[lo:hi], bases[lo:hi], world, dist, msm_fn, sum_fn)
    if rank == 0:
        full = H.oracle_msm("g1", scal, bases, threads=1)
        q.put(bool(np.array_equal(total, full)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1000), (3, 257)])
def test_sharded_msm_gloo(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert ok


def test_shard_ranges_cover():
    for n in (1, 7, 1000, 1 << 20):
        for w in (1, 2, 3, 8):
            rs = [sharded_msm.shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))


def _gpu_worker(rank, world, port, log_total, q):
    """bench.py's sharded step on the HIP library: both ranks on cuda:0 (a 1-GPU box), the
    all-gather over gloo on host copies (RCCL needs one GPU per rank)"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import gpu_helpers
        amd = gpu_helpers.amd
        torch.cuda.set_device(0)
        n = 1 << log_total
        lo, hi = sharded_msm.shard_range(n, world, rank)
        s = torch.zeros((hi - lo, 4), dtype=torch.int64, device="cuda")
        amd.gen_scalars(s, 0x5EED0004, montgomery=True, start=lo)
        b = torch.zeros((hi - lo, 12), dtype=torch.int64, device="cuda")
        amd.gen_bases("g1", b, 0x5EED0013, start=lo)
        part = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
        amd.msm("g1", s, b, icicle="jacobian", scalars_mont=True, out=part, n=hi - lo)
        torch.cuda.synchronize()
        gathered = sharded_msm.gather_partials(part.cpu(), world, dist).cuda()
        tot = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
        amd.sum_jacobian("g1", gathered, tot)
        amd.jacobian_to_icicle("g1", tot)
        torch.cuda.synchronize()
        got = gpu_helpers.decode_icicle("g1", amd.to_numpy_u64(tot)[0])
        if rank == 0:
            lib = H.oracle()
            scal = np.zeros((n, 4), dtype=np.uint64)
            lib.orc_gen_scalars(H.ptr(scal), 0x5EED0004, n)
            bases = np.zeros((n, 12), dtype=np.uint64)
            lib.orc_gen_g1_bases(H.ptr(bases), 0x5EED0013, n, 16)
            ref = H.g1_from_affine_mont(H.oracle_msm("g1", scal, bases, threads=16))
            q.put(got == ref)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent on q.get
        q.put(repr(e))
        raise


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_msm_hip_world(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, 18, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
    assert ok is True, ok
