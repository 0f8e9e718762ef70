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
