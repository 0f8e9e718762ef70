"""Multi-GPU MSM sharding: one process per GPU, torch.distributed.

An MSM of N points is partitioned into contiguous shards, one per rank; each rank runs the
full Pippenger on its shard (bases stay resident on its GPU) and produces ONE partial sum
(Jacobian, Montgomery, 144 B for G1).  The partial sums are exchanged with a single
all_gather (RCCL over xGMI with the "nccl" backend; gloo in the CPU tests) and added on the
device.  RCCL reduce ops cannot add curve points, so this is all-gather + EC reduction, not
all_reduce(sum).  The reference has no multi-GPU path (core/config.rs:524-531)."""
from __future__ import annotations


def shard_range(n_total: int, world: int, rank: int):
    """[lo, hi) of rank's contiguous shard (sizes differ by at most one)."""
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def gather_partials(partial, world, dist, out=None):
    """all_gather one partial point per rank -> tensor [world, limbs] (same device)."""
    import torch
    if world == 1 and not (dist is not None and dist.is_available() and dist.is_initialized()):
        return partial.reshape(1, -1)  # no process group: nothing to exchange
    if out is None:
        out = torch.empty((world, partial.numel()), dtype=partial.dtype, device=partial.device)
    if partial.is_cuda and dist.get_backend() != "nccl":
        # gloo (CPU tests, one-GPU rehearsals): stage through host memory
        host = torch.empty((world, partial.numel()), dtype=partial.dtype)
        dist.all_gather_into_tensor(host, partial.reshape(1, -1).cpu())
        out.copy_(host)
        return out
    dist.all_gather_into_tensor(out, partial.reshape(1, -1).contiguous())
    return out


def sharded_msm(group, scalars_shard, bases_shard, world, dist, msm_fn, sum_fn, stream=None):
    """Run the local MSM with `msm_fn(scalars, bases) -> partial (1, limbs) tensor`, gather
    the partials and reduce with `sum_fn(gathered) -> (1, limbs) tensor`."""
    partial = msm_fn(scalars_shard, bases_shard)
    gathered = gather_partials(partial, world, dist)
    return sum_fn(gathered)
