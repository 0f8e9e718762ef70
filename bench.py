#!/usr/bin/env python3
"""bench.py -- headline benchmark: G1 MSM/s at 2^20 points (+ Fr NTT/s at 2^22), MI355X.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1 launched by
torch.distributed.run, one rank per GPU.  Rank 0 prints ONE JSON line.

Step = one G1 MSM over N * 2^msm_log points, sharded contiguously: each rank runs Pippenger
on its 2^msm_log shard (bases device-resident, scalars Montgomery on device -- the
production path core/msm.rs:594-682), then the partial Jacobian sums are exchanged with one
RCCL all_gather over xGMI and EC-added on device (reference has no multi-GPU).
value = MSMs of 2^msm_log points (per-GPU shard size) completed per second over all GPUs
(weak scaling).  The Fr NTT 2^ntt_log (forward, natural order, best_fft semantics) is timed
in its own loop on every rank (replicas) and reported as `ntt_per_sec`.
Inputs are synthetic: seeded scalars and bases P_i = k_i G generated on the device.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "midnight-bls12-381-cuda_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
MSM_BYTES_PER_POINT = 128  # 32 B scalar + 96 B affine base
NTT_BYTES_PER_ELEM = 64    # one read + one write of 32 B per transform


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--msm-log", type=int, default=20)
    ap.add_argument("--ntt-log", type=int, default=22)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-threads", type=int, default=0)
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import bls12_381_amd as amd
    import sharded_msm

    world =int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    amd.lib()
    stream = torch.cuda.current_stream(dev)

    def barrier_sync():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    # ------------------------------------------------------------------ MSM inputs
    n = 1 << args.msm_log
    scalars = torch.zeros((n, 4), dtype=torch.int64, device=dev)
    bases = torch.zeros((n, 12), dtype=torch.int64, device=dev)
    amd.gen_scalars(scalars, 0x5EED0003 + rank, montgomery=True, stream=stream)
    amd.gen_bases("g1", bases, 0x5EED0013 + rank, stream=stream)
    partial = torch.zeros((1, 18), dtype=torch.int64, device=dev)
    gathered = torch.zeros((world, 18), dtype=torch.int64, device=dev)
    total = torch.zeros((1, 18), dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)

    def msm_step():
        # bls12_381_g1_msm_cuda semantics (reference icicle_curve_api.cu:679): result is a
        # Jacobian Montgomery point left on the device, no host round trip
        amd.msm("g1", scalars, bases, icicle=False, scalars_mont=True, out=partial, stream=stream,
                is_async=True, n=n)
        if world > 1:
            sharded_msm.gather_partials(partial, world, dist, out=gathered)
            amd.sum_jacobian("g1", gathered, total, stream=stream)

    for _ in range(args.warmup):
        msm_step()
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        msm_step()
    barrier_sync()
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    msm_time = float(dt_t.item())
    ms_per_step = msm_time / args.steps * 1e3
    msm_per_sec = world * args.steps / msm_time

    # live per-stage timing (HIP events on this stream) for the roofline
    amd.profile(True)
    for _ in range(max(2, args.steps // 2)):
        msm_step()
    torch.cuda.synchronize(dev)
    msm_prof = amd.profile_read()
    amd.profile(False)

    # ------------------------------------------------------------------ NTT (replicas)
    amd.ntt_init_domain()
    nn = 1 << args.ntt_log
    x = torch.zeros((nn, 4), dtype=torch.int64, device=dev)
    y = torch.zeros_like(x)
    amd.gen_scalars(x, 0x5EED0025 + rank, montgomery=True, stream=stream)
    for _ in range(args.warmup):
        amd.ntt(x, out=y, stream=stream, is_async=True)
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        amd.ntt(x, out=y, stream=stream, is_async=True)
    barrier_sync()
    ndt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ndt, op=dist.ReduceOp.MAX)
    ntt_per_sec = world * args.steps / float(ndt.item())
    amd.profile(True)
    for _ in range(max(2, args.steps // 2)):
        amd.ntt(x, out=y, stream=stream, is_async=True)
    torch.cuda.synchronize(dev)
    ntt_prof = amd.profile_read()
    amd.profile(False)

    # ------------------------------------------------------------------ CPU baseline (rank 0, N=1)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args, amd, scalars, bases, n)

    if rank == 0:
        def avg(prof, key):
            ms, cnt = prof.get(key, (0.0, 0))
            return ms / cnt if cnt else None

        acc_ms = avg(msm_prof, "msm.accumulate")
        msm_total_ms = avg(msm_prof, "msm.total")
        ntt_ms = avg(ntt_prof, "ntt.transform")
        ntt_pass_ms = avg(ntt_prof, "ntt.pass")
        stages = {k: round(v[0] / v[1], 4) for k, v in sorted(msm_prof.items()) if v[1]}
        msm_ach = MSM_BYTES_PER_POINT * n / (acc_ms * 1e-3) / 1e9 if acc_ms else None
        ntt_ach = NTT_BYTES_PER_ELEM * nn / (ntt_ms * 1e-3) / 1e9 if ntt_ms else None
        out = {
            "metric": "G1 MSM/sec at 2^20 points + Fr NTT/sec at 2^22 (bit-exact vs BLST)",
            "value": round(msm_per_sec, 3),
            "unit": "MSM/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32-limb Montgomery (Fq 381-bit / Fr 255-bit integer)",
            "data": "synthetic: seeded scalars, bases k_i*G generated on device",
            "config": {"workload": f"G1 MSM 2^{args.msm_log} points per GPU (sharded, RCCL all-gather of "
                                   f"partial sums) + Fr NTT 2^{args.ntt_log}",
                       "msm_points_per_gpu": n, "ntt_size": nn, "parallelism": f"msm-shard{world}"},
            "ntt_per_sec": round(ntt_per_sec, 3),
            "ntt_ms": round(ntt_ms, 4) if ntt_ms else None,
            "msm_stage_ms": stages,
            "roofline": {"kernel": "k_accumulate<G1> (MSM bucket accumulation, dominant)",
                         "bound": "hbm", "achieved": round(msm_ach, 2) if msm_ach else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(msm_ach / HBM_PEAK_GBS, 5) if msm_ach else None,
                         "traffic": None,
                         "note": "VALU-bound (v_mad_u64_u32); HBM fraction reported as the contract asks"},
            "roofline_ntt": {"kernel": "k_ntt_pass x passes (one transform)", "bound": "hbm",
                             "achieved": round(ntt_ach, 2) if ntt_ach else None, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(ntt_ach / HBM_PEAK_GBS, 5) if ntt_ach else None,
                             "traffic": None, "pass_ms": round(ntt_pass_ms, 4) if ntt_pass_ms else None},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(args, amd, scalars, bases, n):
    """The oracle (C port of the reference CPU semantics, multithreaded Pippenger) on the
    host cores, on the same 2^msm_log inputs copied back from the device."""
    import ctypes
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import helpers as H
    o = H.oracle()
    threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    s_mont = np.ascontiguousarray(amd.to_numpy_u64(scalars))
    b = np.ascontiguousarray(amd.to_numpy_u64(bases))
    # Montgomery -> standard (mont_mul by 1) on the CPU, untimed: the oracle extracts bits
    s_std = np.zeros((n, 4), dtype=np.uint64)
    one = np.zeros((n, 4), dtype=np.uint64)
    one[:, 0] = 1
    o.orc_vec_mul(H.ptr(s_std), H.ptr(s_mont), H.ptr(one), n)
    t0 = time.perf_counter()
    H.oracle_msm("g1", s_std, b, threads=threads)
    t = time.perf_counter() - t0
    return {"value": round(1.0 / t, 4), "unit": "MSM/s", "cores": threads, "kind": "port",
            "sample": f"one full G1 MSM of 2^{args.msm_log} points (same inputs), oracle/bls12_381_oracle.c "
                      f"multithreaded Pippenger, {threads} threads; BLST not available"}


if __name__ == "__main__":
    main()
