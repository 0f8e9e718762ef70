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
# HBM bytes per launch from the committed rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
# (tools/gpu_pmc.sh on tools/pmc_probe.py's fixed workload; gfx950 FETCH_SIZE x2 correction)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r01", "pmc_summary.json")


def pmc_traffic(kernel, n_launches_per_unit=1):
    try:
        with open(PMC_SUMMARY) as f:
            k = json.load(f)["kernels"].get(kernel)
        return None if not k or k.get("hbm_bytes_per_launch") is None else k["hbm_bytes_per_launch"] * n_launches_per_unit
    except (OSError, ValueError, KeyError):
        return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--msm-log", type=int, default=20)
    ap.add_argument("--ntt-log", type=int, default=22)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-mix", action="store_true", help="skip the G2 MSM + batched NTT overlap leg (config #5)")
    ap.add_argument("--mix-batch", type=int, default=4, help="NTT polynomials in the config #5 batch")
    ap.add_argument("--msm-batch", type=int, default=8, help="members of the batched-MSM leg (0: skip)")
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

    # batched MSMs (ICICLE batch_size, shared device bases, device results): members pipelined
    # on two streams so each member's latency-bound reduction overlaps the next accumulation
    batch_leg = None
    if args.msm_batch > 1:
        B = args.msm_batch
        sb = torch.zeros((B * n, 4), dtype=torch.int64, device=dev)
        amd.gen_scalars(sb, 0x5EED0033 + rank, montgomery=True, stream=stream)
        rb = torch.zeros((B, 18), dtype=torch.int64, device=dev)

        def batch_step():
            amd.msm("g1", sb, bases, icicle=True, scalars_mont=True, batch=B, out=rb, stream=stream,
                    is_async=True, n=n)

        batch_step()
        barrier_sync()
        reps = max(2, args.steps // 4)
        t0 = time.perf_counter()
        for _ in range(reps):
            batch_step()
        barrier_sync()
        bdt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(bdt, op=dist.ReduceOp.MAX)
        batch_leg = {"batch": B, "reps": reps, "ms_per_batch": round(float(bdt.item()) / reps * 1e3, 3),
                     "msm_per_sec": round(world * B * reps / float(bdt.item()), 3),
                     "note": "ICICLE batch_size (core/msm.rs msm_batch_with_device_bases), members pipelined on two HIP streams"}
        del sb

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

    # NTT 2^20 forward + inverse round trip (BASELINE config #2), device-resident
    x20 = x[: 1 << 20]
    y20 = torch.zeros_like(x20)
    z20 = torch.zeros_like(x20)
    reps = max(3, args.steps)
    for _ in range(2):
        amd.ntt(x20, out=y20, stream=stream, is_async=True)
        amd.ntt(y20, inverse=True, out=z20, stream=stream, is_async=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        amd.ntt(x20, out=y20, stream=stream, is_async=True)
        amd.ntt(y20, inverse=True, out=z20, stream=stream, is_async=True)
    torch.cuda.synchronize(dev)
    ntt20_rt_ms = (time.perf_counter() - t0) / reps * 1e3
    ntt20_exact = bool(torch.equal(z20, x20))
    del y20, z20

    # ------------------------------------------------------------------ config #5 mix (replicas)
    mix = None
    if not args.no_mix:
        mix = mix_leg(args, amd, torch, dev, rank)

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
                         "traffic": pmc_traffic("k_accumulate"),
                         "traffic_source": "profiles/r01/pmc_summary.json (bytes per launch)",
                         "note": "VALU-bound (v_mad_u64_u32); HBM fraction reported as the contract asks"},
            "msm_batch": batch_leg,
            "ntt20_roundtrip_ms": round(ntt20_rt_ms, 4),
            "ntt20_roundtrip_exact": ntt20_exact,
            "mix_g2msm_batched_ntt": mix,
            "roofline_ntt": {"kernel": "k_ntt_pass x passes (one transform)", "bound": "hbm",
                             "achieved": round(ntt_ach, 2) if ntt_ach else None, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(ntt_ach / HBM_PEAK_GBS, 5) if ntt_ach else None,
                             "traffic": ntt_traffic(args.ntt_log),
                             "traffic_source": "profiles/r01/pmc_summary.json (first + middle + last pass)",
                             "pass_ms": round(ntt_pass_ms, 4) if ntt_pass_ms else None},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def ntt_traffic(log_n):
    """HBM bytes of one forward 2^22 transform: first + middle + last pass (pmc_probe sizes)"""
    if log_n != 22:
        return None
    parts = [pmc_traffic(k) for k in ("k_ntt_pass<true, false, false>", "k_ntt_pass<false, false, false>",
                                      "k_ntt_pass<false, true, false>")]
    return None if any(p is None for p in parts) else sum(parts)


def mix_leg(args, amd, torch, dev, rank):
    """BASELINE config #5: G2 MSM 2^msm_log and a batch of Fr NTTs 2^ntt_log enqueued on two
    HIP streams at once (PLONK-prover-shaped mix); reports each alone and the overlapped wall."""
    n = 1 << args.msm_log
    nn = 1 << args.ntt_log
    B = args.mix_batch
    s_a = torch.cuda.Stream(dev)
    s_b = torch.cuda.Stream(dev)
    sc = torch.zeros((n, 4), dtype=torch.int64, device=dev)
    bs = torch.zeros((n, 24), dtype=torch.int64, device=dev)
    amd.gen_scalars(sc, 0x5EED0005 + rank, montgomery=True, stream=s_a)
    amd.gen_bases("g2", bs, 0x5EED0015 + rank, stream=s_a)
    res = torch.zeros((1, 36), dtype=torch.int64, device=dev)
    xb = torch.zeros((B * nn, 4), dtype=torch.int64, device=dev)
    yb = torch.zeros_like(xb)
    amd.gen_scalars(xb, 0x5EED0025 + rank, montgomery=True, stream=s_b)
    torch.cuda.synchronize(dev)

    def g2():
        amd.msm("g2", sc, bs, icicle=False, scalars_mont=True, out=res, stream=s_a, is_async=True, n=n)

    def ntts():
        amd.ntt(xb, out=yb, batch=B, stream=s_b, is_async=True)

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / reps * 1e3

    reps = max(2, min(args.steps, 5))
    g2_ms = timed(g2, reps)
    ntt_ms = timed(ntts, reps)
    both_ms = timed(lambda: (g2(), ntts()), reps)
    return {"g2_msm_points": n, "ntt_batch": B, "ntt_size": nn, "g2_msm_ms": round(g2_ms, 3),
            "g2_msm_per_sec": round(1e3 / g2_ms, 3), "batched_ntt_ms": round(ntt_ms, 3),
            "overlapped_ms": round(both_ms, 3), "sum_isolated_ms": round(g2_ms + ntt_ms, 3),
            "streams": 2}


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
