#!/usr/bin/env python3
"""bench.py -- headline benchmark: G1 MSM/s at 2^20 points (+ Fr NTT/s at 2^22), MI355X.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1 launched by
torch.distributed.run, one rank per GPU.  Rank 0 prints ONE JSON line.

Headline (`value`, BASELINE config #3): one step = one G1 MSM of 2^msm_log points per rank on
the PRODUCTION path core/msm.rs:594-682 uses -- scalars in Montgomery form and bases resident
in HBM, the ICICLE entry (bls12_381_icicle_g1_msm: Montgomery flags honoured, ICICLE (x, y, 1)
standard-form result left on the device).  At N > 1 every rank runs its 2^msm_log shard of one
global input stream (mbls_g1_msm_jacobian), the Jacobian partials are exchanged with ONE RCCL
all_gather over xGMI, added on the device and normalised once (the reference has
no multi-GPU path).  value = MSMs of 2^msm_log points completed per second over all GPUs
(weak scaling), from the median of the K per-step hipEvent times (the max
over ranks), with mean / min / max and the wall-clock rate of the same K steps in `msm_step_ms`.  The other BASELINE configs are legs of the same run (see `configs` below):
#1 vecops (GPU and the CPU path), #2 NTT 2^20 round trip, #4 the 2^24 MSM split over the N
ranks (strong scaling, digest comparable across N), #5 G2 MSM 2^20 + 4 x NTT 2^22 on two
streams.  Inputs are synthetic: seeded scalars and bases P_i = k_i G generated on the device.
"""
import argparse
import hashlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "midnight-bls12-381-cuda_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
MSM_BYTES_PER_POINT = 128  # 32 B scalar + 96 B affine base
G2_BYTES_PER_POINT = 224   # 32 B scalar + 192 B affine base
NTT_BYTES_PER_ELEM = 64    # one read + one write of 32 B per transform
VEC_BYTES_PER_ELEM = 96    # read a, b; write out
PROFILES = os.path.join(ROOT, "profiles")


def pmc_summary():
    for rnd in ("r06/closing", "r05/closing", "r04/closing", "r03", "r02", "r01"):
        path = os.path.join(PROFILES, rnd, "pmc_summary.json")
        try:
            with open(path) as f:
                return json.load(f), os.path.relpath(path, ROOT)
        except (OSError, ValueError):
            continue
    return {}, None


def _pmc_kernel(kernel):
    """per-launch counters of `kernel` (round-2 summaries keyed G1's accumulation "k_accumulate")"""
    ks = pmc_summary()[0].get("kernels", {})
    if kernel not in ks and kernel == "k_accumulate<G1>":
        kernel = "k_accumulate"
    return ks.get(kernel)


def pmc_traffic(kernel):
    k = _pmc_kernel(kernel)
    return None if not k or k.get("hbm_bytes_per_launch") is None else k["hbm_bytes_per_launch"]


def pmc_counter(kernel, counter):
    return (_pmc_kernel(kernel) or {}).get(counter)


# VALU issue model, MEASURED (tools/valu_ceiling.hip, profiles/r05/valu_ceiling.json): on gfx950 a
# wave64 VALU instruction issues over ~4 SIMD cycles whether it is v_mad_u64_u32 (4.4 at the
# throttled 2.16 GHz a pure-mad loop runs at) or v_add_co / v_addc_co (4.1); the round-1..4 model
# (8 cycles per INT64 instruction, 2 otherwise, 2.4 GHz) was wrong on both and is gone.
SIMDS = 1024


def valu_issue_bound_ms(kernel, cyc_per_instr, mhz):
    """a kernel's VALU issue time from its committed instruction count (all VALU at the measured
    cycles per wave-instruction, all SIMDs busy, the measured clock)"""
    v = pmc_counter(kernel, "SQ_INSTS_VALU")
    if v is None or not cyc_per_instr or not mhz:
        return None
    return v * cyc_per_instr / SIMDS / (mhz * 1e3)


CEILING_BIN = os.path.join(ROOT, "tools", "valu_ceiling")


_CEILING = []


def valu_ceiling():
    """the measured ceilings, run once per bench process (main and the mix leg share them)"""
    if not _CEILING:
        _CEILING.append(_valu_ceiling())
    return _CEILING[0]


def _valu_ceiling():
    """Measured VALU ceilings (tools/valu_ceiling.hip): k_accumulate<G1>'s
    arithmetic (same madd / mmadd code, same 168-VGPR / 3-wave bounds, points from LDS) and
    k_ntt_pass's radix-4 body, register-resident.  Run live on this box as a child process when
    the binary is built (build() builds it), else the committed measurement."""
    import subprocess
    if os.path.exists(CEILING_BIN):
        try:
            out = subprocess.run([CEILING_BIN, "24"], capture_output=True, text=True, timeout=120)
            if out.returncode == 0:
                d = json.loads(out.stdout)
                d["source"] = "live: tools/valu_ceiling 24 on this box"
                return d
        except (OSError, ValueError, subprocess.TimeoutExpired):
            pass
    path = os.path.join(PROFILES, "r06", "valu_ceiling.json")
    if not os.path.exists(path):
        path = os.path.join(PROFILES, "r05", "valu_ceiling.json")
    try:
        with open(path) as f:
            d = json.load(f)
        d["source"] = f"committed: {os.path.relpath(path, ROOT)}"
        return d
    except (OSError, ValueError):
        return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--msm-log", type=int, default=20)
    ap.add_argument("--ntt-log", type=int, default=22)
    ap.add_argument("--msm-total-log", type=int, default=24,
                    help="config #4: one MSM of 2^k points split over the ranks (0: skip)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-budget-s", type=float, default=20.0, help="bound on the CPU MSM leg's repeats")
    ap.add_argument("--no-cpu-total", action="store_true", help="skip the CPU config #4 MSM (2^msm_total_log, once)")
    ap.add_argument("--no-mix", action="store_true", help="skip the G2 MSM + batched NTT overlap leg (config #5)")
    ap.add_argument("--mix-batch", type=int, default=4, help="NTT polynomials in the config #5 batch")
    ap.add_argument("--msm-batch", type=int, default=8, help="members of the batched-MSM leg (0: skip)")
    ap.add_argument("--headline-only", action="store_true", help="headline MSM + NTT loops only (profiling)")
    ap.add_argument("--no-stage-profile", action="store_true",
                    help="skip the stage-profiler passes (their hipEvent markers add ~10 us before each stage "
                         "in a kernel trace; use for timelines)")
    return ap.parse_args()


def digest(t):
    import numpy as np
    return hashlib.sha256(t.detach().cpu().numpy().view(np.uint64).tobytes()).hexdigest()[:16]


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`--gpus N` is authoritative.  Without a launcher (no WORLD_SIZE) and N > 1, start
    torch.distributed.run with N ranks as a CHILD process (never exec: nothing here has touched
    the GPU, and the child must not replace this process), let rank 0's JSON line through, and
    return the child's exit code.  Returns None when this process is a rank itself."""
    env_world = os.environ.get("WORLD_SIZE")
    same_dev = os.environ.get("MBLS_BENCH_SAME_DEVICE") == "1"
    if env_world is not None:
        if int(env_world) != args.gpus:
            sys.stderr.write(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} "
                             f"ranks; refusing to print a line for a run that was not asked for\n")
            return 2
        return None
    if args.gpus <= 1:
        return None
    import torch  # device_count() does not initialise the GPU on this image
    have = torch.cuda.device_count()
    if have < args.gpus and not same_dev:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {have}; "
                         f"(rehearsal on one GPU: MBLS_BENCH_SAME_DEVICE=1 MBLS_BENCH_BACKEND=gloo)\n")
        return 2
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ))


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    import torch
    import torch.distributed as dist
    import bls12_381_amd as amd
    import sharded_msm

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-rank path on a one-GPU box (never the driver's runs):
    # MBLS_BENCH_SAME_DEVICE=1 puts every rank on GPU 0, MBLS_BENCH_BACKEND=gloo replaces RCCL
    # (which refuses two ranks on one device); the digests must match the N = 1 run
    same_dev = os.environ.get("MBLS_BENCH_SAME_DEVICE") == "1"
    if same_dev:
        local = 0
    backend = os.environ.get("MBLS_BENCH_BACKEND", "nccl")
    if world > 1 and not same_dev and torch.cuda.device_count() < world:
        sys.stderr.write(f"bench.py: rank {rank}: WORLD_SIZE={world} but {torch.cuda.device_count()} GPUs visible\n")
        sys.exit(2)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    amd.lib()
    stream = torch.cuda.current_stream(dev)
    # which device every rank ran on (the line proves the N it claims)
    props = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "device": local, "uuid": str(getattr(props, "uuid", "")), "name": props.name}
    ranks_devices = [me]
    if world > 1:
        ranks_devices = [None] * world
        dist.all_gather_object(ranks_devices, me)
    dist_world = dist.get_world_size() if world > 1 else 1

    def barrier_sync():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def max_over_ranks(x):
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed(fn, reps, warm=1, sync_all=False):
        """wall ms per call of fn over `reps` calls (stream-ordered, synchronised at both ends)"""
        for _ in range(warm):
            fn()
        (barrier_sync if sync_all else lambda: torch.cuda.synchronize(dev))()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        (barrier_sync if sync_all else lambda: torch.cuda.synchronize(dev))()
        return (time.perf_counter() - t0) / reps * 1e3

    # ------------------------------------------------------------------ headline MSM inputs
    n = 1 << args.msm_log
    scalars = torch.zeros((n, 4), dtype=torch.int64, device=dev)
    bases = torch.zeros((n, 12), dtype=torch.int64, device=dev)
    # rank r holds elements [r n, (r + 1) n) of one global stream (N = 1: the test's inputs)
    amd.gen_scalars(scalars, 0x5EED0003, montgomery=True, stream=stream, start=rank * n)
    amd.gen_bases("g1", bases, 0x5EED0013, stream=stream, start=rank * n)
    result = torch.zeros((1, 18), dtype=torch.int64, device=dev)
    partial = torch.zeros((1, 18), dtype=torch.int64, device=dev)
    gathered = torch.zeros((world, 18), dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)

    def sharded_step(sc, bs, m):
        """one rank's production-path MSM; N > 1: Jacobian partial -> all_gather -> EC sum ->
        one (x, y, 1) normalisation (result: ICICLE form on every rank)"""
        if world == 1:
            amd.msm("g1", sc, bs, icicle=True, scalars_mont=True, out=result, stream=stream, is_async=True, n=m)
            return
        amd.msm("g1", sc, bs, icicle="jacobian", scalars_mont=True, out=partial, stream=stream, is_async=True, n=m)
        sharded_msm.gather_partials(partial, world, dist, out=gathered)
        amd.sum_jacobian("g1", gathered, result, stream=stream)
        amd.jacobian_to_icicle("g1", result, stream=stream)

    def msm_step():
        sharded_step(scalars, bases, n)

    for _ in range(args.warmup):
        msm_step()
    # per-call hipEvent times (events on the MSM's own stream, recorded
    # between back-to-back steps: the queue never drains), `value` from their median; the K steps
    # are also bracketed by a barrier + synchronize on both sides and wall-timed (max over ranks)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    barrier_sync()
    t0 = time.perf_counter()
    evs[0].record(stream)
    for i in range(args.steps):
        msm_step()
        evs[i + 1].record(stream)
    barrier_sync()
    msm_time = max_over_ranks(time.perf_counter() - t0)
    step_ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
    med_ms = max_over_ranks(statistics.median(step_ms))
    ms_per_step = med_ms
    msm_per_sec = world * 1e3 / med_ms
    step_stats = {"median_ms": round(med_ms, 4), "mean_ms": round(max_over_ranks(sum(step_ms) / len(step_ms)), 4),
                  "min_ms": round(max_over_ranks(step_ms[0]), 4), "max_ms": round(max_over_ranks(step_ms[-1]), 4),
                  "wall_ms_per_step": round(msm_time / args.steps * 1e3, 4),
                  "wall_msm_per_sec": round(world * args.steps / msm_time, 3),
                  "n": args.steps, "source": "hipEvents on the MSM stream, max over ranks of each statistic"}
    headline_result = result.clone()

    # live per-stage timing (HIP events recorded on the MSM's own stream) for the roofline; the
    # timed steps above run without these events (each marker delays the next dispatch ~10 us)
    msm_prof = {}
    if not args.no_stage_profile:
        amd.profile(True)
        for _ in range(max(3, args.steps // 2)):
            msm_step()
        torch.cuda.synchronize(dev)
        msm_prof = amd.profile_read()
        amd.profile(False)

    extra = {}
    if not args.headline_only:
        extra.update(msm_variants(args, amd, torch, dev, stream, scalars, bases, n, timed, max_over_ranks, world))
    # ------------------------------------------------------------------ config #4: 2^total split over ranks
    cfg4, cfg4_result = None, None
    if args.msm_total_log and not args.headline_only:
        total = 1 << args.msm_total_log
        lo, hi = sharded_msm.shard_range(total, world, rank)
        m = hi - lo
        s4 = torch.zeros((m, 4), dtype=torch.int64, device=dev)
        b4 = torch.zeros((m, 12), dtype=torch.int64, device=dev)
        amd.gen_scalars(s4, 0x5EED0004, montgomery=True, stream=stream, start=lo)
        amd.gen_bases("g1", b4, 0x5EED0013, stream=stream, start=lo)
        torch.cuda.synchronize(dev)
        reps = max(2, args.steps // 4)
        ms4 = max_over_ranks(timed(lambda: sharded_step(s4, b4, m), reps, warm=1, sync_all=True))
        cfg4 = {"workload": f"G1 MSM 2^{args.msm_total_log} points sharded {world}-way (strong scaling)",
                "points_per_rank": m, "reps": reps, "ms_per_msm": round(ms4, 3),
                "msm_per_sec": round(1e3 / ms4, 4),
                "points_per_sec": round(total / ms4 * 1e3, 1),
                "result_digest": digest(result),
                "note": "same result_digest at every N = bit-identical sharded sum; the 1-GPU result is "
                        "pinned to the oracle by tests/test_gpu_parity.py::test_msm_g1_2_24_single_and_sharded"}
        cfg4_result = result.clone()
        del s4, b4
        torch.cuda.empty_cache()

    # ------------------------------------------------------------------ NTT 2^ntt_log (replicas)
    amd.ntt_init_domain()
    nn = 1 << args.ntt_log
    x = torch.zeros((nn, 4), dtype=torch.int64, device=dev)
    y = torch.zeros_like(x)
    amd.gen_scalars(x, 0x5EED0025, montgomery=True, stream=stream)
    ntt_ms_wall = max_over_ranks(timed(lambda: amd.ntt(x, out=y, stream=stream, is_async=True), args.steps,
                                       warm=args.warmup, sync_all=True))
    ntt_per_sec = world * 1e3 / ntt_ms_wall
    ntt_prof = {}
    if not args.no_stage_profile:
        amd.profile(True)
        for _ in range(max(3, args.steps // 2)):
            amd.ntt(x, out=y, stream=stream, is_async=True)
        torch.cuda.synchronize(dev)
        ntt_prof = amd.profile_read()
        amd.profile(False)

    legs = {}
    if not args.headline_only:
        # config #2: NTT 2^20 forward + inverse round trip, device-resident
        x20 = x[: 1 << 20]
        y20 = torch.zeros_like(x20)
        z20 = torch.zeros_like(x20)

        def rt():
            amd.ntt(x20, out=y20, stream=stream, is_async=True)
            amd.ntt(y20, inverse=True, out=z20, stream=stream, is_async=True)
        rt_ms = timed(rt, max(3, args.steps), warm=2)
        legs["ntt20_roundtrip_ms"] = round(rt_ms, 4)
        legs["ntt20_roundtrip_exact"] = bool(torch.equal(z20, x20))
        del y20, z20
        legs["vecops"] = vecops_leg(amd, torch, dev, stream, timed)
        if not args.no_mix:
            legs["mix_g2msm_batched_ntt"] = mix_leg(args, amd, torch, dev, rank, timed)

    # ------------------------------------------------------------------ CPU baseline (rank 0, N=1)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and not args.headline_only:
        cpu = cpu_baseline(args, amd, torch, scalars, bases, n, headline_result, x, cfg4_result)

    if rank == 0:
        def avg(prof, key):
            ms, cnt = prof.get(key, (0.0, 0))
            return ms / cnt if cnt else None

        acc_ms = avg(msm_prof, "msm.accumulate")
        ntt_ms = avg(ntt_prof, "ntt.transform")
        ntt_pass_ms = avg(ntt_prof, "ntt.pass")
        stages = {k: round(v[0] / v[1], 4) for k, v in sorted(msm_prof.items()) if v[1]}
        # dominant kernel: k_accumulate<G1>; algorithmic bytes = 128 B x points per launch
        msm_ach = MSM_BYTES_PER_POINT * n / (acc_ms * 1e-3) / 1e9 if acc_ms else None
        contributions = 2 * n * ((128 + 16 - 1) // 16)  # GLV: 2n digit streams x 8 windows (c = 16)
        ntt_ach = NTT_BYTES_PER_ELEM * nn / (ntt_ms * 1e-3) / 1e9 if ntt_ms else None
        _, pmc_src = pmc_summary()
        ceil = valu_ceiling() or {}
        # G1's accumulation is k_accumulate_r28 (round 5): its own arithmetic's ceiling when measured
        acc_c = ceil.get("acc28x_ceiling") or ceil.get("acc28_ceiling") or ceil.get("acc_ceiling") or {}
        # the shipped pass multiplies in radix 2^29 (round 6): its own body's ceiling when measured
        ntt_c = ceil.get("ntt29_ceiling") or ceil.get("ntt_ceiling") or {}
        isa = ceil.get("isa_2") or {}
        cyc = isa.get("simd_cycles_per_wave_instr")
        # the ceiling's ns per contribution at this MSM's contribution count
        acc_ceiling_ms = acc_c["ns_per_contribution_chip"] * contributions * 1e-6 if acc_c else None
        ntt_ceiling_ms = (ntt_c["ms_per_2^22_transform_10_pairs"] * (args.ntt_log - 2) / 20
                          if ntt_c and args.ntt_log % 2 == 0 else None)
        acc_issue = valu_issue_bound_ms("k_accumulate<G1>", cyc, acc_c.get("mhz_med"))
        passes = [valu_issue_bound_ms(k, cyc, ntt_c.get("mhz_med"))
                  for k in ("k_ntt_pass<true, false, false>", "k_ntt_pass<false, false, false>",
                            "k_ntt_pass<false, true, false>")]
        ntt_issue_ms = round(sum(passes), 4) if args.ntt_log == 22 and all(p is not None for p in passes) else None
        out = {
            "metric": "G1 MSM/sec at 2^20 points + Fr NTT/sec at 2^22 (bit-exact vs BLST)",
            "value": round(msm_per_sec, 3),
            "unit": "MSM/s",
            "n_gpus": world,
            "world_size": dist_world,
            "rank_devices": ranks_devices,
            "same_device_rehearsal": same_dev and world > 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32-limb Montgomery (Fq 381-bit / Fr 255-bit integer)",
            "data": "synthetic: seeded scalars, bases k_i*G generated on device",
            "config": {"workload": f"G1 MSM 2^{args.msm_log} points per GPU, production path (ICICLE entry, "
                                   f"Montgomery scalars + bases in HBM, (x,y,1) result on device); N>1: "
                                   f"sharded, RCCL all-gather of partial sums",
                       "msm_points_per_gpu": n, "ntt_size": nn, "parallelism": f"msm-shard{world}"},
            "msm_step_ms": step_stats,
            "bit_exact": cpu.get("bit_exact") if cpu else None,
            "ntt_per_sec": round(ntt_per_sec, 3),
            "ntt_ms": round(ntt_ms, 4) if ntt_ms else None,
            "msm_stage_ms": stages,
            "roofline": {"kernel": "k_accumulate<G1> (MSM bucket accumulation, dominant)",
                         "bound": "hbm", "achieved": round(msm_ach, 2) if msm_ach else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(msm_ach / HBM_PEAK_GBS, 5) if msm_ach else None,
                         "traffic": pmc_traffic("k_accumulate<G1>"),
                         "traffic_source": f"{pmc_src} (HBM bytes per launch)" if pmc_src else None,
                         "note": "VALU-bound (v_mad_u64_u32): see roofline_valu"},
            "roofline_valu": {"kernel": "k_accumulate<G1>", "bound": "valu",
                              "achieved": round(contributions / (acc_ms * 1e-3) / 1e9, 3) if acc_ms else None,
                              "peak": round(contributions / (acc_ceiling_ms * 1e-3) / 1e9, 3) if acc_ceiling_ms else None,
                              "unit": "G mixed additions/s",
                              "frac": round(acc_ceiling_ms / acc_ms, 4) if acc_ceiling_ms and acc_ms else None,
                              "ceiling_source": "microbench", "ceiling_ms": round(acc_ceiling_ms, 4) if acc_ceiling_ms else None,
                              "ceiling": acc_c or None, "ceiling_run": ceil.get("source"),
                              "measured_cycles_per_valu_instr": cyc,
                              "counter_valu_insts_per_launch": pmc_counter("k_accumulate<G1>", "SQ_INSTS_VALU"),
                              "counter_issue_ms": round(acc_issue, 4) if acc_issue else None,
                              "counter_issue_frac": round(acc_issue / acc_ms, 4) if acc_issue and acc_ms else None,
                              "counter_source": f"{pmc_src} (SQ_INSTS_VALU per launch)" if pmc_src else None,
                              "note": f"{contributions} mixed additions per launch; peak = k_acc28x_ceiling "
                                      "(tools/valu_ceiling.hip: the same radix-2^28 XYZZ xmadd / xmmadd code, launch bounds and chunk "
                                      "structure with the points in LDS: no random gathers), measured on the box; "
                                      "frac = ceiling time / kernel time.  counter_issue_ms = the committed VALU "
                                      "instruction count at the measured cycles per wave-instruction and clock"},
            "roofline_ntt": {"kernel": "k_ntt_pass x passes (one transform)", "bound": "hbm",
                             "achieved": round(ntt_ach, 2) if ntt_ach else None, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(ntt_ach / HBM_PEAK_GBS, 5) if ntt_ach else None,
                             "traffic": ntt_traffic(args.ntt_log),
                             "valu_ceiling_ms": round(ntt_ceiling_ms, 4) if ntt_ceiling_ms else None,
                             "valu_frac": round(ntt_ceiling_ms / ntt_ms, 4) if ntt_ceiling_ms and ntt_ms else None,
                             "valu_ceiling_source": "microbench (k_ntt29_ceiling: the shipped pass's radix-4 body -- "
                                                    "radix-2^29 products, lazy [0, 2r) additions -- register-"
                                                    "resident, twiddle limb planes in LDS; 10 stage pairs, i.e. "
                                                    "the transform's 22 stages minus the first pair's trivial "
                                                    "products)",
                             "counter_issue_ms": ntt_issue_ms,
                             "counter_issue_frac": round(ntt_issue_ms / ntt_ms, 4) if ntt_issue_ms and ntt_ms else None,
                             "pass_ms": round(ntt_pass_ms, 4) if ntt_pass_ms else None},
            "config4_msm_sharded": cfg4,
            "cpu_baseline": cpu,
        }
        out.update(extra)
        out.update(legs)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def msm_variants(args, amd, torch, dev, stream, scalars, bases, n, timed, max_over_ranks, world):
    """the same 2^20 G1 MSM through the reference's raw entry, host-staged scalars, and the
    batched ICICLE call (rank-local: no exchange)"""
    out = {}
    res = torch.zeros((1, 18), dtype=torch.int64, device=dev)
    reps = max(3, args.steps // 2)
    # the reference's raw entry bls12_381_g1_msm_cuda (icicle_curve_api.cu:679): standard scalars,
    # Jacobian Montgomery result, no normalisation (round 1's headline)
    s_std = torch.zeros_like(scalars)
    amd.gen_scalars(s_std, 0x5EED0003, montgomery=False, stream=stream)
    raw_ms = max_over_ranks(timed(lambda: amd.msm("g1", s_std, bases, icicle=False, out=res, stream=stream,
                                                  is_async=True, n=n), reps))
    out["msm_raw_entry_per_sec"] = round(world * 1e3 / raw_ms, 3)
    del s_std
    # prepared bases (precompute_factor 2 = the [P, phi P] table, built once per base set as the
    # prover uploads its SRS once): the MSM's front only splits scalars
    table = torch.zeros((2 * n, 12), dtype=torch.int64, device=dev)
    amd.precompute_bases("g1", bases, 2, n, out=table)
    pres = torch.zeros((1, 18), dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    prep_ms = max_over_ranks(timed(lambda: amd.msm("g1", scalars, table, icicle=True, scalars_mont=True, points_mont=False,
                                                   precompute_factor=2, out=pres, stream=stream, is_async=True, n=n),
                                   reps))
    amd.msm("g1", scalars, bases, icicle=True, scalars_mont=True, out=res, stream=stream, n=n)
    torch.cuda.synchronize(dev)
    amd.profile(True)
    for _ in range(3):
        amd.msm("g1", scalars, table, icicle=True, scalars_mont=True, points_mont=False, precompute_factor=2, out=pres,
                stream=stream, is_async=True, n=n)
    torch.cuda.synchronize(dev)
    pprof = amd.profile_read()
    amd.profile(False)
    out["msm_prepared_bases"] = {"msm_per_sec": round(world * 1e3 / prep_ms, 3), "ms": round(prep_ms, 4),
                                 "equal_to_plain": bool(torch.equal(pres, res)),
                                 "stage_ms": {k: round(v[0] / v[1], 4) for k, v in sorted(pprof.items()) if v[1]},
                                 "note": "precompute_factor 2 = point-major [P, phi P] table built once "
                                         "(precompute_bases); same scalars and (x,y,1) result as `value`"}
    del table
    # the reference's recommended MIDNIGHT_GPU_PRECOMPUTE=4 (core/config.rs:101-125) and 8: the
    # point-major 2^(64 f) / 2^(32 f) shift tables (fewer windows: smaller tail, shorter fold)
    pre = {}
    for F in (4, 8):
        tabF = torch.zeros((F * n, 12), dtype=torch.int64, device=dev)
        amd.precompute_bases("g1", bases, F, n, out=tabF)
        rF = torch.zeros((1, 18), dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)
        f_ms = max_over_ranks(timed(lambda: amd.msm("g1", scalars, tabF, icicle=True, scalars_mont=True,
                                                    points_mont=False, precompute_factor=F, out=rF, stream=stream,
                                                    is_async=True, n=n), reps))
        amd.profile(True)
        for _ in range(3):
            amd.msm("g1", scalars, tabF, icicle=True, scalars_mont=True, points_mont=False, precompute_factor=F,
                    out=rF, stream=stream, is_async=True, n=n)
        torch.cuda.synchronize(dev)
        fprof = amd.profile_read()
        amd.profile(False)
        pre[f"factor_{F}"] = {"msm_per_sec": round(world * 1e3 / f_ms, 3), "ms": round(f_ms, 4),
                              "equal_to_plain": bool(torch.equal(rF, res)),
                              "table_bytes": F * n * 96,
                              "stage_ms": {k: round(v[0] / v[1], 4) for k, v in sorted(fprof.items()) if v[1]}}
        del tabF
    out["msm_precompute_tables"] = dict(pre, note="precompute_bases once (core/msm.rs:401-506 with "
                                        "MIDNIGHT_GPU_PRECOMPUTE=F), then MSMs of the same scalars; never `value` "
                                        "(the reference's benchmark uploads plain bases)")
    # host-inclusive: scalars in pinned host memory, staged by the call (end-to-end
    # rate with the scalar H2D; never `value`)
    host_s = scalars.cpu().pin_memory()
    torch.cuda.synchronize(dev)
    hi_ms = max_over_ranks(timed(lambda: amd.msm("g1", host_s, bases, icicle=True, scalars_mont=True, out=res,
                                                 stream=stream, is_async=True, n=n), reps))
    out["msm_host_scalars_per_sec"] = round(world * 1e3 / hi_ms, 3)
    del host_s
    # the reference's production call shape (core/msm.rs:594-682, msm_with_device_bases): PAGEABLE
    # host Montgomery scalars (HostSlice over a Rust Vec), device bases, device result, then
    # copy_to_host of the one point -- every byte through the boundary, timed per call
    page_s = scalars.cpu().numpy().copy()  # ordinary (pageable) host memory
    host_r = None

    def pageable_call():
        nonlocal host_r
        amd.msm("g1", page_s, bases, icicle=True, scalars_mont=True, out=res, stream=stream, is_async=False, n=n)
        host_r = res.cpu()
    torch.cuda.synchronize(dev)
    pg_ms = max_over_ranks(timed(pageable_call, reps))
    out["msm_pageable_host_per_sec"] = round(world * 1e3 / pg_ms, 3)
    out["msm_pageable_host_note"] = ("core/msm.rs:665-675 shape: pageable host scalars (32 MiB H2D), device bases, "
                                     "device result copied to the host; PCIe-inclusive, never `value`")
    del page_s
    # independent MSMs on alternating streams (the reference's async shape: core/msm.rs:742 makes a
    # stream per call): one MSM's latency-bound tail overlaps the next one's front and
    # accumulation; each stream's calls lease their own scratch context (no false dependency)
    s2 = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    r2 = [torch.zeros((1, 18), dtype=torch.int64, device=dev) for _ in range(2)]
    torch.cuda.synchronize(dev)

    def two_stream_pair():
        for k in range(2):
            amd.msm("g1", scalars, bases, icicle=True, scalars_mont=True, out=r2[k], stream=s2[k], is_async=True, n=n)
    pair_ms = max_over_ranks(timed(two_stream_pair, max(3, args.steps // 2), warm=2))
    out["msm_two_streams"] = {"msm_per_sec": round(world * 2e3 / pair_ms, 3), "ms_per_pair": round(pair_ms, 4),
                              "results_equal": bool(torch.equal(r2[0], res) and torch.equal(r2[1], res)),
                              "note": "the same 2^20 MSM issued alternately on two caller streams (async, device "
                                      "result), as an async prover issues independent commitments; never `value`"}
    # skewed scalar columns (selector-like 0 / 1, small values): the heavy-bucket paths
    # (DESIGN.md section 5 "Skewed scalars"; parity in tests/test_gpu_parity.py::test_msm_skewed_scalars)
    sk = torch.zeros_like(scalars)
    amd.gen_scalars(sk, 0x5EED0003, montgomery=False, stream=stream)
    torch.cuda.synchronize(dev)
    even = torch.arange(n, device=dev) % 2 == 0
    skew = {}
    for name in ("half_one", "bits8", "ones"):
        if name == "half_one":
            sk[even] = torch.tensor([1, 0, 0, 0], dtype=torch.int64, device=dev)
        elif name == "bits8":
            sk[:, 1:] = 0
            sk[:, 0] = torch.randint(0, 256, (n,), device=dev, generator=torch.Generator(dev).manual_seed(8))
        else:
            sk[:] = torch.tensor([1, 0, 0, 0], dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)
        sk_ms = max_over_ranks(timed(lambda: amd.msm("g1", sk, bases, icicle=True, scalars_mont=False, out=res,
                                                     stream=stream, is_async=True, n=n), reps))
        skew[f"{name}_ms"] = round(sk_ms, 4)
    out["msm_skewed_scalars"] = dict(skew, note="G1 2^20, standard-form scalars: half the scalars 1 (the rest "
                                     "random), 8-bit scalars, every scalar 1; never `value`")
    del sk
    # batched MSMs (ICICLE batch_size, shared device bases): members pipelined on two streams
    if args.msm_batch > 1:
        B = args.msm_batch
        sb = torch.zeros((B * n, 4), dtype=torch.int64, device=dev)
        amd.gen_scalars(sb, 0x5EED0033, montgomery=True, stream=stream)
        rb = torch.zeros((B, 18), dtype=torch.int64, device=dev)
        breps = max(2, args.steps // 4)
        b_ms = max_over_ranks(timed(lambda: amd.msm("g1", sb, bases, icicle=True, scalars_mont=True, batch=B,
                                                    out=rb, stream=stream, is_async=True, n=n), breps))
        # the first and last members against single ICICLE MSMs of the same scalars
        one = torch.zeros((1, 18), dtype=torch.int64, device=dev)
        same = True
        for k in (0, B - 1):
            amd.msm("g1", sb[k * n:(k + 1) * n], bases, icicle=True, scalars_mont=True, out=one, stream=stream, n=n)
            torch.cuda.synchronize()
            same = same and bool(torch.equal(one[0], rb[k]))
        out["msm_batch"] = {"batch": B, "reps": breps, "ms_per_batch": round(b_ms, 3),
                            "msm_per_sec": round(world * B * 1e3 / b_ms, 3),
                            "members_equal_single_msm": same,
                            "note": "ICICLE batch_size (core/msm.rs msm_batch_with_device_bases); member b's front "
                                    "(digits, sort) and tail (reduction, fold, (x,y,1)) on two side streams beside "
                                    "the accumulations of members b - 1 / b + 1 (TailPipe, msm_core.hpp)"}
        del sb
    return out


def vecops_leg(amd, torch, dev, stream, timed):
    """config #1 on the GPU: vector add / mul at 2^16 (launch-bound) and 2^24 (HBM roofline)"""
    out = {}
    for log_n in (16, 24):
        n = 1 << log_n
        a = torch.zeros((n, 4), dtype=torch.int64, device=dev)
        b = torch.zeros_like(a)
        c = torch.zeros_like(a)
        amd.gen_scalars(a, 0x5EED0001, montgomery=True, stream=stream)
        amd.gen_scalars(b, 0x5EED0101, montgomery=True, stream=stream)
        for op in ("add", "mul"):
            reps = 200 if log_n == 16 else 20
            ms = timed(lambda: amd.vec_op(op, a, b, out=c, stream=stream, is_async=True), reps, warm=3)
            gbs = VEC_BYTES_PER_ELEM * n / (ms * 1e-3) / 1e9
            out[f"{op}_2^{log_n}"] = {"ms": round(ms, 5), "gb_per_s": round(gbs, 1),
                                      "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}
        del a, b, c
    out["note"] = "96 B/elem algorithmic; wall time per call (host launch included at 2^16)"
    return out


def ntt_traffic(log_n):
    """HBM bytes of one forward 2^22 transform: first + middle + last pass (pmc_probe sizes)"""
    if log_n != 22:
        return None
    names = ("k_ntt_pass<true, false, false>", "k_ntt_pass<false, false, false>", "k_ntt_pass<false, true, false>")
    parts = [pmc_traffic(k) for k in names]
    return None if any(p is None for p in parts) else sum(parts)


def mix_leg(args, amd, torch, dev, rank, timed):
    """BASELINE config #5: G2 MSM 2^msm_log (ICICLE entry) and a batch of Fr NTTs 2^ntt_log
    enqueued on two HIP streams at once (PLONK-prover-shaped mix); each alone and overlapped."""
    n = 1 << args.msm_log
    nn = 1 << args.ntt_log
    B = args.mix_batch
    # the G2 MSM on a HIGH-priority stream, the NTT batch on a normal one: the hardware dispatches
    # the NTT's workgroups only when the MSM leaves slots free -- its front and its latency-bound
    # tail (bucket sums, reduction levels, final fold: ~2 ms of few-wave chains) -- instead of
    # time-slicing the SIMDs with its VALU-bound accumulation (round 4: equal priorities,
    # overlapped == sum of isolated)
    s_a = torch.cuda.Stream(dev, priority=-1)
    s_b = torch.cuda.Stream(dev)
    s_a0 = torch.cuda.Stream(dev)  # equal-priority reference run
    sc = torch.zeros((n, 4), dtype=torch.int64, device=dev)
    bs = torch.zeros((n, 24), dtype=torch.int64, device=dev)
    amd.gen_scalars(sc, 0x5EED0005, montgomery=True, stream=s_a)
    amd.gen_bases("g2", bs, 0x5EED0015, stream=s_a)
    res = torch.zeros((1, 36), dtype=torch.int64, device=dev)
    xb = torch.zeros((B * nn, 4), dtype=torch.int64, device=dev)
    yb = torch.zeros_like(xb)
    amd.gen_scalars(xb, 0x5EED0025, montgomery=True, stream=s_b)
    torch.cuda.synchronize(dev)

    def g2(stream=None):
        amd.msm("g2", sc, bs, icicle=True, scalars_mont=True, out=res, stream=stream or s_a, is_async=True, n=n)

    def ntts():
        amd.ntt(xb, out=yb, batch=B, stream=s_b, is_async=True)

    reps = max(2, min(args.steps, 5))
    g2_ms = timed(g2, reps)
    res_iso = res.clone()
    ntt_ms = timed(ntts, reps)
    yb_iso = yb.clone()
    res.zero_()
    yb.zero_()
    torch.cuda.synchronize(dev)
    # the NTT batch made to wait for the G2 MSM's accumulation (mbls_msm_accumulate_event): it runs in
    # the MSM's latency-bound tail instead of slowing its front (round 5 timeline: without the event
    # the low-priority NTT filled the slots of the G2 front and the front took 2 ms instead of 0.4)
    acc_ev = amd.HipEvent()

    def overlapped():
        amd.msm_accumulate_event(s_a, acc_ev.handle)
        g2()
        acc_ev.wait(s_b)
        ntts()
    both_ms = timed(overlapped, reps)
    # the overlapped run must reproduce the isolated outputs bit for bit (the G2 result is pinned
    # to the oracle by tests/test_gpu_parity.py::test_bench_msm_2_20_production_path[g2], the
    # batch members by ::test_bench_ntt_2_22_single_and_batch4)
    g2_same, ntt_same = bool(torch.equal(res, res_iso)), bool(torch.equal(yb, yb_iso))
    assert g2_same and ntt_same, f"config #5 overlapped outputs differ from isolated: g2 {g2_same} ntt {ntt_same}"
    res.zero_()
    yb.zero_()
    torch.cuda.synchronize(dev)
    both_eq_ms = timed(lambda: (g2(s_a0), ntts()), reps)  # the same with equal stream priorities
    assert torch.equal(res, res_iso) and torch.equal(yb, yb_iso), "config #5 equal-priority outputs differ"
    del yb_iso
    # G2 with prepared bases (precompute_factor 4 = [P, psi P, psi^2 P, psi^3 P], built once)
    table = torch.zeros((4 * n, 24), dtype=torch.int64, device=dev)
    amd.precompute_bases("g2", bs, 4, n, out=table)
    pres = torch.zeros_like(res)
    torch.cuda.synchronize(dev)
    g2p_ms = timed(lambda: amd.msm("g2", sc, table, icicle=True, scalars_mont=True, points_mont=False,
                                   precompute_factor=4, out=pres, stream=s_a, is_async=True, n=n), reps)
    g2p_same = bool(torch.equal(pres, res_iso))
    del table, pres
    acc_ms = g2_stage_ms(amd, torch, dev, g2, s_a)
    contributions = 4 * n * ((64 + 16 - 1) // 16)  # psi split: 4n digit streams x 4 windows (c = 16)
    ceil = valu_ceiling() or {}
    g2c = ceil.get("acc28px_ceiling") or ceil.get("acc28p_ceiling") or {}
    g2_ceiling_ms = g2c["ms_per_2^20_g2_msm_contributions"] * contributions / 16777216.0 if g2c else None
    return {"g2_msm_points": n, "ntt_batch": B, "ntt_size": nn, "g2_msm_ms": round(g2_ms, 3),
            "g2_msm_per_sec": round(1e3 / g2_ms, 3),
            "g2_prepared_bases_ms": round(g2p_ms, 3), "g2_prepared_equal_to_plain": g2p_same,
            "g2_roofline_hbm_frac": round(G2_BYTES_PER_POINT * n / (g2_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            "g2_accumulate_ms": round(acc_ms, 4) if acc_ms else None,
            "g2_roofline_valu": {"kernel": "k_accumulate_r28p<G2> (pair-sliced radix-2^28 Fq2 lanes)", "bound": "valu",
                                 "achieved": round(contributions / (acc_ms * 1e-3) / 1e9, 3) if acc_ms else None,
                                 "peak": round(contributions / (g2_ceiling_ms * 1e-3) / 1e9, 3)
                                 if g2_ceiling_ms else None,
                                 "unit": "G mixed additions/s",
                                 "frac": round(g2_ceiling_ms / acc_ms, 4) if g2_ceiling_ms and acc_ms else None,
                                 "ceiling_ms": round(g2_ceiling_ms, 4) if g2_ceiling_ms else None,
                                 "ceiling": g2c or None,
                                 "ceiling_source": ceil.get("source", "live: tools/valu_ceiling") if g2c else None,
                                 "note": f"{contributions} mixed additions per launch (psi split: 4n digit streams x 4 "
                                         "windows); peak = k_acc28px_ceiling (tools/valu_ceiling.hip: the same "
                                         "pair-sliced XYZZ xmadd / xmmadd and launch bounds with the points in LDS), "
                                         "measured on the box; frac = ceiling time / kernel time"},
            "batched_ntt_ms": round(ntt_ms, 3), "overlapped_ms": round(both_ms, 3),
            "sum_isolated_ms": round(g2_ms + ntt_ms, 3), "streams": 2,
            "overlap_ratio": round(both_ms / (g2_ms + ntt_ms), 4),
            "overlapped_equal_priority_ms": round(both_eq_ms, 3),
            "overlap_note": "G2 MSM on a high-priority stream; the NTT batch on a normal-priority stream waits for "
                            "an event the MSM records when its accumulation is enqueued (mbls_msm_accumulate_event), "
                            "so its workgroups fill the slots the MSM's latency-bound tail (bucket sums, reduction "
                            "levels, final fold) leaves idle.  overlapped_equal_priority_ms: both enqueued at once on "
                            "equal-priority streams, no event -- both VALU-bound legs time-slice the SIMDs",
            "overlapped_outputs_bit_identical": g2_same and ntt_same,
            "g2_result_digest": digest(res)}


def g2_stage_ms(amd, torch, dev, g2, st):
    """average k_accumulate<G2> stage time (HIP events on the MSM's stream)"""
    amd.profile(True)
    for _ in range(3):
        g2()
    st.synchronize()
    prof = amd.profile_read()
    amd.profile(False)
    ms, cnt = prof.get("msm.accumulate", (0.0, 0))
    return ms / cnt if cnt else None


def cpu_baseline(args, amd, torch, scalars, bases, n, headline_result, ntt_in, cfg4_result=None):
    """The oracle (oracle/bls12_381_oracle.c: C restatement of the reference CPU semantics,
    OpenMP Pippenger / radix-2 NTT / vecops) on the host cores, on the SAME inputs as the GPU
    legs.  Protocol: one untimed warmup, then the median of >= 5 runs for the
    2^msm_log G1 MSM (bounded by --cpu-budget-s), the NTTs and the G2 MSM; config #4's 2^24 G1 MSM
    once.  Each MSM result must equal the GPU's (bit_exact).  BLST is not available."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import gpu_helpers
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

    def med(fn, runs=5, budget_s=None):
        fn()  # warmup
        ts, t_start = [], time.perf_counter()
        while len(ts) < runs and (budget_s is None or len(ts) < 2 or time.perf_counter() - t_start < budget_s):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts), len(ts)

    got = gpu_helpers.decode_icicle("g1", amd.to_numpy_u64(headline_result)[0])
    # the baseline: the BLST-shaped Pippenger (signed digits, XYZZ buckets, window-parallel:
    # orc_g1_msm_fast); the checker's plain restatement timed beside it
    ref = H.oracle_msm("g1", s_std, b, threads=threads, fast=True)
    msm_s, runs = med(lambda: H.oracle_msm("g1", s_std, b, threads=threads, fast=True), 5, args.cpu_budget_s)
    bit_exact = got == H.g1_from_affine_mont(ref)
    ref_c = H.oracle_msm("g1", s_std, b, threads=threads)
    chk_s, chk_runs = med(lambda: H.oracle_msm("g1", s_std, b, threads=threads), 3, args.cpu_budget_s)
    out = {"value": round(1.0 / msm_s, 4), "unit": "MSM/s", "cores": threads, "kind": "port",
           "sample": f"full G1 MSM of 2^{args.msm_log} points on the headline's inputs, median of {runs} runs after "
                     f"one warmup, oracle/bls12_381_oracle.c orc_g1_msm_fast (BLST-shaped: signed c-bit digits, "
                     f"XYZZ buckets, windows split evenly over {threads} OpenMP threads, C __int128 Montgomery "
                     f"products); BLST itself is not available (no network, not in the image)",
           "bit_exact": bool(bit_exact),
           "checker_port_msm_per_sec": round(1.0 / chk_s, 4), "checker_port_runs": chk_runs,
           "checker_port_bit_exact": bool(got == H.g1_from_affine_mont(ref_c)),
           "checker_port_note": "the oracle's plain restatement (orc_g1_msm: unsigned windows, Jacobian buckets, "
                                "points split over threads), the round-5 baseline"}
    # NTT (config #2 / the metric's second half): oracle radix-2 best_fft, all threads
    xn = np.ascontiguousarray(amd.to_numpy_u64(ntt_in))
    for log_n in (20, args.ntt_log):
        a = np.ascontiguousarray(xn[: 1 << log_n])
        t, _ = med(lambda: H.oracle_ntt(a, log_n, False, threads=threads), 5)
        out[f"ntt_2^{log_n}_ms"] = round(t * 1e3, 2)
    # vecops 2^16 (config #1: the CPU path of MIDNIGHT_DEVICE=cpu, core/vecops.rs:575-610)
    va = np.ascontiguousarray(xn[: 1 << 16])
    vb = np.ascontiguousarray(xn[1 << 16: 2 << 16])
    vc = np.zeros_like(va)
    for th, tag in ((1, "1t"), (threads, f"{threads}t")):
        o.orc_set_threads(th)
        for op, fn in (("add", o.orc_vec_add), ("mul", o.orc_vec_mul)):
            t, _ = med(lambda: fn(H.ptr(vc), H.ptr(va), H.ptr(vb), 1 << 16), 20)
            out[f"vec_{op}_2^16_{tag}_us"] = round(t * 1e6, 1)
    o.orc_set_threads(0)
    out["protocol"] = "median of >= 5 runs after one untimed warmup (MSM 2^20, NTT, G2); 20 runs for vecops"
    # G2 MSM (config #5) on the mix leg's inputs
    if not args.no_mix:
        g2s = torch.zeros((n, 4), dtype=torch.int64, device=scalars.device)
        g2b = torch.zeros((n, 24), dtype=torch.int64, device=scalars.device)
        amd.gen_scalars(g2s, 0x5EED0005, montgomery=False)
        amd.gen_bases("g2", g2b, 0x5EED0015)
        torch.cuda.synchronize()
        g2sn = np.ascontiguousarray(amd.to_numpy_u64(g2s))
        g2bn = np.ascontiguousarray(amd.to_numpy_u64(g2b))
        del g2s, g2b
        t, runs = med(lambda: H.oracle_msm("g2", g2sn, g2bn, threads=threads, fast=True), 5)
        out[f"g2_msm_2^{args.msm_log}_ms"] = round(t * 1e3, 1)
        out["g2_msm_runs"] = runs
        del g2sn, g2bn
    # config #4: the 2^msm_total_log G1 MSM once, bit-exact against the GPU's (1-GPU) result
    if args.msm_total_log and not args.no_cpu_total and cfg4_result is not None:
        total = 1 << args.msm_total_log
        s4 = torch.zeros((total, 4), dtype=torch.int64, device=scalars.device)
        amd.gen_scalars(s4, 0x5EED0004, montgomery=False)
        s4n = np.ascontiguousarray(amd.to_numpy_u64(s4))
        del s4
        b4 = torch.zeros((total, 12), dtype=torch.int64, device=scalars.device)
        amd.gen_bases("g1", b4, 0x5EED0013)
        b4n = np.ascontiguousarray(amd.to_numpy_u64(b4))
        del b4
        torch.cuda.empty_cache()
        t0 = time.perf_counter()
        r4 = H.oracle_msm("g1", s4n, b4n, threads=threads, fast=True)
        t4 = time.perf_counter() - t0
        got4 = gpu_helpers.decode_icicle("g1", amd.to_numpy_u64(cfg4_result)[0])
        out[f"g1_msm_2^{args.msm_total_log}_ms"] = round(t4 * 1e3, 1)
        out[f"g1_msm_2^{args.msm_total_log}_note"] = "config #4 on the CPU: timed once (SURVEY.md 8d row #4)"
        out[f"g1_msm_2^{args.msm_total_log}_bit_exact"] = bool(got4 == H.g1_from_affine_mont(r4))
        del s4n, b4n
    return out


if __name__ == "__main__":
    main()
