"""Prepared bases (DESIGN.md "prepared bases"): precompute_bases with precompute_factor equal to the
group's endomorphism split writes the point-major image table -- G1 factor 2: [P, phi P]; G2
factor 4: [P, psi P, psi^2 P, psi^3 P] -- once per base set (core/msm.rs:308-332 uploads the bases
once per proof, :401-506 precomputes them); an MSM with that factor splits only its scalars.
Checked against the oracle: the table contents (pyref phi / psi), split-boundary scalars, small
bit sizes (the prepared table always takes the split), msm_size < bases_size, c > 16 for G2, the
benchmark seeds at 2^20 and a batch with per-member tables."""
import numpy as np
import pytest

import helpers as H
from helpers import pyref as pr

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


def _std_scalars(seed, n):
    s = np.zeros((n, 4), dtype=np.uint64)
    H.oracle().orc_gen_scalars(H.ptr(s), seed, n)
    return s


def test_prepared_tables_hold_the_images(amd):
    import torch
    n = 37
    b1 = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b1, 0x5EED0F01)
    t1 = amd.precompute_bases("g1", b1, 2, n)
    bn = amd.to_numpy_u64(b1)
    for i in range(n):
        p = H.g1_from_affine_mont(bn[i])
        assert H.g1_from_affine_mont(t1[2 * i]) == p
        assert H.g1_from_affine_mont(t1[2 * i + 1]) == pr.glv_phi(p)
    n2 = 9
    b2 = torch.zeros((n2, 24), dtype=torch.int64, device="cuda")
    amd.gen_bases("g2", b2, 0x5EED0F02)
    t2 = amd.precompute_bases("g2", b2, 4, n2)
    bn2 = amd.to_numpy_u64(b2)
    for i in range(n2):
        p = H.g2_from_affine_mont(bn2[i])
        q = p
        for j in range(4):
            assert H.g2_from_affine_mont(t2[4 * i + j]) == q, (i, j)
            q = pr.psi(q)


def test_prepared_g1_boundaries_and_bitsizes(amd, gh):
    import torch
    edge = H.glv_edge_scalars()
    g = pr.rng(31)
    sc = edge + [g.randrange(pr.R) for _ in range(96 - len(edge))]
    n = len(sc)
    nb = n + 17  # msm_size < bases_size: a prefix of the point-major table
    b = torch.zeros((nb, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0F03)
    bn = amd.to_numpy_u64(b)
    table = amd.precompute_bases("g1", b, 2, nb)
    for bits in (0, 128, 64):
        vals = sc if bits == 0 else [x % (1 << bits) for x in sc]
        s = H.ints_to_limbs(vals, 4)
        ref = H.g1_from_affine_mont(H.oracle_msm("g1", s, np.ascontiguousarray(bn[:n])))
        for c in (0, 5, 16, 18):
            r = amd.msm("g1", s, table, c=c, bitsize=bits, precompute_factor=2, n=n)
            assert gh.decode_icicle("g1", r[0]) == ref, (bits, c)


def test_prepared_g2_boundaries_and_large_c(amd, gh):
    import torch
    edge = H.psi_edge_scalars()
    g = pr.rng(32)
    sc = edge + [g.randrange(pr.R) for _ in range(48 - len(edge))]
    n = len(sc)
    b = torch.zeros((n, 24), dtype=torch.int64, device="cuda")
    amd.gen_bases("g2", b, 0x5EED0F04)
    bn = amd.to_numpy_u64(b)
    table = amd.precompute_bases("g2", b, 4, n)
    s = H.ints_to_limbs(sc, 4)
    ref = H.g2_from_affine_mont(H.oracle_msm("g2", s, bn))
    for c in (0, 6, 16, 18):  # c > 16 runs as 16 (the psi digits)
        r = amd.msm("g2", s, table, c=c, precompute_factor=4, n=n)
        assert gh.decode_icicle("g2", r[0]) == ref, c
    r = amd.msm("g2", s, table, icicle=False, precompute_factor=4, n=n)
    assert gh.decode_jacobian_mont("g2", r[0]) == ref
    small = H.ints_to_limbs([x % (1 << 100) for x in sc], 4)
    ref = H.g2_from_affine_mont(H.oracle_msm("g2", small, bn))
    r = amd.msm("g2", small, table, bitsize=100, precompute_factor=4, n=n)
    assert gh.decode_icicle("g2", r[0]) == ref


@pytest.mark.parametrize("group,log_n", [("g1", 20), ("g2", 16)])
def test_prepared_bench_seeds(amd, gh, group, log_n):
    """the benchmark's inputs (bench.py seeds, ICICLE entry, Montgomery scalars, device result)
    through the prepared table, equal to the oracle"""
    import torch
    n = 1 << log_n
    w, f = (12, 2) if group == "g1" else (24, 4)
    seed_s, seed_b = (0x5EED0003, 0x5EED0013) if group == "g1" else (0x5EED0005, 0x5EED0015)
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, seed_s, montgomery=True)
    b = torch.zeros((n, w), dtype=torch.int64, device="cuda")
    amd.gen_bases(group, b, seed_b)
    table = torch.zeros((n * f, w), dtype=torch.int64, device="cuda")
    amd.precompute_bases(group, b, f, n, out=table)
    out = torch.zeros((1, 18 if group == "g1" else 36), dtype=torch.int64, device="cuda")
    amd.msm(group, s, table, icicle=True, scalars_mont=True, points_mont=False, precompute_factor=f, out=out,
            is_async=True, n=n)
    torch.cuda.synchronize()
    ref = H.oracle_msm(group, _std_scalars(seed_s, n), amd.to_numpy_u64(b), threads=ORACLE_THREADS)
    dec = H.g1_from_affine_mont if group == "g1" else H.g2_from_affine_mont
    assert gh.decode_icicle(group, amd.to_numpy_u64(out)[0]) == dec(ref)


def test_prepared_batch_per_member_tables(amd, gh):
    """batch of 3 (pipelined members) with per-member prepared tables and with one shared table"""
    import torch
    n, B = 5000, 3
    s = torch.zeros((B * n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0F05, montgomery=True)
    b = torch.zeros((B * n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0F06)
    tables = torch.cat([amd.torch_u64(amd.precompute_bases("g1", b[k * n:(k + 1) * n], 2, n)) for k in range(B)])
    torch.cuda.synchronize()
    sn, bn = amd.to_numpy_u64(s), amd.to_numpy_u64(b)
    std = _std_scalars(0x5EED0F05, B * n)
    r = amd.msm("g1", s, tables, scalars_mont=True, batch=B, shared_bases=False, precompute_factor=2, n=n)
    for k in range(B):
        ref = H.oracle_msm("g1", np.ascontiguousarray(std[k * n:(k + 1) * n]),
                           np.ascontiguousarray(bn[k * n:(k + 1) * n]), threads=ORACLE_THREADS)
        assert gh.decode_icicle("g1", r[k]) == H.g1_from_affine_mont(ref), k
    r = amd.msm("g1", s, tables[:2 * n], scalars_mont=True, batch=B, shared_bases=True, precompute_factor=2, n=n)
    for k in range(B):
        ref = H.oracle_msm("g1", np.ascontiguousarray(std[k * n:(k + 1) * n]), np.ascontiguousarray(bn[:n]),
                           threads=ORACLE_THREADS)
        assert gh.decode_icicle("g1", r[k]) == H.g1_from_affine_mont(ref), k
    del sn


def test_large_shift_tables_at_2e20(amd, gh):
    """G1 tables at 2^20 through every plan make_plan has for them: F = 3 and 16 (1.6 GB, above
    1 GiB) run the GLV plan on slot 0 of the table with a compact per-call [P, phi P] (make_plan
    bstride), F = 4 and 8 (403 / 805 MB) the shift plan; the benchmark inputs, Montgomery
    scalars, equal to the oracle"""
    import torch
    n = 1 << 20
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0003, montgomery=True)
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0013)
    torch.cuda.synchronize()
    ref = H.g1_from_affine_mont(H.oracle_msm("g1", _std_scalars(0x5EED0003, n), amd.to_numpy_u64(b),
                                             threads=ORACLE_THREADS))
    for F in (3, 4, 8, 16):
        table = torch.zeros((n * F, 12), dtype=torch.int64, device="cuda")
        amd.precompute_bases("g1", b, F, n, out=table)
        out = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
        amd.msm("g1", s, table, icicle=True, scalars_mont=True, points_mont=False, precompute_factor=F, out=out, n=n)
        torch.cuda.synchronize()
        assert gh.decode_icicle("g1", amd.to_numpy_u64(out)[0]) == ref, F
        del table
        torch.cuda.empty_cache()


@pytest.mark.parametrize("group,n,factors", [
    ("g1", 200, (3, 4, 8, 16, 32)),
    ("g1", 5000, (3, 4, 5, 6, 7, 8, 16)),
    ("g1", (1 << 13) + 3, (4, 8, 16)),
    ("g2", 200, (2, 3, 8, 16)),
    ("g2", 3000, (2, 3, 5, 8, 16)),
])
def test_shift_and_slot0_plans(amd, gh, group, n, factors):
    """every precompute factor, whichever plan make_plan picks for it (shift plan with the
    measured windows for F = 4 / 8 / 16, the split plan on slot 0 of the table for the others),
    full-width and 64-bit scalars and a caller's c, edge scalars and equal points, equal to the
    oracle"""
    import torch
    w = 12 if group == "g1" else 24
    g = pr.rng(40 + n)
    # block and window boundaries of every table shape (2^16 k - 1, 2^(sF f)), the split
    # boundaries, and one scalar repeated 40 times (a heavy bucket in every window)
    edge = (H.glv_edge_scalars() if group == "g1" else H.psi_edge_scalars()) + \
        [(1 << k) - 1 for k in (8, 11, 13, 16, 32, 37, 43, 52, 64, 86, 128, 172, 192, 240)] + \
        [1 << k for k in (16, 32, 64, 128, 192, 240)] + [0x5EED << 100] * 40
    sc = [x % pr.R for x in edge][:n] + [g.randrange(pr.R) for _ in range(max(0, n - len(edge)))]
    b = torch.zeros((n, w), dtype=torch.int64, device="cuda")
    amd.gen_bases(group, b, 0x5EED0F10 + n)
    b[1] = b[0]  # equal points: a doubling inside a bucket chain
    b[3] = b[2]
    bn = amd.to_numpy_u64(b)
    dec = H.g1_from_affine_mont if group == "g1" else H.g2_from_affine_mont
    cases = []
    for bits in (0, 64):
        vals = sc if bits == 0 else [x % (1 << 64) for x in sc]
        s = H.ints_to_limbs(vals, 4)
        cases.append((bits, s, dec(H.oracle_msm(group, s, bn, threads=ORACLE_THREADS))))
    for F in factors:
        table = amd.precompute_bases(group, b, F, n)
        for bits, s, ref in cases:
            for c in ((0, 13) if bits == 0 else (0,)):
                r = amd.msm(group, s, table, c=c, bitsize=bits, precompute_factor=F, n=n)
                assert gh.decode_icicle(group, r[0]) == ref, (F, bits, c)
