"""CPU-only checks of the MSM schedule the library picks (make_plan through the host-only
mbls_msm_plan diagnostics export; no device work): the split plans and their windows, prepared
tables, and which precompute factors run the shift plan or the split plan on slot 0 of the table
("Shift tables: which plan" and "Window sizes below 2^20").  The results of
every plan are checked against the oracle by tests/test_gpu_prepared.py on the GPU."""
import os
import subprocess
import sys

import pytest

import helpers as H

PKG = os.path.join(H.ROOT, "midnight-bls12-381-cuda_amd")
LIB = os.path.join(PKG, "lib", "libbls12_381_mi355x.so")


@pytest.fixture(scope="module")
def amd():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", PKG, "-j8", "-s"])
    sys.path.insert(0, PKG)
    import bls12_381_amd
    return bls12_381_amd


@pytest.mark.parametrize("log_n,c", [(8, 8), (13, 8), (14, 11), (15, 11), (16, 16), (20, 16), (24, 16)])
def test_g1_plain_bases_take_the_glv_split(amd, log_n, c):
    p = amd.msm_plan("g1", 1 << log_n)
    assert (p["split"], p["c"], p["F"], p["bstride"], p["prepared"]) == (2, c, 1, 1, 0)
    assert p["W"] == (128 + c - 1) // c
    assert p["buckets"] == p["W"] * (1 << (c - 1))


@pytest.mark.parametrize("log_n,c", [(8, 11), (12, 11), (13, 13), (15, 13), (16, 16), (20, 16)])
def test_g2_plain_bases_take_the_psi_split(amd, log_n, c):
    p = amd.msm_plan("g2", 1 << log_n)
    assert (p["split"], p["c"], p["W"]) == (4, c, (64 + c - 1) // c)


def test_narrow_scalars_and_large_windows_stay_unsplit(amd):
    assert amd.msm_plan("g1", 1 << 16, bitsize=128)["split"] == 1
    assert amd.msm_plan("g2", 1 << 16, bitsize=192)["split"] == 1
    assert amd.msm_plan("g2", 1 << 16, c=18)["split"] == 1  # psi digits need c <= 16
    # a caller's c that leaves the split's top window nearly empty becomes 16
    assert amd.msm_plan("g1", 1 << 20, c=15)["c"] == 16
    assert amd.msm_plan("g1", 1 << 20, c=13)["c"] == 13


@pytest.mark.parametrize("group,F", [("g1", 2), ("g2", 4)])
def test_prepared_tables_take_the_split(amd, group, F):
    for log_n in (8, 16, 20):
        for bits in (0, 64):
            p = amd.msm_plan(group, 1 << log_n, precompute_factor=F, bitsize=bits)
            assert (p["prepared"], p["split"], p["F"], p["bstride"]) == (1, F, 1, 1)
    assert amd.msm_plan("g2", 1 << 16, precompute_factor=4, c=18)["c"] == 16


@pytest.mark.parametrize("F,log_n,c", [(4, 8, 8), (4, 12, 11), (4, 14, 13), (4, 16, 16), (4, 20, 16), (4, 21, 16),
                                       (8, 10, 11), (8, 13, 11), (8, 14, 16), (8, 20, 16),
                                       (16, 8, 8), (16, 10, 16), (16, 19, 16)])
def test_g1_shift_plans_and_windows(amd, F, log_n, c):
    p = amd.msm_plan("g1", 1 << log_n, precompute_factor=F)
    sF = (256 + F - 1) // F
    assert (p["split"], p["F"], p["sF"], p["c"], p["bstride"]) == (1, F, sF, c, 1)
    assert p["Wg"] == (sF + c - 1) // c and p["W"] == F * p["Wg"]


@pytest.mark.parametrize("F,log_n", [(4, 22), (8, 21), (16, 20), (16, 24)])
def test_g1_shift_tables_above_1gib_run_slot0(amd, F, log_n):
    assert (1 << log_n) * F * 96 > 1 << 30
    p = amd.msm_plan("g1", 1 << log_n, precompute_factor=F)
    assert (p["split"], p["bstride"], p["F"], p["c"]) == (2, F, 1, 16)


@pytest.mark.parametrize("group,F", [("g1", 3), ("g1", 5), ("g1", 6), ("g1", 7), ("g1", 32), ("g1", 64),
                                     ("g2", 2), ("g2", 3), ("g2", 5), ("g2", 32)])
def test_other_factors_run_the_split_plan_on_slot0(amd, group, F):
    S = 2 if group == "g1" else 4
    for log_n in (8, 14, 20):
        p = amd.msm_plan(group, 1 << log_n, precompute_factor=F)
        assert (p["split"], p["bstride"], p["F"], p["prepared"]) == (S, F, 1, 0)
        assert p["c"] == amd.msm_plan(group, 1 << log_n)["c"]  # the plain split's window


@pytest.mark.parametrize("F,log_n,c", [(8, 12, 11), (8, 14, 11), (8, 15, 16), (8, 20, 16), (16, 8, 8),
                                       (16, 14, 16)])
def test_g2_shift_plans(amd, F, log_n, c):
    p = amd.msm_plan("g2", 1 << log_n, precompute_factor=F)
    assert (p["split"], p["F"], p["c"], p["bstride"]) == (1, F, c, 1)


def test_plan_argument_errors(amd):
    with pytest.raises(amd.IcicleError):
        amd.msm_plan("g1", 1 << 10, precompute_factor=65)
    with pytest.raises(amd.IcicleError):
        amd.msm_plan("g1", 1 << 10, c=21)
    with pytest.raises(amd.IcicleError):
        amd.msm_plan("g1", 1 << 10, bitsize=257)
