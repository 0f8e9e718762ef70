"""Shared test helpers: fixture loading, limb conversion, oracle loader.

The oracle (oracle/liboracle_bls12_381.so, oracle/pyref.py) is the CHECKER only."""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
ORACLE_DIR = os.path.join(ROOT, "oracle")
sys.path.insert(0, ORACLE_DIR)
sys.path.insert(0, ROOT)

import pyref  # noqa: E402


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def hx(s):
    return None if s is None else int(s, 16)


def ints_to_limbs(vals, nlimbs):
    """list of python ints -> (n, nlimbs) uint64 array"""
    out = np.zeros((len(vals), nlimbs), dtype=np.uint64)
    for i, v in enumerate(vals):
        for j in range(nlimbs):
            out[i, j] = (v >> (64 * j)) & 0xFFFFFFFFFFFFFFFF
    return out


def limbs_to_ints(arr):
    arr = np.asarray(arr, dtype=np.uint64)
    if arr.ndim == 1:
        arr = arr[None, :]
    return [pyref.limbs_to_int([int(x) for x in row]) for row in arr]


# ---- point encodings ----------------------------------------------------------------
def g1_affine_mont(pt):
    """std affine (x, y) or None -> 12 u64 limbs, Montgomery (identity -> zeros)"""
    if pt is None:
        return [0] * 12
    x, y = pt
    return pyref.int_to_limbs(pyref.fq_to_mont(x), 6) + pyref.int_to_limbs(pyref.fq_to_mont(y), 6)


def g2_affine_mont(pt):
    if pt is None:
        return [0] * 24
    (x0, x1), (y0, y1) = pt
    out = []
    for v in (x0, x1, y0, y1):
        out += pyref.int_to_limbs(pyref.fq_to_mont(v), 6)
    return out


def g1_from_affine_mont(limbs):
    limbs = [int(v) for v in limbs]
    if not any(limbs):
        return None
    return (pyref.fq_from_mont(pyref.limbs_to_int(limbs[0:6])),
            pyref.fq_from_mont(pyref.limbs_to_int(limbs[6:12])))


def g2_from_affine_mont(limbs):
    limbs = [int(v) for v in limbs]
    if not any(limbs):
        return None
    c = [pyref.fq_from_mont(pyref.limbs_to_int(limbs[6 * i:6 * i + 6])) for i in range(4)]
    return ((c[0], c[1]), (c[2], c[3]))


def pt_from_json(p, group):
    if p is None:
        return None
    if group == "g1":
        return (hx(p[0]), hx(p[1]))
    return ((hx(p[0][0]), hx(p[0][1])), (hx(p[1][0]), hx(p[1][1])))


# ---- oracle -------------------------------------------------------------------------
_ORACLE = None


def oracle():
    """Load (building if needed) the CPU oracle shared library."""
    global _ORACLE
    if _ORACLE is not None:
        return _ORACLE
    so = os.path.join(ORACLE_DIR, "liboracle_bls12_381.so")
    src = os.path.join(ORACLE_DIR, "bls12_381_oracle.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["make", "-C", ORACLE_DIR, "-s"])
    lib = ctypes.CDLL(so)
    P = ctypes.c_void_p
    sz = ctypes.c_size_t
    for nm in ("orc_fr_mul", "orc_fr_add", "orc_fr_sub", "orc_fq_mul", "orc_g1_add_affine",
               "orc_g2_add_affine"):
        getattr(lib, nm).argtypes = [P, P, P]
    for nm in ("orc_fr_inv", "orc_fr_to_mont", "orc_fr_from_mont", "orc_fq_inv", "orc_fq_to_mont",
               "orc_fq_from_mont", "orc_g1_mul_gen", "orc_g2_mul_gen"):
        getattr(lib, nm).argtypes = [P, P]
    for nm in ("orc_vec_add", "orc_vec_sub", "orc_vec_mul", "orc_scalar_mul_vec", "orc_scalar_add_vec"):
        getattr(lib, nm).argtypes = [P, P, P, sz]
    lib.orc_omega.argtypes = [P, ctypes.c_int]
    lib.orc_ntt.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    for nm in ("orc_g1_msm", "orc_g2_msm", "orc_g1_msm_fast", "orc_g2_msm_fast"):
        getattr(lib, nm).argtypes = [P, P, P, sz, ctypes.c_int]
        getattr(lib, nm).restype = ctypes.c_int
    lib.orc_gen_scalars.argtypes = [P, ctypes.c_uint64, sz]
    lib.orc_set_threads.argtypes = [ctypes.c_int]
    lib.orc_set_threads.restype = None
    lib.orc_max_threads.restype = ctypes.c_int
    for nm in ("orc_gen_g1_bases", "orc_gen_g2_bases"):
        getattr(lib, nm).argtypes = [P, ctypes.c_uint64, sz, ctypes.c_int]
    _ORACLE = lib
    return lib


def ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def oracle_msm(group, scalars_std: np.ndarray, bases_mont: np.ndarray, threads=0, fast=False):
    """fast: the window-parallel XYZZ Pippenger (orc_g*_msm_fast, the bench's CPU baseline) instead of
    the checker's restatement"""
    lib = oracle()
    n = scalars_std.shape[0]
    out = np.zeros(12 if group == "g1" else 24, dtype=np.uint64)
    if fast:
        fn = lib.orc_g1_msm_fast if group == "g1" else lib.orc_g2_msm_fast
    else:
        fn = lib.orc_g1_msm if group == "g1" else lib.orc_g2_msm
    fn(ptr(out), ptr(np.ascontiguousarray(scalars_std)), ptr(np.ascontiguousarray(bases_mont)), n, threads)
    return out


def oracle_ntt(data_mont: np.ndarray, log_n: int, inverse: bool, threads=0):
    a = np.ascontiguousarray(data_mont.copy())
    oracle().orc_ntt(ptr(a), log_n, 1 if inverse else 0, threads)
    return a


def glv_edge_scalars():
    """scalars on the GLV split's balancing boundaries (k1, k2 around lam/2, lam, lam + 1)"""
    lam, h = pyref.GLV_LAMBDA, pyref.GLV_LAMBDA >> 1
    out = [0, 1, 2, pyref.R - 1, pyref.R - 2, h, h + 1, lam - 1, lam, lam + 1, lam * lam, lam * lam + lam,
           (h + 1) * lam, h * lam + h, h * lam + h + 1, (h + 1) * lam + h + 1, (h + 2) * lam - 1, (lam + 1) * lam - 1,
           lam * lam + lam - 1, (1 << 254), (1 << 255) - 1]
    return [s % pyref.R for s in out]


def psi_edge_scalars():
    """scalars on the G2 psi split's boundaries: base-|z| digits at 0, x/2, x/2 + 1, x - 1, the
    folded fifth digit (s >= x^4 - ... near r), and powers of x"""
    x, h = pyref.PSI_X, pyref.PSI_X >> 1
    out = [0, 1, 2, pyref.R - 1, pyref.R - 2, h, h + 1, x - 1, x, x + 1, x * x, x ** 3, x ** 3 - 1,
           h * (1 + x + x * x + x ** 3), (h + 1) * (1 + x + x * x + x ** 3), (x - 1) * (1 + x + x * x),
           pyref.R - x ** 3, pyref.R - h * x ** 3, (1 << 254), (1 << 255) - 1]
    return [s % pyref.R for s in out]
