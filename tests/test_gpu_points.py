"""Batch point-form conversions of the reference's C ABI (point_ops.cu:759,844,924) on the GPU,
against the pure-Python restatement (oracle/pyref.py):

* bls12_381_g1_affine_to_projective: Montgomery affine -> (x, y, 1), identity -> (0, 1, 0);
* bls12_381_g1_projective_to_affine / bls12_381_g2_projective_to_affine: Jacobian with random Z
  (x = X / Z^2, y = Y / Z^3) -> affine, Z = 0 -> (0, 0);
* host and device placement, sizes that are not a multiple of the per-thread run, identities
  inside a run, and the reference's argument errors (null, size <= 0) -> INVALID_ARGUMENT."""
import random

import numpy as np
import pytest

import helpers as H
from helpers import pyref as pr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def amd():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import gpu_helpers
    gpu_helpers.amd.lib()
    return gpu_helpers.amd


def _g1_points(n, seed):
    rnd = random.Random(seed)
    base = pr.g1_mul(rnd.randrange(1, pr.R), pr.G1)
    pts, acc = [], base
    for i in range(n):  # consecutive multiples: cheap and all distinct
        pts.append(acc)
        acc = pr.g1_add(acc, base)
    return pts


def _g2_points(n, seed):
    rnd = random.Random(seed)
    base = pr.g2_mul(rnd.randrange(1, pr.R), pr.G2)
    pts, acc = [], base
    for i in range(n):
        pts.append(acc)
        acc = pr.g2_add(acc, base)
    return pts


def _fq_limbs(v):
    return pr.int_to_limbs(pr.fq_to_mont(v % pr.P), 6)


def _g1_jac_mont(pt, z):
    """Jacobian Montgomery limbs of affine std `pt` with Z = z (identity: Z = 0)"""
    if pt is None:
        return _fq_limbs(1) + _fq_limbs(1) + [0] * 6
    x, y = pt
    return _fq_limbs(x * z * z) + _fq_limbs(y * z * z * z) + _fq_limbs(z)


def _g2_jac_mont(pt, z):
    if pt is None:
        return _fq_limbs(1) + [0] * 6 + _fq_limbs(1) + [0] * 6 + [0] * 12
    x, y = pt
    z2 = pr.f2_mul(z, z)
    X, Y = pr.f2_mul(x, z2), pr.f2_mul(y, pr.f2_mul(z2, z))
    out = []
    for v in (X[0], X[1], Y[0], Y[1], z[0], z[1]):
        out += _fq_limbs(v)
    return out


@pytest.mark.parametrize("where", ["host", "device"])
def test_g1_affine_to_projective(amd, where):
    import torch
    pts = _g1_points(37, 1) + [None] + _g1_points(5, 2) + [None]
    aff = np.array([H.g1_affine_mont(p) for p in pts], dtype=np.uint64)
    src = aff if where == "host" else amd.torch_u64(aff)
    out = None if where == "host" else torch.zeros((len(pts), 18), dtype=torch.int64, device="cuda")
    got = amd.convert_points("g1", "to_projective", src, out=out)
    got = got if where == "host" else amd.to_numpy_u64(got)
    one = _fq_limbs(1)
    for i, p in enumerate(pts):
        row = [int(v) for v in got[i]]
        if p is None:  # Projective::identity(): (0, 1, 0) with 1 in Montgomery form
            assert row == [0] * 6 + one + [0] * 6, i
        else:
            assert row == H.g1_affine_mont(p) + one, i


@pytest.mark.parametrize("where", ["host", "device"])
@pytest.mark.parametrize("n", [1, 8, 61])
def test_g1_projective_to_affine(amd, where, n):
    import torch
    rnd = random.Random(n)
    pts = _g1_points(n, 10 + n)
    if n > 2:
        pts[1] = None  # identity inside a run
        pts[-1] = None
    jac = np.array([_g1_jac_mont(p, rnd.randrange(1, pr.P)) for p in pts], dtype=np.uint64)
    src = jac if where == "host" else amd.torch_u64(jac)
    out = None if where == "host" else torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    got = amd.convert_points("g1", "to_affine", src, out=out)
    got = got if where == "host" else amd.to_numpy_u64(got)
    for i, p in enumerate(pts):
        assert [int(v) for v in got[i]] == H.g1_affine_mont(p), i


@pytest.mark.parametrize("n", [3, 29])
def test_g2_projective_to_affine(amd, n):
    rnd = random.Random(100 + n)
    pts = _g2_points(n, 20 + n)
    pts[n // 2] = None
    jac = np.array([_g2_jac_mont(p, (rnd.randrange(pr.P), rnd.randrange(1, pr.P))) for p in pts], dtype=np.uint64)
    got = amd.convert_points("g2", "to_affine", jac)
    for i, p in enumerate(pts):
        assert [int(v) for v in got[i]] == H.g2_affine_mont(p), i


def test_g1_round_trip_generated_bases(amd):
    """2^16 + 5 device-generated bases: affine -> projective -> affine is the identity map"""
    import torch
    n = (1 << 16) + 5
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0E01)
    proj = torch.zeros((n, 18), dtype=torch.int64, device="cuda")
    back = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.convert_points("g1", "to_projective", b, out=proj)
    amd.convert_points("g1", "to_affine", proj, out=back)
    torch.cuda.synchronize()
    assert torch.equal(back, b)


def test_conversion_argument_errors(amd):
    import ctypes
    L = amd.lib()
    cfg = amd.vec_config()
    buf = np.zeros((4, 18), dtype=np.uint64)
    for name in ("bls12_381_g1_affine_to_projective", "bls12_381_g1_projective_to_affine",
                 "bls12_381_g2_projective_to_affine"):
        fn = getattr(L, name)
        assert fn(None, 4, ctypes.byref(cfg), amd._p(buf)) == amd.INVALID_ARGUMENT
        assert fn(amd._p(buf), 0, ctypes.byref(cfg), amd._p(buf)) == amd.INVALID_ARGUMENT
        assert fn(amd._p(buf), -1, ctypes.byref(cfg), amd._p(buf)) == amd.INVALID_ARGUMENT
        assert fn(amd._p(buf), 4, None, amd._p(buf)) == amd.INVALID_ARGUMENT
        assert fn(amd._p(buf), (1 << 26) + 1, ctypes.byref(cfg), amd._p(buf)) == amd.INVALID_ARGUMENT
