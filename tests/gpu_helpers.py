"""Helpers for the -m gpu parity tests: load the HIP binding, decode results."""
import os
import sys

import numpy as np

import helpers as H
from helpers import pyref as pr

PKG = os.path.join(H.ROOT, "midnight-bls12-381-cuda_amd")
sys.path.insert(0, PKG)
import bls12_381_amd as amd  # noqa: E402


def decode_icicle(group, row):
    """ICICLE standard projective (x, y, 1) / identity (0, 1, 0) -> affine std or None"""
    row = [int(v) for v in row]
    if group == "g1":
        x, y, z = (pr.limbs_to_int(row[6 * k:6 * k + 6]) for k in range(3))
        if z == 0:
            assert x == 0 and y == 1, "malformed identity"
            return None
        assert z == 1
        return (x, y)
    c = [pr.limbs_to_int(row[6 * k:6 * k + 6]) for k in range(6)]
    if c[4] == 0 and c[5] == 0:
        assert c[0] == c[1] == 0 and c[2] == 1 and c[3] == 0, "malformed identity"
        return None
    assert c[4] == 1 and c[5] == 0
    return ((c[0], c[1]), (c[2], c[3]))


def decode_jacobian_mont(group, row):
    """Jacobian Montgomery (x = X/Z^2, y = Y/Z^3) -> affine std or None"""
    row = [int(v) for v in row]
    if group == "g1":
        X, Y, Z = (pr.fq_from_mont(pr.limbs_to_int(row[6 * k:6 * k + 6])) for k in range(3))
        if Z == 0:
            return None
        zi = pow(Z, -1, pr.P)
        return ((X * zi * zi) % pr.P, (Y * zi * zi * zi) % pr.P)
    c = [pr.fq_from_mont(pr.limbs_to_int(row[6 * k:6 * k + 6])) for k in range(6)]
    X, Y, Z = (c[0], c[1]), (c[2], c[3]), (c[4], c[5])
    if Z == (0, 0):
        return None
    zi = pr.f2_inv(Z)
    zi2 = pr.f2_mul(zi, zi)
    return (pr.f2_mul(X, zi2), pr.f2_mul(Y, pr.f2_mul(zi2, zi)))


def affine_mont_array(group, pts):
    enc = H.g1_affine_mont if group == "g1" else H.g2_affine_mont
    nl = 12 if group == "g1" else 24
    return np.array([enc(p) for p in pts], dtype=np.uint64).reshape(-1, nl)
