"""Parity of the HIP path (through the C ABI) against the oracle and the golden fixtures.
Bit-exact for everything (integer arithmetic).  Run with -m gpu on an MI355X."""
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


@pytest.fixture(scope="module")
def gh():
    import gpu_helpers
    return gpu_helpers


# ----------------------------------------------------------------------------- vecops
@pytest.mark.parametrize("op", ["add", "sub", "mul", "scalar_mul", "scalar_add"])
def test_vecops_golden_host(amd, op):
    g = H.load_golden("vecops.json")
    a = H.ints_to_limbs([H.hx(x) for x in g["a"]], 4)
    b = H.ints_to_limbs([H.hx(x) for x in g["b"]], 4)
    s = H.ints_to_limbs([H.hx(g["scalar"])], 4)[0]
    out = amd.vec_op(op, s if op.startswith("scalar") else a, b)
    assert H.limbs_to_ints(out) == [H.hx(x) for x in g[op]]


@pytest.mark.parametrize("op", ["add", "sub", "mul"])
def test_vecops_device_2_16_vs_oracle(amd, op):
    import torch
    n = 1 << 16
    a = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    b = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(a, 0x5EED0001, montgomery=True)
    amd.gen_scalars(b, 0x5EED0101, montgomery=True)
    out = torch.zeros_like(a)
    amd.vec_op(op, a, b, out=out)
    torch.cuda.synchronize()
    an, bn = amd.to_numpy_u64(a), amd.to_numpy_u64(b)
    ref = np.zeros_like(an)
    fn = {"add": H.oracle().orc_vec_add, "sub": H.oracle().orc_vec_sub, "mul": H.oracle().orc_vec_mul}[op]
    fn(H.ptr(ref), H.ptr(an), H.ptr(bn), n)
    assert np.array_equal(amd.to_numpy_u64(out), ref)


def test_vecops_raw_entry_points(amd):
    import ctypes
    import torch
    g = H.load_golden("vecops.json")
    a = H.ints_to_limbs([H.hx(x) for x in g["a"]], 4)
    b = H.ints_to_limbs([H.hx(x) for x in g["b"]], 4)
    s = np.ascontiguousarray(H.ints_to_limbs([H.hx(g["scalar"])], 4)[0])
    da, db = amd.torch_u64(a), amd.torch_u64(b)
    out = torch.zeros_like(da)
    cfg = amd.vec_config(is_a_on_device=True, is_b_on_device=True, is_result_on_device=True)
    L = amd.lib()
    n = a.shape[0]
    for name, key, first in [("vec_add_cuda", "add", da), ("vec_sub_cuda", "sub", da), ("vec_mul_cuda", "mul", da),
                             ("scalar_mul_vec_cuda", "scalar_mul", s), ("scalar_add_vec_cuda", "scalar_add", s)]:
        amd.check(getattr(L, name)(amd._p(out), amd._p(first), amd._p(db), n, ctypes.byref(cfg)), name)
        torch.cuda.synchronize()
        assert H.limbs_to_ints(amd.to_numpy_u64(out)) == [H.hx(x) for x in g[key]], name


def test_vecops_empty_and_errors(amd):
    z = np.zeros((0, 4), dtype=np.uint64)
    out = amd.vec_op("add", z, z)
    assert out.shape == (0, 4)
    with pytest.raises(amd.IcicleError) as e:
        amd.check(amd.lib().bls12_381_vector_add(None, None, 4, None, None), "null")
    assert e.value.code == amd.INVALID_POINTER


def _bitrev_perm(log_n):
    n = 1 << log_n
    return np.array([int(format(i, f"0{log_n}b")[::-1], 2) if log_n else 0 for i in range(n)], dtype=np.int64)


@pytest.mark.parametrize("columns", [False, True])
def test_vecops_batched_scalar_ops(amd, columns):
    """ICICLE v4 batch: one scalar per member, row or columns_batch layout; host and device scalars"""
    import torch
    n, batch = 1000, 3
    g = pr.rng(17)
    vals = [g.randrange(pr.R) for _ in range(n * batch)]
    sc = [g.randrange(pr.R) for _ in range(batch)]
    b = H.ints_to_limbs(vals, 4)
    s = H.ints_to_limbs(sc, 4)
    member = [(i % batch) if columns else (i // n) for i in range(n * batch)]
    for op, fn in (("scalar_mul", lambda x, y: pr.fr_mont_mul(x, y)), ("scalar_add", lambda x, y: (x + y) % pr.R)):
        expect = [fn(sc[member[i]], v) for i, v in enumerate(vals)]
        out = amd.vec_op(op, s, b, batch=batch, columns_batch=columns)
        assert H.limbs_to_ints(out) == expect, op
        out_d = torch.zeros((n * batch, 4), dtype=torch.int64, device="cuda")
        amd.vec_op(op, amd.torch_u64(s), amd.torch_u64(b), out=out_d, batch=batch, columns_batch=columns)
        torch.cuda.synchronize()
        assert H.limbs_to_ints(amd.to_numpy_u64(out_d)) == expect, op


@pytest.mark.parametrize("n", [1, 5, 256, 1000, 1 << 16])
def test_vec_sum(amd, n):
    g = pr.rng(n)
    vals = [g.randrange(pr.R) for _ in range(n)]
    out = amd.vec_sum(amd.torch_u64(H.ints_to_limbs(vals, 4)))
    assert H.limbs_to_ints(out)[0] == sum(vals) % pr.R


@pytest.mark.parametrize("n", [1, 63, 64, 65, 4097])
def test_batch_inv(amd, n):
    """Montgomery-form inverses (x R -> x^-1 R), zeros map to zero; out of place and in place"""
    import torch
    g = pr.rng(100 + n)
    xs = [g.randrange(pr.R) for _ in range(n)]
    for k in range(0, n, 7):
        xs[k] = 0
    mont = [pr.fr_to_mont(v) for v in xs]
    expect = [pr.fr_to_mont(pow(v, -1, pr.R)) if v else 0 for v in xs]
    x = amd.torch_u64(H.ints_to_limbs(mont, 4))
    out = torch.zeros_like(x)
    amd.batch_inv(x, out)
    torch.cuda.synchronize()
    assert H.limbs_to_ints(amd.to_numpy_u64(out)) == expect
    amd.batch_inv(x, x)
    torch.cuda.synchronize()
    assert H.limbs_to_ints(amd.to_numpy_u64(x)) == expect


# ----------------------------------------------------------------------------- NTT
@pytest.mark.parametrize("ordering", ["NN", "NR", "RN", "RR", "NM", "MN"])
def test_ntt_orderings(amd, ordering):
    """R (and M, defined as bit-reversed) on the input and/or output side, both directions"""
    amd.ntt_init_domain()
    log_n = 9
    n = 1 << log_n
    g = pr.rng(31)
    x = H.ints_to_limbs([pr.fr_to_mont(g.randrange(pr.R)) for _ in range(n)], 4)
    rev = _bitrev_perm(log_n)
    in_rev = ordering[0] in "RM"
    out_rev = ordering[1] in "RM"
    for inverse in (False, True):
        got = amd.ntt(x[rev] if in_rev else x, inverse=inverse, ordering=ordering)
        ref = H.oracle_ntt(x, log_n, inverse)
        assert np.array_equal(got, ref[rev] if out_rev else ref), (ordering, inverse)
    # NR forward then RN inverse round-trips without any explicit permutation
    y = amd.ntt(x, ordering="NR")
    assert np.array_equal(amd.ntt(y, inverse=True, ordering="RN"), x)


@pytest.mark.parametrize("ordering", ["NN", "RR"])
def test_ntt_columns_batch(amd, ordering):
    """columns_batch: element i of polynomial b at i*batch + b (host and device buffers)"""
    import torch
    amd.ntt_init_domain()
    log_n, batch = 8, 3
    n = 1 << log_n
    g = pr.rng(41)
    polys = [H.ints_to_limbs([pr.fr_to_mont(g.randrange(pr.R)) for _ in range(n)], 4) for _ in range(batch)]
    rev = _bitrev_perm(log_n)
    r = ordering == "RR"
    inter = np.stack([p[rev] if r else p for p in polys], axis=1).reshape(n * batch, 4)
    for inverse in (False, True):
        expect = np.stack([(lambda o: o[rev] if r else o)(H.oracle_ntt(p, log_n, inverse)) for p in polys],
                          axis=1).reshape(n * batch, 4)
        got = amd.ntt(np.ascontiguousarray(inter), inverse=inverse, batch=batch, ordering=ordering, columns_batch=True)
        assert np.array_equal(got, expect), inverse
        d = amd.torch_u64(np.ascontiguousarray(inter))
        amd.ntt(d, inverse=inverse, out=d, batch=batch, ordering=ordering, columns_batch=True)  # in place
        torch.cuda.synchronize()
        assert np.array_equal(amd.to_numpy_u64(d), expect), inverse


def test_ntt_golden(amd):
    amd.ntt_init_domain()
    g = H.load_golden("ntt.json")
    for case in g["cases"]:
        x = H.ints_to_limbs([H.hx(v) for v in case["input"]], 4)
        fwd = amd.ntt(x, inverse=False)
        inv = amd.ntt(x, inverse=True)
        assert H.limbs_to_ints(fwd) == [H.hx(v) for v in case["forward"]], case["name"]
        assert H.limbs_to_ints(inv) == [H.hx(v) for v in case["inverse"]], case["name"]


@pytest.mark.parametrize("log_n", [11, 12, 15, 17, 20])
def test_ntt_vs_oracle(amd, log_n):
    import torch
    amd.ntt_init_domain()
    n = 1 << log_n
    x = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(x, 0x5EED0002 + log_n, montgomery=True)
    y = torch.zeros_like(x)
    amd.ntt(x, inverse=False, out=y)
    z = torch.zeros_like(x)
    amd.ntt(y, inverse=True, out=z)
    torch.cuda.synchronize()
    xn = amd.to_numpy_u64(x)
    ref = H.oracle_ntt(xn, log_n, False)
    assert np.array_equal(amd.to_numpy_u64(y), ref)
    assert np.array_equal(amd.to_numpy_u64(z), xn)  # exact round trip


@pytest.mark.parametrize("log_n", [23, 24])
def test_ntt_past_init_tables_vs_oracle(amd, log_n):
    """sizes above the 2^22 stage tables built at init_domain: the tables are extended on first
    use (ntt.hip build_domain); forward against the oracle's best_fft DFT, exact round trip, and
    (2^24) a forward-NTT linearity check; three 8-stage passes"""
    import torch
    amd.ntt_init_domain()
    n = 1 << log_n
    x = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(x, 0x5EED0060 + log_n, montgomery=True)
    y = torch.zeros_like(x)
    amd.ntt(x, inverse=False, out=y)
    z = torch.zeros_like(x)
    amd.ntt(y, inverse=True, out=z)
    torch.cuda.synchronize()
    xn = amd.to_numpy_u64(x)
    assert np.array_equal(amd.to_numpy_u64(z), xn)  # exact round trip
    # forward output against the oracle's best_fft at both sizes (2^24: ~2 s on 16 host threads)
    assert np.array_equal(amd.to_numpy_u64(y), H.oracle_ntt(xn, log_n, False, threads=16))
    if log_n == 24:
        # NTT(x + x) == NTT(x) + NTT(x): the sum through vec add (both canonical Montgomery)
        xx = torch.zeros_like(x)
        amd.vec_op("add", x, x, out=xx)
        yy = torch.zeros_like(x)
        amd.ntt(xx, inverse=False, out=yy)
        y2 = torch.zeros_like(x)
        amd.vec_op("add", y, y, out=y2)
        torch.cuda.synchronize()
        assert torch.equal(yy, y2)
    del x, y, z


def test_ntt_batch_and_inplace(amd):
    import torch
    amd.ntt_init_domain()
    log_n, batch = 10, 5
    n = 1 << log_n
    x = torch.zeros((n * batch, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(x, 77, montgomery=True)
    xn = amd.to_numpy_u64(x)
    y = x.clone()
    amd.ntt(y, inverse=False, out=y, batch=batch)  # in place
    torch.cuda.synchronize()
    yn = amd.to_numpy_u64(y)
    for b in range(batch):
        assert np.array_equal(yn[b * n:(b + 1) * n], H.oracle_ntt(xn[b * n:(b + 1) * n], log_n, False))


def test_ntt_coset(amd):
    amd.ntt_init_domain()
    g = pr.rng(5)
    n = 64
    xs = [g.randrange(pr.R) for _ in range(n)]
    gen = 7
    x = H.ints_to_limbs([pr.fr_to_mont(v) for v in xs], 4)
    gm = np.array(pr.int_to_limbs(pr.fr_to_mont(gen), 4), dtype=np.uint64)
    fwd = amd.ntt(x, inverse=False, coset_gen=gm)
    expect = pr.ntt_forward([(v * pow(gen, i, pr.R)) % pr.R for i, v in enumerate(xs)])
    assert [pr.fr_from_mont(v) for v in H.limbs_to_ints(fwd)] == expect
    back = amd.ntt(fwd, inverse=True, coset_gen=gm)
    assert np.array_equal(back, x)


def test_ntt_rejects_bad_sizes(amd):
    amd.ntt_init_domain()
    x = np.zeros((12, 4), dtype=np.uint64)
    with pytest.raises(amd.IcicleError) as e:
        amd.ntt(x)
    assert e.value.code == amd.INVALID_ARGUMENT


# ----------------------------------------------------------------------------- MSM
def _case_arrays(gh, case, group):
    sc = [H.hx(s) for s in case["scalars"]]
    pts = [H.pt_from_json(b, group) for b in case["bases"]]
    n = len(sc)
    s_std = H.ints_to_limbs(sc, 4) if n else np.zeros((0, 4), dtype=np.uint64)
    s_mont = H.ints_to_limbs([pr.fr_to_mont(s) for s in sc], 4) if n else np.zeros((0, 4), dtype=np.uint64)
    nl = 12 if group == "g1" else 24
    b_mont = gh.affine_mont_array(group, pts) if n else np.zeros((0, nl), dtype=np.uint64)
    return s_std, s_mont, b_mont


@pytest.mark.parametrize("group", ["g1", "g2"])
def test_msm_golden_icicle_semantics(amd, gh, group):
    g = H.load_golden(f"msm_{group}.json")
    for case in g["cases"]:
        s_std, s_mont, b_mont = _case_arrays(gh, case, group)
        expect = H.pt_from_json(case["result"], group)
        r1 = amd.msm(group, s_mont, b_mont, icicle=True, scalars_mont=True, n=len(case["scalars"]))
        assert gh.decode_icicle(group, r1[0]) == expect, case["name"]
        r2 = amd.msm(group, s_std, b_mont, icicle=True, scalars_mont=False, n=len(case["scalars"]))
        assert gh.decode_icicle(group, r2[0]) == expect, case["name"]


@pytest.mark.parametrize("group", ["g1", "g2"])
def test_msm_golden_raw_entry(amd, gh, group):
    g = H.load_golden(f"msm_{group}.json")
    for case in g["cases"]:
        s_std, _, b_mont = _case_arrays(gh, case, group)
        r = amd.msm(group, s_std, b_mont, icicle=False, n=len(case["scalars"]))
        assert gh.decode_jacobian_mont(group, r[0]) == H.pt_from_json(case["result"], group), case["name"]


def test_msm_window_sizes(amd, gh):
    g = H.load_golden("msm_g1.json")
    case = [c for c in g["cases"] if c["name"] == "random_300"][0]
    s_std, _, b_mont = _case_arrays(gh, case, "g1")
    expect = H.pt_from_json(case["result"], "g1")
    for c in (2, 5, 8, 11, 13, 14, 15, 16, 18):  # 14 / 15 / 18 run as 16 with the GLV split
        r = amd.msm("g1", s_std, b_mont, c=c)
        assert gh.decode_icicle("g1", r[0]) == expect, c
    # c > 16 without a split (G2 keeps the plain 255-bit digits there): the digit + scatter sort
    g2 = H.load_golden("msm_g2.json")
    case2 = [c for c in g2["cases"] if c["name"] == "random_64"][0]
    s2, _, b2 = _case_arrays(gh, case2, "g2")
    expect2 = H.pt_from_json(case2["result"], "g2")
    for c in (15, 17, 18):
        r = amd.msm("g2", s2, b2, c=c)
        assert gh.decode_icicle("g2", r[0]) == expect2, c


def test_msm_points_standard_form(amd, gh):
    g = H.load_golden("msm_g1.json")
    case = [c for c in g["cases"] if c["name"] == "random_100"][0]
    s_std, _, _ = _case_arrays(gh, case, "g1")
    pts = [H.pt_from_json(b, "g1") for b in case["bases"]]
    b_std = np.array([pr.int_to_limbs(p[0], 6) + pr.int_to_limbs(p[1], 6) for p in pts], dtype=np.uint64)
    r = amd.msm("g1", s_std, b_std, points_mont=False)
    assert gh.decode_icicle("g1", r[0]) == H.pt_from_json(case["result"], "g1")


def test_generated_inputs_match_oracle(amd, gh):
    import torch
    n = 257
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0003)
    b1 = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b1, 0x5EED0013)
    b2 = torch.zeros((64, 24), dtype=torch.int64, device="cuda")
    amd.gen_bases("g2", b2, 0x5EED0015)
    torch.cuda.synchronize()
    o = H.oracle()
    rs = np.zeros((n, 4), dtype=np.uint64)
    o.orc_gen_scalars(H.ptr(rs), 0x5EED0003, n)
    r1 = np.zeros((n, 12), dtype=np.uint64)
    o.orc_gen_g1_bases(H.ptr(r1), 0x5EED0013, n, 0)
    r2 = np.zeros((64, 24), dtype=np.uint64)
    o.orc_gen_g2_bases(H.ptr(r2), 0x5EED0015, 64, 0)
    assert np.array_equal(amd.to_numpy_u64(s), rs)
    assert np.array_equal(amd.to_numpy_u64(b1), r1)
    assert np.array_equal(amd.to_numpy_u64(b2), r2)


@pytest.mark.parametrize("log_n", [10, 14, 16])
def test_msm_g1_device_vs_oracle(amd, gh, log_n):
    import torch
    n = 1 << log_n
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0003 + log_n, montgomery=True)
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0013 + log_n)
    out = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
    amd.msm("g1", s, b, scalars_mont=True, out=out)
    torch.cuda.synchronize()
    s_std = np.zeros((n, 4), dtype=np.uint64)
    H.oracle().orc_gen_scalars(H.ptr(s_std), 0x5EED0003 + log_n, n)
    ref = H.oracle_msm("g1", s_std, amd.to_numpy_u64(b))
    assert gh.decode_icicle("g1", amd.to_numpy_u64(out)[0]) == H.g1_from_affine_mont(ref)


@pytest.mark.parametrize("c", [0, 15])
def test_msm_adversarial_heavy_buckets(amd, gh, c):
    """all scalars equal (every window's contributions land in ONE bucket) and c = 15 (whose
    top window holds only carries): heavy buckets must still reduce exactly."""
    import torch
    n = 1 << 13
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 99)
    s_one = H.ints_to_limbs([pr.R - 12345] * n, 4)
    out = amd.msm("g1", amd.torch_u64(s_one), b, icicle=True, c=c, n=n)
    bn = amd.to_numpy_u64(b)
    ref = H.oracle_msm("g1", s_one, bn)
    assert gh.decode_icicle("g1", out[0]) == H.g1_from_affine_mont(ref)
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 1234)
    out = amd.msm("g1", s, b, icicle=True, c=c, n=n)
    ref = H.oracle_msm("g1", amd.to_numpy_u64(s), bn)
    assert gh.decode_icicle("g1", out[0]) == H.g1_from_affine_mont(ref)


def test_msm_g2_heavy_buckets_raw_xyzz_level0(amd, gh):
    """G2 at c = 16 (4 psi windows of 2^15 buckets: reduction level 0 in lanes, so the bucket sums
    stay raw pair-sliced XYZZ): all scalars equal (one heavy bucket per window, summed by slice
    workgroups and converted from the row layout) and random scalars (light buckets), vs the oracle."""
    import torch
    n = 1 << 12
    b = torch.zeros((n, 24), dtype=torch.int64, device="cuda")
    amd.gen_bases("g2", b, 77)
    bn = amd.to_numpy_u64(b)
    s_one = H.ints_to_limbs([pr.R - 54321] * n, 4)
    out = amd.msm("g2", amd.torch_u64(s_one), b, icicle=True, c=16, n=n)
    assert gh.decode_icicle("g2", out[0]) == H.g2_from_affine_mont(H.oracle_msm("g2", s_one, bn))
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 4321)
    out = amd.msm("g2", s, b, icicle=True, c=16, n=n)
    assert gh.decode_icicle("g2", out[0]) == H.g2_from_affine_mont(H.oracle_msm("g2", amd.to_numpy_u64(s), bn))


@pytest.mark.parametrize("group", ["g1", "g2"])
def test_msm_chunk_start_exceptional_pairs(amd, gh, group):
    """the accumulation adds a chunk's second point with the affine + affine formula (its first
    point left the accumulator at Z = 1): equal points (doubling), opposite points (identity) and
    identity bases must reach that step.  All bases equal (every chunk opens with P + P), +-P
    alternating with equal scalars (P + (-P)), and a pattern with identities, vs the oracle."""
    import torch
    n = 4096
    nl = 12 if group == "g1" else 24
    one = torch.zeros((1, nl), dtype=torch.int64, device="cuda")
    amd.gen_bases(group, one, 4242)
    pt = amd.to_numpy_u64(one)[0]
    half = nl // 2
    y = pr.limbs_to_int([int(v) for v in pt[half:half + 6]])
    neg = pt.copy()
    neg[half:half + 6] = pr.int_to_limbs((pr.P - y) % pr.P, 6)
    if group == "g2":  # y = (y0, y1): negate both components
        y1 = pr.limbs_to_int([int(v) for v in pt[half + 6:]])
        neg[half + 6:] = pr.int_to_limbs((pr.P - y1) % pr.P, 6)
    zero = np.zeros(nl, dtype=np.uint64)
    rnd = np.random.default_rng(11)
    s_rand = H.ints_to_limbs([int(rnd.integers(1, 2 ** 62)) * int(rnd.integers(1, 2 ** 62)) * int(rnd.integers(1, 2 ** 62)) % pr.R
                              for _ in range(n)], 4)
    s_same = H.ints_to_limbs([pr.R - 77777] * n, 4)
    cases = [
        ("all equal", np.tile(pt, (n, 1)), s_rand),
        ("+-P alternating, equal scalars", np.stack([pt if i % 2 == 0 else neg for i in range(n)]), s_same),
        ("P, P, identity, -P pattern", np.stack([(pt, pt, zero, neg)[i % 4] for i in range(n)]), s_rand),
    ]
    for name, bases, scal in cases:
        bases = np.ascontiguousarray(bases.astype(np.uint64))
        out = amd.msm(group, amd.torch_u64(scal), amd.torch_u64(bases), icicle=True, n=n)
        ref = H.oracle_msm(group, scal, bases)
        want = H.g1_from_affine_mont(ref) if group == "g1" else H.g2_from_affine_mont(ref)
        assert gh.decode_icicle(group, out[0]) == want, name


def test_msm_precompute_factor(amd, gh):
    g = H.load_golden("msm_g1.json")
    case = [c for c in g["cases"] if c["name"] == "random_300"][0]
    s_std, _, b_mont = _case_arrays(gh, case, "g1")
    n = s_std.shape[0]
    expect = H.pt_from_json(case["result"], "g1")
    for c, factor in [(8, 2), (8, 4), (10, 26), (13, 5), (3, 64)]:
        pre = amd.precompute_bases("g1", b_mont, factor, n, c=c)
        r = amd.msm("g1", s_std, pre, c=c, precompute_factor=factor, n=n)
        assert gh.decode_icicle("g1", r[0]) == expect, (c, factor)


@pytest.mark.parametrize("group", ["g1", "g2"])
def test_msm_precompute_replays_rust_caller(amd, gh, group):
    """core/msm.rs flag for flag: precompute_bases (:441-454: c = 0, bases Montgomery, factor
    1..8) once over the whole base set, then msm_with_device_bases (:630-650): host scalars in
    Montgomery form, the FULL precomputed buffer, are_bases_montgomery_form = !is_precomputed()
    (false for a table), c = MIDNIGHT_MSM_WINDOW (0 = auto) and msm_size <= bases_size.  The
    table's shift depends on the factor only, so every c / msm_size must give the oracle's sum."""
    import torch
    nb, n = (3000, 2500) if group == "g1" else (700, 600)
    w = 12 if group == "g1" else 24
    b = torch.zeros((nb, w), dtype=torch.int64, device="cuda")
    amd.gen_bases(group, b, 0x5EED00C1)
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED00C2, montgomery=False)
    sm = torch.zeros_like(s)
    amd.gen_scalars(sm, 0x5EED00C2, montgomery=True)  # same stream, Montgomery form (host copy below)
    torch.cuda.synchronize()
    s_std, s_mont = amd.to_numpy_u64(s), np.ascontiguousarray(amd.to_numpy_u64(sm))
    bn = amd.to_numpy_u64(b)
    ref = H.oracle_msm(group, s_std, np.ascontiguousarray(bn[:n]))
    dec = H.g1_from_affine_mont if group == "g1" else H.g2_from_affine_mont
    for factor in (1, 2, 3, 4, 8) if group == "g1" else (1, 4, 7):
        table = torch.zeros((nb * factor, w), dtype=torch.int64, device="cuda")
        amd.precompute_bases(group, b, factor, nb, c=0, out=table)  # core/msm.rs:451: cfg.c = 0
        for c in (0, 11, 16):
            r = amd.msm(group, s_mont, table, scalars_mont=True, points_mont=(factor == 1), c=c,
                        precompute_factor=factor, n=n)
            assert gh.decode_icicle(group, r[0]) == dec(ref), (factor, c)
    # standard-form input to the precompute is converted (the output is always Montgomery)
    pts_std = np.ascontiguousarray(bn.copy())
    for k in range(pts_std.shape[0]):
        pts_std[k] = [v for fq in range(w // 6) for v in pr.int_to_limbs(pr.fq_from_mont(pr.limbs_to_int(
            [int(x) for x in bn[k, 6 * fq:6 * fq + 6]])), 6)]
    table = amd.precompute_bases(group, pts_std, 2, nb, points_mont=False)
    r = amd.msm(group, s_std, table, points_mont=False, precompute_factor=2, n=n)
    assert gh.decode_icicle(group, r[0]) == dec(ref)


def test_msm_batch(amd, gh):
    g = H.load_golden("msm_g1.json")
    cases = [c for c in g["cases"] if c["name"] in ("random_16", "max_digit_patterns")]
    # shared bases: same bases, different scalars
    base_case = [c for c in g["cases"] if c["name"] == "random_16"][0]
    s_std, _, b_mont = _case_arrays(gh, base_case, "g1")
    n = s_std.shape[0]
    rng = pr.rng(11)
    batches = [s_std] + [H.ints_to_limbs([rng.randrange(pr.R) for _ in range(n)], 4) for _ in range(3)]
    allsc = np.ascontiguousarray(np.concatenate(batches))
    r = amd.msm("g1", allsc, b_mont, batch=4, n=n)
    pts = [H.pt_from_json(p, "g1") for p in base_case["bases"]]
    for k in range(4):
        expect = pr.msm_shared_doubling(H.limbs_to_ints(batches[k]), pts)
        assert gh.decode_icicle("g1", r[k]) == expect, k
    assert cases


@pytest.mark.parametrize("group,shared,log_n,batch", [("g1", True, 12, 5), ("g1", False, 12, 5), ("g2", True, 12, 5),
                                                     ("g1", True, 16, 7), ("g2", False, 14, 4)])
def test_msm_batch_pipelined_device(amd, gh, group, shared, log_n, batch):
    """batch members run on pipeline streams (member b's front beside member b - 1's
    accumulation, its tail beside member b + 1's; two scratch regions reused every other member):
    each member equals the single-MSM result (itself pinned to the oracle), device-resident
    operands, odd and even batch sizes, shared and per-member bases, G1 at the production window
    size (2^16: c = 16, the fused chunk counts)"""
    import torch
    n = 1 << log_n
    w = 12 if group == "g1" else 24
    s = torch.zeros((batch * n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED00B0, montgomery=True)
    nb = n if shared else n * batch
    b = torch.zeros((nb, w), dtype=torch.int64, device="cuda")
    amd.gen_bases(group, b, 0x5EED00B1)
    out = torch.zeros((batch, w * 3 // 2), dtype=torch.int64, device="cuda")
    amd.msm(group, s, b, scalars_mont=True, batch=batch, shared_bases=shared, out=out, n=n)
    torch.cuda.synchronize()
    got = amd.to_numpy_u64(out)
    for k in range(batch):
        bk = b if shared else b[k * n:(k + 1) * n]
        one = amd.msm(group, s[k * n:(k + 1) * n], bk, scalars_mont=True, n=n)
        assert gh.decode_icicle(group, got[k]) == gh.decode_icicle(group, one[0]), k


def test_msm_sum_jacobian_and_convert(amd, gh):
    import torch
    # partial results of a split MSM summed on device == full MSM (the multi-GPU reduction)
    g = H.load_golden("msm_g1.json")
    case = [c for c in g["cases"] if c["name"] == "random_300"][0]
    s_std, _, b_mont = _case_arrays(gh, case, "g1")
    parts = torch.zeros((3, 18), dtype=torch.int64, device="cuda")
    for k, (lo, hi) in enumerate([(0, 100), (100, 230), (230, 300)]):
        r = amd.msm("g1", np.ascontiguousarray(s_std[lo:hi]), np.ascontiguousarray(b_mont[lo:hi]), icicle=False)
        parts[k] = amd.torch_u64(r[0])
    tot = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
    amd.sum_jacobian("g1", parts, tot)
    amd.jacobian_to_icicle("g1", tot)
    torch.cuda.synchronize()
    assert gh.decode_icicle("g1", amd.to_numpy_u64(tot)[0]) == H.pt_from_json(case["result"], "g1")


def test_msm_glv_split_boundaries(amd, gh):
    """G1 runs the GLV split (phi(P) = lam P, half-width digits): scalars on its balancing
    boundaries, full-width and <= 128-bit (bitsize 128 keeps the plain path) against the oracle"""
    import torch
    edge = H.glv_edge_scalars()
    g = pr.rng(21)
    sc = edge + [g.randrange(pr.R) for _ in range(64 - len(edge))]
    n = len(sc)
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 77)
    bn = amd.to_numpy_u64(b)
    s = H.ints_to_limbs(sc, 4)
    ref = H.g1_from_affine_mont(H.oracle_msm("g1", s, bn))
    for c in (0, 4, 9, 16):
        r = amd.msm("g1", s, bn, c=c, n=n)
        assert gh.decode_icicle("g1", r[0]) == ref, c
    small = H.ints_to_limbs([x % (1 << 128) for x in sc], 4)
    ref = H.g1_from_affine_mont(H.oracle_msm("g1", small, bn))
    r = amd.msm("g1", small, bn, bitsize=128, n=n)
    assert gh.decode_icicle("g1", r[0]) == ref


def test_msm_psi_split_boundaries(amd, gh):
    """G2 runs the psi split (psi = [z], four quarter-width digit streams): scalars on its
    balancing boundaries, full-width and <= 192-bit (bitsize 192 keeps the plain path) against
    the oracle, through both entry points"""
    import torch
    edge = H.psi_edge_scalars()
    g = pr.rng(22)
    sc = edge + [g.randrange(pr.R) for _ in range(48 - len(edge))]
    n = len(sc)
    b = torch.zeros((n, 24), dtype=torch.int64, device="cuda")
    amd.gen_bases("g2", b, 78)
    bn = amd.to_numpy_u64(b)
    s = H.ints_to_limbs(sc, 4)
    ref = H.g2_from_affine_mont(H.oracle_msm("g2", s, bn))
    for c in (0, 5, 13, 16):
        r = amd.msm("g2", s, bn, c=c, n=n)
        assert gh.decode_icicle("g2", r[0]) == ref, c
    r = amd.msm("g2", s, bn, icicle=False, n=n)
    assert gh.decode_jacobian_mont("g2", r[0]) == ref
    small = H.ints_to_limbs([x % (1 << 192) for x in sc], 4)
    ref = H.g2_from_affine_mont(H.oracle_msm("g2", small, bn))
    r = amd.msm("g2", small, bn, bitsize=192, n=n)
    assert gh.decode_icicle("g2", r[0]) == ref


@pytest.mark.parametrize("group", ["g1", "g2"])
def test_msm_noncanonical_scalars(amd, gh, group):
    """Standard-form scalars >= r.  The reference's raw entry digitises all
    256 bits (msm_kernels.cu:86-142, W = ceil(256 / c) at :648), so any 32-byte s gives s P, and
    its MSM test plan lists scalars >= the modulus (test_msm_security.cu:48).  Every plan the
    library has -- GLV / psi split (per-call images and prepared tables), shift tables, the split
    on slot 0 of a table, c > 16, a batch -- through the raw entry and the ICICLE entry with
    are_scalars_montgomery_form = false, against the oracle's 256-bit Pippenger (and pyref, which
    reduces mod r).  Montgomery scalars: any 32-byte word string x stands for x R^-1 mod r."""
    import torch
    R = pr.R
    g = pr.rng(91 if group == "g1" else 92)
    odd = [R, R + 1, R + 5, 2 * R - 1, 2 * R, 2 * R + 1, (1 << 255), (1 << 255) + 3, (1 << 256) - 1,
           (1 << 256) - R, (1 << 256) - 2, 3 * R - (1 << 256) + R]
    odd += [g.randrange(R, 1 << 256) for _ in range(20)]
    edge = H.glv_edge_scalars() if group == "g1" else H.psi_edge_scalars()
    sc = odd + [e + R for e in edge if e + R < (1 << 256)] + [g.randrange(R) for _ in range(24)]
    n = len(sc)
    w, split = (12, 2) if group == "g1" else (24, 4)
    b = torch.zeros((n, w), dtype=torch.int64, device="cuda")
    amd.gen_bases(group, b, 0x5EED0E01 if group == "g1" else 0x5EED0E02)
    b[1] = b[0]  # equal points: exceptional additions inside a bucket
    bn = amd.to_numpy_u64(b)
    s = H.ints_to_limbs(sc, 4)
    dec = H.g1_from_affine_mont if group == "g1" else H.g2_from_affine_mont
    ref = dec(H.oracle_msm(group, s, bn))
    assert ref == dec(H.oracle_msm(group, H.ints_to_limbs([x % R for x in sc], 4), bn))
    if group == "g1":  # pyref (independent big-integer restatement) on a prefix
        k = 12
        pts = [H.g1_from_affine_mont(bn[i]) for i in range(k)]
        assert dec(H.oracle_msm(group, np.ascontiguousarray(s[:k]), np.ascontiguousarray(bn[:k]))) == \
            pr.msm_shared_doubling(sc[:k], pts, "g1")
    for c in (0, 5, 13, 16, 18):
        r = amd.msm(group, s, bn, c=c, n=n)
        assert gh.decode_icicle(group, r[0]) == ref, ("icicle", c)
    r = amd.msm(group, s, bn, icicle=False, n=n)
    assert gh.decode_jacobian_mont(group, r[0]) == ref, "raw"
    # device scalars, async on a stream
    sd = amd.torch_u64(s)
    out = torch.zeros((1, 18 if group == "g1" else 36), dtype=torch.int64, device="cuda")
    amd.msm(group, sd, b, out=out, is_async=True, n=n)
    torch.cuda.synchronize()
    assert gh.decode_icicle(group, amd.to_numpy_u64(out)[0]) == ref, "device"
    # prepared table (the split against [P, endo P, ...]), shift tables and slot 0 of a table
    factors = (split, 3, 4, 8) if group == "g1" else (split, 2, 3, 8)
    for F in factors:
        table = amd.precompute_bases(group, b, F, n)
        for c in (0, 16):
            r = amd.msm(group, s, table, c=c, precompute_factor=F, n=n)
            assert gh.decode_icicle(group, r[0]) == ref, ("table", F, c)
        r = amd.msm(group, s, table, icicle=False, precompute_factor=F, n=n)
        assert gh.decode_jacobian_mont(group, r[0]) == ref, ("table raw", F)
    # batch of 2 with shared bases: member 0 the odd scalars, member 1 the same reversed
    s2 = np.ascontiguousarray(np.concatenate([s, s[::-1]]))
    r = amd.msm(group, s2, bn, batch=2, n=n)
    ref1 = dec(H.oracle_msm(group, np.ascontiguousarray(s[::-1]), bn))
    assert gh.decode_icicle(group, r[0]) == ref and gh.decode_icicle(group, r[1]) == ref1, "batch"
    # Montgomery-form words >= r: the ICICLE entry converts x -> x R^-1 mod r
    mont = H.ints_to_limbs(sc, 4)
    ref_m = dec(H.oracle_msm(group, H.ints_to_limbs([(x * pr.FR_RINV) % R for x in sc], 4), bn))
    r = amd.msm(group, mont, bn, scalars_mont=True, n=n)
    assert gh.decode_icicle(group, r[0]) == ref_m, "montgomery"


# ----------------------------------------------------------------------------- benchmarked workloads
# bench.py's inputs exactly (seeds, sizes, entry points, flags), bit-exact against the oracle
ORACLE_THREADS = 16  # the GPU box's CPU share


def _oracle_std_scalars(seed, n, start=0):
    s = np.zeros((start + n, 4), dtype=np.uint64)
    H.oracle().orc_gen_scalars(H.ptr(s), seed, start + n)
    return np.ascontiguousarray(s[start:])


@pytest.mark.parametrize("group,seeds", [("g1", (0x5EED0003, 0x5EED0013)), ("g2", (0x5EED0005, 0x5EED0015))])
def test_bench_msm_2_20_production_path(amd, gh, group, seeds):
    """bench.py headline (G1) and config #5 (G2) MSM: 2^20 points, Montgomery scalars and bases
    resident on the device, ICICLE entry ((x, y, 1) result on the device), async on a stream --
    the call core/msm.rs:594-682 makes (core/traits/cpu_impl.rs:117-165 is the CPU semantics)"""
    import torch
    n = 1 << 20
    w = 12 if group == "g1" else 24
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, seeds[0], montgomery=True)
    b = torch.zeros((n, w), dtype=torch.int64, device="cuda")
    amd.gen_bases(group, b, seeds[1])
    out = torch.zeros((1, w * 3 // 2), dtype=torch.int64, device="cuda")
    # torch's side streams are non-blocking: they do not order behind the null stream the
    # generators ran on
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    amd.msm(group, s, b, scalars_mont=True, out=out, stream=st, is_async=True, n=n)
    st.synchronize()
    got = gh.decode_icicle(group, amd.to_numpy_u64(out)[0])
    ref = H.oracle_msm(group, _oracle_std_scalars(seeds[0], n), amd.to_numpy_u64(b), threads=ORACLE_THREADS)
    dec = H.g1_from_affine_mont if group == "g1" else H.g2_from_affine_mont
    assert got == dec(ref)


def test_bench_ntt_2_22_single_and_batch4(amd):
    """bench.py NTT 2^22 (seed 0x5EED0025, forward, natural order) and the config #5 batch of 4 x
    2^22 (the mix leg's inputs), each member vs the oracle's best_fft DFT (core/ntt.rs:1488-1603)"""
    import torch
    amd.ntt_init_domain()
    log_n, B = 22, 4
    n = 1 << log_n
    x = torch.zeros((B * n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(x, 0x5EED0025, montgomery=True)
    y1 = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.ntt(x[:n], out=y1)
    yb = torch.zeros_like(x)
    amd.ntt(x, out=yb, batch=B)
    torch.cuda.synchronize()
    xn = amd.to_numpy_u64(x)
    ybn = amd.to_numpy_u64(yb)
    for k in range(B):
        ref = H.oracle_ntt(xn[k * n:(k + 1) * n], log_n, False, threads=ORACLE_THREADS)
        if k == 0:
            assert np.array_equal(amd.to_numpy_u64(y1), ref)
        assert np.array_equal(ybn[k * n:(k + 1) * n], ref), k
    # inverse of the batch returns the inputs exactly
    z = torch.zeros_like(x)
    amd.ntt(yb, inverse=True, out=z, batch=B)
    torch.cuda.synchronize()
    assert torch.equal(z, x)


@pytest.mark.parametrize("log_n", [21, 22])
def test_msm_g1_chunk_scaling_sizes(amd, gh, log_n):
    """the accumulation chunk scales with the bucket size (16 at 2^21, 32 at 2^22, 128 at 2^24:
    msm_core.hpp accumulate_chunk); 2^21 / 2^22 G1 MSMs through the ICICLE entry equal the
    oracle (2^24 is test_msm_g1_2_24_single_and_sharded)"""
    import torch
    n = 1 << log_n
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0006, montgomery=True)
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0016)
    out = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
    amd.msm("g1", s, b, scalars_mont=True, out=out)
    torch.cuda.synchronize()
    got = gh.decode_icicle("g1", amd.to_numpy_u64(out)[0])
    ref = H.oracle_msm("g1", _oracle_std_scalars(0x5EED0006, n), amd.to_numpy_u64(b), threads=ORACLE_THREADS)
    assert got == H.g1_from_affine_mont(ref)


@pytest.mark.slow
def test_msm_g1_2_24_single_and_sharded(amd, gh):
    """north-star size (BASELINE config #4): G1 MSM of 2^24 points (scalars 0x5EED0004, bases
    0x5EED0013) on one GPU through the ICICLE entry, the C-ABI multi-device entry with 8 shards
    on this GPU (mbls_g1_msm_multi_device), and the bench's sharded sequence for 8
    ranks -- each shard of 2^21 generated from its slice of the global streams, one Jacobian
    partial per shard (mbls_g1_msm_jacobian), partials stacked as the all-gather would, summed
    (mbls_g1_sum_jacobian) and normalised once (mbls_g1_jacobian_to_icicle) -- both equal to
    the oracle's multithreaded Pippenger bit-exactly"""
    import sharded_msm
    import torch
    n, world = 1 << 24, 8
    s = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    amd.gen_scalars(s, 0x5EED0004, montgomery=True)
    b = torch.zeros((n, 12), dtype=torch.int64, device="cuda")
    amd.gen_bases("g1", b, 0x5EED0013)
    out = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
    amd.msm("g1", s, b, scalars_mont=True, out=out)
    torch.cuda.synchronize()
    single = gh.decode_icicle("g1", amd.to_numpy_u64(out)[0])
    # the single-process multi-device entry with the shard loop forced to 8 shards on this GPU
    # (mbls_g1_msm_multi_device, devs = [0] * 8; each shard's bases are its slice of the table)
    shard_b = [b[sharded_msm.shard_range(n, world, r)[0]:sharded_msm.shard_range(n, world, r)[1]] for r in range(world)]
    multi = gh.decode_icicle("g1", amd.msm_multi_device("g1", s, shard_b, [0] * world, n)[0])
    bn = amd.to_numpy_u64(b)
    del s, b, shard_b
    parts = torch.zeros((world, 18), dtype=torch.int64, device="cuda")
    for r in range(world):
        lo, hi = sharded_msm.shard_range(n, world, r)
        ss = torch.zeros((hi - lo, 4), dtype=torch.int64, device="cuda")
        amd.gen_scalars(ss, 0x5EED0004, montgomery=True, start=lo)
        bs = torch.zeros((hi - lo, 12), dtype=torch.int64, device="cuda")
        amd.gen_bases("g1", bs, 0x5EED0013, start=lo)
        amd.msm("g1", ss, bs, icicle="jacobian", scalars_mont=True, out=parts[r:r + 1], n=hi - lo)
    tot = torch.zeros((1, 18), dtype=torch.int64, device="cuda")
    amd.sum_jacobian("g1", parts, tot)
    amd.jacobian_to_icicle("g1", tot)
    torch.cuda.synchronize()
    sharded = gh.decode_icicle("g1", amd.to_numpy_u64(tot)[0])
    ref = H.g1_from_affine_mont(H.oracle_msm("g1", _oracle_std_scalars(0x5EED0004, n), bn, threads=ORACLE_THREADS))
    assert single == ref
    assert sharded == ref
    assert multi == ref


def _skewed(case, n, g):
    """prover-shaped scalar columns: selector-like 0 / 1, small values, one set bit, one repeated
    value (tools/skew_probe.py times them)"""
    if case == "ones":
        return [1] * n
    if case == "half_one":
        return [1 if i % 2 == 0 else g.randrange(pr.R) for i in range(n)]
    if case == "bits8":
        return [g.randrange(256) for _ in range(n)]
    if case == "bit_of_64":
        return [1 << (i % 63) for i in range(n)]
    if case == "repeated":
        return [g.randrange(pr.R)] * n
    if case == "few_values":  # 2048 distinct values: thousands of heavy buckets (the fixed slice plan)
        pool = [g.randrange(pr.R) for _ in range(2048)]
        return [pool[g.randrange(2048)] for _ in range(n)]
    raise ValueError(case)


@pytest.mark.parametrize("group,log_n,case", [("g1", 15, "ones"), ("g1", 15, "half_one"), ("g1", 15, "bits8"),
                                              ("g1", 15, "bit_of_64"), ("g1", 15, "repeated"), ("g1", 20, "ones"),
                                              ("g1", 20, "half_one"), ("g1", 20, "repeated"), ("g1", 20, "few_values"),
                                              ("g1", 22, "ones"), ("g2", 14, "ones"), ("g2", 14, "bits8"),
                                              ("g2", 14, "repeated"), ("g2", 16, "repeated"), ("g2", 16, "half_one")])
def test_msm_skewed_scalars(amd, gh, group, log_n, case):
    """skewed scalar distributions put most contributions into a few buckets (heavy parts of the
    partitioned sort and their helper workgroups -- parts above 2^15 entries: G1 2^20, G2 2^16 --,
    long owner ranges, heavy bucket slices: planned and grouped, or the fixed plan past 1024 heavy
    buckets with `few_values`) -- equal to the oracle"""
    import torch
    n = 1 << log_n
    w = 12 if group == "g1" else 24
    sc = H.ints_to_limbs(_skewed(case, n, pr.rng(77)), 4)
    b = torch.zeros((n, w), dtype=torch.int64, device="cuda")
    amd.gen_bases(group, b, 0x5EED0F20 + log_n)
    out = amd.msm(group, amd.torch_u64(sc), b, icicle=True, n=n)
    ref = H.oracle_msm(group, sc, amd.to_numpy_u64(b), threads=16)
    dec = H.g1_from_affine_mont if group == "g1" else H.g2_from_affine_mont
    assert gh.decode_icicle(group, out[0]) == dec(ref)
