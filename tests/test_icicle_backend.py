"""ICICLE backend shims: the three libraries an unchanged
midnight-zk reaches through ICICLE core.

ICICLE core is not in this image, so tests/icicle_mock/mock_icicle.cpp stands in for it: it
defines the icicle::register_* entry points, dlopens the backend libraries like ICICLE's loader
and records what registered under which device type.  CPU tests check the registrations and
that every symbol the libraries import from ICICLE core mangles to the signature the
reference declares (icicle_backend_api.cuh:98-226); the GPU test drives every registered op
through the registered HIP DeviceAPI and compares each result byte-for-byte with the direct C
ABI call (which test_gpu_parity.py pins to the oracle)."""
import json
import os
import subprocess

import pytest

import helpers as H

PKG = os.path.join(H.ROOT, "midnight-bls12-381-cuda_amd")
ICICLE_DIR = os.path.join(PKG, "lib", "icicle")
LIBS = {
    "device": "libicicle_backend_cuda_device.so",
    "field": "libicicle_backend_cuda_field_bls12_381.so",
    "curve": "libicicle_backend_cuda_curve_bls12_381.so",
}
MOCK_SRC = os.path.join(H.ROOT, "tests", "icicle_mock", "mock_icicle.cpp")

STR = "std::__cxx11::basic_string<char, std::char_traits<char>, std::allocator<char> > const&"
FR = "Field<bls12_381::fp_config>"
FQ = "Field<bls12_381::fq_config>"
FQ2 = f"ComplexExtensionField<bls12_381::fq_config, {FQ} >"
DEV = "icicle::Device const&"
ERR = "icicle::eIcicleError"
# reference icicle_backend_api.cuh:118-199 (impl types) x :141-199 (register functions)
EXPECTED_IMPORTS = {
    "field": {
        f"icicle::register_ntt({STR}, std::function<{ERR} ({DEV}, {FR} const*, int, icicle::NTTDir, "
        f"icicle::NTTConfig<{FR} > const&, {FR}*)>)",
        f"icicle::register_ntt_init_domain({STR}, std::function<{ERR} ({DEV}, {FR} const&, "
        f"icicle::NTTInitDomainConfig const&)>)",
        f"icicle::register_ntt_release_domain({STR}, std::function<{ERR} ({DEV}, {FR} const&)>)",
        f"icicle::register_vector_add({STR}, std::function<{ERR} ({DEV}, {FR} const*, {FR} const*, unsigned long, "
        f"icicle::VecOpsConfig const&, {FR}*)>)",
        f"icicle::register_vector_mul({STR}, std::function<{ERR} ({DEV}, {FR} const*, {FR} const*, unsigned long, "
        f"icicle::VecOpsConfig const&, {FR}*)>)",
        f"icicle::register_scalar_mul_vec({STR}, std::function<{ERR} ({DEV}, {FR} const*, {FR} const*, "
        f"unsigned long, icicle::VecOpsConfig const&, {FR}*)>)",
    },
    "curve": {
        f"icicle::register_msm({STR}, std::function<{ERR} ({DEV}, {FR} const*, Affine<{FQ} > const*, int, "
        f"icicle::MSMConfig const&, Projective<{FQ}, {FR}, bls12_381::G1>*)>)",
        f"icicle::register_msm_precompute_bases({STR}, std::function<{ERR} ({DEV}, Affine<{FQ} > const*, int, "
        f"icicle::MSMConfig const&, Affine<{FQ} >*)>)",
    },
    "device": {
        f"icicle::register_deviceAPI({STR}, std::shared_ptr<icicle::DeviceAPI>)",
    },
}
EXPECTED_REGS = ["register_deviceAPI", "register_ntt", "register_ntt_init_domain", "register_ntt_release_domain",
                 "register_ntt_get_rou_from_domain", "register_vector_add", "register_vector_sub",
                 "register_vector_mul", "register_scalar_mul_vec", "register_scalar_add_vec", "register_vector_sum",
                 "register_msm", "register_msm_precompute_bases", "register_g2_msm",
                 "register_g2_msm_precompute_bases"]


def _need_libs():
    if not all(os.path.exists(os.path.join(ICICLE_DIR, f)) for f in LIBS.values()):
        subprocess.check_call(["make", "-C", PKG, "-j8", "-s"])


def _mock(tmp_path_factory):
    _need_libs()
    exe = str(tmp_path_factory.mktemp("mock") / "mock_icicle")
    lib = os.path.join(PKG, "lib")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-rdynamic", "-D__HIP_PLATFORM_AMD__",
                           "-I", os.path.join(PKG, "csrc"), "-I", os.path.join(H.ROOT, "include"),
                           MOCK_SRC, "-o", exe,
                           "-L", ICICLE_DIR, "-licicle_backend_cuda_curve_bls12_381",
                           "-L", lib, "-lbls12_381_mi355x", f"-Wl,-rpath,{ICICLE_DIR}:{lib}", "-ldl"])
    return exe


@pytest.fixture(scope="module")
def mock(tmp_path_factory):
    return _mock(tmp_path_factory)


def _imports(lib):
    out = subprocess.check_output(["nm", "-D", "-C", "--undefined-only", os.path.join(ICICLE_DIR, lib)]).decode()
    return {l.split(None, 1)[1].strip(): l.split(None, 1)[0] for l in out.splitlines() if l.strip()}


def test_backend_libraries_import_icicle_registration_abi():
    _need_libs()
    for part, expected in EXPECTED_IMPORTS.items():
        imp = _imports(LIBS[part])
        for sig in expected:
            assert sig in imp, f"{LIBS[part]} does not import {sig}"
            assert imp[sig] == "w", f"{sig} should be a weak import (loads without ICICLE core)"


def test_backend_libraries_resolve_their_dependencies():
    """field / curve forward to the HIP library (found through the $ORIGIN rpath); the device
    API needs only the HIP runtime"""
    _need_libs()
    for part, lib in LIBS.items():
        out = subprocess.check_output(["ldd", os.path.join(ICICLE_DIR, lib)]).decode()
        assert "not found" not in out, out
        assert "libamdhip64" in out, out
        if part != "device":
            assert "libbls12_381_mi355x.so" in out, out


def test_registrations_under_cuda_device_type(mock):
    out = subprocess.check_output([mock, ICICLE_DIR]).decode().strip().splitlines()[0]
    regs = json.loads(out)
    for name in EXPECTED_REGS:
        assert regs.get(name) == ["CUDA"], (name, regs.get(name))


@pytest.mark.gpu
def test_registered_ops_match_direct_abi(mock):
    p = subprocess.run([mock, ICICLE_DIR, "--run"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "gpu run ok" in p.stdout, p.stdout + p.stderr
