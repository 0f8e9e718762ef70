"""CPU-only checks of the drop-in boundary: the HIP library builds/loads, exports every symbol
include/bls12_381_mi355x.h declares, and the ctypes config structs match the C layout."""
import ctypes
import os
import re
import subprocess

import pytest

import helpers as H

HEADER = os.path.join(H.ROOT, "include", "bls12_381_mi355x.h")
PKG = os.path.join(H.ROOT, "midnight-bls12-381-cuda_amd")
LIB = os.path.join(PKG, "lib", "libbls12_381_mi355x.so")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^(?:eIcicleError|MSMConfig|NTTConfig|VecOpsConfig|const char\*|void|int)\s+(\w+)\s*\(",
                       src, flags=re.M)
    return sorted(set(names))


def _amd():
    import sys
    sys.path.insert(0, PKG)
    import bls12_381_amd
    return bls12_381_amd


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", PKG, "-j8", "-s"])
    return LIB


def test_header_declares_reference_entry_points():
    fns = header_functions()
    # the reference's exported C symbols for this path
    for ref in ["bls12_381_g1_msm_cuda", "bls12_381_g2_msm_cuda", "bls12_381_ntt_cuda",
                "bls12_381_ntt_init_domain_cuda", "bls12_381_ntt_release_domain_cuda", "bls12_381_coset_ntt_cuda",
                "bls12_381_field_ntt_cuda", "bls12_381_field_ntt_init_domain_cuda",
                "bls12_381_field_ntt_release_domain_cuda", "bls12_381_vector_add", "bls12_381_vector_sub",
                "bls12_381_vector_mul", "vec_add_cuda", "vec_sub_cuda", "vec_mul_cuda", "scalar_mul_vec_cuda",
                "scalar_add_vec_cuda"]:
        assert ref in fns, ref


def test_library_exports_every_declared_symbol(built):
    out = subprocess.check_output(["nm", "-D", "--defined-only", built]).decode()
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing
    amd = _amd()
    assert sorted(amd.EXPORTED) == header_functions()


def test_library_loads_and_reports_version(built):
    amd = _amd()
    L = amd.lib()
    assert b"gfx950" in L.mbls_version()
    assert L.mbls_error_string(11) == b"INVALID_ARGUMENT"
    assert L.mbls_error_string(14) == b"UNKNOWN_ERROR"


def test_default_configs(built):
    amd = _amd()
    c = amd.lib().mbls_default_msm_config()
    assert c.batch_size == 1 and c.precompute_factor == 1 and c.are_points_shared_in_batch
    n = amd.lib().mbls_default_ntt_config()
    assert n.batch_size == 1 and n.ordering == 0
    assert [int(x) for x in n.coset_gen.limbs][0] == 0x00000001fffffffe
    v = amd.lib().mbls_default_vec_ops_config()
    assert v.batch_size == 1


def test_struct_layouts_match_c(tmp_path):
    amd = _amd()
    probe = tmp_path / "probe.c"
    probe.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "bls12_381_mi355x.h"
int main(void) {
  printf("%zu %zu %zu %zu\n", sizeof(MSMConfig), offsetof(MSMConfig, ext), offsetof(MSMConfig, is_async), offsetof(MSMConfig, batch_size));
  printf("%zu %zu %zu %zu\n", sizeof(NTTConfig), offsetof(NTTConfig, ordering), offsetof(NTTConfig, ext), offsetof(NTTConfig, batch_size));
  printf("%zu %zu\n", sizeof(NTTInitDomainConfig), offsetof(NTTInitDomainConfig, ext));
  printf("%zu %zu %zu\n", sizeof(VecOpsConfig), offsetof(VecOpsConfig, batch_size), offsetof(VecOpsConfig, ext));
  printf("%zu %zu %zu %zu\n", sizeof(mbls_g1_affine_t), sizeof(mbls_g1_projective_t), sizeof(mbls_g2_affine_t), sizeof(mbls_g2_projective_t));
  return 0;
}
''')
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), str(probe), "-o", str(exe)])
    lines = subprocess.check_output([str(exe)]).decode().split("\n")
    c = ctypes
    assert lines[0].split() == [str(x) for x in (c.sizeof(amd.MSMConfig), amd.MSMConfig.ext.offset,
                                                 amd.MSMConfig.is_async.offset, amd.MSMConfig.batch_size.offset)]
    assert lines[1].split() == [str(x) for x in (c.sizeof(amd.NTTConfig), amd.NTTConfig.ordering.offset,
                                                 amd.NTTConfig.ext.offset, amd.NTTConfig.batch_size.offset)]
    assert lines[2].split() == [str(x) for x in (c.sizeof(amd.NTTInitDomainConfig), amd.NTTInitDomainConfig.ext.offset)]
    assert lines[3].split() == [str(x) for x in (c.sizeof(amd.VecOpsConfig), amd.VecOpsConfig.batch_size.offset,
                                                 amd.VecOpsConfig.ext.offset)]
    assert lines[4].split() == ["96", "144", "192", "288"]
