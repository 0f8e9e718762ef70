"""Static instruction counts per kernel of the shipped library (DESIGN.md's ISA tables).

Extracts the gfx950 code object from the .so's .hip_fatbin (a clang offload bundle), disassembles
it with llvm-objdump and counts, per kernel symbol matching a substring: VALU / SALU / LDS / VMEM
instructions and the mnemonics asked for (default: v_mad_u64_u32, v_addc_co_u32, v_lshl_add_u64,
s_nop, v_mov_b32).  Usage: python tools/isa_count.py [--lib PATH] SUBSTRING [MNEMONIC ...]"""
import argparse
import collections
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(lib):
    """every gfx950 code object of the .hip_fatbin section (one offload bundle per translation unit)"""
    out = subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", ".hip_fatbin=/dev/stdout", lib, "/dev/null"],
                         capture_output=True, check=True).stdout
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = out.find(magic)
    assert pos >= 0, "no offload bundle"
    while pos >= 0:
        n = struct.unpack_from("<Q", out, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", out, p)
            triple = out[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple:
                yield out[pos + off:pos + off + size]
        pos = out.find(magic, pos + 32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "midnight-bls12-381-cuda_amd", "lib", "libbls12_381_mi355x.so"))
    ap.add_argument("kernel")
    ap.add_argument("mnemonics", nargs="*", default=["v_mad_u64_u32", "v_addc_co_u32", "v_lshl_add_u64", "v_mov_b32", "s_nop"])
    a = ap.parse_args()
    dis = ""
    for co in code_objects(a.lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            dis += subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", "--no-show-raw-insn", f.name],
                                  capture_output=True, text=True, check=True).stdout
    sym = None
    counts = collections.defaultdict(collections.Counter)
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
        if m:
            sym = m.group(1)
            continue
        if sym is None or a.kernel not in sym:
            continue
        t = line.strip().split()
        if not t or t[0].startswith(";"):
            continue
        op = t[0]
        c = counts[sym]
        c["total"] += 1
        cls = ("lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_"))
               else "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "other")
        c[cls] += 1
        if op in a.mnemonics:
            c[op] += 1
    if not counts:
        sys.exit(f"no kernel matching {a.kernel!r}")
    for s, c in counts.items():
        dem = subprocess.run(["c++filt", s], capture_output=True, text=True).stdout.strip()
        print(dem)
        print("  " + ", ".join(f"{k} {c[k]}" for k in ["total", "valu", "salu", "lds", "vmem"] + a.mnemonics))


if __name__ == "__main__":
    main()
