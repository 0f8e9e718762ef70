"""Register / LDS / scratch metadata per kernel of the shipped library (code-object notes).
Usage: python tools/kernel_meta.py [--lib PATH] SUBSTRING"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_count  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=os.path.join(isa_count.ROOT, "midnight-bls12-381-cuda_amd", "lib", "libbls12_381_mi355x.so"))
ap.add_argument("kernel")
a = ap.parse_args()
KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count", ".group_segment_fixed_size",
        ".private_segment_fixed_size")
for co in isa_count.code_objects(a.lib):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        notes = subprocess.run([f"{isa_count.LLVM}/llvm-readelf", "--notes", f.name], capture_output=True, text=True).stdout
    # one YAML map per kernel: split at "- .agpr_count" style entries by ".name:" grouping
    for block in re.split(r"\n\s+- \.", notes):
        m = re.search(r"\.name:\s+(\S+)", block)
        if not m or a.kernel not in m.group(1) or m.group(1).endswith(".kd"):
            continue
        vals = {k: re.search(re.escape(k.lstrip(".")) + r":\s+(\d+)", block) for k in KEYS}
        dem = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        print(dem[:110], {k.lstrip("."): int(v.group(1)) for k, v in vals.items() if v})
