#!/usr/bin/env python3
"""Per-kernel register / scratch usage of one compiled object of the library.

  python tools/kres.py retinex-image-enhancement_amd/lib/obj/conv_hw2.hip.o [regex]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    obj, filt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else ".")
    with tempfile.TemporaryDirectory() as d:
        fat, dev = os.path.join(d, "fat.bin"), os.path.join(d, "dev.o")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj])
        subprocess.check_call(["/opt/rocm/llvm/bin/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"])
        notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", dev], text=True)
    rows = []
    for line in notes.splitlines():
        if line.startswith("  - .agpr_count:"):  # a kernel entry begins
            rows.append({})
        m = re.match(r"\s+(?:- )?\.(name|vgpr_count|agpr_count|sgpr_count|private_segment_fixed_size|"
                     r"vgpr_spill_count|sgpr_spill_count|group_segment_fixed_size):\s+(\S+)", line)
        if m and rows and m.group(1) not in rows[-1]:
            rows[-1][m.group(1)] = m.group(2)
    for r in rows:
        if re.search(filt, r["name"]):
            print(f"{r.get('vgpr_count', '?'):>4}v {r.get('agpr_count', '?'):>4}a {r.get('sgpr_count', '?'):>4}s "
                  f"scratch {r.get('private_segment_fixed_size', '?'):>4} spill {r.get('vgpr_spill_count', '?'):>3} sspill {r.get('sgpr_spill_count', '?'):>3}  "
                  f"{r['name'][:120]}")


if __name__ == "__main__":
    main()
