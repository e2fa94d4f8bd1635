#!/usr/bin/env python3
"""Per-kernel VGPR/AGPR/SGPR/scratch from a hipcc -save-temps gfx950 .s file (AMDGPU metadata).

usage: kernel_resources.py file.s [name_substring]
"""
import re
import subprocess
import sys


def main():
    s = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    meta = s[s.index("amdhsa.kernels:"):]
    for block in meta.split("\n  - ")[1:]:
        name = re.search(r"\.name:\s+(\S+)", block)
        if not name or sub not in name.group(1):
            continue
        fields = {k: re.search(r"\." + k + r":\s+(\d+)", block) for k in
                  ("vgpr_count", "agpr_count", "sgpr_count", "private_segment_fixed_size", "group_segment_fixed_size")}
        dem = subprocess.run(["c++filt", name.group(1)], capture_output=True, text=True).stdout.strip()
        print(f"{dem[:70]:70s} " + " ".join(f"{k.split('_')[0]}={v.group(1) if v else '-'}" for k, v in fields.items()))


if __name__ == "__main__":
    main()
