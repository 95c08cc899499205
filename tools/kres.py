#!/usr/bin/env python3
"""Per-kernel resources from a hipcc --offload-device-only -S listing: VGPRs (arch + acc),
SGPRs, scratch bytes, LDS. Usage: tools/kres.py file.s [name-substring]"""
import re
import sys

src = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", src, re.S):
    name, body = m.group(1), m.group(2)
    if pat not in name:
        continue
    g = lambda k: int(re.search(r"\.amdhsa_" + k + r"\s+(\d+)", body).group(1))
    print(f"{name[:90]:90s} vgpr {g('next_free_vgpr'):4d} acc_off {g('accum_offset'):4d} "
          f"sgpr {g('next_free_sgpr'):3d} scratch {g('private_segment_fixed_size'):4d}")
