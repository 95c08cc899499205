#!/usr/bin/env python3
"""Per-loop instruction summary of one kernel in a hipcc -S listing (experiment tooling):
VALU / MFMA / LDS / buffer / scratch counts and vmcnt waits per loop header.
Usage: tools/isa_loops.py file.s kernel-symbol-substring"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2]
st = [i for i, l in enumerate(src) if re.match(r"^\S*" + re.escape(pat) + r"\S*:", l)][0]
en = [i for i in range(st, len(src)) if src[i].startswith(".Lfunc_end")][0]
body = src[st:en]
blocks, cur = [], None
for l in body:
    m = re.match(r"^(\.LBB\w+):\s*(;.*)?$", l)
    if m:
        cur = [m.group(1), m.group(2) or "", []]
        blocks.append(cur)
        continue
    s = l.strip()
    if not s or s.startswith(";") or s.startswith("."):
        continue
    if cur:
        cur[2].append(s)
loops = {}
for name, ann, ins in blocks:
    h = re.search(r"Header=(\w+)", ann)
    hh = ("BB" + name[4:]) if "Loop Header" in ann else (h.group(1) if h else None)
    if hh:
        loops.setdefault(hh, []).append((name, ins))
for h, bl in loops.items():
    c = Counter()
    waits = []
    for n, ins in bl:
        for s in ins:
            c[s.split()[0]] += 1
            if s.startswith("s_waitcnt") and "vmcnt" in s:
                waits.append(s.split()[1])
    valu = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
    if valu < 40:
        continue
    print(f"{h}: blocks {len(bl)} valu {valu} mfma {c['v_mfma_f32_16x16x32_f16']} trans "
          f"{c['v_sin_f32_e32'] + c['v_cos_f32_e32']} ds_w {sum(v for k, v in c.items() if k.startswith('ds_write'))} "
          f"ds_r {sum(v for k, v in c.items() if k.startswith('ds_read'))} buf {sum(v for k, v in c.items() if k.startswith('buffer_'))} "
          f"glob {sum(v for k, v in c.items() if k.startswith('global_'))} scratch {sum(v for k, v in c.items() if k.startswith('scratch_'))} "
          f"salu {sum(v for k, v in c.items() if k.startswith('s_'))} vmcnt {waits[:12]}")
