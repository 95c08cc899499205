#!/usr/bin/env python3
"""Instruction mix of one loop of a kernel in a hipcc -S listing (experiment tooling): all
blocks from label A up to (not including) label B. Usage: tools/loopmix.py file.s kernel A B"""
import sys
from collections import Counter
f, kern, a, b = sys.argv[1:5]
src = open(f).read().split('\n')
st = [i for i, l in enumerate(src) if l.startswith(kern + ':')][0]
ia = [i for i in range(st, len(src)) if src[i].startswith(a + ':')][0]
ib = [i for i in range(ia, len(src)) if src[i].startswith(b + ':')][0]
ins = [l.strip().split()[0] for l in src[ia:ib] if l.strip() and not l.strip().startswith((';', '.')) and not l.startswith('.L')]
c = Counter(ins)
valu = sum(v for k, v in c.items() if k.startswith('v_') and 'mfma' not in k)
pk = sum(v for k, v in c.items() if k.startswith('v_pk_'))
salu = sum(v for k, v in c.items() if k.startswith('s_'))
print(f"n {len(ins)} valu {valu} (pk {pk}) salu {salu} nop {c['s_nop']} waitcnt {c['s_waitcnt']} "
      f"trans {c['v_sin_f32_e32'] + c['v_cos_f32_e32']} mfma {c['v_mfma_f32_16x16x32_f16']} "
      f"ds {sum(v for k, v in c.items() if k.startswith('ds_'))} buf {sum(v for k, v in c.items() if k.startswith('buffer'))}")
