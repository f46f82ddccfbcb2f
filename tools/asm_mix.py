#!/usr/bin/env python
"""Instruction mix of one kernel in an amdgcn .s file: python tools/asm_mix.py FILE.s SUBSTRING..."""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
for sub in sys.argv[2:]:
    for m in re.finditer(r'^(_Z\S*):\s*;', s, re.M):
        name = m.group(1)
        if sub not in name:
            continue
        end = s.find('.Lfunc_end', m.end())
        body = s[m.end():end]
        ins = [l.strip().split()[0] for l in body.split('\n')
               if l.strip() and not l.strip().startswith(('.', ';')) and not l.strip().endswith(':')]
        c = Counter(ins)
        kinds = Counter()
        for k, v in c.items():
            kinds['valu' if k.startswith('v_') else 'salu' if k.startswith('s_') and not k.startswith(('s_load', 's_buffer', 's_waitcnt', 's_barrier', 's_cbranch', 's_branch')) else
                  'vmem' if k.startswith(('global_', 'buffer_', 'flat_')) else 'lds' if k.startswith('ds_') else
                  'smem' if k.startswith(('s_load', 's_buffer')) else 'other'] += v
        meta = s[s.find('.amdhsa_kernel ' + name):]
        vg = re.search(r'\.amdhsa_next_free_vgpr (\d+)', meta)
        print(name, 'static instrs', len(ins), dict(kinds), 'vgpr', vg.group(1) if vg else '?')
        print('  ', c.most_common(14))
