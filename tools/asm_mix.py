"""Instruction mix of one kernel in a gfx950 .s file: python tools/asm_mix.py file.s <kernel substring>"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
names = [m.group(1) for m in re.finditer(r"^(\S+):", s, re.M) if sys.argv[2] in m.group(1) and not m.group(1).startswith('.')]
name = names[0]
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
c = collections.Counter()
for line in s[i:j].split('\n'):
    t = line.strip().split(' ')[0]
    if not t or t.startswith(('.', ';')) or t.endswith(':'):
        continue
    cls = ('mfma' if 'mfma' in t else 'valu' if t.startswith('v_') else 'salu' if t.startswith('s_') and not t.startswith(('s_load', 's_buffer', 's_waitcnt', 's_nop', 's_barrier', 's_cbranch', 's_branch')) else
           'smem' if t.startswith(('s_load', 's_buffer')) else 'lds' if t.startswith('ds_') else 'vmem' if t.startswith(('global_', 'buffer_', 'flat_', 'scratch_')) else 'ctl')
    c[cls] += 1
print(name[:80], dict(c), 'total', sum(c.values()))
