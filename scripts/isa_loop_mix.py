"""Instruction mix of the hottest loop of a kernel in an llvm-objdump disassembly (ISA study helper).
usage: python scripts/isa_loop_mix.py DISASM KERNEL_SUBSTRING [STEPS_PER_ITERATION]"""
import re
import sys
from collections import Counter

txt = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2]
steps = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
funcs, cur = {}, None
for l in txt:
    m = re.match(r'^([0-9a-f]+) <(.+)>:$', l)
    if m:
        cur = m.group(2)
        funcs[cur] = []
        continue
    m = re.match(r'^\s+(\S+)(.*?)//\s*([0-9A-F]+):', l)
    if cur and m:
        funcs[cur].append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
name = [n for n in funcs if pat in n][0]
body = funcs[name]
loops = []
for addr, op, args in body:
    if op.startswith('s_cbranch') or op == 's_branch':
        off = int(args.split()[0])
        if off >= 32768:
            tgt = addr + 4 + (off - 65536) * 4
            loops.append((addr - tgt, tgt, addr))
size, lo, hi = max(loops)
ins = [op for a, op, _ in body if lo <= a <= hi]
c = Counter(ins)
print(name[:100])
print(f'loop {len(ins)} instructions, {size} bytes; per step ({steps:g} steps per iteration):')
valu = sum(v for k, v in c.items() if k.startswith('v_'))
lds = sum(v for k, v in c.items() if k.startswith('ds_'))
print(f'  VALU {valu / steps:.1f}  LDS {lds / steps:.1f}')
print('  ' + ', '.join(f'{k} {v / steps:g}' for k, v in c.most_common(40)))
