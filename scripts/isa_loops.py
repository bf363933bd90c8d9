"""Every backward branch (loop) of one kernel in an llvm-objdump disassembly with its VALU / LDS / SALU counts and
spill traffic (v_readlane / v_writelane); with LO HI (hex addresses) also the instruction histogram of that range.
usage: python scripts/isa_loops.py DISASM KERNEL_SUBSTRING [LO HI]"""
import re, sys
from collections import Counter
txt = open(sys.argv[1]).read().split('\n'); pat = sys.argv[2]
funcs, cur = {}, None
for l in txt:
    m = re.match(r'^([0-9a-f]+) <(.+)>:$', l)
    if m: cur = m.group(2); funcs[cur] = []; continue
    m = re.match(r'^\s+(\S+)(.*?)//\s*([0-9A-F]+):', l)
    if cur and m: funcs[cur].append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
name = [n for n in funcs if pat in n][0]; body = funcs[name]
for addr, op, args in body:
    if op.startswith('s_cbranch') or op == 's_branch':
        off = int(args.split()[0])
        if off >= 32768:
            tgt = addr + 4 + (off - 65536) * 4
            ins = [o for a, o, _ in body if tgt <= a <= addr]
            c = Counter(ins)
            valu = sum(v for k, v in c.items() if k.startswith('v_'))
            lds = sum(v for k, v in c.items() if k.startswith('ds_'))
            print(f"loop {tgt:x}-{addr:x} {op} n={len(ins)} VALU={valu} LDS={lds} readlane={c['v_readlane_b32']} writelane={c['v_writelane_b32']} salu={sum(v for k,v in c.items() if k.startswith('s_'))} saveexec={c['s_and_saveexec_b64']}")
if len(sys.argv) > 3:
    lo, hi = int(sys.argv[3], 16), int(sys.argv[4], 16)
    c = Counter(o for a, o, _ in body if lo <= a <= hi)
    print(sorted(c.items(), key=lambda x: -x[1]))
