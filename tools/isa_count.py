#!/usr/bin/env python3
"""Static instruction counts of one kernel in a `make asm` listing, by class and by opcode:
    python3 tools/isa_count.py <hrt_kernels.s> <mangled kernel name> [top N opcodes]"""
import collections
import sys

src = open(sys.argv[1]).read()
name = sys.argv[2]
start = src.index("\n" + name + ":") + 1
end = src.index(".Lfunc_end", start)
c = collections.Counter()
for l in src[start:end].splitlines()[1:]:
    l = l.strip()
    if not l or l.startswith(('.', ';', '//')) or l.split()[0].endswith(':'):
        continue
    op = l.split()[0]
    c['v_pk' if op.startswith('v_pk_') else op.split('_')[0]] += 1
    c['op:' + op] += 1
print({k: v for k, v in c.items() if not k.startswith('op:')})
n = int(sys.argv[3]) if len(sys.argv) > 3 else 25
print([(k[3:], v) for k, v in c.most_common() if k.startswith('op:')][:n])
