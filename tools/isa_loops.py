#!/usr/bin/env python3
"""Static instruction counts per loop of one kernel in a `make asm` listing (blocks grouped by the
innermost loop header the compiler's comments name):
    python3 tools/isa_loops.py <hrt_kernels.s> <mangled kernel name>"""
import collections
import re
import sys

src = open(sys.argv[1]).read()
name = sys.argv[2]
start = src.index("\n" + name + ":") + 1
end = src.index(".Lfunc_end", start)
loops = collections.OrderedDict()
cur = "entry"
for l in src[start:end].splitlines()[1:]:
    s = l.strip()
    m = re.match(r"^(\.LBB\d+_\d+):\s*(;.*)?$", s)
    if m:
        c = m.group(2) or ""
        h = re.search(r"Header=BB(\d+_\d+) Depth=(\d+)", c)
        hl = re.search(r"Loop Header: Depth=(\d+)", c)
        if h:
            cur = "BB%s d%s" % (h.group(1), h.group(2))
        elif hl:
            cur = "%s d%s" % (m.group(1)[2:], hl.group(1))
        else:
            cur = "outside"
        continue
    if not s or s.startswith((".", ";", "//")):
        continue
    op = s.split()[0]
    d = loops.setdefault(cur, collections.Counter())
    d["all"] += 1
    d[op.split("_")[0]] += 1
    if op.startswith("v_") and ("f32" in op or "f16" in op):
        d["vf"] += 1
for k, v in loops.items():
    print(k, dict(v))
