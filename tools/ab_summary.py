#!/usr/bin/env python3
"""Summarise tools/ab.sh output files: per file and library, the min over rounds of the min ms per frame."""
import json
import sys
from collections import defaultdict

for path in sys.argv[1:]:
    best = defaultdict(list)
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "result" in d:
            best[d["lib"].split("/")[-2] if "lib" in d else (d["args"] or "(default)")].append(min(d["result"]["ms"]))
    print(path)
    for k, v in best.items():
        print(f"  {k:16s} min {min(v):.3f}  per round {v}")
