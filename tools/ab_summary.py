#!/usr/bin/env python3
"""Summarise tools/ab.sh output: per library, the min over rounds of the min ms per frame."""
import json
import sys
from collections import defaultdict

best = defaultdict(list)
for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    if "result" in d:
        best[d["lib"].split("/")[-2]].append(min(d["result"]["ms"]))
for k, v in best.items():
    print(f"{k:12s} min {min(v):.3f}  per round {v}")
