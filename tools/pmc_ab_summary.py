"""Per-frame instruction counters of the trace kernel for each A/B build profiled by tools/pmc_ab.sh.

    python tools/pmc_ab_summary.py gpurun_out/<tag>"""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

out = sys.argv[1]
for d in sorted(glob.glob(os.path.join(out, "*"))):
    if not os.path.isdir(d):
        continue
    for k, passes in load(d).items():
        if "<false>" not in k:
            continue
        cs, dur = passes[0]
        row = {"build": os.path.basename(d), "kernel": k, "ms_per_frame": round(dur * 1e3 / 64, 3)}
        row.update({c: round(v / 64 / 1e6, 2) for c, v in sorted(cs.items())})  # millions per frame
        print(json.dumps(row))
