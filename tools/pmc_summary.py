"""Summarise rocprofv3 --pmc passes (counter_collection.csv) per trace-kernel dispatch."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(out):
    per = defaultdict(lambda: defaultdict(float))
    durations = {}
    for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r.get("Kernel_Name", "")
                if "trace" not in k:
                    continue
                per[k][r["Counter_Name"]] += float(r["Counter_Value"])
                per[k]["_dispatches_" + r["Counter_Name"]] += 1
    for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*kernel_trace.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "trace" in r["Kernel_Name"]:
                    durations.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    res = {}
    for k, c in per.items():
        # counters are summed over dispatches of that kernel in a pass; normalise per dispatch
        d = {n: v / max(c["_dispatches_" + n], 1) for n, v in c.items() if not n.startswith("_")}
        # rows are per (dispatch, counter) possibly per-XCD/SE instance: dispatches counted per row
        res[k] = d
    print(json.dumps({"per_dispatch_counters": res, "durations_ns": durations}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
