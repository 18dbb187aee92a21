"""Summarise rocprofv3 --pmc passes (counter_collection.csv) for the trace-kernel dispatches.

    python tools/pmc_summary.py gpurun_out/<tag> [--traffic-json profiles/pmc_traffic.json --workload k=v ...]

Per dispatch: the counters summed over their instances, the kernel duration (kernel trace of the same
pass), effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), VALU issue utilisation, executed FP32
FLOP rate ((2*FMA + MUL + ADD) wave-instructions * 64 lanes / duration) and HBM traffic:
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads half the bytes of a wide coalesced
stream (MI355X_MICROARCH.md, HBM section), so read bytes = 2 * FETCH_SIZE * 1024.
"""
import argparse
import csv
import glob
import json
import os
import statistics
from collections import defaultdict


def load(out):
    counters = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    durations = defaultdict(list)
    for pdir in sorted(glob.glob(os.path.join(out, "p*"))):
        per_dispatch = defaultdict(lambda: defaultdict(float))
        names = {}
        for f in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = r.get("Kernel_Name", "")
                    if "trace" not in k:
                        continue
                    did = r.get("Dispatch_Id", r.get("Correlation_Id", "0"))
                    per_dispatch[did][r["Counter_Name"]] += float(r["Counter_Value"])
                    names[did] = k
        for did, cs in per_dispatch.items():
            for n, v in cs.items():
                counters[names[did]][n].append(v)
        for f in glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if "trace" in r["Kernel_Name"]:
                        durations[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return counters, durations


def summarise(counters, durations):
    res = {}
    for k, cs in counters.items():
        c = {n: statistics.median(v) for n, v in cs.items()}
        dur = statistics.median(durations[k]) * 1e-9 if durations.get(k) else None
        d = {"counters_per_dispatch": c, "duration_s_median": dur}
        if dur:
            if "GRBM_GUI_ACTIVE" in c:
                d["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9
            if "SQ_INSTS_VALU" in c and "effective_clock_ghz" in d:
                slots = 256 * 4 * d["effective_clock_ghz"] * 1e9 * dur / 2  # wave64 VALU = 2 cycles on SIMD32
                d["valu_issue_utilisation"] = c["SQ_INSTS_VALU"] / slots
            if "SQ_INSTS_VALU_FMA_F32" in c:
                fl = 64 * (2 * c["SQ_INSTS_VALU_FMA_F32"] + c.get("SQ_INSTS_VALU_MUL_F32", 0) +
                           c.get("SQ_INSTS_VALU_ADD_F32", 0))
                d["executed_fp32_tflops"] = fl / dur / 1e12
                d["executed_fp32_flops"] = fl
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                rd = 2 * c["FETCH_SIZE"] * 1024
                wr = c["WRITE_SIZE"] * 1024
                d["hbm_read_bytes"] = rd
                d["hbm_write_bytes"] = wr
                d["hbm_bytes"] = rd + wr
                d["hbm_gbs"] = (rd + wr) / dur / 1e9
        res[k] = d
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--traffic-json", default=None)
    ap.add_argument("--workload", nargs="*", default=[])
    a = ap.parse_args()
    counters, durations = load(a.out)
    res = summarise(counters, durations)
    print(json.dumps(res, indent=1))
    if a.traffic_json:
        wl = {}
        for kv in a.workload:
            k, v = kv.split("=", 1)
            wl[k] = int(v) if v.isdigit() else v
        # the default (auto) trace kernel of the run
        k = max(res, key=lambda n: res[n].get("duration_s_median") or 0)
        d = res[k]
        ref_tests = None  # the reference's triangle tests per launch (kbench JSON line of pass 1)
        try:
            with open(os.path.join(a.out, "p1.log")) as fh:
                for line in fh:
                    if line.startswith("{"):
                        ref_tests = json.loads(line).get("tri_tests", ref_tests)
        except (OSError, ValueError):
            pass
        with open(a.traffic_json, "w") as f:
            json.dump({"workload": wl, "kernel": k, "hbm_bytes_per_trace_launch": d.get("hbm_bytes"),
                       "hbm_read_bytes": d.get("hbm_read_bytes"), "hbm_write_bytes": d.get("hbm_write_bytes"),
                       "duration_s_median": d.get("duration_s_median"),
                       "effective_clock_ghz": d.get("effective_clock_ghz"),
                       "executed_fp32_tflops": d.get("executed_fp32_tflops"),
                       "executed_fp32_flops_per_trace_launch": d.get("executed_fp32_flops"),
                       "reference_tests_per_trace_launch": ref_tests,
                       "executed_flops_per_reference_test": (d.get("executed_fp32_flops") / ref_tests
                                                             if ref_tests and d.get("executed_fp32_flops") else None),
                       "valu_issue_utilisation": d.get("valu_issue_utilisation"),
                       "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KiB->bytes; separate --pmc passes, "
                               "kernel-trace only"}, f, indent=1)


if __name__ == "__main__":
    main()
