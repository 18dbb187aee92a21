"""Summarise rocprofv3 --pmc passes (counter_collection.csv) for the trace-kernel dispatches.

    python tools/pmc_summary.py gpurun_out/<tag> [--traffic-json profiles/pmc_traffic.json --frames F
                                                  --workload k=v ...]

Each pass p<i>/ is one rocprofv3 run (--kernel-trace --pmc <counters>) of the same deterministic
command (tools/pmc.sh: bench.py itself, so the profiled launch has the timed launch's shape).  Per
trace kernel the summary takes the LONGEST dispatch of each pass (the bench's timed launch of F
frames; the warm-up launch and the planning probe are shorter or differently named) and reports its
counters, duration, effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), VALU issue utilisation,
executed FP32 FLOP ((2*FMA + MUL + ADD) wave-instructions * 64 lanes) and HBM traffic, per launch and
per frame (/ F).  HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced stream (MI355X_MICROARCH.md, HBM section), so read bytes = 2 * FETCH_SIZE
* 1024 (the guide calls other access widths uncalibrated: this kernel's reads are scalar loads and
8-byte band entries, so the absolute figure carries that caveat; ratios between builds do not).
The traffic JSON is stamped with the library's hrt_build_id() so bench.py never applies counters of
another build.
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(out):
    """kernel -> list (one per pass) of (counters of its longest dispatch, duration in s)."""
    res = defaultdict(list)
    for pdir in sorted(glob.glob(os.path.join(out, "p*"))):
        if not os.path.isdir(pdir):
            continue
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
        dur = {}
        for f in glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if "trace" in r["Kernel_Name"]:
                        dur[r.get("Dispatch_Id", "")] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        best = {}
        for did, cs in per_dispatch.items():
            k, d = names[did], dur.get(did)
            if d is not None and (k not in best or d > best[k][1]):
                best[k] = (dict(cs), d)
        for k, v in best.items():
            res[k].append(v)
    return res


def summarise(passes, frames):
    out = {}
    for k, lst in passes.items():
        c = {}
        for cs, _ in lst:
            c.update(cs)
        dur = sorted(d for _, d in lst)[len(lst) // 2]
        d = {"counters_per_launch": c, "duration_s": dur, "frames_per_launch": frames}
        if "GRBM_GUI_ACTIVE" in c:
            d["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9
        if "SQ_INSTS_VALU" in c and "effective_clock_ghz" in d:
            slots = 256 * 4 * d["effective_clock_ghz"] * 1e9 * dur / 2  # wave64 VALU = 2 cycles on SIMD32
            d["valu_issue_utilisation"] = c["SQ_INSTS_VALU"] / slots
        if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_ANY" in c:
            d["wait_any_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        if "SQ_INSTS_LDS" in c and "SQ_LDS_BANK_CONFLICT" in c and c["SQ_INSTS_LDS"]:
            d["lds_conflict_cycles_per_lds_inst"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"]
        if "SQ_INSTS_VALU_FMA_F32" in c:
            fl = 64 * (2 * c["SQ_INSTS_VALU_FMA_F32"] + c.get("SQ_INSTS_VALU_MUL_F32", 0) +
                       c.get("SQ_INSTS_VALU_ADD_F32", 0))
            d["executed_fp32_flops_per_launch"] = fl
            d["executed_fp32_flops_per_frame"] = fl / frames
            d["executed_fp32_tflops"] = fl / dur / 1e12
        if "SQ_INSTS_VALU_FLOPS_FP32" in c:
            # (tools/probe/flops_probe.hip, r05a: FLOPS_FP32 counts per WAVE-instruction -- fma 2, mul / add /
            # trans 1 -- whatever the exec mask, i.e. the same as 2 FMA + MUL + ADD (+ TRANS) above / 64)
            d["fp32_flops_counter_per_frame"] = 64 * c["SQ_INSTS_VALU_FLOPS_FP32"] / frames
            d["fp32_trans_ops_counter_per_frame"] = 64 * c.get("SQ_INSTS_VALU_FLOPS_FP32_TRANS", 0) / frames
        if "SQ_THREAD_CYCLES_VALU" in c and c.get("SQ_ACTIVE_INST_VALU"):
            # lanes active per VALU instruction (rocprof's VALUUtilization; r05b: exactly the exec mask's
            # share on the probe), and the FP32 FLOPs the ACTIVE lanes execute at that share
            d["valu_lane_utilisation"] = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
            if "executed_fp32_flops_per_frame" in d:
                d["lane_fp32_flops_per_frame"] = d["executed_fp32_flops_per_frame"] * d["valu_lane_utilisation"]
                d["lane_fp32_tflops"] = d["lane_fp32_flops_per_frame"] * frames / dur / 1e12
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rd, wr = 2 * c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
            d.update(hbm_read_bytes_per_frame=rd / frames, hbm_write_bytes_per_frame=wr / frames,
                     hbm_bytes_per_frame=(rd + wr) / frames, hbm_gbs=(rd + wr) / dur / 1e9)
        out[k] = d
    return out


def bench_line(out):
    """The bench JSON line of pass 1 (reference triangle tests per frame, segments)."""
    try:
        with open(os.path.join(out, "p1.log")) as fh:
            for line in fh:
                if line.startswith("{"):
                    return json.loads(line)
    except (OSError, ValueError):
        pass
    return {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--traffic-json", default=None)
    ap.add_argument("--frames", type=int, default=1, help="frames traced by the profiled (longest) launch")
    ap.add_argument("--workload", nargs="*", default=[])
    a = ap.parse_args()
    res = summarise(load(a.out), a.frames)
    print(json.dumps(res, indent=1))
    if a.traffic_json:
        sys.path.insert(0, ROOT)
        from epq_raytracer_amd import _lib
        wl = {}
        for kv in a.workload:
            k, v = kv.split("=", 1)
            wl[k] = int(v) if v.lstrip("-").isdigit() else v
        k = max(res, key=lambda n: res[n]["duration_s"])  # the dominant trace kernel
        d = res[k]
        b = bench_line(a.out)
        ref_tests = b.get("tri_tests_per_step")
        fl = d.get("executed_fp32_flops_per_frame")
        with open(a.traffic_json, "w") as f:
            json.dump({"build_id": _lib.build_id(), "workload": wl, "kernel": k, "frames_per_launch": a.frames,
                       "hbm_bytes_per_frame": d.get("hbm_bytes_per_frame"),
                       "hbm_read_bytes_per_frame": d.get("hbm_read_bytes_per_frame"),
                       "hbm_write_bytes_per_frame": d.get("hbm_write_bytes_per_frame"),
                       "launch_duration_s": d["duration_s"], "effective_clock_ghz": d.get("effective_clock_ghz"),
                       "executed_fp32_flops_per_frame": fl, "executed_fp32_tflops": d.get("executed_fp32_tflops"),
                       "reference_tests_per_frame": ref_tests,
                       "executed_flops_per_reference_test": fl / ref_tests if fl and ref_tests else None,
                       "valu_issue_utilisation": d.get("valu_issue_utilisation"),
                       "valu_lane_utilisation": d.get("valu_lane_utilisation"),
                       "lane_fp32_flops_per_frame": d.get("lane_fp32_flops_per_frame"),
                       "fp32_flops_counter_per_frame": d.get("fp32_flops_counter_per_frame"),
                       "wait_any_frac": d.get("wait_any_frac"),
                       "lds_conflict_cycles_per_lds_inst": d.get("lds_conflict_cycles_per_lds_inst"),
                       "counters_per_launch": d["counters_per_launch"],
                       "note": "longest dispatch of each separate --pmc pass (kernel-trace only) of the bench "
                               "command; FETCH_SIZE x2 (gfx950) + WRITE_SIZE, KiB->bytes; per frame = / "
                               "frames_per_launch"}, f, indent=1)


if __name__ == "__main__":
    main()
