#!/usr/bin/env python3
"""Benchmark: Mrays/s of the MI355X path tracer on the headline workload of BASELINE.json
(island.obj, 1920x1080, 64 spp, 8 bounces) -- one "step" = one progressive frame: one trace of 64
samples per pixel (rng_offset = frame index) + one accumulate.  The K timed steps are the frame loop
of compute_n_then_render (src/raytracing_app.rs:198-227): one hrt_compute_n call of K frames (the
persistent kernel traces up to --frames-per-launch of them per launch, each frame its own image, the
combiner folding them in order -- byte for byte the per-frame loop), then, when N > 1, the row-tile
gather of the accumulated framebuffer for its present -- hrt_read_image on a context joined to an RCCL
communicator (hrt_comm_init: one ncclGather to rank 0 + the row un-interleave on rank 0's device,
behind the C ABI).  --frames-per-launch 1 runs the realtime loop instead (compute_then_render: trace
+ accumulate + gather per frame); the line also reports per_frame_dispatch_ms, a short realtime loop
measured after the timed steps.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Without a launcher (WORLD_SIZE unset) and --gpus N > 1, this process starts the N rank processes itself
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, 127.0.0.1) before anything in it touches a GPU, and
exits with the first failing rank's status; under a launcher --gpus must equal WORLD_SIZE.  For N > 1
--verify is on by default: rank 0 re-renders the frames on one full-frame context and the line's
gather_check says whether the gathered framebuffer is byte-identical to it.

A "ray" is one segment = one world_hit call (assets/raytracing.glsl:317), counted exactly on the
device.  value = segments of all ranks / max-over-ranks wall time of the K timed steps.
Prints ONE JSON line on rank 0 (fields: DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector (= FP32 MFMA) peak
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E spec peak
FLOP_PER_TEST = 38         # algorithmic fp32 FLOP per ray-triangle test (raytracing.glsl:213-241)
BYTES_PER_PIXEL_FRAME = 32  # 16 B ray centre + 4 B trace store + 12 B combiner (r, r, w)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)   # the driver's shape: --steps 20 --warmup 5
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scene", default="island")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64, help="samples per pixel per frame (num_samples)")
    ap.add_argument("--bounces", type=int, default=8, help="max_bounces")
    ap.add_argument("--variant", type=int, default=0,
                    help="hrt_kernel: 0 auto, 1 literal, 2 brute, 3 brute_lds, 4 bundle, 5 bundle_cull")
    ap.add_argument("--row-tile", type=int, default=8)
    ap.add_argument("--frames-per-launch", type=int, default=64,
                    help="> 1: steps run as hrt_compute_n (compute_n_then_render) with up to this many frames per "
                         "trace launch; 1: one trace + accumulate (+ gather) dispatch per step (compute_then_render)")
    ap.add_argument("--verify", action=argparse.BooleanOptionalAction, default=None,
                    help="N>1 (default on): rank 0 re-renders all frames on one full-frame context and compares "
                         "the gathered frame byte for byte (gather_check)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = the library's RCCL gather over xGMI (default); gloo = torch all-gather of the "
                         "local blocks through the host (rehearsal with several ranks on one GPU)")
    ap.add_argument("--realtime-frames", type=int, default=32,
                    help="after the timed steps: frames of the per-frame dispatch loop (compute_then_render) "
                         "reported as per_frame_dispatch_ms (0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample length (0 = skip)")
    ap.add_argument("--comm-timeout-ms", type=int, default=60000,
                    help="HRT_OPT_COMM_TIMEOUT_MS: a collective (hrt_comm_init, the gather) whose peers do not "
                         "arrive within this fails on every rank instead of hanging")
    ap.add_argument("--pmc-json", default=None,
                    help="rocprofv3 PMC record of this build and workload (tools/pmc.sh); default "
                         "profiles/pmc_traffic.json for island, profiles/pmc_traffic_<scene>.json otherwise")
    a = ap.parse_args()
    if a.pmc_json is None:
        a.pmc_json = os.path.join(ROOT, "profiles", "pmc_traffic.json" if a.scene == "island"
                                  else f"pmc_traffic_{a.scene}.json")
    return a


def resolve_launch(gpus: int, env) -> tuple:
    """("spawn", N): no launcher (WORLD_SIZE unset) and N > 1 -- this process starts the N ranks;
    ("rank", world): run as one rank of world.  A --gpus that contradicts the launcher's WORLD_SIZE is
    an error, never a silent single-rank line."""
    if gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in env:
        return ("spawn", gpus) if gpus > 1 else ("rank", 1)
    world = int(env["WORLD_SIZE"])
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
    return ("rank", world)


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv, cmd=None, poll_s: float = 0.1) -> int:
    """Start n rank processes (cmd + argv, default this script) with the torch.distributed.run
    environment, one per GPU, and wait for them.  Returns 0, or the first failing rank's exit status
    after terminating the others (by their own PIDs).  Nothing here touches a GPU: the ranks are fresh
    processes, not forks of an initialised runtime."""
    port = free_port()
    base = cmd or [sys.executable, os.path.abspath(__file__)]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BENCH_SPAWNED="1")
        procs.append(subprocess.Popen(base + list(argv), env=env))
    status = 0
    try:
        while True:
            codes = [p.poll() for p in procs]  # (every rank polled: no short-circuit)
            if all(c is not None for c in codes):
                break
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                status = bad[0]
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if status == 0:
        status = next((p.returncode for p in procs if p.returncode != 0), 0)
    return status


def rank_record(ctx, rank, world, lib_gather, kern_ms, gather_ms, segs) -> dict:
    """What one rank reports to rank 0 for an N > 1 line: the communicator the LIBRARY has
    (hrt_comm_info: did RCCL see N ranks?), its per-frame kernel time and its gather's wall time."""
    # (no library communicator on the gloo rehearsal: the rccl fields are null there)
    crank, cworld, transport = ctx.comm_info() if lib_gather else (None, None, 0)
    return {"rank": rank, "rccl_rank": None if crank is None else int(crank),
            "rccl_world": None if cworld is None else int(cworld), "transport": int(transport),
            "kernel_ms": round(float(kern_ms), 4), "gather_ms": None if gather_ms is None else round(gather_ms, 4),
            "segments": int(segs)}


def assemble_ranks(recs: list, world: int) -> dict:
    """The line's "ranks" object from every rank's rank_record (rank 0 first or not): the
    communicator's world size as the ranks see it (min / max: 8 and 8 when RCCL joined all 8), the rank
    ids it gave them, each rank's kernel time and gather time (max = what the step waited for)."""
    recs = sorted(recs, key=lambda r: r["rank"])
    worlds = [r["rccl_world"] for r in recs if r["rccl_world"] is not None]
    gms = [r["gather_ms"] for r in recs if r["gather_ms"] is not None]
    rccl = len(worlds) == len(recs)  # every rank joined a library communicator (not the gloo rehearsal)
    return {"reported": len(recs), "world": world,
            "rccl_world": {"min": min(worlds), "max": max(worlds)} if rccl else None,
            "rccl_ranks": [r["rccl_rank"] for r in recs] if rccl else None,
            "rccl_ok": (len(recs) == world and min(worlds) == max(worlds) == world
                        and sorted(r["rccl_rank"] for r in recs) == list(range(world))) if rccl else None,
            "transport": sorted({r["transport"] for r in recs}),
            "kernel_ms": [r["kernel_ms"] for r in recs],
            "kernel_ms_max": max(r["kernel_ms"] for r in recs),
            "gather_ms": [r["gather_ms"] for r in recs],
            "gather_ms_max": max(gms) if gms else None,
            "segments": [r["segments"] for r in recs]}


def main():
    args = parse()
    how, world = resolve_launch(args.gpus, os.environ)
    if how == "spawn":
        sys.exit(spawn_ranks(world, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.verify is None:
        args.verify = world > 1

    import torch
    import torch.distributed as dist

    dist_on = world > 1
    gloo = args.dist_backend == "gloo"
    ndev = torch.cuda.device_count()  # (counts devices without initialising the runtime)
    if dist_on and not gloo and world > ndev:
        raise SystemExit(f"bench.py: --gpus {world} with the RCCL gather needs {world} GPUs, {ndev} visible "
                         "(--dist-backend gloo rehearses several ranks on one GPU)")
    device = local_rank % max(ndev, 1)  # one rank per GPU; ranks > GPUs only for gloo rehearsals
    if dist_on:
        torch.cuda.set_device(device)
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
    coll_dev = "cpu" if gloo else f"cuda:{device}"

    import epq_raytracer_amd as E
    from epq_raytracer_amd import _lib, rowtiles

    W, H = args.width, args.height
    camera, settings = E.preset(args.scene)
    settings.num_samples, settings.max_bounces = args.spp, args.bounces
    partition = (args.row_tile, rank, world) if dist_on else None
    ctx = E.HrtContext((W, H), device=device, mode=_lib.MODE_RGBA8, partition=partition)
    raytrace = E.RayTracePipeline(ctx, (W, H), settings)
    diffuse = E.DiffusePipeline(ctx, (W, H))
    ctx.set_option(_lib.OPT_KERNEL_VARIANT, args.variant)
    fpl = max(1, args.frames_per_launch)
    ctx.set_option(_lib.OPT_FRAMES_PER_LAUNCH, fpl)
    raytrace.init()
    diffuse.next_frame(0, raytrace.image())
    frame = 1

    lib_gather = dist_on and not gloo
    lib_comm_error = None
    if lib_gather:  # RCCL communicator inside the library: rank 0's id shared through torch.distributed
        ctx.set_option(_lib.OPT_COMM_TIMEOUT_MS, args.comm_timeout_ms)
        uid = [E.HrtContext.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        failed = 0
        try:
            ctx.comm_init(uid[0], rank, world)
        except _lib.HrtError as e:  # (the library's error text; every rank fails, none waits past the timeout)
            print(f"bench.py rank {rank}/{world}: library communicator: {e}", file=sys.stderr, flush=True)
            lib_comm_error = str(e)
            failed = 1
        # (decided together: if any rank has no library communicator, no rank enters its gather)
        flag = torch.tensor([failed], dtype=torch.int32, device=coll_dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if int(flag[0]):
            # the frame is still gathered, by torch.distributed's own all-gather of the same row blocks
            # (RCCL through torch), and the line says so -- a scaling curve with the reason beside it
            lib_gather = False
            lib_comm_error = lib_comm_error or "another rank's hrt_comm_init failed"
    torch_gather = dist_on and not lib_gather  # the gloo rehearsal, or the fallback above
    local = torch.empty((ctx.local_rows, W, 4), dtype=torch.uint8, device=coll_dev) if torch_gather else None
    full = torch.empty((H, W, 4), dtype=torch.uint8, device=f"cuda:{device}") if lib_gather and rank == 0 else None

    def present():
        nonlocal full
        if lib_gather:  # the framebuffer gather behind the C ABI: one ncclGather + un-interleave on rank 0
            if rank == 0:
                ctx.read_into(_lib.IMG_ACCUM, _lib.FMT_RGBA8, full.data_ptr(), full.numel())
            else:
                ctx.read_into(_lib.IMG_ACCUM, _lib.FMT_RGBA8, 0, 0)
        elif dist_on:  # gloo rehearsal: all-gather of the equal-size row-tile blocks through the host
            ctx.read_into(_lib.IMG_ACCUM, _lib.FMT_RGBA8, local.data_ptr(), local.numel())
            full = rowtiles.gather_frame(local, H, args.row_tile)

    def steps(k):
        nonlocal frame
        if k <= 0:
            return
        if fpl > 1:  # compute_n_then_render(k): k frames, then one present
            ctx.compute_n(raytrace.push_constants(camera, frame, False), k)
            frame += k
            present()
            return
        for _ in range(k):  # compute_then_render per frame
            raytrace.compute(camera, frame)
            diffuse.next_frame(frame, raytrace.image())
            frame += 1
            present()

    steps(args.warmup)
    ctx.synchronize()
    torch.cuda.synchronize()
    ctx.reset_stats()

    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps(args.steps)
    ctx.synchronize()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    st = ctx.stats()
    segs, tests = st.segments, st.tri_tests
    # the gather's own wall time (one more present after the timed region: the library's status
    # all-reduce + ncclGather + row assembly, or the gloo all-gather)
    gather_ms = None
    if dist_on:
        dist.barrier()
        tg = time.perf_counter()
        present()
        ctx.synchronize()
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3
    last_trace = ctx.read(_lib.IMG_TRACE, _lib.FMT_RGBA8) if world == 1 else None
    gathered = full.cpu().numpy() if (dist_on and rank == 0 and full is not None) else None
    # the realtime loop (compute_then_render per frame, src/main.rs:41-57): consecutive traces overlap
    # on the context's trace lanes (three by default); measured after the timed steps, separately reported
    rt_ms = None
    if args.realtime_frames > 0 and fpl > 1:
        saved = fpl
        fpl = 1
        steps(6)  # untimed: every trace lane's first (probe-planned) trace
        if dist_on:
            dist.barrier()
        ctx.synchronize()
        t1 = time.perf_counter()
        steps(args.realtime_frames)
        ctx.synchronize()
        if dist_on:
            dist.barrier()
        rt_ms = (time.perf_counter() - t1) * 1e3 / args.realtime_frames
        fpl = saved
    kern_ms = st.total_trace_ms / max(st.traces, 1)  # per frame (a launch of f frames counts f traces)
    launches = -(-args.steps // fpl) if fpl > 1 else args.steps
    last_frame = frame - 1 - (args.realtime_frames + 6 if rt_ms is not None else 0)
    kernel_sym = _lib.kernel_symbol(st.last_kernel, st.last_block,  # what HRT_KERNEL_AUTO resolved to
                                    node_r=_lib.wq_node_radius(ctx.scene_info()))
    ranks = None
    if dist_on:
        recs = [None] * world
        dist.all_gather_object(recs, rank_record(ctx, rank, world, lib_gather, kern_ms, gather_ms, segs))
        ranks = assemble_ranks(recs, world)
        t = torch.tensor([elapsed, kern_ms, rt_ms or 0.0], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_max = float(t[0]), float(t[1])
        rt_ms = float(t[2]) if rt_ms is not None else None
        c = torch.tensor([segs, tests], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        segs_all, tests_all = int(c[0]), int(c[1])
    else:
        kern_ms_max, segs_all, tests_all = kern_ms, segs, tests

    if rank == 0:
        ms_per_step = elapsed * 1e3 / args.steps
        value = segs_all / elapsed / 1e6
        # roofline of the dominant kernel (trace), rank 0's launches: algorithmic FLOP / launch time
        tests_per_frame = tests / max(st.traces, 1)
        # reference-equivalent work: 38 FLOP per triangle test the reference performs;
        # the tuned kernel skips most of them exactly, so this rate can exceed the hardware peak.
        algorithmic_tf = FLOP_PER_TEST * tests_per_frame / (kern_ms * 1e-3) / 1e12
        pix_local = ctx.local_rows * W
        algo_bytes = BYTES_PER_PIXEL_FRAME * pix_local + (len(raytrace.tris) * 64 + len(raytrace.meshes) * 80)
        # the timed launch's frames (the PMC record must be of the same launch shape)
        roof = pmc_roofline(args, world, kernel_sym, kern_ms, tests_per_frame, ctx.local_rows / H,
                            max(1, st.last_frames))  # (as the library split the steps into launches)
        line = {
            "metric": (f"Mrays/s ({args.scene}.obj {W}x{H} {args.spp}spp {args.bounces}-bounce path-trace segments "
                       "per second)"),
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": (f"synthetic: reference scene preset ({args.scene} geometry + src/main.rs materials/camera"
                     + (", build-defined for cave" if args.scene == "cave" else "") +
                     "), deterministic RNG seeds rng_offset = frame index"),
            "config": {"workload": f"{args.scene}.obj {W}x{H} {args.spp}spp {args.bounces}-bounce, 1 frame/step "
                                   + (f"(trace + accumulate; the {args.steps} steps as compute_n_then_render: "
                                      f"{launches} trace launch(es) of <= {fpl} frames"
                                      f"{', then the row-tile gather' if dist_on else ''})" if fpl > 1 else
                                      f"(trace + accumulate{' + row-tile gather' if dist_on else ''} per frame)"),
                       "frames_per_launch": fpl if fpl > 1 else 1,
                       "launch_frames": int(st.last_frames),  # the timed launches' frames, as the library split them
                       "scene": args.scene, "width": W, "height": H, "spp": args.spp, "bounces": args.bounces,
                       "parallelism": (f"row-tiles{world}x{args.row_tile} (" +
                                       ("RCCL ncclGather behind hrt_read_image" if lib_gather else
                                        "gloo all-gather" if gloo else
                                        "torch.distributed all-gather: the library's communicator failed")
                                       + ")" if dist_on else "single-gpu"),
                       "launcher": ("bench.py --gpus (own rank processes)" if os.environ.get("BENCH_SPAWNED")
                                    else "torch.distributed.run" if dist_on else "single process"),
                       "kernel_variant": _lib.KERNEL_NAMES[args.variant]},
            "segments_per_step": segs_all // args.steps,
            "tri_tests_per_step": tests_all // args.steps,
            "paths_per_s": W * H * args.spp / (elapsed / args.steps),
            "per_frame_dispatch_ms": round(rt_ms, 3) if rt_ms is not None else None,
            "roofline": {"bound": "valu-fp32", **roof,
                         "algorithmic_tflops": round(algorithmic_tf, 3),
                         "kernel": kernel_sym,
                         "kernel_ms": round(kern_ms, 3),
                         "launch_ms": round(kern_ms * args.steps / launches, 3),
                         "kernel_ms_basis": "per frame: launch time / frames per launch (HIP events on the "
                                            "context's stream)",
                         "flop_per_test": FLOP_PER_TEST,
                         "tests_per_frame": int(tests_per_frame), "build_id": _lib.build_id()},
            # BASELINE.md's %HBM-roofline: rocprofv3 counter bytes (FETCH_SIZE x2 + WRITE_SIZE) per frame /
            # the live per-frame kernel time / 8 TB/s; the compulsory (algorithmic) bytes beside it
            "hbm_roofline": {"achieved": (round(roof["traffic"] / (kern_ms * 1e-3) / 1e9, 3)
                                          if roof["traffic"] else None),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": (round(roof["traffic"] / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                                      if roof["traffic"] else None),
                             "basis": "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per frame / live kernel time per frame",
                             "traffic_per_frame": roof["traffic"],
                             "algorithmic_bytes_per_frame": algo_bytes,
                             "algorithmic_gbs": round(algo_bytes / (kern_ms * 1e-3) / 1e9, 3),
                             "traffic_over_algorithmic": (round(roof["traffic"] / algo_bytes, 2)
                                                          if roof["traffic"] else None)},
        }
        if world == 1 and args.cpu_seconds > 0:
            line["cpu_baseline"], line["parity_sample"] = cpu_baseline(args, raytrace, camera, last_frame,
                                                                       last_trace)
        if ranks is not None:
            line["ranks"] = ranks
        if lib_comm_error is not None:
            line["lib_comm_error"] = lib_comm_error
        if dist_on and args.verify:
            line["gather_check"] = verify_gather(args, gathered, settings, camera, device, last_frame)
        print(json.dumps(line), flush=True)

    ctx.close()
    if dist_on:
        dist.destroy_process_group()


def pmc_roofline(args, world, kernel_sym, kern_ms, tests_per_frame, row_frac, launch_frames):
    """roofline.achieved / frac / traffic from the committed rocprofv3 PMC record of THIS build
    (profiles/pmc_traffic.json, tools/pmc.sh): executed FP32 FLOP per frame / the live per-frame
    kernel time.  A record of another build (hrt_build_id), kernel or workload gives null."""
    from epq_raytracer_amd import _lib
    out = {"achieved": None, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": None, "traffic": None,
           "achieved_basis": "unmeasured (no rocprofv3 PMC record of this build, kernel and workload)",
           "pmc_source": None}
    if not os.path.exists(args.pmc_json):
        return out
    with open(args.pmc_json) as f:
        pmc = json.load(f)
    wl = pmc.get("workload", {})
    want = {"scene": args.scene, "width": args.width, "height": args.height, "spp": args.spp,
            "bounces": args.bounces, "kernel_variant": _lib.KERNEL_NAMES[args.variant],
            "frames_per_launch": launch_frames}
    if pmc.get("build_id") != _lib.build_id():
        out["achieved_basis"] = (f"unmeasured: the PMC record is of build {pmc.get('build_id')}, this library is "
                                 f"{_lib.build_id()}")
        return out
    if pmc.get("kernel") != kernel_sym or any(wl.get(k) != v for k, v in want.items()):
        out["achieved_basis"] = "unmeasured: the PMC record is of another kernel or workload"
        return out
    flops = pmc.get("executed_fp32_flops_per_frame")
    traffic = pmc.get("hbm_bytes_per_frame")
    if world > 1:  # this rank's rows: the record's FLOPs per reference test x the rank's own tests
        per_test = pmc.get("executed_flops_per_reference_test")
        flops = per_test * tests_per_frame if per_test else None
        traffic = traffic * row_frac if traffic else None
    if flops:
        tf = flops / (kern_ms * 1e-3) / 1e12
        out.update(achieved=round(tf, 3), frac=round(tf / FP32_PEAK_TFLOPS, 4),
                   achieved_basis=("executed FP32 FLOP per frame (rocprofv3 PMC of this build and launch shape) / "
                                   "live per-frame kernel time" + (", scaled to this rank's triangle tests"
                                                                  if world > 1 else "")))
    out["traffic"] = round(traffic) if traffic else None
    out["valu_issue_utilisation"] = pmc.get("valu_issue_utilisation")
    # lane-weighted: the FP32 FLOPs the ACTIVE lanes execute (executed x the VALU lane utilisation,
    # SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU) of the same record); frac above counts every
    # wave-instruction as 64 lanes whatever the exec mask
    lane_util = pmc.get("valu_lane_utilisation")
    if flops and lane_util:
        lane_tf = flops * lane_util / (kern_ms * 1e-3) / 1e12
        out.update(lane_flops=round(lane_tf, 3), lane_frac=round(lane_tf / FP32_PEAK_TFLOPS, 4),
                   live_lane_ratio=round(lane_util, 4))
    else:
        out.update(lane_flops=None, lane_frac=None, live_lane_ratio=None)
    out["pmc_source"] = os.path.relpath(args.pmc_json, ROOT)
    return out


def verify_gather(args, full, settings, camera, device, last_frame):
    """Rank 0: render frames 1..last_frame on one full-frame context (same accumulation sequence) and
    compare its accumulator with the row-tile-gathered one byte for byte."""
    import epq_raytracer_amd as E
    from epq_raytracer_amd import _lib
    W, H = args.width, args.height
    ref_ctx = E.HrtContext((W, H), device=device, mode=_lib.MODE_RGBA8)
    rt = E.RayTracePipeline(ref_ctx, (W, H), settings)
    df = E.DiffusePipeline(ref_ctx, (W, H))
    ref_ctx.set_option(_lib.OPT_KERNEL_VARIANT, args.variant)
    rt.init()
    df.next_frame(0, rt.image())
    for k in range(1, last_frame + 1):
        rt.compute(camera, k)
        df.next_frame(k, rt.image())
    ref = ref_ctx.read(_lib.IMG_ACCUM)
    ref_ctx.close()
    got = full if isinstance(full, np.ndarray) else full.cpu().numpy()
    return {"frames": last_frame, "bit_exact": bool(np.array_equal(got, ref)),
            "pixels_differing": int(np.any(got != ref, axis=-1).sum())}


def cpu_baseline(args, raytrace, camera, last_frame, gpu):
    """The oracle (oracle/rt_oracle.c, OpenMP) on a bounded sample of the same workload: whole rows
    spread evenly over the last timed frame (rng_offset = last_frame).  Also checks those rows of the
    GPU's trace image of that frame (as the timed loop left it) byte for byte against it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from epq_raytracer_amd import _lib

    W, H = args.width, args.height
    pc = raytrace.push_constants(camera, last_frame, False)
    rays = raytrace.rays
    threads = pyoracle.num_threads()
    # calibrate on one row, then pick a row count for ~cpu_seconds
    t = time.perf_counter()
    pyoracle.trace(pc, rays, raytrace.spheres, raytrace.tris, raytrace.meshes, rows=(H // 2, H // 2 + 1))
    per_row = max(time.perf_counter() - t, 1e-4)
    nrows = int(min(H, max(2, args.cpu_seconds / per_row)))
    rows = np.unique(np.linspace(0, H - 1, nrows).astype(int))
    segs = 0
    cpu_img = np.zeros((H, W, 4), np.uint8)
    t = time.perf_counter()
    for y in rows:
        img, _, s, _ = pyoracle.trace(pc, rays, raytrace.spheres, raytrace.tris, raytrace.meshes, rows=(int(y), int(y) + 1))
        cpu_img[y] = img[y]
        segs += s
    dt = time.perf_counter() - t
    same = bool(np.array_equal(gpu[rows], cpu_img[rows]))
    base = {"value": round(segs / dt / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{len(rows)} of {H} rows (evenly spaced) of the same frame (rng_offset={last_frame}), "
                      f"{segs} segments, "
                      f"{dt:.1f} s on {threads} OpenMP threads (oracle/rt_oracle.c -O2 -ffp-contract=off)"}
    parity = {"rows_checked": int(len(rows)), "frame": last_frame, "bit_exact": same}
    return base, parity


if __name__ == "__main__":
    main()
