#!/usr/bin/env python3
"""bench.py — throughput of the MI355X path tracer on BASELINE.json's headline metric.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

A step is one pass of the hot path over one batch: every rank renders its
row-block-cyclic share of the config's image for all of that step's samples (one
kernel launch), and for N > 1 the shards are gathered to rank 0 over RCCL and
assembled there (the gather of step k overlaps the render of step k+1; the timed
region ends after the last gather and assembly).

Scaling is WEAK by default: per-GPU work is fixed at the config's frame
(W x H x spp pixel-samples); with N GPUs the frame gets N x spp samples per pixel
(each GPU renders 1/N of the rows at N x spp). --scaling strong keeps spp fixed.

`value` = counted rays of all ranks / max-over-ranks wall time of the K steps, in
Mray/s, the reference's own formula (src/cpu/main.cpp:188-189; rays counted as
parallel.cpp:122,204). Inputs are resident in HBM (the scene is uploaded once); no
host transfer is inside the timed region.

Rank 0 prints ONE JSON line on stdout; progress goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mray/s at 1280×720, 4 spp, 8-bounce; 1/2/4/8-GPU scaling"
CONFIGS = {
    2: dict(width=1280, height=720, spp=4, depth=8, scene="default"),
    3: dict(width=1920, height=1080, spp=16, depth=50, scene="default"),
    4: dict(width=3840, height=2160, spp=64, depth=8, scene="random1000"),
    5: dict(width=7680, height=4320, spp=256, depth=8, scene="random1000"),
}
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md, chip-level parameters (spec)
BYTES_PER_PIXEL_SAMPLE = 24.0    # 12 B read + 12 B write of RGB per pixel-sample


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(cfg, budget_s: float):
    """Time the reference's own TraceRowJob body (oracle/_ref, forked worker processes,
    per-pixel seeds) -- or the C restatement if _ref is absent -- on this host."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the baseline leg only

    cores = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    cores = max(1, min(cores, os.cpu_count() or 1))
    w, h, depth = cfg["width"], cfg["height"], cfg["depth"]
    if cfg["scene"] == "default":
        x0, xc, y0, yc = 0, w, 0, h
        spheres = mats = None
        what = f"full {w}x{h} frames"
    else:
        from learnraytracing_amd.scene import random_scene, scene_arrays
        import numpy as np
        s, m = scene_arrays(*random_scene(1000, 1))
        spheres, mats = np.array(s, np.float32), np.array(m, np.float32)
        xc, yc = 128, 32
        x0, y0 = (w - xc) // 2, (h - yc) // 2
        what = f"{xc}x{yc} centre crop of {w}x{h}"
    use_ref = oracle.have_ref() and spheres is None
    kind = "reference" if use_ref else "port"
    rays = 0
    frames = 0
    t0 = time.perf_counter()
    while True:
        if use_ref:
            _, r = oracle.ref_render_p(w, h, 1, depth, frames, x0, xc, y0, yc, procs=cores)
        else:
            _, r = oracle.orc_render(w, h, 1, depth, frames, x0, xc, y0, yc, spheres=spheres, mats=mats,
                                     threads=cores)
        if r < 0:
            raise RuntimeError("cpu baseline failed")
        rays += r
        frames += 1
        dt = time.perf_counter() - t0
        if dt >= budget_s:
            break
    src = "oracle/_ref (reference maths.cpp+parallel.cpp, clang -O2)" if use_ref else "oracle/lrt_oracle.c"
    return {"value": rays / dt / 1e6, "unit": "Mray/s", "cores": cores, "kind": kind,
            "sample": f"{what}, {frames} frame(s) x 1 spp, {depth} bounces, per-pixel seeds, "
                      f"{rays} rays in {dt:.2f} s, {cores} {'processes' if use_ref else 'threads'}; {src}"}


def kernel_name(kernel: str, frames: int) -> str:
    if kernel == "auto":   # mirrors render_device's policy in lrt_hip.hip
        kernel = "v0"
    return {"v0": "trace_kernel", "v1": "paths_kernel", "v3": "regen_kernel", "wf": "wf_extend"}.get(kernel, "paths2_kernel")


def read_traffic(cfg_name: str):
    """HBM bytes per launch of trace_kernel from the committed PMC run, if any."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(cfg_name)
        return (e["bytes_per_launch"], os.path.relpath(p, ROOT)) if e else (None, None)
    except (OSError, ValueError, KeyError):
        return None, None


def read_valu(cfg_name: str):
    """VALU issue fraction and lane utilisation of trace_kernel from the summary of the
    committed PMC run that pmc_traffic.json points at (the path's real bound)."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            src = json.load(f)[cfg_name]["source"]
        sp = os.path.join(ROOT, "profiles", src, "summary.json")
        with open(sp) as f:
            s = json.load(f)
        c = s["counters_per_launch"]
        return {"issue_frac": round(s["valu_issue_frac_of_peak"], 4),
                "valu_insts_per_launch": c["SQ_INSTS_VALU"],
                "lane_util": round(c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64), 4),
                "note": "wave64 VALU instructions issued / (1024 SIMDs x 1 per 2 cycles at 2.4 GHz); "
                        "lane_util = active lanes per VALU instruction / 64",
                "source": os.path.relpath(sp, ROOT)}
    except (OSError, ValueError, KeyError, ZeroDivisionError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--streams", type=int, default=2,
                    help="render streams the steps rotate over: step k+1 starts in the CU slots step k's "
                         "persistent grid frees during its tail (each step writes its own buffer)")
    ap.add_argument("--spp", type=int, default=None, help="diagnostic: override the config's spp per GPU")
    ap.add_argument("--depth", type=int, default=None, help="diagnostic: override the config's bounce budget")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="diagnostic (1 process): render only rank 0's shard of an N-GPU weak-scaling run, "
                         "no gather -- the per-GPU render time at N GPUs, measured on one")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=None, help="seconds of CPU-baseline timing")
    ap.add_argument("--scene-global", action="store_true", help="read spheres from global memory, not LDS")
    ap.add_argument("--reserve-cus", type=int, default=None,
                    help="CUs the render stream leaves free for other streams (default 0)")
    ap.add_argument("--kernel", choices=["auto", "v0", "v1", "v2", "v2s", "v3", "wf"], default="auto",
                    help="auto: the library's policy (default); v0: one pixel per lane (LRT_F_SIMPLE); "
                         "v1: unscheduled state machine; v2: phase-scheduled persistent; v2s[N]: "
                         "phase-scheduled, N static pixels per lane")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus {args.gpus}; using WORLD_SIZE")
    cfg = dict(CONFIGS[args.config])
    if args.spp:
        cfg["spp"] = args.spp
    if args.depth is not None:
        cfg["depth"] = args.depth
    cfg_name = f"config{args.config}"

    # CPU baseline first: rank 0 at N=1 only, before anything touches the GPU.
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
        budget = args.cpu_budget if args.cpu_budget is not None else max(1.5, 15.0 / max(1, cores))
        log(f"cpu baseline ({budget:.1f} s budget) ...")
        cpu = cpu_baseline(cfg, budget)
        log(f"cpu baseline: {cpu['value']:.1f} Mray/s ({cpu['kind']}, {cpu['cores']} cores)")

    import torch
    import torch.distributed as dist

    backend = os.environ.get("LRT_DIST_BACKEND", "nccl")   # nccl = RCCL; gloo only to rehearse on 1 GPU
    # LRT_BENCH_SAME_GPU=1 puts every rank on GPU 0 (rehearsing the RCCL path on a 1-GPU box)
    gpu = 0 if (backend != "nccl" or os.environ.get("LRT_BENCH_SAME_GPU") == "1") else local_rank
    torch.cuda.set_device(gpu)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    import learnraytracing_amd as lrt
    from learnraytracing_amd.dist import gather_to_root, max_shard_rows, shard_rows
    from learnraytracing_amd.renderer import unshard_tensor

    lrt.InitializeTest()
    # --reserve-cus R: render on a CU-masked stream (lrt_stream_create) leaving R CUs to
    # other streams. Off by default: a kernel on another stream only starts beside the
    # persistent render once >= 8 CUs per XCD are free (64 CUs, -23 % render throughput;
    # tools/overlap_probe.py), which costs more than the gather it would hide
    reserve = args.reserve_cus if args.reserve_cus is not None else 0
    rstream = None
    if reserve > 0:
        from learnraytracing_amd.renderer import RenderStream
        rstream = RenderStream(reserve)
        torch.cuda.set_stream(rstream.torch)
    if cfg["scene"] == "random1000":
        lrt.set_scene(*lrt.random_scene(1000, 1))
    W, H, D = cfg["width"], cfg["height"], cfg["depth"]
    shards = world if world > 1 else max(1, args.shard_of)   # row shards of the frame
    spp_total = cfg["spp"] * shards if args.scaling == "weak" else cfg["spp"]
    rb = H if shards == 1 else args.row_block
    max_rows = max_shard_rows(H, rb, shards)
    rows = shard_rows(H, rb, shards, rank)
    flags = (1 if args.scene_global else 0) | {"auto": 0, "v0": 2, "v1": 4, "v2": 16, "v2s": 8, "v3": 128, "wf": 256}[args.kernel]
    job = lrt.Job(width=W, height=H, frame0=0, frames=spp_total, max_depth=D, row_block=rb,
                  row_period=shards, row_phase=rank, row_count=rows, flags=flags)
    dev = torch.device("cuda", torch.cuda.current_device())
    nstreams = max(1, args.streams)
    nslots = max(2, nstreams)
    bufs = [torch.zeros((max_rows, W, 4), dtype=torch.float32, device=dev) for _ in range(nslots)]
    rays = torch.zeros(1, dtype=torch.int64, device=dev)
    gathered = [torch.empty((world, max_rows, W, 4), dtype=torch.float32, device=dev) if rank == 0 and world > 1
                else None for _ in range(nslots)]
    frame = torch.empty((H, W, 4), dtype=torch.float32, device=dev) if rank == 0 and world > 1 else None
    stream = torch.cuda.current_stream(dev)
    # render streams (the first is the current stream); frame assembly on its own stream
    rstreams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(nstreams - 1)]
    astream = torch.cuda.Stream(device=dev) if world > 1 else stream

    pending = []   # (work, slot) of gathers not yet assembled

    def assemble(work, slot):
        with torch.cuda.stream(astream):
            if work is not None:
                work.wait()   # the assembly stream waits for the gather
            if rank == 0:
                unshard_tensor(gathered[slot], frame, W, H, rb, world, astream)
            done = torch.cuda.Event()
            done.record(astream)
        # the slot's next render (and so its next gather) waits until this one was gathered
        rstreams[slot % nstreams].wait_event(done)

    def step(k, events=None):
        slot = k % nslots
        rs = rstreams[k % nstreams]
        if events is not None:
            events[0].record(rs)
        lrt.render_tensor(job, bufs[slot], rays, rs)
        if events is not None:
            events[1].record(rs)
        if world > 1:
            with torch.cuda.stream(rs):   # the gather is ordered after this step's render
                _, work = gather_to_root(bufs[slot], max_rows, world, rank, gathered=gathered[slot], async_op=True)
            while pending:
                assemble(*pending.pop(0))
            pending.append((work, slot))

    def drain():
        while pending:
            assemble(*pending.pop(0))

    log(f"rank {rank}/{world}: {cfg_name} {W}x{H} spp_total={spp_total} depth={D} rows={rows} "
        f"row_block={rb} scaling={args.scaling}")
    # at least one warmup step per render stream: a stream's first launch grows the
    # stream-ordered pool for its per-launch buffers (overflow stack, sample planes)
    warmup = max(args.warmup, nstreams)
    for k in range(warmup):
        step(k)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    rays.zero_()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(warmup + k, ev[k])
    drain()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / max(1, args.steps)

    stats = torch.tensor([elapsed, float(rays.item()), kernel_ms], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
    if world > 1:
        t = stats[0:1].clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        r = stats[1:2].clone()
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        km = stats[2:3].clone()
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        stats = torch.cat([t, r, km])
    elapsed, total_rays, kernel_ms = (float(x) for x in stats.tolist())

    if rank == 0:
        value = total_rays / elapsed / 1e6
        pix_samples = rows * W * spp_total                     # one launch on rank 0
        alg_bytes = BYTES_PER_PIXEL_SAMPLE * pix_samples
        achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
        traffic, traffic_src = read_traffic(f"{cfg_name}_n{world}")
        valu = read_valu(f"{cfg_name}_n{world}")
        if valu:   # the committed launch's VALU instructions over this run's wall time per launch
            valu["issue_frac_effective"] = round(valu["valu_insts_per_launch"] / (elapsed / args.steps)
                                                 / (256 * 4 * 2.4e9 / 2), 4)
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: procedural sphere scene (no dataset), per-pixel seeded XorShift32 streams",
            "config": {
                "workload": f"{cfg_name}: {W}x{H}, {cfg['spp']} spp per GPU, {D} bounces, "
                            f"{'reference 9-sphere scene' if cfg['scene'] == 'default' else 'random_scene(1000, seed=1)'}",
                "width": W, "height": H, "spp_per_gpu": cfg["spp"], "spp_total": spp_total, "max_depth": D,
                "rays_per_step": int(total_rays / args.steps),
                "parallelism": f"rows: row-block-cyclic x{world} (block {rb}), RCCL gather to rank 0"
                if world > 1 else ("single GPU" if shards == 1 else
                                   f"DIAGNOSTIC: rank 0's shard of {shards} (block {rb}), no gather"),
                "scene_reads": "global" if args.scene_global else "LDS-staged",
                "reserved_cus": reserve,
                "render_streams": nstreams,
                "kernel": args.kernel,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": traffic,
                "kernel": kernel_name(args.kernel, spp_total),
                "kernel_ms": round(kernel_ms, 4),
                "algorithmic_bytes_per_launch": alg_bytes,
                "effective_ms_per_launch": round(elapsed / args.steps * 1e3, 4),
                "achieved_effective": round(alg_bytes / (elapsed / args.steps) / 1e9, 3),
                "note": "24 B per pixel-sample (SURVEY 8(d)); the path is VALU-bound, HBM frac is "
                        "reported as north_star asks" + (f"; traffic from {traffic_src}" if traffic_src else "")
                        + (f"; consecutive steps run on {nstreams} streams and their launches overlap "
                           "(each fills the CU slots the previous one frees in its tail), so kernel_ms "
                           "includes the overlap; achieved_effective uses the wall time per launch"
                           if nstreams > 1 else ""),
            },
            "valu": valu,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if rstream is not None:
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
        rstream.close()
    lrt.ShutdownTest()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
