#!/usr/bin/env python3
"""bench.py — throughput of the MI355X path tracer on BASELINE.json's headline metric.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5] [--scaling strong|weak]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

A step is one pass of the hot path over one batch: every rank renders its
row-block-cyclic share of the config's W x H image at the config's spp (one kernel
launch). For N > 1 the frame is assembled on rank 0 by the renders themselves: each
rank's render stores its finished pixels into rank 0's frame over xGMI (IPC-mapped;
--exchange rccl instead packs to RGB, gathers over RCCL and assembles with the unshard
kernel, the gather of step k overlapping the render of step k+1); the timed region ends when
every rank's last render (and gather/assembly) has completed.

Scaling is STRONG by default: the frame (W x H x spp) is fixed and split over the N
GPUs, so config 2 at N = 8 is still 1280x720 at 4 spp (each GPU renders 1/8 of the
rows) and config 5 is 7680x4320 at 256 spp in total. --scaling weak keeps the per-GPU
work fixed instead (N x spp samples per pixel).

`value` = counted rays of all ranks / max-over-ranks wall time of the K steps, in
Mray/s, the reference's own formula (src/cpu/main.cpp:188-189; rays counted as
parallel.cpp:122,204). Inputs are resident in HBM (the scene is uploaded once); no
host transfer is inside the timed region.

Besides the timed region (unless --no-extra-legs; the DrawTest legs first, then the W warmup
steps, then the end-to-end and launch-alone legs, then the K timed steps -- the ~35 launches of
those legs hold the render's load while the power controller raises the shader clock, which
otherwise ramps through a short timed region, profiles/r6_g):
  * `ms_per_launch_alone`: the same launches one at a time on one stream, each kernel
    bracketed by HIP events the library records on that stream right around it
    (lrt_kernel_timing) -- the duration the roofline objects divide by; `ms_per_call_alone`:
    the same launches with the events around the whole render call (its other stream
    commands and dispatch included);
  * `end_to_end`: render (+ gather and assembly) + the D2H copy of the frame into pinned
    host memory on rank 0 (N = 1: packed to RGB, 12 B/pixel, 4 frames in flight), beside the
    box's own pinned D2H bandwidth (`copy_ceiling_gbs`);
  * `cpu_baseline` (all host cores) and `cpu_baseline_1core`: the reference's own
    TraceRowJob body (oracle/_ref, rank 0 at N = 1 only, before the GPU is touched).

Rank 0 prints ONE JSON line on stdout; progress goes to stderr.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
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
# timed steps by default: a timed region of tens of ms (config 2: 200 x 0.22 ms)
DEFAULT_STEPS = {2: 200, 3: 40, 4: 10, 5: 3}
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md, chip-level parameters (spec)
BYTES_PER_PIXEL_SAMPLE = 24.0    # 12 B read + 12 B write of RGB per pixel-sample
# VALU: 256 CUs x 4 SIMD32 x 32 lanes per clock x 2.4 GHz = 78.6 T lane-operations/s
# (the 157.3 TFLOP/s FP32 vector peak of MI355X_MICROARCH.md counts an FMA as 2)
VALU_LANE_PEAK_T = 256 * 4 * 32 * 2.4e9 / 1e12
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2   # wave64 VALU instructions/s (2 cycles each per SIMD)
FP32_PEAK_T = 157.3              # MI355X_MICROARCH.md: peak FP32 (vector), TFLOP/s
# algorithmic FLOPs per counted ray = 17 per sphere test (HitSphere, maths.cpp:54-59,
# one per sphere of the linear scan) + ~60 of shading = 213 for the reference's 9-sphere scene
ALG_FLOP_PER_SPHERE, ALG_FLOP_SHADING = 17, 60
PMC_INDEX = os.path.join(ROOT, "profiles", "pmc_index.json")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Watchdog:
    """Bounds every phase of the run (the first multi-GPU run on the driver's 8-GPU node must
    end in a diagnosable line, not a hung job): enter(name) starts a phase with its own time
    limit (LRT_BENCH_TIMEOUT, seconds, default 600); when one expires on any rank, that rank
    reports the phase on stderr and rank 0 prints a partial JSON line naming it (value null),
    then the process exits with status 3. A rank blocked in a collective because a peer
    stalled times out in its own phase, so rank 0 always reports. The thread only reads state
    and prints; nothing is re-executed. LRT_BENCH_STALL=<phase> (tests) makes every rank, or
    rank LRT_BENCH_STALL_RANK, hang at the start of that phase."""

    def __init__(self, rank, world, base):
        self.rank, self.world, self.base = rank, world, base
        self.limit = float(os.environ.get("LRT_BENCH_TIMEOUT", "600"))
        self.phase, self.deadline, self.started = "start", time.monotonic() + self.limit, time.monotonic()
        self.done = []   # phases completed, in order
        self.lock = threading.Lock()
        self.stall = os.environ.get("LRT_BENCH_STALL")
        self.stall_rank = os.environ.get("LRT_BENCH_STALL_RANK")
        threading.Thread(target=self._run, name="bench-watchdog", daemon=True).start()

    def enter(self, name, limit=None):
        with self.lock:
            if self.phase != "start":
                self.done.append(self.phase)
            self.phase = name
            self.started = time.monotonic()
            self.deadline = self.started + (limit or self.limit)
        if self.stall == name and (self.stall_rank is None or int(self.stall_rank) == self.rank):
            log(f"rank {self.rank}: LRT_BENCH_STALL={name}: hanging here")
            while True:
                time.sleep(3600)

    def _run(self):
        while True:
            time.sleep(0.25)
            with self.lock:
                expired = time.monotonic() > self.deadline
                phase, waited, done = self.phase, time.monotonic() - self.started, list(self.done)
            if expired:
                break
        msg = f"timeout: phase '{phase}' ran {waited:.1f} s on rank {self.rank} of {self.world} (limit {self.limit:.0f} s)"
        log(msg)
        if self.rank != 0:   # rank 0 reports first: the launcher stops every rank once one has exited
            time.sleep(min(10.0, self.limit))
        if self.rank == 0:
            line = dict(self.base)
            line.update({"value": None, "error": msg, "failed_phase": phase, "phases_completed": done})
            print(json.dumps(line), flush=True)
        os._exit(3)


def workload(config: int, world: int = 1, scaling: str = "strong", spp=None, depth=None, shard_of: int = 1):
    """The per-rank render of `config` at N = world: shards = row shards of the frame,
    spp_total = samples per pixel of the whole frame (each rank renders its rows at that
    spp). Pure function (tested on CPU)."""
    if scaling not in ("strong", "weak"):
        raise ValueError("scaling must be strong or weak")
    cfg = dict(CONFIGS[config])
    if spp:
        cfg["spp"] = spp
    if depth is not None:
        cfg["depth"] = depth
    shards = world if world > 1 else max(1, shard_of)
    cfg["shards"] = shards
    cfg["spp_total"] = cfg["spp"] * shards if scaling == "weak" else cfg["spp"]
    cfg["pixel_samples_total"] = cfg["width"] * cfg["height"] * cfg["spp_total"]
    return cfg


def cpu_baseline(cfg, budget_s: float, cores: int):
    """Time the reference's own TraceRowJob body (oracle/_ref: libref.so, or libref1000.so
    whose static scene is random_scene(1000, 1)) in forked worker processes with per-pixel
    seeds -- or the C restatement if _ref is absent -- on this host, for about budget_s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle  # test infrastructure: the baseline leg only

    w, h, depth = cfg["width"], cfg["height"], cfg["depth"]
    n = 9 if cfg["scene"] == "default" else 1000
    if n == 9:
        x0, xc, y0, yc = 0, w, 0, h
        spheres = mats = None
        what = f"full {w}x{h} frames"
    else:
        from learnraytracing_amd.scene import random_scene, scene_arrays
        s, m = scene_arrays(*random_scene(1000, 1))
        spheres, mats = np.array(s, np.float32), np.array(m, np.float32)
        xc, yc = 128, 32
        x0, y0 = (w - xc) // 2, (h - yc) // 2
        what = f"{xc}x{yc} centre crop of {w}x{h}"
    use_ref = oracle.have_ref(n)
    kind = "reference" if use_ref else "port"
    rays = 0
    frames = 0
    t0 = time.perf_counter()
    while True:
        if use_ref:
            _, r = oracle.ref_render_p(w, h, 1, depth, frames, x0, xc, y0, yc, procs=cores, n=n)
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
    src = (f"oracle/_ref/{'libref.so' if n == 9 else 'libref1000.so'} (reference maths.cpp+parallel.cpp, clang -O2)"
           if use_ref else "oracle/lrt_oracle.c")
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mray/s", "cores": cores, "kind": kind,
            "sample": f"{what}, {frames} frame(s) x 1 spp, {depth} bounces, per-pixel seeds, "
                      f"{rays} rays in {dt:.2f} s, {cores} {'processes' if use_ref else 'threads'}; {src}"}


def drawtest_leg(lrt, frames: int = 200):
    """lrt_draw_test as src/cpu/main.cpp drives DrawTest: one pageable `new float[]` backbuffer
    (main.cpp:40) handed to every frame (main.cpp:165) at 1280x720, kMaxDepth 20, frameCount
    counting up. Each call page-locks the buffer for itself only (nothing is kept between
    calls). The first two frames are untimed; the rate is rays / wall time over the next
    `frames` frames, the same unit as cpu_reference_drawtest (the reference's DrawTest on the
    host cores)."""
    import numpy as np

    from learnraytracing_amd import _lib as L
    w, h = 1280, 720
    lrt.set_scene(*lrt.default_scene())   # DrawTest renders the reference's scene (parallel.cpp:15-51)
    bb = np.zeros(w * h * 4, np.float32)
    for f in range(2):
        lrt.DrawTest(0.0, f, w, h, bb)
    rays = 0
    t0 = time.perf_counter()
    for f in range(2, 2 + frames):
        rays += lrt.DrawTest(0.0, f, w, h, bb)
    dt = time.perf_counter() - t0
    info = L.last_launch()
    return {"value": round(rays / dt / 1e6, 1), "unit": "Mray/s", "ms_per_frame": round(dt / frames * 1e3, 4),
            "frames": frames, "host_path": info.get("host"), "lookahead": info.get("lookahead"),
            "what": "lrt_draw_test(0, f, 1280, 720, pageable backbuffer) per frame, host wall clock (H2D of the "
                    "previous values, render, lerp written back over PCIe)"}


def cpu_reference_drawtest(cores: int, budget_s: float):
    """Context beside cpu_baseline: the reference as it ships -- its own
    DrawTest (parallel.cpp:297-323) with enkiTS over `cores` workers, kMaxDepth 20 and the
    shared racy RNG, at main.cpp's 1280x720, 1 spp per call, progressive frames on one
    buffer. Not the same work as the metric (20 bounces, racy streams), so never a ratio."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the baseline legs only

    if not oracle.have_ref(9):
        return None
    rate, frames, rays, dt = oracle.ref_drawtest_rate(1280, 720, budget_s, cores)
    return {"value": round(rate, 3), "unit": "Mray/s", "cores": cores, "kind": "reference",
            "sample": f"reference DrawTest (enkiTS, {cores} workers, kMaxDepth 20, shared RNG) at 1280x720, "
                      f"{frames} progressive frame(s) x 1 spp, {rays} rays in {dt:.2f} s; oracle/_ref/libref.so"}


def scene_reads(info: dict) -> str:
    """Where the launched instance reads the scene from, taken from lrt_last_launch()'s
    lds= / acc= words (not from the flags asked for)."""
    lds, bvh = info.get("lds"), info.get("bvh")
    if info.get("acc") == "grid":
        return ("uniform grid: cell lists + cell-ordered spheres through L1/L2 (global memory), materials "
                + ("LDS-staged" if lds == "1" else "through L1/L2"))
    if bvh == "1":
        return ("BVH nodes + leaf spheres through L1/L2 (global memory), materials "
                + ("LDS-staged" if lds == "1" else "through L1/L2"))
    if lds == "1":
        return "LDS-staged spheres, materials and lights"
    if lds == "0":
        return "global memory (L1/L2)"
    return "unknown"


def read_pmc(key: str):
    """Per-launch counters of trace_kernel for `key` (e.g. "config2_n1") from the committed
    rocprofv3 passes (profiles/pmc_index.json -> profiles/<run>/summary_<config>.json)."""
    try:
        with open(PMC_INDEX) as f:
            src = json.load(f)[key]
        p = os.path.join(ROOT, "profiles", src)
        with open(p) as f:
            s = json.load(f)
        s["path"] = os.path.relpath(p, ROOT)
        return s
    except (OSError, ValueError, KeyError):
        return None


def base_line(args, world, cfg):
    """The fields every line carries, the failure lines included (value null)."""
    return {"metric": METRIC, "value": None, "unit": "Mray/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"config{args.config}: {cfg['width']}x{cfg['height']}, "
                                   f"{cfg['spp_total']} spp, {cfg['depth']} bounces"}}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(args, argv) -> int:
    """`--gpus N` (N > 1) without a launcher: start N ranks as ONE child process,
    `python -m torch.distributed.run --nproc-per-node N ... bench.py <same args>`, forward rank
    0's JSON line and return the child's exit code. This process never imports torch or touches
    a GPU (the child is started, not exec'd). If the child cannot start, or ends without a line,
    print a line with value null naming the reason and return non-zero: a run asked for N GPUs
    never reports a one-GPU number."""
    import collections
    import subprocess

    n = args.gpus
    base = base_line(args, n, workload(args.config, n, args.scaling, args.spp, args.depth))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    log(f"bench: --gpus {n} without a launcher: starting {n} ranks: {' '.join(cmd)}")

    def fail(reason, rc):
        line = dict(base)
        line.update({"error": reason, "launcher": "bench.py self-launch (torch.distributed.run)"})
        print(json.dumps(line), flush=True)
        return rc if rc else 1

    try:
        p = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, bufsize=1)
    except OSError as e:
        return fail(f"could not start torch.distributed.run: {e}", 2)
    tail = collections.deque(maxlen=30)

    def pump_err():
        for ln in p.stderr:
            tail.append(ln.rstrip())
            sys.stderr.write(ln)
            sys.stderr.flush()

    t = threading.Thread(target=pump_err, daemon=True)
    t.start()
    lines = 0
    for ln in p.stdout:
        if ln.startswith("{"):
            lines += 1
            sys.stdout.write(ln)
            sys.stdout.flush()
        else:
            sys.stderr.write(ln)
    rc = p.wait()
    t.join(timeout=5)
    if lines == 0:
        return fail(f"the {n}-rank run exited with status {rc} without a result line; stderr tail: "
                    + " | ".join(list(tail)[-8:]), rc)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: per config, a timed region of tens of ms: config 2 200 steps "
                         "-- 20 steps of 0.22 ms left launch and drain edges at ~8 %% of a 4.5-ms region)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--streams", type=int, default=2,
                    help="render streams the steps rotate over: step k+1 starts in the CU slots step k's "
                         "persistent grid frees during its tail (each step writes its own buffer)")
    ap.add_argument("--spp", type=int, default=None, help="diagnostic: override the config's spp")
    ap.add_argument("--depth", type=int, default=None, help="diagnostic: override the config's bounce budget")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="diagnostic (1 process): render only rank 0's shard of an N-GPU run, no gather -- "
                         "the per-GPU render at N GPUs, measured on one")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra-legs", action="store_true",
                    help="only the timed region (profiling runs): no launch-alone, end-to-end or CPU legs")
    ap.add_argument("--cpu-budget", type=float, default=None, help="seconds of all-core CPU-baseline timing")
    ap.add_argument("--scene-global", action="store_true", help="read spheres from global memory, not LDS")
    ap.add_argument("--exchange", choices=["remote", "rccl"], default="remote",
                    help="N > 1 frame assembly: remote = each rank's render stores its finished pixels straight "
                         "into rank 0's frame over xGMI (IPC-mapped, lrt_render_device_to_frame); rccl = pack to "
                         "RGB, RCCL gather to rank 0, unshard kernel")
    ap.add_argument("--reserve-cus", type=int, default=None,
                    help="CUs the render stream leaves free for other streams (default 0)")
    ap.add_argument("--kernel", choices=["auto", "v0", "wf", "pool"], default="auto",
                    help="auto: the library's policy; v0: frame lanes; wf: wavefront; "
                         "pool: sample-pool regeneration (A/B)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = DEFAULT_STEPS.get(args.config, 20)

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    cfg = workload(args.config, world, args.scaling, args.spp, args.depth, args.shard_of)
    cfg_name = f"config{args.config}"
    if world != args.gpus:   # a launcher's rank count and --gpus disagree: refuse, never relabel
        if rank == 0:
            line = base_line(args, args.gpus, cfg)
            line["error"] = f"WORLD_SIZE={world} but --gpus {args.gpus}: the launcher and --gpus disagree"
            print(json.dumps(line), flush=True)
        log(f"error: WORLD_SIZE={world} but --gpus {args.gpus}")
        sys.exit(2)
    extra = not args.no_extra_legs
    wd = Watchdog(rank, world, base_line(args, world, cfg))

    # CPU baselines first: rank 0 at N=1 only, before anything touches the GPU.
    cpu = cpu1 = cpu_dt = None
    if rank == 0 and world == 1 and extra and not args.no_cpu_baseline:
        wd.enter("cpu_baseline")
        cores = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
        cores = max(1, min(cores, os.cpu_count() or 1))
        budget = args.cpu_budget if args.cpu_budget is not None else max(1.5, 15.0 / cores)
        log(f"cpu baseline ({budget:.1f} s on {cores} cores, then 6 s on 1 core) ...")
        cpu = cpu_baseline(cfg, budget, cores)
        cpu1 = cpu_baseline(cfg, 6.0, 1)
        log(f"cpu baseline: {cpu['value']:.1f} Mray/s ({cpu['kind']}, {cores} cores), 1 core {cpu1['value']:.2f}")
        cpu_dt = cpu_reference_drawtest(cores, 3.0)
        if cpu_dt:
            log(f"reference DrawTest (enkiTS, {cores} threads): {cpu_dt['value']:.1f} Mray/s")

    wd.enter("import_torch", max(wd.limit, 300.0))   # (a fresh box pages the image in: 1-2 minutes)
    import datetime

    import torch
    import torch.distributed as dist

    backend = os.environ.get("LRT_DIST_BACKEND", "nccl")   # nccl = RCCL; gloo only to rehearse on 1 GPU
    # LRT_BENCH_SAME_GPU=1 puts every rank on GPU 0 (rehearsing the RCCL path on a 1-GPU box)
    one_gpu = backend != "nccl" or os.environ.get("LRT_BENCH_SAME_GPU") == "1"
    gpu = 0 if one_gpu else local_rank
    def check_devices():
        """Refuse a world the visible GPUs cannot hold (one rank per GPU over RCCL), rank 0
        printing the line -- never fewer GPUs than the line's n_gpus. (Counting devices does
        not initialise the GPU.)"""
        ndev = torch.cuda.device_count()
        need = 1 if one_gpu else world
        if ndev >= need:
            return
        msg = f"--gpus {world} needs {need} visible GPU(s), {ndev} visible"
        if rank == 0:
            line = dict(wd.base)
            line.update({"error": msg, "failed_phase": "device_count"})
            print(json.dumps(line), flush=True)
        log(f"rank {rank}: error: {msg}")
        os._exit(2)

    if world > 1:   # the rendezvous itself is bounded too (the store's timeout)
        wd.enter("init_process_group")
        tmo = datetime.timedelta(seconds=wd.limit * 1.5)   # (the watchdog reports first)
        if backend == "nccl":
            check_devices()
            torch.cuda.set_device(gpu)
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
    wd.enter("device_init", max(wd.limit, 300.0))
    check_devices()
    torch.cuda.set_device(gpu)
    import learnraytracing_amd as lrt
    from learnraytracing_amd import _lib as L
    from learnraytracing_amd.dist import gather_to_root, max_shard_rows, open_shared_frames, shard_rows
    from learnraytracing_amd.renderer import pack_rgb_tensor, render_tensor_to_frame, unshard_rgb_tensor

    lrt.InitializeTest()
    # ---- the reference API as its own caller uses it (rank 0, N = 1): DrawTest per frame, on
    # one device and split over two contexts of it (lrt_initialize_devices([0, 0]): the
    # multi-device host path's own cost, rehearsed on the one GPU this process drives). Run
    # first, on their own context: the config's render below starts from a fresh one.
    drawtest = drawtest_multi = None
    if extra and world == 1:
        wd.enter("drawtest")
        drawtest = drawtest_leg(lrt)
        torch.cuda.synchronize()
        lrt.ShutdownTest()
        lrt.InitializeDevices([gpu, gpu])
        drawtest_multi = drawtest_leg(lrt, frames=100)
        drawtest_multi["devices"] = f"[{gpu}, {gpu}] (lrt_initialize_devices, direct exchange)"
        lrt.ShutdownTest()
        lrt.InitializeTest()
        torch.cuda.synchronize()
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
    shards, spp_total = cfg["shards"], cfg["spp_total"]
    rb = H if shards == 1 else args.row_block
    max_rows = max_shard_rows(H, rb, shards)
    rows = shard_rows(H, rb, shards, rank)
    flags = (1 if args.scene_global else 0) | {"auto": 0, "v0": 2, "wf": 256, "pool": 512}[args.kernel]
    job = lrt.Job(width=W, height=H, frame0=0, frames=spp_total, max_depth=D, row_block=rb,
                  row_period=shards, row_phase=rank, row_count=rows, flags=flags)
    dev = torch.device("cuda", torch.cuda.current_device())
    nstreams = max(1, args.streams)
    nslots = max(2, nstreams)
    # the end-to-end leg's frames in flight: a render must not wait for the copy of the frame
    # before it (2 slots serialised render and copy: 0.43 = 0.225 + 0.203 ms/step, profiles/r6_e);
    # a multiple of the render streams, so that slot s is always rendered on stream s % nstreams
    e2e_slots = 2 * nstreams if world == 1 else nslots
    bufs = [torch.zeros((max_rows, W, 4), dtype=torch.float32, device=dev) for _ in range(max(nslots, e2e_slots))]
    rays = torch.zeros(1, dtype=torch.int64, device=dev)
    # remote exchange: rank 0's frames mapped into every rank; each render stores its finished
    # pixels there itself (no pack, gather or unshard launch per step)
    remote = world > 1 and args.exchange == "remote"
    # with N > 1 both exchanges are timed (the other one as a second leg, unless
    # --no-extra-legs): the fused remote stores, and north_star's RCCL gather over xGMI
    both = world > 1 and extra
    shared = None
    ipc_refused = None
    if remote or both:
        wd.enter("open_shared_frames")
        dev_b = dev if backend == "nccl" else torch.device("cpu")
        # LRT_BENCH_FORCE_IPC_FAIL=1 (tests): every rank reports a refused mapping
        shared = open_shared_frames(W, H, nslots, rank, dev_b,
                                    force_fail=os.environ.get("LRT_BENCH_FORCE_IPC_FAIL") == "1")
        if shared is None:   # IPC mapping refused on some rank: the RCCL exchange instead
            log("note: IPC frame mapping failed on a rank; falling back to --exchange rccl")
            ipc_refused = "lrt_ipc_open refused on at least one rank: the remote-store exchange was not run"
            remote = False
    have_rccl = world > 1 and (not remote or both)
    # the RCCL exchange carries RGB only (lrt_pack_rgb): 12 of the 16 bytes per pixel cross xGMI
    packed = [torch.empty((max_rows, W, 3), dtype=torch.float32, device=dev) if have_rccl else None
              for _ in range(nslots)]
    gathered = [torch.empty((world, max_rows, W, 3), dtype=torch.float32, device=dev) if rank == 0 and have_rccl
                else None for _ in range(nslots)]
    frames_out = [torch.empty((H, W, 4), dtype=torch.float32, device=dev) if rank == 0 and have_rccl else None
                  for _ in range(nslots)]
    stream = torch.cuda.current_stream(dev)
    # render streams (the first is the current stream); frame assembly and D2H on their own
    rstreams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(nstreams - 1)]
    for rs_ in rstreams[1:]:   # the buffers' zero fills (current stream) come before any render
        rs_.wait_stream(stream)
    astream = torch.cuda.Stream(device=dev) if world > 1 else stream
    cstream = torch.cuda.Stream(device=dev)
    host = None   # pinned frame copies (end-to-end leg)
    e2e_rgb = []  # N = 1: the packed RGB frames the end-to-end leg copies
    # N = 1, LRT_BENCH_E2E=fused (A/B): no copy -- the render's lerp stores each pixel (RGBA) straight
    # into the pinned host frame over PCIe (lrt_render_device_to_frame)
    e2e_fused = os.environ.get("LRT_BENCH_E2E", "copy") == "fused"

    def d2h_ceiling(src, dst, reps=10):
        """Pinned D2H bandwidth of this box (GB/s): reps copies of src into the page-locked dst
        on the copy stream, timed with events -- the end-to-end leg's own ceiling."""
        with torch.cuda.stream(cstream):
            dst.copy_(src, non_blocking=True)   # (first touch of the pinned pages, untimed)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cstream)
            for _ in range(reps):
                dst.copy_(src, non_blocking=True)
            e1.record(cstream)
        e1.synchronize()
        return src.numel() * 4 * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    pending = []   # (mode, work, slot, d2h, rdone) of steps whose gather / D2H is not yet enqueued
    slot_done = {}   # (slot, d2h) -> event: that slot's gather / assembly / copy has completed

    def finish(mode, work, slot, d2h, rdone):
        """Assemble slot's frame on rank 0 (after its gather), then optionally copy it to
        pinned host memory; the slot's next render waits for both."""
        done = None
        gather_ex = mode == "rccl"
        if gather_ex:
            done = torch.cuda.Event()
            with torch.cuda.stream(astream):
                if work is not None:
                    work.wait()   # the assembly stream waits for the gather
                if rank == 0:
                    unshard_rgb_tensor(gathered[slot], frames_out[slot], W, H, rb, world, astream)
                done.record(astream)
        if d2h and rank == 0:
            cstream.wait_event(done if done is not None else rdone)
            with torch.cuda.stream(cstream):
                if not (world == 1 and e2e_fused):
                    host[slot].copy_(frames_out[slot] if gather_ex else e2e_rgb[slot] if world == 1 else bufs[slot],
                                     non_blocking=True)
            done = torch.cuda.Event()
            done.record(cstream)
        if done is not None:   # the slot's next render waits for its gather / copy (step())
            slot_done[(slot, d2h)] = done

    def step(k, mode, d2h=False):
        """mode: "remote" (stores into rank 0's IPC frame), "rccl" (pack + gather + unshard), or
        "local" (N = 1). d2h: the end-to-end leg, which cycles over e2e_slots buffers."""
        slot = k % (e2e_slots if d2h else nslots)
        rs = rstreams[k % nstreams]
        prev = slot_done.pop((slot, d2h), None)
        if prev is not None:   # (only this render waits: the stream's other renders run on)
            rs.wait_event(prev)
        if mode == "remote":
            render_tensor_to_frame(job, bufs[slot], rays, shared.ptrs[slot], rs)
        elif d2h and world == 1 and e2e_fused:   # the render's own stores land in pinned host memory
            render_tensor_to_frame(job, bufs[slot], rays, host[slot].data_ptr(), rs)
        else:
            lrt.render_tensor(job, bufs[slot], rays, rs)
        rdone = None
        if d2h and world == 1:
            if not e2e_fused:
                pack_rgb_tensor(bufs[slot], e2e_rgb[slot], rs)
            rdone = torch.cuda.Event()
            rdone.record(rs)
        work = None
        if mode == "rccl":
            with torch.cuda.stream(rs):   # the gather is ordered after this step's render
                pack_rgb_tensor(bufs[slot], packed[slot], rs)
                _, work = gather_to_root(packed[slot], max_rows, world, rank, gathered=gathered[slot], async_op=True)
        while pending:
            finish(*pending.pop(0))
        pending.append((mode, work, slot, d2h, rdone))

    def drain():
        while pending:
            finish(*pending.pop(0))

    def sync_all():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    log(f"rank {rank}/{world}: {cfg_name} {W}x{H} spp_total={spp_total} depth={D} rows={rows} "
        f"row_block={rb} scaling={args.scaling}")
    # at least one warmup step per render stream: a stream's first launch grows the
    # stream-ordered pool for its per-launch buffers (overflow stack, sample planes)
    warmup = max(args.warmup, nstreams)

    warm = {}

    def warmup_steps(mode):
        """The W untimed warmup steps of `mode`; their own time is kept (warm[mode], ms per step)
        as the record of a cold start (first launches record and sort the tile order)."""
        wd.enter(f"warmup_{mode}")
        sync_all()
        tw = time.perf_counter()
        for k in range(warmup):
            step(k, mode)
        drain()
        torch.cuda.synchronize()
        warm[mode] = (time.perf_counter() - tw) / warmup * 1e3
        sync_all()

    def timed(mode):
        """K timed steps of `mode`: (seconds, counted rays of this rank)."""
        rays.zero_()
        sync_all()
        wd.enter(f"timed_{mode}")
        t0 = time.perf_counter()
        for k in range(args.steps):
            step(warmup + k, mode)
        drain()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if world > 1:
            dist.barrier()
        return t1 - t0, float(rays.item())

    mode = ("remote" if remote else "rccl") if world > 1 else "local"
    warmup_steps(mode)
    remote = mode == "remote"
    # ---- extra legs, BEFORE the timed region: end to end (D2H included), then each launch alone
    # (the roofline's duration). Under a render's full load the shader clock starts near 2.18 GHz
    # and the power controller raises it to ~2.39 GHz over ~50 launches (~13 ms); the cycles per
    # wave stay the same (tools/clock_ramp.py, profiles/r6_g). Timed right after W warmup steps, a
    # 20-step region measured that ramp (0.241 against 0.224 ms/step at the held clock). These
    # legs are the same render (the alone leg at least 64 launches); the timed steps are unchanged.
    alone_ms = e2e_s = call_ms = None
    # the alone leg averages at least LRT_BENCH_ALONE_MIN launches (default 64; K if larger)
    alone_n = max(args.steps, int(os.environ.get("LRT_BENCH_ALONE_MIN", "64")))
    copy_ceiling = host_identical = None
    e2e_steps = 0

    def leg_end_to_end():
        nonlocal host, copy_ceiling, host_identical, e2e_steps, e2e_s
        if rank == 0:
            # N = 1: the frame leaves as packed RGB (12 of the 16 B per pixel: the render never
            # writes alpha; lrt_pack_rgb on the render stream); N > 1: rank 0's assembled RGBA frame
            shape = (H, W, 4) if world > 1 or e2e_fused else tuple(bufs[0].shape[:2]) + (3,)   # --shard-of: the shard
            host = [torch.empty(shape, dtype=torch.float32, pin_memory=True) for _ in range(e2e_slots)]
            if world == 1:
                e2e_rgb[:] = [torch.empty(shape, dtype=torch.float32, device=dev) for _ in range(e2e_slots)]
                copy_ceiling = d2h_ceiling(e2e_rgb[0], host[0])
        e2e_steps = max(1, min(args.steps, 20))
        wd.enter("end_to_end")
        if remote:   # a frame is complete once every rank's render of it is: barrier, then D2H
            def e2e_step(k):
                step(k, mode)
                sync_all()
                if rank == 0:
                    host[k % nslots].copy_(shared.tensor(k % nslots))
            for k in range(nslots):
                e2e_step(k)
            sync_all()
            t2 = time.perf_counter()
            for k in range(e2e_steps):
                e2e_step(k)
            e2e_s = time.perf_counter() - t2
            dist.barrier()
        else:
            for k in range(e2e_slots):   # untimed: each pinned buffer's first copy maps its pages
                step(k, mode, d2h=True)
            drain()
            sync_all()
            t2 = time.perf_counter()
            for k in range(e2e_steps):
                step(k, mode, d2h=True)
            drain()
            torch.cuda.synchronize()
            e2e_s = time.perf_counter() - t2
            if world == 1:   # the last frame on the host, bit for bit the device's RGB
                last = (e2e_steps - 1) % e2e_slots
                hv = host[last][..., :3] if e2e_fused else host[last]
                host_identical = bool(torch.equal(hv.contiguous().view(torch.int32),
                                                  bufs[last][..., :3].contiguous().cpu().view(torch.int32)))
            if world > 1:
                dist.barrier()
        drain()
        sync_all()

    def leg_alone():
        nonlocal call_ms, alone_ms
        wd.enter("launch_alone")
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(alone_n)]
        scratch = torch.zeros(1, dtype=torch.int64, device=dev)
        L.check(L.lib().lrt_kernel_timing(1))
        for k in range(alone_n):
            ev[k][0].record(stream)
            if remote:
                render_tensor_to_frame(job, bufs[0], scratch, shared.ptrs[0], stream)
            else:
                lrt.render_tensor(job, bufs[0], scratch, stream)
            ev[k][1].record(stream)
        torch.cuda.synchronize()
        call_ms = sum(a.elapsed_time(b) for a, b in ev) / alone_n
        kt = (ctypes.c_float * alone_n)()
        nk = ctypes.c_int(0)
        L.check(L.lib().lrt_kernel_times(kt, alone_n, ctypes.byref(nk)))
        L.check(L.lib().lrt_kernel_timing(0))
        # one render kernel per launch: the kernel's own events; else the call's
        alone_ms = sum(kt[:nk.value]) / nk.value if nk.value == alone_n else call_ms


    # LRT_BENCH_LEGS (A/B of the order; default: both legs before the timed steps)
    legs = os.environ.get("LRT_BENCH_LEGS", "e2e,alone,timed").split(",") if extra else ["timed"]
    for leg in legs[:legs.index("timed")]:
        {"e2e": leg_end_to_end, "alone": leg_alone}[leg]()
    elapsed, timed_rays = timed(mode)
    launch_info = L.last_launch()
    for leg in legs[legs.index("timed") + 1:]:
        {"e2e": leg_end_to_end, "alone": leg_alone}[leg]()
    exchange_legs = None
    if both and shared is None:   # the RCCL leg alone: the line still carries the exchange's timing
        wd.enter("exchange_legs")
        st = torch.tensor([elapsed, timed_rays], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        mx, sm = st.clone(), st.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        exchange_legs = {
            "primary": mode, "frames_identical": None,
            "legs": {"rccl": {"ms_per_step": round(float(mx[0]) / args.steps * 1e3, 4),
                              "value": round(float(sm[1]) / float(mx[0]) / 1e6, 3), "unit": "Mray/s",
                              "what": "pack to RGB + RCCL gather (dist.gather over nccl = RCCL) to rank 0 + unshard"},
                     "remote": {"refused": ipc_refused}},
        }
    if both and shared is not None:
        # the other exchange, same steps; then both legs' assembled frames, bit for bit, on rank 0
        other = "rccl" if mode == "remote" else "remote"
        warmup_steps(other)
        e2, r2 = timed(other)
        wd.enter("exchange_legs")
        legs = {mode: (elapsed, timed_rays), other: (e2, r2)}
        st = torch.tensor([legs["remote"][0], legs["rccl"][0], legs["remote"][1], legs["rccl"][1]],
                          dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        mx, sm = st.clone(), st.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        same = None
        if rank == 0:
            a, b = shared.tensor(0)[..., :3].contiguous(), frames_out[0][..., :3].contiguous()
            same = bool(torch.equal(a.view(torch.int32), b.view(torch.int32)))
        exchange_legs = {
            "primary": mode,
            "frames_identical": same,
            "legs": {m: {"ms_per_step": round(float(mx[i]) / args.steps * 1e3, 4),
                         "value": round(float(sm[2 + i]) / float(mx[i]) / 1e6, 3), "unit": "Mray/s",
                         "what": ("each render stores its finished pixels into rank 0's frame over xGMI (IPC)"
                                  if m == "remote" else
                                  "pack to RGB + RCCL gather (dist.gather over nccl = RCCL) to rank 0 + unshard")}
                     for i, m in enumerate(("remote", "rccl"))},
        }
    torch.cuda.synchronize()

    wd.enter("stats")
    stats = torch.tensor([elapsed, timed_rays, alone_ms or 0.0, e2e_s or 0.0], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
    if world > 1:
        r = stats[1:2].clone()
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        stats = torch.cat([mx[0:1], r, mx[2:4]])
    elapsed, total_rays, alone_ms, e2e_s = (float(x) for x in stats.tolist())

    if rank == 0:
        value = total_rays / elapsed / 1e6
        rays_per_step = total_rays / args.steps
        ms_step = elapsed / args.steps * 1e3
        pix_samples = rows * W * spp_total                     # one launch on rank 0
        alg_bytes = BYTES_PER_PIXEL_SAMPLE * pix_samples
        key = f"{cfg_name}_n{shards}" if args.scaling == "strong" or shards == 1 else f"{cfg_name}_n{shards}_weak"
        pmc = read_pmc(key) if not (args.spp or args.depth is not None or args.kernel != "auto") else None
        if pmc and pmc.get("kernel") != launch_info.get("kernel"):
            pmc = None   # counters of another kernel than this run's
        kname = launch_info.get("kernel", "trace_kernel")
        dur_ms = alone_ms if alone_ms else ms_step
        hbm = {"bound": "hbm", "achieved": round(alg_bytes / (dur_ms * 1e-3) / 1e9, 3), "peak": HBM_PEAK_GBS,
               "unit": "GB/s", "frac": round(alg_bytes / (dur_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6),
               "traffic": pmc["hbm_bytes_per_launch"] if pmc and "hbm_bytes_per_launch" in pmc else None,
               "algorithmic_bytes_per_launch": alg_bytes,
               "note": "24 B per pixel-sample (SURVEY 8(d)) x the launch's pixel-samples over one launch's "
                       "duration alone (ms_per_launch_alone); traffic = corrected 2 x FETCH_SIZE + WRITE_SIZE "
                       "per launch from the committed PMC pass"}
        roof = hbm
        valu = None
        if pmc and "lane_ops_per_launch" in pmc:
            lane_ops = pmc["lane_ops_per_launch"]
            achieved_t = lane_ops / (dur_ms * 1e-3) / 1e12
            valu = {"bound": "valu", "achieved": round(achieved_t, 3), "peak": round(VALU_LANE_PEAK_T, 2),
                    "unit": "TFLOP/s", "frac": round(achieved_t / VALU_LANE_PEAK_T, 4),
                    "traffic": hbm["traffic"], "kernel": kname,
                    "lane_ops_per_launch": lane_ops,
                    "issue_frac": round(pmc["valu_insts_per_launch"] / (dur_ms * 1e-3) / VALU_ISSUE_PEAK, 4),
                    "lane_util": pmc["lane_util"],
                    "duration_ms": round(dur_ms, 4),
                    "source": pmc["path"],
                    "note": "ISSUED work, not algorithmic: FP32 VALU lane-operations/s = SQ_INSTS_VALU x 64 x "
                            "lane_util per launch (lane_util = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64), "
                            "committed PMC pass) over one launch's duration alone; peak = 256 CU x 4 SIMD x 32 "
                            "lanes x 2.4 GHz = 78.6 T lane-ops/s; frac = issue_frac x lane_util"}
        if cfg["scene"] == "default":
            # the algorithmic roofline of the prompt: SURVEY §8(d)'s FLOPs per counted ray x the rays
            # one launch counts (rank 0's launch) / that launch's duration alone, against the FP32
            # vector peak. (For the 1000-sphere scene §8(d)'s 17 N per ray is the linear scan's
            # work, which the BVH does not do; there the counter line above is the roofline.)
            nsph = 9
            flop_ray = ALG_FLOP_PER_SPHERE * nsph + ALG_FLOP_SHADING
            rays_launch = rays_per_step / max(1, world)
            alg_t = flop_ray * rays_launch / (dur_ms * 1e-3) / 1e12
            roof = {"bound": "valu", "achieved": round(alg_t, 3), "peak": FP32_PEAK_T, "unit": "TFLOP/s",
                    "frac": round(alg_t / FP32_PEAK_T, 4),
                    "traffic": hbm["traffic"], "kernel": kname,
                    "algorithmic_flop_per_ray": flop_ray,
                    "rays_per_launch": int(rays_launch),
                    "duration_ms": round(dur_ms, 4),
                    "note": f"ALGORITHMIC: SURVEY 8(d) {flop_ray} FLOP per counted ray (17 per sphere x {nsph} + 60 "
                            "shading) x the launch's counted rays over one launch's duration alone (HIP events on "
                            "its stream); peak = MI355X FP32 vector peak 157.3 TFLOP/s, which counts an FMA as 2 "
                            "(the bit-exact path is built with -ffp-contract=off, so its own ceiling is half that); "
                            "traffic = corrected HBM bytes per launch from the committed PMC pass"}
        elif valu:
            roof = valu
        # the same algorithmic work per step over the timed region's own step time: launches
        # overlap there (two render streams), so this is the rate the chip sustains, not a
        # launch's duration (the roofline object above keeps the prompt's per-launch form)
        piped = None
        if cfg["scene"] == "default":
            alg_step = (ALG_FLOP_PER_SPHERE * 9 + ALG_FLOP_SHADING) * rays_per_step / (ms_step * 1e-3) / 1e12
            peak_all = FP32_PEAK_T * world
            piped = {"bound": "valu", "achieved": round(alg_step, 3), "peak": peak_all, "unit": "TFLOP/s",
                     "frac": round(alg_step / peak_all, 4), "duration_ms": round(ms_step, 4),
                     "note": "213 FLOP per counted ray x rays per step (all ranks) / ms_per_step (pipelined "
                             "timed region), against the FP32 vector peak of the n_gpus GPUs"}
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": warmup,
            "ms_per_step": round(ms_step, 4),
            "ms_per_launch_alone": round(alone_ms, 4) if alone_ms else None,
            "ms_per_call_alone": round(call_ms, 4) if call_ms else None,
            "alone_launches": alone_n if alone_ms else None,
            "ms_per_step_warmup": round(warm[mode], 4),
            "timing_note": "ms_per_step: the K timed steps, pipelined over the render streams (a step's launch "
                           "overlaps its neighbours' tails); ms_per_launch_alone: one launch with nothing beside "
                           "it, the roofline's duration; ms_per_step_warmup: rank 0's W untimed warmup steps (first "
                           "launches record the tile order). Order: W warmup steps, the end_to_end and launch-alone "
                           "legs (min(K, 20) + 4 and max(K, 64) launches), then the K timed steps: under a render's load the shader clock "
                           "rises from ~2.18 to ~2.39 GHz over ~50 launches at constant cycles per wave "
                           "(profiles/r6_g), which a 20-step region right after the warmup measured (0.241 vs "
                           "0.224 ms/step)",
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: procedural sphere scene (no dataset), per-pixel seeded XorShift32 streams",
            "config": {
                "workload": f"{cfg_name}: {W}x{H}, {spp_total} spp"
                            + (" per pixel over the whole frame" if args.scaling == "strong" else
                               f" ({cfg['spp']} per GPU, weak scaling)")
                            + f", {D} bounces, "
                            + ("reference 9-sphere scene" if cfg["scene"] == "default" else "random_scene(1000, seed=1)"),
                "width": W, "height": H, "spp_total": spp_total, "max_depth": D,
                "rays_per_step": int(rays_per_step),
                "parallelism": f"rows: row-block-cyclic x{world} (block {rb}), "
                               + ("each render stores its pixels into rank 0's frame over xGMI (IPC)" if remote
                                  else "RCCL gather of RGB to rank 0")
                if world > 1 else ("single GPU" if shards == 1 else
                                   f"DIAGNOSTIC: rank 0's shard of {shards} (block {rb}), no gather"),
                "scene_reads": scene_reads(launch_info),
                "render_streams": nstreams,
                "kernel": launch_info.get("kernel", args.kernel),
                "instance": " ".join(f"{k}={v}" for k, v in launch_info.items() if k != "kernel"),
            },
            "roofline": roof,
            "roofline_valu_issue": valu if valu is not roof else None,
            "roofline_pipelined": piped,
            "roofline_hbm": hbm,
            "end_to_end": {
                "value": round(total_rays / args.steps * e2e_steps / e2e_s / 1e6, 3), "unit": "Mray/s",
                "ms_per_step": round(e2e_s / e2e_steps * 1e3, 4), "steps": e2e_steps,
                "what": "render" + ((" + remote stores into rank 0's frame, barrier" if remote else
                                     " + RCCL gather + assembly") if world > 1 else " + pack to RGB")
                        + (" + D2H of the RGBA frame" if world > 1 else " + D2H of the RGB frame (12 B/pixel)")
                        + " into pinned host memory on rank 0"
                        + (", one step at a time" if remote else f", pipelined over {e2e_slots} frames in flight"),
                "frames_in_flight": e2e_slots if not remote else 1,
                "untimed_steps": e2e_slots if not remote else nslots,
                "copy_ceiling_gbs": round(copy_ceiling, 2) if copy_ceiling else None,
                "copy_ms_at_ceiling": (round(H * W * 12 / (copy_ceiling * 1e9) * 1e3, 4)
                                       if copy_ceiling and world == 1 else None),
                "host_frame_identical": host_identical,
            } if e2e_s else None,
            "cpu_baseline": cpu,
            "cpu_baseline_1core": cpu1,
            "cpu_reference_drawtest": cpu_dt,
            "drawtest": drawtest,
            "drawtest_multi": drawtest_multi,
            "exchange": exchange_legs,
        }
        print(json.dumps(out), flush=True)
    wd.enter("teardown")
    if rstream is not None:
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
        rstream.close()
    if shared is not None:   # importers unmap first, then rank 0 frees
        if rank != 0:
            shared.close()
        dist.barrier()
        if rank == 0:
            shared.close()
    lrt.ShutdownTest()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
