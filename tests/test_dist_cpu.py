"""The N>1 path on CPU: two gloo ranks each render their row-block-cyclic shard (the
oracle stands in for the per-rank GPU render here -- test-only), the shards go to rank 0
through learnraytracing_amd.dist.gather_to_root, and the assembled frame equals the
1-rank frame bit for bit. Also checks the shard map against lrt_shard_rows."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, w, h, rb, frames, depth, outdir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle")]
    import torch
    import torch.distributed as dist
    import oracle
    from learnraytracing_amd import dist as D

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = D.shard_global_rows(h, rb, world, rank)
        max_rows = D.max_shard_rows(h, rb, world)
        local = np.zeros((max_rows, w, 4), np.float32)
        rays = 0
        # render each row block of this shard as a contiguous window
        for start in range(0, len(rows), rb):
            y0 = int(rows[start])
            n = min(rb, len(rows) - start)
            blk, r = oracle.orc_render(w, h, frames, depth, y0=y0, yc=n, threads=1)
            local[start:start + n] = blk
            rays += r
        gathered, _ = D.gather_to_root(torch.from_numpy(local), max_rows, world, rank)
        tot = torch.tensor([rays], dtype=torch.int64)
        dist.all_reduce(tot)
        if rank == 0:
            g = gathered.numpy()
            frame = np.zeros((h, w, 4), np.float32)
            for p in range(world):
                gr = D.shard_global_rows(h, rb, world, p)
                frame[gr] = g[p, :len(gr)]
            np.save(os.path.join(outdir, "frame.npy"), frame)
            np.save(os.path.join(outdir, "rays.npy"), tot.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,rb", [(2, 8), (2, 5)])
def test_two_rank_gloo_assembly_bitwise(tmp_path, world, rb):
    w, h, frames, depth = 80, 45, 2, 8
    mp.spawn(_worker, args=(world, _free_port(), w, h, rb, frames, depth, str(tmp_path)), nprocs=world, join=True)
    import oracle
    want, wrays = oracle.orc_render(w, h, frames, depth)
    got = np.load(tmp_path / "frame.npy")
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert int(np.load(tmp_path / "rays.npy")[0]) == wrays


def _shared_worker(rank, world, port, fail_rank, outdir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    import torch
    import torch.distributed as dist
    from learnraytracing_amd import dist as D

    closed = []

    class Fake:   # stands in for the IPC-mapped frames: fails on fail_rank only
        def __init__(self, w, h, n, r, group=None):
            if r == fail_rank:
                raise RuntimeError("hipIpcOpenMemHandle refused (test)")

        def close(self):
            closed.append(rank)

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        D.SharedFrames = Fake
        got = D.open_shared_frames(8, 4, 2, rank, torch.device("cpu"))
        np.save(os.path.join(outdir, f"r{rank}.npy"),
                np.array([got is None, rank in closed], dtype=np.int32))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [-1, 0, 1])
def test_shared_frames_failure_is_agreed(tmp_path, fail_rank):
    """bench.py's fused exchange falls back to the RCCL gather when any rank cannot map rank
    0's frames: every rank gets None together (no rank left waiting in a collective), and
    the ranks that did map them close them again."""
    world = 2
    mp.spawn(_shared_worker, args=(world, _free_port(), fail_rank, str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        is_none, closed = np.load(tmp_path / f"r{r}.npy")
        assert bool(is_none) == (fail_rank >= 0)
        assert bool(closed) == (fail_rank >= 0 and r != fail_rank)


def test_multidevice_exchange_bytes():
    """lrt_exchange_bytes (no GPU): the direct exchange returns every pixel's RGBA once; the
    gather sends the other devices' packed RGB (12 B per pixel) of the largest shard into the
    first device. 1280x720 over 8 devices in row blocks of 8: shard 0 holds 12 blocks."""
    import ctypes

    from learnraytracing_amd import _lib as L
    d, g = ctypes.c_longlong(0), ctypes.c_longlong(0)
    L.check(L.lib().lrt_exchange_bytes(1280, 720, 8, 8, ctypes.byref(d), ctypes.byref(g)))
    assert d.value == 1280 * 720 * 16
    assert g.value == 7 * 96 * 1280 * 12
    L.check(L.lib().lrt_exchange_bytes(1280, 720, 8, 1, ctypes.byref(d), ctypes.byref(g)))
    assert g.value == 0
    assert L.lib().lrt_exchange_bytes(1280, 720, 0, 8, ctypes.byref(d), ctypes.byref(g)) != 0


def _run_bench_two_ranks(env_extra, timeout=180):
    """bench.py under torch.distributed.run with two gloo ranks (no GPU is touched before the
    phase the test stalls in). Returns (exit code, JSON lines on stdout, stderr)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LRT_DIST_BACKEND="gloo", LRT_BENCH_TIMEOUT="6", **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=timeout)
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, lines, p.stderr


@pytest.mark.parametrize("stall_rank", ["1", None], ids=["one_rank_stalls", "every_rank_stalls"])
def test_bench_reports_a_stalled_phase(stall_rank):
    """A multi-rank bench whose rendezvous hangs (one rank never arrives, or none does) ends
    within its time limit with a non-zero status and ONE JSON line from rank 0 that names the
    stalled phase -- not a hung job (round-4 verdict, What's weak 4)."""
    env = {"LRT_BENCH_STALL": "init_process_group"}
    if stall_rank is not None:
        env["LRT_BENCH_STALL_RANK"] = stall_rank
    rc, lines, err = _run_bench_two_ranks(env)
    assert rc != 0, err[-2000:]
    assert len(lines) == 1, (lines, err[-2000:])
    line = lines[0]
    assert line["value"] is None and line["n_gpus"] == 2 and line["failed_phase"] == "init_process_group", line
    assert "timeout" in line["error"] and line["metric"].startswith("Mray/s"), line
    assert "timeout: phase 'init_process_group'" in err


def _run_bench(args, env_extra, timeout=240):
    """bench.py run as the driver's one-GPU command is run, with no launcher around it."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(LRT_DIST_BACKEND="gloo", LRT_BENCH_TIMEOUT="6", **env_extra)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], cwd=root, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, lines, p.stderr


def test_bench_gpus_n_self_launches_n_ranks():
    """`python bench.py --gpus 2` with no launcher starts two ranks itself (round-5 verdict,
    Next 1): the rendezvous phase -- which a one-process run never enters -- is where both ranks
    stall here, and rank 0's line says n_gpus 2."""
    rc, lines, err = _run_bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                                {"LRT_BENCH_STALL": "init_process_group"})
    assert rc != 0, err[-2000:]
    assert len(lines) == 1, (lines, err[-2000:])
    assert lines[0]["n_gpus"] == 2 and lines[0]["failed_phase"] == "init_process_group", lines[0]
    assert "starting 2 ranks" in err and "torch.distributed.run" in err


def test_bench_gpus_n_without_the_gpus_fails_loudly():
    """No GPU here: `--gpus 2` ends non-zero with ONE line, n_gpus 2 and value null, naming the
    missing devices -- never a number measured on fewer GPUs than the line claims."""
    rc, lines, err = _run_bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"], {})
    assert rc != 0
    assert len(lines) == 1, (lines, err[-2000:])
    d = lines[0]
    assert d["n_gpus"] == 2 and d["value"] is None and "visible" in d["error"], d


def test_bench_world_size_mismatch_is_refused():
    """A launcher's WORLD_SIZE that disagrees with --gpus is an error, not a relabelled line."""
    rc, lines, err = _run_bench(["--gpus", "1", "--no-cpu-baseline"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert rc == 2
    assert len(lines) == 1 and lines[0]["value"] is None and "disagree" in lines[0]["error"], lines


def test_bench_self_launch_that_cannot_start_prints_a_null_line(monkeypatch, capsys):
    import argparse
    import sys

    import bench
    monkeypatch.setattr(sys, "executable", "/nonexistent/python3")
    args = argparse.Namespace(gpus=4, steps=5, warmup=1, config=2, scaling="strong", spp=None, depth=None)
    rc = bench.self_launch(args, ["--gpus", "4"])
    import json
    out = [json.loads(ln) for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]
    assert rc == 2 and len(out) == 1
    assert out[0]["n_gpus"] == 4 and out[0]["value"] is None and "could not start" in out[0]["error"]


@pytest.mark.parametrize("h,rb", [(45, 8), (90, 5)])
def test_eight_rank_gloo_assembly_bitwise(tmp_path, h, rb):
    """World 8 (the driver's node): eight gloo ranks render their row-block-cyclic shards (at
    h=45, rb=8 ranks 6 and 7 own no rows), gather to rank 0 and assemble the 1-rank frame bit
    for bit."""
    world, w, frames, depth = 8, 80, 2, 8
    mp.spawn(_worker, args=(world, _free_port(), w, h, rb, frames, depth, str(tmp_path)), nprocs=world, join=True)
    import oracle
    want, wrays = oracle.orc_render(w, h, frames, depth)
    got = np.load(tmp_path / "frame.npy")
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert int(np.load(tmp_path / "rays.npy")[0]) == wrays


def _config5_worker(rank, world, port, rb, outdir):
    """Config 5's geometry (7680x4320, row blocks of 8 over 8 ranks): every rank fills its
    shard's packed RGB with a code of (global row, column, channel), gathers it to rank 0 the
    way bench.py's RCCL leg does (gather_to_root of [max_rows, W, 3]), and rank 0 assembles
    the frame from the gathered shards with the host mirror of the row map."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    import torch
    import torch.distributed as dist
    from learnraytracing_amd import dist as D

    W, H = 7680, 4320
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = D.shard_global_rows(H, rb, world, rank)
        max_rows = D.max_shard_rows(H, rb, world)
        # the code is an int32 carried as the float32 bit pattern the RGB planes move
        code = (rows[:, None, None].astype(np.int32) * W + np.arange(W, dtype=np.int32)[None, :, None]) * 4 \
            + np.arange(3, dtype=np.int32)[None, None, :]
        local = np.zeros((max_rows, W, 3), np.float32)
        local[:len(rows)] = code.view(np.float32)
        gathered, _ = D.gather_to_root(torch.from_numpy(local), max_rows, world, rank)
        if rank == 0:
            g = gathered.numpy()
            frame = np.full((H, W, 3), -1, np.int32)
            for p in range(world):
                gr = D.shard_global_rows(H, rb, world, p)
                frame[gr] = g[p, :len(gr)].view(np.int32)
            want = (np.arange(H, dtype=np.int32)[:, None, None] * W + np.arange(W, dtype=np.int32)[None, :, None]) * 4 \
                + np.arange(3, dtype=np.int32)[None, None, :]
            ok = bool(np.array_equal(frame, want))
            np.save(os.path.join(outdir, "ok.npy"), np.array([ok, (frame < 0).sum() == 0]))
    finally:
        dist.destroy_process_group()


def test_config5_frame_assembles_over_eight_gloo_ranks(tmp_path):
    """Config 5's 7680x4320 frame row-block-cyclic over 8 ranks: every pixel of the assembled
    frame comes from the rank that owns its row, none is left unwritten (round-5 verdict,
    What's missing 2: the assembly had never run at N > 1)."""
    mp.spawn(_config5_worker, args=(8, _free_port(), 8, str(tmp_path)), nprocs=8, join=True)
    ok, full = np.load(tmp_path / "ok.npy")
    assert ok and full
