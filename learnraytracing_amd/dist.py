"""Multi-GPU frame rendering: one process per GPU, the image's rows dealt to GPUs in
blocks of `row_block` rows round-robin (row-block-cyclic), each GPU rendering its
rows densely into a local buffer, then ONE collective (a gather over RCCL/xGMI) brings
the shards to rank 0, where the unshard kernel assembles the frame.

Why row-block-cyclic: contiguous row bands are imbalanced (the sky rows are cheap;
max/mean work 1.31 at 8 GPUs), interleaved blocks are within 0.4 %.
Per-pixel seeding makes the assembled frame bit-identical to a 1-GPU render for any
G and row_block (tests/test_gpu_parity.py, tests/test_dist_cpu.py).

The collective is torch.distributed (backend "nccl" = RCCL on ROCm; "gloo" on CPU
for tests). The reference has no distributed code at all.

SharedFrames is the other exchange: rank 0's frames are mapped into every rank over IPC and
each rank's render stores its finished pixels straight into them (xGMI writes from the render
kernel, lrt_render_device_to_frame) -- no pack, gather or assembly launch per step.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np


def shard_rows(height: int, row_block: int, period: int, phase: int) -> int:
    """Rows GPU `phase` owns (same formula as lrt_shard_rows)."""
    if row_block < 1 or period < 1 or not (0 <= phase < period) or height < 0:
        raise ValueError("invalid shard geometry")
    blocks = (height + row_block - 1) // row_block
    return sum(min((b + 1) * row_block, height) - b * row_block for b in range(phase, blocks, period))


def shard_global_rows(height: int, row_block: int, period: int, phase: int) -> np.ndarray:
    """Global row index of each local row of shard `phase` (the map of lrt_render_desc)."""
    n = shard_rows(height, row_block, period, phase)
    ly = np.arange(n)
    return (ly // row_block) * row_block * period + phase * row_block + ly % row_block


def max_shard_rows(height: int, row_block: int, period: int) -> int:
    return shard_rows(height, row_block, period, 0)


def gather_to_root(local, max_rows: int, world: int, rank: int, gathered=None, group=None,
                   async_op: bool = False):
    """Gather every rank's [max_rows, W, 4] shard buffer into rank 0's
    [world, max_rows, W, 4] tensor (`gathered`, allocated if None).
    Returns (gathered_or_None, work_or_None).

    ONE code path for every backend: `dist.gather` of the shard into the rows of
    `gathered`. RCCL ("nccl") moves the device tensors over xGMI directly; gloo moves host
    tensors only, so a cuda shard under gloo (rehearsing N > 1 on one GPU) is staged
    through host copies around the same call -- CPU tensors under gloo (tests) take the
    exact lines the RCCL run takes."""
    import torch
    import torch.distributed as dist

    if local.shape[0] != max_rows:
        raise ValueError("shard buffers must be padded to max_rows rows")
    if world == 1 and not dist.is_initialized():
        return local.unsqueeze(0), None   # no process group: nothing to exchange
    # (a one-rank group takes the collective too, so the RCCL gather is exercised at N = 1)
    stage = local.is_cuda and dist.get_backend(group) == "gloo"
    send = local.cpu() if stage else local
    out: Optional[List] = None
    recv = None
    if rank == 0:
        if gathered is None:
            gathered = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
        recv = torch.empty(gathered.shape, dtype=gathered.dtype) if stage else gathered
        out = list(recv.unbind(0))
    else:
        gathered = None
    work = dist.gather(send, gather_list=out, dst=0, group=group, async_op=async_op and not stage)
    if stage and rank == 0:
        gathered.copy_(recv)
    return gathered, work


class SharedFrames:
    """`count` RGBA frames (height x width) allocated on rank 0 (lrt_ipc_alloc) and mapped into
    every other rank (lrt_ipc_open, peer access over xGMI), for the fused exchange: rank r's
    render writes its rows into rank 0's frame directly. `ptrs[i]` is frame i's device address
    in this process; rank 0 can view frame i as a tensor with `tensor(i)`."""

    def __init__(self, width: int, height: int, count: int, rank: int, group=None):
        import ctypes
        import torch.distributed as dist

        from . import _lib as L
        self.width, self.height, self.count, self.rank = width, height, count, rank
        self.bytes = width * height * 16
        self._owned, self._opened, self.ptrs = [], [], []
        handles = None
        err = None
        if rank == 0:
            handles = []
            try:
                for _ in range(count):
                    p = ctypes.c_void_p()
                    h = (ctypes.c_char * L.IPC_HANDLE_BYTES)()
                    L.check(L.lib().lrt_ipc_alloc(self.bytes, ctypes.byref(p), ctypes.cast(h, ctypes.c_void_p)))
                    self._owned.append(p.value)
                    handles.append(bytes(h))
            except Exception as e:   # still broadcast (None), so no rank waits on a dead root
                err, handles = e, None
            self.ptrs = list(self._owned)
        box = [handles]
        if dist.is_initialized():
            dist.broadcast_object_list(box, src=0, group=group)
        if err is not None:
            self.close()
            raise err
        if box[0] is None:
            raise RuntimeError("rank 0 could not allocate the shared frames")
        if rank != 0:
            try:
                for hb in box[0]:
                    h = (ctypes.c_char * L.IPC_HANDLE_BYTES).from_buffer_copy(hb)
                    p = ctypes.c_void_p()
                    L.check(L.lib().lrt_ipc_open(ctypes.cast(h, ctypes.c_void_p), ctypes.byref(p)))
                    self._opened.append(p.value)
            except Exception:
                self.close()
                raise
            self.ptrs = list(self._opened)

    def tensor(self, i: int):
        """Frame i as a (height, width, 4) float32 cuda tensor over rank 0's own memory (no copy)."""
        if self.rank != 0:
            raise ValueError("only rank 0 owns the frames")
        return _tensor_from_ptr(self.ptrs[i], (self.height, self.width, 4))

    def close(self) -> None:
        import ctypes

        from . import _lib as L
        for p in self._opened:
            L.lib().lrt_ipc_close(ctypes.c_void_p(p))
        for p in self._owned:
            L.lib().lrt_ipc_free(ctypes.c_void_p(p))
        self._opened, self._owned, self.ptrs = [], [], []


class _CudaArray:
    """__cuda_array_interface__ of float32 device memory, for torch.as_tensor (no copy)."""

    def __init__(self, ptr: int, shape):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": "<f4", "data": (int(ptr), False),
                                         "version": 3, "strides": None}


def open_shared_frames(width: int, height: int, count: int, rank: int, device, group=None, force_fail=False):
    """SharedFrames on every rank, or None on every rank when any rank fails to allocate or
    map them (the ranks agree through one all-reduce), so the caller can fall back to the
    RCCL exchange instead of one rank dying while the others wait in a collective.
    force_fail: this rank reports a refused mapping without trying (tests of the fallback)."""
    import torch
    import torch.distributed as dist

    frames, err = None, None
    if force_fail:
        err = RuntimeError("IPC mapping refused (forced)")
    else:
        try:
            frames = SharedFrames(width, height, count, rank, group=group)
        except Exception as e:
            err = e
    if not dist.is_initialized():
        if err is not None:
            raise err
        return frames
    bad = torch.tensor([0 if err is None else 1], dtype=torch.int32, device=device)
    dist.all_reduce(bad, op=dist.ReduceOp.MAX, group=group)
    if int(bad.item()):
        if frames is not None:
            frames.close()
        return None
    return frames


def _tensor_from_ptr(ptr: int, shape):
    import torch
    return torch.as_tensor(_CudaArray(ptr, shape), device="cuda")
