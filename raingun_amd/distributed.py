"""Row-tile sharding of one frame across ranks (one process per GPU).

Pixels are independent (rendering.rs:27-33), so the frame is cut into
`tile_rows`-row tiles dealt round-robin: tile t belongs to rank t % world
(interleaving balances sky-heavy and geometry-heavy bands).  Each rank renders
its tiles densely packed into one buffer of `slot_rows(...)` rows (the last
ranks' buffers are zero-padded so every rank sends the same byte count), and
ONE gather (torch.distributed; backend "nccl" is RCCL over xGMI) brings the
buffers to rank 0, which re-interleaves them into image order.

Rank 0's share (`root` > 1, rg_frames_set_root_tiles): the tiles are dealt in
periods of root + world - 1 -- the first `root` of each period to rank 0, then
one to each other rank.  Rank 0's rows never cross the interconnect, so every
other rank's part of the gather shrinks; rank 0's own part is larger than the
equal-size slots of the others and is not sent.

There is no other collective on the data path.
"""
from __future__ import annotations

from typing import Callable, Optional

TILE_ROWS = 16


def n_tiles(height: int, tile_rows: int = TILE_ROWS) -> int:
    return (height + tile_rows - 1) // tile_rows


def tiles_per_rank(height: int, world: int, tile_rows: int = TILE_ROWS) -> int:
    return (n_tiles(height, tile_rows) + world - 1) // world


def slot_rows(height: int, world: int, tile_rows: int = TILE_ROWS) -> int:
    """Rows of every rank's gather buffer (equal across ranks)."""
    return tiles_per_rank(height, world, tile_rows) * tile_rows


def rank_tiles(height: int, rank: int, world: int, tile_rows: int = TILE_ROWS, root: int = 1) -> list:
    """Image tiles of `rank`, in the order its part holds them."""
    n = n_tiles(height, tile_rows)
    if root == 1:
        return list(range(rank, n, world))
    P = root + world - 1
    if rank == 0:
        return [t for t in range(n) if t % P < root]
    return list(range(root + rank - 1, n, P))


def root_slot_rows(height: int, world: int, tile_rows: int = TILE_ROWS, root: int = 1) -> int:
    """Rows of the other ranks' equal-size gather slots with rank 0's share `root` (root 1: slot_rows)."""
    if root == 1 or world == 1:
        return slot_rows(height, world, tile_rows)
    return len(rank_tiles(height, 1, world, tile_rows, root)) * tile_rows


def tilings(rank: int, world: int, tile_rows: int = TILE_ROWS, root: int = 1) -> list:
    """The rg_tiling(s) whose selected tiles, interleaved one by one, make up `rank`'s part: ONE for
    every rank but rank 0 with root > 1, whose `root` tiles per period are `root` strided tilings
    (the native loop renders them in one launch: rg_frames.hip, RgKernelArgs::tile_group)."""
    from ._abi import rg_tiling

    if root == 1:
        return [rg_tiling(tile_rows, world, rank)]
    P = root + world - 1
    if rank == 0:
        return [rg_tiling(tile_rows, P, j) for j in range(root)]
    return [rg_tiling(tile_rows, P, root + rank - 1)]


def tiling(rank: int, world: int, tile_rows: int = TILE_ROWS):
    """The rg_tiling a rank passes to rg_render_tiles[_async]."""
    from ._abi import rg_tiling

    return rg_tiling(tile_rows, world, rank)


def assemble(gathered, height: int, world: int, tile_rows: int = TILE_ROWS, root: int = 1):
    """Re-interleave the per-rank buffers into image order.

    `gathered` is a list (index = rank) of (slot_rows, W, C) tensors or arrays,
    or one stacked (world, slot_rows, W, C) tensor/array.  Returns (height, W, C).
    With rank 0's share `root` > 1, gathered[0] is rank 0's own (larger) part."""
    import numpy as np

    if root > 1 and world > 1:
        T = tile_rows
        out = None
        for r in range(world):
            part = gathered[r]
            for j, t in enumerate(rank_tiles(height, r, world, T, root)):
                rows = part[j * T:(j + 1) * T][:height - t * T]
                if out is None:
                    out = (np.empty((height,) + tuple(part.shape[1:]), dtype=part.dtype) if isinstance(part, np.ndarray)
                           else part.new_empty((height,) + tuple(part.shape[1:])))
                out[t * T:t * T + rows.shape[0]] = rows
        return out

    is_np = isinstance(gathered, np.ndarray) or (isinstance(gathered, (list, tuple)) and
                                                 isinstance(gathered[0], np.ndarray))
    if is_np:
        g = np.stack(gathered) if isinstance(gathered, (list, tuple)) else gathered
    else:
        import torch

        if isinstance(gathered, (list, tuple)):
            base = gathered[0]._base if gathered[0]._base is not None else None
            # views of one (world, slot, W, C) tensor (gather_buffers()): no stacking copy
            if (base is not None and base.dim() == 4 and base.shape[0] == len(gathered) and
                    all(t._base is base for t in gathered) and gathered[0].data_ptr() == base.data_ptr()):
                g = base
            else:
                g = torch.stack(list(gathered))
        else:
            g = gathered
    tpr = tiles_per_rank(height, world, tile_rows)
    w, c = g.shape[-2], g.shape[-1]
    g = g.reshape(world, tpr, tile_rows, w, c)
    # tile j*world + r lives in g[r, j]
    g = g.transpose(1, 0, 2, 3, 4) if is_np else g.transpose(0, 1)
    return g.reshape(world * tpr * tile_rows, w, c)[:height]


def gather_buffers(part, world: int):
    """Rank 0's receive buffers for render_frame: `world` views of ONE
    (world, slot_rows, W, C) tensor, so assemble() re-interleaves them with a
    single copy."""
    big = part.new_empty((world,) + tuple(part.shape))
    return list(big.unbind(0))


def _root_part(render_tiles, height: int, world: int, tile_rows: int, root: int):
    """Rank 0's part with share `root` > 1: its `root` strided tilings rendered and interleaved
    tile by tile (local tile p * root + s = tile p of tiling s)."""
    T, subs = tile_rows, [render_tiles(t) for t in tilings(0, world, tile_rows, root)]
    n = len(rank_tiles(height, 0, world, T, root))
    part = subs[0].new_zeros((n * T,) + tuple(subs[0].shape[1:]))
    for i in range(n):
        p, s = divmod(i, root)
        part[i * T:(i + 1) * T] = subs[s][p * T:(p + 1) * T]
    return part


def render_frame(render_tiles: Callable[[object], object], height: int, rank: int, world: int,
                 tile_rows: int = TILE_ROWS, group=None, out=None, gather_bufs=None, root: int = 1):
    """Render this rank's tiles with `render_tiles(tiling) -> (slot_rows, W, 4)
    tensor` and gather the frame to rank 0.  Returns the (height, W, 4) frame on
    rank 0 and None on the other ranks.  root > 1: rank 0's share (module doc);
    render_tiles then returns that tiling's rows, zero-padded to root_slot_rows."""
    if root > 1 and world > 1:
        import torch.distributed as dist

        slot = root_slot_rows(height, world, tile_rows, root)
        if rank == 0:
            mine = _root_part(render_tiles, height, world, tile_rows, root)
            dummy = mine.new_zeros((slot,) + tuple(mine.shape[1:]))  # rank 0's slot of the gather is not read
            bufs = [dummy.new_empty(dummy.shape) for _ in range(world)]
            dist.gather(dummy, bufs, dst=0, group=group)
            return assemble([mine] + bufs[1:], height, world, tile_rows, root)
        part = render_tiles(tilings(rank, world, tile_rows, root)[0])[:slot]
        dist.gather(part.contiguous(), None, dst=0, group=group)
        return None
    part = render_tiles(tiling(rank, world, tile_rows))
    if world == 1:
        return part[:height]
    import torch.distributed as dist

    if part.is_cuda and dist.get_backend(group) == "gloo":
        # rehearsal only (gloo gathers host tensors): stage through host memory
        host = part.cpu()
        if rank == 0:
            hb = [host.new_empty(host.shape) for _ in range(world)]
            dist.gather(host, hb, dst=0, group=group)
            frame = assemble(hb, height, world, tile_rows).to(part.device)
            if out is not None:
                out.copy_(frame)
                return out
            return frame
        dist.gather(host, None, dst=0, group=group)
        return None
    if rank == 0:
        bufs = gather_bufs if gather_bufs is not None else [part.new_empty(part.shape) for _ in range(world)]
        dist.gather(part, bufs, dst=0, group=group)
        frame = assemble(bufs, height, world, tile_rows)
        if out is not None:
            out.copy_(frame)
            return out
        return frame
    dist.gather(part, None, dst=0, group=group)
    return None


def assemble_into(frame_padded, gathered, world: int, tile_rows: int = TILE_ROWS):
    """Re-interleave a (world, slot_rows, W, C) gather result into
    `frame_padded` ((world * slot_rows, W, C), image order, the last rows
    padding) with ONE strided copy: tile j*world + r lives in gathered[r, j]."""
    w, c = gathered.shape[-2], gathered.shape[-1]
    tpr = gathered.shape[1] // tile_rows
    src = gathered.reshape(world, tpr, tile_rows, w, c)
    dst = frame_padded.view(tpr, world, tile_rows, w, c)
    if hasattr(dst, "copy_"):
        dst.copy_(src.transpose(0, 1))
    else:  # numpy
        dst[...] = src.transpose(1, 0, 2, 3, 4)
    return frame_padded


class FramePipeline:
    """Row-tile frames over `world` ranks, `depth` frames in flight.

    Step k: this rank renders its tiles of frame k into part buffer k % depth
    (on the current stream), the gather of that buffer to rank 0 is issued
    asynchronously (torch.distributed, backend "nccl" = RCCL: it runs on RCCL's
    own stream after the render), and rank 0 re-interleaves it on a side
    stream once the gather has landed.  So the gather and the re-interleave
    of frame k overlap the render of frame k+1; a buffer is reused only after
    its previous frame's gather (and, on rank 0, re-interleave) finished.
    `flush()` completes every frame in flight.  On CPU tensors (gloo) the
    same sequence runs synchronously, and `on_frame(k, frame)` (rank 0) sees
    each assembled frame.  One collective per frame: the gather.

    `streams=True` (CUDA) renders frame k on render stream k % depth, so the
    renders of consecutive frames may also overlap: the next frame's blocks
    take the CUs the current frame's slowest tiles leave idle (a rank's share
    of a frame is tail-bound: its makespan is set by its slowest 8x8 tiles,
    not by its average work).  The library keeps separate launch state per
    stream, so the two launches never share counters or tile queues."""

    def __init__(self, part_shape, height: int, rank: int, world: int, tile_rows: int = TILE_ROWS,
                 device=None, depth: int = 2, group=None, on_frame=None, streams=False,
                 gather: bool = None):
        import torch

        self.H, self.rank, self.world, self.T, self.group = height, rank, world, tile_rows, group
        self.depth, self.on_frame = depth, on_frame
        self.gather = world > 1 if gather is None else gather  # gather=True at world 1: rehearse the collective path
        self.cuda = device is not None and torch.device(device).type == "cuda"
        kw = dict(dtype=torch.uint8, device=device)
        self.parts = [torch.zeros(part_shape, **kw) for _ in range(depth)]
        self.works = [None] * depth
        self.frames = [None] * depth          # frame index held by each buffer
        self.asm_done = [None] * depth        # rank 0, CUDA: re-interleave finished (event)
        if rank == 0 and self.gather:
            self.gathered = [torch.empty((world,) + tuple(part_shape), **kw) for _ in range(depth)]
            self.recv = [list(g.unbind(0)) for g in self.gathered]
            self.frame_padded = torch.empty((world * part_shape[0],) + tuple(part_shape[1:]), **kw)
            self.side = torch.cuda.Stream(device) if self.cuda else None
            if self.cuda:  # assemble_into's strided copy, its views built once
                tpr = part_shape[0] // tile_rows
                self.asm_src = [g.reshape((world, tpr, tile_rows) + tuple(part_shape[1:])).transpose(0, 1)
                                for g in self.gathered]
                self.asm_dst = self.frame_padded.view((tpr, world, tile_rows) + tuple(part_shape[1:]))
                self.asm_done = [torch.cuda.Event() for _ in range(depth)]
        # streams: True -> `depth` new render streams; a list -> those (a caller that times several
        # pipelines in one process keeps one set, so every one runs on the same hardware queues)
        if isinstance(streams, (list, tuple)):
            assert len(streams) >= depth
            self.streams = list(streams[:depth]) if self.cuda else None
        else:
            self.streams = [torch.cuda.Stream(device) for _ in range(depth)] if (self.cuda and streams) else None
        self.k = 0

    @property
    def frame(self):
        """Rank 0's latest assembled frame (image order, `height` rows)."""
        if not self.gather:  # one rank: its part is the frame
            return self.parts[(self.k - 1) % self.depth][:self.H]
        return self.frame_padded[:self.H]

    def _retire(self, b):
        """Make buffer b reusable: its frame's gather (+ rank 0's re-interleave) done."""
        import torch

        w = self.works[b]
        if w is None:
            return
        if self.cuda:
            if self.rank == 0:
                torch.cuda.current_stream().wait_event(self.asm_done[b])
            else:
                w.wait()
        self.works[b] = None

    def step(self, render):
        """Enqueue one frame: `render(part)` writes this rank's tiles into `part`
        on the current stream (render stream k % depth with `streams`)."""
        import torch

        b = self.k % self.depth
        if self.streams is None:
            self._step(render, b)
        else:
            # frame k depends only on frame k - depth (its buffer) and the scene:
            # the render stream does not wait for the caller's stream (host cost
            # per frame is the N > 1 bound at small shares: scripts/host_overhead_probe.py)
            with torch.cuda.stream(self.streams[b]):
                self._step(render, b)

    def _step(self, render, b):
        import torch
        import torch.distributed as dist

        self._retire(b)
        part = self.parts[b]
        render(part)
        if not self.gather:  # one rank: nothing to gather, the part is the frame
            self.frames[b] = self.k
            if not self.cuda and self.on_frame is not None:
                self.on_frame(self.k, self.frame_of(b))
            self.k += 1
            return
        work = dist.gather(part, self.recv[b] if self.rank == 0 else None, dst=0, group=self.group, async_op=True)
        self.works[b], self.frames[b] = work, self.k
        if self.rank == 0:
            if self.cuda:
                with torch.cuda.stream(self.side):
                    work.wait()  # side stream waits for the gather
                    self.asm_dst.copy_(self.asm_src[b])  # re-interleave (assemble_into, views made once)
                    self.asm_done[b].record(self.side)
            else:
                work.wait()
                assemble_into(self.frame_padded, self.gathered[b], self.world, self.T)
                if self.on_frame is not None:
                    self.on_frame(self.k, self.frame)
        elif not self.cuda:
            work.wait()
        self.k += 1

    def frame_of(self, b):
        return self.parts[b][:self.H]

    def flush(self):
        """Complete every frame in flight (the current stream then holds them all)."""
        import torch

        for b in range(self.depth):
            self._retire(b)
        if self.streams is not None:  # the renders (one rank: nothing else follows them)
            for s in self.streams:
                torch.cuda.current_stream().wait_stream(s)


class RcclComm:
    """The library's own RCCL communicator over the ranks of a torch.distributed
    group (include/raingun_frames.h rg_comm_*): rank 0 makes the ncclUniqueId,
    torch.distributed's public broadcast_object_list hands its bytes to every
    rank, and every rank joins with ncclCommInitRank on `device` -- no private
    torch API, no communicator borrowed from torch."""

    def __init__(self, rank: int, world: int, device: int, group=None):
        import ctypes as C

        import torch.distributed as dist

        from . import _abi

        self._lib = _abi.lib()
        if not hasattr(self._lib, "rg_comm_init_rank"):
            raise RuntimeError("libraingun_hip.so predates rg_comm_init_rank: rebuild it")
        n = self._lib.rg_comm_id_bytes()
        uid = (C.c_uint8 * n)()
        status = _abi.RG_OK
        if rank == 0:
            status = int(self._lib.rg_comm_unique_id(uid))
        # (status, id) travel together, so a failure on rank 0 raises on EVERY rank instead of
        # leaving the others blocked in the broadcast; the source is group rank 0's global rank
        obj = [(status, bytes(uid))]
        if world > 1:
            src = 0 if group is None else dist.get_global_rank(group, 0)
            dist.broadcast_object_list(obj, src=src, group=group)
        status, raw = obj[0]
        _abi.check(status, "rg_comm_unique_id (rank 0)")
        uid = (C.c_uint8 * n).from_buffer_copy(raw)
        h = C.c_void_p()
        _abi.check(self._lib.rg_comm_init_rank(uid, world, rank, int(device), C.byref(h)), "rg_comm_init_rank")
        self.handle = h
        self.gather_fn = self._lib.rg_comm_gather_fn()
        if not self.gather_fn:
            raise RuntimeError("rg_comm_gather_fn: no ncclGather")

    def info(self) -> dict:
        """ncclCommCount / ncclCommUserRank / ncclCommCuDevice of the communicator."""
        import ctypes as C

        from . import _abi

        n, r, d = C.c_int32(-1), C.c_int32(-1), C.c_int32(-1)
        _abi.check(self._lib.rg_comm_info(self.handle, C.byref(n), C.byref(r), C.byref(d)), "rg_comm_info")
        return {"nranks": n.value, "rank": r.value, "device": d.value}

    def close(self):
        if getattr(self, "handle", None):
            self._lib.rg_comm_destroy(self.handle)
            self.handle = None


class NativeFramePipeline:
    """FramePipeline's N > 1 loop in C++ (include/raingun_frames.h): frame k
    renders on render stream k % depth, ONE ncclGather per frame (or per two
    frames) runs on a communication stream in frame order, rank 0
    re-interleaves on a side stream -- a handful of HIP/RCCL calls per frame
    instead of ~70 us of Python on rank 0, which would otherwise bound a small
    share (1/8 of a 4K test1 frame renders in ~40 us).  The communicator is the
    library's own (RcclComm, over the ranks of `group`); failures raise."""

    def __init__(self, scene, width: int, height: int, rank: int, world: int, tile_rows: int = TILE_ROWS,
                 depth: int = 4, group=None, device=None, root_tiles: int = 1):
        import ctypes as C

        import torch

        from . import _abi

        self.W, self.H, self.rank = width, height, rank
        self._lib = _abi.lib()
        # a DeviceScene is kept alive as long as the pipeline (raingun_frames.h: the scene
        # must outlive its frames); a raw handle is the caller's to keep
        self._scene = scene
        scene_handle = getattr(scene, "handle", scene)
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        # the rank's device first: the id broadcast (NCCL object tensors) and rg_frames_create
        # (it binds the current device) both use it
        torch.cuda.set_device(dev)
        self.comm = RcclComm(rank, world, dev.index if dev.index is not None else torch.cuda.current_device(), group)
        h = C.c_void_p()
        st = self._lib.rg_frames_create(scene_handle, width, height, tile_rows, rank, world, depth,
                                        self.comm.handle, C.c_void_p(self.comm.gather_fn), C.byref(h))
        _abi.check(st, "rg_frames_create")
        self._h = h
        if root_tiles != 1:  # rank 0's share (include/raingun_frames.h rg_frames_set_root_tiles)
            _abi.check(self._lib.rg_frames_set_root_tiles(h, int(root_tiles)), "rg_frames_set_root_tiles")

    def step(self, render=None):
        from . import _abi

        _abi.check(self._lib.rg_frames_step(self._h), "rg_frames_step")

    def flush(self):
        from . import _abi

        _abi.check(self._lib.rg_frames_flush(self._h), "rg_frames_flush")

    def read_frame(self):
        """Rank 0: the latest assembled frame as a (H, W, 4) uint8 numpy array.
        Local (no collective): call flush() on EVERY rank first -- with two
        frames per gather, a batch cut short is gathered only by flush(), and
        reading while it is pending raises (rg_frames_read_image)."""
        import numpy as np

        from . import _abi

        out = np.empty((self.H, self.W, 4), dtype=np.uint8)
        _abi.check(self._lib.rg_frames_read_image(self._h, out.ctypes.data), "rg_frames_read_image")
        return out

    def close(self):
        if getattr(self, "_h", None):
            self._lib.rg_frames_destroy(self._h)
            self._h = None
        if getattr(self, "comm", None) is not None:
            self.comm.close()  # after the frames: their gathers ran on it
            self.comm = None
        self._scene = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown: the runtime may already be gone
            pass
