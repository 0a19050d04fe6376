"""Host-side cost per frame of the N>1 frame pipeline, on one GPU (world 1 over
RCCL): enqueue time of K frames without synchronising, for a tiny frame (so
the GPU never holds the host back).  Separates the library launch, the
pipeline's Python/stream bookkeeping, the RCCL gather and rank 0's
re-interleave.  Prints JSON {case: us_per_frame}."""
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from raingun_amd import _abi, distributed as rd  # noqa: E402
from raingun_amd.scene import DeviceScene  # noqa: E402
from raingun_amd.synth import synthetic_scene  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
dev = torch.device("cuda", 0)
W, H, K, T = 256, 144, 400, rd.TILE_ROWS
ds = DeviceScene(synthetic_scene(16, 1, 1))  # cheap frames: the GPU keeps up with the host
lib = _abi.lib()
tiling = rd.tiling(0, 1, T)
slot = rd.slot_rows(H, 1, T)
out = {}


def timed(name, fn):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    out[name] = {"enqueue_us": round(t_enq * 1e6 / K, 1), "total_us": round((time.perf_counter() - t0) * 1e6 / K, 1)}


buf = torch.zeros((slot, W, 4), dtype=torch.uint8, device=dev)
sh = C.c_void_p(torch.cuda.current_stream().cuda_stream)


def launch(part=None, s=None):
    p = buf if part is None else part
    st = sh if s is None else C.c_void_p(s.cuda_stream)
    _abi.check(lib.rg_render_tiles_pipelined(ds.handle, W, H, C.byref(tiling), C.c_void_p(p.data_ptr()), None, st))


timed("rg_render_tiles_pipelined", launch)
for f, gather in ((1, False), (4, False), (4, True)):
    pipe = rd.FramePipeline((slot, W, 4), H, 0, 1, T, device=dev, depth=f, streams=f > 1, gather=gather)
    timed(f"pipeline_F{f}{'_gather' if gather else ''}",
          lambda: pipe.step(lambda part: launch(part, torch.cuda.current_stream())))
    pipe.flush()
native = rd.NativeFramePipeline(ds.handle, W, H, 0, 1, T, depth=4, device=dev)
timed("native_pipeline_F4_gather", native.step)
native.flush()
native.close()
# the same loop with a no-op in place of ncclGather: the library's own host cost
NOOP = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p, C.c_void_p)(
    lambda *a: 0)
h = C.c_void_p()
_abi.check(lib.rg_frames_create(ds.handle, W, H, T, 0, 1, 4, C.c_void_p(1), C.cast(NOOP, C.c_void_p), C.byref(h)))
timed("native_pipeline_F4_noop_gather", lambda: _abi.check(lib.rg_frames_step(h)))
lib.rg_frames_flush(h)
lib.rg_frames_destroy(h)
# rank 0 of an 8-rank loop: the library's native no-op gather in place of
# ncclGather, so the numbers are the loop's own host work per frame; two frames per gather
# (batch 2, the default at world > 1) halve the per-frame gather and bookkeeping calls
noop = C.cast(lib.rg_debug_gather_noop, C.c_void_p)
for world in (8,):
    for batch in (1, 2):
        h = C.c_void_p()
        _abi.check(lib.rg_frames_create(ds.handle, W, H, T, 0, world, 8, C.c_void_p(1), noop, C.byref(h)))
        _abi.check(lib.rg_frames_set_batch(h, batch))
        timed(f"native_pipeline_world{world}_rank0_F8_batch{batch}_noop_gather",
              lambda: _abi.check(lib.rg_frames_step(h)))
        _abi.check(lib.rg_frames_flush(h))
        lib.rg_frames_destroy(h)
# RCCL's own host cost per ncclGather call (world 1): what batching halves per frame
native = rd.NativeFramePipeline(ds.handle, W, H, 0, 1, T, depth=8, device=dev)
timed("native_pipeline_F8_world1_rccl_gather", native.step)
native.flush()
native.close()
recv = [torch.empty_like(buf)]
timed("dist.gather_alone", lambda: dist.gather(buf, recv, dst=0, async_op=True))
print(json.dumps(out, indent=1))
dist.destroy_process_group()
