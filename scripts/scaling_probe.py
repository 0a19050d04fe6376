"""Single-GPU probe of the per-step costs a rank pays at N GPUs (test1 4K d5):
kernel time of its 1/N share of tiles, host-side step time (launch + counters
memset + events), and rank 0's re-interleave of N gathered buffers.  RCCL
itself cannot be timed on a 1-GPU box; this bounds everything else."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from raingun_amd import _abi, distributed as rd  # noqa: E402
from raingun_amd.scene import DeviceScene, load_scene  # noqa: E402

G = Path(__file__).resolve().parent.parent / "tests" / "golden"
sc = load_scene(G / "examples" / "test1.yml", texture_root=G)
sc.max_recursion_depth = 5
W, H = 3840, 2160
ds = DeviceScene(sc)
lib = _abi.lib()
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
sh = C.c_void_p(stream.cuda_stream)
res = {}
for N, order in [(n, o) for n in (1, 2, 4, 8) for o in (True, False)]:
    ds.set_tile_order(order)
    t = rd.tiling(0, N, rd.TILE_ROWS)
    slot = rd.slot_rows(H, N)
    out = torch.zeros((slot, W, 4), dtype=torch.uint8, device=dev)
    def launch():
        _abi.check(lib.rg_render_tiles_async(ds.handle, W, H, C.byref(t), C.c_void_p(out.data_ptr()), None, sh, None))
    for _ in range(5):
        launch()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    t0 = time.perf_counter()
    for e0, e1 in ev:
        e0.record(stream); launch(); e1.record(stream)
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) * 1e3 / len(ev)
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    # rank 0's assemble of N buffers into the frame
    bufs = rd.gather_buffers(out, N)
    for b in bufs:
        b.copy_(out)
    frame = torch.empty((H, W, 4), dtype=torch.uint8, device=dev)
    for _ in range(3):
        frame.copy_(rd.assemble(bufs, H, N))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        frame.copy_(rd.assemble(bufs, H, N))
    torch.cuda.synchronize()
    asm_ms = (time.perf_counter() - t0) * 1e3 / 20
    res[f"N{N}_order{int(order)}"] = dict(kernel_ms=round(kern_ms, 4), launch_loop_ms=round(step_ms, 4), assemble_ms=round(asm_ms, 4),
                  frame_bytes_per_rank=slot * W * 4)
print(json.dumps(res, indent=1))
