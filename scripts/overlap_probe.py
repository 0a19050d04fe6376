"""Per-rank render throughput of a 1/N share of a frame with F frames in flight
(frame k on render stream k % F), on one GPU: what a rank of the N-GPU frame
pipeline can sustain before the gather (bench.py --frames-in-flight F).
Frames in flight let the next frame's blocks take the CUs the current frame's
slowest tiles leave idle.  Prints JSON: {workload: {N: {F: ms_per_frame}}}."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from raingun_amd import _abi, distributed as rd  # noqa: E402
from raingun_amd.scene import DeviceScene, load_scene  # noqa: E402
from raingun_amd.synth import synthetic_scene  # noqa: E402

G = Path(__file__).resolve().parent.parent / "tests" / "golden"
W, H = 3840, 2160
K = 40


def scene(name):
    if name == "test1":
        sc = load_scene(G / "examples" / "test1.yml", texture_root=G)
        sc.max_recursion_depth = 5
        return sc
    return synthetic_scene(int(name[5:]), 2, 5)


lib = _abi.lib()
dev = torch.device("cuda", 0)
FMAX = int(__import__("os").environ.get("FMAX", "4"))
STREAMS = [torch.cuda.Stream(dev) for _ in range(FMAX)]  # created once: distinct hardware queues
out = {}
for name in sys.argv[1:] or ("test1", "synth1024"):
    ds = DeviceScene(scene(name))
    res = {}
    for n in (1, 2, 4, 8):
        t = rd.tiling(0, n, rd.TILE_ROWS)
        slot = rd.slot_rows(H, n)
        res[n] = {}
        for f in range(1, FMAX + 1):
            streams = STREAMS[:f]
            bufs = [torch.zeros((slot, W, 4), dtype=torch.uint8, device=dev) for _ in range(f)]

            def launch(k):
                s = streams[k % f]
                _abi.check(lib.rg_render_tiles_async(ds.handle, W, H, C.byref(t), C.c_void_p(bufs[k % f].data_ptr()),
                                                     None, C.c_void_p(s.cuda_stream), None))
            for k in range(2 * f):
                launch(k)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(K):
                launch(k)
            torch.cuda.synchronize()
            res[n][f] = round((time.perf_counter() - t0) * 1e3 / K, 4)
    ds.close()
    out[name] = res
print(json.dumps(out, indent=1))
