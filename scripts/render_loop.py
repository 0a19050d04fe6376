"""Render K frames of a workload (for rocprofv3 kernel traces).
usage: python scripts/render_loop.py [test1|synth1024|synth4096] [frames]"""
import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from raingun_amd import _abi  # noqa: E402
from raingun_amd.scene import DeviceScene, load_scene  # noqa: E402
from raingun_amd.synth import synthetic_scene  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "test1"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 10
G = Path(__file__).resolve().parent.parent / "tests" / "golden"
if wl == "test1":
    sc = load_scene(G / "examples" / "test1.yml", texture_root=G)
    sc.max_recursion_depth = 5
else:
    sc = synthetic_scene(int(wl[5:]), 2, 5)
ds = DeviceScene(sc)
buf = torch.empty((2160, 3840, 4), dtype=torch.uint8, device="cuda")
t = _abi.rg_tiling(2160, 1, 0)
for _ in range(frames):
    _abi.check(_abi.lib().rg_render_tiles_async(ds.handle, 3840, 2160, C.byref(t), C.c_void_p(buf.data_ptr()), None,
                                                None, None))
torch.cuda.synchronize()
print("done", wl, frames)
