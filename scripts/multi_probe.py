"""Components of one device's rg_render_multi timeline (direct mode), on one GPU:
the device's share rendered alone (rg_render_tiles_async, latency-sized launch),
the same with its rows' strided device-to-host copy, and the full call with the
stand-in only_rank rehearsal.  Prints JSON (ms)."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from raingun_amd import _abi  # noqa: E402
from raingun_amd.scene import DeviceScene  # noqa: E402

W, H, N, T = 3840, 2160, 8, 8
out = {}


def timeit(fn, k=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / k * 1e3, 4)


lib = _abi.lib()
for wl in sys.argv[1:] or ["test1", "synth1024"]:
    scene = bench.load_workload(wl, W, H)[0]
    ds = DeviceScene(scene)
    r = {}
    t = _abi.rg_tiling(T, N, 0)
    rows = lib.rg_tiling_rows(H, C.byref(t))
    part = torch.empty((rows, W, 4), dtype=torch.uint8, device="cuda")
    st = _abi.rg_stats()

    def render_sync():
        _abi.check(lib.rg_render_tiles_async(ds.handle, W, H, C.byref(t), C.c_void_p(part.data_ptr()), None, None,
                                             C.byref(st)))
    r["share_render_sync_ms"] = timeit(render_sync)
    r["share_kernel_ms"] = round(st.kernel_ms, 4)
    host = np.empty((H, W, 4), dtype=np.uint8)
    reg = _abi.HostRegistration(host)
    hip = C.CDLL(str(Path(torch.__file__).parent / "lib" / "libamdhip64.so"))
    hip.hipMemcpy2D.restype = C.c_int
    hip.hipMemcpy2D.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int]
    hip.hipMemcpy.restype = C.c_int
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    row4 = W * 4
    ntile = rows // T

    def copy2d():
        assert hip.hipMemcpy2D(host.ctypes.data, N * T * row4, part.data_ptr(), T * row4, T * row4, ntile, 2) == 0
    r["share_copy2d_ms"] = timeit(copy2d)

    def copy1d():
        assert hip.hipMemcpy(host.ctypes.data, part.data_ptr(), rows * row4, 2) == 0
    r["share_copy1d_contiguous_ms"] = timeit(copy1d)
    for rk in (0, 7):
        ds.set_multi(0, stand_in=True, bands=0, only_rank=rk)
        r[f"multi_only_rank{rk}_ms"] = timeit(lambda: ds.render_multi(W, H, N, T, out=host), k=10)
    ds.set_multi(0, stand_in=True, bands=0, only_rank=-1)
    r["multi_stand_in_all8_one_gpu_ms"] = timeit(lambda: ds.render_multi(W, H, N, T, out=host), k=5)
    reg.close()
    ds.close()
    out[wl] = r
print(json.dumps(out, indent=1))
