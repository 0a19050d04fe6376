#!/usr/bin/env python3
"""Same scene, several DeviceScene instances in one process: does the frame time depend on the
instance (where its tables landed in HBM)?  profiles/r06/s19: one north-star instance rendered the
pinned host frame in 2.32-2.34 ms, a second one in 2.13 ms, with either host buffer.

    python scripts/scene_instance_probe.py [workload] [instances]   -> JSON lines: per instance the
    pinned host-visible frame (rg_render_image) and a device-resident single launch (rg_render_tiles)
"""
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

W, H = 3840, 2160


def timed(fn, n):
    for _ in range(3):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return round((time.perf_counter() - t0) / n * 1e3, 4)


def kernel_ms(ds, reps=9):
    """Median kernel time of a whole-frame device-resident launch (HIP events, rg_stats.kernel_ms)."""
    lib = _abi.lib()
    import ctypes as C
    t = _abi.rg_tiling(H, 1, 0)
    part = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    st = _abi.rg_stats()
    ks = []
    for i in range(reps + 2):
        _abi.check(lib.rg_render_tiles_async(ds.handle, W, H, C.byref(t), C.c_void_p(part.data_ptr()), None, None,
                                             C.byref(st)))
        if i >= 2:
            ks.append(st.kernel_ms)
    return round(float(np.median(ks)), 4)


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "synth1024"
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    scene = bench.load_workload(wl, W, H)[0]
    buf = np.empty((H, W, 4), dtype=np.uint8)
    reg = _abi.HostRegistration(buf)
    keep = []
    try:
        for i in range(k):
            ds = DeviceScene(scene)
            keep.append(ds)
            host = timed(lambda: ds.render_image(W, H, out=buf), 30)
            dev = kernel_ms(ds)
            print(json.dumps({"workload": wl, "instance": i, "host_pinned_ms": host, "device_single_launch_ms": dev}),
                  flush=True)
        # again, in reverse order: is it the instance or the time it ran?
        for i in reversed(range(k)):
            ds = keep[i]
            host = timed(lambda: ds.render_image(W, H, out=buf), 30)
            print(json.dumps({"workload": wl, "instance": i, "again_host_pinned_ms": host}), flush=True)
    finally:
        for ds in keep:
            ds.close()
        reg.close()


if __name__ == "__main__":
    main()
