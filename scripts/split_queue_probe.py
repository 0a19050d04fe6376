#!/usr/bin/env python3
"""The light path's split host frame (rg_render_image into page-locked memory: a device-resident
part + DMA on one render stream, a one-launch part writing host memory on another) against where
its streams land among the process's hardware queues: before each fresh DeviceScene, K extra HIP
streams are created (and kept until the scene is closed), shifting the queues its streams get.
profiles/r06/s32: two of three test1 instances ran the split frame at 1.06 ms instead of 0.80.

    GPU_MAX_HW_QUEUES=16 python scripts/split_queue_probe.py [workload] [kmax]   -> JSON lines
"""
import ctypes
import json
import os
import sys
import time
from pathlib import Path

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from raingun_amd import _abi  # noqa: E402
from raingun_amd.scene import DeviceScene  # noqa: E402

W, H = 3840, 2160


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "test1"
    kmax = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    hip = ctypes.CDLL("libamdhip64.so")
    scene = bench.load_workload(wl, W, H)[0]
    buf = np.empty((H, W, 4), dtype=np.uint8)
    reg = _abi.HostRegistration(buf)
    try:
        for k in range(kmax):
            extra = []
            for _ in range(k):
                s = ctypes.c_void_p()
                assert hip.hipStreamCreate(ctypes.byref(s)) == 0
                extra.append(s)
            ds = DeviceScene(scene)
            for _ in range(3):
                ds.render_image(W, H, out=buf)
            t0 = time.perf_counter()
            for _ in range(30):
                ds.render_image(W, H, out=buf)
            ms = (time.perf_counter() - t0) / 30 * 1e3
            ds.close()
            for s in extra:
                hip.hipStreamDestroy(s)
            print(json.dumps({"workload": wl, "extra_streams": k, "pinned_ms": round(ms, 4)}), flush=True)
    finally:
        reg.close()


if __name__ == "__main__":
    main()
