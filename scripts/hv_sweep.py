#!/usr/bin/env python3
"""Host-visible rg_render_image: ms per 4K frame against the host path
setting, into a page-locked and a pageable buffer.  A setting is `bands`
(rg_debug_set_image_bands: 0 automatic, -1 one launch writing host memory,
k row bands), `-1:<tile_wlog>` (one launch with that tile shape; 0 automatic)
or `-1:<tile_wlog>:<tile order>` (rg_debug_set_tile_order: -1 automatic,
0 raster, 1 cost-ordered); `-2:0:-1:<pct>`: split frames with pct percent of
the rows rendered into device memory and copied by DMA.
  python scripts/hv_sweep.py [--workload test1|synth1024] [--pinned] [setting ...]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from bench import load_workload
    from raingun_amd import _abi
    from raingun_amd.scene import DeviceScene

    W, H = 3840, 2160
    args = sys.argv[1:]
    wl = "test1"
    if args[:1] == ["--workload"]:
        wl, args = args[1], args[2:]
    scene, *_ = load_workload(wl, W, H)
    ds = DeviceScene(scene, device=0)
    lib = _abi.lib()
    ref = ds.render_image(W, H)
    kinds = ("pinned", "pageable")
    if args[:1] == ["--pinned"]:
        kinds, args = ("pinned",), args[1:]
    settings = args or ["0", "-1:6", "-1:5", "-1:3", "3"]
    for kind in kinds:
        buf = np.empty((H, W, 4), dtype=np.uint8)
        reg = _abi.HostRegistration(buf) if kind == "pinned" else None
        for setting in settings:
            k, _, rest = setting.partition(":")
            shape, _, rest = rest.partition(":")
            order, _, pct = rest.partition(":")
            k = int(k)
            ds.set_tile_order(int(order) if order else -1)
            if hasattr(_abi.lib(), "rg_debug_set_host_split"):
                ds.set_host_split(int(pct) if pct else 0)
            _abi.check(lib.rg_debug_set_image_bands(ds.handle, k))
            if shape and int(shape):
                ds.set_host_tile_shape(int(shape))
            else:  # the automatic shape (libraries before round 3's tile ring reject 0: their default is 8x8)
                lib.rg_debug_set_host_tile_shape(ds.handle, 0)
            for _ in range(3):
                ds.render_image(W, H, out=buf)
            n, t0 = 0, time.perf_counter()
            while n < 40:
                ds.render_image(W, H, out=buf)
                n += 1
            dt = (time.perf_counter() - t0) / n
            assert np.array_equal(buf, ref)
            print(json.dumps({"workload": wl, "kind": kind, "setting": setting, "ms": round(dt * 1e3, 4),
                              "GBps": round(W * H * 4 / dt / 1e9, 2)}), flush=True)
        if reg is not None:
            reg.close()
    ds.close()


if __name__ == "__main__":
    main()
