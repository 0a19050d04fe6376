"""Single-launch latency of a rank's share (diagnostic).

For each workload: one latency-sized launch (rg_render_tiles_async with stats,
HIP events on its stream) of the whole frame and of every rank's 1/8 share
(8-row tiles, tile t -> rank t % 8), on an otherwise idle GPU; then, unless
--no-multi, the 1-GPU host-visible frame (pinned, rg_render_image) and the
8-device rg_render_multi rehearsal (each device's timeline alone, bench.py's
multi_rehearsal).  RAINGUN_HIP_LIB selects a variant library.

    python scripts/latency_probe.py [--no-multi] [--tile-order] [--lane-depth=N] [workload ...]   -> JSON on stdout
"""
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


def share_ms(ds, lib, stride, offset, reps=7):
    t = _abi.rg_tiling(T if stride > 1 else H, stride, offset)
    rows = lib.rg_tiling_rows(H, C.byref(t))
    part = torch.empty((rows, W, 4), dtype=torch.uint8, device="cuda")
    st = _abi.rg_stats()
    ks = []
    for i in range(reps + 2):
        _abi.check(lib.rg_render_tiles_async(ds.handle, W, H, C.byref(t), C.c_void_p(part.data_ptr()), None, None,
                                             C.byref(st)))
        if i >= 2:
            ks.append(st.kernel_ms)
    return float(np.median(ks)), st.rays.primary + st.rays.shadow + st.rays.secondary


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    multi = "--no-multi" not in sys.argv
    order = 1 if "--tile-order" in sys.argv else -1  # --tile-order: probe-ordered tiles on every path
    lane_depth = next((int(a.split("=", 1)[1]) for a in sys.argv if a.startswith("--lane-depth=")), -1)
    lib = _abi.lib()
    out = {"lib": str(getattr(lib, "_name", "")), "width": W, "height": H}
    for wl in args or ["test1", "synth1024"]:
        scene = bench.load_workload(wl, W, H)[0]
        ds = DeviceScene(scene)
        ds.set_tile_order(order)
        ds.set_lane_depth(lane_depth)
        r = {"tile_order": order, "lane_depth": lane_depth}
        r["whole_kernel_ms"], rays = share_ms(ds, lib, 1, 0)
        per = [share_ms(ds, lib, N, k) for k in range(N)]
        r["share8_kernel_ms"] = [round(p[0], 4) for p in per]
        r["share8_max_ms"] = round(max(p[0] for p in per), 4)
        r["whole_over_share8_max"] = round(r["whole_kernel_ms"] / r["share8_max_ms"], 2)
        r["whole_kernel_ms"] = round(r["whole_kernel_ms"], 4)
        r["rays_whole"] = rays
        if multi:
            buf = np.empty((H, W, 4), dtype=np.uint8)
            reg = _abi.HostRegistration(buf)
            try:
                for _ in range(3):
                    ds.render_image(W, H, out=buf)
                k, t0 = 0, time.perf_counter()
                while k < 10 or time.perf_counter() - t0 < 0.5:
                    ds.render_image(W, H, out=buf)
                    k += 1
                r["host_pinned_1gpu_ms"] = round((time.perf_counter() - t0) / k * 1e3, 4)
            finally:
                reg.close()

            class A:
                steps = 100
            r["multi_8gpu_rehearsal"] = bench.multi_rehearsal(ds, W, H, r["host_pinned_1gpu_ms"], A())
        ds.close()
        out[wl] = r
        print(json.dumps({wl: r}), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
