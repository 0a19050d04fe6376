"""Per-wave timeline of ONE launch (diagnostic; VERDICT r3 item 1: "per-wave
start/end stamps").  Needs a -DRG_WAVE_TIMES build (RAINGUN_HIP_LIB): every
wave of rg_render_kernel writes its start (before LDS staging), staging end,
end (100 MHz wall clock) and tile count into the rgb buffer.

For the whole 4K frame and rank 0's 1/8 share (8-row tiles) of each workload,
one latency-sized launch (rg_render_tiles_async): how fast the waves start (the
dispatch ramp), how long they live, how many run at once, when they end.
    RAINGUN_HIP_LIB=abvar/wt/libraingun_hip.so python scripts/wave_times.py [workload ...]
"""
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from raingun_amd import _abi  # noqa: E402
from raingun_amd.scene import DeviceScene  # noqa: E402

W, H = 3840, 2160


def pct(v, qs=(0, 10, 50, 90, 99, 100)):
    return [round(float(x), 1) for x in np.percentile(v, qs)]


def one(ds, lib, stride):
    t = _abi.rg_tiling(8 if stride > 1 else H, stride, 0)
    rows = lib.rg_tiling_rows(H, C.byref(t))
    rgba = torch.empty((rows, W, 4), dtype=torch.uint8, device="cuda")
    res = None
    for rep in range(3):
        rgb = torch.zeros((rows * W * 3,), dtype=torch.float32, device="cuda")
        st = _abi.rg_stats()
        _abi.check(lib.rg_render_tiles_async(ds.handle, W, H, C.byref(t), C.c_void_p(rgba.data_ptr()),
                                             C.c_void_p(rgb.data_ptr()), None, C.byref(st)))
        torch.cuda.synchronize()
        w = rgb.view(torch.int32).cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        w = w[: (w.size // 4) * 4].reshape(-1, 4)
        live = w[(w[:, 2] > 0) | (w[:, 3] > 0)]
        s0 = live[:, 0]
        s0 = np.where(s0 - s0.min() > (1 << 31), s0 - (1 << 32), s0)  # 32-bit wrap
        start = (s0 - s0.min()) * 0.01  # us
        staged = start + live[:, 1] * 0.01
        end = start + live[:, 2] * 0.01
        ev = np.concatenate([start, end])
        order = np.argsort(ev, kind="stable")
        conc = np.cumsum(np.where(order < len(start), 1, -1))
        res = {"kernel_ms": round(st.kernel_ms, 4), "waves": int(len(live)),
               "start_us_p0_10_50_90_99_100": pct(start),
               "staging_us_p50_p99": [round(float(x), 2) for x in np.percentile(live[:, 1] * 0.01, (50, 99))],
               "life_us_p0_10_50_90_99_100": pct(end - start),
               "end_us_p0_10_50_90_99_100": pct(end),
               "tiles_per_wave_p0_50_100": [int(x) for x in np.percentile(live[:, 3], (0, 50, 100))],
               "max_concurrent_waves": int(conc.max()),
               "waves_alive_at_25_50_75pct_of_makespan": [
                   int(((start <= f * end.max()) & (end > f * end.max())).sum()) for f in (0.25, 0.5, 0.75)]}
        del staged
    return res


def main():
    lib = _abi.lib()
    out = {"lib": str(getattr(lib, "_name", ""))}
    for wl in sys.argv[1:] or ["test1", "synth1024"]:
        ds = DeviceScene(bench.load_workload(wl, W, H)[0])
        out[wl] = {"whole": one(ds, lib, 1), "share8": one(ds, lib, 8)}
        print(json.dumps({wl: out[wl]}), file=sys.stderr, flush=True)
        ds.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
