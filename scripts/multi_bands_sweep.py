"""rg_render_multi's 8-device rehearsal (bench.py multi_rehearsal) for several band
counts per device share (rg_debug_set_multi bands: -1 = one launch writing the
caller's pinned frame, 0 = automatic, K > 0 = K bands with per-band copies).
    python scripts/multi_bands_sweep.py [workload ...]   -> JSON lines"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from raingun_amd import _abi  # noqa: E402
from raingun_amd.scene import DeviceScene  # noqa: E402

W, H, N = 3840, 2160, 8


def device_ms(ds, buf, bands, r, budget_s=0.4):
    ds.set_multi(0, stand_in=True, bands=bands, only_rank=r)
    for _ in range(2):
        ds.render_multi(W, H, N, 8, out=buf)
    k, t0 = 0, time.perf_counter()
    while k < 5 or (time.perf_counter() - t0 < budget_s and k < 200):
        ds.render_multi(W, H, N, 8, out=buf)
        k += 1
    return (time.perf_counter() - t0) / k * 1e3


def main():
    for wl in sys.argv[1:] or ["test1"]:
        ds = DeviceScene(bench.load_workload(wl, W, H)[0])
        ref = ds.render_image(W, H)
        buf = np.empty((H, W, 4), dtype=np.uint8)
        reg = _abi.HostRegistration(buf)
        try:
            for bands in (0, -1, 1, 2, 3, 4):
                per = [device_ms(ds, buf, bands, r) for r in range(N)]
                ds.set_multi(0, stand_in=True, bands=bands, only_rank=-1)
                ds.render_multi(W, H, N, 8, out=buf)  # all 8 stand-in devices: the whole frame
                ok = bool(np.array_equal(buf, ref))
                print(json.dumps({"workload": wl, "bands": bands, "projected_ms": round(max(per), 4),
                                  "per_device_ms": [round(x, 4) for x in per], "frame_equal": ok}), flush=True)
        finally:
            ds.set_multi(0, stand_in=False, bands=0, only_rank=-1)
            reg.close()
            ds.close()


if __name__ == "__main__":
    main()
