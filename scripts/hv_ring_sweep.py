#!/usr/bin/env python3
"""Light-path host frames: sweep of the one-launch host-frame kernels' knobs (rg_debug_set_host_ring)
on the two consumers -- the 1-GPU frame into a pinned buffer (rg_render_image: split frames, part B
one launch of ~65 % of the frame) and rg_render_multi's 8-device rehearsal with each device's share
as ONE launch storing its rows over its own link (bench.multi_rehearsal, stand-in devices).

    python scripts/hv_ring_sweep.py [workload]   -> JSON lines on stdout
"""
import itertools
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from raingun_amd import _abi  # noqa: E402
from raingun_amd.scene import DeviceScene  # noqa: E402

W, H = 3840, 2160


def pinned_ms(ds, buf, budget=0.4):
    for _ in range(3):
        ds.render_image(W, H, out=buf)
    k, t0 = 0, time.perf_counter()
    while k < 10 or time.perf_counter() - t0 < budget:
        ds.render_image(W, H, out=buf)
        k += 1
    return (time.perf_counter() - t0) / k * 1e3


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "test1"
    scene = bench.load_workload(wl, W, H)[0]
    ds = DeviceScene(scene)
    ref = ds.render_image(W, H)
    buf = np.empty((H, W, 4), dtype=np.uint8)
    reg = _abi.HostRegistration(buf)

    class A:
        steps = 60
    try:
        for flush in (16, 8, 4):
            ds.set_host_ring(flush_big=flush, group_big=flush, multi_light_one=0)
            ms = pinned_ms(ds, buf)
            assert np.array_equal(buf, ref)
            print(json.dumps({"workload": wl, "case": "pinned_1gpu", "flush_big": flush, "ms": round(ms, 4)}), flush=True)
        ds.set_host_ring(flush_big=8, group_big=8, multi_light_one=0)
        r = bench.multi_rehearsal(ds, W, H, 1.0, A(), budget_s=0.25)
        print(json.dumps({"workload": wl, "case": "multi_bands", "per_device_ms": r["per_device_ms"],
                          "projected_ms": r["projected_ms_per_step"]}), flush=True)
        for flush, group in ((8, 1), (4, 1), (4, 2), (2, 1), (2, 2), (1, 1)):
            ds.set_host_ring(flush_small=flush, group_small=group, multi_light_one=1)
            r = bench.multi_rehearsal(ds, W, H, 1.0, A(), budget_s=0.25)
            print(json.dumps({"workload": wl, "case": "multi_one_launch", "flush_small": flush, "group_small": group,
                              "per_device_ms": r["per_device_ms"], "projected_ms": r["projected_ms_per_step"]}),
                  flush=True)
        # the whole frame over 8 stand-in devices with the last setting equals the 1-GPU frame
        ds.set_multi(0, stand_in=True, bands=0, only_rank=-1)
        got = ds.render_multi(W, H, 8, 8, out=buf)
        assert np.array_equal(buf, ref)
        print(json.dumps({"workload": wl, "case": "verify_multi_equals_image", "ok": True}), flush=True)
    finally:
        ds.set_multi(0, stand_in=False, bands=0, only_rank=-1)
        reg.close()
        ds.close()


if __name__ == "__main__":
    main()
