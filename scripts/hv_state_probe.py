#!/usr/bin/env python3
"""Why bench.py's host_visible_north_star line reads 2.36-2.38 ms after a second 4K pipelined
line but 2.0-2.13 ms otherwise (profiles/r06/s17): in ONE process, time the north-star frame into
page-locked memory (rg_render_image) before and after a pipelined 4K measure (bench.measure of
`between`), into the buffer registered before it and into a freshly allocated and registered one.

    python scripts/hv_state_probe.py [between_workload]   -> JSON lines
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


def frames_ms(ds, buf, n=40):
    for _ in range(3):
        ds.render_image(W, H, out=buf)
    t0 = time.perf_counter()
    for _ in range(n):
        ds.render_image(W, H, out=buf)
    return round((time.perf_counter() - t0) / n * 1e3, 4)


def main():
    between = sys.argv[1] if len(sys.argv) > 1 else "test3"
    args = bench.parse_args(["--no-cpu-baseline"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    bench.measure("test1", args, 1, 0, 0, dev, False)  # what bench.py runs first

    scene = bench.load_workload("synth1024", W, H)[0]
    ds = DeviceScene(scene)
    old = np.empty((H, W, 4), dtype=np.uint8)
    reg_old = _abi.HostRegistration(old)
    out = {"before": frames_ms(ds, old)}
    r = bench.measure(between, args, 1, 0, 0, dev, False, warmup=5, budget_s=3.0)
    out["between"] = f"{between}: {r['ms_per_step']} ms"
    out["after_old_buffer_same_scene"] = frames_ms(ds, old)
    new = np.empty((H, W, 4), dtype=np.uint8)
    reg_new = _abi.HostRegistration(new)
    out["after_new_buffer_same_scene"] = frames_ms(ds, new)
    ds2 = DeviceScene(scene)
    out["after_new_buffer_new_scene"] = frames_ms(ds2, new)
    out["after_old_buffer_new_scene"] = frames_ms(ds2, old)
    ds2.close()
    torch.cuda.empty_cache()
    out["after_empty_cache_old_buffer"] = frames_ms(ds, old)
    reg_new.close()
    reg_old.close()
    ds.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
