"""Kernel time of the per-lane BVH walk settings (rg_debug_set_lane_depth) on the
sphere workloads, whole frame (N=1) and one rank's 1/8 share (N=8).
  python scripts/lane_probe.py [depths...]   (default: 99 1 0)"""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from raingun_amd import _abi  # noqa: E402
from raingun_amd.synth import synthetic_scene  # noqa: E402
from raingun_amd.scene import DeviceScene  # noqa: E402

W, H = 3840, 2160
depths = [int(x) for x in sys.argv[1:]] or [99, 1, 0]
out = {}
for n, planes in ((1024, 2), (4096, 8)):
    ds = DeviceScene(synthetic_scene(n, planes, 5))
    for dpt in depths:
        ds.set_lane_depth(dpt)
        for share in (1, 8):
            ks = []
            for _ in range(5):
                st = _abi.rg_stats()
                ds.render_tiles(W, H, 16, share, 0, stats=st)
                ks.append(st.kernel_ms)
            out[f"synth{n}_lane{dpt}_N{share}"] = round(float(np.median(ks[1:])), 4)
            print(f"synth{n} lane_depth {dpt} share 1/{share}: {out[f'synth{n}_lane{dpt}_N{share}']:.3f} ms", flush=True)
    ds.close()
print(json.dumps(out))
