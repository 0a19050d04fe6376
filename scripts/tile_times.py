"""Per-8x8-tile wall time distribution (diagnostic; needs a -DRG_TILE_TIMES
build via RAINGUN_HIP_LIB).  Shows whether a frame's makespan at small
per-GPU shares is bounded by its slowest tiles."""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from raingun_amd.scene import DeviceScene, load_scene  # noqa: E402
from raingun_amd.synth import synthetic_scene  # noqa: E402

G = Path(__file__).resolve().parent.parent / "tests" / "golden"
out = {}
for name in ("test1", "synth1024"):
    if name == "test1":
        sc = load_scene(G / "examples" / "test1.yml", texture_root=G)
        sc.max_recursion_depth = 5
    else:
        sc = synthetic_scene(1024, 2, 5)
    ds = DeviceScene(sc)
    W, H = 3840, 2160
    ntiles = (W // 8) * (H // 8)
    for _ in range(2):
        _, rgb = ds.render_tiles(W, H, want_rgb=True)
    t = rgb.reshape(-1)[:ntiles].astype(np.float64)
    it = rgb.reshape(-1)[ntiles:2 * ntiles].astype(np.float64)
    q = np.percentile(t, [50, 90, 99, 99.9, 100])
    grid = t.reshape(H // 8, W // 8)
    out[name] = {"tiles": ntiles, "mean_us": round(float(t.mean()), 2),
                 "p50_p90_p99_p999_max_us": [round(float(x), 2) for x in q],
                 "sum_ms": round(float(t.sum()) / 1e3, 2),
                 "iters_p50_p99_max": [float(x) for x in np.percentile(it, [50, 99, 100])],
                 "us_per_iter_p50_p99": [round(float(x), 2) for x in np.percentile(t / np.maximum(it, 1), [50, 99])],
                 "slowest_tiles_iters": [int(it[i]) for i in np.argsort(t)[-5:]],
                 "slowest_tiles_rc": [[int(i // (W // 8)), int(i % (W // 8))] for i in np.argsort(t)[-5:]],
                 "row_band_mean_us": [round(float(grid[r:r + 27].mean()), 1) for r in range(0, H // 8, 27)]}
    ds.close()
print(json.dumps(out, indent=1))
