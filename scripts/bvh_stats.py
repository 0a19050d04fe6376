"""BVH traversal statistics on the north-star scene (diagnostic).

Run with RAINGUN_HIP_LIB pointing at a -DRG_BVH_STATS build
(scripts/build_variants.sh bvhstats=-DRG_BVH_STATS).  Prints, per ray class
mix of a 3840x2160 depth-5 frame: wave traversals, node visits and leaf visits
per traversal, lanes per traversal (coherence), fallback lanes.
clock_traversal_frac is the wave-coherent walk's share of wave time and
clock_fullscan_frac the per-lane walk's (with the full scans, ~0.05 %)."""
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from raingun_amd import _abi  # noqa: E402
from raingun_amd.scene import DeviceScene  # noqa: E402
from raingun_amd.synth import synthetic_scene  # noqa: E402

out = {}
for name, (n, planes, depth, w, h) in {"synth1024_4k_d5": (1024, 2, 5, 3840, 2160),
                                      "synth4096p8_1080p_d8": (4096, 8, 8, 1920, 1080)}.items():
    ds = DeviceScene(synthetic_scene(n, planes, depth))
    st = _abi.rg_stats()
    ds.set_image_bands(1)  # one launch: rg_debug_counters reads the last launch's words
    ds.render_tiles(w, h, stats=st)
    c = (C.c_uint64 * 16)()
    _abi.check(_abi.lib().rg_debug_counters(ds.handle, c))
    trav, nodes, leaves, lanes, fallback = c[4], c[5], c[6], c[7], c[8]
    rays = st.rays.total()
    out[name] = dict(rays=rays, kernel_ms=round(st.kernel_ms, 3), traversals=trav, lanes_per_traversal=lanes / max(trav, 1),
                     nodes_per_traversal=nodes / max(trav, 1), leaves_per_traversal=leaves / max(trav, 1),
                     scan_lanes=fallback, scan_frac=fallback / max(rays, 1),
                     clipped_start_lanes=c[9], no_sphere_lanes=c[10], nan_lanes=c[11],
                     clock_traversal_frac=c[12] / max(c[14], 1), clock_fullscan_frac=c[13] / max(c[14], 1),
                     waves=c[15])
    ds.close()
print(json.dumps(out, indent=1))
