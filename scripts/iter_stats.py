#!/usr/bin/env python3
"""SIMD use of the render loop's query iterations (library built with
-DRG_ITER_STATS, e.g. scripts/build_variants.sh iter="-DRG_ITER_STATS", run
with RAINGUN_HIP_LIB=abvar/iter/libraingun_hip.so): per workload at 3840x2160,
the mean querying lanes per wave iteration overall, in iterations holding a
ray of depth >= 1, the share of iterations with <= 16 querying lanes.
  python scripts/iter_stats.py [workload ...]"""
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from bench import load_workload
    from raingun_amd import _abi
    from raingun_amd.scene import DeviceScene

    for wl in sys.argv[1:] or ["test1", "synth1024", "synth1024p2d1"]:
        scene, *_ = load_workload(wl, 3840, 2160)
        ds = DeviceScene(scene, device=0)
        st = _abi.rg_stats()
        ds.set_image_bands(1)  # one launch: rg_debug_counters reads the last launch's words
        ds.render_tiles(3840, 2160, stats=st)
        w = (C.c_uint64 * 16)()
        _abi.check(_abi.lib().rg_debug_counters(ds.handle, w))
        ds.close()
        it, lanes, it2, lanes2, sec2, low, its, shl, lw_it, lw_l, lf_it, lf_l = (int(w[k]) for k in range(4, 16))
        print(json.dumps({"workload": wl, "rays": st.rays.as_dict(), "query_iterations": it,
                          "lanes_per_iteration": round(lanes / max(it, 1), 2),
                          "iterations_with_depth_ge1": it2, "lanes_per_such_iteration": round(lanes2 / max(it2, 1), 2),
                          "depth_ge1_lanes_per_such_iteration": round(sec2 / max(it2, 1), 2),
                          "share_iterations_le16_lanes": round(low / max(it, 1), 3),
                          "iterations_with_shadow_lanes": its, "shadow_lanes_per_such": round(shl / max(its, 1), 2),
                          "lane_walk_iterations": lw_it, "lane_walk_active_lanes": round(lw_l / max(lw_it, 1), 2),
                          "leaf_iterations": lf_it, "leaf_lanes": round(lf_l / max(lf_it, 1), 2),
                          # light path: words 14/15 count iterations with closest-hit lanes instead
                          "light_mixed_iterations": its + lf_it - it if wl.startswith("test") else None}),
              flush=True)


if __name__ == "__main__":
    main()
