"""Makespan anatomy of one rank's share of a frame (diagnostic).

  python scripts/tail_probe.py curve      kernel ms vs share 1/N (normal build)
  RAINGUN_HIP_LIB=build/variants/tt/libraingun_hip.so python scripts/tail_probe.py timeline
                                          per-tile start/duration at N=1 and N=8
                                          (-DRG_TILE_TIMES build)

The timeline shows where a share's kernel time goes: the instant the queue
drained (last tile start), the slowest tiles, and how long the kernel ran on
after most waves had finished."""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from raingun_amd import _abi  # noqa: E402
from raingun_amd.scene import DeviceScene, load_scene  # noqa: E402
from raingun_amd.synth import synthetic_scene  # noqa: E402

G = Path(__file__).resolve().parent.parent / "tests" / "golden"
W, H = 3840, 2160


def scene(name):
    if name == "test1":
        sc = load_scene(G / "examples" / "test1.yml", texture_root=G)
        sc.max_recursion_depth = 5
        return sc
    return synthetic_scene(int(name[5:]), 2, 5)


def curve():
    out = {}
    for name in ("test1", "synth1024"):
        ds = DeviceScene(scene(name))
        res = {}
        for n in (1, 2, 4, 8, 16, 32, 64, 135):
            ks = []
            for _ in range(6):
                st = _abi.rg_stats()
                ds.render_tiles(W, H, 16, n, 0, stats=st)
                ks.append(st.kernel_ms)
            res[n] = round(float(np.median(ks[1:])), 4)
        out[name] = res
        ds.close()
    print(json.dumps(out, indent=1))


def timeline():
    out = {}
    for name in ("test1", "synth1024"):
        ds = DeviceScene(scene(name))
        for n in (1, 8):
            for _ in range(2):
                _, rgb = ds.render_tiles(W, H, 16, n, 0, want_rgb=True)
            rows = rgb.shape[0]
            nt = (W // 8) * ((rows + 7) // 8)
            f = rgb.reshape(-1)
            dur = f[:nt].astype(np.float64)
            iters = f[nt:2 * nt].astype(np.float64)
            tq = f[3 * nt:4 * nt].astype(np.float64)
            start = f[2 * nt:3 * nt].astype(np.int64)
            s0 = start.min()
            if start.max() - s0 > (1 << 23):  # 24-bit wrap
                start = np.where(start - s0 > (1 << 23), start - (1 << 24), start)
                s0 = start.min()
            st_us = (start - s0) * 0.01
            end_us = st_us + dur
            order = np.argsort(end_us)
            out[f"{name}_N{n}"] = {
                "tiles": int(nt),
                "makespan_us": round(float(end_us.max()), 1),
                "last_start_us": round(float(st_us.max()), 1),
                "end_p50_p90_p99_us": [round(float(x), 1) for x in np.percentile(end_us, [50, 90, 99])],
                "dur_p50_p99_max_us": [round(float(x), 1) for x in np.percentile(dur, [50, 99, 100])],
                "slowest5": [[round(float(st_us[i]), 1), round(float(dur[i]), 1)] for i in np.argsort(dur)[-5:]],
                "slowest5_iters_query_us": [[int(iters[i]), round(float(tq[i]), 1)] for i in np.argsort(dur)[-5:]],
                "query_frac_all": round(float(tq.sum() / dur.sum()), 3),
                # -DRG_BVH_STATS builds: [full-scan us, traversal us, scan lanes, wave traversals, traversal loop trips] of the slowest tiles
                "slowest5_scan_trav_us_lanes": [[round(float(f[k * nt + i]), 1) for k in (4, 5, 6, 7, 8)]
                                                for i in np.argsort(dur)[-5:]],
                "last5_end": [[round(float(st_us[i]), 1), round(float(dur[i]), 1)] for i in order[-5:]],
                "mean_dur_us": round(float(dur.mean()), 2),
            }
        ds.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    {"curve": curve, "timeline": timeline}[sys.argv[1]]()
