#!/usr/bin/env python3
"""A/B kernel variants in interleaved rounds (one subprocess per variant per round).

usage: python scripts/bench_variants.py [--rounds R] [--frames K] [--workloads test1,synth1024] v1 v2 ...
Each variant is abvar/<name>/libraingun_hip.so.  Every run first checks
the variant bit-exactly against the CPU restatement on small frames.
"""
import argparse, json, os, subprocess, sys, time
from pathlib import Path
REPO = Path(__file__).resolve().parent.parent

CHILD = r'''
import sys, time, json, ctypes as C
sys.path.insert(0, %(repo)r)
import numpy as np
from raingun_amd import _abi
from raingun_amd.scene import DeviceScene, SceneDesc, load_scene
from raingun_amd.synth import synthetic_scene
import oracle
G = %(repo)r + "/tests/golden"
out = {}
# parity gate (skipped for timing-only ablations)
for name, sc, w, h in [("test1", load_scene(G + "/examples/test1.yml", texture_root=G), 160, 120),
                       ("synth64", synthetic_scene(64, 2, 5), 160, 90)]:
    ds = DeviceScene(sc); g = ds.render_tiles(w, h); ds.close()
    st, o, _, _, _ = oracle.render(SceneDesc(sc), w, h)
    assert %(noparity)r or np.array_equal(g, o), "variant differs from oracle on " + name
for wl in %(workloads)r:
    if wl == "test1":
        sc = load_scene(G + "/examples/test1.yml", texture_root=G); sc.max_recursion_depth = 5
    elif wl.startswith("synth"):
        sc = synthetic_scene(int(wl[5:]), 2, 5)
    ds = DeviceScene(sc)
    stt = _abi.rg_stats()
    ds.render_tiles(3840, 2160, stats=stt)
    ms = []
    import torch
    buf = torch.empty((2160, 3840, 4), dtype=torch.uint8, device="cuda")
    t = _abi.rg_tiling(2160, 1, 0)
    for i in range(%(frames)d):
        s2 = _abi.rg_stats()
        st = _abi.lib().rg_render_tiles_async(ds.handle, 3840, 2160, C.byref(t), C.c_void_p(buf.data_ptr()), None, None, C.byref(s2))
        assert st == 0
        ms.append(s2.kernel_ms)
    ds.close()
    rays = stt.rays.primary + stt.rays.shadow + stt.rays.secondary
    out[wl] = {"ms_med": float(np.median(ms)), "ms_min": float(np.min(ms)), "mrays": rays / np.median(ms) / 1e3}
print("RESULT " + json.dumps(out))
'''

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--workloads", default="test1,synth1024")
    ap.add_argument("--no-parity", action="store_true", help="timing-only ablation builds")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    wls = a.workloads.split(",")
    res = {v: [] for v in a.variants}
    for r in range(a.rounds):
        for v in a.variants:
            lib = REPO / "build" / "variants" / v / "libraingun_hip.so"
            env = dict(os.environ, RAINGUN_HIP_LIB=str(lib))
            code = CHILD % {"repo": str(REPO), "workloads": wls, "frames": a.frames, "noparity": a.no_parity}
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
            line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(f"[{v}] FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            d = json.loads(line[0][7:])
            res[v].append(d)
            print(f"round {r} {v}: " + "  ".join(f"{w} {d[w]['ms_med']:.3f}ms {d[w]['mrays']:.0f}Mr/s" for w in wls), flush=True)
    print("SUMMARY")
    for v in a.variants:
        flags = (REPO / "build" / "variants" / v / "flags.txt").read_text().strip()
        print(f"{v:>12} [{flags}]: " + "  ".join(
            f"{w} best {min(x[w]['ms_med'] for x in res[v]):.3f}ms" for w in wls))

if __name__ == "__main__":
    main()
