#!/usr/bin/env python3
"""Region visit counts of the render loop (library built with -DRG_REGION_STATS, e.g.
scripts/build_variants.sh region="-DRG_REGION_STATS", run with RAINGUN_HIP_LIB=abvar/region/...).

One whole-frame launch (the headline instantiation: 3840x2160, 16 tiles per wave) per workload;
prints, per RG_REGION marker (rg_kernels.hip), how many times a wave entered the region and the
mean active lanes on entry.  scripts/isa_budget.py --visits multiplies these by each region's
static instructions.

    python scripts/region_stats.py [workload] [--size WxH] [--json out.json] [--lib abvar/region/libraingun_hip.so]
"""
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

BASE = 144


def names():
    txt = (Path(__file__).resolve().parents[1] / "raingun_amd" / "csrc" / "rg_kernels.hip").read_text()
    body = txt[txt.index("RGR_LOOP = 0"):txt.index("RGR_COUNT")]
    return [n.split("=")[0].strip() for n in body.replace("\n", " ").split(",") if n.strip()]


def main():
    if "--lib" in sys.argv:  # the RG_REGION_STATS build (before _abi loads the default library)
        import os
        k = sys.argv.index("--lib")
        os.environ["RAINGUN_HIP_LIB"] = str(Path(sys.argv[k + 1]).resolve())
        del sys.argv[k:k + 2]
    from bench import load_workload
    from raingun_amd import _abi
    from raingun_amd.scene import DeviceScene

    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    size = sys.argv[sys.argv.index("--size") + 1] if "--size" in sys.argv else "3840x2160"
    for v in (out, size):
        if v in args:
            args.remove(v)
    W, H = (int(v) for v in size.split("x"))
    wl = args[0] if args else "test1"
    scene, *_ = load_workload(wl, W, H)
    ds = DeviceScene(scene, device=0)
    st = _abi.rg_stats()
    ds.set_image_bands(1)
    ds.render_tiles(W, H, stats=st)
    rn = names()
    w = (C.c_uint64 * (2 * len(rn)))()
    _abi.check(_abi.lib().rg_debug_counter_words(ds.handle, BASE, 2 * len(rn), w))
    ds.close()
    regs = {n: {"visits": int(w[2 * k]), "lanes_per_visit": round(int(w[2 * k + 1]) / max(int(w[2 * k]), 1), 2)}
            for k, n in enumerate(rn)}
    res = {"workload": wl, "width": W, "height": H, "rays": st.rays.as_dict(), "regions": regs}
    text = json.dumps(res, indent=1)
    if out:
        Path(out).write_text(text)
    print(text)


if __name__ == "__main__":
    main()
