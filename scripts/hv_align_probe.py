#!/usr/bin/env python3
"""Host-visible frame into page-locked memory against the caller buffer's placement: the same
rg_render_image of one workload into buffers at different offsets from a 2 MiB boundary, with and
without MADV_HUGEPAGE, interleaved.  The kernel's stores cross PCIe into these pages, so the
buffer's page size (IOMMU translations) can matter.

    python scripts/hv_align_probe.py [workload] [rounds]   -> JSON lines
"""
import ctypes
import json
import mmap
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from raingun_amd import _abi  # noqa: E402
from raingun_amd.scene import DeviceScene  # noqa: E402

W, H = 3840, 2160
MB2 = 2 << 20
MADV_HUGEPAGE, MADV_NOHUGEPAGE = 14, 15


def thp_setting():
    try:
        return Path("/sys/kernel/mm/transparent_hugepage/enabled").read_text().strip()
    except OSError:
        return "?"


def placed(nbytes, offset, advice):
    """nbytes at `offset` past a 2 MiB boundary of a fresh anonymous mapping, madvise'd."""
    m = mmap.mmap(-1, nbytes + 2 * MB2, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    raw = np.frombuffer(m, dtype=np.uint8)
    base = raw.ctypes.data
    start = (-base) % MB2 + offset
    if advice is not None:
        libc = ctypes.CDLL(None, use_errno=True)
        libc.madvise(ctypes.c_void_p(base), ctypes.c_size_t(len(raw)), ctypes.c_int(advice))
    buf = raw[start:start + nbytes]
    buf[:] = 0  # fault the pages in (with the advice in force)
    return m, buf.reshape(H, W, 4)


def time_frames(ds, buf, n=40):
    for _ in range(3):
        ds.render_image(W, H, out=buf)
    t0 = time.perf_counter()
    for _ in range(n):
        ds.render_image(W, H, out=buf)
    return (time.perf_counter() - t0) / n * 1e3


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "synth1024"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    scene = bench.load_workload(wl, W, H)[0]
    ds = DeviceScene(scene)
    ref = ds.render_image(W, H)
    cases = [("aligned_2M_huge", 0, MADV_HUGEPAGE), ("aligned_2M_nohuge", 0, MADV_NOHUGEPAGE),
             ("offset_4K_huge", 4096, MADV_HUGEPAGE), ("offset_1M_default", 1 << 20, None),
             ("numpy_empty", None, None)]
    print(json.dumps({"thp": thp_setting(), "workload": wl}), flush=True)
    try:
        for r in range(rounds):
            for name, off, adv in cases:
                if off is None:
                    m, buf = None, np.empty((H, W, 4), dtype=np.uint8)
                else:
                    m, buf = placed(H * W * 4, off, adv)
                reg = _abi.HostRegistration(buf)
                try:
                    ms = time_frames(ds, buf)
                    ok = bool(np.array_equal(buf, ref))
                finally:
                    reg.close()
                print(json.dumps({"round": r, "case": name, "addr_mod_2M": buf.ctypes.data % MB2, "ms": round(ms, 4),
                                  "ok": ok}), flush=True)
                del buf
                if m is not None:
                    m.close()
    finally:
        ds.close()


if __name__ == "__main__":
    main()
