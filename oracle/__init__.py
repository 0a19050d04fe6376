"""ctypes wrapper of oracle/liboracle.so — the CPU restatement of raingun's
render path (raingun_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, and only as the checker / CPU baseline.  The
product path (raingun_amd, libraingun_hip.so) never imports this package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "liboracle.so"

_LIB = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)
    return LIB_PATH


def lib():
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            build()
        from raingun_amd import _abi

        l = C.CDLL(str(LIB_PATH))
        P = C.POINTER
        l.rgo_render.restype = C.c_int32
        l.rgo_render.argtypes = [P(_abi.rg_scene_desc), C.c_uint32, C.c_uint32, P(_abi.rg_tiling), C.c_void_p,
                                 C.c_void_p, P(_abi.rg_ray_counts), C.c_int32, P(C.c_int64)]
        l.rgo_trace.restype = C.c_int32
        l.rgo_trace.argtypes = [P(_abi.rg_scene_desc), C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
        l.rgo_fresnel.restype = C.c_double
        l.rgo_fresnel.argtypes = [C.c_double] * 6 + [C.c_float]
        l.rgo_wrap.restype = C.c_uint32
        l.rgo_wrap.argtypes = [C.c_float, C.c_uint32]
        l.rgo_f32_to_u8.restype = C.c_uint8
        l.rgo_f32_to_u8.argtypes = [C.c_float]
        l.rgo_f32_to_i32.restype = C.c_int32
        l.rgo_f32_to_i32.argtypes = [C.c_float]
        l.rgo_fov_adjustment.restype = C.c_double
        l.rgo_fov_adjustment.argtypes = [C.c_double]
        l.rgo_tiling_rows.restype = C.c_uint32
        l.rgo_tiling_rows.argtypes = [C.c_uint32, P(_abi.rg_tiling)]
        _LIB = l
    return _LIB


def default_threads() -> int:
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return max(1, min(len(os.sched_getaffinity(0)), 64))
    except AttributeError:  # pragma: no cover
        return max(1, min(os.cpu_count() or 1, 64))


def render(scene_desc, width: int, height: int, tile_rows: int = 0, stride: int = 1, offset: int = 0,
           want_rgb: bool = False, threads: int = 0):
    """Render with the CPU restatement.  Returns (status, rgba, rgb|None, counts dict, error_pixel)."""
    from raingun_amd import _abi

    t = _abi.rg_tiling(tile_rows or height, stride, offset)
    rows = lib().rgo_tiling_rows(height, C.byref(t))
    rgba = np.zeros((rows, width, 4), dtype=np.uint8)
    rgb = np.zeros((rows, width, 3), dtype=np.float32) if want_rgb else None
    counts = _abi.rg_ray_counts()
    err = C.c_int64(-1)
    st = lib().rgo_render(scene_desc.ptr(), width, height, C.byref(t), rgba.ctypes.data,
                          rgb.ctypes.data if rgb is not None else None, C.byref(counts),
                          threads or default_threads(), C.byref(err))
    return st, rgba, rgb, counts.as_dict(), int(err.value)


def trace(scene_desc, rays: np.ndarray):
    rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
    n = rays.shape[0]
    dist = np.empty(n, dtype=np.float64)
    body = np.empty(n, dtype=np.int32)
    st = lib().rgo_trace(scene_desc.ptr(), rays.ctypes.data, n, dist.ctypes.data, body.ctypes.data)
    return st, dist, body
