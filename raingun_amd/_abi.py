"""ctypes mirror of include/raingun.h and the loader for libraingun_hip.so.

The product path is the HIP library.  There is no CPU fallback: if the
shared object is missing or fails to load, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
LIB_PATH = PKG_DIR / "libraingun_hip.so"

# ---------------------------------------------------------------- enums
RG_OK = 0
RG_ERR_INVALID_ARGUMENT = -1
RG_ERR_PORTRAIT = -2
RG_ERR_AABB_NORMAL = -3
RG_ERR_NAN_DISTANCE = -4
RG_ERR_TRANSMISSION = -5
RG_ERR_TEXTURE = -6
RG_ERR_DEVICE = -10
RG_ERR_OUT_OF_MEMORY = -11
RG_ERR_CANCELLED = -12
RG_ERR_COLLECTIVE = -13
RG_ERR_PENDING = -14

BODY_SPHERE, BODY_PLANE, BODY_DISK, BODY_AABB = 0, 1, 2, 3
COLORATION_COLOR, COLORATION_TEXTURE = 0, 1
SURFACE_DIFFUSE, SURFACE_REFLECTING, SURFACE_REFRACTIVE = 0, 1, 2
LIGHT_DIRECTIONAL, LIGHT_SPHERICAL = 0, 1


# ---------------------------------------------------------------- structs
class rg_material(C.Structure):
    _fields_ = [
        ("coloration", C.c_uint32),
        ("color", C.c_float * 3),
        ("texture", C.c_int32),
        ("x_offset", C.c_float),
        ("y_offset", C.c_float),
        ("albedo", C.c_float),
        ("surface", C.c_uint32),
        ("reflectivity", C.c_float),
        ("index", C.c_float),
        ("transparency", C.c_float),
    ]


class rg_body(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32),
        ("_pad", C.c_uint32),
        ("p", C.c_double * 7),
        ("material", rg_material),
    ]


class rg_light(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32),
        ("color", C.c_float * 3),
        ("intensity", C.c_float),
        ("_pad", C.c_uint32),
        ("v", C.c_double * 3),
    ]


class rg_texture(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("rgba", C.POINTER(C.c_uint8))]


class rg_scene_desc(C.Structure):
    _fields_ = [
        ("fov", C.c_double),
        ("default_color", C.c_float * 3),
        ("max_recursion_depth", C.c_uint32),
        ("n_bodies", C.c_uint32),
        ("bodies", C.POINTER(rg_body)),
        ("n_lights", C.c_uint32),
        ("lights", C.POINTER(rg_light)),
        ("n_textures", C.c_uint32),
        ("textures", C.POINTER(rg_texture)),
    ]


class rg_ray_counts(C.Structure):
    _fields_ = [("primary", C.c_uint64), ("shadow", C.c_uint64), ("secondary", C.c_uint64)]

    def as_dict(self) -> dict:
        return {"primary": int(self.primary), "shadow": int(self.shadow), "secondary": int(self.secondary)}

    def total(self) -> int:
        return int(self.primary) + int(self.shadow) + int(self.secondary)


class rg_stats(C.Structure):
    _fields_ = [
        ("rays", rg_ray_counts),
        ("kernel_ms", C.c_float),
        ("error_pixel", C.c_int32),
        ("_pad", C.c_uint32),
    ]


class rg_tiling(C.Structure):
    _fields_ = [("tile_rows", C.c_uint32), ("tile_stride", C.c_uint32), ("tile_offset", C.c_uint32)]


class rg_bvh_info(C.Structure):  # include/raingun_debug.h
    _fields_ = [("built", C.c_int32), ("enabled", C.c_int32), ("nodes", C.c_int32), ("leaves", C.c_int32),
                ("depth", C.c_int32), ("margin", C.c_float), ("origin_bound", C.c_float), ("lane_stack", C.c_int32),
                ("lbuf_bytes", C.c_int64)]


TILE_CALLBACK = C.CFUNCTYPE(C.c_int32, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint8), C.c_void_p)

# Every symbol include/raingun.h declares (tests/test_abi.py checks the export table).
EXPORTED_SYMBOLS = (
    "rg_abi_version",
    "rg_status_string",
    "rg_device_count",
    "rg_scene_create",
    "rg_scene_destroy",
    "rg_scene_set_max_depth",
    "rg_render_image",
    "rg_render_tiles_async",
    "rg_render_tiles_pipelined",
    "rg_render_tiles",
    "rg_tiling_rows",
    "rg_render_stream",
    "rg_trace",
    "rg_host_register",
    "rg_host_unregister",
    "rg_scene_release_stream",
    "rg_stream_status",
    "rg_render_multi",
)
# include/raingun_debug.h
DEBUG_SYMBOLS = ("rg_debug_set_path", "rg_debug_set_bvh", "rg_debug_bvh_info", "rg_debug_counters",
                 "rg_debug_set_lightbuf", "rg_debug_lightbuf_count",
                 "rg_debug_set_tile_order", "rg_debug_set_lane_depth", "rg_debug_set_image_bands", "rg_debug_set_host_split",
                 "rg_debug_fail_split_a", "rg_debug_set_host_ring", "rg_debug_set_host_tile_shape", "rg_debug_set_multi", "rg_debug_gather_noop",
                 "rg_debug_counter_words")
# include/raingun_frames.h
FRAMES_SYMBOLS = ("rg_frames_create", "rg_frames_destroy", "rg_frames_step", "rg_frames_flush", "rg_frames_image",
                  "rg_frames_read_image", "rg_frames_status", "rg_frames_set_batch", "rg_frames_set_root_tiles", "rg_comm_id_bytes",
                  "rg_comm_unique_id", "rg_comm_init_rank", "rg_comm_info", "rg_comm_destroy", "rg_comm_gather_fn")
PATH_AUTO, PATH_LIGHT, PATH_HEAVY = -1, 0, 1


class RaingunError(RuntimeError):
    """A non-zero rg_status (the reference would have panicked)."""

    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = status_string(status) if _LIB is not None else str(status)
        super().__init__(f"{what}: {msg} (status {status})" if what else f"{msg} (status {status})")


_LIB: C.CDLL | None = None


def _declare(lib: C.CDLL) -> None:
    P = C.POINTER
    lib.rg_abi_version.restype = C.c_int32
    lib.rg_status_string.restype = C.c_char_p
    lib.rg_status_string.argtypes = [C.c_int32]
    lib.rg_device_count.restype = C.c_int32
    lib.rg_scene_create.restype = C.c_int32
    lib.rg_scene_create.argtypes = [P(rg_scene_desc), C.c_int32, P(C.c_void_p)]
    lib.rg_scene_destroy.restype = None
    lib.rg_scene_destroy.argtypes = [C.c_void_p]
    lib.rg_scene_set_max_depth.restype = C.c_int32
    lib.rg_scene_set_max_depth.argtypes = [C.c_void_p, C.c_uint32]
    lib.rg_render_image.restype = C.c_int32
    lib.rg_render_image.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, P(rg_stats)]
    lib.rg_render_tiles_async.restype = C.c_int32
    lib.rg_render_tiles_async.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, P(rg_tiling), C.c_void_p,
                                          C.c_void_p, C.c_void_p, P(rg_stats)]
    if hasattr(lib, "rg_render_tiles_pipelined"):  # absent from pre-round-3 builds (A/B runs against them)
        lib.rg_render_tiles_pipelined.restype = C.c_int32
        lib.rg_render_tiles_pipelined.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, P(rg_tiling), C.c_void_p,
                                                  C.c_void_p, C.c_void_p]
    lib.rg_render_tiles.restype = C.c_int32
    lib.rg_render_tiles.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, P(rg_tiling), C.c_void_p, C.c_void_p,
                                    P(rg_stats)]
    lib.rg_tiling_rows.restype = C.c_uint32
    lib.rg_tiling_rows.argtypes = [C.c_uint32, P(rg_tiling)]
    lib.rg_render_stream.restype = C.c_int32
    lib.rg_render_stream.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, TILE_CALLBACK, C.c_void_p,
                                     P(rg_stats)]
    lib.rg_debug_set_path.restype = C.c_int32
    lib.rg_debug_set_path.argtypes = [C.c_void_p, C.c_int32]
    lib.rg_debug_set_bvh.restype = C.c_int32
    lib.rg_debug_set_bvh.argtypes = [C.c_void_p, C.c_int32]
    if hasattr(lib, "rg_debug_set_lightbuf"):  # absent from older builds A/B runs load (RAINGUN_HIP_LIB)
        lib.rg_debug_set_lightbuf.restype = C.c_int32
        lib.rg_debug_set_lightbuf.argtypes = [C.c_void_p, C.c_int32]
        lib.rg_debug_lightbuf_count.restype = C.c_int32
        lib.rg_debug_lightbuf_count.argtypes = [C.c_void_p]
    lib.rg_debug_bvh_info.restype = C.c_int32
    lib.rg_debug_bvh_info.argtypes = [C.c_void_p, P(rg_bvh_info)]
    lib.rg_debug_set_tile_order.restype = C.c_int32
    lib.rg_debug_set_tile_order.argtypes = [C.c_void_p, C.c_int32]
    lib.rg_debug_set_lane_depth.restype = C.c_int32
    lib.rg_debug_set_lane_depth.argtypes = [C.c_void_p, C.c_int32]
    lib.rg_debug_set_image_bands.restype = C.c_int32
    lib.rg_debug_set_image_bands.argtypes = [C.c_void_p, C.c_int32]
    if hasattr(lib, "rg_debug_set_host_split"):  # absent from pre-round-5 builds A/B runs load (RAINGUN_HIP_LIB)
        lib.rg_debug_set_host_split.restype = C.c_int32
        lib.rg_debug_set_host_split.argtypes = [C.c_void_p, C.c_int32]
    if hasattr(lib, "rg_debug_set_host_ring"):  # absent from pre-round-6 builds
        lib.rg_debug_set_host_ring.restype = C.c_int32
        lib.rg_debug_set_host_ring.argtypes = [C.c_void_p] + [C.c_int32] * 5
    if hasattr(lib, "rg_debug_fail_split_a"):  # absent from pre-round-6 builds
        lib.rg_debug_fail_split_a.restype = C.c_int32
        lib.rg_debug_fail_split_a.argtypes = [C.c_void_p, C.c_int32]
    if hasattr(lib, "rg_debug_set_multi"):  # absent from pre-round-3 builds
        lib.rg_debug_set_multi.restype = C.c_int32
        lib.rg_debug_set_multi.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32]
    if hasattr(lib, "rg_debug_set_host_tile_shape"):  # absent from older builds A/B runs load (RAINGUN_HIP_LIB)
        lib.rg_debug_set_host_tile_shape.restype = C.c_int32
        lib.rg_debug_set_host_tile_shape.argtypes = [C.c_void_p, C.c_int32]
    lib.rg_debug_counters.restype = C.c_int32
    lib.rg_debug_counters.argtypes = [C.c_void_p, P(C.c_uint64)]
    if hasattr(lib, "rg_debug_counter_words"):  # absent from pre-round-6 builds
        lib.rg_debug_counter_words.restype = C.c_int32
        lib.rg_debug_counter_words.argtypes = [C.c_void_p, C.c_int32, C.c_int32, P(C.c_uint64)]
    lib.rg_frames_create.restype = C.c_int32
    lib.rg_frames_create.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int32, C.c_int32,
                                     C.c_int32, C.c_void_p, C.c_void_p, P(C.c_void_p)]
    lib.rg_frames_destroy.restype = None
    lib.rg_frames_destroy.argtypes = [C.c_void_p]
    lib.rg_frames_step.restype = C.c_int32
    lib.rg_frames_step.argtypes = [C.c_void_p]
    lib.rg_frames_flush.restype = C.c_int32
    lib.rg_frames_flush.argtypes = [C.c_void_p]
    lib.rg_frames_image.restype = C.c_void_p
    lib.rg_frames_image.argtypes = [C.c_void_p]
    lib.rg_frames_read_image.restype = C.c_int32
    lib.rg_frames_read_image.argtypes = [C.c_void_p, C.c_void_p]
    lib.rg_trace.restype = C.c_int32
    lib.rg_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
    lib.rg_host_register.restype = C.c_int32
    lib.rg_host_register.argtypes = [C.c_void_p, C.c_size_t]
    lib.rg_host_unregister.restype = C.c_int32
    lib.rg_host_unregister.argtypes = [C.c_void_p]
    lib.rg_scene_release_stream.restype = C.c_int32
    lib.rg_scene_release_stream.argtypes = [C.c_void_p, C.c_void_p]
    lib.rg_stream_status.restype = C.c_int32
    lib.rg_stream_status.argtypes = [C.c_void_p, C.c_void_p, P(C.c_int32)]
    lib.rg_render_multi.restype = C.c_int32
    lib.rg_render_multi.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int32, C.c_uint32, C.c_void_p,
                                    P(rg_stats)]
    lib.rg_frames_status.restype = C.c_int32
    lib.rg_frames_status.argtypes = [C.c_void_p, P(C.c_int32)]
    if hasattr(lib, "rg_frames_set_batch"):  # absent from pre-round-3 builds
        lib.rg_frames_set_batch.restype = C.c_int32
        lib.rg_frames_set_batch.argtypes = [C.c_void_p, C.c_int32]
    if hasattr(lib, "rg_frames_set_root_tiles"):  # absent from pre-round-6 builds
        lib.rg_frames_set_root_tiles.restype = C.c_int32
        lib.rg_frames_set_root_tiles.argtypes = [C.c_void_p, C.c_int32]
    if hasattr(lib, "rg_comm_init_rank"):  # absent from pre-round-4 builds
        lib.rg_comm_id_bytes.restype = C.c_int32
        lib.rg_comm_unique_id.restype = C.c_int32
        lib.rg_comm_unique_id.argtypes = [C.c_void_p]
        lib.rg_comm_init_rank.restype = C.c_int32
        lib.rg_comm_init_rank.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, P(C.c_void_p)]
        lib.rg_comm_info.restype = C.c_int32
        lib.rg_comm_info.argtypes = [C.c_void_p, P(C.c_int32), P(C.c_int32), P(C.c_int32)]
        lib.rg_comm_destroy.restype = C.c_int32
        lib.rg_comm_destroy.argtypes = [C.c_void_p]
        lib.rg_comm_gather_fn.restype = C.c_void_p
        lib.rg_comm_gather_fn.argtypes = []


def lib() -> C.CDLL:
    """Load libraingun_hip.so (built by ``make -C raingun_amd/csrc``).  Raises if absent."""
    global _LIB
    if _LIB is None:
        path = os.environ.get("RAINGUN_HIP_LIB") or str(LIB_PATH)
        if not Path(path).exists():
            raise RuntimeError(
                f"{path} is missing: build it with `make -C raingun_amd/csrc` (or __graft_entry__.build()). "
                "There is no CPU fallback for the render path.")
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64,
        # which satisfies this library's libamdhip64.so.7 dependency when torch
        # is imported first.  Loading /opt/rocm's runtime first would leave two
        # runtimes in the process and torch would then see no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:  # pragma: no cover - torch is part of the image
            pass
        lib_ = C.CDLL(path)
        _declare(lib_)
        _LIB = lib_
    return _LIB


def status_string(status: int) -> str:
    return lib().rg_status_string(int(status)).decode()


def check(status: int, what: str = "") -> None:
    if status != RG_OK:
        raise RaingunError(status, what)


class HostRegistration:
    """Page-lock a numpy array for direct DMA (rg_host_register) while in scope."""

    def __init__(self, arr):
        self.arr = arr
        check(lib().rg_host_register(arr.ctypes.data, arr.nbytes), "rg_host_register")

    def close(self) -> None:
        if self.arr is not None:
            lib().rg_host_unregister(self.arr.ctypes.data)
            self.arr = None

    def __enter__(self):
        return self.arr

    def __exit__(self, *exc):
        self.close()

