"""ctypes binding of include/raingun_host.h (libraingun_host.so): the native
host layer — YAML scene loading, JPEG/PNG decoding and PNG writing.

Like the renderer, this library is required: :func:`lib` builds it in-tree
if it is missing (g++ only, seconds) and raises if it cannot be loaded.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading
from pathlib import Path
from typing import Optional, Tuple

import numpy as np

from . import _abi

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "libraingun_host.so"
SRC_DIR = PKG_DIR / "host"
CLI_PATH = PKG_DIR / "bin" / "raingun"

RGH_OK = 0
RGH_ERR_INVALID_ARGUMENT = -1
RGH_ERR_OUT_OF_MEMORY = -11
RGH_ERR_IO = -20
RGH_ERR_YAML = -21
RGH_ERR_SCHEMA = -22
RGH_ERR_IMAGE = -23

JPEG_REFERENCE, JPEG_LIBJPEG = 0, 1

EXPORTED_SYMBOLS = (
    "rgh_abi_version",
    "rgh_last_error",
    "rgh_scene_load_file",
    "rgh_scene_load_string",
    "rgh_scene_desc",
    "rgh_scene_texture_path",
    "rgh_scene_clamp_depth",
    "rgh_scene_free",
    "rgh_image_decode",
    "rgh_image_decode_file",
    "rgh_png_encode",
    "rgh_png_write",
    "rgh_free",
)


class HostError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(message)
        self.status = status


_lib = None
_lock = threading.Lock()


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(SRC_DIR), "lib"], check=True)


def lib() -> C.CDLL:
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = Path(os.environ.get("RAINGUN_HOST_LIB", LIB_PATH))
        if not path.exists() and path == LIB_PATH:
            build()
        l = C.CDLL(str(path))
        u8p = C.POINTER(C.c_uint8)
        l.rgh_abi_version.restype = C.c_int32
        l.rgh_last_error.restype = C.c_char_p
        l.rgh_scene_load_file.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_void_p)]
        l.rgh_scene_load_string.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.POINTER(C.c_void_p)]
        l.rgh_scene_desc.argtypes = [C.c_void_p]
        l.rgh_scene_desc.restype = C.POINTER(_abi.rg_scene_desc)
        l.rgh_scene_texture_path.argtypes = [C.c_void_p, C.c_uint32]
        l.rgh_scene_texture_path.restype = C.c_char_p
        l.rgh_scene_clamp_depth.argtypes = [C.c_void_p, C.c_uint32]
        l.rgh_scene_free.argtypes = [C.c_void_p]
        l.rgh_image_decode.argtypes = [C.c_void_p, C.c_size_t, C.c_int32, C.POINTER(C.c_uint32),
                                       C.POINTER(C.c_uint32), C.POINTER(u8p)]
        l.rgh_image_decode_file.argtypes = [C.c_char_p, C.c_int32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                            C.POINTER(u8p)]
        l.rgh_png_encode.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(u8p), C.POINTER(C.c_size_t)]
        l.rgh_png_write.argtypes = [C.c_char_p, C.c_void_p, C.c_uint32, C.c_uint32]
        l.rgh_free.argtypes = [C.c_void_p]
        if l.rgh_abi_version() != 1:
            raise RuntimeError(f"{path}: unexpected host ABI version {l.rgh_abi_version()}")
        _lib = l
        return l


def _check(status: int) -> None:
    if status != RGH_OK:
        raise HostError(status, lib().rgh_last_error().decode("utf-8", "replace"))


def _take_image(w: C.c_uint32, h: C.c_uint32, p) -> np.ndarray:
    try:
        n = w.value * h.value * 4
        return np.ctypeslib.as_array(p, shape=(n,)).copy().reshape(h.value, w.value, 4)
    finally:
        lib().rgh_free(p)


def decode_image_file(path, flavor: int = JPEG_REFERENCE) -> np.ndarray:
    """image::open(path) -> (h, w, 4) uint8 RGBA (material.rs:34-47)."""
    w, h, p = C.c_uint32(), C.c_uint32(), C.POINTER(C.c_uint8)()
    _check(lib().rgh_image_decode_file(os.fsencode(str(path)), flavor, C.byref(w), C.byref(h), C.byref(p)))
    return _take_image(w, h, p)


def decode_image(data: bytes, flavor: int = JPEG_REFERENCE) -> np.ndarray:
    w, h, p = C.c_uint32(), C.c_uint32(), C.POINTER(C.c_uint8)()
    buf = C.create_string_buffer(data, len(data))
    _check(lib().rgh_image_decode(buf, len(data), flavor, C.byref(w), C.byref(h), C.byref(p)))
    return _take_image(w, h, p)


def encode_png(rgba: np.ndarray) -> bytes:
    rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
    h, w, c = rgba.shape
    if c != 4:
        raise ValueError("expected (h, w, 4) RGBA8")
    p, n = C.POINTER(C.c_uint8)(), C.c_size_t()
    _check(lib().rgh_png_encode(rgba.ctypes.data, w, h, C.byref(p), C.byref(n)))
    try:
        return C.string_at(p, n.value)
    finally:
        lib().rgh_free(p)


class LoadedScene:
    """A scene loaded by the native loader (rgh_scene_load_*): owns the
    rg_scene_desc that rg_scene_create consumes."""

    def __init__(self, handle: C.c_void_p):
        self.handle = handle

    @classmethod
    def from_file(cls, path, texture_root=None) -> "LoadedScene":
        h = C.c_void_p()
        root = os.fsencode(str(texture_root)) if texture_root is not None else None
        _check(lib().rgh_scene_load_file(os.fsencode(str(path)), root, C.byref(h)))
        return cls(h)

    @classmethod
    def from_string(cls, text: str, texture_root=None) -> "LoadedScene":
        h = C.c_void_p()
        b = text.encode("utf-8")
        root = os.fsencode(str(texture_root)) if texture_root is not None else None
        _check(lib().rgh_scene_load_string(b, len(b), root, C.byref(h)))
        return cls(h)

    @property
    def desc(self) -> _abi.rg_scene_desc:
        return lib().rgh_scene_desc(self.handle).contents

    def ptr(self):
        return lib().rgh_scene_desc(self.handle)

    def texture_path(self, index: int) -> str:
        p = lib().rgh_scene_texture_path(self.handle, int(index))
        if p is None:
            raise IndexError(index)
        return p.decode("utf-8")

    def clamp_depth(self, limit: int) -> None:
        lib().rgh_scene_clamp_depth(self.handle, int(limit))

    def close(self) -> None:
        if self.handle:
            lib().rgh_scene_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def desc_tuple(d: _abi.rg_scene_desc) -> Tuple:
    """A comparable, hashable snapshot of an rg_scene_desc (textures by content digest)."""
    import hashlib

    def mat(m):
        return (m.coloration, tuple(m.color), m.texture, m.x_offset, m.y_offset, m.albedo, m.surface,
                m.reflectivity, m.index, m.transparency)

    bodies = tuple((d.bodies[i].kind, tuple(d.bodies[i].p), mat(d.bodies[i].material)) for i in range(d.n_bodies))
    lights = tuple((d.lights[i].kind, tuple(d.lights[i].color), d.lights[i].intensity, tuple(d.lights[i].v))
                   for i in range(d.n_lights))
    texs = []
    for i in range(d.n_textures):
        t = d.textures[i]
        data = C.string_at(t.rgba, t.width * t.height * 4)
        texs.append((t.width, t.height, hashlib.sha256(data).hexdigest()))
    return (d.fov, tuple(d.default_color), d.max_recursion_depth, bodies, lights, tuple(texs))
