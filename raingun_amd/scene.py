"""Host-side mirror of raingun-lib's public API (scene.rs, bodies.rs, lights.rs,
material.rs) above the C ABI of libraingun_hip.so.

* :func:`load_scene` runs the native C++ loader (include/raingun_host.h), which
  reproduces the serde schema of `Scene` (scene.rs:11-31) as serde_yaml 0.6
  over yaml-rust 0.3.5 reads it: camelCase top-level keys with
  `deny_unknown_fields`; externally tagged enums (`Sphere:`/`Plane:`/`Disk:`/
  `AABB:`, `Directional:`/`Spherical:`, `Color:`/`Texture:`, `Diffuse` /
  `{Diffuse: null}` / `{Reflecting: {...}}` / `{Refractive: {...}}`); Point3 and
  Vector3 as `[x, y, z]` or `{x:, y:, z:}` (cgmath "eders"); f32 fields rounded
  to f32; textures decoded eagerly at load time relative to the working
  directory (material.rs:34-47) by the native decoder (libraingun_host.so),
  which rounds like the reference's jpeg-decoder 0.1.11.  This module only
  converts the loaded rg_scene_desc into the dataclasses below.
* :class:`Scene` keeps the reference's `render_image(width, height)` /
  `streaming_render(...)` / `trace(ray)` entry points (scene.rs:34-51); every
  one of them runs on the GPU through the C ABI.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Callable, List, Optional, Sequence, Union

import numpy as np

from . import _abi
from .color import Color



class SceneError(ValueError):
    """The YAML does not deserialise into a Scene (serde_yaml's Err)."""


# ---------------------------------------------------------------- data model
@dataclass
class Texture:                 # material.rs:26-32
    path: str
    image: np.ndarray          # (h, w, 4) uint8 RGBA
    x_offset: float
    y_offset: float


@dataclass
class Material:                # material.rs:7-12
    coloration: Union[Color, Texture]
    albedo: float
    surface: str = "Diffuse"   # Diffuse | Reflecting | Refractive
    reflectivity: float = 0.0
    index: float = 0.0
    transparency: float = 0.0


@dataclass
class Sphere:                  # bodies.rs:13-18
    center: tuple
    radius: float
    material: Material


@dataclass
class Plane:                   # bodies.rs:20-25
    origin: tuple
    normal: tuple
    material: Material


@dataclass
class Disk:                    # bodies.rs:27-33
    origin: tuple
    normal: tuple
    radius: float
    material: Material


@dataclass
class AABB:                    # bodies.rs:35-39
    bounds: tuple              # ((x0,y0,z0), (x1,y1,z1))
    material: Material


@dataclass
class DirectionalLight:        # lights.rs:8-13
    direction: tuple
    color: Color
    intensity: float


@dataclass
class SphericalLight:          # lights.rs:15-20
    position: tuple
    color: Color
    intensity: float


Body = Union[Sphere, Plane, Disk, AABB]
Light = Union[DirectionalLight, SphericalLight]


# ---------------------------------------------------------------- loading
def load_scene(source: Union[str, os.PathLike], texture_root: Optional[Union[str, os.PathLike]] = None) -> "Scene":
    """serde_yaml::from_reader::<Scene> (main.rs:116-118) through the native
    loader (rgh_scene_load_*, raingun_amd/host/scene_loader.cpp).  `source` is
    a path or YAML text.  Texture paths resolve against `texture_root`
    (default: the current working directory, as image::open does)."""
    from . import _host

    try:
        if isinstance(source, os.PathLike) or (isinstance(source, str) and "\n" not in source
                                               and Path(source).exists()):
            loaded = _host.LoadedScene.from_file(source, texture_root)
        else:
            loaded = _host.LoadedScene.from_string(str(source), texture_root)
    except _host.HostError as e:
        raise SceneError(str(e)) from None
    try:
        return _scene_from_desc(loaded)
    finally:
        loaded.close()


_SURFACES = {_abi.SURFACE_DIFFUSE: "Diffuse", _abi.SURFACE_REFLECTING: "Reflecting",
             _abi.SURFACE_REFRACTIVE: "Refractive"}


def _scene_from_desc(loaded) -> "Scene":
    d = loaded.desc
    textures = []
    for i in range(d.n_textures):
        t = d.textures[i]
        img = np.ctypeslib.as_array(t.rgba, shape=(t.height * t.width * 4,)).copy().reshape(t.height, t.width, 4)
        textures.append((loaded.texture_path(i), img))

    def material(m) -> Material:
        if m.coloration == _abi.COLORATION_TEXTURE:
            path, img = textures[m.texture]
            col: Union[Color, Texture] = Texture(path, img, m.x_offset, m.y_offset)
        else:
            col = Color(*m.color)
        return Material(col, m.albedo, _SURFACES[m.surface], m.reflectivity, m.index, m.transparency)

    bodies: List[Body] = []
    for i in range(d.n_bodies):
        b = d.bodies[i]
        p = tuple(b.p)
        mat = material(b.material)
        if b.kind == _abi.BODY_SPHERE:
            bodies.append(Sphere(p[0:3], p[3], mat))
        elif b.kind == _abi.BODY_PLANE:
            bodies.append(Plane(p[0:3], p[3:6], mat))
        elif b.kind == _abi.BODY_DISK:
            bodies.append(Disk(p[0:3], p[3:6], p[6], mat))
        else:
            bodies.append(AABB((p[0:3], p[3:6]), mat))
    lights: List[Light] = []
    for i in range(d.n_lights):
        l = d.lights[i]
        cls = DirectionalLight if l.kind == _abi.LIGHT_DIRECTIONAL else SphericalLight
        lights.append(cls(tuple(l.v), Color(*l.color), l.intensity))
    return Scene(d.fov, Color(*d.default_color), d.max_recursion_depth, bodies, lights)


# ---------------------------------------------------------------- flat descriptor
class SceneDesc:
    """Owns the ctypes arrays behind an rg_scene_desc (pass `.desc` to the ABI)."""

    def __init__(self, scene: "Scene"):
        nb, nl = len(scene.bodies), len(scene.lights)
        self.bodies = (_abi.rg_body * max(nb, 1))()
        self.lights = (_abi.rg_light * max(nl, 1))()
        tex_index: dict = {}
        self._images: List[np.ndarray] = []
        for i, b in enumerate(scene.bodies):
            rb = self.bodies[i]
            if isinstance(b, Sphere):
                rb.kind, p = _abi.BODY_SPHERE, [*b.center, b.radius]
            elif isinstance(b, Plane):
                rb.kind, p = _abi.BODY_PLANE, [*b.origin, *b.normal]
            elif isinstance(b, Disk):
                rb.kind, p = _abi.BODY_DISK, [*b.origin, *b.normal, b.radius]
            elif isinstance(b, AABB):
                rb.kind, p = _abi.BODY_AABB, [*b.bounds[0], *b.bounds[1]]
            else:
                raise TypeError(f"not a body: {b!r}")
            for k, v in enumerate(p):
                rb.p[k] = v
            m = b.material
            rm = rb.material
            if isinstance(m.coloration, Texture):
                key = id(m.coloration.image)
                if key not in tex_index:
                    tex_index[key] = len(self._images)
                    self._images.append(np.ascontiguousarray(m.coloration.image, dtype=np.uint8))
                rm.coloration = _abi.COLORATION_TEXTURE
                rm.texture = tex_index[key]
                rm.x_offset = m.coloration.x_offset
                rm.y_offset = m.coloration.y_offset
            else:
                rm.coloration = _abi.COLORATION_COLOR
                rm.color[:] = [float(m.coloration.red), float(m.coloration.green), float(m.coloration.blue)]
                rm.texture = -1
            rm.albedo = m.albedo
            rm.surface = {"Diffuse": _abi.SURFACE_DIFFUSE, "Reflecting": _abi.SURFACE_REFLECTING,
                          "Refractive": _abi.SURFACE_REFRACTIVE}[m.surface]
            rm.reflectivity = m.reflectivity
            rm.index = m.index
            rm.transparency = m.transparency
        for i, l in enumerate(scene.lights):
            rl = self.lights[i]
            if isinstance(l, DirectionalLight):
                rl.kind, v = _abi.LIGHT_DIRECTIONAL, l.direction
            else:
                rl.kind, v = _abi.LIGHT_SPHERICAL, l.position
            rl.v[:] = list(v)
            rl.color[:] = [float(l.color.red), float(l.color.green), float(l.color.blue)]
            rl.intensity = l.intensity
        self.textures = (_abi.rg_texture * max(len(self._images), 1))()
        for i, im in enumerate(self._images):
            self.textures[i].height, self.textures[i].width = im.shape[0], im.shape[1]
            self.textures[i].rgba = im.ctypes.data_as(C.POINTER(C.c_uint8))
        d = _abi.rg_scene_desc()
        d.fov = scene.fov
        d.default_color[:] = [float(scene.default_color.red), float(scene.default_color.green),
                              float(scene.default_color.blue)]
        d.max_recursion_depth = scene.max_recursion_depth
        d.n_bodies, d.bodies = nb, C.cast(self.bodies, C.POINTER(_abi.rg_body))
        d.n_lights, d.lights = nl, C.cast(self.lights, C.POINTER(_abi.rg_light))
        d.n_textures, d.textures = len(self._images), C.cast(self.textures, C.POINTER(_abi.rg_texture))
        self.desc = d

    def ptr(self):
        return C.byref(self.desc)


# ---------------------------------------------------------------- device scene
class DeviceScene:
    """An rg_scene handle: the scene uploaded to one GPU."""

    def __init__(self, scene: "Scene", device: int = 0, path: Optional[int] = None, bvh: Optional[bool] = None):
        self._desc = SceneDesc(scene)
        h = C.c_void_p()
        _abi.check(_abi.lib().rg_scene_create(self._desc.ptr(), int(device), C.byref(h)), "rg_scene_create")
        self.handle = h
        self.device = device
        if path is not None:
            self.set_path(path)
        if bvh is not None:
            self.set_bvh(bvh)

    def close(self) -> None:
        if getattr(self, "handle", None):
            _abi.lib().rg_scene_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_path(self, path: int) -> None:
        """Force a kernel path (_abi.PATH_AUTO / PATH_LIGHT / PATH_HEAVY; include/raingun_debug.h)."""
        _abi.check(_abi.lib().rg_debug_set_path(self.handle, int(path)))

    def set_bvh(self, enable: bool) -> None:
        """Use (default) or bypass the sphere BVH (include/raingun_debug.h)."""
        _abi.check(_abi.lib().rg_debug_set_bvh(self.handle, 1 if enable else 0))

    def set_lightbuf(self, enable: bool) -> None:
        """Shadow rays test their light buffer cell's spheres (default) or walk the BVH (include/raingun_debug.h)."""
        _abi.check(_abi.lib().rg_debug_set_lightbuf(self.handle, 1 if enable else 0))

    def lightbuf_count(self) -> int:
        """Lights with a shadow-ray light buffer in use (include/raingun_debug.h)."""
        return int(_abi.lib().rg_debug_lightbuf_count(self.handle))

    def set_tile_order(self, mode) -> None:
        """Tile scheduling: True/1 probe-ordered, False/0 raster, -1 auto (include/raingun_debug.h)."""
        _abi.check(_abi.lib().rg_debug_set_tile_order(self.handle, int(mode)))

    def set_lane_depth(self, min_depth: int) -> None:
        """Rays at recursion depth >= min_depth walk the BVH per lane (0: all
        non-primary rays, large: none, -1: default) (include/raingun_debug.h)."""
        _abi.check(_abi.lib().rg_debug_set_lane_depth(self.handle, int(min_depth)))

    def set_image_bands(self, bands: int) -> None:
        """Row bands of host-visible renders (0: by frame size; include/raingun_debug.h)."""
        _abi.check(_abi.lib().rg_debug_set_image_bands(self.handle, int(bands)))

    def set_multi(self, mode: int = 0, stand_in: bool = False, bands: int = 0, only_rank: int = -1) -> None:
        """rg_render_multi delivery (raingun_debug.h): 0 per-device copies to the host, 1 RCCL gather;
        stand_in: every device is this one (ngpus > 1 on one GPU); only_rank: rehearse one device's work."""
        _abi.check(_abi.lib().rg_debug_set_multi(self.handle, int(mode), 1 if stand_in else 0, int(bands),
                                                 int(only_rank)))

    def set_host_ring(self, flush_small: int = -1, group_small: int = -1, flush_big: int = -1, group_big: int = -1,
                      multi_light_one: int = -1) -> None:
        """Light-path host frames: LDS-ring flush size and queue group of small / big launches,
        rg_render_multi's one launch per device for light scenes; -1 keeps a setting
        (include/raingun_debug.h rg_debug_set_host_ring)."""
        _abi.check(_abi.lib().rg_debug_set_host_ring(self.handle, int(flush_small), int(group_small), int(flush_big),
                                                     int(group_big), int(multi_light_one)))

    def set_host_split(self, pct: int) -> None:
        """Image bands -2 (split host frames): percent of the rows rendered into device
        memory and copied by DMA beside the one-launch rest; 0 = default (raingun_debug.h)."""
        _abi.check(_abi.lib().rg_debug_set_host_split(self.handle, int(pct)))

    def set_host_tile_shape(self, tile_wlog: int) -> None:
        """Tile shape of one-launch host-visible renders: log2 of the tile width, 3 (8x8) .. 6 (64x1);
        0 = automatic (16x4 for heavy-path scenes, 64x1 for light-path scenes)."""
        _abi.check(_abi.lib().rg_debug_set_host_tile_shape(self.handle, int(tile_wlog)))

    def bvh_info(self) -> _abi.rg_bvh_info:
        info = _abi.rg_bvh_info()
        _abi.check(_abi.lib().rg_debug_bvh_info(self.handle, C.byref(info)))
        return info

    def set_max_depth(self, depth: int) -> None:
        _abi.check(_abi.lib().rg_scene_set_max_depth(self.handle, int(depth)))

    def render_image(self, width: int, height: int, stats: Optional[_abi.rg_stats] = None,
                     out: Optional[np.ndarray] = None) -> np.ndarray:
        """rendering::render_image (rendering.rs:24-38) into host memory.  `out`
        (optional, (height, width, 4) uint8, C-contiguous) may be a buffer
        registered with register_host() for direct DMA."""
        if out is None:
            out = np.empty((height, width, 4), dtype=np.uint8)
        assert out.shape == (height, width, 4) and out.dtype == np.uint8 and out.flags.c_contiguous
        st = stats if stats is not None else _abi.rg_stats()
        _abi.check(_abi.lib().rg_render_image(self.handle, width, height, out.ctypes.data, C.byref(st)),
                   "rg_render_image")
        return out

    def render_multi(self, width: int, height: int, ngpus: int, tile_rows: int = 0,
                     stats: Optional[_abi.rg_stats] = None, out: Optional[np.ndarray] = None) -> np.ndarray:
        """rg_render_multi: the frame over `ngpus` devices of this process (row
        tiles, one RCCL gather to this scene's device), delivered to host memory."""
        if out is None:
            out = np.empty((height, width, 4), dtype=np.uint8)
        st = stats if stats is not None else _abi.rg_stats()
        _abi.check(_abi.lib().rg_render_multi(self.handle, width, height, int(ngpus), int(tile_rows),
                                              out.ctypes.data, C.byref(st)), "rg_render_multi")
        return out

    def render_stream(self, width: int, height: int, on_tile, tile_rows: int = 16,
                      stats: Optional[_abi.rg_stats] = None) -> int:
        """rg_render_stream: on_tile(row0, band) gets each band of finished RGBA8
        rows (a copy); return True to cancel.  Returns the rg_status."""
        st = stats if stats is not None else _abi.rg_stats()

        def cb(row0, rows, w, ptr, _user):
            band = np.ctypeslib.as_array(ptr, shape=(rows * w * 4,)).reshape(rows, w, 4).copy()
            return 1 if on_tile(int(row0), band) else 0

        fn = _abi.TILE_CALLBACK(cb)
        return _abi.lib().rg_render_stream(self.handle, width, height, tile_rows, fn, None, C.byref(st))

    def stream_status(self, stream: int):
        """(status, error_pixel) of the launches on `stream` (a hipStream_t value) since the last call."""
        px = C.c_int32(-1)
        st = _abi.lib().rg_stream_status(self.handle, C.c_void_p(stream), C.byref(px))
        return st, px.value

    def release_stream(self, stream: int) -> None:
        _abi.check(_abi.lib().rg_scene_release_stream(self.handle, C.c_void_p(stream)), "rg_scene_release_stream")

    def render_tiles(self, width: int, height: int, tile_rows: int = 0, stride: int = 1, offset: int = 0,
                     want_rgb: bool = False, stats: Optional[_abi.rg_stats] = None):
        t = _abi.rg_tiling(tile_rows or height, stride, offset)
        rows = _abi.lib().rg_tiling_rows(height, C.byref(t))
        rgba = np.empty((rows, width, 4), dtype=np.uint8)
        rgb = np.empty((rows, width, 3), dtype=np.float32) if want_rgb else None
        st = stats if stats is not None else _abi.rg_stats()
        status = _abi.lib().rg_render_tiles(self.handle, width, height, C.byref(t), rgba.ctypes.data,
                                            rgb.ctypes.data if rgb is not None else None, C.byref(st))
        _abi.check(status, "rg_render_tiles")
        return (rgba, rgb) if want_rgb else rgba

    def trace(self, rays: np.ndarray):
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        n = rays.shape[0]
        dist = np.empty(n, dtype=np.float64)
        body = np.empty(n, dtype=np.int32)
        _abi.check(_abi.lib().rg_trace(self.handle, rays.ctypes.data, n, dist.ctypes.data, body.ctypes.data),
                   "rg_trace")
        return dist, body


# ---------------------------------------------------------------- Scene
@dataclass
class Scene:                   # scene.rs:11-31
    fov: float = 90.0
    default_color: Color = field(default_factory=Color.black)
    max_recursion_depth: int = 10
    bodies: List[Body] = field(default_factory=list)
    lights: List[Light] = field(default_factory=list)

    from_yaml = staticmethod(load_scene)

    def to_device(self, device: int = 0) -> DeviceScene:
        return DeviceScene(self, device)

    # scene.rs:41-43 -> rendering::render_image (rendering.rs:24-38), on the GPU
    def render_image(self, width: int, height: int, device: int = 0) -> np.ndarray:
        ds = DeviceScene(self, device)
        try:
            return ds.render_image(width, height)
        finally:
            ds.close()

    # scene.rs:45-51 -> rendering::render_image_stream (rendering.rs:40-69).  The
    # reference sends one RenderedPixel per pixel; here the callback receives
    # bands of `tile_rows` finished RGBA8 rows.  Return True from it to cancel.
    def streaming_render(self, width: int, height: int,
                         on_tile: Callable[[int, np.ndarray], Optional[bool]],
                         tile_rows: int = 16, device: int = 0) -> _abi.rg_stats:
        ds = DeviceScene(self, device)
        stats = _abi.rg_stats()
        try:
            _abi.check(ds.render_stream(width, height, on_tile, tile_rows, stats), "rg_render_stream")
        finally:
            ds.close()
        return stats

    # scene.rs:34-39
    def trace(self, origin: Sequence[float], direction: Sequence[float], device: int = 0):
        ds = DeviceScene(self, device)
        try:
            dist, body = ds.trace(np.array([*origin, *direction], dtype=np.float64))
        finally:
            ds.close()
        if body[0] < 0:
            return None
        return float(dist[0]), int(body[0])
