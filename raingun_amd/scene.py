"""Host-side mirror of raingun-lib's public API (scene.rs, bodies.rs, lights.rs,
material.rs) above the C ABI of libraingun_hip.so.

* :func:`load_scene` reproduces the serde schema of `Scene` (scene.rs:11-31)
  as serde_yaml 0.6 reads it: camelCase top-level keys with
  `deny_unknown_fields`; externally tagged enums (`Sphere:`/`Plane:`/`Disk:`/
  `AABB:`, `Directional:`/`Spherical:`, `Color:`/`Texture:`, `Diffuse` /
  `{Diffuse: null}` / `{Reflecting: {...}}` / `{Refractive: {...}}`); Point3 and
  Vector3 as `[x, y, z]` or `{x:, y:, z:}` (cgmath "eders"); f32 fields rounded
  to f32; textures decoded eagerly at load time relative to the working
  directory (material.rs:34-47).
* :class:`Scene` keeps the reference's `render_image(width, height)` /
  `streaming_render(...)` / `trace(ray)` entry points (scene.rs:34-51); every
  one of them runs on the GPU through the C ABI.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Callable, List, Optional, Sequence, Union

import numpy as np

from . import _abi
from .color import Color

F32 = np.float32


class SceneError(ValueError):
    """The YAML does not deserialise into a Scene (serde_yaml's Err)."""


# ---------------------------------------------------------------- data model
@dataclass
class Texture:                 # material.rs:85-91
    path: str
    image: np.ndarray          # (h, w, 4) uint8 RGBA
    x_offset: float
    y_offset: float


@dataclass
class Material:                # material.rs:66-71
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


# ---------------------------------------------------------------- YAML schema
def _f64(v, what: str) -> float:
    if isinstance(v, bool) or v is None:
        raise SceneError(f"{what}: expected a number, got {v!r}")
    if isinstance(v, (int, float)):
        return float(v)
    if isinstance(v, str):  # PyYAML (YAML 1.1) leaves e.g. "1e-13" as a string; yaml-rust parses it
        try:
            return float(v.strip())
        except ValueError:
            pass
    raise SceneError(f"{what}: expected a number, got {v!r}")


def _f32(v, what: str) -> float:
    return float(F32(_f64(v, what)))


def _u32(v, what: str) -> int:
    if isinstance(v, bool) or not isinstance(v, int) or v < 0 or v > 0xFFFFFFFF:
        raise SceneError(f"{what}: expected a u32, got {v!r}")
    return int(v)


def _vec3(v, what: str) -> tuple:
    if isinstance(v, (list, tuple)):
        if len(v) != 3:
            raise SceneError(f"{what}: expected 3 components, got {len(v)}")
        return tuple(_f64(c, what) for c in v)
    if isinstance(v, dict):
        try:
            return (_f64(v["x"], what), _f64(v["y"], what), _f64(v["z"], what))
        except KeyError as e:
            raise SceneError(f"{what}: missing field {e.args[0]}") from None
    raise SceneError(f"{what}: expected a point/vector, got {v!r}")


def _color(v, what: str) -> Color:
    if not isinstance(v, str):
        raise SceneError(f"{what}: a string of a simple hex color (#000000 - #ffffff), got {v!r}")
    try:
        return Color.from_str(v)
    except ValueError as e:
        raise SceneError(f"{what}: {e}") from None


def _variant(v, what: str):
    """Externally tagged enum: 'Name' (unit variant) or {Name: content}."""
    if isinstance(v, str):
        return v, None
    if isinstance(v, dict) and len(v) == 1:
        (k, val), = v.items()
        return k, val
    raise SceneError(f"{what}: expected an enum variant, got {v!r}")


def _req(d, key: str, what: str):
    if not isinstance(d, dict):
        raise SceneError(f"{what}: expected a mapping, got {d!r}")
    if key not in d:
        raise SceneError(f"{what}: missing field `{key}`")
    return d[key]


def _load_image(path: str, base: Path) -> np.ndarray:
    p = Path(path)
    if not p.is_absolute():
        p = base / p
    try:
        from PIL import Image  # decoder used by the host loader only (image::open, material.rs:42)
        with Image.open(p) as im:
            return np.ascontiguousarray(np.asarray(im.convert("RGBA"), dtype=np.uint8))
    except Exception as e:  # serde Error::custom (material.rs:43-46)
        raise SceneError(f"Could not load texture file {path}: {e}") from None


def _material(v, what: str, base: Path, cache: dict) -> Material:
    kind, col = _variant(_req(v, "coloration", what), what + ".coloration")
    if kind == "Color":
        coloration = _color(col, what + ".coloration.Color")
    elif kind == "Texture":
        tw = what + ".coloration.Texture"
        img_path = _req(col, "image", tw)
        if not isinstance(img_path, str):
            raise SceneError(f"{tw}.image: expected a path string")
        if img_path not in cache:
            cache[img_path] = _load_image(img_path, base)
        coloration = Texture(img_path, cache[img_path], _f32(_req(col, "x_offset", tw), tw + ".x_offset"),
                             _f32(_req(col, "y_offset", tw), tw + ".y_offset"))
    else:
        raise SceneError(f"{what}.coloration: unknown variant `{kind}`, expected `Color` or `Texture`")
    albedo = _f32(_req(v, "albedo", what), what + ".albedo")
    skind, sval = _variant(_req(v, "surface", what), what + ".surface")
    m = Material(coloration, albedo, skind)
    if skind == "Diffuse":
        if sval is not None:
            raise SceneError(f"{what}.surface: Diffuse takes no fields")
    elif skind == "Reflecting":
        m.reflectivity = _f32(_req(sval, "reflectivity", what + ".surface"), what + ".reflectivity")
    elif skind == "Refractive":
        m.index = _f32(_req(sval, "index", what + ".surface"), what + ".index")
        m.transparency = _f32(_req(sval, "transparency", what + ".surface"), what + ".transparency")
    else:
        raise SceneError(f"{what}.surface: unknown variant `{skind}`")
    return m


def _body(v, i: int, base: Path, cache: dict) -> Body:
    what = f"bodies[{i}]"
    kind, b = _variant(v, what)
    w = f"{what}.{kind}"
    if kind == "Sphere":
        return Sphere(_vec3(_req(b, "center", w), w + ".center"), _f64(_req(b, "radius", w), w + ".radius"),
                      _material(_req(b, "material", w), w + ".material", base, cache))
    if kind == "Plane":
        return Plane(_vec3(_req(b, "origin", w), w + ".origin"), _vec3(_req(b, "normal", w), w + ".normal"),
                     _material(_req(b, "material", w), w + ".material", base, cache))
    if kind == "Disk":
        return Disk(_vec3(_req(b, "origin", w), w + ".origin"), _vec3(_req(b, "normal", w), w + ".normal"),
                    _f64(_req(b, "radius", w), w + ".radius"),
                    _material(_req(b, "material", w), w + ".material", base, cache))
    if kind == "AABB":
        bounds = _req(b, "bounds", w)
        if not isinstance(bounds, (list, tuple)) or len(bounds) != 2:
            raise SceneError(f"{w}.bounds: expected two points")
        return AABB((_vec3(bounds[0], w + ".bounds[0]"), _vec3(bounds[1], w + ".bounds[1]")),
                    _material(_req(b, "material", w), w + ".material", base, cache))
    raise SceneError(f"{what}: unknown variant `{kind}`, expected one of `Sphere`, `Plane`, `Disk`, `AABB`")


def _light(v, i: int) -> Light:
    what = f"lights[{i}]"
    kind, l = _variant(v, what)
    w = f"{what}.{kind}"
    if kind == "Directional":
        return DirectionalLight(_vec3(_req(l, "direction", w), w + ".direction"),
                                _color(_req(l, "color", w), w + ".color"),
                                _f32(_req(l, "intensity", w), w + ".intensity"))
    if kind == "Spherical":
        return SphericalLight(_vec3(_req(l, "position", w), w + ".position"),
                              _color(_req(l, "color", w), w + ".color"),
                              _f32(_req(l, "intensity", w), w + ".intensity"))
    raise SceneError(f"{what}: unknown variant `{kind}`, expected `Directional` or `Spherical`")


_SCENE_KEYS = ("fov", "defaultColor", "maxRecursionDepth", "bodies", "lights")


def load_scene(source: Union[str, os.PathLike], texture_root: Optional[Union[str, os.PathLike]] = None) -> "Scene":
    """serde_yaml::from_reader::<Scene> (main.rs:116-118).  `source` is a path or
    YAML text.  Texture paths resolve against `texture_root` (default: the
    current working directory, as image::open does)."""
    import yaml

    text = None
    if isinstance(source, os.PathLike) or (isinstance(source, str) and "\n" not in source and Path(source).exists()):
        text = Path(source).read_text()
    else:
        text = str(source)
    try:
        doc = yaml.safe_load(text)
    except yaml.YAMLError as e:
        raise SceneError(f"Could not load YAML: {e}") from None
    if doc is None:
        doc = {}
    if not isinstance(doc, dict):
        raise SceneError("invalid type: expected struct Scene")
    for k in doc:
        if k not in _SCENE_KEYS:  # deny_unknown_fields (scene.rs:12)
            raise SceneError(f"unknown field `{k}`, expected one of {', '.join('`%s`' % s for s in _SCENE_KEYS)}")
    base = Path(texture_root) if texture_root is not None else Path.cwd()
    cache: dict = {}
    s = Scene()
    if "fov" in doc:
        s.fov = _f64(doc["fov"], "fov")
    if "defaultColor" in doc:
        s.default_color = _color(doc["defaultColor"], "defaultColor")
    if "maxRecursionDepth" in doc:
        s.max_recursion_depth = _u32(doc["maxRecursionDepth"], "maxRecursionDepth")
    bodies = doc.get("bodies", []) or []
    lights = doc.get("lights", []) or []
    if not isinstance(bodies, list) or not isinstance(lights, list):
        raise SceneError("bodies/lights: expected a sequence")
    s.bodies = [_body(b, i, base, cache) for i, b in enumerate(bodies)]
    s.lights = [_light(l, i) for i, l in enumerate(lights)]
    return s


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

    def __init__(self, scene: "Scene", device: int = 0, path: Optional[int] = None):
        self._desc = SceneDesc(scene)
        h = C.c_void_p()
        _abi.check(_abi.lib().rg_scene_create(self._desc.ptr(), int(device), C.byref(h)), "rg_scene_create")
        self.handle = h
        self.device = device
        if path is not None:
            self.set_path(path)

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

    def set_max_depth(self, depth: int) -> None:
        _abi.check(_abi.lib().rg_scene_set_max_depth(self.handle, int(depth)))

    def render_image(self, width: int, height: int, stats: Optional[_abi.rg_stats] = None) -> np.ndarray:
        out = np.empty((height, width, 4), dtype=np.uint8)
        st = stats if stats is not None else _abi.rg_stats()
        _abi.check(_abi.lib().rg_render_image(self.handle, width, height, out.ctypes.data, C.byref(st)),
                   "rg_render_image")
        return out

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

        def cb(row0, rows, w, ptr, _user):
            band = np.ctypeslib.as_array(ptr, shape=(rows * w * 4,)).reshape(rows, w, 4).copy()
            return 1 if on_tile(int(row0), band) else 0

        fn = _abi.TILE_CALLBACK(cb)
        try:
            _abi.check(_abi.lib().rg_render_stream(ds.handle, width, height, tile_rows, fn, None, C.byref(stats)),
                       "rg_render_stream")
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
