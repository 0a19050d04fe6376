"""raingun_amd — MI355X-native renderer for raingun's per-pixel ray-trace path.

Host-side mirror of raingun-lib's API (Scene / render_image / streaming_render /
trace) above the C ABI of libraingun_hip.so (include/raingun.h).
"""
from .color import Color
from .scene import (AABB, DeviceScene, DirectionalLight, Disk, Material, Plane, Scene, SceneDesc, SceneError,
                    Sphere, SphericalLight, Texture, load_scene)
from ._abi import RaingunError

__all__ = ["AABB", "Color", "DeviceScene", "DirectionalLight", "Disk", "Material", "Plane", "RaingunError",
           "Scene", "SceneDesc", "SceneError", "Sphere", "SphericalLight", "Texture", "load_scene"]
