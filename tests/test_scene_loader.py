"""The YAML loader reproduces the serde schema of Scene (scene.rs:11-31,
bodies.rs:13-47, lights.rs:8-26, material.rs:7-54)."""
import numpy as np
import pytest

from raingun_amd.color import Color
from raingun_amd.scene import (AABB, DirectionalLight, Disk, Plane, Scene, SceneDesc, SceneError, Sphere,
                               SphericalLight, Texture, load_scene)

MINI = """
bodies:
  - Sphere:
      center: [0.0, 0.0, -5.0]
      radius: 1
      material:
        coloration:
          Color: "#ff0000"
        albedo: 0.18
        surface: Diffuse
"""


def test_defaults():  # scene.rs:21-31
    s = load_scene("bodies: []\n")
    assert s.fov == 90.0 and s.max_recursion_depth == 10 and s.default_color == Color.black()
    assert s.bodies == [] and s.lights == []
    assert load_scene("{}\n").fov == 90.0


def test_examples_load(example_scenes):
    t1 = example_scenes["test1"]
    assert [type(b) for b in t1.bodies] == [Plane, Plane, Sphere, Sphere, Sphere, Sphere]
    assert [type(l) for l in t1.lights] == [DirectionalLight, SphericalLight, SphericalLight]
    # Point3 as a mapping (test1.yml:5-8) and as a sequence (test1.yml:13)
    assert t1.lights[0].direction == (0.4, -1.0, -0.9)
    assert t1.lights[1].position == (-6.0, 3.2, -5.0)
    assert t1.lights[2].position == (30.0, 20.0, -30.0)
    # `surface: Diffuse` (test1.yml:32) and `surface: {Diffuse: null}` (test1.yml:42-43)
    assert t1.bodies[0].material.surface == "Diffuse" and t1.bodies[1].material.surface == "Diffuse"
    assert t1.bodies[3].material.surface == "Reflecting"
    assert t1.bodies[3].material.reflectivity == float(np.float32(0.75))
    assert t1.bodies[5].material.surface == "Refractive"
    assert t1.bodies[5].material.index == float(np.float32(1.33))
    tex = t1.bodies[2].material.coloration
    assert isinstance(tex, Texture) and tex.image.shape == (1024, 2048, 4)
    assert tex.x_offset == float(np.float32(0.9))
    t2 = example_scenes["test2"]
    assert [type(b) for b in t2.bodies] == [Plane, Disk, Disk, AABB]
    assert t2.bodies[3].bounds == ((2.0, -2.0, -3.2), (2.8, -0.4, -3.0))
    t3 = example_scenes["test3"]
    assert t3.default_color == Color.from_str("#444444")


def test_f32_fields_are_rounded():
    s = load_scene(MINI.replace("0.18", "0.1"))
    assert s.bodies[0].material.albedo == float(np.float32(0.1))
    assert s.bodies[0].radius == 1.0


def test_deny_unknown_fields_on_scene_only():
    with pytest.raises(SceneError, match="unknown field `camera`"):
        load_scene("camera: 1\n")
    # unknown fields inside bodies are ignored by serde (no deny_unknown_fields there)
    s = load_scene(MINI.replace("radius: 1", "radius: 1\n      extra: 7"))
    assert isinstance(s.bodies[0], Sphere)


@pytest.mark.parametrize("yaml_text,msg", [
    (MINI.replace("Sphere:", "Cube:"), "unknown variant `Cube`"),
    (MINI.replace('"#ff0000"', '"red"'), "not a valid color"),
    (MINI.replace("      radius: 1\n", ""), "missing field `radius`"),
    (MINI.replace("surface: Diffuse", "surface: Glossy"), "unknown variant `Glossy`"),
    (MINI.replace("[0.0, 0.0, -5.0]", "[0.0, 0.0]"), "expected 3 components"),
    ("maxRecursionDepth: -1\n", "u32"),
    ("lights:\n  - Ambient:\n      color: \"#ffffff\"\n", "unknown variant `Ambient`"),
])
def test_errors(yaml_text, msg):
    with pytest.raises(SceneError, match=msg):
        load_scene(yaml_text)


def test_missing_texture_file(tmp_path):
    y = MINI.replace('Color: "#ff0000"', 'Texture:\n            image: "nope.jpg"\n            x_offset: 0.0\n'
                                         '            y_offset: 0.0')
    with pytest.raises(SceneError, match="Could not load texture file nope.jpg"):
        load_scene(y, texture_root=tmp_path)


def test_exponent_floats():
    s = load_scene("fov: 1e2\n")  # YAML 1.1 leaves 1e2 a string; yaml-rust parses it as a float
    assert s.fov == 100.0


def test_desc_layout(example_scenes):
    d = SceneDesc(example_scenes["test1"])
    assert d.desc.n_bodies == 6 and d.desc.n_lights == 3 and d.desc.n_textures == 2
    assert d.desc.bodies[2].material.coloration == 1 and d.desc.bodies[2].material.texture in (0, 1)
    assert d.desc.bodies[5].material.surface == 2
    assert tuple(d.desc.bodies[3].p[:4]) == (-10.0, 3.0, -15.2, 5.0)


def test_programmatic_scene():
    from raingun_amd.scene import Material
    m = Material(Color.from_str("#00ff00"), 0.5)
    s = Scene(bodies=[Sphere((0.0, 0.0, -3.0), 1.0, m)], lights=[DirectionalLight((0, -1, 0), Color(1, 1, 1), 2.0)])
    d = SceneDesc(s)
    assert d.desc.n_bodies == 1 and d.desc.lights[0].kind == 0
