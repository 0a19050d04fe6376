"""Pin the CPU restatement (oracle/) to the reference's own golden renders.

examples/test{1,2,3}.png are 800x600 RGBA8 renders produced by the reference
(examples/render-examples.sh:7-10: default 800x600, YAML default depth 10).
All three must be reproduced byte for byte.  test1/test3 sample JPEG
textures, so this also pins the texture decoder: the native host decoder
(raingun_amd/host/jpeg_decode.cpp) rounds like the reference's jpeg-decoder
0.1.11 (Cargo.lock:400-406); decoding with IJG/libjpeg rounding instead moves
1,172 / 6,977 texture-dependent pixels by up to 3 LSB (kept below as a
negative control, so the test cannot pass vacuously).
"""
import numpy as np
import pytest
from PIL import Image

from raingun_amd.scene import SceneDesc, Texture, load_scene


def _golden(golden_dir, name):
    return np.asarray(Image.open(golden_dir / "examples" / f"{name}.png").convert("RGBA"))


def test_test2_exact(oracle_lib, example_scenes, golden_dir):
    st, rgba, _, counts, err = oracle_lib.render(SceneDesc(example_scenes["test2"]), 800, 600)
    assert st == 0 and err == -1
    assert np.array_equal(rgba, _golden(golden_dir, "test2"))
    assert counts["primary"] == 480000


@pytest.mark.parametrize("name", ["test1", "test3"])
def test_textured_examples_exact(oracle_lib, golden_dir, name):
    scene = load_scene(golden_dir / "examples" / f"{name}.yml", texture_root=golden_dir)
    st, rgba, _, _, err = oracle_lib.render(SceneDesc(scene), 800, 600)
    assert st == 0 and err == -1
    assert np.array_equal(rgba, _golden(golden_dir, name))


@pytest.mark.parametrize("name,n_diff", [("test1", 1172), ("test3", 6977)])
def test_libjpeg_rounding_is_detected(oracle_lib, golden_dir, name, n_diff):
    """Negative control: libjpeg-rounded textures must NOT reproduce the goldens,
    and every pixel they change must be texture-dependent."""
    from raingun_amd import _host

    scene = load_scene(golden_dir / "examples" / f"{name}.yml", texture_root=golden_dir)
    for b in scene.bodies:
        c = b.material.coloration
        if isinstance(c, Texture):
            c.image = _host.decode_image_file(golden_dir / c.path, _host.JPEG_LIBJPEG)
    _, rgba, _, _, _ = oracle_lib.render(SceneDesc(scene), 800, 600)
    gold = _golden(golden_dir, name)
    diff = np.abs(rgba.astype(int) - gold.astype(int)).max(axis=2)
    assert int((diff > 0).sum()) == n_diff and diff.max() <= 3
    dep = np.zeros(diff.shape, bool)
    for val in (0, 128, 255):
        for b in scene.bodies:
            c = b.material.coloration
            if isinstance(c, Texture):
                img = np.full_like(c.image, val)
                img[..., 3] = 255
                c.image = img
        _, alt, _, _, _ = oracle_lib.render(SceneDesc(scene), 800, 600)
        dep |= (alt != rgba).any(axis=2)
    assert not ((diff > 0) & ~dep).any()


def test_hand_kats(oracle_lib, example_scenes):
    """Pixel values derived by hand from the formulas."""
    _, rgba, _, _, _ = oracle_lib.render(SceneDesc(example_scenes["test2"]), 800, 600)
    assert tuple(rgba[299, 790]) == (85, 85, 85, 255)       # sky = defaultColor #555555 (test2.yml:2)
    # floor just below the horizon: yellow * (n.l = 0.7125) * 7.0 * 0.15/pi -> 0.238 -> 60 (test2.yml:3-10,18-25)
    f32 = np.float32
    lit = f32(f32(f32(1.0) * f32(0.7125)) * f32(7.0)) * f32(f32(0.15) / f32(np.pi))
    assert int(lit * f32(255.0)) == 60
    assert tuple(rgba[300, 790]) == (60, 60, 0, 255)
    _, rgba3, _, _, _ = oracle_lib.render(SceneDesc(example_scenes["test3"]), 800, 600)
    assert tuple(rgba3[0, 0]) == (48, 32, 20, 255)          # wall #ffaa77 * light * n.l * 9 * 0.3 / pi


def test_ray_count_fixture(oracle_lib, example_scenes, golden_dir):
    """Per-class ray counts of the examples at 800x600 (tests/golden/ray_counts.json,
    made by tests/golden/make_fixtures.py) stay fixed."""
    import json

    want = json.loads((golden_dir / "ray_counts.json").read_text())
    for name, scene in example_scenes.items():
        _, _, _, counts, _ = oracle_lib.render(SceneDesc(scene), 800, 600)
        assert counts == want[name], name


def test_tiling_packs_rows(oracle_lib, example_scenes):
    d = SceneDesc(example_scenes["test2"])
    _, whole, _, _, _ = oracle_lib.render(d, 200, 150)
    _, part, _, _, _ = oracle_lib.render(d, 200, 150, 16, 3, 1)
    tiles = list(range(1, (150 + 15) // 16, 3))
    assert part.shape[0] == 16 * len(tiles)
    for j, t in enumerate(tiles):
        rows = whole[t * 16:(t + 1) * 16]
        assert np.array_equal(part[j * 16:j * 16 + rows.shape[0]], rows)
