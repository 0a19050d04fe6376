"""GPU (libraingun_hip.so, through the C ABI) vs the CPU restatement (oracle).

The bar: RGBA8 output byte-identical, pre-quantisation f32 RGB within 1e-4 per
channel (north_star tolerance; observed 0), and per-class ray counts exactly
equal.  Scenes: the reference's three examples at its default 800x600 and at
the BASELINE configs' 3840x2160, plus seeded synthetic N-sphere scenes.
"""
import copy

import numpy as np
import pytest

from raingun_amd import _abi
from raingun_amd.scene import AABB, DeviceScene, Material, Scene, SceneDesc
from raingun_amd.color import Color
from raingun_amd.synth import synthetic_scene

pytestmark = pytest.mark.gpu

RGB_TOL = 1e-4  # per-channel |delta| bound stated by the north_star


@pytest.fixture(scope="module", autouse=True)
def _device():
    lib = _abi.lib()  # raises if the HIP library is missing: no fallback
    assert lib.rg_device_count() > 0, "no HIP device visible"


def _compare(oracle_lib, scene, w, h, tile_rows=0, stride=1, offset=0, path=None, bvh=None, lane=None,
             lightbuf=None):
    desc = SceneDesc(scene)
    ds = DeviceScene(scene, path=path, bvh=bvh)
    if lane is not None:
        ds.set_lane_depth(lane)
    if lightbuf is not None:
        ds.set_lightbuf(lightbuf)
    st = _abi.rg_stats()
    g_rgba, g_rgb = ds.render_tiles(w, h, tile_rows, stride, offset, want_rgb=True, stats=st)
    o_st, o_rgba, o_rgb, o_counts, o_err = oracle_lib.render(desc, w, h, tile_rows, stride, offset, want_rgb=True)
    assert o_st == 0
    assert st.rays.as_dict() == o_counts, "ray counts differ"
    diff = np.abs(g_rgb.astype(np.float64) - o_rgb.astype(np.float64))
    assert np.nanmax(diff) <= RGB_TOL
    mism = np.count_nonzero((g_rgba != o_rgba).any(axis=2))
    assert mism == 0, f"{mism} RGBA8 pixels differ"
    ds.close()
    return st


PATHS = [_abi.PATH_LIGHT, _abi.PATH_HEAVY]  # both kernel paths on every scene
# (kernel path, sphere BVH, per-lane walk depth): the light path never
# traverses; the heavy path with >= 16 spheres traverses the BVH by default,
# rays of depth >= 1 per lane; lane depth 0 = every non-primary ray per lane,
# 99 = wave-coherent walk only
PATH_BVH = [(_abi.PATH_LIGHT, False, None), (_abi.PATH_HEAVY, False, None), (_abi.PATH_HEAVY, True, None),
            (_abi.PATH_HEAVY, True, 0), (_abi.PATH_HEAVY, True, 99)]


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("name", ["test1", "test2", "test3"])
def test_examples_800x600(oracle_lib, example_scenes, name, path):
    st = _compare(oracle_lib, example_scenes[name], 800, 600, path=path)
    assert st.rays.primary == 800 * 600


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("name", ["test1", "test2", "test3"])
def test_examples_reproduce_reference_golden_png(example_scenes, golden_dir, name, path):
    """The GPU output equals the reference's own renders byte for byte
    (examples/test{1,2,3}.png, 800x600, YAML depth), textures included."""
    from PIL import Image

    ds = DeviceScene(example_scenes[name], path=path)
    got = ds.render_image(800, 600)
    ds.close()
    gold = np.asarray(Image.open(golden_dir / "examples" / f"{name}.png").convert("RGBA"))
    assert np.array_equal(got, gold)


def test_config2_test1_4k_depth5(oracle_lib, example_scenes):
    s = copy.copy(example_scenes["test1"])
    s.max_recursion_depth = 5
    _compare(oracle_lib, s, 3840, 2160)


def test_config3_test3_4k(oracle_lib, example_scenes):
    _compare(oracle_lib, example_scenes["test3"], 3840, 2160)


@pytest.mark.parametrize("n,planes,depth,w,h", [
    (16, 2, 5, 320, 240),
    (64, 8, 8, 256, 144),
    (1024, 2, 5, 192, 108),
    (200, 2, 0, 160, 90),
    (200, 2, 1, 160, 90),
    (200, 2, 2, 160, 90),
    (40, 4, 20, 160, 90),
])
@pytest.mark.parametrize("path,bvh,lane", PATH_BVH)
def test_synthetic(oracle_lib, n, planes, depth, w, h, path, bvh, lane):
    _compare(oracle_lib, synthetic_scene(n, planes, depth), w, h, path=path, bvh=bvh, lane=lane)


@pytest.mark.parametrize("keep", [[0], [1], [0, 1], [1, 2], [0, 1, 2]])
@pytest.mark.parametrize("path", PATHS)
def test_light_counts(oracle_lib, example_scenes, keep, path):
    """test1 with 1, 2 or 3 of its lights: the light path runs a 2-light shadow batch for scenes
    with at most RG_LB_SMALL (2) lights and the 3-light one otherwise (rg_kernels.hip launch_depth)."""
    scene = copy.deepcopy(example_scenes["test1"])
    scene.lights = [scene.lights[i] for i in keep]
    _compare(oracle_lib, scene, 320, 240, path=path)


@pytest.mark.parametrize("n,planes,depth,w,h", [(16, 2, 5, 320, 240), (1024, 2, 5, 192, 108), (40, 4, 20, 160, 90)])
@pytest.mark.parametrize("lane", [None, 0])
def test_synthetic_shadow_rays_walk_the_bvh(oracle_lib, n, planes, depth, w, h, lane):
    """The heavy path with the shadow-ray light buffers off: every shadow ray walks the BVH
    (the default path since round 5 tests its cell's spheres instead)."""
    _compare(oracle_lib, synthetic_scene(n, planes, depth), w, h, path=_abi.PATH_HEAVY, bvh=True, lane=lane,
             lightbuf=False)


def _lights_scene(n=1024):
    """The synthetic scene plus lights that stress the light buffers: a point light inside the
    sphere field, one far away, one inside a sphere, an axis-aligned and an oblique directional light."""
    from raingun_amd.scene import DirectionalLight, SphericalLight

    s = synthetic_scene(n, 2, 5)
    c0 = s.bodies[2].center  # the first sphere (after the two planes)
    s.lights += [SphericalLight(position=(0.5, 4.0, -40.0), color=Color(1.0, 0.9, 0.8), intensity=20000.0),
                 SphericalLight(position=(300.0, 500.0, 200.0), color=Color(0.5, 0.5, 1.0), intensity=9e6),
                 SphericalLight(position=tuple(c0), color=Color(1.0, 1.0, 1.0), intensity=100.0),
                 DirectionalLight(direction=(0.0, -1.0, 0.0), color=Color(0.9, 1.0, 0.9), intensity=2.0),
                 DirectionalLight(direction=(-0.3, -0.2, 1.0), color=Color(1.0, 0.8, 0.8), intensity=2.0)]
    return s


def test_lightbuf_is_built_for_sphere_scenes():
    ds = DeviceScene(synthetic_scene(1024, 2, 5))
    assert ds.lightbuf_count() == 3  # 1 directional + 2 spherical lights
    ds.set_bvh(False)
    assert ds.lightbuf_count() == 0  # the buffers ride on the BVH's bounds and path
    ds.set_bvh(True)
    ds.set_lightbuf(False)
    assert ds.lightbuf_count() == 0  # built, but not in use
    ds.set_lightbuf(True)
    assert ds.lightbuf_count() == 3
    ds.close()
    ds = DeviceScene(_lights_scene())
    assert ds.lightbuf_count() >= 6
    ds.close()


@pytest.mark.parametrize("lightbuf", [True, False])
@pytest.mark.parametrize("lane", [None, 0])
def test_lightbuf_stress_lights(oracle_lib, lightbuf, lane):
    """Eight lights (inside the sphere field, far away, inside a sphere, axis-aligned and oblique
    directional) on the 1024-sphere scene: with and without the light buffers, against the CPU
    restatement."""
    _compare(oracle_lib, _lights_scene(), 192, 108, path=_abi.PATH_HEAVY, bvh=True, lane=lane, lightbuf=lightbuf)


def _lights_scene_past_buffers():
    """Eleven lights: more than the RG_LB_MAX_LIGHTS (8) that get a light buffer, so shadow rays of
    lights 8.. walk the BVH, beside the camera buffer's slot in the same descriptor array."""
    from raingun_amd.scene import DirectionalLight, SphericalLight

    s = _lights_scene()
    s.lights += [SphericalLight(position=(-20.0, 30.0, -60.0), color=Color(0.7, 1.0, 0.7), intensity=30000.0),
                 DirectionalLight(direction=(0.5, -0.7, -0.2), color=Color(1.0, 1.0, 0.6), intensity=1.5),
                 SphericalLight(position=(10.0, 2.0, -25.0), color=Color(0.9, 0.6, 1.0), intensity=5000.0)]
    assert len(s.lights) == 11
    return s


@pytest.mark.parametrize("lightbuf", [True, False])
def test_lightbuf_more_lights_than_buffers(oracle_lib, lightbuf):
    """Lights beyond the buffered ones fall back to the BVH walk: both settings against
    the CPU restatement on the 1024-sphere scene."""
    s = _lights_scene_past_buffers()
    ds = DeviceScene(s)
    assert ds.lightbuf_count() <= 8
    ds.close()
    _compare(oracle_lib, s, 160, 90, path=_abi.PATH_HEAVY, bvh=True, lightbuf=lightbuf)


def test_bvh_is_built_for_sphere_scenes():
    ds = DeviceScene(synthetic_scene(1024, 2, 5))
    info = ds.bvh_info()
    assert info.built == 1 and info.enabled == 1 and info.nodes > 64 and info.leaves >= 1024 // 4
    assert 0 < info.margin < 0.05 and info.origin_bound > 100
    assert 0 < info.lbuf_bytes < 4 * (1 << 25)  # 3 lights + the camera buffer, under the scene's cap
    ds.set_bvh(False)
    assert ds.bvh_info().enabled == 0
    ds.close()
    small = DeviceScene(synthetic_scene(8, 2, 5))
    assert small.bvh_info().built == 0
    small.close()


@pytest.mark.parametrize("bvh,lane", [(True, None), (True, 0), (True, 99), (False, None)])
def test_config5_shape_4096_spheres_8_planes(oracle_lib, bvh, lane):
    """BASELINE configs[4]'s scene (4096 spheres + 8 planes, depth 8; the sphere
    tables exceed LDS, so the BVH kernel reads nodes through the scalar cache)
    at a reduced resolution the CPU restatement finishes quickly."""
    _compare(oracle_lib, synthetic_scene(4096, 8, 8), 256, 144, path=_abi.PATH_HEAVY, bvh=bvh, lane=lane)


@pytest.mark.parametrize("lane", [None, 0])
def test_north_star_scene_4k_bvh(oracle_lib, lane):
    """The north-star scene (1024 spheres) at the full 3840x2160, depth 5,
    every 9th 16-row tile (the restatement scans all 1026 bodies per ray)."""
    _compare(oracle_lib, synthetic_scene(1024, 2, 5), 3840, 2160, 16, 9, 4, lane=lane)


def test_odd_sizes_and_square(oracle_lib, example_scenes):
    for w, h in [(1, 1), (17, 3), (97, 61), (64, 64)]:
        _compare(oracle_lib, example_scenes["test1"], w, h)


@pytest.mark.parametrize("tile_rows,stride,offset", [(8, 3, 1), (16, 4, 3), (7, 2, 0), (600, 1, 0)])
def test_tiles_match_oracle(oracle_lib, example_scenes, tile_rows, stride, offset):
    _compare(oracle_lib, example_scenes["test1"], 800, 600, tile_rows, stride, offset)


def test_interleaved_tiles_assemble_to_frame(example_scenes):
    """N row-tile shards (the multi-GPU partition) reassemble to the 1-GPU frame bit-exactly."""
    s = example_scenes["test3"]
    ds = DeviceScene(s)
    w, h, T, N = 640, 480, 16, 4
    whole = ds.render_image(w, h)
    tiles = (h + T - 1) // T
    frame = np.zeros((tiles * T, w, 4), np.uint8)
    for r in range(N):
        part = ds.render_tiles(w, h, T, N, r)
        for j, t in enumerate(range(r, tiles, N)):
            frame[t * T:(t + 1) * T] = part[j * T:(j + 1) * T]
    assert np.array_equal(frame[:h], whole)


def test_stream_bands(example_scenes):
    s = example_scenes["test2"]
    w, h = 320, 240
    whole = DeviceScene(s).render_image(w, h)
    got = np.zeros_like(whole)
    seen = []

    def on_tile(row0, band):
        got[row0:row0 + band.shape[0]] = band
        seen.append(row0)
        return False

    stats = s.streaming_render(w, h, on_tile, tile_rows=32)
    assert np.array_equal(got, whole)
    assert seen == list(range(0, h, 32))
    assert stats.rays.primary == w * h


def test_stream_cancel(example_scenes):
    s = example_scenes["test2"]
    calls = []
    with pytest.raises(_abi.RaingunError) as ei:
        s.streaming_render(320, 240, lambda r, b: calls.append(r) or True, tile_rows=32)
    assert ei.value.status == _abi.RG_ERR_CANCELLED
    assert calls == [0]


@pytest.mark.parametrize("bvh", [True, False])
def test_trace_matches_oracle(oracle_lib, bvh):
    s = synthetic_scene(256, 2, 5)
    rng = np.random.default_rng(7)
    n = 4096
    o = rng.uniform(-30, 30, size=(n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d], axis=1)
    gd, gb = DeviceScene(s, bvh=bvh).trace(rays)
    st, od, ob = oracle_lib.trace(SceneDesc(s), rays)
    assert st == 0
    assert np.array_equal(gb, ob)
    hit = ob >= 0
    assert np.array_equal(gd[hit], od[hit])
    assert 0 < hit.sum() < n


def test_portrait_is_rejected(example_scenes):
    ds = DeviceScene(example_scenes["test2"])
    with pytest.raises(_abi.RaingunError) as ei:
        ds.render_image(60, 80)
    assert ei.value.status == _abi.RG_ERR_PORTRAIT


def test_aabb_normal_error_matches_oracle(oracle_lib):
    """bodies.rs:324 panics when no face is within 1e-8 of the hit point; far
    from the origin the f64 hit point misses every face by more than that."""
    m = Material(Color.from_str("#ffffff"), 0.5)
    s = Scene(bodies=[AABB(((-3e8, -3e8, -7e8), (3e8, 3e8, -5e8)), m)])
    desc = SceneDesc(s)
    o_st, _, _, _, o_err = oracle_lib.render(desc, 64, 48)
    st = _abi.rg_stats()
    ds = DeviceScene(s)
    with pytest.raises(_abi.RaingunError) as ei:
        ds.render_tiles(64, 48, stats=st)
    assert o_st == _abi.RG_ERR_AABB_NORMAL
    assert ei.value.status == o_st
    assert st.error_pixel == o_err


@pytest.mark.parametrize("scale", [1.0, 40.0, 3000.0])
def test_f32_prefilter_tangent_rays(oracle_lib, scale):
    """Rays grazing sphere silhouettes (opp within 1e-9 relative of r^2), from
    near and far origins at several scene scales: the heavy path's f32
    pre-filter must never reject a sphere the exact f64 test accepts."""
    from raingun_amd.color import Color
    from raingun_amd.scene import Material, Sphere
    rng = np.random.default_rng(11)
    m = Material(Color.from_str("#ffffff"), 0.5)
    centers = rng.uniform(-1, 1, size=(64, 3)) * scale * 4 + np.array([0, 0, -8 * scale])
    radii = rng.uniform(0.01, 0.2, size=64) * scale
    s = Scene(bodies=[Sphere(tuple(c), float(r), m) for c, r in zip(centers, radii)])
    rays, targets = [], []
    for _ in range(8192):
        k = rng.integers(64)
        c, r = centers[k], radii[k]
        o = rng.uniform(-3, 3, size=3) * scale
        d = c - o                                   # aim at the centre ...
        perp = np.cross(d, rng.normal(size=3))
        perp /= np.linalg.norm(perp)
        o = o + perp * r * (1.0 + rng.uniform(-1e-9, 1e-9))  # ... then slide off by ~r, across d
        if rng.integers(2):
            d /= np.linalg.norm(d)
        rays.append(np.concatenate([o, d]))
        targets.append(k)
    rays, targets = np.array(rays), np.array(targets)
    for path, bvh, lane in PATH_BVH:  # rg_trace walks per lane at lane depth <= 1
        ds = DeviceScene(s, path=path, bvh=bvh)
        if lane is not None:
            ds.set_lane_depth(lane)
        gd, gb = ds.trace(rays)
        ds.close()
        st, od, ob = oracle_lib.trace(SceneDesc(s), rays)
        assert st == 0
        assert np.array_equal(gb, ob), f"path {path} bvh {bvh} lane {lane}: {np.count_nonzero(gb != ob)} rays differ"
        hit = ob >= 0
        assert np.array_equal(gd[hit], od[hit])
    # where nothing else is in the way, grazing rays split between hitting and
    # missing their target: the boundary really is exercised
    own = (ob == targets) | (ob == -1)
    assert own.sum() > 1000
    assert 0.2 < (ob[own] == targets[own]).mean() < 0.8


@pytest.mark.parametrize("scene_kind", ["synth200", "test1", "test3"])
def test_tile_order_changes_nothing(oracle_lib, example_scenes, scene_kind):
    """Probe-ordered tile scheduling (include/raingun_debug.h) only changes the
    dequeue order: frame, f32 RGB and ray counts equal the raster-order render
    and the CPU restatement, for whole frames and row tilings."""
    scene = synthetic_scene(200, 2, 5) if scene_kind == "synth200" else example_scenes[scene_kind]
    w, h = 320, 180
    for order in (1, 0):
        ds = DeviceScene(scene)
        ds.set_tile_order(order)
        st = _abi.rg_stats()
        rgba, rgb = ds.render_tiles(w, h, want_rgb=True, stats=st)
        part = ds.render_tiles(w, h, 16, 3, 2)
        ds.close()
        o_st, o_rgba, o_rgb, o_counts, _ = oracle_lib.render(SceneDesc(scene), w, h, want_rgb=True)
        _, o_part, _, _, _ = oracle_lib.render(SceneDesc(scene), w, h, 16, 3, 2)
        assert np.array_equal(rgba, o_rgba) and np.array_equal(part, o_part)
        assert float(np.abs(rgb - o_rgb).max()) <= RGB_TOL
        assert st.rays.as_dict() == o_counts


@pytest.mark.parametrize("scene_kind", ["synth200", "test1"])
def test_frames_in_flight_on_concurrent_streams(oracle_lib, example_scenes, scene_kind):
    """Frames in flight (bench.py, FramePipeline): launches of one scene on
    distinct streams run concurrently, each with its own launch state (ray
    counters, tile queues, tile-order scratch).  Every part must still equal
    the CPU restatement, and a counted launch afterwards must count exactly."""
    import ctypes as C

    import torch

    scene = synthetic_scene(200, 2, 5) if scene_kind == "synth200" else example_scenes[scene_kind]
    w, h, T, F = 320, 180, 16, 3
    ds = DeviceScene(scene)
    lib = _abi.lib()
    streams = [torch.cuda.Stream() for _ in range(F)]
    tilings = [_abi.rg_tiling(T, F, i) for i in range(F)]
    rows = [lib.rg_tiling_rows(h, C.byref(t)) for t in tilings]
    bufs = [[torch.full((rows[i], w, 4), 7, dtype=torch.uint8, device="cuda") for _ in range(2)] for i in range(F)]
    for rnd in range(4):  # several rounds: each stream's launches queue behind the others' in flight
        for i in range(F):
            b = bufs[i][rnd % 2]
            _abi.check(lib.rg_render_tiles_async(ds.handle, w, h, C.byref(tilings[i]), C.c_void_p(b.data_ptr()),
                                                 None, C.c_void_p(streams[i].cuda_stream), None))
    torch.cuda.synchronize()
    for i in range(F):
        _, o_part, _, _, _ = oracle_lib.render(SceneDesc(scene), w, h, T, F, i)
        for b in bufs[i]:
            assert np.array_equal(b.cpu().numpy(), o_part), f"stream {i}"
    st = _abi.rg_stats()
    ds.render_tiles(w, h, stats=st)
    ds.close()
    assert st.rays.as_dict() == oracle_lib.render(SceneDesc(scene), w, h)[3]


@pytest.mark.parametrize("path, bvh, lane", PATH_BVH)
def test_point_lights_in_plane_surfaces(oracle_lib, path, bvh, lane):
    """Spherical lights lying exactly in plane surfaces: every shadow ray
    towards them meets the plane at (almost) the light's own distance, so the
    occlusion test fl(num/den) <= light distance (bodies.rs:137-148,
    rendering.rs:152-155) is decided by the last rounding: the kernels'
    unfused f64 division and comparison must agree with the restatement pixel
    for pixel.  (A division-free pre-decision of this comparison was tried
    against this test and rejected as slower: profiles/r02/heavy_path_experiments.txt.)"""
    from raingun_amd.scene import DirectionalLight, Plane, Sphere, SphericalLight
    rng = np.random.default_rng(23)
    m = Material(Color.from_str("#c0c0c0"), 0.6)
    mr = Material(Color.from_str("#ffffff"), 0.5)
    mr.surface = "Reflecting"
    mr.reflectivity = 0.4
    bodies = [Plane((0.0, -2.0, 0.0), (0.0, -1.0, 0.0), m),        # floor (normal away from the camera)
              Plane((0.0, 0.0, -30.0), (0.0, 0.0, -1.0), m)]        # back wall
    for _ in range(40):
        c = (rng.uniform(-9, 9), rng.uniform(-1.5, 4), rng.uniform(-25, -6))
        bodies.append(Sphere(c, float(rng.uniform(0.3, 1.2)), mr if rng.integers(3) == 0 else m))
    lights = [SphericalLight((1.37, -2.0, -11.3), Color.from_str("#ffeedd"), 900.0),   # in the floor
              SphericalLight((-4.1, 2.9, -30.0), Color.from_str("#ddeeff"), 1500.0),   # in the back wall
              DirectionalLight((0.3, -1.0, -0.5), Color.from_str("#ffffff"), 0.6)]
    s = Scene(bodies=bodies, lights=lights, max_recursion_depth=4)
    _compare(oracle_lib, s, 320, 180, path=path, bvh=bvh, lane=lane)
