"""The native host layer (include/raingun_host.h, raingun_amd/host/): C-ABI
exports, the JPEG/PNG codecs, the YAML scene loader and the `raingun` binary.
CPU only (the binary's render call is covered by tests/test_gpu_cli.py)."""
import hashlib
import io
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest
from PIL import Image

from raingun_amd import _abi, _host
from raingun_amd.color import Color
from raingun_amd.scene import SceneDesc, SceneError, Texture, load_scene

INCLUDE = Path(__file__).resolve().parent.parent / "include"
TEXTURES = Path(__file__).resolve().parent / "golden" / "textures"
JPEGS = ["clay-ground-seamless.jpg", "land_ocean_ice_cloud_2048.jpg", "tile1/color.jpg"]


def declared(header):
    text = re.sub(r"/\*.*?\*/", "", header.read_text(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*(rgh_[a-z0-9_]+)\s*\(", text,
                                 flags=re.M)))


# ---------------------------------------------------------------- ABI
def test_header_matches_binding_and_exports():
    assert declared(INCLUDE / "raingun_host.h") == sorted(_host.EXPORTED_SYMBOLS)
    _host.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", str(_host.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    assert not [s for s in _host.EXPORTED_SYMBOLS if s not in exported]


def test_null_arguments_fail_loudly():
    import ctypes as C
    l = _host.lib()
    assert l.rgh_scene_load_file(None, None, None) == _host.RGH_ERR_INVALID_ARGUMENT
    assert l.rgh_png_encode(None, 1, 1, None, None) == _host.RGH_ERR_INVALID_ARGUMENT
    assert not l.rgh_scene_desc(None)  # NULL in, NULL out
    w, h, p = C.c_uint32(), C.c_uint32(), C.POINTER(C.c_uint8)()
    assert l.rgh_image_decode(b"xx", 2, 0, C.byref(w), C.byref(h), C.byref(p)) == _host.RGH_ERR_IMAGE
    assert "could not be determined" in l.rgh_last_error().decode()


# ---------------------------------------------------------------- JPEG
# sha256 of the reference-flavour RGBA8 decode.  These are the texels with
# which tests/test_oracle_golden.py reproduces examples/test{1,3}.png exactly.
REFERENCE_DIGESTS = {
    "clay-ground-seamless.jpg": "f7e711383ed83620361e9568c15e3cd010d8946cdd29df013f55477331481a5f",
    "land_ocean_ice_cloud_2048.jpg": "ce8cc6bd5131e743fb8cca8958b4c9f784fd600c9fb54c4f91cbebe5f75e69db",
    "tile1/color.jpg": "4f20d834b6ef9b9db028fe634d02dcb8f9f01efbfeea5dd17d6b9d7623aac419",
}


@pytest.mark.parametrize("name", JPEGS)
def test_jpeg_reference_flavour_digest(name):
    img = _host.decode_image_file(TEXTURES / name)
    assert hashlib.sha256(img.tobytes()).hexdigest() == REFERENCE_DIGESTS[name]
    assert (img[..., 3] == 255).all()


@pytest.mark.parametrize("name", JPEGS)
def test_jpeg_libjpeg_flavour_equals_pil(name):
    """The reference's textures cover baseline 4:2:0 (tile1), baseline 4:4:4
    (earth) and progressive 4:4:4 (clay)."""
    ours = _host.decode_image_file(TEXTURES / name, _host.JPEG_LIBJPEG)
    pil = np.asarray(Image.open(TEXTURES / name).convert("RGBA"))
    assert np.array_equal(ours, pil)


def _synthetic_jpeg(w, h, mode="RGB", seed=0, **save):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = np.stack([(xx * 7 + yy * 3) % 256, (xx * 2 + yy * 11) % 256, (xx * yy) % 256], axis=-1)
    noise = rng.integers(0, 40, size=(h, w, 3))
    arr = np.clip(base + noise, 0, 255).astype(np.uint8)
    im = Image.fromarray(arr, "RGB")
    if mode == "L":
        im = im.convert("L")
    b = io.BytesIO()
    im.save(b, "JPEG", **save)
    return b.getvalue()


@pytest.mark.parametrize("w,h,mode,save", [
    (64, 48, "RGB", dict(quality=90, subsampling=0)),
    (61, 37, "RGB", dict(quality=75, subsampling=1)),            # 4:2:2, ragged edges
    (61, 37, "RGB", dict(quality=75, subsampling=2)),            # 4:2:0, ragged edges
    (97, 65, "RGB", dict(quality=60, subsampling=2, progressive=True)),
    (97, 65, "RGB", dict(quality=95, subsampling=0, progressive=True)),
    (50, 30, "L", dict(quality=80)),
    (50, 30, "L", dict(quality=80, progressive=True)),
    (80, 40, "RGB", dict(quality=85, subsampling=2, restart_marker_blocks=3)),
    (80, 40, "RGB", dict(quality=85, subsampling=2, progressive=True, restart_marker_rows=1)),
    (3, 2, "RGB", dict(quality=50, subsampling=2)),              # narrower than one MCU
    (17, 9, "RGB", dict(quality=100, subsampling=0, optimize=True)),
])
def test_jpeg_variants_equal_pil(w, h, mode, save):
    data = _synthetic_jpeg(w, h, mode, **save)
    ours = _host.decode_image(data, _host.JPEG_LIBJPEG)
    pil = np.asarray(Image.open(io.BytesIO(data)).convert("RGBA"))
    assert ours.shape == pil.shape
    assert np.array_equal(ours, pil)
    ref = _host.decode_image(data, _host.JPEG_REFERENCE)  # stb-style rounding: same image within a few LSB
    assert np.abs(ref.astype(int) - pil.astype(int)).max() <= 8


def test_jpeg_truncated_and_garbage():
    data = (TEXTURES / JPEGS[2]).read_bytes()
    with pytest.raises(_host.HostError):
        _host.decode_image(data[:2])
    with pytest.raises(_host.HostError):
        _host.decode_image(b"\xff\xd8\xff\xc3\x00\x02")  # lossless process: unsupported
    _host.decode_image(data[: len(data) // 2])  # truncated scan data decodes (IJG pads with zeros)


# ---------------------------------------------------------------- PNG
@pytest.mark.parametrize("name", ["test1", "test2", "test3"])
def test_png_decode_golden(golden_dir, name):
    p = golden_dir / "examples" / f"{name}.png"
    assert np.array_equal(_host.decode_image_file(p), np.asarray(Image.open(p).convert("RGBA")))


@pytest.mark.parametrize("mode", ["L", "LA", "RGB", "RGBA", "P", "1", "P-trns"])
def test_png_modes_equal_pil(mode):
    rng = np.random.default_rng(5)
    arr = rng.integers(0, 256, size=(23, 41, 4), dtype=np.uint8)
    im = Image.fromarray(arr, "RGBA")
    if mode == "P-trns":
        im = im.convert("RGB").convert("P", palette=Image.ADAPTIVE, colors=16)
        im.info["transparency"] = 3
    elif mode == "P":
        im = im.convert("RGB").convert("P", palette=Image.ADAPTIVE, colors=200)
    else:
        im = im.convert(mode)
    b = io.BytesIO()
    if mode == "P-trns":
        im.save(b, "PNG", transparency=3)
    else:
        im.save(b, "PNG")
    ours = _host.decode_image(b.getvalue())
    pil = np.asarray(Image.open(io.BytesIO(b.getvalue())).convert("RGBA"))
    assert np.array_equal(ours, pil)


def test_png_16bit_keeps_high_byte():
    import struct
    import zlib
    w, h = 5, 3
    vals = np.arange(w * h * 3, dtype=np.uint16).reshape(h, w, 3) * 4099
    raw = b"".join(b"\x00" + vals[y].astype(">u2").tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    png = (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 16, 2, 0, 0, 0)) +
           chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b""))
    out = _host.decode_image(png)
    assert np.array_equal(out[..., :3], (vals >> 8).astype(np.uint8)) and (out[..., 3] == 255).all()


def test_png_encode_roundtrip(tmp_path):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, size=(37, 53, 4), dtype=np.uint8)
    assert np.array_equal(np.asarray(Image.open(io.BytesIO(_host.encode_png(img))).convert("RGBA")), img)
    assert np.array_equal(_host.decode_image(_host.encode_png(img)), img)
    import ctypes as C
    out = tmp_path / "x.png"
    assert _host.lib().rgh_png_write(str(out).encode(), img.ctypes.data, 53, 37) == 0
    assert np.array_equal(np.asarray(Image.open(out).convert("RGBA")), img)


# ---------------------------------------------------------------- YAML + serde schema
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


def _load(text, root=None):
    return load_scene(text, texture_root=root)


def test_yaml_flow_and_block_forms_agree():
    block = _load(MINI)
    flow = _load('bodies: [{Sphere: {center: {x: 0.0, y: 0.0, z: -5.0}, radius: 1,\n'
                 '   material: {coloration: {Color: "#ff0000"}, albedo: 0.18, surface: Diffuse}}}]\n')
    quoted = _load(MINI.replace("center:", "'center':").replace("radius:", '"radius":'))
    docmark = _load("%YAML 1.2\n---\n" + MINI + "...\n")
    commented = _load("# scene\n" + MINI.replace("radius: 1", "radius: 1   # one unit\n      # more"))
    for s in (flow, quoted, docmark, commented):
        assert s.bodies == block.bodies


def test_yaml_anchors_and_aliases():
    s = _load("""
bodies:
  - Sphere:
      center: [0, 0, -5]
      radius: 1
      material: &red
        coloration: {Color: "#ff0000"}
        albedo: 0.5
        surface: Diffuse
  - Sphere:
      center: [2, 0, -5]
      radius: 1
      material: *red
""")
    assert s.bodies[0].material == s.bodies[1].material


def test_yaml_sequence_at_parent_indentation_and_block_scalar():
    s = _load('defaultColor: >-\n  #102030\nlights:\n- Directional:\n    direction: [0, -1, 0]\n'
              '    color: "#ffffff"\n    intensity: 2\n')
    assert s.default_color == Color.from_str("#102030")
    assert len(s.lights) == 1 and s.lights[0].intensity == 2.0


@pytest.mark.parametrize("text,value", [
    ("fov: 1e2\n", 100.0), ("fov: .5\n", 0.5), ("fov: 5.\n", 5.0), ("fov: +7\n", 7.0), ("fov: -3\n", -3.0),
    ("fov: 0x10\n", 16.0), ("fov: 0o17\n", 15.0), ("fov: 1E-1\n", 0.1), ("fov: inf\n", float("inf")),
])
def test_yaml_rust_number_resolution(text, value):
    assert _load(text).fov == value


@pytest.mark.parametrize("text,msg", [
    ('fov: "90"\n', "invalid type: string"),            # quoted scalars are strings, never numbers
    ("fov: 1_000\n", "invalid type: string"),           # YAML 1.1 digit separators: a string in yaml-rust
    ("fov: true\n", "invalid type: boolean"),
    ("maxRecursionDepth: 2.0\n", "expected u32"),
    ("maxRecursionDepth: 4294967296\n", "expected u32"),
    ("bodies: ~\n", "expected a sequence"),
    ("bodies: {}\n", "expected a sequence"),
    ("- 1\n", "expected struct Scene"),
    ("fov: [1\n", "flow collection"),
    ("a:\n\tb: 1\n", "tab"),
    ("fov: 90\n  bad: 1\n", "indentation"),
    ("defaultColor: '#ffff'\n", "not a valid color"),
    ("defaultColor: '#gg0000'\n", "not a valid color"),
    ("lights: [Directional]\n", "unit variant"),
    (MINI.replace("surface: Diffuse", "surface: {Diffuse: {a: 1}}"), "Diffuse takes no fields"),
    (MINI.replace("surface: Diffuse", "surface: Reflecting"), "unit variant"),
    (MINI.replace("surface: Diffuse", "surface: {Refractive: {index: 1.3}}"), "missing field `transparency`"),
    (MINI.replace("Sphere:", "AABB:").replace("center: [0.0, 0.0, -5.0]", "bounds: [[0, 0, 0]]"),
     "expected two points"),
    (MINI.replace("[0.0, 0.0, -5.0]", "{x: 0, y: 0}"), "missing field `z`"),
    (MINI.replace("coloration:\n          Color", "coloration:\n          Colour"), "unknown variant `Colour`"),
])
def test_schema_errors(text, msg):
    with pytest.raises(SceneError, match=msg):
        _load(text)


def test_color_parsing_follows_from_str_radix():
    assert _load("defaultColor: '#+fffff'\n").default_color == Color.from_str("#0fffff")
    assert _load("defaultColor: \"#FfA07a\"\n").default_color == Color.from_str("#ffa07a")


def test_textures_shared_by_path(tmp_path, golden_dir):
    src = golden_dir / "textures" / "tile1" / "color.jpg"
    (tmp_path / "a.jpg").write_bytes(src.read_bytes())
    (tmp_path / "b.jpg").write_bytes(src.read_bytes())
    tex = 'Texture: {{image: "{}", x_offset: 0, y_offset: 0}}'
    body = ("  - Sphere: {{center: [0, 0, -5], radius: 1, material: {{coloration: {{{}}}, albedo: 1, "
            "surface: Diffuse}}}}\n")
    text = "bodies:\n" + "".join(body.format(tex.format(p)) for p in ("a.jpg", "a.jpg", "b.jpg"))
    ls = _host.LoadedScene.from_string(text, tmp_path)
    d = ls.desc
    assert d.n_textures == 2
    assert [d.bodies[i].material.texture for i in range(3)] == [0, 0, 1]
    assert ls.texture_path(1) == "b.jpg"
    s = _load(text, tmp_path)
    assert isinstance(s.bodies[0].material.coloration, Texture)
    assert s.bodies[0].material.coloration.image is s.bodies[1].material.coloration.image
    ls.close()


def test_clamp_depth_only_lowers():
    ls = _host.LoadedScene.from_string("maxRecursionDepth: 3\n")
    ls.clamp_depth(4)
    assert ls.desc.max_recursion_depth == 3
    ls.clamp_depth(2)
    assert ls.desc.max_recursion_depth == 2
    ls.close()


def test_synthetic_scene_loads_fast_and_complete():
    from raingun_amd import synth
    import time
    y = synth.synthetic_yaml(4096, 8)
    t0 = time.perf_counter()
    ls = _host.LoadedScene.from_string(y)
    dt = time.perf_counter() - t0
    assert ls.desc.n_bodies == 4096 + 8
    assert dt < 2.0
    ls.close()


# ---------------------------------------------------------------- the `raingun` binary (no render)
@pytest.fixture(scope="module")
def cli():
    if not (_abi.PKG_DIR / "libraingun_hip.so").exists():
        subprocess.run(["make", "-s", "-C", str(_abi.PKG_DIR / "csrc")], check=True)
    subprocess.run(["make", "-s", "-C", str(_host.SRC_DIR)], check=True)
    return str(_host.CLI_PATH)


def _run(cli, *args, cwd=None):
    return subprocess.run([cli, *args], capture_output=True, text=True, cwd=cwd, timeout=120)


def test_cli_help_and_version(cli):
    r = _run(cli, "--help")
    assert r.returncode == 0 and "USAGE" in r.stdout and "--4k" in r.stdout
    r = _run(cli, "--version")
    assert r.returncode == 0 and r.stdout.strip() == "raingun 0.1.0"


def test_cli_argument_errors(cli):
    r = _run(cli)
    assert r.returncode == 1 and "<FILE>" in r.stderr
    r = _run(cli, "--bogus", "x.yml")
    assert r.returncode == 1 and "wasn't expected" in r.stderr
    r = _run(cli, "--width")
    assert r.returncode == 1 and "requires a value" in r.stderr


def test_cli_panics_like_the_reference(cli, tmp_path):
    r = _run(cli, "--width", "wide", "x.yml")
    assert r.returncode == 101 and "Could not parse width" in r.stderr
    r = _run(cli, str(tmp_path / "missing.yml"))
    assert r.returncode == 101 and "Could not open input file" in r.stderr
    bad = tmp_path / "bad.yml"
    bad.write_text("camera: 1\n")
    r = _run(cli, str(bad))
    assert r.returncode == 101 and "Could not load YAML" in r.stderr and "unknown field `camera`" in r.stderr
    r = _run(cli, "..")
    assert r.returncode == 2 and "Could not guess output filename" in r.stdout
