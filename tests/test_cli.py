"""CLI parity with the reference's own tests (src/main.rs:134-179) plus the
PNG writer and duration formatting (src/render.rs:218-244)."""
import io

import numpy as np
import pytest
from PIL import Image

from raingun_amd.cli import encode_png, format_duration, parse_arguments


def test_it_parses_resolution_arguments():  # main.rs:143-169
    o = parse_arguments(["file"])
    assert (o.width, o.height) == (800, 600)
    o = parse_arguments(["--width", "640", "--height", "480", "file"])
    assert (o.width, o.height) == (640, 480)
    o = parse_arguments(["--hd", "file"])
    assert (o.width, o.height) == (1920, 1080)
    o = parse_arguments(["--hd", "--4k", "file"])
    assert (o.width, o.height) == (3840, 2160)
    o = parse_arguments(["--hd", "--width", "2000", "file"])
    assert (o.width, o.height) == (2000, 1080)


def test_it_parses_draft_argument():  # main.rs:171-178
    o = parse_arguments(["--hd", "--width", "2000", "--draft", "file"])
    assert (o.width, o.height) == (800, 600)
    assert o.max_recursion_depth == 4


def test_4k_then_hd_last_wins():
    o = parse_arguments(["--4k", "--hd", "file"])
    assert (o.width, o.height) == (1920, 1080)


def test_short_flags():
    o = parse_arguments(["-w", "320", "-h", "200", "file"])
    assert (o.width, o.height) == (320, 200)


def test_bad_width():
    with pytest.raises(SystemExit, match="Could not parse width"):
        parse_arguments(["--width", "wide", "file"])


def test_png_roundtrip():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, size=(37, 53, 4), dtype=np.uint8)
    back = np.asarray(Image.open(io.BytesIO(encode_png(img))).convert("RGBA"))
    assert np.array_equal(back, img)


@pytest.mark.parametrize("ms,want", [(0, "0ms"), (800, "800ms"), (801, "0.80s"), (12345, "12.35s"),
                                     (60000, "60.00s"), (61500, "1m 1.50s")])
def test_format_duration(ms, want):  # render.rs:229-244
    assert format_duration(ms) == want
