"""Colour KATs: the reference's own unit tests (raingun-lib/src/color.rs:162-203)
plus the quantisation rules the render path relies on (color.rs:26-43)."""
import numpy as np
import pytest

from raingun_amd.color import Color


def test_it_parses_strings():  # color.rs:162-185
    assert Color.from_str("#000000") == Color(0.0, 0.0, 0.0)
    assert Color.from_str("#ffffff") == Color(1.0, 1.0, 1.0)
    assert Color.from_str("#ff7f11") == Color(1.0, 0.498039216, 0.066666667)


def test_it_displays_strings():  # color.rs:187-191
    assert str(Color.black()) == "#000000"
    assert str(Color(1.0, 0.5, 0.0)) == "#ff7f00"


@pytest.mark.parametrize("sample", ["#000000", "#123456", "#ffeecc", "#fef0fa", "#010203"])
def test_it_returns_same_color_as_input(sample):  # color.rs:193-203 (made non-tautological)
    assert str(Color.from_str(sample)) == sample


@pytest.mark.parametrize("bad", ["#12345", "123456", "#12345g", "#1234567", "", None, "#-12345"])
def test_rejects_invalid(bad):
    with pytest.raises(ValueError):
        Color.from_str(bad)


def test_parse_is_f32_division():
    c = Color.from_str("#7f0001")
    assert c.red == np.float32(127) / np.float32(255)
    assert c.blue == np.float32(1) / np.float32(255)


def test_rgba_truncates_and_saturates():  # color.rs:32-37 (`as u8`)
    assert Color(1.0, 0.5, 0.0).rgba() == (255, 127, 0, 255)
    assert Color(2.0, -1.0, float("nan")).rgba() == (255, 0, 0, 255)
    assert Color(0.999, 0.0039215, 0.0039216).rgba() == (254, 0, 1, 255)


def test_clamp():  # color.rs:39-43 (f32::min/max ignore NaN -> NaN clamps to 1)
    c = Color(1.5, -0.25, float("nan")).clamp()
    assert (float(c.red), float(c.green), float(c.blue)) == (1.0, 0.0, 1.0)


def test_ops_are_f32():
    a, b = Color(0.1, 0.2, 0.3), Color(0.7, 0.11, 0.5)
    assert (a + b).red == np.float32(0.1) + np.float32(0.7)
    assert (a * b).green == np.float32(0.2) * np.float32(0.11)
    assert (a * 3.0).blue == np.float32(0.3) * np.float32(3.0)
