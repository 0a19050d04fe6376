"""Colour, mirroring raingun-lib/src/color.rs.

f32 RGB.  Parsing follows `FromStr` (color.rs:114-130): exactly "#rrggbb",
each channel `(byte as f32) / 255.0` in f32.  Display follows color.rs:52-60:
`floor(c * 255)` per channel, formatted as lower-case hex.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32


class Color:
    __slots__ = ("red", "green", "blue")

    def __init__(self, red: float, green: float, blue: float):
        self.red = F32(red)
        self.green = F32(green)
        self.blue = F32(blue)

    # color.rs:22-24
    @staticmethod
    def black() -> "Color":
        return Color(0.0, 0.0, 0.0)

    # color.rs:114-130
    @staticmethod
    def from_str(s: str) -> "Color":
        if isinstance(s, str) and len(s) == len("#123456") and s.startswith("#"):
            digits = s[1:]
            # u64::from_str_radix(.., 16): hex digits only (a leading '+' is also accepted by Rust)
            body = digits[1:] if digits.startswith("+") else digits
            if body and all(ch in "0123456789abcdefABCDEF" for ch in body):
                num = int(body, 16)
                red = F32((num & 0xFF0000) >> 16)
                grn = F32((num & 0x00FF00) >> 8)
                blu = F32(num & 0x0000FF)
                d = F32(255.0)
                return Color(red / d, grn / d, blu / d)
        raise ValueError(f"{s} is not a valid color")

    # color.rs:26-30
    @staticmethod
    def from_rgba(rgba) -> "Color":
        d = F32(255.0)
        return Color(F32(rgba[0]) / d, F32(rgba[1]) / d, F32(rgba[2]) / d)

    # color.rs:32-37 (`as u8` saturating, NaN -> 0)
    def rgba(self) -> tuple:
        return (_to_u8(self.red * F32(255.0)), _to_u8(self.green * F32(255.0)), _to_u8(self.blue * F32(255.0)), 255)

    # color.rs:39-43
    def clamp(self) -> "Color":
        return Color(*(_clamp01(c) for c in (self.red, self.green, self.blue)))

    def __add__(self, o: "Color") -> "Color":
        return Color(self.red + o.red, self.green + o.green, self.blue + o.blue)

    def __mul__(self, o) -> "Color":
        if isinstance(o, Color):
            return Color(self.red * o.red, self.green * o.green, self.blue * o.blue)
        s = F32(o)
        return Color(self.red * s, self.green * s, self.blue * s)

    def __eq__(self, o) -> bool:
        return isinstance(o, Color) and (self.red, self.green, self.blue) == (o.red, o.green, o.blue)

    def __repr__(self) -> str:
        return f"Color({float(self.red)!r}, {float(self.green)!r}, {float(self.blue)!r})"

    # color.rs:52-60: floor(c as f32 * 255.0) as u8
    def __str__(self) -> str:
        return "#" + "".join(f"{_to_u8(F32(math.floor(F32(c) * F32(255.0)))):02x}"
                             for c in (self.red, self.green, self.blue))

    def as_tuple(self) -> tuple:
        return (float(self.red), float(self.green), float(self.blue))


def _to_u8(v) -> int:
    v = float(v)
    if not v > 0.0:
        return 0
    if v >= 255.0:
        return 255
    return int(v)


def _clamp01(v):
    v = F32(v)
    # f32::min(1.0) then f32::max(0.0); both ignore a NaN operand
    m = F32(1.0) if (np.isnan(v) or v > 1.0) else v
    return F32(0.0) if m < 0.0 else m
