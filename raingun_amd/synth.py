"""Synthetic N-sphere scenes in the reference's YAML schema.

The reference ships no synthetic scenes; BASELINE.json's configs C4/C5 name
"1024 spheres" and "4096 spheres + 8 planes".  This generator is the committed
definition: a SplitMix64 stream (seed 0x5EED) drives every choice, floats are
emitted with repr() (shortest round-trip), so the YAML -> f64 values are exact
and the scene is identical on every machine.  `python -m raingun_amd.synth N`
prints the YAML; `scene_md5` identifies it in bench output.
"""
from __future__ import annotations

import hashlib
import sys

SEED = 0x5EED
MASK64 = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed: int = SEED):
        self.state = seed & MASK64

    def next_u64(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def uniform(self, lo: float, hi: float) -> float:
        # 53-bit mantissa in [0,1), then scale; rounded to 6 decimals so the YAML is readable
        u = (self.next_u64() >> 11) * (1.0 / (1 << 53))
        return round(lo + (hi - lo) * u, 6)

    def below(self, n: int) -> int:
        return self.next_u64() % n


def _vec(v) -> str:
    return "[" + ", ".join(repr(float(c)) for c in v) + "]"


def synthetic_yaml(n_spheres: int = 1024, n_planes: int = 2, max_depth: int = 5, seed: int = SEED) -> str:
    """Spheres: centre x in [-24,24], y in [-1.5,14], z in [-90,-8], radius in [0.25,1.25];
    material mix 60% Diffuse (random colour, albedo 0.18-0.9), 25% Reflecting (0.2-0.8),
    15% Refractive (index 1.1-1.6, transparency 0.8).  Planes: floor + back wall, then up to
    6 more one-sided planes (ceiling, side walls, three far walls).  Lights: 1 directional +
    2 spherical.  defaultColor #334466, fov 90."""
    rng = SplitMix64(seed)
    out = ["---", 'defaultColor: "#334466"', "fov: 90.0", f"maxRecursionDepth: {int(max_depth)}", "lights:",
           "  - Directional:", "      direction: [0.4, -1.0, -0.9]", '      color: "#ffffee"',
           "      intensity: 7.0",
           "  - Spherical:", "      position: [-6.0, 12.0, -20.0]", '      color: "#ee7700"',
           "      intensity: 40000.0",
           "  - Spherical:", "      position: [18.0, 20.0, -50.0]", '      color: "#ffffee"',
           "      intensity: 90000.0",
           "bodies:"]
    planes = [
        ((0.0, -2.0, 0.0), (0.0, -1.0, 0.0), "#c8c8b4", 0.18),      # floor
        ((0.0, 0.0, -100.0), (0.0, 0.0, -1.0), "#6677ff", 0.9),     # back wall
        ((0.0, 40.0, 0.0), (0.0, 1.0, 0.0), "#ffffff", 0.5),        # ceiling
        ((-60.0, 0.0, 0.0), (-1.0, 0.0, 0.0), "#ff8888", 0.5),      # left wall
        ((60.0, 0.0, 0.0), (1.0, 0.0, 0.0), "#88ff88", 0.5),        # right wall
        ((0.0, 0.0, -110.0), (0.1, 0.0, -1.0), "#8888ff", 0.5),     # far walls (behind the back wall)
        ((0.0, 0.0, -120.0), (-0.1, 0.0, -1.0), "#ffff88", 0.5),
        ((0.0, 0.0, -130.0), (0.0, 0.1, -1.0), "#88ffff", 0.5),
    ]
    for origin, normal, col, albedo in planes[:max(0, min(n_planes, len(planes)))]:
        out += ["  - Plane:", f"      origin: {_vec(origin)}", f"      normal: {_vec(normal)}", "      material:",
                "        coloration:", f'          Color: "{col}"', f"        albedo: {albedo!r}",
                "        surface: Diffuse"]
    for _ in range(n_spheres):
        c = (rng.uniform(-24.0, 24.0), rng.uniform(-1.5, 14.0), rng.uniform(-90.0, -8.0))
        r = rng.uniform(0.25, 1.25)
        kind = rng.below(100)
        col = "#%06x" % (rng.next_u64() & 0xFFFFFF)
        albedo = rng.uniform(0.18, 0.9)
        out += ["  - Sphere:", f"      center: {_vec(c)}", f"      radius: {r!r}", "      material:",
                "        coloration:", f'          Color: "{col}"', f"        albedo: {albedo!r}"]
        if kind < 60:
            out += ["        surface: Diffuse"]
        elif kind < 85:
            out += ["        surface:", "          Reflecting:", f"            reflectivity: {rng.uniform(0.2, 0.8)!r}"]
        else:
            out += ["        surface:", "          Refractive:", f"            index: {rng.uniform(1.1, 1.6)!r}",
                    "            transparency: 0.8"]
    return "\n".join(out) + "\n"


def scene_md5(text: str) -> str:
    return hashlib.md5(text.encode()).hexdigest()


def synthetic_scene(n_spheres: int = 1024, n_planes: int = 2, max_depth: int = 5, seed: int = SEED):
    from .scene import load_scene

    return load_scene(synthetic_yaml(n_spheres, n_planes, max_depth, seed))


if __name__ == "__main__":  # pragma: no cover
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    p = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    d = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    sys.stdout.write(synthetic_yaml(n, p, d))
