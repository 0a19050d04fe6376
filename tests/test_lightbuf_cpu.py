"""CPU check of the shadow-ray light buffers (raingun_amd/csrc/rg_lightbuf.cpp +
the kernel's cell lookup rg_lightbuf_ray.h): tests/native/lightbuf_sim.cpp
casts shadow rays from sphere surfaces (with the shadow bias), from random
points in and around the scene, and grazing rays that pass at r (1 +- 1e-9)
and r (1 +- 1e-13) from a sphere's centre, towards directional and spherical
lights, and compares the any-hit answer of each ray's cell list with the
brute-force scan over every sphere.  A negative control drops the margins and
must be caught."""
import json
import subprocess
from pathlib import Path

import pytest

from raingun_amd import synth
from raingun_amd._host import LoadedScene

REPO = Path(__file__).resolve().parent.parent
SRC = [REPO / "tests" / "native" / "lightbuf_sim.cpp", REPO / "raingun_amd" / "csrc" / "rg_lightbuf.cpp",
       REPO / "raingun_amd" / "csrc" / "rg_bvh.cpp"]


def _build(tmp_path_factory, extra=()):
    out = tmp_path_factory.mktemp("lb") / "lightbuf_sim"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", *extra, "-o", str(out), *map(str, SRC)],
                   check=True)
    return out


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    return _build(tmp_path_factory)


def _scene_text(*args, extra_lights=()):
    ls = LoadedScene.from_string(synth.synthetic_yaml(*args))
    d = ls.desc
    sp = [tuple(d.bodies[i].p[:4]) for i in range(d.n_bodies) if d.bodies[i].kind == 0]
    lights = [(d.lights[i].kind, tuple(d.lights[i].v)) for i in range(d.n_lights)]
    ls.close()
    lights += list(extra_lights)
    lines = [str(len(sp))] + [" ".join(repr(float(v)) for v in p) for p in sp]
    lines += [str(len(lights))] + [f"{k} " + " ".join(repr(float(x)) for x in v) for k, v in lights]
    return "\n".join(lines) + "\n"


def _run(exe, text, rays=3000):
    r = subprocess.run([str(exe), str(rays)], input=text, capture_output=True, text=True, timeout=600)
    return r.returncode, (json.loads(r.stdout) if r.stdout.strip() else None), r.stderr


# extra lights: a point light inside the sphere field, one far away, an axis-aligned and an
# oblique directional light (the synthetic scenes bring one directional and two spherical lights)
EXTRA = ((1, (0.5, 4.0, -40.0)), (1, (300.0, 500.0, 200.0)), (0, (0.0, -1.0, 0.0)), (0, (-0.3, -0.2, 1.0)))


@pytest.mark.parametrize("args", [(16,), (256,), (1024,), (4096, 8)])
def test_lightbuf_matches_brute_force(sim, args):
    rc, res, err = _run(sim, _scene_text(*args, extra_lights=EXTRA))
    assert rc == 0, err
    assert res["mismatches"] == 0 and res["camera_mismatches"] == 0
    assert res["lights_built"] >= 5 and res["camera_built"] == 1
    assert res["camera_hits"] > 1000
    assert res["occluded"] > 1000 and res["grazing"] > 1000 and res["empty_cells"] > 100
    if args[0] >= 1024:  # the point of the structure: few exact tests per shadow ray
        assert res["tests_per_ray"] < 16 and res["camera_tests_per_ray"] < 16


def test_light_inside_a_sphere(sim):
    # a point light inside sphere 0 and another exactly on a sphere's surface: the always list
    # (plus 17 small spheres around them: the buffers, like the BVH, are built for >= 16 spheres)
    sph = ["0 0 -10 2", "5 0 -10 1", "0 5 -12 1.5"] + [f"{-8 + i} {(-1) ** i * 3} {-14 - i % 3} 0.4" for i in range(17)]
    lines = [str(len(sph))] + sph + ["2", "1 0.5 0 -10", "1 6 0 -10"]
    rc, res, err = _run(sim, "\n".join(lines) + "\n", rays=20000)
    assert rc == 0, err
    assert res["mismatches"] == 0 and res["occluded"] > 0


def test_dropped_margins_are_caught(tmp_path_factory):
    exe = _build(tmp_path_factory, ["-DRG_LB_TEST_NO_MARGIN"])
    rc, res, _ = _run(exe, _scene_text(1024, extra_lights=EXTRA), rays=4000)
    assert rc == 1 and res["mismatches"] > 0
