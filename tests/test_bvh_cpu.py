"""CPU check of the sphere BVH (raingun_amd/csrc/rg_bvh.cpp + the kernel's slab
test rg_bvh_ray.h): tests/native/bvh_sim.cpp traces primary, surface-origin,
grazing (r(1 +- 1e-9), r(1 +- 1e-13)) and far-origin rays (up to 1e5 x the
scene, through the clipped-start path of rg_bvh_classify) through the BVH and
through the brute-force reference scan; closest hits (t bits, YAML index) and
shadow any-hit answers must agree on every ray, for both the wave-coherent walk
and the per-lane nearest-first walk (bounded stack, pruning at pop).  A negative control shrinks the
boxes and must be caught."""
import json
import os
import subprocess
from pathlib import Path

import pytest

from raingun_amd import synth
from raingun_amd._host import LoadedScene

REPO = Path(__file__).resolve().parent.parent
SRC = [REPO / "tests" / "native" / "bvh_sim.cpp", REPO / "raingun_amd" / "csrc" / "rg_bvh.cpp"]


def _build(tmp_path_factory, extra=()):
    out = tmp_path_factory.mktemp("bvh") / "bvh_sim"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", *extra, "-o", str(out), *map(str, SRC)],
                   check=True)
    return out


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    return _build(tmp_path_factory)


def _spheres(*args):
    ls = LoadedScene.from_string(synth.synthetic_yaml(*args))
    d = ls.desc
    sp = [tuple(d.bodies[i].p[:4]) for i in range(d.n_bodies) if d.bodies[i].kind == 0]
    ls.close()
    return f"{len(sp)}\n" + "\n".join(" ".join(repr(float(v)) for v in p) for p in sp) + "\n"


def _run(exe, text, rays=6000, env=None):
    r = subprocess.run([str(exe), str(rays)], input=text, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **(env or {})))
    return r.returncode, (json.loads(r.stdout) if r.stdout.strip() else None), r.stderr


@pytest.mark.parametrize("args", [(16,), (64,), (1024,), (4096, 8)])
def test_bvh_matches_brute_force(sim, args):
    rc, res, err = _run(sim, _spheres(*args))
    assert rc == 0, err
    assert res["mismatches"] == 0
    assert res["hits"] > 0 and res["occluded"] > 0 and res["fallback"] > 0
    assert res["shifted"] > 1000 and res["no_sphere"] > 1000  # far origins: clipped start / skipped
    assert res["grown"] > 100  # very far origins: boxes grown by the exact test's slack
    if args[0] >= 1024:  # the point of the structure: a handful of exact tests per ray
        assert res["exact_tests_per_ray"] < 16 and res["nodes_per_ray"] < 16
        assert res["lane_steps_per_ray"] < 16  # the per-lane nearest-first walk prunes as well
    # the per-lane walk's stack stays within the bound the host sizes it to
    assert 0 < res["lane_stack_used"] <= res["lane_stack"] <= 16


def test_degenerate_and_clustered_spheres(sim):
    # identical centres (no SAH split possible), a tight cluster and a far outlier
    lines = ["0 0 -10 1"] * 40 + [f"{0.001 * i} 0 -20 0.5" for i in range(40)] + ["500 500 -900 30"]
    rc, res, err = _run(sim, f"{len(lines)}\n" + "\n".join(lines) + "\n")
    assert rc == 0, err
    assert res["mismatches"] == 0


def test_shrunken_boxes_are_caught(tmp_path_factory):
    exe = _build(tmp_path_factory, ["-DRG_BVH_MARGIN_ULPS=-200.0"])
    rc, res, _ = _run(exe, _spheres(1024), env={"BVH_SIM_SKIP_STRUCT": "1"})
    assert rc == 1 and res["mismatches"] > 0
