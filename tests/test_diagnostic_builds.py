"""The render kernel's diagnostic builds still compile (CPU, no GPU needed).

rg_kernels.hip keeps four default-off diagnostic switches (per-tile and per-wave
timelines, per-iteration SIMD-use counters, BVH statistics) that scripts under
scripts/ build into variant libraries for profiling sessions.  Every other
default-off experiment was removed; these must not rot, so each
one is compiled here (hipcc semantic analysis of the whole translation unit,
every template instantiation included, for gfx950)."""
import shutil
import subprocess
from pathlib import Path

import pytest

CSRC = Path(__file__).resolve().parent.parent / "raingun_amd" / "csrc"
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(shutil.which(HIPCC) is None and not Path(HIPCC).exists(), reason="hipcc not installed")
@pytest.mark.parametrize("flag", ["", "-DRG_TILE_TIMES", "-DRG_WAVE_TIMES", "-DRG_ITER_STATS", "-DRG_BVH_STATS",
                                  "-DRG_REGION_STATS"])
def test_diagnostic_build_compiles(flag):
    cmd = [HIPCC, "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fsyntax-only", "-Werror=return-type",
           "rg_kernels.hip"]
    if flag:
        cmd.append(flag)
    r = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert " error:" not in r.stderr, r.stderr[-3000:]
