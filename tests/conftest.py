import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
GOLDEN = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def golden_dir() -> Path:
    return GOLDEN


@pytest.fixture(scope="session")
def example_scenes():
    """The reference's example scenes (examples/test{1,2,3}.yml) with textures
    resolved against tests/golden (the reference resolves them against the CWD,
    which is the repository root in examples/render-examples.sh)."""
    from raingun_amd.scene import load_scene

    return {t: load_scene(GOLDEN / "examples" / f"{t}.yml", texture_root=GOLDEN) for t in ("test1", "test2", "test3")}


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle

    oracle.build()
    return oracle
