"""End to end on the GPU: the CLI renders examples/test2.yml exactly as the
reference's examples/render-examples.sh did (default 800x600, YAML depth), and
the PNG it writes is pixel-identical to the reference's golden test2.png."""
import numpy as np
import pytest
from PIL import Image

from raingun_amd.cli import main

pytestmark = pytest.mark.gpu


def test_cli_renders_golden_test2(golden_dir, tmp_path, capsys):
    out = tmp_path / "test2.png"
    assert main([str(golden_dir / "examples" / "test2.yml"), "-o", str(out)]) == 0
    got = np.asarray(Image.open(out).convert("RGBA"))
    gold = np.asarray(Image.open(golden_dir / "examples" / "test2.png").convert("RGBA"))
    assert np.array_equal(got, gold)
    line = capsys.readouterr().out
    assert "→" in line and "render" in line and "write" in line


def test_cli_draft_caps_depth(golden_dir, tmp_path):
    out = tmp_path / "d.png"
    assert main([str(golden_dir / "examples" / "test2.yml"), "--hd", "--draft", "-o", str(out)]) == 0
    assert Image.open(out).size == (800, 600)
