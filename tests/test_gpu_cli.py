"""End to end on the GPU: both front ends render the reference's examples
exactly as its examples/render-examples.sh did (default 800x600, YAML depth),
and the PNGs they write are pixel-identical to the reference's golden
test{1,2,3}.png.  `raingun` is the native C++ binary (raingun_amd/bin/raingun,
main.rs:98-132); raingun_amd.cli is the Python mirror."""
import subprocess

import numpy as np
import pytest
from PIL import Image

from raingun_amd import _abi, _host
from raingun_amd.cli import main

pytestmark = pytest.mark.gpu


def _png(path):
    return np.asarray(Image.open(path).convert("RGBA"))


@pytest.fixture(scope="module")
def native_cli():
    if not _host.CLI_PATH.exists():
        subprocess.run(["make", "-s", "-C", str(_host.SRC_DIR)], check=True)
    return str(_host.CLI_PATH)


@pytest.mark.parametrize("name", ["test1", "test2", "test3"])
def test_native_cli_reproduces_golden(native_cli, golden_dir, tmp_path, name):
    out = tmp_path / f"{name}.png"
    # textures resolve against the working directory, as image::open does
    r = subprocess.run([native_cli, str(golden_dir / "examples" / f"{name}.yml"), "-o", str(out)],
                       cwd=golden_dir, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "\t→\t" in r.stdout and "render" in r.stdout and "write" in r.stdout
    assert np.array_equal(_png(out), _png(golden_dir / "examples" / f"{name}.png"))


def test_native_cli_default_output_name_and_draft(native_cli, golden_dir, tmp_path):
    yml = tmp_path / "scene.yml"
    yml.write_text((golden_dir / "examples" / "test2.yml").read_text())
    r = subprocess.run([native_cli, "--hd", "--draft", str(yml)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = tmp_path / "scene.png"  # PathBuf::set_extension("png") (main.rs:104-111)
    assert Image.open(out).size == (800, 600)
    r = subprocess.run([native_cli, "-w", "100", "-h", "200", str(yml)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 101 and "width must be" in r.stderr  # assert!(width >= height), ray.rs:42


def test_python_cli_renders_golden_test2(golden_dir, tmp_path, capsys):
    out = tmp_path / "test2.png"
    assert main([str(golden_dir / "examples" / "test2.yml"), "-o", str(out)]) == 0
    assert np.array_equal(_png(out), _png(golden_dir / "examples" / "test2.png"))
    line = capsys.readouterr().out
    assert "→" in line and "render" in line and "write" in line


def test_python_cli_draft_caps_depth(golden_dir, tmp_path):
    out = tmp_path / "d.png"
    assert main([str(golden_dir / "examples" / "test2.yml"), "--hd", "--draft", "-o", str(out)]) == 0
    assert Image.open(out).size == (800, 600)
