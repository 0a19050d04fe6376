"""Host-code sanitizers (CPU): the native host layer's parsers (YAML scene
loader, JPEG decoder in both rounding flavours, PNG codec) and the CPU
restatement, built with -fsanitize=address,undefined (leak checking on,
every report fatal) and driven over the reference's fixtures and over
truncated / byte-flipped copies of them (tests/native/sanitize_host.cpp).
GPU code is out of reach: GPU AddressSanitizer is not available on this pool.
"""
import json
import shutil
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
HOST = REPO / "raingun_amd" / "host"
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1",
       "-ffp-contract=off", "-fwrapv", f"-I{REPO / 'include'}"]


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if shutil.which("g++") is None or shutil.which("gcc") is None:
        pytest.skip("no host compiler")
    d = tmp_path_factory.mktemp("sanitize")
    srcs = [REPO / "tests" / "native" / "sanitize_host.cpp"] + [HOST / f for f in
                                                                ("yaml.cpp", "jpeg_decode.cpp", "png_codec.cpp",
                                                                 "scene_loader.cpp")]
    subprocess.run(["g++", "-std=c++17", *SAN, "-c", *map(str, srcs)], cwd=d, check=True)
    subprocess.run(["gcc", "-std=c11", *SAN, "-c", str(REPO / "oracle" / "raingun_oracle.c")], cwd=d, check=True)
    exe = d / "sanitize_host"
    subprocess.run(["g++", "-fsanitize=address,undefined", "-o", str(exe), *map(str, sorted(d.glob("*.o"))),
                    "-lz", "-lm", "-pthread"], check=True)
    return exe


def test_host_parsers_and_oracle_under_asan_ubsan(harness):
    p = subprocess.run([str(harness), str(REPO / "tests" / "golden"), "40"], capture_output=True, text=True,
                       timeout=600, env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                         "UBSAN_OPTIONS": "print_stacktrace=1", "PATH": "/usr/bin:/bin"})
    assert p.returncode == 0, p.stderr[-4000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["fixtures"] == 9
    assert res["mutants_rejected"] > 0 and res["mutants_accepted"] > 0
