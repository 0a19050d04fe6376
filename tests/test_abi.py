"""The C-ABI library loads and exports every function include/raingun.h
declares (no compute calls: this runs without a GPU)."""
import re
import subprocess
from pathlib import Path

import pytest

from raingun_amd import _abi

INCLUDE = Path(__file__).resolve().parent.parent / "include"
HEADER = INCLUDE / "raingun.h"


def declared_functions(header=HEADER):
    text = re.sub(r"/\*.*?\*/", "", header.read_text(), flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*(rg_[a-z0-9_]+)\s*\(", text, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def libpath():
    if not _abi.LIB_PATH.exists():
        subprocess.run(["make", "-s", "-C", str(_abi.PKG_DIR / "csrc")], check=True)
    return _abi.LIB_PATH


def test_header_matches_binding_table():
    assert declared_functions() == sorted(_abi.EXPORTED_SYMBOLS)
    assert declared_functions(INCLUDE / "raingun_debug.h") == sorted(_abi.DEBUG_SYMBOLS)
    assert declared_functions(INCLUDE / "raingun_frames.h") == sorted(_abi.FRAMES_SYMBOLS)


def test_library_exports_every_symbol(libpath):
    out = subprocess.run(["nm", "-D", "--defined-only", str(libpath)], capture_output=True, text=True,
                         check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    declared = (declared_functions() + declared_functions(INCLUDE / "raingun_debug.h")
                + declared_functions(INCLUDE / "raingun_frames.h"))
    missing = [s for s in declared if s not in exported]
    assert not missing, missing


def test_library_loads_and_answers_host_only_calls(libpath):
    lib = _abi.lib()
    assert lib.rg_abi_version() == 1
    assert lib.rg_status_string(_abi.RG_ERR_PORTRAIT).decode().startswith("width must be")
    t = _abi.rg_tiling(16, 3, 1)
    import ctypes as C
    assert lib.rg_tiling_rows(600, C.byref(t)) == 16 * len(range(1, 38, 3))
    bad = _abi.rg_tiling(16, 3, 3)
    assert lib.rg_tiling_rows(600, C.byref(bad)) == 0
    assert lib.rg_device_count() >= 0


def test_invalid_arguments_fail_loudly(libpath):
    import ctypes as C
    lib = _abi.lib()
    assert lib.rg_scene_create(None, 0, None) == _abi.RG_ERR_INVALID_ARGUMENT
    assert lib.rg_render_image(None, 8, 8, None, None) == _abi.RG_ERR_INVALID_ARGUMENT
    assert lib.rg_trace(None, None, 1, None, None) == _abi.RG_ERR_INVALID_ARGUMENT
    out = C.c_void_p(7)
    assert lib.rg_frames_create(None, 8, 8, 16, 0, 1, 2, None, None, C.byref(out)) == _abi.RG_ERR_INVALID_ARGUMENT
    assert out.value is None
    assert lib.rg_frames_step(None) == _abi.RG_ERR_INVALID_ARGUMENT
    assert lib.rg_frames_image(None) is None
    px = C.c_int32(5)
    assert lib.rg_frames_status(None, C.byref(px)) == _abi.RG_ERR_INVALID_ARGUMENT
    assert lib.rg_frames_read_image(None, None) == _abi.RG_ERR_INVALID_ARGUMENT
    assert lib.rg_frames_flush(None) == _abi.RG_ERR_INVALID_ARGUMENT


def test_comm_entry_points_validate_arguments(libpath):
    """The library's own RCCL communicator (raingun_frames.h rg_comm_*): argument
    errors come back as status codes before any RCCL or HIP call."""
    import ctypes as C
    lib = _abi.lib()
    assert lib.rg_comm_id_bytes() == 128
    assert lib.rg_comm_unique_id(None) == _abi.RG_ERR_INVALID_ARGUMENT
    uid = (C.c_uint8 * 128)()
    comm = C.c_void_p(9)
    assert lib.rg_comm_init_rank(None, 2, 0, 0, C.byref(comm)) == _abi.RG_ERR_INVALID_ARGUMENT
    assert comm.value is None  # cleared on every failure
    for world, rank, dev in ((0, 0, 0), (2, 2, 0), (2, -1, 0), (2, 0, -1)):
        assert lib.rg_comm_init_rank(uid, world, rank, dev, C.byref(comm)) == _abi.RG_ERR_INVALID_ARGUMENT
    assert lib.rg_comm_init_rank(uid, 1, 0, 0, None) == _abi.RG_ERR_INVALID_ARGUMENT
    assert lib.rg_comm_info(None, None, None, None) == _abi.RG_ERR_INVALID_ARGUMENT
    assert lib.rg_comm_destroy(None) == _abi.RG_ERR_INVALID_ARGUMENT


def test_struct_sizes_match_header():
    import ctypes as C
    # rg_body: kind, pad, 7 doubles, material (12 x 4 B)
    assert C.sizeof(_abi.rg_material) == 48
    assert C.sizeof(_abi.rg_body) == 8 + 56 + 48
    assert C.sizeof(_abi.rg_light) == 24 + 24
    assert C.sizeof(_abi.rg_stats) == 24 + 16
