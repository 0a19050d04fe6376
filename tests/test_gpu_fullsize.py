"""BASELINE configs[3] and configs[4] at their full sizes, on one GPU.

The CPU restatement cannot render 33 M or 268 M pixels in test time, so the
full frames are checked through properties that hold at any size, and against
the oracle on a sample of row tiles:

* the frame rendered as N interleaved row-tile partitions (the N-rank split of
  bench.py / raingun_amd.distributed) and re-assembled equals the one-launch
  frame byte for byte, and the partitions' ray counts add up exactly to the
  frame's (a checksum of checksums);
* sampled 16-row tiles of the full frame equal the CPU restatement's render of
  the same tiles byte for byte, with exactly equal per-class ray counts.
"""
import ctypes as C

import numpy as np
import pytest

from raingun_amd import _abi
from raingun_amd import distributed as rd
from raingun_amd.scene import DeviceScene, SceneDesc
from raingun_amd.synth import synthetic_scene

pytestmark = pytest.mark.gpu
T = 16


def _render(ds, w, h, tiling, torch):
    lib = _abi.lib()
    rows = lib.rg_tiling_rows(h, C.byref(tiling))
    buf = torch.empty((rows, w, 4), dtype=torch.uint8, device="cuda")
    st = _abi.rg_stats()
    _abi.check(lib.rg_render_tiles_async(ds.handle, w, h, C.byref(tiling), C.c_void_p(buf.data_ptr()), None, None,
                                         C.byref(st)), "rg_render_tiles_async")
    return buf, st.rays.as_dict()


def _full_size_check(oracle_lib, scene, w, h, ranks, sample_stride, sample_offset):
    import torch

    ds = DeviceScene(scene)
    frame, counts = _render(ds, w, h, _abi.rg_tiling(h, 1, 0), torch)
    # N-rank split, assembled as rank 0 does after the gather
    parts, total = [], {"primary": 0, "shadow": 0, "secondary": 0}
    slot = rd.slot_rows(h, ranks, T)
    for r in range(ranks):
        p, c = _render(ds, w, h, _abi.rg_tiling(T, ranks, r), torch)
        padded = torch.zeros((slot, w, 4), dtype=torch.uint8, device="cuda")
        padded[:p.shape[0]] = p
        parts.append(padded)
        for k in total:
            total[k] += c[k]
    assembled = rd.assemble(parts, h, ranks, T)
    assert torch.equal(assembled, frame), "assembled partitions differ from the one-launch frame"
    assert total == counts, (total, counts)
    del parts, assembled
    # sampled tiles against the CPU restatement
    sample, s_counts = _render(ds, w, h, _abi.rg_tiling(T, sample_stride, sample_offset), torch)
    ds.close()
    o_st, o_rgba, _, o_counts, _ = oracle_lib.render(SceneDesc(scene), w, h, T, sample_stride, sample_offset)
    assert o_st == 0
    assert s_counts == o_counts
    got = sample.cpu().numpy()
    assert np.array_equal(got[:o_rgba.shape[0]], o_rgba)
    # and the sampled tiles are the frame's own rows
    tiles = range(sample_offset, (h + T - 1) // T, sample_stride)
    rows = torch.cat([frame[t * T:min((t + 1) * T, h)] for t in tiles])
    assert np.array_equal(rows.cpu().numpy(), o_rgba[:rows.shape[0]])
    return counts


def test_config4_north_star_8k_row_tiled_8_ways(oracle_lib):
    """configs[3]: synthetic 1024 spheres, 7680x4320, depth 5, row-tiled across 8 ranks."""
    counts = _full_size_check(oracle_lib, synthetic_scene(1024, 2, 5), 7680, 4320, 8, 27, 5)
    assert counts["primary"] == 7680 * 4320


def test_config5_4096_spheres_8_planes_16384_depth8(oracle_lib):
    """configs[4]: synthetic 4096 spheres + 8 planes, 16384x16384, depth 8 (the
    LDS-spill / stack-depth stress case: the sphere tables exceed the LDS
    budget, frame stacks of 7), split 8 ways."""
    counts = _full_size_check(oracle_lib, synthetic_scene(4096, 8, 8), 16384, 16384, 8, 128, 37)
    assert counts["primary"] == 16384 * 16384
