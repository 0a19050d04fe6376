"""The multi-GPU partition (raingun_amd/distributed.py) on CPU: world_size 2
and 3 gloo process groups, each rank renders its round-robin row tiles (with
the CPU restatement standing in for the GPU, so this runs without one), ONE
gather to rank 0, re-interleave -> byte-identical to the 1-rank frame."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from raingun_amd import distributed as rd


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, W, H, T, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from raingun_amd.scene import SceneDesc, load_scene
        from pathlib import Path
        g = Path(__file__).resolve().parent / "golden"
        desc = SceneDesc(load_scene(g / "examples" / "test2.yml", texture_root=g))
        slot = rd.slot_rows(H, world, T)

        def render_tiles(t):
            st, rgba, _, _, _ = oracle.render(desc, W, H, t.tile_rows, t.tile_stride, t.tile_offset, threads=2)
            assert st == 0
            buf = np.zeros((slot, W, 4), np.uint8)  # equal-size slots, zero-padded
            buf[:rgba.shape[0]] = rgba
            return torch.from_numpy(buf)

        frame = rd.render_frame(render_tiles, H, rank, world, T)
        if rank == 0:
            np.save(out_path, frame.numpy())
        else:
            assert frame is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,T", [(2, 16), (3, 8)])
def test_gloo_gather_reassembles_frame(oracle_lib, example_scenes, world, T, tmp_path):
    from raingun_amd.scene import SceneDesc
    W, H = 160, 120
    _, whole, _, _, _ = oracle_lib.render(SceneDesc(example_scenes["test2"]), W, H)
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), W, H, T, out), nprocs=world, join=True)
    frame = np.load(out)
    assert frame.shape == (H, W, 4)
    assert np.array_equal(frame, whole)


def test_assemble_index_math():
    H, world, T = 50, 3, 8
    tiles = rd.n_tiles(H, T)
    img = np.arange(H)[:, None, None].repeat(2, 1).repeat(1, 2)
    parts = []
    for r in range(world):
        buf = np.full((rd.slot_rows(H, world, T), 2, 1), -1)
        for j, t in enumerate(rd.rank_tiles(H, r, world, T)):
            rows = img[t * T:(t + 1) * T]
            buf[j * T:j * T + rows.shape[0]] = rows
        parts.append(buf)
    assert np.array_equal(rd.assemble(parts, H, world, T), img)
    tparts = [torch.from_numpy(p) for p in parts]
    assert torch.equal(rd.assemble(tparts, H, world, T), torch.from_numpy(img))
    assert tiles == 7 and rd.tiles_per_rank(H, world, T) == 3


@pytest.mark.parametrize("world,root", [(2, 2), (3, 2), (3, 4), (8, 2), (8, 3)])
def test_root_share_index_math(world, root):
    """Rank 0's share: periods of root + world - 1 tiles, the first `root` to
    rank 0.  Every image tile belongs to exactly one rank, the other ranks' slots are equal up to
    one tile, rank 0's tilings interleave to its tile list, and assemble() restores the image."""
    H, T = 203, 8
    tiles = rd.n_tiles(H, T)
    owned = sorted(t for r in range(world) for t in rd.rank_tiles(H, r, world, T, root))
    assert owned == list(range(tiles))
    counts = [len(rd.rank_tiles(H, r, world, T, root)) for r in range(1, world)]
    assert max(counts) - min(counts) <= 1 and rd.root_slot_rows(H, world, T, root) == max(counts) * T
    P = root + world - 1
    ts = rd.tilings(0, world, T, root)
    assert [(t.tile_stride, t.tile_offset) for t in ts] == [(P, j) for j in range(root)]
    inter = []
    for p in range(tiles // P + 1):
        inter += [p * P + t.tile_offset for t in ts if p * P + t.tile_offset < tiles]
    assert inter == rd.rank_tiles(H, 0, world, T, root)
    img = np.arange(H)[:, None, None].repeat(3, 1).repeat(1, 2)
    parts = []
    for r in range(world):
        mine = rd.rank_tiles(H, r, world, T, root)
        rows = len(mine) * T if r == 0 else rd.root_slot_rows(H, world, T, root)
        buf = np.full((rows, 3, 1), -1)
        for j, t in enumerate(mine):
            blk = img[t * T:(t + 1) * T]
            buf[j * T:j * T + blk.shape[0]] = blk
        parts.append(buf)
    assert np.array_equal(rd.assemble(parts, H, world, T, root), img)
    assert torch.equal(rd.assemble([torch.from_numpy(p) for p in parts], H, world, T, root), torch.from_numpy(img))


def _root_worker(rank, world, root, port, W, H, T, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from raingun_amd.scene import SceneDesc, load_scene
        from pathlib import Path
        g = Path(__file__).resolve().parent / "golden"
        desc = SceneDesc(load_scene(g / "examples" / "test2.yml", texture_root=g))
        slot = max(rd.root_slot_rows(H, world, T, root), len(rd.rank_tiles(H, 0, world, T, root)) * T)

        def render_tiles(t):
            st, rgba, _, _, _ = oracle.render(desc, W, H, t.tile_rows, t.tile_stride, t.tile_offset, threads=2)
            assert st == 0
            buf = np.zeros((slot, W, 4), np.uint8)
            buf[:rgba.shape[0]] = rgba
            return torch.from_numpy(buf)

        frame = rd.render_frame(render_tiles, H, rank, world, T, root=root)
        if rank == 0:
            np.save(out_path, frame.numpy())
        else:
            assert frame is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,root,T", [(2, 2, 8), (3, 3, 16)])
def test_gloo_gather_root_share(oracle_lib, example_scenes, world, root, T, tmp_path):
    """World 2/3 over gloo with rank 0's share > 1: rank 0 renders its `root` tiles per period (its
    strided tilings, interleaved), the others one each; ONE gather of the others' equal slots;
    the assembled frame equals the 1-rank render."""
    from raingun_amd.scene import SceneDesc
    W, H = 160, 117
    _, whole, _, _, _ = oracle_lib.render(SceneDesc(example_scenes["test2"]), W, H)
    out = str(tmp_path / "frame.npy")
    mp.spawn(_root_worker, args=(world, root, _free_port(), W, H, T, out), nprocs=world, join=True)
    assert np.array_equal(np.load(out), whole)


def _pipe_worker(rank, world, port, W, H, T, K, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from raingun_amd.scene import SceneDesc, load_scene
        from pathlib import Path
        g = Path(__file__).resolve().parent / "golden"
        desc = SceneDesc(load_scene(g / "examples" / "test2.yml", texture_root=g))
        t = rd.tiling(rank, world, T)
        st, rgba, _, _, _ = oracle.render(desc, W, H, t.tile_rows, t.tile_stride, t.tile_offset, threads=2)
        assert st == 0
        got = {}
        pipe = rd.FramePipeline((rd.slot_rows(H, world, T), W, 4), H, rank, world, T, device=None,
                                on_frame=lambda k, f: got.__setitem__(k, f.numpy().copy()))
        for k in range(K):
            def render(part, k=k):  # frame k: the rank's tiles with every byte offset by k
                part.zero_()
                part[:rgba.shape[0]] = torch.from_numpy((rgba.astype(np.int32) + k).astype(np.uint8))
            pipe.step(render)
        pipe.flush()
        if rank == 0:
            np.save(out_path, np.stack([got[k] for k in range(K)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,T", [(2, 16), (3, 8)])
def test_frame_pipeline_gathers_every_frame(oracle_lib, example_scenes, world, T, tmp_path):
    """The multi-frame pipeline (double-buffered parts, async gather, re-interleave
    into the padded frame) delivers each frame k intact and in order."""
    from raingun_amd.scene import SceneDesc
    W, H, K = 96, 70, 5
    _, whole, _, _, _ = oracle_lib.render(SceneDesc(example_scenes["test2"]), W, H)
    out = str(tmp_path / "frames.npy")
    mp.spawn(_pipe_worker, args=(world, _free_port(), W, H, T, K, out), nprocs=world, join=True)
    frames = np.load(out)
    for k in range(K):
        assert np.array_equal(frames[k], (whole.astype(np.int32) + k).astype(np.uint8)), k


def test_assemble_into_matches_assemble():
    H, world, T, W = 50, 3, 8, 5
    slot = rd.slot_rows(H, world, T)
    g = torch.randint(0, 255, (world, slot, W, 4), dtype=torch.uint8)
    fp = torch.empty((world * slot, W, 4), dtype=torch.uint8)
    rd.assemble_into(fp, g, world, T)
    assert torch.equal(fp[:H], rd.assemble(list(g.unbind(0)), H, world, T))


def test_frame_pipeline_single_rank_needs_no_collective():
    """At N = 1 the pipeline only rotates render buffers (no process group, no
    gather): frame k is the part it rendered, delivered in order."""
    H, W, T, K, depth = 40, 6, 16, 7, 3
    slot = rd.slot_rows(H, 1, T)
    got = {}
    pipe = rd.FramePipeline((slot, W, 4), H, 0, 1, T, depth=depth, on_frame=lambda k, f: got.__setitem__(k, f.clone()))
    for k in range(K):
        pipe.step(lambda part, k=k: part.fill_(k))
        assert pipe.frame.shape == (H, W, 4) and int(pipe.frame[0, 0, 0]) == k
    pipe.flush()
    assert sorted(got) == list(range(K))
    for k in range(K):
        assert bool((got[k] == k).all())


class _FakeCommLib:
    """Stands in for libraingun_hip.so's rg_comm_* entry points (no GPU, no RCCL)."""

    def __init__(self, fail_unique_id):
        self.fail = fail_unique_id
        self.init_calls = 0

    def rg_comm_init_rank(self, *a):
        self.init_calls += 1
        return 0

    def rg_comm_id_bytes(self):
        return 128

    def rg_comm_unique_id(self, uid):
        if self.fail:
            return -13  # RG_ERR_COLLECTIVE
        for i in range(len(uid)):
            uid[i] = (7 * i) & 0xFF
        return 0

    def rg_comm_gather_fn(self):
        return 1

    def rg_comm_destroy(self, h):
        return 0


def _comm_worker(rank, world, port, fail, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from raingun_amd import _abi
        fake = _FakeCommLib(fail)
        _abi.lib = lambda: fake  # this spawned process only
        try:
            c = rd.RcclComm(rank, world, 0)
            res = "ok" if fake.init_calls == 1 and c.gather_fn == 1 else "bad"
        except _abi.RaingunError as e:
            res = f"raised {e.status}" if hasattr(e, "status") else "raised"
        with open(os.path.join(out_dir, f"r{rank}"), "w") as f:
            f.write(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail", [False, True])
def test_rccl_comm_id_failure_raises_on_every_rank(fail, tmp_path):
    """rank 0's rg_comm_unique_id failing must not leave the other ranks blocked in the
    id broadcast -- the status travels with the id and every rank raises (gloo, world 3)."""
    world = 3
    mp.spawn(_comm_worker, args=(world, _free_port(), fail, str(tmp_path)), nprocs=world, join=True)
    res = [open(tmp_path / f"r{r}").read() for r in range(world)]
    if fail:
        assert all(r.startswith("raised") for r in res), res
    else:
        assert res == ["ok"] * world, res
