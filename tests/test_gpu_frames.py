"""The native frames-in-flight pipeline (include/raingun_frames.h) on one GPU:
a world-1 RCCL process group runs the same per-frame loop an N-GPU node runs
(render on stream k % depth, ncclGather on the communication stream, rank 0's
re-interleave on a side stream).  Every delivered frame must equal a one-shot
render byte for byte."""
import ctypes as C
import os
import socket

import numpy as np
import pytest

from raingun_amd import distributed as rd
from raingun_amd.scene import DeviceScene
from raingun_amd.synth import synthetic_scene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl_world1():
    import torch
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("scene_kind,w,h,depth", [("test1", 320, 240, 3), ("synth200", 256, 144, 4),
                                                  ("test1", 97, 61, 1)])
def test_native_pipeline_frames_equal_one_shot_render(nccl_world1, example_scenes, scene_kind, w, h, depth):
    import torch

    scene = synthetic_scene(200, 2, 5) if scene_kind == "synth200" else example_scenes[scene_kind]
    ds = DeviceScene(scene)
    ref = ds.render_image(w, h)
    pipe = rd.NativeFramePipeline(ds.handle, w, h, 0, 1, depth=depth, device=torch.device("cuda", 0))
    for k in range(2 * depth + 1):
        pipe.step()
        if k % depth == 0:
            assert np.array_equal(pipe.read_frame(), ref), k
    pipe.flush()
    assert np.array_equal(pipe.read_frame(), ref)
    pipe.close()
    ds.close()


# ncclGather's signature (rccl.h:745) as rg_gather_fn (include/raingun_frames.h)
GATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p, C.c_void_p)


def _hip_runtime():
    """The HIP runtime PyTorch loaded (the instance libraingun_hip.so binds to)."""
    import torch

    hip = C.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    hip.hipMemcpyAsync.restype = C.c_int
    hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    return hip


def _fake_gather(world, others, calls):
    """A stand-in for ncclGather on rank 0 of `world` ranks: slot 0 of the
    receive buffer gets this rank's send buffer, slot r rank r's pre-rendered
    part as that rank would send it (`others[r]`, packed RGB) -- device copies
    on the stream the pipeline hands over, as RCCL would."""
    hip = _hip_runtime()

    slot = others[1].numel() if world > 1 else 0

    def gather(send, recv, count, dtype, root, comm, stream):
        assert dtype == 1 and root == 0 and recv
        calls.append(count)
        if hip.hipMemcpyAsync(recv, send, count, 3, stream) != 0:  # hipMemcpyDeviceToDevice
            return 1
        # a batch of count // slot frames: rank r's chunk holds its packed parts back to back
        for r in range(1, world):
            for h in range(count // slot):
                if hip.hipMemcpyAsync(recv + r * count + h * slot, others[r].data_ptr(), slot, 3, stream) != 0:
                    return 1
        return 0

    return GATHER_FN(gather)


@pytest.mark.parametrize("world,w,h,T,depth,batch,root", [(2, 320, 243, 8, 3, 1, 1), (3, 256, 144, 16, 2, 2, 1),
                                                          (8, 640, 357, 8, 4, 2, 1), (8, 640, 357, 8, 4, 1, 1),
                                                          (8, 97, 61, 8, 1, 1, 1), (2, 64, 40, 8, 8, 0, 1),
                                                          (8, 640, 357, 8, 4, 2, 2), (3, 320, 243, 8, 3, 1, 3),
                                                          (2, 256, 149, 16, 4, 2, 4), (8, 97, 61, 8, 2, 0, 2)])
def test_native_pipeline_world_n_reinterleave(example_scenes, world, w, h, T, depth, batch, root):
    """The N > 1 native loop on one GPU: rank 0 of `world` ranks,
    the other ranks' parts (tiling {T, world, r}) pre-rendered and delivered by
    a stand-in gather.  The re-interleave, the slot offsets and the padding of
    heights that are not a multiple of T all run; every frame equals the
    one-shot render byte for byte.  root > 1: rank 0 renders
    `root` consecutive tiles of every period of root + world - 1 in one launch
    (grouped tiling), the others tile root + r - 1 of each period."""
    import torch

    from raingun_amd import _abi

    ds = DeviceScene(example_scenes["test1"])
    ref = ds.render_image(w, h)
    lib = _abi.lib()
    slot = rd.root_slot_rows(h, world, T, root)
    slot_bytes = (slot * w * 3 + 15) // 16 * 16  # off the root a part travels as packed RGB (rg_frames.hip)
    parts = [torch.zeros((max(slot, 8), w, 4), dtype=torch.uint8, device="cuda") for _ in range(world)]
    others = [torch.zeros(slot_bytes, dtype=torch.uint8, device="cuda") for _ in range(world)]
    for r in range(1, world):
        t = rd.tilings(r, world, T, root)[0]
        assert lib.rg_tiling_rows(h, C.byref(t)) <= slot
        _abi.check(lib.rg_render_tiles_async(ds.handle, w, h, C.byref(t), C.c_void_p(parts[r].data_ptr()), None,
                                             None, None))
        torch.cuda.synchronize()
        others[r][:slot * w * 3] = parts[r][..., :3].reshape(-1)
    torch.cuda.synchronize()
    calls = []
    fn = _fake_gather(world, others, calls)
    hdl = C.c_void_p()
    _abi.check(lib.rg_frames_create(ds.handle, w, h, T, 0, world, depth, C.c_void_p(1), C.cast(fn, C.c_void_p),
                                    C.byref(hdl)))
    if batch:  # 0: the default (two frames per gather at world > 1 with an even depth)
        _abi.check(lib.rg_frames_set_batch(hdl, batch))
    if root != 1:
        _abi.check(lib.rg_frames_set_root_tiles(hdl, root))
    out = np.empty((h, w, 4), np.uint8)
    b = batch or (2 if depth % 2 == 0 else 1)
    for k in range(2 * depth + 1):
        _abi.check(lib.rg_frames_step(hdl))
        if k % 3 == 0:
            if b == 2 and (k % depth) % 2 == 0:  # slot k % depth opens a batch of two
                # a batch waits for its gather: reading (or asking for the status) must not
                # start the catch-up gather, a collective, on rank 0 alone
                n_calls = len(calls)
                px = C.c_int32(-2)
                assert lib.rg_frames_read_image(hdl, out.ctypes.data) == _abi.RG_ERR_PENDING, k
                assert lib.rg_frames_status(hdl, C.byref(px)) == _abi.RG_OK and px.value == -1
                assert len(calls) == n_calls, k
            _abi.check(lib.rg_frames_flush(hdl))  # every rank flushes: a batch cut short is gathered then
            _abi.check(lib.rg_frames_read_image(hdl, out.ctypes.data))
            assert np.array_equal(out, ref), k
    _abi.check(lib.rg_frames_flush(hdl))
    _abi.check(lib.rg_frames_read_image(hdl, out.ctypes.data))
    assert np.array_equal(out, ref)
    lib.rg_frames_destroy(hdl)
    ds.close()
    assert calls and all(c in (slot_bytes, b * slot_bytes) for c in calls)
    assert sum(calls) == (2 * depth + 1) * slot_bytes  # every frame gathered exactly once
    if b == 2:
        assert 2 * slot_bytes in calls


def test_native_pipeline_reports_device_errors():
    """a frame that raises a device error (the AABB-normal panic,
    bodies.rs:324) is still delivered, and rg_frames_flush / _status /
    _read_image report the error and its first pixel."""
    from raingun_amd import _abi
    from raingun_amd.color import Color
    from raingun_amd.scene import AABB, Material, Scene

    m = Material(Color.from_str("#ffffff"), 0.5)
    bad = Scene(bodies=[AABB(((-3e8, -3e8, -7e8), (3e8, 3e8, -5e8)), m)])
    ds = DeviceScene(bad)
    st = _abi.rg_stats()
    with pytest.raises(_abi.RaingunError):
        ds.render_tiles(64, 48, stats=st)
    lib = _abi.lib()
    calls = []
    fn = _fake_gather(1, [None], calls)
    hdl = C.c_void_p()
    _abi.check(lib.rg_frames_create(ds.handle, 64, 48, 8, 0, 1, 2, C.c_void_p(1), C.cast(fn, C.c_void_p),
                                    C.byref(hdl)))
    for _ in range(3):
        _abi.check(lib.rg_frames_step(hdl))
    px = C.c_int32(-2)
    assert lib.rg_frames_status(hdl, C.byref(px)) == _abi.RG_ERR_AABB_NORMAL
    assert px.value == st.error_pixel
    out = np.empty((48, 64, 4), np.uint8)
    assert lib.rg_frames_read_image(hdl, out.ctypes.data) == _abi.RG_ERR_AABB_NORMAL
    lib.rg_frames_destroy(hdl)
    ds.close()
