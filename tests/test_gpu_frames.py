"""The native frames-in-flight pipeline (include/raingun_frames.h) on one GPU:
a world-1 RCCL process group runs the same per-frame loop an N-GPU node runs
(render on stream k % depth, ncclGather on the communication stream, rank 0's
re-interleave on a side stream).  Every delivered frame must equal a one-shot
render byte for byte."""
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
