"""bench.py's launch contract on CPU (no GPU work: --plan exits before any):
`--gpus N` outside a launcher starts N ranks itself, inside one it must equal
WORLD_SIZE -- never a silent one-GPU run reported as n_gpus 1."""
import json
import re
import os
import subprocess
import sys
from pathlib import Path

BENCH = Path(__file__).resolve().parent.parent / "bench.py"


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(BENCH), *args], capture_output=True, text=True, env=env, timeout=240)


def test_gpus_2_outside_a_launcher_runs_two_ranks():
    p = _run(["--gpus", "2", "--plan", "--backend", "gloo"])
    assert p.returncode == 0, p.stderr[-2000:]
    plans = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", p.stdout)]  # ranks share the pipe
    assert sorted(x["rank"] for x in plans) == [0, 1]
    assert all(x["world"] == 2 and x["n_gpus"] == 2 for x in plans)
    assert sorted(x["local_rank"] for x in plans) == [0, 1]
    # the N > 1 line always proves its gathered frame against a 1-rank render
    assert all(x["verify_against_1_rank_frame"] is True for x in plans)


def test_gpus_mismatching_world_size_fails_loudly():
    p = _run(["--gpus", "2", "--plan"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr
    assert '"n_gpus": 1' not in p.stdout


def test_default_is_one_gpu():
    p = _run(["--plan"])
    assert p.returncode == 0
    line = json.loads(p.stdout.strip())
    assert line["n_gpus"] == 1
    assert line["verify_against_1_rank_frame"] is False  # nothing gathered at N = 1 ...
    p = _run(["--plan", "--rccl-rehearsal"])
    assert json.loads(p.stdout.strip())["verify_against_1_rank_frame"] is True  # ... unless rehearsed


def test_check_frame_rejects_a_different_frame():
    import numpy as np
    import pytest

    sys.path.insert(0, str(BENCH.parent))
    import bench

    a = np.zeros((4, 6, 4), np.uint8)
    assert bench.check_frame(a.copy(), a, 2) is True
    b = a.copy()
    b[2, 3, 1] = 9
    with pytest.raises(SystemExit, match="1 pixels differ"):
        bench.check_frame(b, a, 8)
    with pytest.raises(SystemExit):
        bench.check_frame(a[:3], a, 8)


def _times_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, str(BENCH.parent))
        import bench

        res = bench.gather_rank_times(0.01 * (rank + 1), 10, 0.5 + rank, world, rank)
        Path(out_dir, f"r{rank}.json").write_text(json.dumps(res))
    finally:
        dist.destroy_process_group()


def test_per_rank_times_reach_every_rank(tmp_path):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_times_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        res = json.loads((tmp_path / f"r{r}.json").read_text())
        assert [x["rank"] for x in res] == [0, 1]
        assert [x["ms_per_step"] for x in res] == [1.0, 2.0]
        assert [x["share_kernel_ms"] for x in res] == [0.5, 1.5]
