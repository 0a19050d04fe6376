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


def test_gpus_mismatching_world_size_fails_loudly():
    p = _run(["--gpus", "2", "--plan"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr
    assert '"n_gpus": 1' not in p.stdout


def test_default_is_one_gpu():
    p = _run(["--plan"])
    assert p.returncode == 0
    assert json.loads(p.stdout.strip())["n_gpus"] == 1
