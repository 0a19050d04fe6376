#!/usr/bin/env python3
"""bench.measure() of several workloads in sequence in ONE process (frames in flight, 4K): does a
line's time depend on what ran before it?  profiles/r06/s29: test3 as bench.py's main line
0.219 ms, as an extra line after test1 0.243 ms.

    python scripts/measure_order_probe.py wl[,wl...] [--reuse-streams]   -> one JSON line
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    wls = sys.argv[1].split(",") if len(sys.argv) > 1 else ["test3", "test3"]
    extra = [a for a in sys.argv[2:]]
    args = bench.parse_args(["--no-cpu-baseline", "--steps", "100", *extra])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    out = []
    for wl in wls:
        r = bench.measure(wl, args, 1, 0, 0, dev, False)
        out.append({"workload": wl, "ms_per_step": r["ms_per_step"]})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
