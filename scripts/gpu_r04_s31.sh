#!/bin/bash
# Round-4 session 31: the round-end checks on the libraries __graft_entry__.build()
# produced at HEAD -- the whole -m gpu suite, smoke(), the driver's bench configuration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s31; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cfg.json 2> $O/bench_driver_cfg.err || { tail -20 $O/bench_driver_cfg.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_driver_cfg.json').read().strip().splitlines()[-1]);print('driver-cfg', d['value'], d['ms_per_step'], d['roofline']['frac'], d['host_visible']['pinned']['ms_per_step'], d['host_visible']['pageable']['ms_per_step'], d['north_star_1024_spheres']['ms_per_step'])"
echo session done
