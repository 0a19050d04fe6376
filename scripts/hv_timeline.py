"""Host-visible frames under a trace: rg_render_image of one workload into a
page-locked buffer, back to back (run under rocprofv3 --kernel-trace
--memory-copy-trace to see band renders and their copies on the timeline)."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from raingun_amd import _abi  # noqa: E402
from raingun_amd.scene import DeviceScene  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "test1"
bands = int(sys.argv[2]) if len(sys.argv) > 2 else 0
W, H = 3840, 2160
ds = DeviceScene(bench.load_workload(wl, W, H)[0])
ds.set_image_bands(bands)
buf = np.empty((H, W, 4), dtype=np.uint8)
reg = _abi.HostRegistration(buf)
for _ in range(5):
    ds.render_image(W, H, out=buf)
t0 = time.perf_counter()
n = 20
for _ in range(n):
    ds.render_image(W, H, out=buf)
print(wl, "bands", bands, "ms per frame", round((time.perf_counter() - t0) / n * 1e3, 4))
reg.close()
ds.close()
