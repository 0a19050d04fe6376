import sys; sys.path.insert(0, '.')
import bench
from raingun_amd.scene import DeviceScene
for wl in ("synth1024", "synth4096p8d8"):
    ds = DeviceScene(bench.load_workload(wl, 3840, 2160)[0])
    b = ds.bvh_info()
    print(wl, {k: getattr(b, k) for k in ("nodes", "leaves", "depth", "lane_stack")})
    ds.close()
