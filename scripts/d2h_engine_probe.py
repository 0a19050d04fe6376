"""Which engine carries a device-to-host copy into page-locked memory, and how
fast: hipMemcpyAsync of a 4K RGBA8 frame (33.2 MB) and of a 1/3 band into
(a) hipHostMalloc'd memory, (b) a hipHostRegister'ed numpy buffer (rg_host_register),
alone and while a render kernel runs.  Run under rocprofv3 --kernel-trace
--memory-copy-trace: SDMA copies appear as memory copies, blit copies as
__amd_rocclr_copyBuffer kernels."""
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from raingun_amd import _abi  # noqa: E402

print({k: v for k, v in os.environ.items() if any(s in k for s in ("SDMA", "HSA", "HIP", "GPU_", "ROC"))},
      file=sys.stderr)
hip = C.CDLL(str(Path(torch.__file__).parent / "lib" / "libamdhip64.so"))
hip.hipHostMalloc.restype = C.c_int
hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipMemcpyAsync.restype = C.c_int
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
N = 3840 * 2160 * 4
src = torch.empty(N, dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
res = {}
p = C.c_void_p()
assert hip.hipHostMalloc(C.byref(p), N, 0) == 0
reg_buf = np.empty(N, np.uint8)
reg = _abi.HostRegistration(reg_buf)
for name, dst in (("hipHostMalloc", p.value), ("registered", reg_buf.ctypes.data)):
    for size in (N, N // 3):
        for _ in range(3):
            assert hip.hipMemcpyAsync(dst, src.data_ptr(), size, 2, C.c_void_p(s.cuda_stream)) == 0
        s.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            assert hip.hipMemcpyAsync(dst, src.data_ptr(), size, 2, C.c_void_p(s.cuda_stream)) == 0
        s.synchronize()
        dt = (time.perf_counter() - t0) / 10
        res[f"{name}_{size}"] = {"ms": round(dt * 1e3, 4), "GBps": round(size / dt / 1e9, 2)}
reg.close()
print(json.dumps(res, indent=1))
