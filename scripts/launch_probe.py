"""Why is one launch of a small share slow?  (diagnostic, round 4)

For the whole frame and rank 0's 1/8 share (8-row tiles), time the latency-sized
launch (rg_render_tiles_async) three ways on one stream:
  sync     each launch followed by a host synchronisation (the single-shot case),
  b2b      K launches enqueued back to back, no host gap (events around all K),
  spaced   K launches, each after a short host sleep (idle gaps, GPU not drained of work)
and the pipelined launch (rg_render_tiles_pipelined) on 8 streams round-robin.
RAINGUN_HIP_LIB selects a variant library.  JSON on stdout.
    python scripts/launch_probe.py [workload ...]
"""
import ctypes as C
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import bench  # noqa: E402
from raingun_amd import _abi  # noqa: E402
from raingun_amd.scene import DeviceScene  # noqa: E402

W, H, K = 3840, 2160, 20


def main():
    lib = _abi.lib()
    out = {}
    for wl in sys.argv[1:] or ["test1", "synth1024"]:
        ds = DeviceScene(bench.load_workload(wl, W, H)[0])
        r = {}
        for name, stride in (("whole", 1), ("share8", 8)):
            t = _abi.rg_tiling(8 if stride > 1 else H, stride, 0)
            rows = lib.rg_tiling_rows(H, C.byref(t))
            bufs = [torch.empty((rows, W, 4), dtype=torch.uint8, device="cuda") for _ in range(8)]
            s0 = torch.cuda.current_stream()

            def launch(i=0, stream=None, pipelined=False):
                sh = C.c_void_p((stream or s0).cuda_stream)
                if pipelined:
                    _abi.check(lib.rg_render_tiles_pipelined(ds.handle, W, H, C.byref(t),
                                                             C.c_void_p(bufs[i % 8].data_ptr()), None, sh))
                else:
                    _abi.check(lib.rg_render_tiles_async(ds.handle, W, H, C.byref(t),
                                                         C.c_void_p(bufs[0].data_ptr()), None, sh, None))

            for _ in range(5):
                launch()
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
            for e0, e1 in ev:  # sync
                e0.record(s0)
                launch()
                e1.record(s0)
                torch.cuda.synchronize()
            sync_ms = sorted(e0.elapsed_time(e1) for e0, e1 in ev)[K // 2]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s0)
            for _ in range(K):  # back to back
                launch()
            b.record(s0)
            torch.cuda.synchronize()
            b2b_ms = a.elapsed_time(b) / K
            for e0, e1 in ev:  # spaced: ~0.3 ms of host time between launches, stream never drained
                e0.record(s0)
                launch()
                e1.record(s0)
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < 3e-4:
                    pass
            torch.cuda.synchronize()
            spaced_ms = sorted(e0.elapsed_time(e1) for e0, e1 in ev)[K // 2]
            streams = [torch.cuda.Stream() for _ in range(8)]
            for i in range(16):
                launch(i, streams[i % 8], True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(8 * K):
                launch(i, streams[i % 8], True)
            torch.cuda.synchronize()
            pipe_ms = (time.perf_counter() - t0) * 1e3 / (8 * K)
            r[name] = {"sync_ms": round(sync_ms, 4), "b2b_ms": round(b2b_ms, 4), "spaced_ms": round(spaced_ms, 4),
                       "pipelined_8_streams_ms": round(pipe_ms, 4)}
            # the same tiles as ONE call split into k concurrent launches on k streams (tile j of the
            # call's selection -> launch j % k), from a start event to the join of all k
            for k in (2, 4, 8):
                subs = [_abi.rg_tiling(8, stride * k, j * stride) for j in range(k)]
                sbufs = [torch.empty((lib.rg_tiling_rows(H, C.byref(u)), W, 4), dtype=torch.uint8, device="cuda")
                         for u in subs]
                ss = streams[:k]
                ts = []
                for rep in range(K + 3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s0)
                    for j in range(k):
                        ss[j].wait_event(e0)
                        _abi.check(lib.rg_render_tiles_async(ds.handle, W, H, C.byref(subs[j]),
                                                             C.c_void_p(sbufs[j].data_ptr()), None,
                                                             C.c_void_p(ss[j].cuda_stream), None))
                    for j in range(k):
                        s0.wait_stream(ss[j])
                    e1.record(s0)
                    torch.cuda.synchronize()
                    if rep >= 3:
                        ts.append(e0.elapsed_time(e1))
                r[name][f"split{k}_ms"] = round(sorted(ts)[len(ts) // 2], 4)
            for st_ in streams:
                ds.release_stream(st_.cuda_stream)
            print(wl, name, r[name], file=sys.stderr, flush=True)
        ds.close()
        out[wl] = r
    print(json.dumps(out))


if __name__ == "__main__":
    main()
