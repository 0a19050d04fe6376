#!/usr/bin/env python3
"""Benchmark: Mrays/s of the per-pixel ray-trace path (BASELINE.json metric).

One step = one frame of the workload rendered by the HIP megakernel, scene and
textures already resident in HBM, framebuffer left in HBM (rank 0 holds the
assembled frame).  At N>1 (one rank per GPU: torchrun, or `--gpus N`, which
launches torch.distributed.run itself) the frame is cut into 8-row tiles dealt
round-robin to the ranks and the tiles are gathered to rank 0 with one RCCL
gather per frame or two (ncclGather over xGMI on the library's own
communicator: ncclCommInitRank, its unique id broadcast by torch.distributed),
then re-interleaved into image order on rank 0 -- the per-frame loop runs in
C++ (include/raingun_frames.h).  The line reports the ranks RCCL saw
(`rccl_nranks`, `rccl.devices`).

`value` is the device-resident kernel throughput: the frame is left in HBM
(rank 0 holds the assembled frame).  SURVEY.md 8(d)'s scope -- "framebuffer
available to host", as the reference's timer around render_image
(src/render.rs:54-56) -- is the `host_visible` line (rg_render_image, the
frame in host memory when each call returns).

Workload (BASELINE.json configs[1]): examples/test1.yml at 3840x2160,
recursion depth 5.  Extra line items on the same N GPUs: configs[2]
(test3.yml 3840x2160), the north_star scene (1024 spheres, 3840x2160, depth
5), configs[3] (the same at 7680x4320) and configs[4] (4096 spheres + 8
planes, 16384x16384, depth 8); at N=1 `host_visible` times the drop-in itself,
rg_render_image, with the frame in host memory when each call returns.
Frames are kept in flight (8, each on its own render stream): the timed
region holds `--steps` complete frames (fewer for the slow extra lines, see
`steps` in each), after `--settle-s` seconds of untimed frames and the
`--warmup` untimed steps.

Prints ONE JSON line on rank 0 (the driver's contract).  `roofline` is the
executed-work VALU roofline: issue cycles of the instructions the kernels
executed per frame (rocprofv3 PMC, profiles/pmc_work.json: FP64 4 cycles, f32
transcendental 4, every other VALU instruction 2 per wave64 on a 32-lane
SIMD; MI355X_MICROARCH.md) over 1,024 SIMDs x 2.4 GHz x the measured time per
frame, as FP64-rate lane-ops/s against 39.3 T.  `roofline_hbm` reports HBM
bytes; `cpu_baseline` the CPU restatement in oracle/ on this host's cores on a
bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

METRIC = "Mrays/sec (primary+shadow+secondary) at 3840×2160, depth 5; 1/2/4/8 MI355X"
FP64_PEAK_TOPS = 39.3     # MI355X FP64 vector 78.6 TFLOP/s spec counts FMA as 2; parity forbids FMA -> 39.3 T ops/s
SIMDS, CLOCK_HZ = 1024, 2.4e9  # 256 CUs x 4 SIMDs; peak engine clock (39.3 T = 1024 x 16 FP64 lanes x 2.4 GHz)
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec
# Algorithmic FP64 ops per body test on the reference's miss path.
OPS_PER_BODY = {"sphere": 16, "plane": 14, "disk": 20, "aabb": 18}
TILE_ROWS = 16


def load_workload(name: str, W: int = 3840, H: int = 2160):
    from raingun_amd.scene import AABB, Disk, Plane, Sphere, load_scene
    from raingun_amd.synth import scene_md5, synthetic_yaml

    golden = REPO / "tests" / "golden"
    if name == "test1":
        scene = load_scene(golden / "examples" / "test1.yml", texture_root=golden)
        scene.max_recursion_depth = 5
        label = f"examples/test1.yml {W}x{H} depth 5 (BASELINE configs[1])"
        src = ("reference example scene examples/test1.yml; textures decoded by the native host layer "
               "(libraingun_host.so, jpeg-decoder 0.1.11 rounding)")
    elif name == "test3":
        scene = load_scene(golden / "examples" / "test3.yml", texture_root=golden)
        label = f"examples/test3.yml {W}x{H} depth 10 (BASELINE configs[2])"
        src = ("reference example scene examples/test3.yml; textures decoded by the native host layer "
               "(libraingun_host.so, jpeg-decoder 0.1.11 rounding)")
    elif name.startswith("synth"):
        import re

        m = re.fullmatch(r"synth(\d*)(?:p(\d+))?(?:d(\d+))?", name)
        if not m:
            raise SystemExit(f"unknown workload {name}")
        n, planes, depth = int(m.group(1) or 1024), int(m.group(2) or 2), int(m.group(3) or 5)
        text = synthetic_yaml(n, planes, depth)
        scene = load_scene(text)
        label = (f"synthetic {n} spheres + {planes} planes {W}x{H} depth {depth} "
                 f"(seed 0x5EED, md5 {scene_md5(text)})")
        if (n, planes, depth, W, H) == (1024, 2, 5, 7680, 4320):
            label += " (BASELINE configs[3])"
        elif (n, planes, depth, W, H) == (4096, 8, 8, 16384, 16384):
            label += " (BASELINE configs[4])"
        elif (n, planes, depth, W, H) == (1024, 2, 5, 3840, 2160):
            label += " (north_star)"
        src = "synthetic seeded scene (raingun_amd/synth.py)"
    else:
        raise SystemExit(f"unknown workload {name}")
    counts = {"sphere": 0, "plane": 0, "disk": 0, "aabb": 0}
    for b in scene.bodies:
        counts[{Sphere: "sphere", Plane: "plane", Disk: "disk", AABB: "aabb"}[type(b)]] += 1
    ops_per_ray = sum(OPS_PER_BODY[k] * v for k, v in counts.items())
    return scene, label, src, counts, ops_per_ray


def texture_bytes(scene) -> int:
    from raingun_amd.scene import Texture

    seen, total = set(), 0
    for b in scene.bodies:
        c = b.material.coloration
        if isinstance(c, Texture) and id(c.image) not in seen:
            seen.add(id(c.image))
            total += c.image.size
    return total


def cpu_baseline(scene, width, height, budget_s: float = 12.0):
    """CPU restatement (oracle/) on this host's cores, on a bounded sample of the
    same frame: every k-th 16-row tile, k grown until one pass fits the budget."""
    import oracle
    from raingun_amd.scene import SceneDesc

    desc = SceneDesc(scene)
    threads = oracle.default_threads()
    tiles = (height + TILE_ROWS - 1) // TILE_ROWS
    stride = max(1, tiles // 64) if width * height > 40_000_000 else 1  # first probe: the whole frame (or 64 tiles)
    while True:
        t0 = time.perf_counter()
        st, _, _, counts, _ = oracle.render(desc, width, height, TILE_ROWS, stride, 0, threads=threads)
        dt = time.perf_counter() - t0
        if st != 0:
            raise RuntimeError(f"oracle status {st}")
        if dt <= budget_s or stride >= tiles:
            break
        stride = min(tiles, int(stride * dt / budget_s * 2) + 1)
    reps, elapsed, rays = 1, dt, sum(counts.values())
    while elapsed < budget_s / 2 and reps < 100:
        t0 = time.perf_counter()
        oracle.render(desc, width, height, TILE_ROWS, stride, 0, threads=threads)
        elapsed += time.perf_counter() - t0
        reps += 1
    rows = oracle.lib().rgo_tiling_rows(height, __import__("raingun_amd")._abi.rg_tiling(TILE_ROWS, stride, 0))
    return {
        "value": round(rays * reps / elapsed / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"every {stride}th 16-row tile of the same frame ({min(rows, height)} of {height} rows, "
                  f"{rays} rays) x{reps} passes, {elapsed:.1f}s; CPU restatement oracle/raingun_oracle.c, "
                  f"-O2 -ffp-contract=off, {threads} pthreads",
    }


def pmc_work(key: str):
    """Executed work per frame of one workload (scripts/pmc_work.py -> profiles/pmc_work.json):
    VALU issue cycles, HBM bytes, instruction mix; None if not profiled."""
    f = REPO / "profiles" / "pmc_work.json"
    if not f.exists():
        return None
    try:
        return json.loads(f.read_text()).get(key)
    except Exception:
        return None


def roofline(key: str, frame_s: float, n_gpus: int, alg_bytes: int, tex: int, alg_ops: float = 0.0):
    """Executed-work VALU roofline of the timed configuration: the issue cycles
    of every VALU instruction the frame's kernels executed (PMC, counted at
    N=1 for the whole frame, which the N ranks split) over the cycles N GPUs
    offer in the measured time per frame."""
    w = pmc_work(key)
    res = {"bound": "valu", "achieved": None, "peak": round(FP64_PEAK_TOPS * n_gpus, 3),
           "unit": "T FP64-rate VALU lane-ops/s", "frac": None, "traffic": None,
           "basis": "not profiled (run scripts/pmc_work.sh for this workload)"}
    if alg_ops:
        # SURVEY.md 8(d)'s algorithmic figure: the reference's brute-force FP64 ops per ray
        # (16 per sphere, 14 per plane ...) x rays per frame over the FP64 lane-op peak.  Shading
        # is not counted and the BVH skips most of the brute-force work, so it is not a
        # utilisation figure (it exceeds 1 on the sphere scenes)
        res["algorithmic_frac"] = round(alg_ops / frame_s / (FP64_PEAK_TOPS * 1e12 * n_gpus), 5)
    if w:
        cyc = w["valu_cycles_per_frame"]
        frac = cyc / (frame_s * n_gpus * SIMDS * CLOCK_HZ)
        fw = w.get("fetch_write_kib_per_frame")  # PMC FETCH_SIZE, WRITE_SIZE (KiB per frame as collected)
        if fw and None not in fw:
            res["traffic_raw"] = {"fetch_size_bytes": round(fw[0] * 1024), "write_size_bytes": round(fw[1] * 1024),
                                  "note": "uncorrected; `traffic` doubles FETCH (gfx950 correction for wide "
                                          "streaming reads, unvalidated for scratch/texel/table reads)"}
        res.update({
            "achieved": round(cyc * 16.0 / frame_s / 1e12, 4),
            "frac": round(frac, 5),
            "traffic": w.get("hbm_bytes_per_frame"),
            "valu_cycles_per_frame": cyc,
            "basis": (f"executed work: {w['valu_insts_per_frame']:.4g} VALU wave64 instructions per frame "
                      f"({w['f64_insts_per_frame']:.4g} FP64 x 4 cycles, {w['trans32_insts_per_frame']:.4g} f32 "
                      f"transcendental x 4, the rest x 2 cycles on a 32-lane SIMD: MI355X_MICROARCH.md) = "
                      f"{cyc:.4g} SIMD issue cycles per frame, over {SIMDS} SIMDs x {CLOCK_HZ / 1e9} GHz x "
                      f"{n_gpus} GPU(s) x the measured {frame_s * 1e3:.4f} ms per frame (ms_per_step); "
                      f"achieved = cycles x 16 FP64 lanes / time.  Counters: {w['source']}"),
        })
    hbm = {"bound": "hbm", "achieved": round(alg_bytes / frame_s / 1e9, 3), "peak": 8000.0 * n_gpus, "unit": "GB/s",
           "frac": round(alg_bytes / frame_s / 1e9 / (8000.0 * n_gpus), 7),
           "traffic": w.get("hbm_bytes_per_frame") if w else None,
           "basis": f"{alg_bytes} B framebuffer written per frame (+{tex} B of textures read, L2/MALL resident) / "
                    f"ms_per_step; traffic = PMC FETCH_SIZE x 2 + WRITE_SIZE (KiB -> B, gfx950 correction)"}
    return res, hbm


def verify_enabled(args, world: int) -> bool:
    """Rank 0 checks the gathered frame against a 1-rank render whenever frames are gathered
    (N > 1, or the world-1 RCCL rehearsal): the first real multi-GPU run proves its frame before
    it reports a rate.  At N = 1 without a gather it runs on request (--verify)."""
    return bool(getattr(args, "verify", False)) or world > 1 or bool(getattr(args, "rccl_rehearsal", False))


def check_frame(got, ref, world: int) -> bool:
    """Byte-for-byte comparison of rank 0's assembled frame with the 1-rank render; a mismatch
    ends the run with a non-zero status (no Mrays/s line is printed)."""
    import numpy as np

    got = np.asarray(got)
    ok = got.shape == ref.shape and bool((got == ref).all())
    if not ok:
        bad = int((got != ref).any(axis=-1).sum()) if got.shape == ref.shape else -1
        raise SystemExit(f"verification: the {world}-rank frame differs from the 1-rank render "
                         f"({bad} pixels differ; shapes {got.shape} vs {ref.shape})")
    return True


def gather_rank_times(elapsed_s: float, steps: int, kernel_ms: float, world: int, rank: int):
    """Every rank's own timed-loop wall time per frame and its single-launch share time, gathered
    to every rank (object collective: gloo or RCCL), so a skewed rank is visible in the line."""
    mine = {"rank": rank, "ms_per_step": round(elapsed_s / max(1, steps) * 1e3, 4), "share_kernel_ms": round(kernel_ms, 4)}
    if world == 1:
        return [mine]
    import torch.distributed as dist

    out = [None] * world
    dist.all_gather_object(out, mine)
    return sorted(out, key=lambda r: r["rank"])


_RENDER_STREAMS = {}


def render_streams(dev, n: int):
    """The render streams of the frames in flight, made once per process and reused by every line
    (--no-reuse-streams: new ones per line).  HIP maps each new stream to a hardware queue, and a
    line's time depends on where its streams land: test3 0.219 ms as the first line, 0.243 ms after
    test1 on new streams (profiles/r06/s29, s30); on the first line's streams 0.218-0.221 ms (s31,
    s38).  (Reuse first moved the host-visible lines' streams so that their split frames' two
    parts shared a queue, 0.80 -> 1.06 ms (s32, s36); the library now gives the one-launch part's
    stream a hardware queue of its own, rg_capi.hip ensure_image_res.)"""
    import torch

    key = (dev.index or 0, n)
    if key not in _RENDER_STREAMS:
        _RENDER_STREAMS[key] = [torch.cuda.Stream(dev) for _ in range(n)]
    return _RENDER_STREAMS[key]


def measure(workload: str, args, world: int, rank: int, local_rank: int, dev, cpu: bool, size=None,
            steps=None, warmup=None, budget_s=None):
    """Time `steps` frames of `workload` on this rank (after `warmup`), frame
    sharded over `world` ranks and gathered to rank 0.  `budget_s`: cap the
    frames so the timed region lasts about that long (slow extra lines).
    Returns the rank-0 result dict (None on other ranks)."""
    import torch
    import torch.distributed as dist

    from raingun_amd import _abi
    from raingun_amd import distributed as rd
    from raingun_amd.scene import DeviceScene

    W, H = size or (args.width, args.height)
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    scene, label, src, body_counts, ops_per_ray = load_workload(workload, W, H)
    if args.depth is not None:  # diagnostic: override the recursion cap
        scene.max_recursion_depth = args.depth
        label += f" (depth overridden: {args.depth})"
    ds = DeviceScene(scene, device=local_rank)  # scene + textures uploaded once, resident in HBM
    if args.tile_order >= 0:
        ds.set_tile_order(args.tile_order)
    if args.lane_depth is not None:
        ds.set_lane_depth(args.lane_depth)
    lib = _abi.lib()
    bvh = ds.bvh_info()

    # --share S (diagnostic, N = 1): render only rank 0's tiles of an S-way split
    split = args.share if (world == 1 and args.share > 1) else world
    TR = args.tile_rows  # rows per interleaved row tile (rank t % N renders tile t)
    tiling = rd.tiling(args.share_rank if split != world else rank, split, TR)
    # rank 0's share (--rank0-share R, native N-rank loop): periods of R + N - 1 tiles, the first R to
    # rank 0 (include/raingun_frames.h rg_frames_set_root_tiles); this rank's tilings, for the counted render
    R0 = args.rank0_share if world > 1 else 1
    my_tilings = rd.tilings(rank, world, TR, R0) if R0 > 1 else [tiling]
    tiling = my_tilings[0]
    my_rows = sum(lib.rg_tiling_rows(H, C.byref(t)) for t in my_tilings)
    slot = rd.slot_rows(H, split, TR)  # equal-size gather slots (last ranks zero-padded)
    out = torch.zeros((max(slot, my_rows), W, 4), dtype=torch.uint8, device=dev)
    # frames in flight, each on its own render stream and hardware queue (16 per
    # process, see main): 8 -- the whole frame is flat from 4 up; a rank's 1/8
    # share of the north-star frame renders in 0.481 / 0.461 / 0.439 / 0.441 ms
    # at 4 / 6 / 8 / 10 (profiles/r02/share_sweep.txt)
    F = args.frames_in_flight if args.frames_in_flight > 0 else 8
    if W * H >= 100_000_000:
        F = min(F, 3)  # 1 GB frames (configs[4]): three in flight fill the GPU as well
    use_pipe = args.backend == "nccl" or world == 1
    gathered = rd.gather_buffers(out, world) if (world > 1 and rank == 0 and not use_pipe) else None
    frame = torch.empty((H, W, 4), dtype=torch.uint8, device=dev) if (rank == 0 and not use_pipe) else None

    stream = torch.cuda.current_stream(dev)
    sh = C.c_void_p(stream.cuda_stream)

    pipelined_fn = getattr(lib, "rg_render_tiles_pipelined", None)

    def render(stats=None, buf=None, pipelined=False):
        # on the current stream: the frame pipeline's render stream for this frame, or the default
        dst = out if buf is None else buf
        cur = torch.cuda.current_stream(dev)
        sh_cur = sh if cur == stream else C.c_void_p(cur.cuda_stream)
        if pipelined and pipelined_fn is not None:  # one of F frames in flight: grid sized for throughput
            st = pipelined_fn(ds.handle, W, H, C.byref(tiling), C.c_void_p(dst.data_ptr()), None, sh_cur)
        elif pipelined:  # a pre-round-3 library (A/B runs): a launch without stats was the pipelined one
            st = lib.rg_render_tiles_async(ds.handle, W, H, C.byref(tiling), C.c_void_p(dst.data_ptr()), None,
                                           sh_cur, None)
        else:  # one launch sized for its own latency
            st = lib.rg_render_tiles_async(ds.handle, W, H, C.byref(tiling), C.c_void_p(dst.data_ptr()), None,
                                           sh_cur, C.byref(stats) if stats is not None else None)
        _abi.check(st, "rg_render_tiles_async")

    def render_tiles(_t):
        render()
        return out

    # Frames in flight (FramePipeline): frame k renders on render stream k % F
    # into its own buffer; at N > 1 its tiles are gathered to rank 0 over RCCL
    # and re-interleaved there while the next frames render.  Consecutive
    # frames' renders overlap: the next frame's blocks take the CUs the current
    # frame's slowest tiles leave idle.  Every frame is complete (rendered, and
    # at N > 1 gathered and assembled on rank 0) when the timed region ends.
    # The gloo rehearsal gathers through host memory one frame at a time.
    pipe = None
    gather = world > 1 or args.rccl_rehearsal
    native = use_pipe and gather and args.backend == "nccl" and not args.python_pipeline
    if R0 > 1 and not native:
        raise SystemExit("--rank0-share needs the native N-rank loop (backend nccl, no --python-pipeline)")
    rccl = None
    if native:  # the per-frame loop in C++ (include/raingun_frames.h): render, ncclGather, re-interleave
        # on the library's own RCCL communicator; a failure raises (the Python loop only on request)
        pipe = rd.NativeFramePipeline(ds, W, H, rank, world, TR, depth=F, device=dev, root_tiles=R0)
        info = pipe.comm.info()
        if info["nranks"] != world or info["rank"] != rank:
            raise SystemExit(f"RCCL communicator {info} does not match rank {rank} of {world}")
        infos = [None] * world
        if world > 1:
            dist.all_gather_object(infos, info)
        else:
            infos = [info]
        rccl = {"nranks": info["nranks"], "devices": [i["device"] for i in infos],
                "communicator": "ncclCommInitRank (rg_comm_init_rank; unique id broadcast by torch.distributed)"}
    if not native and use_pipe:
        pipe = rd.FramePipeline((slot, W, 4), H, rank, world, TR, device=dev, depth=F,
                                streams=(render_streams(dev, F) if args.reuse_streams else True)
                                if F > 1 and not args.one_render_stream else False,
                                gather=gather)

    def step():
        if native:
            pipe.step()
        elif pipe is not None:
            pipe.step(lambda part: render(buf=part, pipelined=True))
        else:
            rd.render_frame(render_tiles, H, rank, world, TR, out=frame, gather_bufs=gathered)

    def finish():
        if pipe is not None:
            pipe.flush()  # the native pipeline raises on a device error of any frame

    # one counted render: ray totals per class (deterministic per frame); rank 0 with a share
    # R > 1 renders its R tilings (the native loop does them in one grouped launch)
    stats = _abi.rg_stats()
    counts = [0, 0, 0]
    for t_ in my_tilings:
        tiling = t_
        render(stats)
        counts = [counts[0] + stats.rays.primary, counts[1] + stats.rays.shadow, counts[2] + stats.rays.secondary]
    tiling = my_tilings[0]
    stats.rays.primary, stats.rays.shadow, stats.rays.secondary = counts
    rays = torch.tensor(counts, dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(rays)
    rays = [int(x) for x in rays.tolist()]
    rays_per_frame = sum(rays)

    # Settle: untimed frames for args.settle_s of wall time before the warm-up
    # steps.  A GPU idle until now runs its first frames slowly (test1 at 20 timed
    # steps: 0.416 ms per frame after 5 warm-up frames, 0.365 after 500;
    # profiles/r02/settle.txt) -- the timed steps measure the steady state.
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle_s:
        for _ in range(F):
            step()
        finish()
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()

    t_w = time.perf_counter()
    for _ in range(warmup):
        step()
    finish()
    torch.cuda.synchronize(dev)
    t_w = (time.perf_counter() - t_w) / max(1, warmup)
    if budget_s is not None and warmup > 0:  # slow lines: as many frames as fit the budget (same on every rank)
        k = torch.tensor([max(3, min(steps, int(budget_s / max(t_w, 1e-6))))], dtype=torch.int64, device=dev)
        if world > 1:
            dist.all_reduce(k, op=dist.ReduceOp.MIN)
        steps = int(k[0])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    finish()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0

    # device errors of frames the Python pipeline rendered asynchronously
    if pipe is not None and not native:
        for s_ in (pipe.streams or [stream]):
            st_, px_ = ds.stream_status(s_.cuda_stream)
            _abi.check(st_, f"frame render (first erroring pixel {px_})")

    # Single-stream kernel time (one latency-sized launch after another, HIP
    # events on that stream): the time ONE launch of this rank's share takes on
    # an otherwise idle GPU (rocprofv3 of `--frames-in-flight 1` gives the same
    # average).  Not the timed configuration (F frames in flight).
    events = []
    for _ in range(max(1, args.roofline_frames)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        render()
        e1.record(stream)
        events.append((e0, e1))
    torch.cuda.synchronize(dev)
    kernel_ms = sum(e0.elapsed_time(e1) for e0, e1 in events) / len(events)

    per_rank = gather_rank_times(elapsed, steps, kernel_ms, world, rank)
    tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt[0])
    verified = None
    if verify_enabled(args, world):  # one extra frame, outside the timed region
        if native:
            step()
            finish()
            final = pipe.read_frame() if rank == 0 else None
        elif pipe is not None:
            step()
            finish()
            final = pipe.frame if rank == 0 else None
        else:
            final = rd.render_frame(render_tiles, H, rank, world, TR, out=frame, gather_bufs=gathered)
        if rank == 0:
            torch.cuda.synchronize(dev)
            ref = ds.render_image(W, H)
            import numpy as np

            got = final if isinstance(final, np.ndarray) else final.cpu().numpy()
            verified = check_frame(got, ref, world)
    if native:
        pipe.close()
    elif pipe is not None and pipe.streams:
        for s_ in pipe.streams:
            ds.release_stream(s_.cuda_stream)
    ds.close()
    if rank != 0:
        return None

    if world > 1:
        via = "RCCL" if args.backend == "nccl" else f"{args.backend} (rehearsal, through host memory)"
        deal = f"round-robin {TR}-row tiles" if R0 == 1 else \
            f"{TR}-row tiles in periods of {R0 + world - 1}: {R0} to rank 0, one to each other rank"
        parallelism = f"row-tiles x{world} ({deal}, one {via} gather per frame to rank 0"
    else:
        parallelism = "one GPU (whole frame"
    if native:
        parallelism += f", {F} frames in flight on {F} render streams; per-frame loop in C++, raingun_frames.h)"
    elif pipe is not None and pipe.streams:
        parallelism += f", {F} frames in flight on {F} render streams)"
    else:
        parallelism += ", frames rendered one after another on one stream)"
    frame_s = elapsed / steps
    value = rays_per_frame * steps / elapsed / 1e6
    my_rays = stats.rays.primary + stats.rays.shadow + stats.rays.secondary
    tex = texture_bytes(scene)
    alg_bytes = H * W * 4  # the frame written once (all ranks together)
    key = f"{workload}@{W}x{H}"
    roof, roof_hbm = roofline(key, frame_s, world if split == world else 1, alg_bytes if split == world else
                              my_rows * W * 4, tex, alg_ops=rays_per_frame * ops_per_ray if split == world else 0.0)
    if split != world:  # --share diagnostic: the PMC figures are whole-frame ones
        roof.update({"achieved": None, "frac": None, "traffic": None, "basis": "--share diagnostic: not computed"})
    ref_equiv = my_rays * ops_per_ray / (kernel_ms * 1e-3) / 1e12
    res = {
        "value": round(value, 3),
        "ms_per_step": round(frame_s * 1e3, 4),
        "steps": steps,
        "warmup": warmup,
        "kernel_ms": round(kernel_ms, 4),
        "kernel_ms_config": "one latency-sized launch at a time on one stream (rg_render_tiles_async), HIP events",
        "data": src,
        "settle_s": args.settle_s,
        "config": {"workload": label, "width": W, "height": H, "max_recursion_depth": scene.max_recursion_depth,
                   "bodies": body_counts, "lights": len(scene.lights), "tile_rows": TR,
                   "frames_in_flight": F, "parallelism": parallelism,
                   **({"rank0_share_tiles": R0} if world > 1 else {})},
        "rays_per_frame": {"primary": rays[0], "shadow": rays[1], "secondary": rays[2], "total": rays_per_frame},
        "roofline": roof,
        "roofline_hbm": roof_hbm,
        # the reference's brute-force work (16 FP64 ops per sphere test, 14 per plane ...)
        # per single-stream launch: what the BVH and f32 pre-filter save, NOT a utilisation figure
        "reference_equivalent_fp64_tops": round(ref_equiv, 3),
    }
    if rccl is not None:
        res["rccl_nranks"] = rccl["nranks"]
        res["rccl"] = rccl
    if bvh.enabled:
        res["bvh"] = {"nodes": bvh.nodes, "leaves": bvh.leaves, "depth": bvh.depth,
                      "box_margin": round(bvh.margin, 6), "near_origin_bound": round(bvh.origin_bound, 3)}
    if verified is not None:
        res["verified_against_1_rank_frame"] = verified
    if world > 1 or args.rccl_rehearsal:
        res["per_rank"] = per_rank  # each rank's own timed-loop ms per frame and single-launch share time
    if cpu:
        res["cpu_baseline"] = cpu_baseline(scene, W, H)
        res["gpu_over_cpu"] = round(value / res["cpu_baseline"]["value"], 1)
    return res


HV_INSTANCES = 3  # scene instances the pinned host-visible frame is timed on (median reported)


def host_visible(workload: str, args, dev, W: int = 3840, H: int = 2160, budget_s: float = 2.0):
    """The drop-in itself: rg_render_image (rendering.rs:24-38) returns the frame
    in HOST memory.  Timed back to back into a page-locked buffer
    (rg_host_register: heavy scenes render in one launch whose pixel stores
    go over PCIe straight into it; others in row bands whose DMA copies land
    in it directly while later bands render) and into a pageable one (banded,
    pinned staging + a parallel host copy).  PCIe alone: 33 MB per 4K frame at
    the measured 56 GB/s = 0.59 ms (profiles/r02/host_visible/d2h_probe.jsonl)."""
    import numpy as np
    import torch

    from raingun_amd import _abi
    from raingun_amd.scene import DeviceScene

    scene, label, _, _, _ = load_workload(workload, W, H)
    ds = DeviceScene(scene, device=dev.index or 0)
    st = _abi.rg_stats()
    ref = ds.render_image(W, H, stats=st)
    rays = st.rays.primary + st.rays.shadow + st.rays.secondary
    res = {"workload": label, "basis": "rg_render_image back to back: frame in host memory when each call returns "
                                       "(PCIe included; scene already in HBM); pinned: the median of "
                                       f"{HV_INSTANCES} scene instances"}

    def frames(d, buf, budget):
        for _ in range(3):
            d.render_image(W, H, out=buf)
        n, t0 = 0, time.perf_counter()
        while n < 5 or (time.perf_counter() - t0 < budget and n < args.steps):
            d.render_image(W, H, out=buf)
            n += 1
        dt = (time.perf_counter() - t0) / n
        if not np.array_equal(buf, ref):
            raise SystemExit("host_visible: frame differs from the first render")
        return dt, n

    def line(dt, n):
        return {"value": round(rays / dt / 1e6, 3), "ms_per_step": round(dt * 1e3, 4), "frames": n,
                "frame_bytes": H * W * 4, "host_GBps": round(H * W * 4 / dt / 1e9, 2)}

    # Pinned: one DeviceScene instance can run its host frame ~12 % slower than another of the same
    # scene in the same process -- 1 instance in 4 on the north star, the same instance every time
    # it is timed, with its device-resident launch unchanged (profiles/r06/s20-s22; most likely the
    # hardware queue its streams land on) -- so the frame is timed on HV_INSTANCES instances
    buf = np.empty((H, W, 4), dtype=np.uint8)
    reg = _abi.HostRegistration(buf)
    inst = []
    try:
        for i in range(HV_INSTANCES):
            d = ds if i == 0 else DeviceScene(scene, device=dev.index or 0)
            try:
                inst.append(frames(d, buf, budget_s / HV_INSTANCES))
            finally:
                if d is not ds:
                    d.close()
    finally:
        reg.close()
    med = sorted(inst)[len(inst) // 2]
    res["pinned"] = line(*med)
    res["pinned"]["instances_ms"] = [round(dt * 1e3, 4) for dt, _ in inst]
    buf = np.empty((H, W, 4), dtype=np.uint8)
    res["pageable"] = line(*frames(ds, buf, budget_s))
    res["multi_8gpu_rehearsal"] = multi_rehearsal(ds, W, H, res["pinned"]["ms_per_step"], args, split=True)
    ds.close()
    torch.cuda.synchronize(dev)
    res["value"] = res["pinned"]["value"]
    res["ms_per_step"] = res["pinned"]["ms_per_step"]
    res["unit"] = "Mrays/s"
    return res


def multi_rehearsal(ds, W: int, H: int, one_gpu_ms: float, args, n: int = 8, budget_s: float = 0.5,
                    split: bool = False):
    """rg_render_multi's host-visible frame on an n-GPU node, rehearsed on one GPU: each device's
    timeline -- its 8-row tiles rendered as ONE launch whose kernel stores the finished rows over
    ITS OWN PCIe link straight into the caller's page-locked buffer (rg_multi.hip render_direct_one;
    light scenes since round 6, trace-heavy scenes since round 4) -- timed alone (rg_debug_set_multi
    stand-in, only_rank = r) for every r.  The frame is done when the slowest device is: projected
    frame time = max over r.  A projection (this GPU's link stands for each device's own; host
    memory bandwidth assumed to take n links at once), not a measurement.  split: also time, per
    device, its share rendered device-resident (one launch, HIP events: `render_ms`) and one D2H copy
    of that many rows into pinned memory (`copy_ms`); overlap = render + copy - timeline."""
    import numpy as np
    import torch

    from raingun_amd import _abi

    buf = np.empty((H, W, 4), dtype=np.uint8)
    reg = _abi.HostRegistration(buf)
    per_rank, render, copy = [], [], []
    lib = _abi.lib()
    try:
        for r in range(n):
            ds.set_multi(0, stand_in=True, bands=0, only_rank=r)
            for _ in range(2):
                ds.render_multi(W, H, n, 8, out=buf)
            # the median call: one host hiccup (the box's other work) must not decide a device's time
            times, t0 = [], time.perf_counter()
            while len(times) < 5 or (time.perf_counter() - t0 < budget_s and len(times) < args.steps):
                t1 = time.perf_counter()
                ds.render_multi(W, H, n, 8, out=buf)
                times.append(time.perf_counter() - t1)
            per_rank.append(float(np.median(times)) * 1e3)
            if split:
                t = _abi.rg_tiling(8, n, r)
                rows = lib.rg_tiling_rows(H, C.byref(t))
                part = torch.empty((rows, W, 4), dtype=torch.uint8, device="cuda")
                host = torch.empty((rows, W, 4), dtype=torch.uint8, pin_memory=True)
                st = _abi.rg_stats()
                ks = []
                for i in range(7):
                    _abi.check(lib.rg_render_tiles_async(ds.handle, W, H, C.byref(t), C.c_void_p(part.data_ptr()),
                                                         None, None, C.byref(st)))
                    if i >= 2:
                        ks.append(st.kernel_ms)
                render.append(float(np.median(ks)))
                cs = []
                for i in range(7):
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    host.copy_(part, non_blocking=True)
                    e1.record()
                    e1.synchronize()
                    if i >= 2:
                        cs.append(e0.elapsed_time(e1))
                copy.append(float(np.median(cs)))
    finally:
        ds.set_multi(0, stand_in=False, bands=0, only_rank=-1)
        reg.close()
    proj = max(per_rank)
    out = {"projected_ms_per_step": round(proj, 4), "projected_speedup_vs_1gpu": round(one_gpu_ms / proj, 2),
           "per_device_ms": [round(x, 4) for x in per_rank], "n_gpus": n,
           "basis": "one GPU times each device's rg_render_multi timeline alone (its 8-row tiles as one launch "
                    "storing its rows into the pinned caller buffer over its own link); projected frame = the "
                    "slowest device"}
    if split:
        out["per_device_split"] = [{"timeline_ms": round(tl, 4), "render_ms": round(rm, 4), "copy_ms": round(cm, 4),
                                    "overlap_ms": round(rm + cm - tl, 4)}
                                   for tl, rm, cm in zip(per_rank, render, copy)]
    return out


# Extra line items: (key, workload, size, CPU baseline?) -- BASELINE configs[2..4] and the north_star scene.
EXTRA_LINES = [
    ("test3_4k", "test3", (3840, 2160), True),                         # configs[2]
    ("north_star_1024_spheres", "synth1024", (3840, 2160), True),      # north_star: 1024 spheres, 4K, depth 5
    ("north_star_1024_spheres_8k", "synth1024", (7680, 4320), False),  # configs[3] (CPU rate: the 4K line's scene)
    ("synth4096_16k", "synth4096p8d8", (16384, 16384), True),          # configs[4]
]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def parse_args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node (one process each).  Outside a launcher, N > 1 starts "
                         "torch.distributed.run with N ranks itself; inside one it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="test1", help="test1 | test3 | synth<N>[p<planes>][d<depth>]")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-north-star", "--no-extra", dest="no_extra", action="store_true",
                    help="skip the extra line items (configs[2..4], the north_star scene, host_visible)")
    ap.add_argument("--extra", default="",
                    help="comma-separated subset of the extra lines to run (test3_4k, north_star_1024_spheres, "
                         "north_star_1024_spheres_8k, synth4096_16k, host_visible, host_visible_north_star); "
                         "default all")
    ap.add_argument("--extra-budget", type=float, default=3.0,
                    help="seconds of timed frames per extra line (at least 3 frames, at most --steps)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL; gloo: rehearsal)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal: every rank renders on GPU 0 (use with --backend gloo)")
    ap.add_argument("--frames-in-flight", type=int, default=0,
                    help="frames in flight, each on its own render stream (N>1: their gathers overlap later renders); "
                         "0 = 8")
    ap.add_argument("--reuse-streams", action=argparse.BooleanOptionalAction, default=True,
                    help="every line's frames in flight on the same render streams, made once per process "
                         "(--no-reuse-streams: new streams per line)")
    ap.add_argument("--one-render-stream", action="store_true",
                    help="render every frame on one stream (N>1: only the gathers overlap the renders)")
    ap.add_argument("--settle-s", type=float, default=0.3,
                    help="seconds of untimed frames before the warm-up steps (steady GPU clocks)")
    ap.add_argument("--roofline-frames", type=int, default=10,
                    help="single-stream launches timed after the timed region (kernel_ms)")
    ap.add_argument("--rccl-rehearsal", action="store_true",
                    help="N=1: run the N>1 path anyway (RCCL process group, per-frame gather, re-interleave)")
    ap.add_argument("--python-pipeline", action="store_true",
                    help="N>1: run the per-frame loop in Python (raingun_amd.distributed.FramePipeline)")
    ap.add_argument("--tile-rows", type=int, default=8,
                    help="rows per interleaved row tile of the N-way split (8: the slowest of 8 shares is 2-4 %% "
                         "faster than with 16, profiles/r01/bench_rank_shares.txt)")
    ap.add_argument("--share-rank", type=int, default=0, help="diagnostic: which rank's share --share times")
    ap.add_argument("--rank0-share", type=int, default=1,
                    help="N > 1: tiles of rank 0 per period of R + N - 1 (rank 0's rows never cross xGMI; "
                         "1 = round robin; include/raingun_frames.h rg_frames_set_root_tiles)")
    ap.add_argument("--depth", type=int, default=None, help="diagnostic: override the workload's recursion depth")
    ap.add_argument("--lane-depth", type=int, default=None,
                    help="diagnostic: rays at recursion depth >= this walk the BVH per lane (rg_debug_set_lane_depth)")
    ap.add_argument("--tile-order", type=int, default=-1,
                    help="diagnostic: 1 = probe-ordered tiles, 0 = raster order, -1 = library default")
    ap.add_argument("--share", type=int, default=1,
                    help="diagnostic at N=1: time rank 0's share of an S-way split (no gather); value counts its rays")
    ap.add_argument("--verify", action="store_true",
                    help="rank 0 checks the frame against a 1-rank render, byte for byte (always at N > 1 and "
                         "with --rccl-rehearsal; this flag adds it at N = 1)")
    ap.add_argument("--plan", action="store_true",
                    help="print this rank's launch plan (rank, world, device) as JSON and exit before any GPU work")
    return ap.parse_args(argv)


def main() -> None:
    args = parse_args()

    # One process per GPU.  `--gpus N` outside a launcher: start torch.distributed.run
    # with N ranks on this node as a CHILD process (nothing here has touched the GPU
    # yet) and exit with its status; inside a launcher WORLD_SIZE must agree.
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve()),
               *sys.argv[1:]]
        sys.exit(subprocess.call(cmd))
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one process per GPU "
                         f"(torchrun --nproc-per-node {args.gpus}) or drop --gpus")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device:
        local_rank = 0
    if args.plan:
        line = {"rank": rank, "world": world, "local_rank": local_rank, "n_gpus": world,
                "verify_against_1_rank_frame": verify_enabled(args, world)}
        if args.backend == "gloo" and world > 1:  # rehearse the rendezvous without a GPU
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")
            dist.barrier()
            dist.destroy_process_group()
        os.write(1, (json.dumps(line) + "\n").encode())  # one write: the ranks share stdout
        return

    # the JSON line is the only thing on stdout: library banners (RCCL prints its
    # version block on stdout when a communicator is created) go to stderr
    json_out = os.fdopen(os.dup(1), "w")
    # frames in flight need a hardware queue per render stream next to RCCL's
    # stream and rank 0's re-interleave stream (HIP's default is 4 per process)
    # (the GPU box exports HIP's default, 4, so raise it rather than default it)
    # 8 render streams + RCCL's + the communication and side streams + the null stream
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 16:
        os.environ["GPU_MAX_HW_QUEUES"] = "16"
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    if world > 1 or args.rccl_rehearsal:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        torch.cuda.set_device(local_rank)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(args.backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local_rank)
    cpu = (not args.no_cpu_baseline) and world == 1

    main_res = measure(args.workload, args, world, rank, local_rank, dev, cpu)
    extras = {}
    if not args.no_extra:
        want = set(filter(None, args.extra.split(","))) or None
        for key, wl, size, with_cpu in EXTRA_LINES:
            if want is not None and key not in want:
                continue
            if (wl, size) == (args.workload, (args.width, args.height)):
                continue
            warm = 2 if size[0] * size[1] >= 100_000_000 else min(args.warmup, 5)
            extras[key] = measure(wl, args, world, rank, local_rank, dev, cpu and with_cpu, size=size,
                                  warmup=warm, budget_s=args.extra_budget)
        if world == 1 and (want is None or "host_visible" in want):
            extras["host_visible"] = host_visible(args.workload, args, dev, args.width, args.height)
        if world == 1 and (want is None or "host_visible_north_star" in want) and args.workload != "synth1024":
            extras["host_visible_north_star"] = host_visible("synth1024", args, dev, 3840, 2160)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": main_res["value"],
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": main_res["ms_per_step"],
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
        }
        line.update({k: v for k, v in main_res.items() if k not in ("value", "ms_per_step", "steps", "warmup")})
        line.update(extras)
        print(json.dumps(line), file=json_out, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
