#!/usr/bin/env python3
"""Benchmark: Mrays/s of the per-pixel ray-trace path (BASELINE.json metric).

One step = one frame of the workload rendered by the HIP megakernel, scene and
textures already resident in HBM, framebuffer left in HBM (rank 0 holds the
assembled frame).  At N>1 (torchrun, one rank per GPU) the frame is cut into
8-row tiles dealt round-robin to the ranks and the tiles are gathered to rank
0 with one RCCL gather per frame (ncclGather on the communicator of the
torch.distributed "nccl" group, i.e. RCCL over xGMI), then re-interleaved into
image order on rank 0 -- the per-frame loop runs in C++ (include/raingun_frames.h).

Workload (BASELINE.json configs[1]): examples/test1.yml at 3840x2160,
recursion depth 5, 1 GPU.  `--workload synth1024` selects the north_star's
1024-sphere 3840x2160 depth-5 scene instead.  Two extra line items report the
north_star scene at 3840x2160 and at 7680x4320 (BASELINE configs[3]) on the
same N GPUs.  Frames are kept in flight (4, each on its own render stream):
the timed region holds `--steps` complete frames.

Prints ONE JSON line on rank 0 (the driver's contract) with `roofline`
(FP64-VALU bound, from HIP events on the render stream), `roofline_hbm`
(achieved HBM bytes, as the north_star asks) and `cpu_baseline` (the CPU
restatement in oracle/, timed on this host's cores on a bounded sample).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

METRIC = "Mrays/sec (primary+shadow+secondary) at 3840×2160, depth 5; 1/2/4/8 MI355X"
FP64_PEAK_TOPS = 39.3     # MI355X FP64 vector 78.6 TFLOP/s spec counts FMA as 2; parity forbids FMA -> 39.3 T ops/s
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
        n = int(name[5:] or 1024)
        text = synthetic_yaml(n, 2, 5)
        scene = load_scene(text)
        label = f"synthetic {n} spheres + 2 planes {W}x{H} depth 5 (seed 0x5EED, md5 {scene_md5(text)})"
        if (W, H) == (7680, 4320):
            label += " (BASELINE configs[3])"
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
    stride = 1  # first probe: the whole frame
    while True:
        t0 = time.perf_counter()
        st, _, _, counts, _ = oracle.render(desc, width, height, TILE_ROWS, stride, 0, threads=threads)
        dt = time.perf_counter() - t0
        if st != 0:
            raise RuntimeError(f"oracle status {st}")
        if dt * stride <= budget_s or stride >= tiles:
            break
        stride = min(tiles, int(stride * (dt * stride / budget_s)) + 1)
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


def load_traffic(workload: str, n_gpus: int, key: str = "hbm_bytes_per_launch"):
    """A PMC figure for this workload's kernel (scripts/pmc.sh -> profiles/traffic.json)."""
    f = REPO / "profiles" / "traffic.json"
    if n_gpus != 1 or not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        return d.get(workload, {}).get(key)
    except Exception:
        return None


def measure(workload: str, args, world: int, rank: int, local_rank: int, dev, cpu: bool, size=None):
    """Time `args.steps` frames of `workload` on this rank (after `args.warmup`),
    frame sharded over `world` ranks and gathered to rank 0.  Returns the
    rank-0 result dict (None on other ranks)."""
    import torch
    import torch.distributed as dist

    from raingun_amd import _abi
    from raingun_amd import distributed as rd
    from raingun_amd.scene import DeviceScene

    W, H = size or (args.width, args.height)
    scene, label, src, body_counts, ops_per_ray = load_workload(workload, W, H)
    ds = DeviceScene(scene, device=local_rank)  # scene + textures uploaded once, resident in HBM
    if args.tile_order >= 0:
        ds.set_tile_order(args.tile_order)
    lib = _abi.lib()
    bvh = ds.bvh_info()

    # --share S (diagnostic, N = 1): render only rank 0's tiles of an S-way split
    split = args.share if (world == 1 and args.share > 1) else world
    TR = args.tile_rows  # rows per interleaved row tile (rank t % N renders tile t)
    tiling = rd.tiling(args.share_rank if split != world else rank, split, TR)
    my_rows = lib.rg_tiling_rows(H, C.byref(tiling))
    slot = rd.slot_rows(H, split, TR)  # equal-size gather slots (last ranks zero-padded)
    out = torch.zeros((slot, W, 4), dtype=torch.uint8, device=dev)
    # frames in flight, each on its own render stream and hardware queue (12 per
    # process, see main): 6 -- the whole frame is flat from 4 up, a 1/8 test1
    # share gains 12 % from 4 to 6 (profiles/r01/bench_frames_in_flight_ab.txt)
    F = args.frames_in_flight if args.frames_in_flight > 0 else 6
    use_pipe = args.backend == "nccl" or world == 1
    gathered = rd.gather_buffers(out, world) if (world > 1 and rank == 0 and not use_pipe) else None
    frame = torch.empty((H, W, 4), dtype=torch.uint8, device=dev) if (rank == 0 and not use_pipe) else None

    stream = torch.cuda.current_stream(dev)
    sh = C.c_void_p(stream.cuda_stream)

    def render(stats=None, buf=None):
        # on the current stream: the frame pipeline's render stream for this frame, or the default
        dst = out if buf is None else buf
        cur = torch.cuda.current_stream(dev)
        sh_cur = sh if cur == stream else C.c_void_p(cur.cuda_stream)
        st = lib.rg_render_tiles_async(ds.handle, W, H, C.byref(tiling), C.c_void_p(dst.data_ptr()), None, sh_cur,
                                       C.byref(stats) if stats is not None else None)
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
    if native:  # the per-frame loop in C++ (include/raingun_frames.h): render, ncclGather, re-interleave
        try:
            pipe = rd.NativeFramePipeline(ds.handle, W, H, rank, world, TR, depth=F, device=dev)
        except Exception as e:  # e.g. no communicator pointer from this torch build: same loop in Python
            print(f"[bench] native frame pipeline unavailable ({e}); using the Python loop", file=sys.stderr)
            native = False
    if not native and use_pipe:
        pipe = rd.FramePipeline((slot, W, 4), H, rank, world, TR, device=dev, depth=F,
                                streams=F > 1 and not args.one_render_stream, gather=gather)

    def step():
        if native:
            pipe.step()
        elif pipe is not None:
            pipe.step(lambda part: render(buf=part))
        else:
            rd.render_frame(render_tiles, H, rank, world, TR, out=frame, gather_bufs=gathered)

    def finish():
        if pipe is not None:
            pipe.flush()

    # one counted render: ray totals per class (deterministic per frame)
    stats = _abi.rg_stats()
    render(stats)
    rays = torch.tensor([stats.rays.primary, stats.rays.shadow, stats.rays.secondary], dtype=torch.float64,
                        device=dev)
    if world > 1:
        dist.all_reduce(rays)
    rays = [int(x) for x in rays.tolist()]
    rays_per_frame = sum(rays)

    for _ in range(args.warmup):
        step()
    finish()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    finish()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0

    # Roofline timing: with frames in flight a launch's start-to-end time
    # includes the CUs it shares with its neighbours, so the kernel time of one
    # launch is measured on its own: this rank's share, one launch after
    # another on one stream, HIP events on that stream (rocprofv3 of
    # `bench.py --frames-in-flight 1` gives the same average: profiles/).
    events = []
    for _ in range(max(1, args.roofline_frames)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        render()
        e1.record(stream)
        events.append((e0, e1))
    torch.cuda.synchronize(dev)
    kernel_ms = sum(e0.elapsed_time(e1) for e0, e1 in events) / len(events)

    tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt[0])
    verified = None
    if getattr(args, "verify", False):
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
            verified = bool((got == ref).all())
            if not verified:
                raise SystemExit(f"--verify: the {world}-rank frame differs from the 1-rank render")
    if native:
        pipe.close()
    ds.close()
    if rank != 0:
        return None

    if world > 1:
        via = "RCCL" if args.backend == "nccl" else f"{args.backend} (rehearsal, through host memory)"
        parallelism = f"row-tiles x{world} (round-robin {TR}-row tiles, one {via} gather per frame to rank 0"
    else:
        parallelism = "one GPU (whole frame"
    if native:
        parallelism += f", {F} frames in flight on {F} render streams; per-frame loop in C++, raingun_frames.h)"
    elif pipe is not None and pipe.streams:
        parallelism += f", {F} frames in flight on {F} render streams)"
    else:
        parallelism += ", frames rendered one after another on one stream)"
    ms_per_step = elapsed * 1e3 / args.steps
    value = rays_per_frame * args.steps / elapsed / 1e6
    my_rays = stats.rays.primary + stats.rays.shadow + stats.rays.secondary
    ops = my_rays * ops_per_ray
    achieved_t = ops / (kernel_ms * 1e-3) / 1e12
    alg_bytes = my_rows * W * 4  # framebuffer written once; scene/texture reads are cache-resident re-reads
    tex = texture_bytes(scene)
    traffic = load_traffic(workload, world)
    res = {
        "value": round(value, 3),
        "ms_per_step": round(ms_per_step, 4),
        "kernel_ms": round(kernel_ms, 4),
        "data": src,
        "config": {"workload": label, "width": W, "height": H, "max_recursion_depth": scene.max_recursion_depth,
                   "bodies": body_counts, "lights": len(scene.lights), "tile_rows": TR,
                   "parallelism": parallelism},
        "rays_per_frame": {"primary": rays[0], "shadow": rays[1], "secondary": rays[2], "total": rays_per_frame},
        "roofline": {
            "bound": "valu_fp64",
            "achieved": round(achieved_t, 4),
            "peak": FP64_PEAK_TOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved_t / FP64_PEAK_TOPS, 5),
            "traffic": traffic,
            "valu_busy_pmc": load_traffic(workload, world, "valu_busy") if (W, H) == (3840, 2160) else None,
            "basis": f"reference-equivalent work: {ops_per_ray} FP64 ops per ray (16/sphere, 14/plane, 20/disk, "
                     f"18/aabb; SURVEY.md 8d) x {my_rays} rays per launch / mean rg_render_kernel time (HIP events "
                     f"around {max(1, args.roofline_frames)} single-stream launches after the timed region)" + (
                         ". The sphere BVH and f32 pre-filter skip most of that work without changing any result, "
                         "so frac > 1 measures the algorithmic saving over the brute-force scan, not hardware "
                         "utilisation (DESIGN.md 4b)" if bvh.enabled else ""),
        },
        "roofline_hbm": {
            "bound": "hbm",
            "achieved": round(alg_bytes / (kernel_ms * 1e-3) / 1e9, 3),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(alg_bytes / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 7),
            "traffic": traffic,
            "basis": f"{alg_bytes} B framebuffer written per launch (+{tex} B of textures, L2/MALL resident)",
        },
    }
    if bvh.enabled:
        res["bvh"] = {"nodes": bvh.nodes, "leaves": bvh.leaves, "depth": bvh.depth,
                      "box_margin": round(bvh.margin, 6), "near_origin_bound": round(bvh.origin_bound, 3)}
    if verified is not None:
        res["verified_against_1_rank_frame"] = verified
    if cpu:
        res["cpu_baseline"] = cpu_baseline(scene, W, H)
        res["gpu_over_cpu"] = round(value / res["cpu_baseline"]["value"], 1)
    return res


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="test1", help="test1 | test3 | synth<N>")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-north-star", action="store_true",
                    help="skip the extra north_star line items (1024 spheres, depth 5, 3840x2160 and 7680x4320)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL; gloo: rehearsal)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal: every rank renders on GPU 0 (use with --backend gloo)")
    ap.add_argument("--frames-in-flight", type=int, default=0,
                    help="frames in flight, each on its own render stream (N>1: their gathers overlap later renders); "
                         "0 = 6")
    ap.add_argument("--one-render-stream", action="store_true",
                    help="render every frame on one stream (N>1: only the gathers overlap the renders)")
    ap.add_argument("--roofline-frames", type=int, default=10,
                    help="single-stream launches timed after the timed region for the roofline's kernel time")
    ap.add_argument("--rccl-rehearsal", action="store_true",
                    help="N=1: run the N>1 path anyway (RCCL process group, per-frame gather, re-interleave)")
    ap.add_argument("--python-pipeline", action="store_true",
                    help="N>1: run the per-frame loop in Python (raingun_amd.distributed.FramePipeline)")
    ap.add_argument("--tile-rows", type=int, default=8,
                    help="rows per interleaved row tile of the N-way split (8: the slowest of 8 shares is 2-4 %% "
                         "faster than with 16, profiles/r01/bench_rank_shares.txt)")
    ap.add_argument("--share-rank", type=int, default=0, help="diagnostic: which rank's share --share times")
    ap.add_argument("--tile-order", type=int, default=-1,
                    help="diagnostic: 1 = probe-ordered tiles, 0 = raster order, -1 = library default")
    ap.add_argument("--share", type=int, default=1,
                    help="diagnostic at N=1: time rank 0's share of an S-way split (no gather); value counts its rays")
    ap.add_argument("--verify", action="store_true",
                    help="rank 0 checks the gathered frame against a 1-rank render, byte for byte")
    args = ap.parse_args()
    # the JSON line is the only thing on stdout: library banners (RCCL prints its
    # version block on stdout when a communicator is created) go to stderr
    json_out = os.fdopen(os.dup(1), "w")
    # frames in flight need a hardware queue per render stream next to RCCL's
    # stream and rank 0's re-interleave stream (HIP's default is 4 per process)
    # (the GPU box exports HIP's default, 4, so raise it rather than default it)
    # 6 render streams + RCCL's + the communication and side streams + the null stream
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 12:
        os.environ["GPU_MAX_HW_QUEUES"] = "12"
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device:
        local_rank = 0
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
    ns_res = ns8k_res = None
    if not args.no_north_star and args.workload != "synth1024":
        ns_res = measure("synth1024", args, world, rank, local_rank, dev, cpu)
    if not args.no_north_star:
        # BASELINE configs[3]: the north-star scene at 7680x4320, row-tiled over the N GPUs
        # (the CPU rate per ray is the 3840x2160 line's: same scene, same rays per pixel)
        ns8k_res = measure("synth1024", args, world, rank, local_rank, dev, False, size=(7680, 4320))

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
        line.update({k: v for k, v in main_res.items() if k not in ("value", "ms_per_step")})
        if ns_res is not None:
            line["north_star_1024_spheres"] = ns_res
        if ns8k_res is not None:
            line["north_star_1024_spheres_8k"] = ns8k_res
        print(json.dumps(line), file=json_out, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
