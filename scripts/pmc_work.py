#!/usr/bin/env python3
"""Summarise scripts/pmc_work.sh runs into profiles/pmc_work.json (read by
bench.py's `roofline`) and profiles/<round>/pmcw/<tag>.json.

Per frame = summed over every rg_* kernel dispatch of the run (render kernel +
the heavy path's tile-order probe/count/scan/scatter), divided by the number
of rg_render_kernel dispatches (every frame launches the same set).

VALU issue cycles per frame (MI355X_MICROARCH.md: a wave64 VALU instruction
issues over 2 cycles on a 32-lane SIMD; FP64 runs at half that lane rate, 4
cycles; f32 transcendentals 4):  4 x FP64 (ADD+MUL+FMA+TRANS) + 4 x TRANS_F32
+ 2 x the rest.  FP64 compares, min/max, div-scale/fixup and conversions are
not in the FP64 counters and are priced at 2: a lower bound on the cycles.

HBM bytes per frame: FETCH_SIZE x 2 + WRITE_SIZE, KiB -> B (gfx950
correction of MI355X_MICROARCH.md §HBM, an upper bound for FETCH).

The kernel trace of the same command at the bench's timed configuration
(frames in flight) gives each launch's start/end; the union of all rg_*
kernel intervals over the timed frames, per frame, is the GPU-busy time per
frame, to compare with the bench line's ms_per_step."""
import collections
import csv
import glob
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")


def counters(tagdir):
    tot = collections.defaultdict(float)
    frames = {}
    for f in sorted(glob.glob(f"{tagdir}/p*/run_counter_collection.csv")):
        renders = set()
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not name.startswith("void rg_") and not name.startswith("rg_"):
                continue
            if "rg_render_kernel" in name:
                renders.add(r["Dispatch_Id"])
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
        for c in {r["Counter_Name"] for r in csv.DictReader(open(f))}:
            frames[c] = len(renders)
    return {c: v / frames[c] for c, v in tot.items() if frames.get(c)}


def trace_union(tagdir, steps, tail=1):
    rows = [r for r in csv.DictReader(open(f"{tagdir}/trace/run_kernel_trace.csv")) if "rg_" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    render = [r for r in rows if "rg_render_kernel" in r["Kernel_Name"]]
    # bench order: 1 counted render, settle frames, warm-up frames, `steps` timed frames, then
    # `tail` single-stream launches (--roofline-frames, 1 in scripts/pmc_work.sh)
    timed = render[len(render) - tail - steps:len(render) - tail]
    lo_id = int(render[len(render) - tail - steps - 1]["Dispatch_Id"]) + 1  # after the last untimed frame
    hi_id = int(timed[-1]["Dispatch_Id"])
    ivs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                 if lo_id <= int(r["Dispatch_Id"]) <= hi_id)
    busy, cur_s, cur_e = 0, None, None
    for s, e in ivs:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = max(e for _, e in ivs) - min(s for s, _ in ivs)
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed]
    return {"timed_frames": len(timed), "busy_ms_per_frame": busy / len(timed) / 1e6,
            "span_ms_per_frame": span / len(timed) / 1e6,
            "render_launch_mean_ms_overlapped": sum(durs) / len(durs) / 1e6,
            "kernel_name": timed[0]["Kernel_Name"]}


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r02"
    root = Path(sys.argv[2]) if len(sys.argv) > 2 else REPO / "gpurun_out" / "pmcw"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    out_f = REPO / "profiles" / "pmc_work.json"
    work = json.loads(out_f.read_text()) if out_f.exists() else {}
    for tagdir in sorted(root.iterdir()):
        tag = tagdir.name                       # <workload>_<W>x<H>
        wl, size = tag.rsplit("_", 1)
        a = counters(tagdir)
        if not a.get("SQ_INSTS_VALU"):
            continue
        f64 = sum(a.get(k, 0.0) for k in F64)
        t32 = a.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
        valu = a["SQ_INSTS_VALU"]
        cyc = 4.0 * f64 + 4.0 * t32 + 2.0 * (valu - f64 - t32)
        d = {"counters_per_frame": a,
             "valu_insts_per_frame": valu, "f64_insts_per_frame": f64, "trans32_insts_per_frame": t32,
             "valu_cycles_per_frame": cyc,
             "hbm_bytes_per_frame": (2.0 * a.get("FETCH_SIZE", 0.0) + a.get("WRITE_SIZE", 0.0)) * 1024.0,
             "fp64_share_of_valu": f64 / valu,
             "wave_time_waiting": a.get("SQ_WAIT_ANY", 0) / a["SQ_WAVE_CYCLES"] if a.get("SQ_WAVE_CYCLES") else None,
             "wave_time_issuing": (a.get("SQ_ACTIVE_INST_ANY", 0) / a["SQ_WAVE_CYCLES"]
                                   if a.get("SQ_WAVE_CYCLES") else None)}
        bj = tagdir / "trace.json"
        b = json.loads(bj.read_text().strip().splitlines()[-1]) if bj.exists() and bj.read_text().strip() else {}
        try:
            d["trace"] = trace_union(tagdir, b.get("steps", steps))
        except Exception as e:  # noqa: BLE001
            d["trace"] = {"error": str(e)}
        if b:
            d["bench_ms_per_step_under_trace"] = b["ms_per_step"]
            d["bench_kernel_ms_single_stream"] = b.get("kernel_ms")
        d["source"] = f"profiles/{rnd}/pmcw/{tag}.json (scripts/pmc_work.sh: rocprofv3 --pmc, the bench's frames in flight)"
        dst = REPO / "profiles" / rnd / "pmcw"
        dst.mkdir(parents=True, exist_ok=True)
        (dst / f"{tag}.json").write_text(json.dumps(d, indent=1) + "\n")
        work[f"{wl}@{size}"] = {k: d[k] for k in ("valu_insts_per_frame", "f64_insts_per_frame",
                                                  "trans32_insts_per_frame", "valu_cycles_per_frame",
                                                  "hbm_bytes_per_frame", "source")}
        work[f"{wl}@{size}"]["fetch_write_kib_per_frame"] = [a.get("FETCH_SIZE"), a.get("WRITE_SIZE")]
        print(tag, json.dumps({k: v for k, v in d.items() if k != "counters_per_frame"}, indent=1))
    out_f.write_text(json.dumps(work, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
