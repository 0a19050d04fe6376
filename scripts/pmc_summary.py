#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (scripts/pmc.sh) for rg_render_kernel:
mean per dispatch of every counter, plus derived quantities.  Writes
profiles/<round>/pmc/<workload>.json and updates profiles/traffic.json.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE counts half the bytes of wide coalesced
streaming reads (x2 correction applied as an upper bound and reported beside
the raw value); WRITE_SIZE is exact for 16-B/lane stores, uncalibrated for the
4-B/lane RGBA stores used here."""
import collections, csv, glob, json, sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def load(workload, root):
    agg = {}
    for f in sorted(glob.glob(f"{root}/pmc_{workload}/p*/run_counter_collection.csv")):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if "rg_render_kernel" in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        byc = collections.defaultdict(list)
        for (_, c), v in per.items():
            byc[c].append(v)
        for c, vs in byc.items():
            agg[c] = sum(vs) / len(vs)
    return agg


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    root = sys.argv[2] if len(sys.argv) > 2 else str(REPO / "gpurun_out")
    traffic_f = REPO / "profiles" / "traffic.json"
    traffic = json.loads(traffic_f.read_text()) if traffic_f.exists() else {}
    for w in ("test1", "synth1024"):
        a = load(w, root)
        if not a:
            continue
        d = {"counters_mean_per_dispatch": a}
        f64 = sum(a.get(k, 0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                       "SQ_INSTS_VALU_TRANS_F64"))
        d["derived"] = {
            "fp64_valu_instructions": f64,
            "fp64_share_of_valu": f64 / a["SQ_INSTS_VALU"] if a.get("SQ_INSTS_VALU") else None,
            "salu_per_valu": a.get("SQ_INSTS_SALU", 0) / a["SQ_INSTS_VALU"] if a.get("SQ_INSTS_VALU") else None,
            "wave_time_waiting_on_memory": a.get("SQ_WAIT_ANY", 0) / a["SQ_WAVE_CYCLES"] if a.get("SQ_WAVE_CYCLES") else None,
            "wave_time_issue_stalled": a.get("SQ_WAIT_INST_ANY", 0) / a["SQ_WAVE_CYCLES"] if a.get("SQ_WAVE_CYCLES") else None,
            "wave_time_issuing": a.get("SQ_ACTIVE_INST_ANY", 0) / a["SQ_WAVE_CYCLES"] if a.get("SQ_WAVE_CYCLES") else None,
            "fetch_bytes_raw": a.get("FETCH_SIZE", 0) * 1024,
            "write_bytes": a.get("WRITE_SIZE", 0) * 1024,
            "hbm_bytes_per_launch": (a.get("FETCH_SIZE", 0) * 2 + a.get("WRITE_SIZE", 0)) * 1024,
            # VALU pipe utilisation: 4 cycles per wave64 VALU instruction on a 16-lane SIMD, over
            # 1,024 SIMDs x kernel cycles (SQ_BUSY_CYCLES is summed over the 32 shader engines)
            "valu_busy": (a["SQ_INSTS_VALU"] * 4.0 / (1024.0 * a["SQ_BUSY_CYCLES"] / 32.0)
                          if a.get("SQ_INSTS_VALU") and a.get("SQ_BUSY_CYCLES") else None),
            "lds_active": (a["SQ_LDS_IDX_ACTIVE"] / 256.0 / (a["SQ_BUSY_CYCLES"] / 32.0)
                           if a.get("SQ_LDS_IDX_ACTIVE") and a.get("SQ_BUSY_CYCLES") else None),
        }
        out = REPO / "profiles" / rnd / "pmc"
        out.mkdir(parents=True, exist_ok=True)
        (out / f"{w}.json").write_text(json.dumps(d, indent=1) + "\n")
        traffic[w] = {"hbm_bytes_per_launch": d["derived"]["hbm_bytes_per_launch"],
                      "valu_busy": d["derived"]["valu_busy"],
                      "source": f"profiles/{rnd}/pmc/{w}.json (FETCH_SIZE x2 + WRITE_SIZE, KiB->B; "
                                f"valu_busy = SQ_INSTS_VALU x 4 / (1024 SIMDs x SQ_BUSY_CYCLES / 32))"}
        print(w, json.dumps(d["derived"], indent=1))
    traffic_f.write_text(json.dumps(traffic, indent=1) + "\n")


if __name__ == "__main__":
    main()
