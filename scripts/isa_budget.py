#!/usr/bin/env python3
"""ISA instruction budget of one rg_render_kernel instantiation, by region of the render loop.

Static side: rg_kernels.hip is compiled for gfx950 with line tables, the kernel disassembled, and
every instruction's full inline chain read back (llvm-symbolizer --inlines), so an instruction of an
inlined sqrt or dot is attributed to the call site it serves.  Regions are the RG_REGION(k) markers
of the kernel (-DRG_REGION_STATS counts how often a wave enters each): a marker's static extent is
the source block `{...}` that encloses it (brace-matched), plus a few function-level regions named
below (the sphere normal, the texel fetch, the spherical-light setup).  An instruction belongs to
the innermost region whose extent holds a frame of its chain.  Classes: FP64 (v_*_f64 and the
division helpers), f32 VALU, int VALU, moves/selects, SALU, LDS, VMEM (global/scratch).

Which binary: the -DRG_REGION_STATS build (--build stats, the default) -- the one whose visits are
counted, so visits and static instructions describe the same code; the marker instrumentation
itself (the instructions at RG_REGION lines) is left out.  The compiler unrolls loops, runtime ones
too, so a marker can exist in several copies: a region's static figure is its instructions in one
template instantiation over the marker copies that instantiation holds (each visit runs one copy).
--build prod reads the production object instead (no marker copies to divide by: unrolled regions
then show their copies' sum).  The sphere tails of the grouped miss tests (sphere_tail inlined into
sph_primary_group / sph_query_group / trace_shadow) are regions of their own (RGR_*_PAIR, a visit
per candidate (sphere, light) pair a wave runs), and raise_error is RGR_ERROR (no visits on a clean
frame).

Dynamic side (--visits region_stats.json from scripts/region_stats.py): each region's wave visits
times its static instructions = the dynamic count; the sum is reconciled with the PMC counters
(SQ_INSTS_VALU, the FP64 counters) of the same frame.

    python scripts/isa_budget.py [--kernel MANGLED] [--heavy] [--visits stats.json] [--json out.json] [hipcc flags...]
"""
import collections
import json
import re
import subprocess
import sys
from pathlib import Path

CSRC = Path(__file__).resolve().parent.parent / "raingun_amd" / "csrc"
SRC = CSRC / "rg_kernels.hip"
DEFAULT = "_Z16rg_render_kernelILi8ELb1ELb1ELi4ELi3ELb0ELb0ELb0ELi0ELb0EEv12RgKernelArgs"
LLVM = "/opt/rocm/lib/llvm/bin"
# callers of sphere_tail -> the pair region its inlined instructions belong to
PAIR_OF = {"sph_primary_group": "RGR_PRIM_PAIR", "sph_query_group": "RGR_QC_PAIR", "trace_shadow": "RGR_SH_PAIR"}
FUNCTION_REGIONS = {"RGR_NORMAL_SPHERE", "RGR_TEXEL", "RGR_UV_SPHERE", "RGR_UV_PLANE", "RGR_LIGHT_SPH"}
CLASSES = ["fp64", "valu_f32", "valu_int", "move_select", "salu", "lds", "vmem"]
VALU = CLASSES[:4]


def region_names():
    txt = SRC.read_text()
    body = txt[txt.index("RGR_LOOP = 0"):txt.index("RGR_COUNT")]
    return [n.split("=")[0].strip() for n in body.replace("\n", " ").split(",") if n.strip()]


def block_of(lines, li):
    """1-based line range of the innermost {...} block enclosing line li (brace matching)."""
    text = "\n".join(lines)
    pos = sum(len(l) + 1 for l in lines[:li - 1])
    depth, i = 0, pos
    while i > 0:  # back to the unmatched '{'
        i -= 1
        ch = text[i]
        if ch == "}":
            depth += 1
        elif ch == "{":
            if depth == 0:
                break
            depth -= 1
    start, depth, j = i, 0, i
    while j < len(text):
        if text[j] == "{":
            depth += 1
        elif text[j] == "}":
            depth -= 1
            if depth == 0:
                break
        j += 1
    return text.count("\n", 0, start) + 1, text.count("\n", 0, j) + 1


def func_at(lines, li):
    """Name of the function whose definition precedes line li."""
    fn = re.compile(r"^(?:template\s*<.*>\s*)?(?:__device__|__global__|static|void).*?\b([A-Za-z_]\w*)\s*\(")
    for k in range(li - 1, -1, -1):
        m = fn.match(lines[k])
        if m and m.group(1) not in ("if", "for", "while", "__launch_bounds__"):
            return m.group(1)
    return "?"


def regions():
    """[(region, function name, first line, last line)] -- innermost-first matching by extent size."""
    lines = SRC.read_text().splitlines()
    out = []
    for i, l in enumerate(lines, 1):
        for m in re.finditer(r"RG_REGION\((RGR_\w+)\)", l):
            name = m.group(1)
            if "#define" in l:
                continue
            stripped = l.strip()
            if stripped.startswith("if (") and not stripped.endswith("{"):
                continue  # conditional one-line markers: function-level regions below
            a, b = block_of(lines, i)
            f = func_at(lines, i)
            if f in ("rg_render_kernel",) or "rg_render_kernel" in lines[a - 1]:
                f = "rg_render_kernel"
            out.append((name, f, a, b))

    def fn_lines(fname, key_start, key_end=None):
        s = next(i for i, l in enumerate(lines, 1) if key_start in l)
        e = s if key_end is None else next(i for i, l in enumerate(lines[s - 1:], s) if key_end in l)
        return (fname, s, e)
    extra = [("RGR_NORMAL_SPHERE",) + fn_lines("surface_normal", "if (b.kind == RG_BODY_SPHERE) { n = normalize"),
             ("RGR_TEXEL",) + fn_lines("texel_fetch", "uint32_t texel_fetch(", "return tg[(size_t)y"),
             ("RGR_UV_SPHERE",) + fn_lines("texture_coords", "const float2 uv = sphere_uv(", "ty = uv.y;"),
             ("RGR_UV_PLANE",) + fn_lines("texture_coords", "V3 xa = cross(n, v3(0.0, 0.0, 1.0));", "ty = (float)dot(hv, ya);"),
             ("RGR_LIGHT_SPH",) + fn_lines("light_dir_dist", "V3 v = sub(v3(l.v[0], l.v[1], l.v[2]), p);", "dist = m;"),
             ("RGR_LIGHT_SPH",) + fn_lines("light_intensity", "V3 d = sub(v3(l.v[0], l.v[1], l.v[2]), p);",
                                           "return l.intensity / (4.0f * PI_F * r2);")]
    return out + [(r, f, a, b) for r, f, a, b in extra]


def klass(op: str) -> str:
    if op.startswith("v_") and ("f64" in op or op.startswith(("v_div_scale", "v_div_fmas", "v_div_fixup"))):
        return "fp64"
    if op.startswith(("v_mov", "v_cndmask", "v_readlane", "v_writelane", "v_readfirstlane", "v_accvgpr")):
        return "move_select"
    if op.startswith("v_") and ("f32" in op or "f16" in op):
        return "valu_f32"
    if op.startswith("v_"):
        return "valu_int"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def disassemble(obj: Path, sym: str):
    d = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", f"--disassemble-symbols={sym}", str(obj)],
                       capture_output=True, text=True, check=True).stdout
    insts = []
    for line in d.splitlines():
        m = re.match(r"\s+(\S+)\b(.*?)//\s*([0-9A-Fa-f]+):", line)
        if m:
            insts.append((int(m.group(3), 16), m.group(1)))
    return insts


def chains(obj: Path, addrs):
    """Inline chain of every address, innermost frame first: [(function, file, line)]."""
    inp = "".join(f"0x{a:x}\n" for a in addrs)
    out = subprocess.run([f"{LLVM}/llvm-symbolizer", f"--obj={obj}", "--inlines", "--output-style=LLVM"], input=inp,
                         capture_output=True, text=True, check=True).stdout
    res = []
    for block in out.strip("\n").split("\n\n"):
        ls = block.split("\n")
        cur = []
        for fn, loc in zip(ls[0::2], ls[1::2]):
            m = re.match(r"(.*):(\d+):(\d+)$", loc)
            full = fn.split("(")[0].strip()
            f = full.split("<")[0].split()[-1].split("::")[-1] if fn.strip() else "?"
            cur.append((f, Path(m.group(1)).name if m else "?", int(m.group(2)) if m else 0, full))
        res.append(cur)
    assert len(res) == len(addrs), (len(res), len(addrs))
    return res


def main():
    args = sys.argv[1:]
    kernel, out_json, visits_path = DEFAULT, None, None
    detail = None
    if "--detail" in args:
        k = args.index("--detail"); detail = args[k + 1]; del args[k:k + 2]
    for flag in ("--kernel", "--json", "--visits"):
        if flag in args:
            k = args.index(flag)
            v = args[k + 1]
            del args[k:k + 2]
            kernel, out_json, visits_path = ((v, out_json, visits_path) if flag == "--kernel" else
                                             (kernel, v, visits_path) if flag == "--json" else (kernel, out_json, v))
    dev_only = "-DRG_DEV_LIGHT_ONLY"
    if "--heavy" in args:  # the heavy-path instantiations (give their --kernel)
        args.remove("--heavy")
        dev_only = "-DRG_DEV_HEAVY_ONLY"
    build = "stats"
    if "--build" in args:
        k = args.index("--build"); build = args[k + 1]; del args[k:k + 2]
    tmp = Path("/tmp/rg_isa_budget")
    tmp.mkdir(exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math",
           "-fPIC", "-gline-tables-only", dev_only, "-DRG_DEV_ONE_DEPTH", "-c", "rg_kernels.hip",
           "-o", str(tmp / "k.o"), "--save-temps=obj", *(["-DRG_REGION_STATS"] if build == "stats" else []), *args]
    r = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-3000:])
        sys.exit(1)
    obj = tmp / "rg_kernels-hip-amdgcn-amd-amdhsa-gfx950.out"
    regs = regions()
    names = region_names()
    src_lines = SRC.read_text().splitlines()
    marker_line = {i: m.group(1) for i, l in enumerate(src_lines, 1)
                   for m in [re.search(r"RG_REGION\((RGR_\w+)\)", l)] if m and "#define" not in l}
    markers = []  # (region, {full names on the chain}) per marker atomic
    per_inst = {}
    detail_lines = collections.defaultdict(collections.Counter)
    for sym, tag in ((kernel, None), ("_ZN3rgk9sphere_uvEdddd", "RGR_UV_SPHERE")):
        insts = disassemble(obj, sym)
        ch = chains(obj, [a for a, _ in insts])
        for (addr, op), chain in zip(insts, ch):
            reg, inst = tag, sym
            mk = next(((fname, line) for _, fname, line, _ in chain if fname == "rg_kernels.hip"), None)
            if build == "stats" and mk and mk[1] in marker_line:
                if op.startswith("global_atomic_add"):
                    markers.append((marker_line[mk[1]], {fr[3] for fr in chain}))
                continue  # the instrumentation itself
            tail = next((i for i, fr in enumerate(chain) if fr[0] == "sphere_tail"), None)
            if reg is None and tail is not None and tail + 1 < len(chain) and chain[tail + 1][0] in PAIR_OF:
                reg, inst = PAIR_OF[chain[tail + 1][0]], chain[tail + 1][3]
            if reg is None:
                best = None
                for depth, (f, fname, line, full) in enumerate(chain):  # innermost first
                    if fname != "rg_kernels.hip":
                        continue
                    for rn, rf, a, b in regs:
                        if rf == f and a <= line <= b:
                            if best is None or (depth, b - a) < best[0]:
                                best = ((depth, b - a), rn, full)
                    if best is not None:
                        break
                reg, inst = (best[1], best[2]) if best else ("(outside the loop)", sym)
                if reg in FUNCTION_REGIONS:
                    inst = "(all)"  # spans several functions (light_dir_dist + light_intensity): one sum
            # per template instantiation of the region's function (sph_query_group<2> and its
            # remainder copy <1> hold the same lines): the largest one is what a visit runs
            per_inst.setdefault(reg, {}).setdefault(inst, collections.Counter())[klass(op)] += 1
            if detail and reg == detail:
                key = " < ".join(f"{f}:{line}" for f, _, line, _ in chain[:4])
                detail_lines[key][klass(op)] += 1
    def copies(reg, inst):
        """Marker copies (atomic pairs) of reg inside instantiation inst, else in the whole kernel."""
        mine = [f for r, f in markers if r == reg]
        n = sum(1 for f in mine if inst in f) or len(mine)
        return max(1, n // 2)
    static, ncopies = {}, {}
    for reg, d in per_inst.items():
        inst, c = max(d.items(), key=lambda kv: sum(kv[1][k] for k in VALU))
        n = copies(reg, inst) if build == "stats" else 1
        ncopies[reg] = n
        static[reg] = collections.Counter({k: round(v / n) for k, v in c.items()})
    if build == "stats":
        print("marker copies per visited instantiation: " +
              ", ".join(f"{k[4:]}={v}" for k, v in sorted(ncopies.items()) if v > 1))
    visits = None
    if visits_path:
        visits = json.loads(Path(visits_path).read_text())["regions"]
    hdr = f"{'region':22s} " + " ".join(f"{k:>10s}" for k in CLASSES)
    print("static instructions per region visit")
    print(hdr + (f" {'visits':>10s} {'dyn VALU':>12s} {'dyn FP64':>12s}" if visits else ""))
    dyn_tot = collections.Counter()
    rows = []
    for rn in names + sorted(k for k in static if k not in names):
        c = static.get(rn, collections.Counter())
        line = f"{rn:22s} " + " ".join(f"{c[k]:10d}" for k in CLASSES)
        if visits:
            v = visits.get(rn, {}).get("visits", 0) if rn in names else 0
            for k in CLASSES:
                dyn_tot[k] += v * c[k]
            line += f" {v:10d} {v * sum(c[k] for k in VALU):12d} {v * c['fp64']:12d}"
        rows.append({"region": rn, "static": dict(c), **({"visits": visits.get(rn, {}).get("visits", 0)} if visits else {})})
        print(line)
    if visits:
        print("dynamic (visits x static): " + ", ".join(f"{k} {dyn_tot[k]:.4g}" for k in CLASSES) +
              f"; VALU {sum(dyn_tot[k] for k in VALU):.4g}")
    if detail:
        print(f"\n{detail}: instructions by inline chain (innermost first)")
        for key, c in sorted(detail_lines.items(), key=lambda kv: -sum(kv[1].values())):
            print(f"  {sum(c.values()):5d}  " + " ".join(f"{k}={c[k]}" for k in CLASSES if c[k]) + f"   {key}")
    if out_json:
        Path(out_json).write_text(json.dumps({"kernel": kernel, "rows": rows, "dynamic_total": dict(dyn_tot)}, indent=1))


if __name__ == "__main__":
    main()
