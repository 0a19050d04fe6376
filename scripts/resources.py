"""Per-instantiation register/scratch summary of rg_render_kernel.

    python scripts/resources.py [extra hipcc flags...]

Compiles rg_kernels.hip with the library's flags and -Rpass-analysis=kernel-resource-usage
and prints VGPRs, spilled VGPRs, scratch bytes per lane, occupancy and static LDS for the
MAXD = 8 instantiations (the ones the bench configurations run; "host": the
host-frame ones, "tpw=-1": the light path's persistent single launches)."""
import re
import subprocess
import sys
from pathlib import Path

CSRC = Path(__file__).resolve().parent.parent / "raingun_amd" / "csrc"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math",
       "-fPIC", "-c", "rg_kernels.hip", "-o", "/tmp/rg_kernels_res.o", "-Rpass-analysis=kernel-resource-usage",
       *sys.argv[1:]]
out = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True)
if out.returncode != 0:
    sys.stderr.write(out.stderr[-4000:])
    sys.exit(out.returncode)
rows, cur = [], None
for line in out.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1)] = int(m.group(2))
for r in rows:
    m = re.match(r"_Z16rg_render_kernelILi(\d+)ELb(\d)ELb(\d)ELi(\d+)ELi(\d+)ELb(\d)ELb(\d)ELb(\d)ELi(n?\d+)ELb(\d)E",
                 r["name"])
    if not m or m.group(1) != "8":
        continue
    maxd, lsph, lcold, wps, lb, f32f, bvh, tasks, tpw, hf = m.groups()
    kind = "light" if int(lb) > 1 else "heavy"
    if tpw != "0":
        kind += f" tpw={tpw.replace('n', '-')}"
    if hf == "1":
        kind += " host"
    print(f"{kind:12s} <{maxd},{lsph},{lcold},{wps},{lb},{f32f},{bvh},{tasks}>  VGPRs {r.get('VGPRs')}  spill {r.get('VGPRs Spill')}"
          f"  scratch {r.get('ScratchSize [bytes/lane]')} B/lane  occ {r.get('Occupancy [waves/SIMD]')}  lds {r.get('LDS Size [bytes/block]')}")
