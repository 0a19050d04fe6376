"""Per-dispatch counter means of rg_render_kernel from one rocprofv3 --pmc run (scripts/pmc_ab.sh)."""
import csv
import glob
import sys
from collections import defaultdict

out, lib = sys.argv[1], sys.argv[2]
vals = defaultdict(lambda: defaultdict(float))
for f in glob.glob(f"{out}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rg_render_kernel" in r["Kernel_Name"]:
            vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for name, d in sorted(vals.items()):
    v = sorted(d.values())
    med = v[len(v) // 2]
    print(f"  {lib}: {name} per frame median {med:.6g} (n={len(v)}, min {v[0]:.6g}, max {v[-1]:.6g})")
