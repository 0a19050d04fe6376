#!/usr/bin/env python3
"""Build and run scripts/bvh_width_sim.cpp (2-, 4- and 8-wide sphere BVHs over the same binary SAH
tree, walked per lane as the heavy kernel does) on a bench workload's spheres and lights.

    python scripts/bvh_width_sim.py [workload] [stride] [--json out.jsonl]

Prints one JSON line per (width, ray kind): walk iterations, child box tests and exact sphere tests
per ray, the tree's worst-case per-lane stack; and the brute-force check (0 mismatches)."""
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def main():
    args = [a for a in sys.argv[1:]]
    out = None
    if "--json" in args:
        k = args.index("--json"); out = args[k + 1]; del args[k:k + 2]
    wl = args[0] if args else "synth1024"
    stride = int(args[1]) if len(args) > 1 else 8
    from bench import load_workload
    from raingun_amd.scene import DirectionalLight, Sphere
    W, H = 3840, 2160
    scene = load_workload(wl, W, H)[0]
    sph = [b for b in scene.bodies if isinstance(b, Sphere)]
    lines = [f"{scene.fov!r}", str(len(sph))]
    lines += [" ".join(repr(float(v)) for v in (*s.center, s.radius)) for s in sph]
    lines.append(str(len(scene.lights)))
    for l in scene.lights:
        if isinstance(l, DirectionalLight):
            lines.append("0 " + " ".join(repr(float(v)) for v in l.direction))
        else:
            lines.append("1 " + " ".join(repr(float(v)) for v in l.position))
    with tempfile.TemporaryDirectory() as td:
        exe = Path(td) / "bvh_width_sim"
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                        str(REPO / "scripts" / "bvh_width_sim.cpp")], check=True)
        r = subprocess.run([str(exe), str(W), str(H), str(stride)], input="\n".join(lines) + "\n",
                           capture_output=True, text=True)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr)
    if out:
        Path(out).write_text(r.stdout)
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
