"""Regenerate tests/golden/ray_counts.json from the CPU restatement (oracle/).

The counts are regression anchors for the examples at the reference's default
800x600 (the reference itself cannot be run here: no Rust toolchain)."""
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))

import oracle  # noqa: E402
from raingun_amd.scene import SceneDesc, load_scene  # noqa: E402

out = {}
for name in ("test1", "test2", "test3"):
    s = load_scene(HERE / "examples" / f"{name}.yml", texture_root=HERE)
    st, _, _, counts, _ = oracle.render(SceneDesc(s), 800, 600)
    assert st == 0
    out[name] = counts
(HERE / "ray_counts.json").write_text(json.dumps(out, indent=1) + "\n")
print(out)
