"""`raingun` command line, mirroring the reference's src/main.rs + src/render.rs.

    python -m raingun_amd.cli [-w PIXELS] [-h PIXELS] [--4k|--hd] [--draft] [-o FILE] FILE

Flags and their precedence follow construct_app / RenderOptions::from
(main.rs:21-96): --draft forces 800x600 and caps the recursion depth at 4
(main.rs:74-75, 119-123); --hd / --4k set 1920x1080 / 3840x2160 and override
each other (the last one wins); explicit --width/--height override presets
(but not --draft, which clap treats as overriding them, main.rs:47-54).  The
render itself runs on the GPU (rg_render_image); the scene is loaded and the
PNG written by the native host layer (libraingun_host.so), and the timing line matches
print_render_message (render.rs:218-244).  `--preview` (piston window) is not
supported: there is no display on an MI355X node.
"""
from __future__ import annotations

import argparse
import sys
import time
from dataclasses import dataclass
from pathlib import Path
from typing import List, Optional

import numpy as np


@dataclass
class RenderOptions:          # render.rs:32-46
    width: int = 800
    height: int = 600
    max_recursion_depth: Optional[int] = None


class _LastWins(argparse.Action):
    """clap `overrides_with`: a later flag of the group cancels earlier ones."""

    def __call__(self, parser, ns, values, option_string=None):
        for other in self.const:
            setattr(ns, other, False)
        setattr(ns, self.dest, True)


def construct_app() -> argparse.ArgumentParser:  # main.rs:21-68
    p = argparse.ArgumentParser(prog="raingun", add_help=False,
                                description="Render a raingun YAML scene on an MI355X GPU.")
    p.add_argument("--help", action="help", help="show this help message and exit")
    p.add_argument("-w", "--width", metavar="PIXELS", help="Width of output image.")
    p.add_argument("-h", "--height", metavar="PIXELS", help="Height of output image.")
    p.add_argument("--4k", dest="uhd", action=_LastWins, nargs=0, const=("hd",), default=False,
                   help="Renders in 4K resolution. Explicit width/height overrides.")
    p.add_argument("--hd", dest="hd", action=_LastWins, nargs=0, const=("uhd",), default=False,
                   help="Renders in 1080 (HD) resolution. Explicit width/height overrides.")
    p.add_argument("--draft", action="store_true", help="Renders in 800x600 and lower quality settings.")
    p.add_argument("--preview", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("-o", "--output", metavar="FILENAME",
                   help='Where to save the rendered image. Defaults to input filename with ".png" extension.')
    p.add_argument("--gpu", type=int, default=0, help="HIP device to render on.")
    p.add_argument("input", metavar="FILE", help="The scene definition file, in YAML format.")
    return p


def options_from(ns: argparse.Namespace) -> RenderOptions:  # main.rs:70-96
    o = RenderOptions()
    if ns.draft:
        o.max_recursion_depth = 4
    elif ns.hd:
        o.width, o.height = 1920, 1080
    elif ns.uhd:
        o.width, o.height = 3840, 2160
    if ns.draft:  # --draft overrides width/height (main.rs:47-54)
        return o
    if ns.width is not None:
        o.width = _parse_u32(ns.width, "Could not parse width")
    if ns.height is not None:
        o.height = _parse_u32(ns.height, "Could not parse height")
    return o


def _parse_u32(s: str, msg: str) -> int:
    try:
        v = int(s, 10)
    except ValueError:
        raise SystemExit(msg) from None
    if not 0 <= v <= 0xFFFFFFFF:
        raise SystemExit(msg)
    return v


def parse_arguments(args: List[str]) -> RenderOptions:
    return options_from(construct_app().parse_args(args))


# ---------------------------------------------------------------- PNG (RGBA8)
def encode_png(rgba: np.ndarray) -> bytes:
    """8-bit RGBA PNG through the native encoder (rgh_png_encode, render.rs:58)."""
    from . import _host

    return _host.encode_png(rgba)


def format_duration(ms: int) -> str:  # render.rs:229-244
    one_minute = 1000 * 60
    if 0 <= ms <= 800:
        return f"{ms}ms"
    if 800 < ms <= one_minute:
        return f"{ms / 1000.0:.2f}s"
    minutes = ms // one_minute
    return f"{minutes}m {(ms - minutes * one_minute) / 1000.0:.2f}s"


def main(argv: Optional[List[str]] = None) -> int:  # main.rs:98-132
    ns = construct_app().parse_args(argv)
    opts = options_from(ns)
    if ns.preview:
        print("--preview is not supported on this build (no display); rendering without preview",
              file=sys.stderr)
    input_path = Path(ns.input)
    if ns.output:
        output_path = Path(ns.output)
    else:
        if input_path.suffix == "" and input_path.name in ("", ".", ".."):
            print(f"Could not guess output filename from {input_path}")
            return 2
        output_path = input_path.with_suffix(".png")

    from .scene import load_scene

    if not input_path.exists():
        raise SystemExit("Could not open input file")
    scene = load_scene(input_path)
    if opts.max_recursion_depth is not None and opts.max_recursion_depth < scene.max_recursion_depth:
        scene.max_recursion_depth = opts.max_recursion_depth

    from .scene import DeviceScene

    ds = DeviceScene(scene, device=ns.gpu)
    t0 = time.perf_counter()                     # render.rs:54-56
    img = ds.render_image(opts.width, opts.height)
    t1 = time.perf_counter()
    output_path.write_bytes(encode_png(img))     # render.rs:58
    t2 = time.perf_counter()
    ds.close()
    print(f"{input_path}\t→\t{output_path}\t({format_duration(int((t1 - t0) * 1000))} render, "
          f"{format_duration(int((t2 - t1) * 1000))} write)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
