"""Cell-growth GIF from one or more ``docs/run.py`` runs (reference ``docs/create_cell_growth_gif.py``
and ``docs/create_cover_gif.py``): the runs' cell-map frames are pasted side by side, frame by
frame; a run that ends early keeps showing its last frame.

Frames come from ``<rundir>/frames/cells_*.png``; runs without frames but with ``step=<i>/``
checkpoints are rendered from the saved ``cell_map.pt`` (loaded with ``weights_only=True``).

    python docs/create_gif.py docs/runs/A docs/runs/B --out cells.gif --fps 10
"""
from __future__ import annotations

import argparse
from pathlib import Path

import numpy as np
import torch
from PIL import Image, ImageOps


def _frames(rundir: Path) -> list[Image.Image]:
    pngs = sorted((rundir / "frames").glob("cells_*.png"))
    if pngs:
        return [Image.open(p).convert("L") for p in pngs]
    states = sorted((d for d in rundir.glob("step=*") if d.is_dir()), key=lambda d: int(d.name.split("=")[1]))
    out = []
    for d in states:
        cmap = torch.load(d / "cell_map.pt", map_location="cpu", weights_only=True)
        out.append(Image.fromarray((cmap.to(torch.uint8) * 255).numpy().astype(np.uint8), mode="L"))
    return out


def create_gif(rundirs: list[Path], outfile: Path, fps: int = 10, border: int = 10, loop: int = 0) -> int:
    runs = [_frames(Path(r)) for r in rundirs]
    runs = [r for r in runs if r]
    if not runs:
        raise ValueError("no frames or checkpoints found")
    n = max(len(r) for r in runs)
    frames = []
    for i in range(n):
        tiles = [ImageOps.expand(r[min(i, len(r) - 1)], border=border, fill=128) for r in runs]
        w = sum(t.width for t in tiles)
        h = max(t.height for t in tiles)
        canvas = Image.new("L", (w, h), 128)
        x = 0
        for t in tiles:
            canvas.paste(t, (x, 0))
            x += t.width
        frames.append(canvas)
    frames[0].save(outfile, save_all=True, append_images=frames[1:], duration=int(1000 / fps), loop=loop)
    return n


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("rundirs", nargs="+")
    ap.add_argument("--out", default="cells.gif")
    ap.add_argument("--fps", type=int, default=10)
    a = ap.parse_args()
    print(create_gif([Path(r) for r in a.rundirs], Path(a.out), fps=a.fps), "frames ->", a.out)
