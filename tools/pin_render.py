"""GPU renders for the example.png pin (tools/make_example_pin.py analyses them).

Writes sums (not bytes) so the analysis can tonemap and estimate noise:
  cornell_<W>.npz      Cornell (cornell.rs:29-96) at W x W, aspect 1.0
  sphere_grid_s<k>.npz SphereGrid (sphere_grid.rs:29-95) at 1920x1080, scene seed k

usage: python tools/pin_render.py OUTDIR [cornell_spp] [grid_spp]
"""
from __future__ import annotations

import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "mass-raytrace_amd"))
import massrt  # noqa: E402


def render(name, w, h, aspect, spp, scene_seed=1, batch=256, sq=False):
    b = massrt.Builder(scene_seed).builtin(name, aspect, REPO / "tests" / "golden")
    ctx = massrt.Context(0)
    ctx.upload(b)
    rgb = np.zeros(w * h * 3, np.float32)
    bo = np.zeros(w * h, np.uint32)
    # per-batch means give a noise estimate (batch means are iid)
    m = []
    t = time.time()
    for s0 in range(0, spp, batch):
        r, _ = ctx.render(w, h, s0, batch, seed=1)
        rgb += r
        m.append(r / batch)
    dt = time.time() - t
    ctx.close()
    m = np.stack(m)
    print(f"{name} {w}x{h} {spp} spp scene seed {scene_seed}: {dt:.1f} s", flush=True)
    return rgb, m.std(0, ddof=1) / np.sqrt(len(m)) if sq else None


def main():
    out = Path(sys.argv[1])
    out.mkdir(parents=True, exist_ok=True)
    cspp = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    gspp = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    rgb, se = render("cornell", 720, 720, 1.0, cspp, batch=512, sq=True)
    np.savez_compressed(out / "cornell_720.npz", rgb=rgb, passes=cspp, se=se.astype(np.float32))
    for k in (1, 2, 3):
        rgb, _ = render("sphere_grid", 1920, 1080, float(massrt.ASPECT_RATIO), gspp, scene_seed=k)
        np.savez_compressed(out / f"sphere_grid_s{k}.npz", rgb=rgb, passes=gspp)


if __name__ == "__main__":
    main()
