"""Does ray order matter for k_trace? Secondary rays of a 1080p frame (first
diffuse-like bounce off the primary hits, uniform random directions) traced
in pixel-tile order and after binning by direction octant + origin Morton
key. Run under rocprofv3 --kernel-trace --stats and compare the k_trace
launches (the order of the calls: tile order first, then binned).
   python tools/coherence_probe.py [scene]"""
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "mass-raytrace_amd"), str(REPO / "tools")]
import massrt  # noqa: E402
from gen_assets import ensure_assets  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "mesh_ply"
assets = ensure_assets(REPO / "assets", mesh=True)
b = massrt.Builder(1).builtin(scene, float(massrt.ASPECT_RATIO), str(assets))
_, cam = b.desc()
f = cam.fields()
org, llc, hor, ver = f[0:3], f[3:6], f[6:9], f[9:12]
W, H = 1920, 1080
# pixels in 8x8-tile order (the renderer's pool order)
ty, tx, py, px = np.meshgrid(np.arange(H // 8 + 1), np.arange(W // 8), np.arange(8), np.arange(8), indexing="ij")
y, x = (ty * 8 + py).ravel(), (tx * 8 + px).ravel()
keep = y < H
y, x = y[keep], x[keep]
rng = np.random.default_rng(1)
s = ((x + rng.random(x.size)) / (W - 1)).astype(np.float32)[:, None]
t = ((H - 1 - y + rng.random(y.size)) / (H - 1)).astype(np.float32)[:, None]
d = (((llc + hor * s) + ver * t) - org).astype(np.float32)
prim = np.concatenate([np.broadcast_to(org, d.shape), d], 1).astype(np.float32)
ctx = massrt.Context(0)
ctx.upload(b)
hit = ctx.trace_rays(prim)
ok = hit[:, 0] != massrt.REF_NONE if hasattr(massrt, "REF_NONE") else hit[:, 0] != 0
tb = hit[:, 2].view(np.float32)
o = (prim[:, :3] + prim[:, 3:] * tb[:, None]).astype(np.float32)[ok]
dirs = rng.normal(size=o.shape).astype(np.float32)
sec = np.concatenate([o, dirs], 1).astype(np.float32)
print(f"{scene}: {prim.shape[0]} primary rays, {sec.shape[0]} secondary rays", flush=True)
# binning key: direction octant (3 bits) over a 10-bit-per-axis origin Morton code
lo, hi = o.min(0), o.max(0)
q = np.clip(((o - lo) / np.maximum(hi - lo, 1e-30) * 1023).astype(np.uint64), 0, 1023)


def spread(v):
    v = v & 0x3FF
    v = (v | (v << 16)) & 0x30000FF
    v = (v | (v << 8)) & 0x300F00F
    v = (v | (v << 4)) & 0x30C30C3
    return (v | (v << 2)) & 0x9249249


morton = spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)
octant = ((dirs[:, 0] < 0).astype(np.uint64) | ((dirs[:, 1] < 0).astype(np.uint64) << 1)
          | ((dirs[:, 2] < 0).astype(np.uint64) << 2))
orders = {
    "tile": np.arange(sec.shape[0]),
    "octant+morton": np.argsort((octant << 30) | morton, kind="stable"),
    "morton+octant": np.argsort((morton << 3) | octant, kind="stable"),
    "octant+tile": np.argsort(octant, kind="stable"),
}
ref = None
for name, perm in orders.items():
    for rep in range(2):
        t0 = time.perf_counter()
        h = ctx.trace_rays(sec[perm])
        dt = time.perf_counter() - t0
    inv = np.empty_like(perm)
    inv[perm] = np.arange(perm.size)
    h = h[inv]
    if ref is None:
        ref = h
    assert np.array_equal(h, ref), name
    print(f"{name:16s} call {dt * 1e3:7.1f} ms (incl. copies); hits identical", flush=True)
ctx.close()
