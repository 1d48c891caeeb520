"""Bisection driver for a GPU/oracle mismatch on the textured/alpha scene of
test_backgrounds_textures_and_alpha: renders with the persistent k_trace and
with MRT_RENDER_SIMPLE_TRACE, and traces random (secondary-like) rays."""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "mass-raytrace_amd"), str(REPO / "tests")]
import numpy as np  # noqa: E402

import massrt  # noqa: E402
import oracle  # noqa: E402

ASPECT = float(massrt.ASPECT_RATIO)
print("debug build:", massrt.lib().mrt_debug_build(), flush=True)
ctx = massrt.Context(0)
rng = np.random.default_rng(7)
tex = rng.integers(0, 256, size=(16, 24, 4), dtype=np.uint8)
tex[..., 3] = np.where(rng.random((16, 24)) < 0.3, 0, 255)
env = rng.integers(0, 256, size=(32, 64, 4), dtype=np.uint8)
grid = np.linspace(-2, 2, 9, dtype=np.float32)
tris = []
for i in range(8):
    for j in range(8):
        x0, x1, y0, y1 = grid[i], grid[i + 1], grid[j], grid[j + 1]
        for tri in ([[x0, y0, 0], [x1, y0, 0], [x1, y1, 0]], [[x0, y0, 0], [x1, y1, 0], [x0, y1, 0]]):
            row = []
            for v in tri:
                row += list(v) + [0, 0, 1] + [v[0] * 0.3 + 0.5, v[1] * 0.3 + 0.5]
            tris.append(row)
tris = np.array(tris, dtype=np.float32)
variants = sys.argv[1:] or ["model", "inst"]
for variant in variants:
    for bg in (massrt.BG_SKY, massrt.BG_SKYSPHERE):
        def scene(x):
            st = x.texture_rgba(tex, massrt.WRAP_REPEAT)
            se = x.texture_rgba(env, massrt.WRAP_CLAMP)
            if bg == massrt.BG_SKY:
                x.background(bg)
            else:
                x.background(bg, se)
            mt = x.material(massrt.MAT_LAMBERTIAN, st)
            mm = x.material(massrt.MAT_METAL, st, 0.3)
            if variant != "none":
                m = x.model(mt, tris, add_to_world="model" in variant, shading=True)
                if "inst" in variant:
                    x.add_instance(m, (0.5, 0.2, -1.5), (0.1, 0.2, 0.05), (1.2, 0.8, 1.0), mm)
            x.add_sphere(x.material(massrt.MAT_DIELECTRIC, 0, 1.4), (0.3, 0.1, 1.0), 0.5)
            x.build_bvh()
            x.camera(45.0, (0.5, 0.8, 6), (0, 0, 0), aspect=ASPECT)
        b, o = massrt.Builder(3), oracle.Scene(3)
        scene(b)
        scene(o)
        ctx.upload(b)
        # random rays around the scene
        n = 200_000
        r = np.random.default_rng(3)
        org = r.uniform(-2.5, 2.5, (n, 3)).astype(np.float32)
        d = r.normal(size=(n, 3)).astype(np.float32)
        rays = np.concatenate([org, d], 1)
        from test_gpu_parity import camera_rays
        _, cam = b.desc()
        rays = np.concatenate([rays, camera_rays(cam, 20000, 9)])
        g, ob = ctx.trace_rays(rays), o.trace_rays(rays)
        bad = np.nonzero((g != ob).any(1))[0]
        print(variant, bg, "random rays mismatches", len(bad), flush=True)
        for k in bad[:5]:
            print("   ray", rays[k].tolist(), "gpu", g[k].tolist(), "orc", ob[k].tolist())
        orgb, obo = o.render(64, 36, 0, 4, seed=8)
        for fl, name in ((0, "persistent"), (massrt.RENDER_SIMPLE_TRACE, "simple"),
                         ):
            rgb, bo = ctx.render(64, 36, 0, 4, seed=8, flags=fl)
            diff = np.nonzero(bo != obo)[0]
            rl = float(np.linalg.norm(rgb.astype(np.float64) - orgb) / max(np.linalg.norm(orgb), 1e-30))
            print(f"   {name}: bounce mismatching pixels {len(diff)} rel_l2 {rl:.3g}", diff[:8].tolist(),
                  bo[diff[:8]].tolist(), obo[diff[:8]].tolist(), flush=True)
