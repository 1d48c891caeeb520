"""Debug driver: the textured/alpha scene of test_backgrounds_textures_and_alpha
on the bounds-checked library (MASSRT_LIB=dbg)."""
import os
import sys
from pathlib import Path

os.environ.setdefault("MASSRT_LIB", "dbg")
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "mass-raytrace_amd"), str(REPO / "tests")]
import numpy as np  # noqa: E402

import massrt  # noqa: E402

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
for variant in sys.argv[1:] or ["model+inst", "model", "inst"]:
    for bg in (massrt.BG_SKY, massrt.BG_SKYSPHERE):
        x = massrt.Builder(3)
        st = x.texture_rgba(tex, massrt.WRAP_REPEAT)
        se = x.texture_rgba(env, massrt.WRAP_CLAMP)
        x.background(bg, se if bg == massrt.BG_SKYSPHERE else 0)
        mt = x.material(massrt.MAT_LAMBERTIAN, st)
        mm = x.material(massrt.MAT_METAL, st, 0.3)
        m = x.model(mt, tris, add_to_world="model" in variant, shading=True)
        if "inst" in variant:
            x.add_instance(m, (0.5, 0.2, -1.5), (0.1, 0.2, 0.05), (1.2, 0.8, 1.0), mm)
        x.add_sphere(x.material(massrt.MAT_DIELECTRIC, 0, 1.4), (0.3, 0.1, 1.0), 0.5)
        x.build_bvh()
        x.camera(45.0, (0.5, 0.8, 6), (0, 0, 0))
        ctx.upload(x)
        try:
            rgb, bo = ctx.render(64, 36, 0, 4, seed=8)
            print(variant, bg, "render ok", float(rgb.mean()), int(bo.sum()), "dbg", ctx.debug_status(), flush=True)
        except Exception as e:
            print(variant, bg, "render FAILED", e, "dbg", ctx.debug_status(), flush=True)
            raise
