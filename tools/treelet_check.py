"""Diagnostics: plain k_trace vs the LDS-treelet variant at scale (no asserts).
   python tools/treelet_check.py [scene] [block] [kb]"""
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "mass-raytrace_amd"), str(REPO / "tests")]
import massrt  # noqa: E402
from test_gpu_parity import camera_rays, random_rays  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "sphere_grid"
block, kb = (sys.argv[2], sys.argv[3]) if len(sys.argv) > 3 else ("1024", "78")
b = massrt.Builder(1).builtin(scene, float(massrt.ASPECT_RATIO), str(REPO / "tests" / "golden"))
_, cam = b.desc()
rays = {"cam2M": camera_rays(cam, 1 << 21, 3), "rand2M": random_rays(1 << 21, 4)}
res = []
for blk, k in (("256", "0"), (block, kb)):
    c = massrt.Context(0, options={"trace_block": int(blk), "treelet_kb": int(k)})
    c.upload(b)
    r = {name: c.trace_rays(v) for name, v in rays.items()}
    for cnt in (False, True):
        r[f"render_cnt{int(cnt)}"] = c.render(640, 360, 0, 4, seed=5, counters=cnt)
    r["render_1080"] = c.render(1920, 1080, 0, 2, seed=5)
    r["debug"] = c.debug_status()
    c.close()
    res.append(r)
a, t = res
for name in rays:
    d = np.nonzero((a[name] != t[name]).any(1))[0]
    print(f"{name}: {len(d)} of {len(rays[name])} rays differ; first {d[:8].tolist()}")
    for i in d[:4]:
        print("   ray", rays[name][i].tolist(), "plain", a[name][i].tolist(), "treelet", t[name][i].tolist())
for name in ("render_cnt0", "render_cnt1", "render_1080"):
    db = np.nonzero(a[name][1] != t[name][1])[0]
    dr = np.nonzero((a[name][0].view(np.uint32) != t[name][0].view(np.uint32)).reshape(-1, 3).any(1))[0]
    print(f"{name}: bounces differ at {len(db)} px, rgb at {len(dr)} px; first {dr[:8].tolist()}")
print("debug", a["debug"], t["debug"])
