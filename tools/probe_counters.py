"""Experiment probe (MRT_PROBE builds): k_trace iteration/coherence counters
for one render of a built-in scene. Usage: MASSRT_LIB=<probe .so> python
tools/probe_counters.py [scene] [W H spp]"""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "mass-raytrace_amd"), str(REPO / "tools")]
import massrt  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "sphere_grid"
W, H, spp = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 8)
d = REPO / "tests" / "golden"
if scene.startswith("mesh") or scene.startswith("menger"):
    from gen_assets import ensure_assets
    d = ensure_assets(REPO / "assets", mesh=scene.startswith("mesh"), textures=scene.endswith("textured"),
                      environment=scene.startswith("menger"))
b = massrt.Builder(1).builtin(scene, float(massrt.ASPECT_RATIO), d)
ctx = massrt.Context(0)
ctx.upload(b)
ctx.reset_counters()
ctx.render(W, H, 0, spp, seed=1, counters=True)
c = ctx.counters()
print(scene, c)
inner, uni, outer = c["texel_taps"], c["wave_slots"], c["model_entries"]
print(f"inner iterations {inner}  uniform {uni} ({uni / max(inner, 1):.3f})  outer iterations {outer}  "
      f"inner share {inner / max(inner + outer, 1):.3f}  lane steps/iter {c['lane_steps'] / max(inner + outer, 1):.1f}  "
      f"node visits {c['node_visits']} sphere tests {c['sphere_tests']} segments {c['segments']}")
