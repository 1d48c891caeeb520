"""Both walks on the GPU, side by side: per-segment traversal counters of a
counted render and the timed k_trace of an uncounted one (option traversal
0 / 1, the same frame). Usage: python tools/nf_counters.py [SCENE ...]
(run on the GPU box; scenes default to the bench scenes)."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "mass-raytrace_amd"))
import massrt  # noqa: E402

REPO = Path(__file__).resolve().parent.parent
W, H, SPP = 1920, 1080, 32
FIELDS = ["node_visits", "triangle_tests", "sphere_tests", "instance_entries", "model_entries", "lane_steps",
          "wave_slots", "box_exact", "vnf_fallbacks"]


def main():
    sys.path.insert(0, str(REPO / "tests"))
    from gen_assets import ensure_assets
    assets = ensure_assets(REPO / "assets", mesh=True, textures=True, environment=True)
    scenes = [a for a in sys.argv[1:] if not a.startswith("--")] or ["sphere_grid", "mesh_ply", "cube_field", "menger"]
    walks = (1,) if "--nf-only" in sys.argv else (0, 1)
    for sc in scenes:
        b = massrt.Builder(1).builtin(sc, 16 / 9, str(REPO / "tests/golden" if sc in ("cornell", "sphere_grid", "cube_field") else assets))
        for trav in walks:
            c = massrt.Context(0, options={**massrt.env_options(), "traversal": trav})
            c.upload(b)
            img = massrt.Image(c, W, H)
            c.reset_counters()
            img.render(5, 0, SPP // 4, counters=True)
            k = c.counters()
            img.render(5, 0, SPP)  # warm
            c.reset_kernel_stats()
            t0 = time.perf_counter()
            img.render(5, 0, SPP, time_kernels=True)
            img.read()  # waits for the render
            dt = time.perf_counter() - t0
            st = c.kernel_stats()
            seg = max(1, k["segments"])
            per = "  ".join(f"{f} {k[f] / seg:.2f}" for f in FIELDS)
            print(f"{sc:12s} trav {trav}: {W * H * SPP / dt / 1e6:8.1f} Msamples/s  trace {st['trace_ms']:.1f} ms "
                  f"shade {st['shade_ms']:.1f} ms  per segment: {per}", flush=True)
            img.close()
            c.close()


if __name__ == "__main__":
    main()
