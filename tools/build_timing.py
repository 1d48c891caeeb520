"""Wall time of World::build_bvh for the built-in scenes: the host builder
(World::bvh_new, the reference's recursion restated in C++) against the
device builder (csrc/device/build.hip), and a check that both trees agree.

usage: python tools/build_timing.py [scene ...]   (needs a GPU)"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "mass-raytrace_amd"))
sys.path.insert(0, str(Path(__file__).resolve().parent))
import massrt  # noqa: E402
from gen_assets import ensure_assets  # noqa: E402

ASPECT = float(massrt.ASPECT_RATIO)


def main(scenes):
    assets = ensure_assets(Path(__file__).resolve().parent.parent / "assets", mesh=True, textures=True,
                           environment=True)
    ctx = massrt.Context(0)
    # warm the device path (module load, hipcub temp allocation)
    massrt.Builder(1).builtin_device("cornell", ctx, ASPECT, assets)
    for s in scenes:
        t0 = time.perf_counter()
        h = massrt.Builder(1).builtin(s, ASPECT, assets)
        t_host = time.perf_counter() - t0
        t0 = time.perf_counter()
        d = massrt.Builder(1).builtin_device(s, ctx, ASPECT, assets)
        t_dev = time.perf_counter() - t0
        hm, dm = d.last_build_ms()
        same = massrt.preorder(h.desc_only())[0] == massrt.preorder(d.desc_only())[0]
        print(f"{s}: generate+build host {t_host * 1e3:.0f} ms, generate+build device {t_dev * 1e3:.0f} ms "
              f"(device tree build: host part {hm:.1f} ms, device part {dm:.1f} ms) same_tree={same}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main(sys.argv[1:] or ["sphere_grid", "cube_field", "menger_l3", "menger"])
