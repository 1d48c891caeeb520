"""The exact call bench.py times: ONE mrt_image_render of
1920x1080x1024 spp with the default options — G = 2,123,366,400 samples in
one call: the default 2^31-sample results slab (98.9% full), the default path
pool refilled hundreds of times, the drain hand-off, and the per-scene walk
(AUTO: the proven near-first walk on all three since round 6; mesh_ply
also on the reference's walk, option traversal = 0) — checked on a ~200-pixel subset against the
oracle at the same 1024 spp: bounce counts bit-exact, radiance within 1e-4
relative L2 (paths are per-(pixel, sample) independent, so the oracle
recomputes any subset exactly; bench.py step: massrt.Image.render + gather).
"""
import numpy as np
import pytest

import massrt
import oracle

pytestmark = pytest.mark.gpu
ASPECT = float(massrt.ASPECT_RATIO)
W, H, SPP = 1920, 1080, 1024


def _pixels(n=200, seed=5):
    """A deterministic spread: a regular stride plus random pixels (edges included)."""
    rng = np.random.default_rng(seed)
    px = np.unique(np.concatenate([np.linspace(0, W * H - 1, n // 2).astype(np.int64),
                                   rng.integers(0, W * H, n // 2), [0, W - 1, W * H - W, W * H - 1]]))
    return px.astype(np.uint32)


@pytest.mark.parametrize("scene,walk", [("sphere_grid", "auto"), ("mesh_ply", "auto"), ("cube_field", "auto"),
                                        ("mesh_ply", "reference")])
def test_bench_call_matches_oracle(golden_dir, assets_dir, scene, walk):
    src = assets_dir if scene == "mesh_ply" else golden_dir
    b = massrt.Builder(1).builtin(scene, ASPECT, src)
    # default options (what bench.py's headline and secondary lines run), or the reference's walk
    c = massrt.Context(0, options={} if walk == "auto" else {"traversal": massrt.TRAVERSAL_REFERENCE})
    try:
        c.upload(b)
        taken = c.tuning()["traversal"]
        assert taken == (massrt.TRAVERSAL_REFERENCE if walk == "reference" else massrt.TRAVERSAL_NEAR_FIRST)
        img = massrt.Image(c, W, H)
        img.render(1, 0, SPP)  # one call: the whole 1024-spp frame (bench.py RankRunner.step)
        img.gather()
        rgb, bo, passes = img.read()
        img.close()
    finally:
        c.close()
    assert passes == SPP
    px = _pixels()
    o = oracle.Scene(1).builtin(scene, ASPECT, src)
    orgb, obo = o.render_pixels(W, H, px, 0, SPP, seed=1, threads=16)
    assert np.array_equal(bo[px], obo), f"{int((bo[px] != obo).sum())} of {px.size} pixels' bounce counts differ"
    a = rgb.reshape(-1, 3)[px].astype(np.float64)
    rel = np.linalg.norm(a - orgb.reshape(-1, 3)) / np.linalg.norm(orgb)
    assert rel <= 1e-4, rel
    # the whole frame was rendered: every pixel took 1024 paths of >= 1 segment
    assert bo.min() >= 0 and int(bo.sum()) > 0
