"""The oracle (and the GPU path) against the one image the reference produced:
/root/reference/example.png's CornellBox panel (fixture
tests/golden/example_cornell.npz, cut out by tools/make_example_pin.py).

What the panel pins (tests/example_pin.py has the measurements):
  * geometry — Camera::new (world.rs:5-51) with cornell.rs:83-96's camera at
    aspect 1.0, the jittered pixel mapping u = (x + rand)/(W-1) (main.rs:258-259),
    cube.ply through PlyLoader + Model::instance transforms (cornell.rs:37-72)
    and the row flip of dump (main.rs:763-766): the wall corners and the
    light's edges fall on the panel's pixels (within EDGE_TOL);
  * light transport — the DiffuseLight(8) light, Lambertian walls and their
    inter-reflection (material.rs:192-246, world.rs:65-79): the walls' linear
    radiance matches the panel's within BAND once the panel is decoded with
    the gamma 2.0 it was encoded with.
What it cannot pin: the panel predates the current tonemap exponent
(main.rs:643 uses 1/2.2; test_panel_encoding_is_gamma_2 documents the
mismatch) and the current box and sphere placement, so those regions are
excluded. The reference's RNG stream is not pinned by an image either.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

import example_pin as ep

GOLDEN = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def panel():
    return np.load(GOLDEN / "example_cornell.npz")["panel"]


def _oracle_cornell(vfov=None):
    import oracle

    sc = oracle.Scene(1).builtin("cornell", 1.0, str(GOLDEN))
    if vfov is not None:  # negative control: the same scene through another camera
        sc.camera(vfov, (0.0, 5.0, 20.0), (0.0, 5.0, 0.0), (0.0, 1.0, 0.0), aspect=1.0, aperture=0.0)
    return sc


def _as_panel(pts, rgb, spp):
    """Scatter per-pixel mean radiance of panel points into a NaN image."""
    L = np.full((ep.PH, ep.PW, 3), np.nan)
    L[pts[:, 0], pts[:, 1]] = rgb.reshape(-1, 3) / spp
    return L


def _bytes(L):
    return 255.0 * np.clip(L, 0.0, 1.0) ** 0.5  # the panel's gamma 2.0 encoding


def _check_edges(L, panel, tol=ep.EDGE_TOL):
    a, b = ep.edge_positions(_bytes(L)), ep.edge_positions(panel.astype(np.float64))
    return {k: a[k] - b[k] for k in a}


def _check_regions(L, panel):
    bad = []
    P = ep.panel_to_linear(panel)
    for name, r in ep.region_ratios(L, panel).items():
        ys, xs = ep.REGIONS[name]
        for c, v in enumerate(r):
            if v is None:  # dark in the panel: must be dark in the render
                lv = L[ys, xs, c]
                m = float(np.nanmean(lv))
                if m > 4 * float(P[ys, xs, c].mean()) + (3 / 255) ** 2:
                    bad.append((name, c, "dark channel", m))
            elif not (ep.BAND[0] <= v <= ep.BAND[1]):
                bad.append((name, c, v))
    return bad


def test_oracle_cornell_matches_example_png(panel):
    """CPU oracle on the panel's pixels: edges (256 spp, every 2nd band line)
    and region radiance (256 spp on a 5-px grid)."""
    sc = _oracle_cornell()
    pe = ep.edge_pixels(step=2)
    rgb, _ = sc.render_pixels(ep.W, ep.H, ep.to_render_index(pe), 0, 256, seed=1, threads=0)
    d = _check_edges(_as_panel(pe, rgb, 256), panel)
    assert all(abs(v) <= ep.EDGE_TOL for v in d.values()), d
    pr = ep.region_pixels(step=5)
    rgb, _ = sc.render_pixels(ep.W, ep.H, ep.to_render_index(pr), 0, 256, seed=2, threads=0)
    bad = _check_regions(_as_panel(pr, rgb, 256), panel)
    assert not bad, bad


def test_registration_detects_a_one_degree_camera_change(panel):
    """Negative control: vfov 36 instead of cornell.rs:89's 37 moves the
    wall corners by ~6 px — the edge check must see it."""
    sc = _oracle_cornell(vfov=36.0)
    pe = ep.edge_pixels(step=2)
    rgb, _ = sc.render_pixels(ep.W, ep.H, ep.to_render_index(pe), 0, 256, seed=1, threads=0)
    d = _check_edges(_as_panel(pe, rgb, 256), panel)
    assert max(abs(d["red wall | back wall"]), abs(d["back wall | green wall"])) > 2 * ep.EDGE_TOL, d


def test_panel_encoding_is_gamma_2(panel):
    """The panel's bytes are 255*sqrt(x): decoded with main.rs:643's 1/2.2
    instead, the walls come out >15% darker than the same radiance decoded
    with 2.0 — the band would reject the pin. This documents why the pin
    decodes with 2.0 (the image predates main.rs:643)."""
    P2, P22 = ep.panel_to_linear(panel, 2.0), ep.panel_to_linear(panel, 2.2)
    ys, xs = ep.REGIONS["back_upper"]
    assert P2[ys, xs].mean() / P22[ys, xs].mean() > 1.15


@pytest.mark.gpu
def test_gpu_cornell_matches_example_png(panel):
    """The product path (libmassrt, k_trace/k_shade) over the whole 720x720
    frame at 2048 spp: every edge and region of the panel."""
    import massrt

    b = massrt.Builder(1).builtin("cornell", 1.0, GOLDEN)
    ctx = massrt.Context(0)
    ctx.upload(b)
    spp = 2048
    rgb, _ = ctx.render(ep.W, ep.H, 0, spp, seed=1)
    ctx.close()
    L = (rgb.reshape(ep.H, ep.W, 3) / spp)[::-1][ep.ROW0:ep.ROW0 + ep.PH, ep.COL0:ep.COL0 + ep.PW]
    d = _check_edges(L, panel)
    assert all(abs(v) <= ep.EDGE_TOL for v in d.values()), d
    bad = _check_regions(L, panel)
    assert not bad, bad
