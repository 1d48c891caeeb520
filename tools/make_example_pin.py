"""Fixture for the example.png pin (tests/test_example_pin.py).

/root/reference/example.png (the only image the reference itself produced) is
a 720x1125 collage. Its top panel is the CornellBox scene
(scenes/cornell.rs:29-96). Measured here:
  * the panel shows pixels [6, 718) x [6, 714) (rows x columns, top row
    first) of a 720x720 render at aspect 1.0: the wall corners and the light
    fall on the predicted pixels of Camera::new (world.rs:5-51, vfov 37,
    look_from (0,5,20)) to within half a pixel; the collage's 6-px border
    covers the rest;
  * its bytes were tone-mapped with gamma 2.0 (byte = 255*sqrt(x), the
    RTIOW convention) — a log-log fit of the panel against a converged
    render gives exponents 0.513 / 0.496 / 0.500 — not the 1/2.2 of the
    current main.rs:643, so the panel predates that line;
  * the tall box and the glass sphere sit elsewhere than cornell.rs:63-81
    places them now (the panel predates those lines too); walls, ceiling,
    floor and the light are where the current source puts them.
The lower-left SphereGrid panel shows a different camera and lighting than
scenes/sphere_grid.rs (no registration found, mean |byte diff| 86 at the best
offset for every scene seed), so it pins nothing.

Writes tests/golden/example_cornell.npz: the Cornell panel crop (uint8,
712x708x3) plus the crop offsets. The fixture is data cut out of the
reference's own image; this script (which reads /root/reference) made it.

  python tools/make_example_pin.py                 # fixture
  python tools/make_example_pin.py --diff R.npz    # diff image + stats of a GPU render
                                                   # (tools/pin_render.py output) under profiles/
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
EXAMPLE = Path("/root/reference/example.png")
OUT = REPO / "tests" / "golden" / "example_cornell.npz"
ROW0, ROW1, COL0, COL1 = 6, 718, 6, 714  # panel = render[ROW0:ROW1, COL0:COL1] (top row first)
RENDER = 720


def make_fixture():
    from PIL import Image  # tooling only (not needed by the tests)

    a = np.asarray(Image.open(EXAMPLE).convert("RGB"))
    assert a.shape == (1125, 720, 3), a.shape
    panel = np.ascontiguousarray(a[ROW0:ROW1, COL0:COL1])
    # the collage border around the panel is black
    assert a[:ROW0, :, :].max() == 0 and a[ROW1:ROW1 + 4, :, :].max() == 0
    np.savez_compressed(OUT, panel=panel, offsets=np.array([ROW0, ROW1, COL0, COL1, RENDER]))
    print(f"wrote {OUT} ({OUT.stat().st_size} bytes)")


def diff(npz: Path):
    from PIL import Image

    sys.path.insert(0, str(REPO / "tests"))
    import example_pin as ep

    panel = np.load(OUT)["panel"]
    z = np.load(npz)
    L = z["rgb"].reshape(RENDER, RENDER, 3) / float(z["passes"])
    L = L[::-1][ROW0:ROW1, COL0:COL1]  # top row first, the panel's window
    shown = 255.0 * np.clip(L, 0, 1) ** 0.5
    d = shown - panel
    out = REPO / "profiles" / "r3_example_pin"
    out.mkdir(parents=True, exist_ok=True)
    vis = np.concatenate([shown, panel, np.clip(128 + 4 * d, 0, 255)], 1).astype(np.uint8)
    Image.fromarray(vis).save(out / "cornell_render_panel_diff.png")
    stats = {"render": str(npz.name), "passes": int(z["passes"]),
             "regions": ep.region_ratios(L, panel),
             "regions_gamma_2_2": ep.region_ratios(L, panel, gamma=2.2),
             "note": "linear radiance ratio render/panel per region and channel (panel decoded with gamma 2.0; "
                     "gamma_2_2 = decoded with the current main.rs:643 exponent instead)"}
    (out / "cornell_regions.json").write_text(json.dumps(stats, indent=1))
    print(json.dumps(stats, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--diff", type=Path, default=None)
    a = ap.parse_args()
    if a.diff:
        diff(a.diff)
    else:
        make_fixture()
