"""Helpers of the example.png pin (test_example_pin.py, tools/make_example_pin.py).

The reference's example.png top panel = pixels [6, 718) x [6, 714) of a
720x720 CornellBox render (cornell.rs:29-96, aspect 1.0), tone-mapped with
gamma 2.0. The box and the sphere were placed differently when it was made,
so only the static geometry (walls, ceiling, floor, light) is compared:
  * registration: the positions of the wall corners and of the light's
    edges (EDGES) in the render and in the panel agree within EDGE_TOL;
  * radiance: linear radiance means over wall / ceiling regions, panel
    decoded as (byte/255)^2, must agree within the band below.
"""
from __future__ import annotations

import numpy as np

W = H = 720           # the panel's source render
ROW0, COL0 = 6, 6     # panel = render rows [6, 718), cols [6, 714), top row first
PH, PW = 712, 708

# panel coordinates (rows, cols): regions clear of the box and the sphere in
# both the panel and the current scene
REGIONS = {
    "left_wall": (slice(200, 560), slice(20, 125)),
    "right_wall": (slice(160, 520), slice(585, 700)),
    "ceiling": (slice(10, 60), slice(160, 550)),
    "back_upper": (slice(150, 260), slice(150, 560)),
    "back_right": (slice(260, 400), slice(380, 560)),
}
# radiance band render/panel per region and channel (channels whose panel
# mean is above DARK); measured 1.01-1.12 at 16384 spp on the GPU
BAND = (0.85, 1.20)
DARK = 20.0  # bytes: a channel this dark in the panel (e.g. G of the red wall) must be dark in the render too

# static edges (panel coordinates): (name, axis, band, window, channel, mode).
# axis "x": the profile runs along columns of `window`, averaged over the rows
# of `band`; axis "y": along rows, averaged over the columns of `band`.
# channel None = the sum of the three. mode "cross": where the profile
# crosses halfway between its ends' levels; "min": its darkest point (the
# shadowed crease of a corner between two walls of equal albedo).
EDGES = (
    ("red wall | back wall", "x", (150, 250), (110, 170), 1, "cross"),
    ("back wall | green wall", "x", (150, 250), (540, 600), 0, "cross"),
    ("ceiling | back wall (left)", "y", (160, 270), (125, 155), None, "min"),
    ("ceiling | back wall (right)", "y", (440, 550), (125, 155), None, "min"),
    ("light, near edge", "y", (330, 380), (55, 86), None, "cross"),
    ("light, far edge", "y", (330, 380), (86, 115), None, "cross"),
    ("light, left edge", "x", (75, 95), (285, 320), None, "cross"),
    ("light, right edge", "x", (75, 95), (390, 420), None, "cross"),
)
EDGE_TOL = 1.5  # pixels (measured <= 0.86 at 16384 spp on the GPU)


def panel_to_linear(panel: np.ndarray, gamma: float = 2.0) -> np.ndarray:
    return (panel.astype(np.float64) / 255.0) ** gamma


def region_ratios(L: np.ndarray, panel: np.ndarray, gamma: float = 2.0) -> dict:
    """{region: [ratio_r, ratio_g, ratio_b]} of render linear means over panel
    linear means (None for channels dark in the panel). L: (PH, PW, 3) mean
    radiance per pixel in panel coordinates (NaN where not rendered)."""
    P = panel_to_linear(panel, gamma)
    out = {}
    for name, (ys, xs) in REGIONS.items():
        lv = L[ys, xs].reshape(-1, 3)
        pv = P[ys, xs].reshape(-1, 3)
        ok = ~np.isnan(lv[:, 0])
        pm = panel[ys, xs].reshape(-1, 3)[ok].astype(np.float64).mean(0)
        r = []
        for c in range(3):
            if pm[c] < DARK:
                r.append(None)
            else:
                r.append(round(float(lv[ok, c].mean() / pv[ok, c].mean()), 4))
        out[name] = r
    return out


def region_pixels(step: int = 6):
    """Panel (row, col) pairs on a grid over every region."""
    pts = []
    for ys, xs in REGIONS.values():
        for y in range(ys.start, ys.stop, step):
            for x in range(xs.start, xs.stop, step):
                pts.append((y, x))
    return np.array(pts, dtype=np.int64)


def edge_pixels(step: int = 1):
    """Panel (row, col) pairs covering every EDGES band x window (bands
    subsampled by `step`)."""
    pts = set()
    for _, axis, band, win, _, _ in EDGES:
        for b in range(band[0], band[1], step):
            for w in range(win[0], win[1]):
                pts.add((b, w) if axis == "x" else (w, b))
    return np.array(sorted(pts), dtype=np.int64)


def to_render_index(pts: np.ndarray) -> np.ndarray:
    """panel (row, col) -> render pixel index p = y*W + x with y = 0 the bottom row."""
    y = (H - 1) - (pts[:, 0] + ROW0)
    x = pts[:, 1] + COL0
    return (y * W + x).astype(np.uint32)


def _crossing(prof: np.ndarray) -> float:
    """Position (index units) where the profile crosses halfway between its
    two ends' levels (first crossing, linear interpolation)."""
    lo, hi = prof[:4].mean(), prof[-4:].mean()
    mid = 0.5 * (lo + hi)
    s = np.sign(prof - mid)
    for i in range(len(prof) - 1):
        if s[i] != s[i + 1] and s[i + 1] != 0:
            return i + (mid - prof[i]) / (prof[i + 1] - prof[i])
    return float("nan")


def _minimum(prof: np.ndarray, half: int = 4) -> float:
    """Position of the profile's minimum: vertex of the least-squares parabola
    through the 2*half+1 samples around the darkest one (noise-robust)."""
    sm = np.convolve(prof, np.array([1, 2, 3, 2, 1]) / 9.0, mode="same")
    k = int(np.argmin(sm[2:-2])) + 2  # the smoothed profile picks the crease, the raw one locates it
    lo, hi = max(0, k - half), min(len(prof), k + half + 1)
    x = np.arange(lo, hi, dtype=np.float64)
    a, b, _ = np.polyfit(x - k, prof[lo:hi], 2)
    return float(k - b / (2 * a)) if a > 0 else float(k)


def edge_positions(img: np.ndarray) -> dict:
    """{edge name: position in panel pixels} of an image in panel
    coordinates ((PH, PW, 3) display bytes, NaN where not rendered)."""
    out = {}
    for name, axis, band, win, ch, mode in EDGES:
        if axis == "x":
            blk = img[band[0]:band[1], win[0]:win[1]]
            prof = np.nanmean(blk, axis=0)
        else:
            blk = img[win[0]:win[1], band[0]:band[1]]
            prof = np.nanmean(blk, axis=1)
        prof = prof.sum(1) if ch is None else prof[:, ch]
        out[name] = win[0] + (_crossing(prof) if mode == "cross" else _minimum(prof))
    return out
