"""Statistical check against the reference's RNG semantics.

The reference draws every random number of a render thread from ONE
thread-local fastrand wyrand stream (math.rs:244-246), consumed in the order
of its pixel loop (main.rs:253-264): jitter u, v, Camera::ray's disk sample
(world.rs:53-63), then the scatter draws of every bounce. The GPU (and the
oracle's parity mode) instead key a xoroshiro128** stream by (pixel, sample)
(DESIGN §2), so images can only agree in distribution. The fixture
tests/golden/refrng_<scene>.npz holds the oracle rendering with the
reference's semantics (tools/make_refrng_fixture.py: 64 workers x 64 passes
= 4096 spp of a 64x36 frame; per-pixel radiance mean and per-sample variance,
bounce-count mean and variance). Here the other side renders 4096 spp of
the same frame in batches and every 4x4-pixel block mean is compared with
Welch's statistic

  z = (mean_here - mean_ref) / sqrt(var_ref / n_ref + var_of_mean_here)

(the fixture's per-sample variance; this side's variance of the mean from
its batch means, so rare bright paths count on the side that drew them).
Pass: max |z| < 5 and mean z^2 in [0.6, 1.6] over all blocks, channels and the bounce counts of both scenes; a wrong draw order,
a missing draw or a biased sampler moves whole regions by many sigmas.
"""
from pathlib import Path

import numpy as np
import pytest

import massrt

GOLDEN = Path(__file__).resolve().parent / "golden"
SCENES = ["cornell", "sphere_grid"]
BLOCK = 4


def batch_stats(render, batches, spp):
    """Per-pixel mean and variance of the mean of `batches` renders of `spp`
    samples each (batch means: heavy-tailed radiance — rare paths to the small
    lights — shows up in this side's own variance)."""
    m, m2, b, b2 = 0.0, 0.0, 0.0, 0.0
    for k in range(batches):
        rgb, bo = render(k * spp, spp)
        x, y = np.asarray(rgb, np.float64) / spp, np.asarray(bo, np.float64) / spp
        m, m2, b, b2 = m + x, m2 + x * x, b + y, b2 + y * y
    m, m2, b, b2 = m / batches, m2 / batches, b / batches, b2 / batches
    f = 1.0 / (batches - 1)
    return m, np.maximum(m2 - m * m, 0) * f, b, np.maximum(b2 - b * b, 0) * f


def block_z(fix, here):
    """Welch z of every 4x4-block mean (radiance channels and bounce counts):
    the fixture's variance of the mean from its per-sample variance, this
    side's from its batch means."""
    W, H, n_ref = int(fix["width"]), int(fix["height"]), int(fix["n"])
    m_here, v_here, b_here, bv_here = here
    zs = []
    for mean_ref, var, mh, vh, ch in ((fix["mean"], fix["var"], m_here, v_here, 3),
                                      (fix["bmean"], fix["bvar"], b_here, bv_here, 1)):
        def blocks(a):
            a = np.asarray(a, dtype=np.float64).reshape(H // BLOCK, BLOCK, W // BLOCK, BLOCK, ch)
            return a.sum(axis=(1, 3)) / BLOCK ** 2
        v = blocks(var) / BLOCK ** 2 / n_ref + blocks(vh) / BLOCK ** 2
        d = blocks(mh) - blocks(mean_ref)
        zero = v == 0
        assert np.all(d[zero] == 0), "a constant block differs"
        zs.append((d[~zero] / np.sqrt(v[~zero])).ravel())
    return np.concatenate(zs)


def check(z):
    assert z.size > 200
    assert np.abs(z).max() < 5.0, f"max |z| {np.abs(z).max():.2f}"
    assert 0.6 <= float(np.mean(z * z)) <= 1.6, f"mean z^2 {np.mean(z * z):.3f}"


@pytest.mark.gpu
def test_gpu_matches_reference_rng_semantics(ctx):
    z = []
    for scene in SCENES:
        fix = np.load(GOLDEN / f"refrng_{scene}.npz")
        W, H = int(fix["width"]), int(fix["height"])
        b = massrt.Builder(1).builtin(scene, float(massrt.ASPECT_RATIO), GOLDEN)
        ctx.upload(b)
        here = batch_stats(lambda s0, n: ctx.render(W, H, s0, n, seed=77), 64, 64)  # 4096 spp
        z.append(block_z(fix, here))
    check(np.concatenate(z))


def test_oracle_per_sample_streams_match_reference_rng_semantics():
    """The same check on the CPU: the oracle's per-(pixel, sample) streams
    (the GPU's scheme, 1024 spp) against the reference-semantics fixture."""
    import oracle

    z = []
    for scene in SCENES:
        fix = np.load(GOLDEN / f"refrng_{scene}.npz")
        W, H = int(fix["width"]), int(fix["height"])
        o = oracle.Scene(1).builtin(scene, float(massrt.ASPECT_RATIO), str(GOLDEN))
        here = batch_stats(lambda s0, n: o.render(W, H, s0, n, seed=78, threads=0), 32, 32)
        z.append(block_z(fix, here))
    check(np.concatenate(z))


def test_check_detects_a_wrong_sampler():
    """Sanity of the statistic: dropping the disk draw of Camera::ray (every
    later draw shifts by two) is invisible to a pinhole camera, so instead a
    biased image (radiance x 1.02) must fail."""
    fix = np.load(GOLDEN / "refrng_sphere_grid.npz")
    n = int(fix["n"])
    rng = np.random.default_rng(0)
    noise = rng.normal(size=fix["mean"].shape) * np.sqrt(fix["var"] / n)
    here = (fix["mean"] * 1.02 + noise, fix["var"] / n, fix["bmean"], fix["bvar"] / n)
    with pytest.raises(AssertionError):
        check(block_z(fix, here))
