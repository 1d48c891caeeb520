"""Full-size properties at BASELINE config 2 (SphereGrid 1920x1080): a sampled
pixel subset against the oracle (paths are per-(pixel, sample) independent,
so the oracle recomputes any subset exactly), determinism, shard additivity."""
import numpy as np
import pytest

import massrt
import oracle

pytestmark = pytest.mark.gpu
ASPECT = float(massrt.ASPECT_RATIO)
W, H = 1920, 1080


@pytest.fixture(scope="module")
def grid(golden_dir):
    return (massrt.Builder(1).builtin("sphere_grid", ASPECT, golden_dir),
            oracle.Scene(1).builtin("sphere_grid", ASPECT, golden_dir))


def test_fullsize_pixel_subset_matches_oracle(ctx, grid):
    b, o = grid
    ctx.upload(b)
    spp = 4
    rgb, bo = ctx.render(W, H, 0, spp, seed=1)
    px = np.arange(0, W * H, 997, dtype=np.uint32)
    orgb, obo = o.render_pixels(W, H, px, 0, spp, seed=1)
    assert np.array_equal(bo[px], obo)
    a = rgb.reshape(-1, 3)[px].astype(np.float64)
    assert np.linalg.norm(a - orgb.reshape(-1, 3)) / np.linalg.norm(orgb) <= 1e-4
    assert 1.0 < bo.mean() / spp < 20.0


def test_fullsize_deterministic_and_shard_additive(ctx, grid):
    b, _ = grid
    ctx.upload(b)
    a = ctx.render(W, H, 0, 2, seed=9)
    acc = (np.zeros(W * H * 3, np.float32), np.zeros(W * H, np.uint32))
    for i in range(4):
        acc = ctx.render(W, H, 0, 2, seed=9, shard_index=i, shard_count=4, accum=acc)
    assert np.array_equal(a[0].view(np.uint32), acc[0].view(np.uint32))
    assert np.array_equal(a[1], acc[1])
