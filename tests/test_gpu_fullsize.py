"""Full-size properties at BASELINE config 2 (SphereGrid 1920x1080), configs 3-4
(cube_field, mesh_ply, mesh_obj at 1080p) and config 5 (4K): a sampled
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


@pytest.mark.parametrize("scene", ["cube_field", "mesh_ply", "mesh_obj"])
def test_fullsize_pixel_subset_other_configs(ctx, golden_dir, assets_dir, scene):
    """BASELINE configs 3 and 4 at their stated 1920x1080: 16.6M paths per
    call, so the pools drain through the adopt-mode hand-off and mesh_*
    (an 82 MB record stream) runs with the large-stream loop thresholds —
    the paths the bench times. A pixel subset must match the oracle (bounces
    bit-exact, radiance rel L2 <= 1e-4)."""
    src = golden_dir if scene == "cube_field" else assets_dir
    b = massrt.Builder(1).builtin(scene, ASPECT, src)
    o = oracle.Scene(1).builtin(scene, ASPECT, src)
    ctx.upload(b)
    spp = 8
    rgb, bo = ctx.render(W, H, 0, spp, seed=3)
    px = np.arange(11, W * H, 1_499, dtype=np.uint32)
    orgb, obo = o.render_pixels(W, H, px, 0, spp, seed=3)
    assert np.array_equal(bo[px], obo)
    a = rgb.reshape(-1, 3)[px].astype(np.float64)
    assert np.linalg.norm(a - orgb.reshape(-1, 3)) / np.linalg.norm(orgb) <= 1e-4
    assert bo.sum() > 0


def test_fullsize_deterministic_and_shard_additive(ctx, grid):
    b, _ = grid
    ctx.upload(b)
    a = ctx.render(W, H, 0, 2, seed=9)
    acc = (np.zeros(W * H * 3, np.float32), np.zeros(W * H, np.uint32))
    for i in range(4):
        acc = ctx.render(W, H, 0, 2, seed=9, shard_index=i, shard_count=4, accum=acc)
    assert np.array_equal(a[0].view(np.uint32), acc[0].view(np.uint32))
    assert np.array_equal(a[1], acc[1])


# ---- BASELINE config 5 size: textured 1M-triangle mesh + SkySphere env map at 3840x2160
W4, H4 = 3840, 2160


@pytest.fixture(scope="module")
def textured(assets_dir):
    return (massrt.Builder(1).builtin("mesh_obj_textured", ASPECT, assets_dir),
            oracle.Scene(1).builtin("mesh_obj_textured", ASPECT, assets_dir))


def test_4k_pixel_subset_across_result_chunks(textured):
    """144 spp of the 4K frame = 1.19G samples. The results slab holds 2^31
    samples by default (258 spp of 8.3M pixels); with results_log2 = 30 the
    library splits this call into chunks of 2^30 samples (129 spp), so it
    crosses a chunk boundary. A pixel subset must match the oracle (bounces
    bit-exact; radiance within 1e-4: acos/atan2 of SkySphere are ocml vs
    glibc ULPs), splitting the call at the chunk boundary must not change a
    bit, and neither must the default slab (one chunk)."""
    b, o = textured
    spp = 144
    c = massrt.Context(0, options={"results_log2": 30})
    try:
        c.upload(b)
        rgb, bo = c.render(W4, H4, 0, spp, seed=5)
        part = c.render(W4, H4, 0, 129, seed=5)
        part = c.render(W4, H4, 129, spp - 129, seed=5, accum=part)
    finally:
        c.close()
    px = np.arange(3, W4 * H4, 15_013, dtype=np.uint32)
    orgb, obo = o.render_pixels(W4, H4, px, 0, spp, seed=5)
    assert np.array_equal(bo[px], obo)
    a = rgb.reshape(-1, 3)[px].astype(np.float64)
    assert np.linalg.norm(a - orgb.reshape(-1, 3)) / np.linalg.norm(orgb) <= 1e-4
    assert np.array_equal(rgb.view(np.uint32), part[0].view(np.uint32)) and np.array_equal(bo, part[1])
    c = massrt.Context(0)
    try:
        c.upload(b)
        whole = c.render(W4, H4, 0, spp, seed=5)
    finally:
        c.close()
    assert np.array_equal(rgb.view(np.uint32), whole[0].view(np.uint32)) and np.array_equal(bo, whole[1])


def test_4k_deterministic_and_shard_additive(ctx, textured):
    b, _ = textured
    ctx.upload(b)
    a = ctx.render(W4, H4, 0, 2, seed=6)
    again = ctx.render(W4, H4, 0, 2, seed=6)
    assert np.array_equal(a[0].view(np.uint32), again[0].view(np.uint32)) and np.array_equal(a[1], again[1])
    acc = (np.zeros(W4 * H4 * 3, np.float32), np.zeros(W4 * H4, np.uint32))
    for i in range(3):
        acc = ctx.render(W4, H4, 0, 2, seed=6, shard_index=i, shard_count=3, accum=acc)
    assert np.array_equal(a[0].view(np.uint32), acc[0].view(np.uint32))
    assert np.array_equal(a[1], acc[1])


@pytest.mark.parametrize("scene", ["sphere_grid", "cube_field", "mesh_ply"])
def test_fullsize_treelet_equals_plain(golden_dir, assets_dir, scene):
    """k_trace with the LDS treelet and parked global loads (1024 threads,
    78 KB) renders full 1080p frames bit-identical to the plain kernel: many
    refills per lane, both queues, every lane state transition at scale."""
    b = massrt.Builder(1).builtin(scene, ASPECT, assets_dir if scene == "mesh_ply" else golden_dir)
    spp = 1 if scene == "mesh_ply" else 2
    out = []
    for block, kb in ((256, 0), (1024, 78)):
        c = massrt.Context(0, options={"trace_block": block, "treelet_kb": kb})
        try:
            c.upload(b)
            out.append(c.render(W, H, 0, spp, seed=5))
            if massrt.lib().mrt_debug_build():  # MASSRT_LIB=dbg: no index out of range
                assert c.debug_status()[3] == 0, c.debug_status()
        finally:
            c.close()
    assert np.array_equal(out[0][1], out[1][1])
    assert np.array_equal(out[0][0].view(np.uint32), out[1][0].view(np.uint32))
