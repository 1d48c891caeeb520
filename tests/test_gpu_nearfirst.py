"""The verified near-first walk (option traversal = MRT_TRAVERSAL_NEAR_FIRST;
nf_tree.cpp, path.h trav_*_nf): surface-area-heuristic trees over the same
primitives walked near child first, the winner checked against the
reference's tree, a fallback to the reference's walk where the check fails.

Bar: the same closest hits as the reference's left-first walk — primitive,
container, t bits, front face — on every ray (the oracle's trace_rays), and
renders bit-identical to the reference walk's (same hits => same shading).
Traversal counters differ by design (fewer box tests); the fallbacks are
counted."""
import numpy as np
import pytest

import massrt
import oracle
from test_gpu_parity import ASPECT, MESH, RTOL, SMALL, _alpha_plane, build_both, camera_rays, random_rays, rel_l2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nf_ctx():
    c = massrt.Context(0, options={"traversal": massrt.TRAVERSAL_NEAR_FIRST})
    yield c
    c.close()


@pytest.fixture(scope="module")
def small(golden_dir):
    return {s: (massrt.Builder(1).builtin(s, ASPECT, golden_dir), oracle.Scene(1).builtin(s, ASPECT, golden_dir))
            for s in SMALL}


def _same(a, b):
    return np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


@pytest.mark.parametrize("scene", SMALL)
def test_rays_equal_the_oracle(nf_ctx, small, scene):
    b, o = small[scene]
    nf_ctx.upload(b)
    assert nf_ctx.tuning()["traversal"] == massrt.TRAVERSAL_NEAR_FIRST
    _, cam = b.desc()
    for rays in (random_rays(60_000, 11), camera_rays(cam, 60_000, 12)):
        nf_ctx.reset_counters()
        o.reset_counters()
        gh, oh = nf_ctx.trace_rays(rays), o.trace_rays(rays)
        assert np.array_equal(gh, oh), f"{int((gh != oh).any(1).sum())} rays differ"
        gc, oc = nf_ctx.counters(), o.counters()
        assert gc["segments"] == oc["segments"] and gc["closest_hits"] == oc["closest_hits"]
        if scene != "cornell":  # a few dozen primitives: the check's 1-2 boxes cost more than the order saves
            assert gc["node_visits"] < oc["node_visits"]  # the point of the walk


@pytest.mark.parametrize("scene", SMALL)
def test_render_equals_the_reference_walk(nf_ctx, small, golden_dir, scene):
    """Same samples, both walks: bit-identical sums and bounce counts; and
    against the oracle as the other parity tests do."""
    b, o = small[scene]
    ref = massrt.Context(0, options={"traversal": massrt.TRAVERSAL_REFERENCE})
    ref.upload(b)
    nf_ctx.upload(b)
    W, H, spp = 160, 90, 4
    a = ref.render(W, H, 0, spp, seed=19)
    nf_ctx.reset_counters()
    n = nf_ctx.render(W, H, 0, spp, seed=19, counters=True)
    ref.close()
    assert _same(a[0], n[0]) and _same(a[1], n[1])
    rgb, bo = nf_ctx.render(40, 23, 0, 2, seed=4)
    orgb, obo = o.render(40, 23, 0, 2, seed=4)
    assert np.array_equal(bo, obo) and rel_l2(rgb, orgb) <= RTOL


@pytest.mark.parametrize("variant", ["model", "instance", "both"])
def test_alpha_mesh_through_model_and_instance(nf_ctx, variant):
    """Alpha-tested triangles in a BLAS entered through a Model and/or an
    Instance (the order keys of BLAS primitives, the object-space check)."""
    tex, tris = _alpha_plane(np.random.default_rng(7))

    def scene(x):
        st = x.texture_rgba(tex, massrt.WRAP_REPEAT)
        x.background(massrt.BG_SKY)
        mt = x.material(massrt.MAT_LAMBERTIAN, st)
        m = x.model(mt, tris, add_to_world=variant in ("model", "both"), shading=True)
        if variant in ("instance", "both"):
            x.add_instance(m, (0.5, 0.2, -1.5), (0.1, 0.2, 0.05), (1.2, 0.8, 1.0), x.material(massrt.MAT_METAL, st, 0.3))
        x.add_sphere(x.material(massrt.MAT_DIELECTRIC, 0, 1.4), (0.3, 0.1, 1.0), 0.5)
        x.build_bvh()
        x.camera(45.0, (0.5, 0.8, 6), (0, 0, 0), aspect=ASPECT)

    b, o = build_both(scene)
    nf_ctx.upload(b)
    assert nf_ctx.tuning()["traversal"] == massrt.TRAVERSAL_NEAR_FIRST
    r = np.random.default_rng(3)
    rays = np.concatenate([r.uniform(-2.5, 2.5, (100_000, 3)), r.normal(size=(100_000, 3))], 1).astype(np.float32)
    g, ob = nf_ctx.trace_rays(rays), o.trace_rays(rays)
    assert (ob[:, 1] >> 28 != 0).sum() > 5_000
    assert np.array_equal(g, ob)


def test_wild_instances(nf_ctx, golden_dir):
    """Instances whose rounding the world margin does not cover ("wild":
    cond(fwd) x cond(inv) far above 2^-14 per unit, nf_tree.cpp wild()) are
    never culled; the nodes on their path force the child and carry no exit
    bound into the instance's BLAS (path.h nf_node_test). Thin
    slabs scaled 1:3000, crossing each other, non-wild cubes and spheres, rays
    from everywhere — and grazing the slabs — against the oracle."""
    def scene(x):
        x.background(massrt.BG_SKY)
        lam = x.material(massrt.MAT_LAMBERTIAN, x.solid(0.6, 0.5, 0.4))
        glow = x.material(massrt.MAT_DIFFUSE_LIGHT, 0, 0.0, (4.0, 4.0, 4.0))
        cube = x.model_from_ply(golden_dir / "cube.ply", lam)
        for k in range(6):  # wild: 12 x 0.004 x 9
            x.add_instance(cube, (0.7 * k - 2.0, 0.3 * k - 0.6, -0.5 * k), (0.1 * k, 0.05, 0.02 * k), (12.0, 0.004, 9.0),
                           glow if k % 2 else NO_MAT)
        for k in range(5):  # ordinary
            x.add_instance(cube, (1.1 * k - 2.0, 0.2, 1.0 - 0.4 * k), (0.0, 0.13 * k, 0.0), (0.4, 0.4, 0.4))
        for k in range(4):
            x.add_sphere(x.material(massrt.MAT_METAL, x.solid(0.8, 0.8, 0.8), 0.1), (k - 1.5, -0.2, 0.3 * k), 0.35)
        x.build_bvh()
        x.camera(45.0, (0.5, 1.5, 7), (0, 0, 0), aspect=ASPECT)

    NO_MAT = massrt.NO_MATERIAL
    b, o = build_both(scene)
    nf_ctx.upload(b)
    assert nf_ctx.tuning()["traversal"] == massrt.TRAVERSAL_NEAR_FIRST
    r = np.random.default_rng(5)
    o1 = r.uniform(-4, 4, (60_000, 3))
    d1 = r.normal(size=(60_000, 3))
    # grazing the slabs: nearly in the y = const plane of the slabs
    o2 = np.concatenate([r.uniform(-6, 6, (60_000, 1)), r.uniform(-1, 1, (60_000, 1)), r.uniform(-6, 6, (60_000, 1))], 1)
    d2 = np.concatenate([r.normal(size=(60_000, 1)), r.normal(size=(60_000, 1)) * 1e-3, r.normal(size=(60_000, 1))], 1)
    rays = np.concatenate([np.concatenate([o1, d1], 1), np.concatenate([o2, d2], 1)]).astype(np.float32)
    g, ob = nf_ctx.trace_rays(rays), o.trace_rays(rays)
    assert (ob[:, 1] >> 28 != 0).sum() > 10_000
    assert np.array_equal(g, ob), f"{int((g != ob).any(1).sum())} rays differ"
    rgb, bo = nf_ctx.render(64, 36, 0, 2, seed=8)
    orgb, obo = o.render(64, 36, 0, 2, seed=8)
    assert np.array_equal(bo, obo) and rel_l2(rgb, orgb) <= RTOL


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_worlds_with_ties(nf_ctx, seed):
    """Coincident and touching primitives: equal t resolved to the later
    primitive of the reference's order (the order keys)."""
    from test_bvh import random_world
    b, o = random_world(seed + 10, 400, ties=True)
    b.camera(50.0, (8, 6, 9), (0, 0, 0), aspect=ASPECT)
    o.camera(50.0, (8, 6, 9), (0, 0, 0), aspect=ASPECT)
    nf_ctx.upload(b)
    rays = random_rays(30_000, seed, span=4.0)
    assert np.array_equal(nf_ctx.trace_rays(rays), o.trace_rays(rays))
    rgb, bo = nf_ctx.render(40, 30, 0, 3, seed=seed)
    orgb, obo = o.render(40, 30, 0, 3, seed=seed)
    assert np.array_equal(bo, obo) and rel_l2(rgb, orgb) <= RTOL


def test_scenes_with_traversal_draws_keep_the_reference_walk(nf_ctx):
    """Volumes and Mix alpha tests draw random numbers during the traversal,
    in the reference's order: those scenes keep the reference's walk."""
    def scene(x):
        x.add_volume((0, 0, 0), 1.0, 0.5, (0.8, 0.8, 0.8))
        x.add_sphere(x.material(massrt.MAT_LAMBERTIAN, x.solid(0.5, 0.5, 0.5)), (0, -101, 0), 100)
        x.build_bvh()
        x.camera(40.0, (0, 1, 5), (0, 0, 0), aspect=ASPECT)

    b, o = build_both(scene)
    nf_ctx.upload(b)
    assert nf_ctx.tuning()["traversal"] == massrt.TRAVERSAL_REFERENCE
    rgb, bo = nf_ctx.render(32, 18, 0, 2, seed=3)
    orgb, obo = o.render(32, 18, 0, 2, seed=3)
    assert np.array_equal(bo, obo)


@pytest.mark.slow
@pytest.mark.parametrize("scene", MESH + ["menger_l3"])
def test_mesh_and_menger_rays(nf_ctx, assets_dir, scene):
    b = massrt.Builder(1).builtin(scene, ASPECT, assets_dir)
    o = oracle.Scene(1).builtin(scene, ASPECT, assets_dir)
    nf_ctx.upload(b)
    assert nf_ctx.tuning()["traversal"] == massrt.TRAVERSAL_NEAR_FIRST
    _, cam = b.desc()
    rays = np.concatenate([camera_rays(cam, 20_000, 5), random_rays(4_000, 6, span=20.0)])
    assert np.array_equal(nf_ctx.trace_rays(rays), o.trace_rays(rays))
    W, H, spp = 48, 27, 2
    rgb, bo = nf_ctx.render(W, H, 0, spp, seed=23)
    orgb, obo = o.render(W, H, 0, spp, seed=23)
    assert np.array_equal(bo, obo) and rel_l2(rgb, orgb) <= RTOL


@pytest.mark.slow
@pytest.mark.parametrize("scene", ["sphere_grid", "cube_field", "mesh_ply"])
def test_fullsize_frame_equals_the_reference_walk(golden_dir, assets_dir, scene):
    """A whole 1080p frame through both walks (both queues, refills, the
    drain hand-off, millions of rays): bit-identical."""
    b = massrt.Builder(1).builtin(scene, ASPECT, assets_dir if scene == "mesh_ply" else golden_dir)
    out = []
    for trav in (massrt.TRAVERSAL_REFERENCE, massrt.TRAVERSAL_NEAR_FIRST):
        c = massrt.Context(0, options={"traversal": trav})
        try:
            c.upload(b)
            c.reset_counters()
            out.append(c.render(1920, 1080, 0, 2, seed=7, counters=True) + (c.counters(),))
        finally:
            c.close()
    (ra, ba, ca), (rn, bn, cn) = out
    assert _same(ra, rn) and _same(ba, bn)
    auto = massrt.Context(0)  # the per-scene default walks near first only where that is the cheaper walk
    try:
        auto.upload(b)
        if auto.tuning()["traversal"] == massrt.TRAVERSAL_NEAR_FIRST:
            assert cn["node_visits"] < ca["node_visits"]
    finally:
        auto.close()
    assert cn["vnf_fallbacks"] < 0.01 * cn["segments"], cn
