"""GPU parity: the gfx950 kernels (through the C ABI) against the oracle.

Bar (BASELINE.json north_star): closest-hit ids / t / front_face, bounce
counts and traversal counters bit-exact; radiance within 1e-4 relative L2
(RTOL below). The GPU folds radiance forward (T *= atten) where the reference
recursion folds it post-order (world.rs:71-72), so radiance differs by ULPs."""
from pathlib import Path

import numpy as np
import pytest

import massrt
import oracle
from conftest import walk_keys

pytestmark = pytest.mark.gpu
ASPECT = float(massrt.ASPECT_RATIO)
RTOL = 1e-4  # relative L2 on accumulated radiance (north_star)
SMALL = ["cornell", "sphere_grid", "cube_field"]
MESH = ["mesh_ply", "mesh_obj", "mesh_obj_textured"]


def rel_l2(a, b):
    return float(np.linalg.norm(a.astype(np.float64) - b) / max(np.linalg.norm(b.astype(np.float64)), 1e-30))


def random_rays(n, seed, span=15.0):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-span, span, (n, 3)).astype(np.float32)
    o[:, 1] = np.abs(o[:, 1]) + 0.5
    d = rng.normal(size=(n, 3)).astype(np.float32)
    return np.concatenate([o, d], 1)


def camera_rays(cam, n, seed):
    """Primary rays in the camera frustum (Camera::ray with jitter, world.rs:53-63)."""
    rng = np.random.default_rng(seed)
    f = cam.fields()
    org, llc, hor, ver = f[0:3], f[3:6], f[6:9], f[9:12]
    s = rng.random(n, dtype=np.float32)[:, None]
    t = rng.random(n, dtype=np.float32)[:, None]
    d = (((llc + hor * s) + ver * t) - org).astype(np.float32)
    return np.concatenate([np.broadcast_to(org, (n, 3)), d], 1).astype(np.float32)


@pytest.fixture(scope="module")
def small_scenes(golden_dir):
    out = {}
    for s in SMALL:
        out[s] = (massrt.Builder(1).builtin(s, ASPECT, golden_dir), oracle.Scene(1).builtin(s, ASPECT, golden_dir))
    return out


@pytest.mark.parametrize("scene", SMALL)
def test_golden_rays_bit_exact(ctx, small_scenes, golden_dir, scene):
    g = np.load(golden_dir / "oracle_golden.npz")
    b, _ = small_scenes[scene]
    ctx.upload(b)
    assert np.array_equal(ctx.trace_rays(g["rays"]), g[f"{scene}_hits"])


@pytest.mark.parametrize("scene", SMALL)
def test_trace_rays_bit_exact(ctx, small_scenes, scene):
    b, o = small_scenes[scene]
    ctx.upload(b)
    _, cam = b.desc()
    for rays in (random_rays(40_000, 1), camera_rays(cam, 40_000, 2)):
        ctx.reset_counters()
        o.reset_counters()
        gh, oh = ctx.trace_rays(rays), o.trace_rays(rays)
        assert np.array_equal(gh, oh), f"{int((gh != oh).any(1).sum())} rays differ"
        gc, oc = ctx.counters(), o.counters()
        for k in walk_keys(ctx, ["segments", "node_visits", "sphere_tests", "triangle_tests", "instance_entries", "closest_hits"]):
            assert gc[k] == oc[k], k


@pytest.mark.parametrize("scene", SMALL)
def test_golden_render(ctx, small_scenes, golden_dir, scene):
    g = np.load(golden_dir / "oracle_golden.npz")
    b, _ = small_scenes[scene]
    ctx.upload(b)
    rgb, bo = ctx.render(32, 18, 0, 2, seed=3)
    assert np.array_equal(bo, g[f"{scene}_bounces"])
    assert rel_l2(rgb, g[f"{scene}_rgb"]) <= RTOL


@pytest.mark.parametrize("scene", SMALL)
def test_render_parity_and_counters(ctx, small_scenes, scene):
    b, o = small_scenes[scene]
    ctx.upload(b)
    W, H, spp = 96, 54, 4
    ctx.reset_counters()
    o.reset_counters()
    rgb, bo = ctx.render(W, H, 0, spp, seed=17, counters=True)
    orgb, obo = o.render(W, H, 0, spp, seed=17, threads=0)
    assert np.array_equal(bo, obo)
    assert rel_l2(rgb, orgb) <= RTOL
    gc, oc = ctx.counters(), o.counters()
    for k in walk_keys(ctx, massrt.COUNTER_FIELDS):
        assert gc[k] == oc[k], (k, gc[k], oc[k])


@pytest.mark.slow
@pytest.mark.parametrize("scene", MESH)
def test_mesh_scene_parity(ctx, assets_dir, scene):
    b = massrt.Builder(1).builtin(scene, ASPECT, assets_dir)
    o = oracle.Scene(1).builtin(scene, ASPECT, assets_dir)
    ctx.upload(b)
    _, cam = b.desc()
    rays = camera_rays(cam, 20_000, 5)
    assert np.array_equal(ctx.trace_rays(rays), o.trace_rays(rays))
    W, H, spp = 48, 27, 2
    ctx.reset_counters()
    o.reset_counters()
    rgb, bo = ctx.render(W, H, 0, spp, seed=23, counters=True)
    orgb, obo = o.render(W, H, 0, spp, seed=23)
    assert np.array_equal(bo, obo)
    assert rel_l2(rgb, orgb) <= RTOL
    gc, oc = ctx.counters(), o.counters()
    for k in walk_keys(ctx, ["samples", "segments", "node_visits", "triangle_tests", "instance_entries", "model_entries",
              "closest_hits", "bounces", "texel_taps"]):
        assert gc[k] == oc[k], (k, gc[k], oc[k])


def test_render_additive_and_shard_invariant(ctx, small_scenes):
    b, _ = small_scenes["sphere_grid"]
    ctx.upload(b)
    W, H = 70, 41
    full = ctx.render(W, H, 0, 4, seed=5)
    half = ctx.render(W, H, 0, 2, seed=5)
    half = ctx.render(W, H, 2, 2, seed=5, accum=half)
    assert np.array_equal(full[0].view(np.uint32), half[0].view(np.uint32)) and np.array_equal(full[1], half[1])
    acc = (np.zeros(W * H * 3, np.float32), np.zeros(W * H, np.uint32))
    for i in range(3):
        acc = ctx.render(W, H, 0, 4, seed=5, shard_index=i, shard_count=3, accum=acc)
    assert np.array_equal(full[0].view(np.uint32), acc[0].view(np.uint32)) and np.array_equal(full[1], acc[1])
    again = ctx.render(W, H, 0, 4, seed=5)
    assert np.array_equal(full[0].view(np.uint32), again[0].view(np.uint32))


def test_depth_limits(ctx, small_scenes):
    b, o = small_scenes["cornell"]
    ctx.upload(b)
    rgb, bo = ctx.render(16, 9, 0, 2, seed=1, max_depth=0)
    assert not rgb.any() and not bo.any()
    for depth in (1, 2, 3):
        g = ctx.render(40, 22, 0, 2, seed=1, max_depth=depth)
        r = o.render(40, 22, 0, 2, seed=1, max_depth=depth)
        assert np.array_equal(g[1], r[1]) and rel_l2(g[0], r[0]) <= RTOL
        assert g[1].max() <= 2 * depth


def build_both(fn):
    b, o = massrt.Builder(3), oracle.Scene(3)
    fn(b)
    fn(o)
    return b, o


@pytest.mark.parametrize("kind,param", [(massrt.MAT_LAMBERTIAN, 0.0), (massrt.MAT_METAL, 0.0),
                                        (massrt.MAT_DIELECTRIC, 1.5)])
def test_furnace_exact_on_gpu(ctx, kind, param):
    def scene(x):
        x.background(massrt.BG_SOLID, 0, (1.0, 1.0, 1.0))
        m = x.material(kind, x.solid(1, 1, 1, 1), param)
        x.add_sphere(m, (0, 0, 0), 1.0)
        x.build_bvh()
        x.camera(40.0, (0, 0, 4), (0, 0, 0), aspect=ASPECT)
    b, o = build_both(scene)
    ctx.upload(b)
    rgb, bo = ctx.render(24, 16, 0, 8, seed=5)
    orgb, obo = o.render(24, 16, 0, 8, seed=5)
    assert np.array_equal(bo, obo)
    assert np.array_equal(rgb, orgb)  # exact: products of 1.0
    assert np.all(rgb == np.round(rgb))


def test_backgrounds_textures_and_alpha(ctx):
    """SkyBackground / SkySphere (acos/atan2 differ by ULPs between ocml and
    glibc: radiance only), textured Lambertian with uvs, and the alpha test
    inside Triangle::intersect (geom.rs:567-571) on a cut-out texture."""
    rng = np.random.default_rng(7)
    tex = rng.integers(0, 256, size=(16, 24, 4), dtype=np.uint8)
    tex[..., 3] = np.where(rng.random((16, 24)) < 0.3, 0, 255)
    env = rng.integers(0, 256, size=(32, 64, 4), dtype=np.uint8)
    grid = np.linspace(-2, 2, 9, dtype=np.float32)
    tris = []
    for i in range(8):
        for j in range(8):
            x0, x1, y0, y1 = grid[i], grid[i + 1], grid[j], grid[j + 1]
            n = [0, 0, 1]
            c = [[x0, y0, 0], [x1, y0, 0], [x1, y1, 0]], [[x0, y0, 0], [x1, y1, 0], [x0, y1, 0]]
            for tri in c:
                row = []
                for v in tri:
                    row += list(v) + n + [v[0] * 0.3 + 0.5, v[1] * 0.3 + 0.5]
                tris.append(row)
    tris = np.array(tris, dtype=np.float32)
    for bg in (massrt.BG_SKY, massrt.BG_SKYSPHERE):
        def scene(x, bg=bg):
            st = x.texture_rgba(tex, massrt.WRAP_REPEAT)
            se = x.texture_rgba(env, massrt.WRAP_CLAMP)
            if bg == massrt.BG_SKY:
                x.background(bg)
            else:
                x.background(bg, se)
            mt = x.material(massrt.MAT_LAMBERTIAN, st)
            mm = x.material(massrt.MAT_METAL, st, 0.3)
            m = x.model(mt, tris, add_to_world=True, shading=True)
            x.add_instance(m, (0.5, 0.2, -1.5), (0.1, 0.2, 0.05), (1.2, 0.8, 1.0), mm)
            x.add_sphere(x.material(massrt.MAT_DIELECTRIC, 0, 1.4), (0.3, 0.1, 1.0), 0.5)
            x.build_bvh()
            x.camera(45.0, (0.5, 0.8, 6), (0, 0, 0), aspect=ASPECT)
        b, o = build_both(scene)
        ctx.upload(b)
        _, cam = b.desc()
        rays = camera_rays(cam, 20_000, 9)
        assert np.array_equal(ctx.trace_rays(rays), o.trace_rays(rays))
        ctx.reset_counters()
        o.reset_counters()
        rgb, bo = ctx.render(64, 36, 0, 4, seed=8, counters=True)
        orgb, obo = o.render(64, 36, 0, 4, seed=8)
        assert np.array_equal(bo, obo)
        assert rel_l2(rgb, orgb) <= RTOL
        gc, oc = ctx.counters(), o.counters()
        assert oc["model_entries"] > 0
        if "model_entries" in walk_keys(ctx, ["model_entries"]):
            assert gc["model_entries"] == oc["model_entries"]
        assert oc["alpha_taps"] > 0


def _alpha_plane(rng):
    tex = rng.integers(0, 256, size=(16, 24, 4), dtype=np.uint8)
    tex[..., 3] = np.where(rng.random((16, 24)) < 0.3, 0, 255)
    grid = np.linspace(-2, 2, 9, dtype=np.float32)
    tris = []
    for i in range(8):
        for j in range(8):
            x0, x1, y0, y1 = grid[i], grid[i + 1], grid[j], grid[j + 1]
            for tri in ([[x0, y0, 0], [x1, y0, 0], [x1, y1, 0]], [[x0, y0, 0], [x1, y1, 0], [x0, y1, 0]]):
                row = []
                for v in tri:
                    row += list(v) + [0, 0, 1] + [v[0] * 0.3 + 0.5, v[1] * 0.3 + 0.5]
                tris.append(row)
    return tex, np.array(tris, dtype=np.float32)


@pytest.mark.parametrize("variant", ["model", "instance", "both"])
def test_trace_rays_model_blas_random(ctx, variant):
    """Random rays in and around an alpha-textured mesh reached through a
    world-level Model and/or an Instance (geom.rs:318-326, 405-419). This is
    the regression test for the SLP-vectoriser miscompile of k_trace (Makefile):
    with it, rays entering the model BLAS lost every hit."""
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
    ctx.upload(b)
    r = np.random.default_rng(3)
    rays = np.concatenate([r.uniform(-2.5, 2.5, (100_000, 3)), r.normal(size=(100_000, 3))], 1).astype(np.float32)
    g, ob = ctx.trace_rays(rays), o.trace_rays(rays)
    assert (ob[:, 1] >> 28 != 0).sum() > 5_000  # many hits inside a BLAS
    assert np.array_equal(g, ob)
    # the one-ray-per-thread debug kernel renders the same image
    rgb, bo = ctx.render(32, 18, 0, 2, seed=5)
    rgb2, bo2 = ctx.render(32, 18, 0, 2, seed=5, flags=massrt.RENDER_SIMPLE_TRACE)
    assert np.array_equal(bo, bo2) and np.array_equal(rgb, rgb2)
    # and so does the fused persistent kernel
    rgb3, bo3 = ctx.render(32, 18, 0, 2, seed=5, flags=massrt.RENDER_FUSED)
    assert np.array_equal(bo, bo3) and np.array_equal(rgb, rgb3)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_worlds_with_ties(ctx, seed):
    from test_bvh import random_world
    b, o = random_world(seed + 10, 400, ties=True)
    b.camera(50.0, (8, 6, 9), (0, 0, 0), aspect=ASPECT)
    o.camera(50.0, (8, 6, 9), (0, 0, 0), aspect=ASPECT)
    ctx.upload(b)
    rays = random_rays(30_000, seed, span=4.0)
    assert np.array_equal(ctx.trace_rays(rays), o.trace_rays(rays))
    rgb, bo = ctx.render(40, 30, 0, 3, seed=seed)
    orgb, obo = o.render(40, 30, 0, 3, seed=seed)
    assert np.array_equal(bo, obo) and rel_l2(rgb, orgb) <= RTOL


def test_tiny_coordinates_keep_the_early_decision(ctx):
    """Vertex coordinates like sin(pi) ~ 1e-16 (and a subnormal) lie outside the
    qfast domain but inside the early slab decision's (path.h make_tray):
    hits and bounces stay bit-exact and most box tests are still settled
    early. Before round 2's split one such coordinate sent every box test of
    the scene to the exact path (mesh_ply: 100% -> 4%)."""
    rng = np.random.default_rng(5)
    b, o = massrt.Builder(3), oracle.Scene(3)
    mb, mo = b.material(massrt.MAT_LAMBERTIAN, b.solid(0.5, 0.5, 0.5)), o.material(1, o.solid(0.5, 0.5, 0.5))
    tiny = np.array([1.2e-16, -3e-17, 7e-39, -0.0], dtype=np.float32)
    for _ in range(3000):
        tri = rng.normal(size=9).astype(np.float32) * 3
        pick = rng.random(9) < 0.25
        tri[pick] = rng.choice(tiny, size=int(pick.sum()))
        b.add_triangle(mb, tri)
        o.add_triangle(mo, tri)
    b.build_bvh()
    o.build_bvh()
    b.camera(50.0, (8, 6, 9), (0, 0, 0), aspect=ASPECT)
    o.camera(50.0, (8, 6, 9), (0, 0, 0), aspect=ASPECT)
    ctx.upload(b)
    rays = random_rays(30_000, 7, span=4.0)
    assert np.array_equal(ctx.trace_rays(rays), o.trace_rays(rays))
    ctx.reset_counters()
    rgb, bo = ctx.render(40, 30, 0, 2, seed=3, counters=True)
    orgb, obo = o.render(40, 30, 0, 2, seed=3)
    assert np.array_equal(bo, obo) and rel_l2(rgb, orgb) <= RTOL
    c = ctx.counters()
    assert 0 < c["box_exact"] < 0.3 * c["node_visits"], c


@pytest.mark.parametrize("scene", ["sphere_grid", "cube_field"])
def test_drain_handoff_is_bit_identical(small_scenes, scene):
    """A queue whose work is exhausted hands its last paths to the fused
    kernel in adopt mode (render.hip launch_finish_v): the image must be
    the per-bounce wavefront's bit for bit — never, at once, by default
    (option finish_paths)."""
    b, _ = small_scenes[scene]
    out = []
    for v in (0, 1000000000, None):
        c = massrt.Context(0)
        if v is not None:
            c.set_option("finish_paths", v)
        c.upload(b)
        c.reset_kernel_stats()
        out.append(c.render(64, 36, 0, 16, seed=11, flags=massrt.RENDER_TIME_KERNELS))
        if v == 1000000000:
            assert c.kernel_stats()["finish_launches"] > 0
        c.close()
    for rgb, bo in out[1:]:
        assert np.array_equal(out[0][0].view(np.uint32), rgb.view(np.uint32)) and np.array_equal(out[0][1], bo)


def test_errors_are_reported(ctx):
    import ctypes as C
    fresh = massrt.Context(0)
    with pytest.raises(massrt.MassrtError, match="no scene"):
        fresh.render(8, 8, 0, 1)
    b = massrt.Builder(1)
    s = b.texture_rgba(np.zeros((2, 2, 4), np.uint8), massrt.WRAP_MIRROR)
    b.add_sphere(b.material(massrt.MAT_LAMBERTIAN, s), (0, 0, 0), 1)
    b.build_bvh()
    d = b.desc_only()
    with pytest.raises(massrt.MassrtError, match="Mirror"):
        fresh.upload_desc(d)
    fresh.close()


def test_device_division_is_correctly_rounded(ctx):
    """The box/sphere tests replace IEEE division by a reciprocal + two FMA
    corrections (path.h div_cr); it must equal a/b bit for bit."""
    assert ctx.selftest_division(1 << 30, seed=1) == 0
    assert ctx.selftest_division(1 << 28, seed=12345) == 0


def test_slab_early_decision_matches_exact(ctx):
    """box_hit_any decides most slab tests from approximate quotients with an
    error margin (path.h); on grazing rays, flat boxes and t_max at a face it
    must agree with the exact (correctly rounded) slab test every time."""
    for seed in (1, 99):
        bad, ties = ctx.selftest_slab(1 << 26, seed=seed)
        assert bad == 0
        assert ties > 100_000  # the near-tie fallback is exercised


def test_tonemap_matches_oracle_bytes(ctx, small_scenes, tmp_path):
    """Image::to_rgb_bytes + dump row flip (main.rs:640-722,760-767) on the GPU:
    byte-exact against the CPU restatement, for a render and for accumulations
    with every edge the formula has (0, >1, NaN, negative, inf, tiny)."""
    b, o = small_scenes["cornell"]
    ctx.upload(b)
    W, H, spp = 48, 27, 3
    rgb, bo = ctx.render(W, H, 0, spp, seed=4)
    for mode in (massrt.DISPLAY_DEFAULT, massrt.DISPLAY_DEPTH):
        for passes in (spp, 0, 1):
            got = ctx.tonemap(W, H, rgb, bo, passes, mode)
            exp = oracle.tonemap(W, H, rgb, bo, passes, mode)
            assert np.array_equal(got, exp), (mode, passes, int((got != exp).sum()))
    rng = np.random.default_rng(11)
    W2, H2 = 257, 129
    x = rng.random(W2 * H2 * 3, dtype=np.float32) * np.float32(3.0)
    specials = np.array([0.0, 1.0, 3.0, np.nan, -1.0, -0.0, np.inf, -np.inf, 1e-38, 1e-45, 2.9999998], np.float32)
    x[: specials.size] = specials
    # values at the gamma thresholds and one ulp either side (x3 passes scaling undone)
    t = massrt.gamma_thresholds()[1:].astype(np.int64)
    edge = np.concatenate([t - 1, t, t + 1]).astype(np.uint32).view(np.float32) * np.float32(3.0)
    x[100:100 + edge.size] = edge
    bb = rng.integers(0, 60, size=W2 * H2, dtype=np.uint32)
    for mode in (massrt.DISPLAY_DEFAULT, massrt.DISPLAY_DEPTH):
        got = ctx.tonemap(W2, H2, x, bb, 3, mode)
        exp = oracle.tonemap(W2, H2, x, bb, 3, mode)
        assert np.array_equal(got, exp), (mode, int((got != exp).sum()))
    massrt.write_png(tmp_path / "cornell.png", ctx.tonemap(W, H, rgb, bo, spp))


@pytest.mark.parametrize("scene", SMALL)
def test_prepass_matches_oracle(ctx, small_scenes, scene):
    """Camera::albedo_normal pre-pass (world.rs:81-92, main.rs:181-222):
    normals bit-exact, albedo bit-exact (no scene here samples an
    environment texture), and the Albedo/Normal views byte-exact."""
    b, o = small_scenes[scene]
    ctx.upload(b)
    W, H = 64, 36
    ga, gn = ctx.prepass(W, H, seed=9)
    oa, on = o.prepass(W, H, seed=9)
    assert np.array_equal(gn, on), int((gn != on).sum())
    assert np.array_equal(ga, oa), int((ga != oa).sum())
    zeros = np.zeros(W * H, np.uint32)
    for mode, buf in ((massrt.DISPLAY_ALBEDO, ga), (massrt.DISPLAY_NORMAL, gn)):
        assert np.array_equal(ctx.tonemap(W, H, buf, zeros, 1, mode), oracle.tonemap(W, H, buf, zeros, 1, mode))


def test_cpp_driver_writes_the_same_image(ctx, small_scenes, golden_dir, tmp_path):
    """examples/mrt_render.cpp (the render()+dump() driver over the C ABI)
    produces exactly the bytes the library's render + tonemap give."""
    import subprocess
    from PIL import Image
    exe = Path(massrt.__file__).parent / "mrt_render"
    out = tmp_path / "cornell.png"
    r = subprocess.run([str(exe), "cornell", "64", "36", "4", str(out), str(golden_dir)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    b, _ = small_scenes["cornell"]
    ctx.upload(b)
    rgb, bo = ctx.render(64, 36, 0, 4, seed=1)
    for suffix, mode in (("", massrt.DISPLAY_DEFAULT), ("_depth", massrt.DISPLAY_DEPTH)):
        png = np.asarray(Image.open(tmp_path / f"cornell{suffix}.png").convert("RGB"))
        assert np.array_equal(png, ctx.tonemap(64, 36, rgb, bo, 4, mode)), suffix
    a, n = ctx.prepass(64, 36, seed=1)
    png = np.asarray(Image.open(tmp_path / "cornell_normal.png").convert("RGB"))
    assert np.array_equal(png, ctx.tonemap(64, 36, n, bo, 4, massrt.DISPLAY_NORMAL))


def test_extended_materials_parity(ctx):
    """Specular, Isotrophic and (nested) Mix, including a Mix whose emit draws
    (material.rs:331-445): GPU render/pre-pass vs the oracle."""
    def scene(x):
        x.background(massrt.BG_SKY)
        red, grey = x.solid(0.9, 0.2, 0.2, 1.0), x.solid(0.6, 0.6, 0.6, 1.0)
        spec = x.material(massrt.MAT_SPECULAR, red, 1.8)
        iso = x.material(massrt.MAT_ISOTROPHIC, 0, 0.0, (0.4, 0.7, 0.3))
        lamb = x.material(massrt.MAT_LAMBERTIAN, grey)
        light = x.material(massrt.MAT_DIFFUSE_LIGHT, 0, 0.0, (4.0, 4.0, 3.0))
        mix = x.mix(0.35, lamb, spec)
        glow = x.mix(0.5, light, x.mix(0.25, x.material(massrt.MAT_METAL, grey, 0.3), x.material(massrt.MAT_DIELECTRIC, 0, 1.5)))
        x.add_sphere(lamb, (0, -100.5, -1), 100.0)
        for k, m in enumerate([spec, iso, mix, glow, spec, mix]):
            x.add_sphere(m, (-2.5 + k, 0.0, -1.0 - 0.3 * (k % 2)), 0.45)
        x.build_bvh()
        x.camera(50.0, (0, 1, 3), (0, 0, -1), aspect=ASPECT)
    b, o = build_both(scene)
    ctx.upload(b)
    ctx.reset_counters()
    o.reset_counters()
    rgb, bo = ctx.render(64, 36, 0, 4, seed=21, counters=True)
    orgb, obo = o.render(64, 36, 0, 4, seed=21)
    assert np.array_equal(bo, obo)
    assert rel_l2(rgb, orgb) <= RTOL
    gc, oc = ctx.counters(), o.counters()
    for k in walk_keys(ctx, ["samples", "segments", "node_visits", "sphere_tests", "closest_hits", "bounces"]):
        assert gc[k] == oc[k], (k, gc[k], oc[k])
    ga, gn = ctx.prepass(64, 36, seed=2)
    oa, on = o.prepass(64, 36, seed=2)
    assert np.array_equal(gn, on) and np.array_equal(ga, oa)


def test_volumes_and_mix_alpha_parity(ctx):
    """Traversal draws (massrt.h mrt_trace_rays): Volume free paths
    (geom.rs:595-653) and the Mix alpha pick on cut-out triangles
    (material.rs:391-426 alpha) come from the ray's own stream, interleaved
    with the scatter draws exactly as in the reference's thread-local rand."""
    rng = np.random.default_rng(11)
    tex, tris = _alpha_plane(rng)
    tex2 = tex.copy()
    tex2[..., 3] = np.where(rng.random((16, 24)) < 0.5, 0, 255)

    def scene(x):
        x.background(massrt.BG_SKY)
        s1, s2 = x.texture_rgba(tex, massrt.WRAP_REPEAT), x.texture_rgba(tex2, massrt.WRAP_REPEAT)
        mix = x.mix(0.4, x.material(massrt.MAT_LAMBERTIAN, s1), x.material(massrt.MAT_METAL, s2, 0.2))
        x.model(mix, tris, add_to_world=True, shading=True)
        x.add_sphere(x.material(massrt.MAT_LAMBERTIAN, x.solid(0.5, 0.5, 0.5, 1)), (0, -101, 0), 100.0)
        x.add_volume((0.4, 0.0, 0.8), 0.7, 1.2, (0.6, 0.7, 0.8))
        x.add_volume((-1.2, 0.3, 1.0), 0.5, 20.0, (0.9, 0.3, 0.2))
        x.add_sphere(x.material(massrt.MAT_DIELECTRIC, 0, 1.5), (1.3, 0.2, 1.2), 0.4)
        x.add_volume((1.3, 0.2, 1.2), 0.3, 3.0, (0.9, 0.9, 0.9))  # medium inside the glass ball
        x.build_bvh()
        x.camera(45.0, (0.3, 0.8, 6), (0, 0, 0), aspect=ASPECT)
    b, o = build_both(scene)
    ctx.upload(b)
    _, cam = b.desc()
    rays = camera_rays(cam, 20_000, 5)
    g, r = ctx.trace_rays(rays), o.trace_rays(rays)
    assert np.array_equal(g, r)
    assert np.any(r[:, 0] >> 28 == massrt.REF_VOLUME)
    ctx.reset_counters()
    o.reset_counters()
    rgb, bo = ctx.render(64, 36, 0, 4, seed=13, counters=True)
    orgb, obo = o.render(64, 36, 0, 4, seed=13)
    assert np.array_equal(bo, obo)
    assert rel_l2(rgb, orgb) <= RTOL
    gc, oc = ctx.counters(), o.counters()
    oc["texel_taps"] += oc["alpha_taps"]  # the device counts alpha-test taps as texel taps
    for k in walk_keys(ctx, massrt.COUNTER_FIELDS):
        assert gc[k] == oc[k], (k, gc[k], oc[k])
    assert oc["alpha_taps"] > 0
    ga, gn = ctx.prepass(64, 36, seed=2)
    oa, on = o.prepass(64, 36, seed=2)
    assert np.array_equal(gn, on) and np.array_equal(ga, oa)


def test_composite_surfaces_and_cubemap_parity(ctx):
    """YCbCrTexture, TextureBlend, SolidColorFallback (texture.rs:197-357) on
    meshes, spheres and in alpha tests, under a CubeMap background
    (material.rs:91-190) whose faces are textures and composites — the EXT
    kernel variants against the oracle. powf(2.2) in YCbCr is ocml vs glibc,
    so radiance and albedo are compared within tolerance, everything else
    bit-exact."""
    rng = np.random.default_rng(23)
    tex, tris = _alpha_plane(rng)
    planes = [rng.integers(0, 256, size=(12, 10, 4), dtype=np.uint8) for _ in range(5)]

    def scene(x):
        cut = x.texture_rgba(tex, massrt.WRAP_REPEAT)
        t = [x.texture_rgba(p, massrt.WRAP_REPEAT if k % 2 else massrt.WRAP_CLAMP) for k, p in enumerate(planes)]
        yc = x.ycbcr(t[0], t[1])
        faces = [t[2], yc, x.solid(0.3, 0.6, 0.9, 1.0), x.blend(massrt.BLEND_LIGHTEN, t[3], x.solid(0.4, 0.1, 0.2, 1)),
                 x.fallback((0.2, 0.3, 0.4, 1.0), cut), t[4]]
        x.background_cubemap(faces, (0.05, 0.1, -0.2))
        glow = x.material(massrt.MAT_LAMBERTIAN, x.blend(massrt.BLEND_ADDITION, cut, yc))
        dark = x.material(massrt.MAT_LAMBERTIAN, x.blend(massrt.BLEND_DARKEN, cut, x.solid(0.9, 0.8, 0.7, 1.0)))
        m = x.model(glow, tris, add_to_world=False, shading=True)
        x.add_instance(m, (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), (1.0, 1.0, 1.0))
        x.add_instance(m, (0.4, 0.3, 1.2), (0.05, 0.1, 0.0), (0.6, 0.6, 0.6), dark)
        sub = x.blend(massrt.BLEND_SUBTRACTION, t[2], x.fallback((1.0, 1.0, 1.0, 1.0), t[3]))
        x.add_sphere(x.material(massrt.MAT_METAL, sub, 0.2), (-1.2, 0.3, 1.0), 0.5)
        x.add_sphere(x.material(massrt.MAT_LAMBERTIAN, yc), (1.3, -0.2, 0.8), 0.4)
        x.build_bvh()
        x.camera(60.0, (0.3, 0.8, 4.5), (0, 0, 0), aspect=ASPECT)
    b, o = build_both(scene)
    ctx.upload(b)
    _, cam = b.desc()
    rays = camera_rays(cam, 20_000, 3)
    assert np.array_equal(ctx.trace_rays(rays), o.trace_rays(rays))
    ctx.reset_counters()
    o.reset_counters()
    rgb, bo = ctx.render(64, 36, 0, 4, seed=29, counters=True)
    orgb, obo = o.render(64, 36, 0, 4, seed=29)
    assert np.array_equal(bo, obo)
    assert rel_l2(rgb, orgb) <= RTOL
    gc, oc = ctx.counters(), o.counters()
    for k in walk_keys(ctx, massrt.COUNTER_FIELDS):
        if k != "texel_taps":  # the reference alpha-tests every uv candidate; the device only can-be-zero surfaces
            assert gc[k] == oc[k], (k, gc[k], oc[k])
    ga, gn = ctx.prepass(64, 36, seed=2)
    oa, on = o.prepass(64, 36, seed=2)
    assert np.array_equal(gn, on)
    assert np.allclose(ga, oa, rtol=1e-5, atol=1e-6)


@pytest.mark.slow
@pytest.mark.parametrize("scene", ["menger_l3", "menger"])
def test_menger_parity(ctx, assets_dir, scene):
    """Menger (menger.rs:20-115): cube instances whose faces
    touch (exact t ties between neighbours, resolved to the later object),
    a 500000-wide Metal ground instance and a CubeMap of
    TextureBlend(stars, YCbCr) faces. menger_l3 = 8,000 cubes, full frame;
    menger = 3.2M instances / 4.19M TLAS nodes, rays + a pixel subset of the
    1080p frame."""
    b = massrt.Builder(1).builtin(scene, ASPECT, assets_dir)
    o = oracle.Scene(1).builtin(scene, ASPECT, assets_dir)
    ctx.upload(b)
    _, cam = b.desc()
    rays = np.concatenate([camera_rays(cam, 20_000, 7), random_rays(4_000, 8, span=400.0)])
    assert np.array_equal(ctx.trace_rays(rays), o.trace_rays(rays))
    if scene == "menger_l3":
        W, H, spp = 64, 36, 2
        ctx.reset_counters()
        o.reset_counters()
        rgb, bo = ctx.render(W, H, 0, spp, seed=31, counters=True)
        orgb, obo = o.render(W, H, 0, spp, seed=31)
        assert np.array_equal(bo, obo)
        assert rel_l2(rgb, orgb) <= RTOL  # YCbCr powf(2.2): ocml vs glibc ULPs
        gc, oc = ctx.counters(), o.counters()
        for k in walk_keys(ctx, massrt.COUNTER_FIELDS):
            assert gc[k] == oc[k], (k, gc[k], oc[k])
    else:
        W, H, spp = 1920, 1080, 2
        rgb, bo = ctx.render(W, H, 0, spp, seed=31)
        px = np.arange(0, W * H, 4999, dtype=np.uint32)
        orgb, obo = o.render_pixels(W, H, px, 0, spp, seed=31)
        assert np.array_equal(bo[px], obo)
        assert rel_l2(rgb.reshape(-1, 3)[px], orgb.reshape(-1, 3)) <= RTOL
        assert bo.mean() / spp > 1.0  # the sponge and the ground are in view


@pytest.mark.parametrize("block,kb", [(256, 0), (256, 1), (256, 4), (256, 24), (512, 48), (1024, 78), (1024, 150)])
def test_treelet_budgets_bit_exact(golden_dir, block, kb):
    """The LDS treelet (upload.cpp build_treelet) at several budgets and
    workgroup sizes: no treelet, a few boxes, the top of the trees, small
    BLAS regions whole, whole small scenes. Closest hits and traversal
    counters must equal the oracle's for every choice of copied records."""
    c = massrt.Context(0, options={"trace_block": block, "treelet_kb": kb})
    try:
        for scene in SMALL:
            b = massrt.Builder(1).builtin(scene, ASPECT, golden_dir)
            o = oracle.Scene(1).builtin(scene, ASPECT, golden_dir)
            c.upload(b)
            _, cam = b.desc()
            for rays in (random_rays(3000, 11), camera_rays(cam, 3000, 12)):
                assert np.array_equal(c.trace_rays(rays), o.trace_rays(rays)), (scene, block, kb)
            c.reset_counters()
            o.reset_counters()
            rgb, bo = c.render(40, 23, 0, 2, seed=4, counters=True)
            orgb, obo = o.render(40, 23, 0, 2, seed=4)
            assert np.array_equal(bo, obo), (scene, block, kb)
            assert rel_l2(rgb, orgb) <= RTOL
            gc, oc = c.counters(), o.counters()
            for k in walk_keys(c, massrt.COUNTER_FIELDS):
                assert gc[k] == oc[k], (scene, block, kb, k, gc[k], oc[k])
    finally:
        c.close()
