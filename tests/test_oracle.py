"""The oracle (CPU restatement) against known answers and its committed golden
fixtures. Known answers are hand-derived from the reference formulas
(geom.rs:56-93 sphere, geom.rs:504-533 Möller-Trumbore, world.rs:65-79 trace),
so they hold for the reference itself; furnace scenes give exact radiance
independent of the RNG."""
import numpy as np
import pytest

import massrt
import oracle

ASPECT = float(massrt.ASPECT_RATIO)
INF = float("inf")


def lambert_world(o, color=(1, 1, 1, 1)):
    s = o.solid(*color)
    return o.material(1, s)


def test_sphere_known_answers():
    o = oracle.Scene(1)
    m = lambert_world(o)
    o.add_sphere(m, (0, 0, -5), 1.0)
    o.build_bvh()
    rays = np.array([[0, 0, 0, 0, 0, -1], [0, 0, -5, 0, 0, -1], [0, 0, 0, 0, 0, 1], [0, 3, 0, 0, 0, -1]],
                    dtype=np.float32)
    h = o.trace_rays(rays, 0.001, INF)
    t = h[:, 2].view(np.float32)
    assert h[0, 0] == (massrt.REF_SPHERE << 28) and t[0] == 4.0 and h[0, 3] == 1  # outside: near root, front
    assert h[1, 0] == (massrt.REF_SPHERE << 28) and t[1] == 1.0 and h[1, 3] == 0  # inside: far root, back face
    assert h[2, 0] == 0 and h[3, 0] == 0  # misses
    # t_max is inclusive (geom.rs:70): a hit exactly at t_max is accepted
    assert o.trace_rays(rays[:1], 0.001, 4.0)[0, 0] != 0
    assert o.trace_rays(rays[:1], 0.001, np.nextafter(np.float32(4.0), np.float32(0)))[0, 0] == 0


def test_triangle_known_answer():
    o = oracle.Scene(1)
    m = lambert_world(o)
    o.add_triangle(m, [0, 0, -2, 1, 0, -2, 0, 1, -2])
    o.build_bvh()
    rays = np.array([[0.25, 0.25, 0, 0, 0, -1], [0.75, 0.75, 0, 0, 0, -1], [0.25, 0.25, 0, 1, 0, 0]],
                    dtype=np.float32)
    h = o.trace_rays(rays)
    assert h[0, 0] == (massrt.REF_TRIANGLE << 28) and h[0, 2].view(np.float32) == 2.0
    assert h[1, 0] == 0  # u + v > 1
    assert h[2, 0] == 0  # |det| < 1e-6 (parallel)


def test_ties_go_to_the_later_object():
    # two identical spheres: BvhNode n=2 keeps the first left; the right child
    # re-tests with t_max = left.t inclusive and wins (geom.rs:192-196)
    for build in (True, False):
        o = oracle.Scene(1)
        m = lambert_world(o)
        o.add_sphere(m, (0, 0, -5), 1.0)
        o.add_sphere(m, (0, 0, -5), 1.0)
        if build:
            o.build_bvh()
        h = o.trace_rays(np.array([[0, 0, 0, 0, 0, -1]], dtype=np.float32))
        assert h[0, 0] == (massrt.REF_SPHERE << 28) | 1


def furnace(kind, param=0.0):
    o = oracle.Scene(1)
    o.background(0, 0, (1.0, 1.0, 1.0))
    s = o.solid(1, 1, 1, 1)
    m = o.material(kind, s, param)
    o.add_sphere(m, (0, 0, 0), 1.0)
    o.build_bvh()
    o.camera(40.0, (0, 0, 4), (0, 0, 0), aspect=ASPECT)
    return o


@pytest.mark.parametrize("kind,param", [(1, 0.0), (2, 0.0), (3, 1.5)])
def test_furnace_exact(kind, param):
    """White materials under a white sky: every sample's radiance is a product
    of 1.0s, i.e. exactly 1 (or 0 for depth-exhausted / absorbed paths)."""
    o = furnace(kind, param)
    spp = 8
    rgb, b = o.render(24, 16, 0, spp, seed=5, threads=4)
    rgb = rgb.reshape(-1, 3)
    assert np.all(rgb == np.round(rgb)) and rgb.max() == spp
    assert np.all(rgb[:, 0] == rgb[:, 1]) and np.all(rgb[:, 1] == rgb[:, 2])
    if kind == 1:
        assert np.all(rgb == spp) and b.max() <= spp  # convex Lambertian: one bounce, never absorbed


def test_golden_fixtures_reproduce(golden_dir):
    g = np.load(golden_dir / "oracle_golden.npz")
    for s in ["cornell", "sphere_grid", "cube_field"]:
        o = oracle.Scene(1).builtin(s, ASPECT, golden_dir)
        rgb, b = o.render(32, 18, 0, 2, seed=3, threads=3)
        assert np.array_equal(b, g[f"{s}_bounces"]), s
        assert np.array_equal(rgb.view(np.uint32), g[f"{s}_rgb"].view(np.uint32)), s
        assert np.array_equal(o.trace_rays(g["rays"]), g[f"{s}_hits"]), s


def test_render_is_deterministic_and_additive(golden_dir):
    """Threads do not change results; [0,4) == [0,2)+[2,4) bit for bit (merge in sample order)."""
    o = oracle.Scene(1).builtin("cornell", ASPECT, golden_dir)
    a = o.render(20, 12, 0, 4, seed=9, threads=1)
    b = o.render(20, 12, 0, 4, seed=9, threads=7)
    c = o.render(20, 12, 0, 2, seed=9, threads=2)
    c = o.render(20, 12, 2, 2, seed=9, threads=5, accum=c)
    for x in (b, c):
        assert np.array_equal(a[0].view(np.uint32), x[0].view(np.uint32)) and np.array_equal(a[1], x[1])


def test_shards_partition_the_frame(golden_dir):
    o = oracle.Scene(1).builtin("sphere_grid", ASPECT, golden_dir)
    full = o.render(40, 24, 0, 1, seed=2, threads=4)
    parts = [o.render(40, 24, 0, 1, seed=2, shard_index=i, shard_count=3, threads=2) for i in range(3)]
    covered = sum((p[1] > 0) | (p[0].reshape(-1, 3).sum(1) > 0) for p in parts)
    assert covered.max() <= 1
    rgb = sum(p[0] for p in parts)
    assert np.array_equal(rgb.view(np.uint32), full[0].view(np.uint32))
    assert np.array_equal(sum(p[1] for p in parts), full[1])


def test_render_pixels_matches_render(golden_dir):
    o = oracle.Scene(1).builtin("cube_field", ASPECT, golden_dir)
    W, H = 30, 17
    rgb, b = o.render(W, H, 0, 3, seed=4, threads=4)
    px = np.array([0, 5, 77, 299, W * H - 1], dtype=np.uint32)
    prgb, pb = o.render_pixels(W, H, px, 0, 3, seed=4, threads=2)
    assert np.array_equal(prgb.reshape(-1, 3), rgb.reshape(-1, 3)[px]) and np.array_equal(pb, b[px])


def test_depth_limits(golden_dir):
    o = oracle.Scene(1).builtin("sphere_grid", ASPECT, golden_dir)
    rgb, b = o.render(16, 9, 0, 2, seed=1, max_depth=0, threads=2)
    assert not rgb.any() and not b.any()  # trace(ray, 0) = (0, 0) (world.rs:66-67)
    rgb, b = o.render(16, 9, 0, 2, seed=1, max_depth=1, threads=2)
    assert b.max() <= 2


@pytest.mark.parametrize("variant", ["specular", "isotrophic", "mix", "mix_nested"])
def test_extended_materials_furnace(variant):
    """Specular (material.rs:331-378), Isotrophic (428-445) and Mix (391-426)
    with white surfaces under a white sky: every radiance is 1 or 0."""
    import massrt
    o = oracle.Scene(3)
    o.background(massrt.BG_SOLID, 0, (1.0, 1.0, 1.0))
    white = o.solid(1, 1, 1, 1)
    if variant == "specular":
        m = o.material(massrt.MAT_SPECULAR, white, 1.8)
    elif variant == "isotrophic":
        m = o.material(massrt.MAT_ISOTROPHIC, 0, 0.0, (1.0, 1.0, 1.0))
    elif variant == "mix":
        m = o.mix(0.3, o.material(massrt.MAT_LAMBERTIAN, white), o.material(massrt.MAT_SPECULAR, white, 1.8))
    else:
        inner = o.mix(0.5, o.material(massrt.MAT_METAL, white, 0.2), o.material(massrt.MAT_DIELECTRIC, 0, 1.5))
        m = o.mix(0.7, inner, o.material(massrt.MAT_LAMBERTIAN, white))
    o.add_sphere(m, (0, 0, 0), 1.0)
    o.build_bvh()
    o.camera(40.0, (0, 0, 4), (0, 0, 0), aspect=1.5)
    spp = 8
    rgb, b = o.render(24, 16, 0, spp, seed=5, threads=4)
    rgb = rgb.reshape(-1, 3)
    assert np.all(rgb == np.round(rgb)) and rgb.max() == spp
    assert b.sum() > 0


def test_volume_free_path_statistics():
    """Volume (geom.rs:595-653): a ray through the centre of a unit sphere of
    density d scatters with probability 1 - exp(-2d); hits lie inside the
    sphere with normal-free front_face = 1; the draw is keyed per ray, so a
    second trace is identical."""
    o = oracle.Scene(1)
    o.add_volume((0, 0, -5), 1.0, 0.5, (0.5, 0.5, 0.5))
    o.build_bvh()
    n = 20_000
    rays = np.zeros((n, 6), np.float32)
    rays[:, 5] = -2.0  # unnormalised direction: distances scale by |d|
    h = o.trace_rays(rays, 0.001, INF)
    hit = h[:, 0] != 0
    assert np.all(h[hit, 0] == (massrt.REF_VOLUME << 28)) and np.all(h[hit, 3] == 1)
    assert abs(hit.mean() - (1 - np.exp(-1.0))) < 0.015
    t = h[hit, 2].view(np.float32)
    assert t.min() >= 2.0 and t.max() <= 3.0  # z in [-6, -4]
    assert np.array_equal(o.trace_rays(rays, 0.001, INF), h)
    # clipped by t_max: nothing past it
    h2 = o.trace_rays(rays, 0.001, 2.25)
    assert np.all(h2[h2[:, 0] != 0, 2].view(np.float32) <= 2.25)


def test_volume_furnace():
    """A white Isotrophic medium under a white sky: every sample is 1 or 0."""
    o = oracle.Scene(3)
    o.background(massrt.BG_SOLID, 0, (1.0, 1.0, 1.0))
    o.add_volume((0, 0, 0), 1.0, 2.0, (1.0, 1.0, 1.0))
    o.build_bvh()
    o.camera(40.0, (0, 0, 4), (0, 0, 0), aspect=1.5)
    spp = 8
    rgb, b = o.render(24, 16, 0, spp, seed=5, threads=4)
    rgb = rgb.reshape(-1, 3)
    assert np.all(rgb == np.round(rgb)) and rgb.max() == spp
    assert b.max() > spp  # multiple scattering inside the medium


def _albedo_of_surface(build_surface, W=4, H=3):
    """Pre-pass albedo of a Lambertian sphere filling the view: the surface's
    get_f(0,0).xyz (material.rs:205-214 attenuation, world.rs:81-92)."""
    o = oracle.Scene(1)
    o.background(massrt.BG_SOLID, 0, (0.0, 0.0, 0.0))
    s = build_surface(o)
    o.add_sphere(o.material(massrt.MAT_LAMBERTIAN, s), (0, 0, 0), 100.0)
    o.build_bvh()
    o.camera(20.0, (0, 0, 0.5), (0, 0, -1), aspect=1.0)
    a, _ = o.prepass(W, H, seed=1, threads=1)
    a = a.reshape(-1, 3)
    assert np.all(a == a[0])
    return a[0]


@pytest.mark.parametrize("mode", [massrt.BLEND_LIGHTEN, massrt.BLEND_DARKEN, massrt.BLEND_ADDITION,
                                  massrt.BLEND_SUBTRACTION])
def test_blend_known_answers(mode):
    """TextureBlend (texture.rs:252-267,303-334) of two solid colours."""
    f = np.float32
    l, r = np.array([0.2, 0.9, 0.5, 1.0], f), np.array([0.6, 0.3, 0.5, 0.5], f)
    got = _albedo_of_surface(lambda o: o.blend(mode, o.solid(*l), o.solid(*r)))
    want = {massrt.BLEND_LIGHTEN: np.maximum(l, r), massrt.BLEND_DARKEN: np.minimum(l, r),
            massrt.BLEND_ADDITION: np.minimum(l + r, f(1)), massrt.BLEND_SUBTRACTION: np.maximum(l - r, f(0))}[mode]
    assert np.array_equal(got, want[:3])


def test_fallback_and_nesting_known_answers():
    """SolidColorFallback (texture.rs:336-357): color*(1-a) + c*a, nested in a blend."""
    f = np.float32
    c, s = np.array([1.0, 0.0, 0.0, 1.0], f), np.array([0.0, 0.0, 1.0, 0.25], f)
    want = c * (f(1) - s[3]) + s * s[3]
    assert np.array_equal(_albedo_of_surface(lambda o: o.fallback(c, o.solid(*s))), want[:3])
    k = np.array([0.1, 0.2, 0.3, 1.0], f)
    got = _albedo_of_surface(lambda o: o.blend(massrt.BLEND_ADDITION, o.solid(*k), o.fallback(c, o.solid(*s))))
    assert np.array_equal(got, np.minimum(k + want, f(1))[:3])


def test_ycbcr_known_answer():
    """YCbCrTexture (texture.rs:197-250) of 1x1 planes: BT.709 matrix as a
    point transform, clamp, powf(2.2)."""
    f = np.float32
    luma = np.array([[[200, 0, 0, 255]]], np.uint8)
    chroma = np.array([[[90, 170, 0, 255]]], np.uint8)
    got = _albedo_of_surface(lambda o: o.ycbcr(o.texture_rgba(luma, massrt.WRAP_CLAMP),
                                               o.texture_rgba(chroma, massrt.WRAP_CLAMP)))
    kr, kg, kb = f(0.2126), f(0.7152), f(0.0722)
    y, u, v = f(200) / f(255), f(90) / f(255) - f(0.5), f(170) / f(255) - f(0.5)
    rgb = np.array([y + f(0) * u + (f(2) - f(2) * kr) * v,
                    y + (-(kb / kg) * (f(2) - f(2) * kb)) * u + (-(kr / kg) * (f(2) - f(2) * kr)) * v,
                    y + (f(2) - f(2) * kb) * u + f(0) * v], f)
    want = np.power(np.clip(rgb, f(0), f(1)), f(2.2))
    assert np.allclose(got, want, rtol=1e-6, atol=0)


def test_cubemap_faces():
    """CubeMap (material.rs:91-190): the major axis of the transformed
    direction picks the face, +y shows the y_neg face and -y the y_pos face
    (the reference's index swap), and all three rotation angles act about x."""
    o = oracle.Scene(1)
    cols = [(1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 0), (0, 1, 1), (1, 0, 1)]
    faces = [o.solid(*c, 1.0) for c in cols]  # x_pos x_neg y_pos y_neg z_pos z_neg

    def centre(look_at, rotation=(0, 0, 0)):
        o.background_cubemap(faces, rotation)
        o.camera(10.0, (0, 0, 0), look_at, view_up=(0, 0, 1) if look_at[2] == 0 and look_at[0] == 0 else (0, 1, 0),
                 aspect=1.0)
        a, _ = o.prepass(3, 3, seed=1, threads=1)
        return tuple(a.reshape(-1, 3)[4])

    o.add_sphere(o.material(massrt.MAT_LAMBERTIAN, o.solid(1, 1, 1, 1)), (700, 800, 900), 1.0)  # off every axis
    o.build_bvh()
    assert centre((1, 0, 0)) == cols[0] and centre((-1, 0, 0)) == cols[1]
    assert centre((0, 1, 0)) == cols[3] and centre((0, -1, 0)) == cols[2]
    assert centre((0, 0, 1)) == cols[4] and centre((0, 0, -1)) == cols[5]
    # a quarter turn about x takes -z to +y (-> the y_neg face); the "y" and
    # "z" angles rotate about x too
    for rot in [(0.25, 0, 0), (0, 0.25, 0), (0, 0, 0.25)]:
        assert centre((0, 0, -1), rot) == cols[3]
