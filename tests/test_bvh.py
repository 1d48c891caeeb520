"""BVH topology: the host builder (product) and the oracle must build the
reference's tree (BvhNode::new, geom.rs:110-161: one fastrand::u8(0..3)
draw per call, stable sort on bbox.min[axis], median split, n=2 pop order)
node for node, box for box."""
import numpy as np
import pytest

import massrt
import oracle


def T(n):
    # node count of BvhNode::new over n items: T(1)=T(2)=1, T(n)=1+T(n//2)+T(n-n//2)
    memo = {1: 1, 2: 1}

    def t(k):
        if k not in memo:
            memo[k] = 1 + t(k // 2) + t(k - k // 2)
        return memo[k]
    return t(n)


def assert_same_tree(b: massrt.Builder, o: oracle.Scene):
    d = b.desc_only()
    lst, boxes = massrt.preorder(d)
    k, bx = o.preorder()
    assert [tuple(x) for x in k.tolist()] == lst
    pb = np.array([x for x in boxes if x is not None], dtype=np.float32).reshape(-1, 6)
    ob = bx[k[:, 0] == 1]
    assert np.array_equal(pb.view(np.uint32), ob.view(np.uint32))
    # every BLAS (Model::new trees) too
    for m in range(o.blas_count()):
        kb, bb = o.blas_preorder(m)
        assert kb[0, 0] == 1
    return d


def test_node_count_formula():
    assert T(12) == 15 and T(10_001) == 11_809 and T(1_000_000) == 1_048_575


@pytest.mark.parametrize("name", ["cornell", "sphere_grid", "cube_field"])
def test_builtin_scene_topology(name, golden_dir):
    aspect = float(massrt.ASPECT_RATIO)
    b = massrt.Builder(1).builtin(name, aspect, golden_dir)
    o = oracle.Scene(1).builtin(name, aspect, golden_dir)
    d = assert_same_tree(b, o)
    cam, _ = b.desc()[1], None
    assert np.array_equal(cam.fields().view(np.uint32), o.camera_fields().view(np.uint32))
    if name == "sphere_grid":
        assert d.n_nodes == T(10_001) + T(12)
        assert d.n_spheres == 10_000 and d.n_instances == 1


@pytest.mark.parametrize("name", ["mesh_ply", "mesh_obj", "mesh_obj_textured"])
def test_mesh_scene_topology(name, assets_dir):
    aspect = float(massrt.ASPECT_RATIO)
    b = massrt.Builder(1).builtin(name, aspect, assets_dir)
    o = oracle.Scene(1).builtin(name, aspect, assets_dir)
    d = b.desc_only()
    assert d.n_triangles == 1_000_000 + 12
    lst, _ = massrt.preorder(d)
    k, _ = o.preorder()
    assert [tuple(x) for x in k.tolist()] == lst
    # the 1M-triangle BLAS, node for node and box for box
    m = d.models[0]
    sub = massrt.MrtSceneDesc()
    sub.nodes = d.nodes
    sub.roots = (massrt.C.c_uint32 * 1)((massrt.REF_NODE << 28) | m.blas_root)
    sub.n_roots = 1
    l2, b2 = massrt.preorder(sub)
    kb, bb = o.blas_preorder(1)
    assert [tuple(x) for x in kb.tolist()] == l2
    pb = np.array([x for x in b2 if x is not None], dtype=np.float32)
    assert np.array_equal(pb.view(np.uint32), bb[kb[:, 0] == 1].view(np.uint32))
    assert sum(1 for x in l2 if x[0] == 1) == T(1_000_000)


def random_world(seed, n_spheres, ties, ctx=None):
    """Same random world built through both builders (the product's top-level
    tree on ctx's device when ctx is given, build.hip)."""
    rng = np.random.default_rng(seed)
    b, o = massrt.Builder(seed), oracle.Scene(seed)
    sb, so = b.solid(0.5, 0.5, 0.5), o.solid(0.5, 0.5, 0.5)
    mb, mo = b.material(massrt.MAT_LAMBERTIAN, sb), o.material(1, so)
    cube = np.array([[1, 1, 1, -1, 1, -1, -1, 1, 1], [1, -1, -1, -1, -1, -1, 1, 1, -1]], dtype=np.float32)
    kb = b.model(mb, cube)
    ko = o.model(mo, cube)
    for i in range(n_spheres):
        c = rng.integers(-3, 3, size=3).astype(np.float32) if ties else rng.normal(size=3).astype(np.float32) * 5
        r = float(rng.choice([0.5, 1.0, -0.5])) if ties else float(rng.uniform(0.1, 1))
        b.add_sphere(mb, c, r)
        o.add_sphere(mo, c, r)
        if i % 7 == 0:
            t, rot, s = rng.normal(size=3), rng.normal(size=3), rng.uniform(0.5, 2, size=3)
            b.add_instance(kb, t, rot, s, mb)
            o.add_instance(ko, t, rot, s, mo)
        if i % 11 == 0:
            tri = rng.integers(-2, 2, size=9).astype(np.float32) if ties else rng.normal(size=9).astype(np.float32)
            b.add_triangle(mb, tri)
            o.add_triangle(mo, tri)
    if ctx is None:
        b.build_bvh()
    else:
        b.build_bvh_device(ctx)
    o.build_bvh()
    return b, o


@pytest.mark.parametrize("seed,n,ties", [(1, 1, False), (2, 2, False), (3, 3, True), (4, 64, True),
                                         (5, 333, False), (6, 1000, True)])
def test_random_worlds_same_tree(seed, n, ties):
    b, o = random_world(seed, n, ties)
    assert_same_tree(b, o)
    assert b.rand_f32() == o.rand_f32()  # same number of scene-stream draws


def test_two_items_pop_order():
    # n == 2: a = items.pop() (last) goes left only if a.min < b.min (geom.rs:122-129)
    for order in [(0.0, 5.0), (5.0, 0.0), (2.0, 2.0)]:
        b, o = massrt.Builder(9), oracle.Scene(9)
        s = b.solid(1, 1, 1)
        m = b.material(massrt.MAT_LAMBERTIAN, s)
        om = o.material(1, o.solid(1, 1, 1))
        for x in order:
            b.add_sphere(m, (x, x, x), 1.0)
            o.add_sphere(om, (x, x, x), 1.0)
        b.build_bvh()
        o.build_bvh()
        lst, _ = massrt.preorder(b.desc_only())
        first = lst[1][1]
        assert first == (1 if order[1] < order[0] else 0)
        assert_same_tree(b, o)


def test_menger_topology(assets_dir):
    """Menger (menger.rs:20-115): 20^3 cubes node for node; the full 20^5 =
    3.2M-instance scene by node/instance counts and the
    number of scene-stream draws (one per BvhNode::new call)."""
    aspect = float(massrt.ASPECT_RATIO)
    b = massrt.Builder(1).builtin("menger_l3", aspect, assets_dir)
    o = oracle.Scene(1).builtin("menger_l3", aspect, assets_dir)
    d = assert_same_tree(b, o)
    assert d.n_instances == 8_001 and d.n_nodes == T(8_001) + 2 * T(12)
    assert np.array_equal(b.desc()[1].fields().view(np.uint32), o.camera_fields().view(np.uint32))
    b = massrt.Builder(1).builtin("menger", aspect, assets_dir)
    o = oracle.Scene(1).builtin("menger", aspect, assets_dir)
    d = b.desc_only()
    assert d.n_instances == 3_200_001 and d.n_nodes == T(3_200_001) + 2 * T(12) == 4_194_333
    assert b.rand_f32() == o.rand_f32()


def test_device_build_needs_context():
    b = massrt.Builder(1)
    m = b.material(massrt.MAT_LAMBERTIAN, b.solid(1, 1, 1))
    b.add_sphere(m, (0, 0, 0), 1.0)
    assert massrt.lib().mrt_builder_build_bvh_device(b.h, None) != 0


# ---- device tree build (csrc/device/build.hip): the same tree, node for node


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,ties", [(1, 1, False), (2, 2, False), (3, 3, True), (4, 64, True),
                                         (5, 333, False), (6, 1000, True), (7, 20_000, False),
                                         (8, 20_000, True)])
def test_device_build_random_worlds(ctx, seed, n, ties):
    b, o = random_world(seed, n, ties, ctx=ctx)
    assert_same_tree(b, o)
    assert b.rand_f32() == o.rand_f32()  # same number of scene-stream draws


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell", "sphere_grid", "cube_field", "menger"])
def test_device_build_builtin_scenes(ctx, name, assets_dir):
    aspect = float(massrt.ASPECT_RATIO)
    h = massrt.Builder(1).builtin(name, aspect, assets_dir)
    b = massrt.Builder(1).builtin_device(name, ctx, aspect, assets_dir)
    lh, bh = massrt.preorder(h.desc_only())
    lb, bb = massrt.preorder(b.desc_only())
    assert lh == lb
    ph = np.array([x for x in bh if x is not None], dtype=np.float32)
    pd = np.array([x for x in bb if x is not None], dtype=np.float32)
    assert np.array_equal(ph.view(np.uint32), pd.view(np.uint32))
    assert h.rand_f32() == b.rand_f32()
    host_ms, dev_ms = b.last_build_ms()
    assert host_ms >= 0 and dev_ms > 0


@pytest.mark.gpu
def test_failed_device_build_leaves_world_unchanged(ctx):
    """A device build that fails (a NaN sort key in a node of >= 3 items) must
    leave the world and the scene stream as they were: the host build after it
    is the reference's tree and draws the same axes."""
    def world(x):
        m = x.material(1 if isinstance(x, oracle.Scene) else massrt.MAT_LAMBERTIAN, x.solid(1, 1, 1))
        for k in range(9):
            x.add_sphere(m, (float(k), 0.5 * k, -1.0 * k), 0.7)
        x.add_sphere(m, (float("nan"),) * 3, 1.0)
        return x

    b, o = world(massrt.Builder(3)), world(oracle.Scene(3))
    with pytest.raises(massrt.MassrtError, match="NaN"):
        b.build_bvh_device(ctx)
    b.build_bvh()
    o.build_bvh()
    assert_same_tree(b, o)
    assert b.rand_f32() == o.rand_f32()


@pytest.mark.gpu
def test_device_build_two_items_with_nan_key(ctx):
    """2 items: the reference compares once (a NaN compares false: the first
    item goes left, geom.rs:122-129); the device build must agree, not fail."""
    for first_nan in (True, False):
        b, o = massrt.Builder(4), oracle.Scene(4)
        mb, mo = b.material(massrt.MAT_LAMBERTIAN, b.solid(1, 1, 1)), o.material(1, o.solid(1, 1, 1))
        centers = [(float("nan"),) * 3, (1.0, 2.0, 3.0)]
        if not first_nan:
            centers.reverse()
        for c in centers:
            b.add_sphere(mb, c, 1.0)
            o.add_sphere(mo, c, 1.0)
        b.build_bvh_device(ctx)
        o.build_bvh()
        lst, boxes = massrt.preorder(b.desc_only())
        k, bx = o.preorder()
        assert [tuple(x) for x in k.tolist()] == lst
        assert b.rand_f32() == o.rand_f32()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_device_build_signed_zeros(ctx, seed):
    """Keys of -0.0 and +0.0 (one key: `<` cannot order them) and node boxes
    whose join picks between -0 and +0: device tree == host tree == oracle,
    boxes compared as bits."""
    rng = np.random.default_rng(seed)
    vals = np.array([-0.0, 0.0, 1.0, -1.0], dtype=np.float32)
    items = [(tuple(float(v) for v in rng.choice(vals, 3)), float(rng.choice([0.0, 1.0]))) for _ in range(300)]

    def world(x, lam):
        m = x.material(lam, x.solid(1, 1, 1))
        for c, r in items:
            x.add_sphere(m, c, r)
        return x

    h = world(massrt.Builder(seed), massrt.MAT_LAMBERTIAN)
    d = world(massrt.Builder(seed), massrt.MAT_LAMBERTIAN)
    o = world(oracle.Scene(seed), 1)
    h.build_bvh()
    d.build_bvh_device(ctx)
    o.build_bvh()
    assert_same_tree(h, o)
    assert_same_tree(d, o)
    lh, bh = massrt.preorder(h.desc_only())
    ld, bd = massrt.preorder(d.desc_only())
    assert lh == ld
    ph = np.array([x for x in bh if x is not None], dtype=np.float32)
    pd = np.array([x for x in bd if x is not None], dtype=np.float32)
    assert np.array_equal(ph.view(np.uint32), pd.view(np.uint32))
    assert (np.signbit(ph) & (ph == 0)).any() and (~np.signbit(ph) & (ph == 0)).any()  # both zeros occur
