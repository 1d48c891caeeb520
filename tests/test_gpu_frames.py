"""Device-resident Image (mrt_image_*), one context over several devices
(mrt_create_multi) and the drop-in render() loop, on the product kernels.

On the 1-GPU box a multi-device context is rehearsed on devices {0, 0, 0}:
three per-device contexts on the one GPU, slabs moved with peer copies (RCCL
needs distinct devices). Every result must equal the one-device render of the
same samples bit for bit (sums are per pixel, in sample order, on one device).
"""
from __future__ import annotations

import numpy as np
import pytest

import massrt
from conftest import walk_keys

pytestmark = pytest.mark.gpu
W, H = 131, 75  # ragged: 8x8 tiles cut by both frame edges
ASPECT = float(massrt.ASPECT_RATIO)


@pytest.fixture(scope="module")
def scene(golden_dir):
    return massrt.Builder(1).builtin("sphere_grid", ASPECT, golden_dir)


def _ctx(scene, devices=None):
    c = massrt.Context(0) if devices is None else massrt.Context(devices=devices)
    c.upload(scene)
    return c


def _same(a, b):
    return np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


def test_image_equals_host_render(scene):
    c = _ctx(scene)
    ref_rgb, ref_b = c.render(W, H, 0, 5, seed=3)
    img = massrt.Image(c, W, H)
    img.render(3, 0, 3)
    img.render(3, 3, 2)  # merges continue the sample order
    rgb, b, passes = img.read()
    assert passes == 5 and _same(rgb, ref_rgb) and _same(b, ref_b)
    assert np.array_equal(img.tonemap(), c.tonemap(W, H, ref_rgb, ref_b, 5))
    img.clear()
    rgb, b, passes = img.read()
    assert passes == 0 and not rgb.any() and not b.any()
    img.close()
    c.close()


def test_image_prepass_views(scene):
    c = _ctx(scene)
    img = massrt.Image(c, W, H)
    assert not img.tonemap(massrt.DISPLAY_ALBEDO).any()  # no pre-pass yet: zeros (main.rs:690-696)
    img.prepass(1)
    a, n = c.prepass(W, H, seed=1)
    assert np.array_equal(img.tonemap(massrt.DISPLAY_ALBEDO), c.tonemap(W, H, a, np.zeros(W * H, np.uint32), 1,
                                                                        massrt.DISPLAY_ALBEDO))
    assert np.array_equal(img.tonemap(massrt.DISPLAY_NORMAL), c.tonemap(W, H, n, np.zeros(W * H, np.uint32), 1,
                                                                        massrt.DISPLAY_NORMAL))
    img.close()
    c.close()


def test_multi_device_context_render_equals_one_device(scene):
    one = _ctx(scene)
    multi = _ctx(scene, devices=[0, 0, 0])
    assert multi.devices() == [0, 0, 0]
    acc1 = (np.zeros(W * H * 3, np.float32), np.zeros(W * H, np.uint32))
    accm = (np.zeros(W * H * 3, np.float32), np.zeros(W * H, np.uint32))
    for s0 in (0, 2):  # host buffers carried across calls (mrt_render adds)
        acc1 = one.render(W, H, s0, 2, seed=5, accum=acc1)
        accm = multi.render(W, H, s0, 2, seed=5, accum=accm)
    assert _same(acc1[0], accm[0]) and _same(acc1[1], accm[1])
    # counters sum over the devices: the same work as one device
    one.reset_counters(), multi.reset_counters()
    one.render(W, H, 0, 1, seed=5, counters=True)
    multi.render(W, H, 0, 1, seed=5, counters=True)
    c1, cm = one.counters(), multi.counters()
    # (the walk's own counters too on the reference's walk; on the near-first
    # walk they depend on which rays the drain hand-off's reference walk takes)
    for k in walk_keys(one, ("samples", "segments", "node_visits", "sphere_tests", "bounces")):
        assert c1[k] == cm[k], k
    # a multi-process split on top: shard 1 of 2 over three devices covers t % 2 == 1 only
    r1, _ = one.render(W, H, 0, 1, seed=5, shard_index=1, shard_count=2)
    rm, _ = multi.render(W, H, 0, 1, seed=5, shard_index=1, shard_count=2)
    assert _same(r1, rm)
    multi.close()
    one.close()


def test_shading_coherence_counters(scene, golden_dir):
    """ABI v9: the counting k_shade reports, per wave with work, the distinct
    material kinds (a miss counts as one more kind) and material indices of
    its lanes. Bounds that hold for any pool order: at least one wave per 64
    shaded paths, at most one per path; 1 <= kinds <= materials <= 64 per
    wave. (finish_paths 0: no drain hand-off, k_shade shades every segment.)"""
    for name, src, w, h in (("sphere_grid", scene, W, H), ("cornell", None, 48, 27)):
        c = massrt.Context(0, options={"finish_paths": 0})
        c.upload(src if src is not None else massrt.Builder(1).builtin(name, ASPECT, golden_dir))
        c.reset_counters()
        c.render(w, h, 0, 2, seed=5, counters=True)
        k = c.counters()
        waves, shaded = k["shade_waves"], k["shaded"]
        assert shaded == k["segments"] > 0 and -(-shaded // 64) <= waves <= shaded, name
        assert waves <= k["shade_kinds"] <= k["shade_materials"] <= 64 * waves, name
        assert k["shade_kinds"] > waves, name  # several kinds share waves (lights, diffuse, glass, metal, sky)
        c.close()


@pytest.mark.parametrize("finish", [0, None])
def test_shade_bin_is_bit_identical(scene, golden_dir, finish):
    """Option shade_bin: k_shade writes each workgroup's survivors into the
    next pool grouped by the material kind they scattered from (1), or split
    by the new ray's y sign between the pool's two ends (2). Paths are
    independent, so the image is the ungrouped one bit for bit (with and
    without the drain hand-off), and so is the work counted. A 64K-path pool
    makes the 236K samples refill it (2: the refill between the two ends, and
    the gap closed once the work runs out)."""
    for src in (scene, massrt.Builder(1).builtin("cube_field", ASPECT, golden_dir)):
        out, cnt = [], []
        for b in (0, 1, 2):
            opts = {"shade_bin": b, "pool_paths": 1 << 16, **({"finish_paths": finish} if finish is not None else {})}
            c = massrt.Context(0, options=opts)
            c.upload(src)
            out.append(c.render(W, H, 0, 24, seed=13))
            c.reset_counters()
            c.render(W, H, 0, 2, seed=13, counters=True)
            cnt.append(c.counters())
            c.close()
        for j in (1, 2):
            assert _same(out[0][0], out[j][0]) and _same(out[0][1], out[j][1]), j
            for k in ("samples", "segments", "bounces", "shaded", "closest_hits"):
                assert cnt[0][k] == cnt[j][k], (j, k)


@pytest.mark.parametrize("traversal", [0, 1])
def test_prim_run_is_bit_identical(scene, golden_dir, traversal):
    """Option trace_prim_run: k_trace steps the lanes at a primitive alone
    while at least that many are at one (65: never, 1: whenever a lane is,
    -1: the per-walk default).
    Only the order of the lanes' steps changes, never a lane's own walk, so
    the image and the work counted are the same bit for bit (the reference
    walk's kernel has no primitive run: the option changes nothing there)."""
    for src in (scene, massrt.Builder(1).builtin("cube_field", ASPECT, golden_dir),
                massrt.Builder(1).builtin("cornell", ASPECT, golden_dir)):
        out, cnt = [], []
        for p in (65, 1, 32, -1):
            c = massrt.Context(0, options={"trace_prim_run": p, "traversal": traversal})
            c.upload(src)
            out.append(c.render(W, H, 0, 16, seed=21))
            c.reset_counters()
            c.render(W, H, 0, 2, seed=21, counters=True)
            cnt.append(c.counters())
            c.close()
        for j in (1, 2, 3):
            assert _same(out[0][0], out[j][0]) and _same(out[0][1], out[j][1]), j
            for k in ("samples", "segments", "bounces", "shaded", "closest_hits", "triangle_tests", "sphere_tests"):
                assert cnt[0][k] == cnt[j][k], (j, k)


@pytest.mark.parametrize("devices", [[0, 0, 0], [0]])
def test_multi_device_shards_accumulate_into_one_host_buffer(scene, devices):
    """A caller that renders shard 0 then shard 1 of 2 into ONE nonzero host
    buffer on a multi-device context keeps both shards' sums and every other
    pixel's starting value (the copy back used to zero the pixels
    of the shards this call did not render)."""
    one = _ctx(scene)
    multi = _ctx(scene, devices=devices)
    rng = np.random.default_rng(7)
    start = (rng.random(W * H * 3, dtype=np.float32), rng.integers(0, 1000, W * H).astype(np.uint32))
    acc1 = (start[0].copy(), start[1].copy())
    accm = (start[0].copy(), start[1].copy())
    for s0, si in ((0, 0), (0, 1), (2, 0)):  # shard 1 once, shard 0 twice
        acc1 = one.render(W, H, s0, 2, seed=4, shard_index=si, shard_count=2, accum=acc1)
        accm = multi.render(W, H, s0, 2, seed=4, shard_index=si, shard_count=2, accum=accm)
        assert _same(acc1[0], accm[0]) and _same(acc1[1], accm[1]), (s0, si)
    assert not _same(accm[0], start[0])
    multi.close()
    one.close()


def test_multi_device_image_gathers_each_tile_once(scene):
    one = _ctx(scene)
    multi = _ctx(scene, devices=[0, 0, 0])
    ref = one.render(W, H, 0, 4, seed=2)
    img = massrt.Image(multi, W, H)
    img.render(2, 0, 1)
    img.render(2, 1, 3)
    rgb, b, passes = img.read()
    assert passes == 4 and _same(rgb, ref[0]) and _same(b, ref[1])
    sent, _ = img.gather_stats()
    n1, n2 = (massrt.shard_pixels(W, H, i, 3).size for i in (1, 2))
    assert sent == 16 * (n1 + n2)  # device 0's own tiles never move
    ms = img.device_stats()  # every device rendered its share of both calls (HIP events)
    assert len(ms) == 3 and all(x > 0 for x in ms), ms
    assert np.array_equal(img.tonemap(), one.tonemap(W, H, ref[0], ref[1], 4))
    img.close()
    multi.close()
    one.close()


def test_dropin_render_frames(scene):
    """massrt.render (= lib.rs render): workers x frame_limit passes per frame,
    the second frame continues the sample index: frame k equals a direct
    render of samples [6k, 6k + 6)."""
    c = _ctx(scene)
    img = massrt.Image(c, W, H)
    st = massrt.SampleStreams(4)
    seen = []
    for k in range(2):
        n = massrt.render(img, st, frame_limit=2, workers=3, batch=4, update=lambda im, p: seen.append(p))
        assert n == 6
        rgb, b, passes = img.read()
        ref = c.render(W, H, 6 * k, 6, seed=4)
        assert passes == 6 and _same(rgb, ref[0]) and _same(b, ref[1])
    assert seen == [4, 6, 4, 6]
    img.close()
    c.close()


def test_prepass_then_wavefront_on_one_stream(scene):
    """a pre-pass (lane-ray slots) or a fused render (queue 0's
    control word, the results slab) queued on a stream, then a wavefront
    render on the same stream with no host sync, must equal the synced run."""
    import torch

    c = _ctx(scene)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    big_w, big_h = 640, 360  # the pre-pass needs as many slots as pixels
    alb = torch.zeros(big_w * big_h * 3, device=dev)
    nrm = torch.zeros_like(alb)
    out = []
    for sync in (True, False):
        rgb = torch.zeros(W * H * 3, device=dev)
        bo = torch.zeros(W * H, dtype=torch.int32, device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            c.render_device(c.args(W, H, 0, 2, 7, flags=massrt.RENDER_FUSED), rgb.data_ptr(), bo.data_ptr(),
                            s.cuda_stream)
            if sync:
                s.synchronize()
            massrt.lib().mrt_prepass_device(c.h, big_w, big_h, 1, massrt.C.c_void_p(alb.data_ptr()),
                                            massrt.C.c_void_p(nrm.data_ptr()), massrt.C.c_void_p(s.cuda_stream))
            if sync:
                s.synchronize()
            c.render_device(c.args(W, H, 2, 3, 7), rgb.data_ptr(), bo.data_ptr(), s.cuda_stream)
        s.synchronize()
        out.append((rgb.cpu().numpy(), bo.cpu().numpy()))
    assert _same(out[0][0], out[1][0]) and _same(out[0][1], out[1][1])
    ref = c.render(W, H, 0, 5, seed=7)
    assert _same(out[1][0], ref[0])
    c.close()


def test_options_and_tuning(scene, golden_dir):
    """mrt_set_option / mrt_get_option / mrt_get_tuning (ABI v8): the loop's
    knobs come from the caller, the per-scene rules fill in -1."""
    c = massrt.Context(0)
    assert c.get_option("queues") == 2 and c.get_option("trace_box_min") == -1
    c.upload(scene)
    t = c.tuning()
    # traversal AUTO: sphere_grid takes the near-first walk (its own rules: refill 40, k_shade at 7)
    assert c.get_option("traversal") == massrt.TRAVERSAL_AUTO and t["traversal"] == massrt.TRAVERSAL_NEAR_FIRST
    assert t["queues"] == 2 and t["trace_box_min"] == 20 and t["trace_chunk"] == 512 and t["shade_waves"] == 7
    assert t["shade_bin"] == 2 and c.get_option("shade_bin") == -1  # grouped survivors, pool split by y sign (near-first)
    c.set_option("shade_bin", 0)
    assert c.tuning()["shade_bin"] == 0
    c.set_option("shade_bin", -1)
    c.set_option("traversal", massrt.TRAVERSAL_REFERENCE)
    t = c.tuning()
    assert t["traversal"] == massrt.TRAVERSAL_REFERENCE and t["trace_refill"] == 32 and t["shade_waves"] == 8
    assert t["shade_bin"] == 1  # the reference walk: grouped survivors, no pool split
    c.set_option("traversal", massrt.TRAVERSAL_NEAR_FIRST)  # its own rules: refill 40, k_shade at 7
    t = c.tuning()
    assert t["traversal"] == massrt.TRAVERSAL_NEAR_FIRST and t["trace_refill"] == 40 and t["shade_waves"] == 7
    c.set_option("traversal", massrt.TRAVERSAL_REFERENCE)
    c.set_option("trace_box_min", 40)
    assert c.tuning()["trace_box_min"] == 40 and c.get_option("trace_box_min") == 40
    cube = massrt.Builder(1).builtin("cube_field", ASPECT, golden_dir)
    c.set_option("trace_box_min", -1)
    c.upload(cube)  # > 1000 instances: box run from 16 lanes, grabs of 128
    assert c.tuning()["trace_box_min"] == 16 and c.tuning()["trace_chunk"] == 128
    assert c.tuning()["trace_refill"] == 32  # 12 only for a big instanced world (Menger)
    for name, bad in (("queues", 5), ("trace_block", 300), ("shade_waves", 6), ("trace_chunk", 8), ("trace_nf_batch", 0),
                      ("traversal", 2)):
        with pytest.raises(massrt.MassrtError, match=name):
            c.set_option(name, bad)
    with pytest.raises(massrt.MassrtError, match="unknown option"):
        c.set_option("no_such_knob", 1)
    ref = c.render(W, H, 0, 2, seed=9)
    c.set_option("queues", 1)  # the pool is re-split: same image
    assert c.tuning()["queues"] == 1
    again = c.render(W, H, 0, 2, seed=9)
    assert _same(ref[0], again[0]) and _same(ref[1], again[1])
    c.close()


def test_transport_and_image_lifetime(scene):
    one = _ctx(scene)
    multi = _ctx(scene, devices=[0, 0])
    assert one.transport() == "none" and multi.transport() == "peer"
    with pytest.raises(massrt.MassrtError, match="distinct devices"):
        multi.set_option("gather", massrt.GATHER_RCCL)
    img = massrt.Image(multi, W, H)
    img.render(1, 0, 2)
    assert img.passes == 2
    assert img.gather_stats()[0] == 0  # the pass count alone gathers nothing
    img.gather()
    assert img.gather_stats()[0] == 16 * massrt.shard_pixels(W, H, 1, 2).size
    # an image must be destroyed before its context: mrt_destroy refuses
    assert massrt.lib().mrt_destroy(multi.h) == 4  # MRT_ERR_STATE
    assert "image" in massrt.lib().mrt_last_error(multi.h).decode()
    multi.close()  # closes the image first
    assert img.h is None and multi.h is None
    one.close()


def test_constrained_memory_renders_in_chunks(scene):
    """a render sizes its pool and results slab to the free device
    memory minus mem_reserve_mb (several contexts may share a device). With
    almost no memory left to it, a multi-device context over repeated devices
    shrinks the pool and the samples per chunk — and renders the same image."""
    import torch

    Wl, Hl, spp = 640, 360, 24
    one = _ctx(scene)
    ref = one.render(Wl, Hl, 0, spp, seed=12)
    one.close()
    multi = massrt.Context(devices=[0, 0, 0])
    multi.upload(scene)
    multi.render(Wl, Hl, 0, 1, seed=12)  # the per-frame buffers, kernels and scratch in place at 1 spp
    free_mb = torch.cuda.mem_get_info(0)[0] >> 20  # what the 24-spp render re-plans its pools and slabs from
    multi.set_option("mem_reserve_mb", max(0, free_mb - 400))
    got = multi.render(Wl, Hl, 0, spp, seed=12)
    t = multi.tuning()
    multi.close()
    assert _same(ref[0], got[0]) and _same(ref[1], got[1]), t
