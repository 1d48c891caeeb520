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
    for k in ("samples", "segments", "node_visits", "sphere_tests", "bounces"):
        assert c1[k] == cm[k], k
    # a multi-process split on top: shard 1 of 2 over three devices covers t % 2 == 1 only
    r1, _ = one.render(W, H, 0, 1, seed=5, shard_index=1, shard_count=2)
    rm, _ = multi.render(W, H, 0, 1, seed=5, shard_index=1, shard_count=2)
    assert _same(r1, rm)
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
