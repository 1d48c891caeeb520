"""Display/export (main.rs:640-722 to_rgb_bytes, 760-783 dump): CPU checks of
the restatement and of the product's host half (gamma table, PNG writer)."""
import numpy as np
import pytest

import massrt
import oracle


def test_gamma_table_is_exact_for_every_float_in_unit_interval():
    """The device maps x in [0,1] to its byte by counting thresholds <= x; the
    oracle checks that against the direct powf formula for all 2^30+1 floats."""
    bad, t = oracle.tonemap_check(threads=0)
    assert bad == 0
    assert np.array_equal(massrt.gamma_thresholds(), t)  # the product derives the same table
    assert t[0] == 0 and np.all(np.diff(t.astype(np.int64)) > 0)


def test_oracle_tonemap_quirks():
    W, H = 4, 2
    rgb = np.array([0.0, 1.0, 2.0, 0.5, 0.25, 4.0, np.nan, -1.0, np.inf, 1e-30, 3.0, 0.9999,
                    0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 1.0, 1.1, 1.2], dtype=np.float32)
    b = np.array([0, 1, 2, 3, 4, 5, 6, 7], dtype=np.uint32)
    out = oracle.tonemap(W, H, rgb, b, 2, massrt.DISPLAY_DEFAULT)
    flat_rows = out[::-1].reshape(-1)  # undo dump()'s row flip -> pixel order
    x = rgb * np.float32(0.5)
    g = np.float32(1.0) / np.float32(2.2)
    with np.errstate(invalid="ignore"):
        v = np.power(x.astype(np.float64), np.float64(g)).astype(np.float32)  # powf up to an ulp
    v = np.where(np.isnan(v), np.float32(1.0), np.minimum(v, np.float32(1.0)))
    v = np.maximum(v, np.float32(0.0))
    exp = np.floor(v * np.float32(255.0)).astype(np.int64)
    assert np.abs(flat_rows.astype(np.int64) - exp).max() <= 1
    # NaN, negative (powf -> NaN) and inf components -> 255 (Rust min returns 1.0); 0 -> 0
    assert flat_rows[6] == 255 and flat_rows[7] == 255 and flat_rows[8] == 255
    assert flat_rows[0] == 0 and flat_rows[1] == 186  # 0.5^(1/2.2) * 255 = 186.3
    # passes == 0 -> black; depth mode
    assert not oracle.tonemap(W, H, rgb, b, 0).any()
    d = oracle.tonemap(W, H, rgb, b, 2, massrt.DISPLAY_DEPTH)[::-1].reshape(-1, 3)
    exp_d = np.floor(np.clip((b.astype(np.float32) * 0.5) / np.float32(7 * 0.5), 0, 1) * np.float32(255)).astype(int)
    assert np.array_equal(d[:, 0], exp_d) and np.array_equal(d[:, 0], d[:, 2])


def test_write_png_roundtrip(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, size=(37, 53, 3), dtype=np.uint8)
    massrt.write_png(tmp_path / "a.png", img)
    back = np.asarray(Image.open(tmp_path / "a.png").convert("RGB"))
    assert np.array_equal(back, img)
    with pytest.raises(massrt.MassrtError):
        massrt.write_png(tmp_path / "no" / "such" / "dir.png", img)


def test_oracle_prepass_furnace_and_views(golden_dir):
    """Camera::albedo_normal (world.rs:81-92): a Lambertian sphere's albedo is
    its colour, misses give the background and a zero normal; the Albedo and
    Normal views follow main.rs:689-718."""
    o = oracle.Scene(3)
    o.background(massrt.BG_SOLID, 0, (0.25, 0.5, 0.75))
    m = o.material(massrt.MAT_LAMBERTIAN, o.solid(0.8, 0.4, 0.2, 1.0))
    o.add_sphere(m, (0, 0, 0), 1.0)
    o.build_bvh()
    o.camera(40.0, (0, 0, 4), (0, 0, 0), aspect=1.0)
    W = H = 33
    a, n = o.prepass(W, H, seed=5)
    a, n = a.reshape(H, W, 3), n.reshape(H, W, 3)
    hit = np.linalg.norm(n, axis=2) > 0
    assert hit[H // 2, W // 2] and not hit[0, 0]
    assert np.allclose(a[hit], np.float32([0.8, 0.4, 0.2])) and np.allclose(a[~hit], np.float32([0.25, 0.5, 0.75]))
    assert np.allclose(np.linalg.norm(n[hit], axis=1), 1.0, atol=1e-5)
    assert n[H // 2, W // 2, 2] > 0.99  # facing the camera
    av = oracle.tonemap(W, H, a.reshape(-1), np.zeros(W * H, np.uint32), 0, massrt.DISPLAY_ALBEDO)
    nv = oracle.tonemap(W, H, n.reshape(-1), np.zeros(W * H, np.uint32), 0, massrt.DISPLAY_NORMAL)
    assert tuple(av[0, 0]) == tuple(np.floor(np.float32([0.25, 0.5, 0.75]) ** np.float32(1 / 2.2) * 255).astype(int))
    assert tuple(nv[0, 0]) == (127, 127, 127)  # (0 + 1) / 2 * 255 = 127.5 -> 127
    # deterministic for a fixed seed
    a2, _ = o.prepass(W, H, seed=5)
    assert np.array_equal(a2, a.reshape(-1))
