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
