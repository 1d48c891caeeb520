"""Random streams: fastrand 1.4.1 wyrand restatement (scene/BVH stream,
math.rs:244-246, geom.rs:111, main.rs:86) and the per-(pixel, sample)
xoroshiro128** path stream shared by the oracle and the GPU.

The wyrand vectors are SURVEY Appendix B (derived from the published
algorithm: fastrand is not vendored in the reference, so they pin the
restatement's arithmetic, not the crate)."""
import numpy as np

import massrt
import oracle

M64 = (1 << 64) - 1


def py_wyrand(seed, n):
    s, out = seed, []
    for _ in range(n):
        s = (s + 0xA0761D6478BD642F) & M64
        t = s * (s ^ 0xE7037ED1A0B428DB)
        out.append(((t >> 64) ^ t) & M64)
    return out


def unit_f32(u32):
    return (np.array([0x3F800000 | (u32 >> 9)], dtype=np.uint32).view(np.float32) - np.float32(1.0))[0]


def test_wyrand_appendix_b():
    want = [0xCDEF1695E1F8ED2C, 0x61D6D24B1C9AAD40, 0x8CF880C22EEBFADF]
    assert py_wyrand(1, 3) == want
    u, f = oracle.wyrand(1, 3)
    assert [int(x) for x in u] == want
    assert np.allclose(f, [0.8827045, 0.111735106, 0.18328822], rtol=0, atol=1e-7)
    assert [unit_f32(w & 0xFFFFFFFF) for w in want] == list(f)


def test_product_and_oracle_scene_streams_agree():
    b = massrt.Builder(1)
    o = oracle.Scene(1)
    a = [b.rand_f32() for _ in range(1000)]
    c = [o.rand_f32() for _ in range(1000)]
    assert np.array_equal(np.float32(a), np.float32(c))
    assert np.array_equal(np.float32(c), oracle.wyrand(1, 1000)[1])


def py_splitmix(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return x, z ^ (z >> 31)


def rotl(v, k):
    return ((v << k) | (v >> (64 - k))) & M64


def py_path_rng(seed, pixel, sample, n):
    x, k = py_splitmix(seed)
    x = k ^ ((pixel << 32) | sample)
    x, s0 = py_splitmix(x)
    x, s1 = py_splitmix(x)
    out = []
    for _ in range(n):
        r = (rotl((s0 * 5) & M64, 7) * 9) & M64
        t = s1 ^ s0
        s0 = rotl(s0, 24) ^ t ^ ((t << 16) & M64)
        s1 = rotl(t, 37)
        out.append(r)
    return out


def test_xoroshiro_first_output_known_answer():
    # xoroshiro128** with state {1, 2}: first output rotl(1*5, 7)*9 = 5760
    assert (rotl(5, 7) * 9) & M64 == 5760


def test_path_rng_restatements_agree():
    for seed, p, s in [(1, 0, 0), (7, 123456, 3), (2**63 + 5, 8294399, 4095)]:
        u, f = oracle.path_rng(seed, p, s, 64)
        assert [int(x) for x in u] == py_path_rng(seed, p, s, 64)
        assert list(f) == [unit_f32(int(x) >> 32) for x in u]
    # distinct streams per pixel and per sample
    a = oracle.path_rng(1, 10, 0, 4)[0]
    b = oracle.path_rng(1, 11, 0, 4)[0]
    c = oracle.path_rng(1, 10, 1, 4)[0]
    assert not np.array_equal(a, b) and not np.array_equal(a, c)


def test_lemire_axis_distribution():
    # u8(0..3) via gen_mod_u32(3): unbiased over many draws
    o = oracle.Scene(1)
    b = massrt.Builder(1)
    tris = np.random.default_rng(1).normal(size=(3000, 9)).astype(np.float32)
    m = b.material(massrt.MAT_NONE)
    b.model(m, tris)
    om = o.material(0)
    o.model(om, tris)
    # both consumed the same number of draws for the same tree
    assert b.rand_f32() == o.rand_f32()
