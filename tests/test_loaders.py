"""Host loaders (ply_loader.rs, stl_loader.rs, obj_loader.rs) against the
reference's own data file (cube.ply) and hand-made fixtures."""
import struct

import numpy as np
import pytest

import massrt

CUBE_VERTS = np.array([[1, 1, 1], [-1, 1, -1], [-1, 1, 1], [1, -1, -1], [-1, -1, -1], [1, 1, -1], [1, -1, 1],
                       [-1, -1, 1]], dtype=np.float32)
CUBE_FACES = [(0, 1, 2), (1, 3, 4), (5, 6, 3), (7, 3, 6), (2, 4, 7), (0, 7, 6), (0, 5, 1), (1, 5, 3), (5, 0, 6),
              (7, 4, 3), (2, 1, 4), (0, 2, 7)]


def test_cube_ply_parses_exactly(golden_dir):
    tris = massrt.load_ply(golden_dir / "cube.ply")
    assert tris.shape == (12, 9)
    want = np.stack([CUBE_VERTS[list(f)].reshape(9) for f in CUBE_FACES])
    assert np.array_equal(tris, want)


def write_ply(path, verts, faces, fmt="binary_little_endian", extra_vertex_prop=False):
    endian = "<" if fmt == "binary_little_endian" else ">"
    hdr = f"ply\nformat {fmt} 1.0\ncomment test\nelement vertex {len(verts)}\n"
    hdr += "property float x\nproperty float y\nproperty float z\n"
    if extra_vertex_prop:
        hdr += "property uchar red\n"
    hdr += f"element face {len(faces)}\nproperty list uchar int vertex_indices\nend_header\n"
    with open(path, "wb") as f:
        f.write(hdr.encode())
        if fmt == "ascii":
            body = ""
            for v in verts:
                body += " ".join(repr(float(x)) for x in v) + (" 7" if extra_vertex_prop else "") + "\n"
            for fc in faces:
                body += f"{len(fc)} " + " ".join(str(i) for i in fc) + "\n"
            f.write(body.encode())
            return
        for v in verts:
            f.write(struct.pack(endian + "3f", *v))
            if extra_vertex_prop:
                f.write(b"\x07")
        for fc in faces:
            f.write(struct.pack(endian + "B" + "i" * len(fc), len(fc), *fc))


@pytest.mark.parametrize("fmt", ["ascii", "binary_little_endian", "binary_big_endian"])
def test_ply_formats_agree_and_drop_non_triangles(tmp_path, fmt):
    rng = np.random.default_rng(3)
    verts = rng.normal(size=(10, 3)).astype(np.float32)
    faces = [(0, 1, 2), (3, 4, 5, 6), (7, 8, 9), (1, 2, 3)]  # the quad is skipped (ply_loader.rs:396)
    p = tmp_path / f"m_{fmt}.ply"
    write_ply(p, verts, faces, fmt, extra_vertex_prop=True)
    tris = massrt.load_ply(p)
    want = np.stack([verts[list(f)].reshape(9) for f in faces if len(f) == 3])
    assert np.array_equal(tris, want)


def test_ply_errors(tmp_path):
    p = tmp_path / "bad.ply"
    p.write_text("not a ply\n")
    with pytest.raises(massrt.MassrtError, match="magic"):
        massrt.load_ply(p)
    p.write_text("ply\nformat binary_middle_endian 1.0\nend_header\n")
    with pytest.raises(massrt.MassrtError, match="unsupported format"):
        massrt.load_ply(p)
    with pytest.raises(massrt.MassrtError):
        massrt.load_ply(tmp_path / "missing.ply")


def test_stl_binary(tmp_path):
    rng = np.random.default_rng(4)
    tris = rng.normal(size=(5, 9)).astype(np.float32)
    p = tmp_path / "m.stl"
    with open(p, "wb") as f:
        f.write(b"\0" * 80)
        f.write(struct.pack("<I", 5))
        for i, t in enumerate(tris):
            f.write(struct.pack("<3f", 0, 0, 1))  # normals are ignored (stl_loader.rs:34-36)
            f.write(struct.pack("<9f", *t))
            attr = 2 if i == 1 else 0
            f.write(struct.pack("<H", attr) + b"\x01" * attr)
    assert np.array_equal(massrt.load_stl(p), tris)


def test_obj_v_vt_vn_and_double_slash(tmp_path):
    p = tmp_path / "m.obj"
    p.write_text("""# test
mtllib none.mtl
o thing
v 0 0 0
v 1 0 0
v 0 1 0
v 0 0 1
vt 0.25 0.5
vt 1 0
vn 0 0 1
vn 1 0 0
usemtl foo
f 1/1/1 2/2/1 3/1/2 4/2/2
f 2//2 3//1 4//2
""")
    t = massrt.load_obj(p).reshape(-1, 3, 8)
    assert t.shape == (2, 3, 8)
    # first face: only the first three corners are used (obj_loader.rs:421-423)
    assert np.array_equal(t[0, :, :3], [[0, 0, 0], [1, 0, 0], [0, 1, 0]])
    assert np.array_equal(t[0, :, 6:], [[0.25, 0.5], [1, 0], [0.25, 0.5]])
    assert np.array_equal(t[0, 2, 3:6], [1, 0, 0])
    # `v//vn` borrows uvs[0] (obj_loader.rs:400-408)
    assert np.array_equal(t[1, :, 6:], [[0.25, 0.5]] * 3)
    assert np.array_equal(t[1, :, 3:6], [[1, 0, 0], [0, 0, 1], [1, 0, 0]])


def test_obj_face_without_uv_is_an_error(tmp_path):
    p = tmp_path / "m.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nf 1//1 2//1 3//1\n")
    with pytest.raises(massrt.MassrtError, match="parse face"):
        massrt.load_obj(p)  # `v//vn` needs uvs[0]; obj_loader.rs:428
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    with pytest.raises(massrt.MassrtError, match="parse face"):
        massrt.load_obj(p)


def test_png_texture_roundtrip(tmp_path):
    PIL = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(5)
    for mode, ch in [("RGBA", 4), ("RGB", 3), ("L", 1), ("LA", 2)]:
        img = rng.integers(0, 256, size=(7, 11, ch), dtype=np.uint8)
        p = tmp_path / f"t_{mode}.png"
        PIL.fromarray(img if ch > 1 else img[..., 0], mode).save(p)
        b = massrt.Builder(1)
        assert b.texture_png(p) == 0
    p = tmp_path / "pal.png"
    im = PIL.fromarray(rng.integers(0, 4, size=(5, 5), dtype=np.uint8), "P")
    im.putpalette([0, 0, 0, 255, 0, 0, 0, 255, 0, 0, 0, 255])
    im.save(p)
    assert massrt.Builder(1).texture_png(p) == 0


def test_png_decoded_texels_match_pillow(tmp_path):
    """Texture::load_png decodes to_rgba8 bytes (texture.rs:36-39)."""
    PIL = pytest.importorskip("PIL.Image")
    import ctypes as C
    rng = np.random.default_rng(6)
    for mode, ch in [("RGBA", 4), ("RGB", 3), ("L", 1), ("LA", 2)]:
        img = rng.integers(0, 256, size=(9, 13, ch), dtype=np.uint8)
        p = tmp_path / f"t_{mode}.png"
        im = PIL.fromarray(img if ch > 1 else img[..., 0], mode)
        im.save(p)
        want = np.asarray(im.convert("RGBA"))
        b = massrt.Builder(1)
        s = b.texture_png(p)
        m = b.material(massrt.MAT_LAMBERTIAN, s)
        b.add_sphere(m, (0, 0, 0), 1.0)
        d = b.desc_only()
        t = d.textures[0]
        got = np.ctypeslib.as_array(C.cast(t.rgba, C.POINTER(C.c_uint8)), shape=(t.height, t.width, 4))
        assert (t.width, t.height) == (13, 9)
        assert np.array_equal(got, want), mode
