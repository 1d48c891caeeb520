"""Synthetic inputs for the BASELINE configs the reference has no asset for
(SURVEY Appendix C). Deterministic; written to assets/ (git-ignored).

  cube.ply             copy of the reference's cube.ply (tests/golden/cube.ply)
  mesh_1m.ply          binary_little_endian PLY, 1,000,000 triangles: a displaced
                       torus, 1000 x 500 quads (configs 3/4, PlyLoader path)
  mesh_1m.obj          the same surface as OBJ with v/vt/vn per corner
                       (obj_loader.rs obj_fns path; ObjLoader needs uv + normal)
  albedo_2048.png      2048^2 RGBA8 albedo (config 5, Lambertian(Texture))
  env_4096x2048.png    4096x2048 RGBA8 equirect sky (config 5, SkySphere; the
                       reference loads 8-bit PNG only, texture.rs:30-69)
  environments/        stand-in for eve::environment("j02") (eve.rs:342-364, whose
                       models/environments/ PNGs are not in the reference):
                       stars01_tile2.png (RGBA star tile) and j02/{0..5}.png (8-bit
                       grey luma) + j02/{0..5}_chroma.png (RGB chroma), 256x256

Usage: python tools/gen_assets.py [--out assets] [--all]
"""
from __future__ import annotations

import argparse
import os
import io
import shutil
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
DEFAULT_DIR = REPO / "assets"
NU, NV = 1000, 500  # quads around / across the torus -> 2*NU*NV = 1,000,000 triangles


def torus_grid(nu=NU, nv=NV):
    """Vertex grid (nu+1) x (nv+1) with duplicated seams (for continuous uvs)."""
    u = np.linspace(0.0, 2.0 * np.pi, nu + 1)
    v = np.linspace(0.0, 2.0 * np.pi, nv + 1)
    U, V = np.meshgrid(u, v, indexing="ij")
    R, r0 = 1.6, 0.62

    def pos(U, V):
        r = r0 * (1.0 + 0.12 * np.sin(7.0 * U) * np.sin(5.0 * V))
        x = (R + r * np.cos(V)) * np.cos(U)
        z = (R + r * np.cos(V)) * np.sin(U)
        y = r * np.sin(V)
        return np.stack([x, y, z], axis=-1)

    P = pos(U, V)
    e = 1e-4
    du = pos(U + e, V) - pos(U - e, V)
    dv = pos(U, V + e) - pos(U, V - e)
    N = np.cross(dv, du)
    N /= np.linalg.norm(N, axis=-1, keepdims=True)
    UV = np.stack([U / (2 * np.pi) * 8.0, V / (2 * np.pi) * 4.0], axis=-1)
    return P.astype(np.float32), N.astype(np.float32), UV.astype(np.float32)


def torus_faces(nu=NU, nv=NV):
    i, j = np.meshgrid(np.arange(nu), np.arange(nv), indexing="ij")
    a = i * (nv + 1) + j
    b = (i + 1) * (nv + 1) + j
    c = (i + 1) * (nv + 1) + j + 1
    d = i * (nv + 1) + j + 1
    t1 = np.stack([a, b, c], -1).reshape(-1, 3)
    t2 = np.stack([a, c, d], -1).reshape(-1, 3)
    f = np.empty((t1.shape[0] * 2, 3), dtype=np.int32)
    f[0::2], f[1::2] = t1, t2
    return f


def write_ply(path: Path, P: np.ndarray, F: np.ndarray):
    hdr = ("ply\nformat binary_little_endian 1.0\ncomment massrt synthetic torus\n"
           f"element vertex {P.shape[0]}\nproperty float x\nproperty float y\nproperty float z\n"
           f"element face {F.shape[0]}\nproperty list uchar int vertex_indices\nend_header\n")
    face_dt = np.dtype([("n", "u1"), ("i", "<i4", (3,))])
    fr = np.empty(F.shape[0], dtype=face_dt)
    fr["n"] = 3
    fr["i"] = F
    with open(path, "wb") as f:
        f.write(hdr.encode())
        f.write(np.ascontiguousarray(P, dtype="<f4").tobytes())
        f.write(fr.tobytes())


def write_obj(path: Path, P, N, UV, F):
    with open(path, "w") as f:
        f.write("# massrt synthetic torus (v/vt/vn)\no torus\n")
        buf = io.StringIO()
        np.savetxt(buf, P, fmt="v %.7g %.7g %.7g")
        np.savetxt(buf, UV, fmt="vt %.7g %.7g")
        np.savetxt(buf, N, fmt="vn %.7g %.7g %.7g")
        G = F + 1
        np.savetxt(buf, np.repeat(G, 3, axis=1), fmt="f %d/%d/%d %d/%d/%d %d/%d/%d")
        f.write(buf.getvalue())


def albedo(n=2048):
    y, x = np.mgrid[0:n, 0:n].astype(np.float32) / n
    check = ((np.floor(x * 16) + np.floor(y * 16)) % 2).astype(np.float32)
    rng = np.random.default_rng(5)
    noise = rng.random((n // 64, n // 64)).repeat(64, 0).repeat(64, 1).astype(np.float32)
    r = 0.35 + 0.45 * check + 0.15 * noise
    g = 0.30 + 0.25 * check + 0.30 * np.sin(6.283 * x * 3) ** 2
    b = 0.25 + 0.20 * (1 - check) + 0.30 * y
    img = np.stack([r, g, b, np.ones_like(r)], -1)
    return (np.clip(img, 0, 1) * 255 + 0.5).astype(np.uint8)


def env(w=4096, h=2048):
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    theta = y / h * np.pi  # row 0 = up (SkySphere v = acos(y)/pi)
    phi = x / w * 2 * np.pi
    up = np.cos(theta)
    sky = np.stack([0.45 + 0.25 * up, 0.6 + 0.25 * up, 0.95 + 0.05 * up], -1)
    ground = np.stack([0.35 + 0 * up, 0.3 + 0 * up, 0.25 + 0 * up], -1)
    img = np.where((up > 0)[..., None], sky, ground)
    # a bright sun disc
    sun_t, sun_p = 0.35 * np.pi, 1.2
    d = np.arccos(np.clip(np.sin(theta) * np.sin(sun_t) * np.cos(phi - sun_p) + np.cos(theta) * np.cos(sun_t), -1, 1))
    img = np.where((d < 0.06)[..., None], np.ones_like(img), img)
    img = np.concatenate([img, np.ones_like(img[..., :1])], -1)
    return (np.clip(img, 0, 1) * 255 + 0.5).astype(np.uint8)


def write_png(path: Path, rgba: np.ndarray):
    from PIL import Image
    mode = {2: "L", 3: "RGB", 4: "RGBA"}[rgba.ndim if rgba.ndim == 2 else rgba.shape[-1]]
    Image.fromarray(rgba, mode).save(path, compress_level=1)


def stars(n=256):
    """Sparse white/blue-ish points on black (alpha 1): the star tile."""
    rng = np.random.default_rng(11)
    img = np.zeros((n, n, 4), dtype=np.uint8)
    img[..., 3] = 255
    k = n * n // 180
    ys, xs = rng.integers(0, n, k), rng.integers(0, n, k)
    lum = rng.integers(90, 256, k)
    img[ys, xs, 0] = lum
    img[ys, xs, 1] = lum
    img[ys, xs, 2] = np.minimum(255, lum + 30)
    return img


def nebula_face(face: int, n=256):
    """One cube face of the nebula: smooth value-noise luma (8-bit grey) and
    chroma (R = Cb+0.5, G = Cr+0.5, B unused) as the YCbCr planes."""
    rng = np.random.default_rng(100 + face)

    def smooth(cells, amp):
        g = rng.random((cells + 1, cells + 1))
        t = np.linspace(0, cells, n, endpoint=False)
        i = t.astype(int)
        f = t - i
        f = f * f * (3 - 2 * f)
        a = g[i][:, i] * (1 - f)[None, :] + g[i][:, i + 1] * f[None, :]
        b = g[i + 1][:, i] * (1 - f)[None, :] + g[i + 1][:, i + 1] * f[None, :]
        return amp * (a * (1 - f)[:, None] + b * f[:, None])

    luma = 0.06 + smooth(4, 0.25) + smooth(12, 0.08)
    cb = 0.5 + smooth(3, 0.16) - 0.08
    cr = 0.5 + smooth(5, 0.16) - 0.08
    l8 = (np.clip(luma, 0, 1) * 255 + 0.5).astype(np.uint8)
    ch = np.stack([cb, cr, np.full_like(cb, 0.5)], -1)
    return l8, (np.clip(ch, 0, 1) * 255 + 0.5).astype(np.uint8)


def ensure_environment(out: Path, name: str = "j02"):
    d = out / "environments" / name
    d.mkdir(parents=True, exist_ok=True)
    if not (out / "environments" / "stars01_tile2.png").exists():
        write_png(out / "environments" / "stars01_tile2.png", stars())
    for f in range(6):
        if not (d / f"{f}_chroma.png").exists():
            luma, chroma = nebula_face(f)
            write_png(d / f"{f}.png", luma)
            write_png(d / f"{f}_chroma.png", chroma)


def ensure_assets(out: Path | str = DEFAULT_DIR, mesh: bool = True, textures: bool = False,
                  environment: bool = False) -> Path:
    """Generate the missing assets under `out`. Safe to call from several
    processes at once (pytest -n, ranks): one holds an exclusive lock while it
    writes, every file appears by rename only when complete."""
    import fcntl

    out = Path(out)
    out.mkdir(parents=True, exist_ok=True)
    with open(out / ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        _ensure_locked(out, mesh, textures, environment)
    return out


def _ensure_locked(out: Path, mesh: bool, textures: bool, environment: bool) -> None:
    def publish(name, write):
        if not (out / name).exists():
            tmp = out / f".tmp{os.getpid()}_{name}"
            write(tmp)
            tmp.rename(out / name)

    publish("cube.ply", lambda p: shutil.copy(REPO / "tests" / "golden" / "cube.ply", p))
    if environment:
        ensure_environment(out)
    if mesh and not ((out / "mesh_1m.ply").exists() and (out / "mesh_1m.obj").exists()):
        P, N, UV = torus_grid()
        F = torus_faces()
        publish("mesh_1m.ply", lambda p: write_ply(p, P.reshape(-1, 3), F))
        publish("mesh_1m.obj", lambda p: write_obj(p, P.reshape(-1, 3), N.reshape(-1, 3), UV.reshape(-1, 2), F))
    if textures:
        publish("albedo_2048.png", lambda p: write_png(p, albedo()))
        publish("env_4096x2048.png", lambda p: write_png(p, env()))

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(DEFAULT_DIR))
    ap.add_argument("--all", action="store_true")
    a = ap.parse_args()
    print(ensure_assets(a.out, mesh=True, textures=a.all, environment=a.all))
