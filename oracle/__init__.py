"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU restatement
(oracle/oracle.cpp). Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module; the product never does.

PARITY UNPINNED against the reference binary itself (no Rust toolchain here,
no golden vectors in the reference); pinned by cube.ply, analytic known
answers and the published fastrand algorithm. See oracle/oracle.h.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "liboracle.so"
NO_MATERIAL = 0xFFFFFFFF
_lib = None


def build() -> Path:
    subprocess.run(["make", "-C", str(HERE), "-s"], check=True)
    return LIB


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB.exists():
        build()
    L = C.CDLL(str(LIB))
    P, U32, U64, F, I, I64 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_float, C.c_int, C.c_int64
    fp, up, dp = C.POINTER(C.c_float), C.POINTER(C.c_uint32), C.POINTER(C.c_double)
    sig = {
        "orc_last_error": (C.c_char_p, []),
        "orc_new": (P, [U64]),
        "orc_free": (None, [P]),
        "orc_builtin": (I, [P, C.c_char_p, F, C.c_char_p]),
        "orc_rand_f32": (F, [P]),
        "orc_solid": (I, [P, F, F, F, F]),
        "orc_texture_rgba": (I, [P, C.POINTER(C.c_uint8), U32, U32, U32]),
        "orc_texture_png": (I, [P, C.c_char_p, U32]),
        "orc_material": (I, [P, U32, U32, F, F, F, F]),
        "orc_background": (I, [P, U32, U32, F, F, F]),
        "orc_ycbcr": (I, [P, U32, U32]),
        "orc_blend": (I, [P, U32, U32, U32]),
        "orc_fallback": (I, [P, F, F, F, F, U32]),
        "orc_background_cubemap": (I, [P, C.POINTER(C.c_uint32), fp]),
        "orc_mix": (I, [P, F, U32, U32]),
        "orc_add_sphere": (I, [P, U32, F, F, F, F]),
        "orc_add_volume": (I, [P, F, F, F, F, F, F, F, F]),
        "orc_add_triangle": (I, [P, U32, fp]),
        "orc_model": (I, [P, U32, U32, fp, U32, I, I]),
        "orc_model_from_ply": (I, [P, C.c_char_p, U32, U32, I]),
        "orc_add_instance": (I, [P, I, fp, fp, fp, U32]),
        "orc_camera": (I, [P, F, fp, fp, fp, F, F, F]),
        "orc_build_bvh": (I, [P]),
        "orc_camera_fields": (I, [P, fp]),
        "orc_export_preorder": (I64, [P, up, fp, U64]),
        "orc_blas_count": (I64, [P]),
        "orc_export_blas": (I64, [P, I64, up, fp, U64]),
        "orc_trace_rays": (I, [P, fp, U32, F, F, P]),
        "orc_render": (I, [P, U32, U32, U32, U32, U64, U32, U32, U32, I, fp, up]),
        "orc_render_pixels": (I, [P, U32, U32, up, U32, U32, U32, U64, U32, I, fp, up]),
        "orc_bench_reference_mode": (C.c_double, [P, U32, U32, U32, U64, U32, I, fp, up, U32, U32, U32]),
        "orc_get_counters": (None, [P, P]),
        "orc_wyrand": (None, [U64, U32, C.POINTER(C.c_uint64), fp]),
        "orc_path_rng": (None, [U64, U32, U32, U32, C.POINTER(C.c_uint64), fp]),
        "orc_reset_counters": (None, [P]),
        "orc_set_counting": (None, [P, I]),
        "orc_tonemap": (I, [U32, U32, fp, up, U32, U32, C.POINTER(C.c_uint8)]),
        "orc_tonemap_check": (U64, [up, I]),
        "orc_prepass": (I, [P, U32, U32, U64, I, fp, fp]),
        "orc_render_refrng": (I, [P, U32, U32, U32, U64, U32, U32, I, dp, dp, dp, dp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


COUNTER_FIELDS = ["samples", "segments", "node_visits", "sphere_tests", "triangle_tests", "instance_entries",
                  "model_entries", "closest_hits", "texel_taps", "bounces", "alpha_taps"]


class _Counters(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in COUNTER_FIELDS]


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _up(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def _f3(v):
    return np.ascontiguousarray(np.asarray(v, dtype=np.float32).reshape(3))


def tonemap(width, height, rgb, bounces, passes, mode=0) -> np.ndarray:
    """Image::to_rgb_bytes + dump row flip (main.rs:640-722,760-767) on the CPU."""
    rgb = np.ascontiguousarray(rgb, dtype=np.float32).reshape(-1)
    b = np.ascontiguousarray(bounces, dtype=np.uint32).reshape(-1)
    out = np.empty(width * height * 3, dtype=np.uint8)
    lib().orc_tonemap(width, height, _fp(rgb), _up(b), passes, mode, out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out.reshape(height, width, 3)


def tonemap_check(threads=0):
    """(mismatches, thresholds): the threshold-table byte vs powf over every f32 in [0, 1]."""
    t = np.zeros(256, dtype=np.uint32)
    bad = lib().orc_tonemap_check(_up(t), threads)
    return int(bad), t


def wyrand(seed: int, n: int):
    u = np.zeros(n, dtype=np.uint64)
    f = np.zeros(n, dtype=np.float32)
    lib().orc_wyrand(seed, n, u.ctypes.data_as(C.POINTER(C.c_uint64)), _fp(f))
    return u, f


def path_rng(seed: int, pixel: int, sample: int, n: int):
    u = np.zeros(n, dtype=np.uint64)
    f = np.zeros(n, dtype=np.float32)
    lib().orc_path_rng(seed, pixel, sample, n, u.ctypes.data_as(C.POINTER(C.c_uint64)), _fp(f))
    return u, f


class OracleError(RuntimeError):
    pass


class Scene:
    """Reference-shaped CPU scene (World + Camera) with the builder API of massrt.Builder."""

    def __init__(self, rng_seed: int = 1):
        self.h = lib().orc_new(rng_seed)

    def __del__(self):
        try:
            if self.h:
                lib().orc_free(self.h)
                self.h = None
        except Exception:
            pass

    def _chk(self, rc):
        if rc < 0:
            raise OracleError(lib().orc_last_error().decode())
        return rc

    def builtin(self, name, aspect, asset_dir=""):
        self._chk(lib().orc_builtin(self.h, name.encode(), aspect, str(asset_dir).encode()))
        return self

    def rand_f32(self):
        return lib().orc_rand_f32(self.h)

    def solid(self, r, g, b, a=1.0):
        return self._chk(lib().orc_solid(self.h, r, g, b, a))

    def texture_rgba(self, rgba, wrap=1):
        rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
        h, w = rgba.shape[:2]
        return self._chk(lib().orc_texture_rgba(self.h, rgba.ctypes.data_as(C.POINTER(C.c_uint8)), w, h, wrap))

    def material(self, kind, surface=0, param=0.0, emit=(0.0, 0.0, 0.0)):
        return self._chk(lib().orc_material(self.h, kind, surface, param, *emit))

    def mix(self, ratio, left, right):
        return self._chk(lib().orc_mix(self.h, ratio, left, right))

    def background(self, kind, surface=0, color=(0.0, 0.0, 0.0)):
        self._chk(lib().orc_background(self.h, kind, surface, *color))

    def ycbcr(self, luma, chroma):
        return self._chk(lib().orc_ycbcr(self.h, luma, chroma))

    def blend(self, mode, left, right):
        return self._chk(lib().orc_blend(self.h, mode, left, right))

    def fallback(self, color, surface):
        return self._chk(lib().orc_fallback(self.h, *[float(c) for c in color], surface))

    def background_cubemap(self, faces, rotation=(0.0, 0.0, 0.0)):
        f = np.ascontiguousarray(faces, dtype=np.uint32).reshape(6)
        r = np.ascontiguousarray(rotation, dtype=np.float32).reshape(3)
        self._chk(lib().orc_background_cubemap(self.h, f.ctypes.data_as(C.POINTER(C.c_uint32)), _fp(r)))

    def add_sphere(self, material, center, radius):
        self._chk(lib().orc_add_sphere(self.h, material, *[float(c) for c in center], radius))

    def add_volume(self, center, radius, density, albedo):
        """geom.rs:595 Volume(Sphere(center, radius), density, albedo)."""
        self._chk(lib().orc_add_volume(self.h, *[float(c) for c in center], float(radius), float(density),
                                       *[float(c) for c in albedo]))

    def add_triangle(self, material, abc):
        a = np.ascontiguousarray(np.asarray(abc, dtype=np.float32).reshape(9))
        self._chk(lib().orc_add_triangle(self.h, material, _fp(a)))

    def model(self, tri_material, tris, override=NO_MATERIAL, add_to_world=False, shading=False):
        t = np.ascontiguousarray(tris, dtype=np.float32)
        return self._chk(lib().orc_model(self.h, tri_material, override, _fp(t), t.shape[0], int(shading),
                                         int(add_to_world)))

    def model_from_ply(self, path, tri_material, override=NO_MATERIAL, add_to_world=False):
        return self._chk(lib().orc_model_from_ply(self.h, str(path).encode(), tri_material, override,
                                                  int(add_to_world)))

    def add_instance(self, model, translation, rotation, scale, material=NO_MATERIAL):
        t, r, s = _f3(translation), _f3(rotation), _f3(scale)
        self._chk(lib().orc_add_instance(self.h, model, _fp(t), _fp(r), _fp(s), material))

    def camera(self, vfov, look_from, look_at, view_up=(0, 1, 0), aspect=16 / 9, aperture=0.0, focus=None):
        f, a, u = _f3(look_from), _f3(look_at), _f3(view_up)
        if focus is None:
            d = (f - a).astype(np.float32)
            focus = float(np.sqrt(np.float32(d[0] * d[0] + d[1] * d[1]) + np.float32(d[2] * d[2])))
        lib().orc_camera(self.h, vfov, _fp(f), _fp(a), _fp(u), aspect, aperture, focus)

    def build_bvh(self):
        self._chk(lib().orc_build_bvh(self.h))

    def camera_fields(self) -> np.ndarray:
        o = np.zeros(19, dtype=np.float32)
        lib().orc_camera_fields(self.h, _fp(o))
        return o

    def _listing(self, n, fill):
        kinds = np.zeros((max(n, 1), 2), dtype=np.uint32)
        boxes = np.zeros((max(n, 1), 6), dtype=np.float32)
        fill(_up(kinds), _fp(boxes), n)
        return kinds[:n], boxes[:n]

    def preorder(self):
        n = lib().orc_export_preorder(self.h, None, None, 0)
        return self._listing(n, lambda k, b, c: lib().orc_export_preorder(self.h, k, b, c))

    def blas_count(self):
        return lib().orc_blas_count(self.h)

    def blas_preorder(self, i):
        n = lib().orc_export_blas(self.h, i, None, None, 0)
        return self._listing(n, lambda k, b, c: lib().orc_export_blas(self.h, i, k, b, c))

    def trace_rays(self, rays, t_min=0.001, t_max=float("inf")):
        r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        out = np.zeros((r.shape[0], 4), dtype=np.uint32)
        self._chk(lib().orc_trace_rays(self.h, _fp(r), r.shape[0], t_min, t_max, out.ctypes.data_as(C.c_void_p)))
        return out

    def render(self, width, height, spp_begin=0, spp_count=1, seed=1, max_depth=50, shard_index=0, shard_count=1,
               threads=0, accum=None):
        if accum is None:
            rgb = np.zeros(width * height * 3, dtype=np.float32)
            b = np.zeros(width * height, dtype=np.uint32)
        else:
            rgb, b = accum
        self._chk(lib().orc_render(self.h, width, height, spp_begin, spp_count, seed, max_depth, shard_index,
                                   shard_count, threads, _fp(rgb), _up(b)))
        return rgb, b

    def prepass(self, width, height, seed=1, threads=0):
        """Camera::albedo_normal pre-pass (world.rs:81-92): (albedo, normal) float32 [H*W*3]."""
        a = np.zeros(width * height * 3, dtype=np.float32)
        n = np.zeros(width * height * 3, dtype=np.float32)
        self._chk(lib().orc_prepass(self.h, width, height, seed, threads, _fp(a), _fp(n)))
        return a, n

    def render_pixels(self, width, height, pixels, spp_begin=0, spp_count=1, seed=1, max_depth=50, threads=0):
        px = np.ascontiguousarray(pixels, dtype=np.uint32)
        rgb = np.zeros(px.size * 3, dtype=np.float32)
        b = np.zeros(px.size, dtype=np.uint32)
        self._chk(lib().orc_render_pixels(self.h, width, height, _up(px), px.size, spp_begin, spp_count, seed,
                                          max_depth, threads, _fp(rgb), _up(b)))
        return rgb, b

    def bench_reference_mode(self, width, height, passes_per_thread, seed=1, max_depth=50, threads=0, row_begin=0,
                             row_end=0, row_step=1):
        rgb = np.zeros(width * height * 3, dtype=np.float32)
        b = np.zeros(width * height, dtype=np.uint32)
        secs = lib().orc_bench_reference_mode(self.h, width, height, passes_per_thread, seed, max_depth, threads,
                                              _fp(rgb), _up(b), row_begin, row_end, row_step)
        if secs < 0:
            raise OracleError("reference-mode bench failed")
        return secs, rgb, b

    def render_refrng(self, width, height, passes, workers, seed=1, max_depth=50, threads=0):
        """Reference RNG semantics (one fastrand stream per worker, pixel-loop
        order): sums and sums of squares of the radiance [H*W*3] and of the
        bounce counts [H*W] over passes x workers samples per pixel (float64)."""
        s = np.zeros(width * height * 3)
        q = np.zeros(width * height * 3)
        b = np.zeros(width * height)
        bq = np.zeros(width * height)
        dp = C.POINTER(C.c_double)
        self._chk(lib().orc_render_refrng(self.h, width, height, passes, seed, max_depth, workers, threads,
                                          s.ctypes.data_as(dp), q.ctypes.data_as(dp), b.ctypes.data_as(dp),
                                          bq.ctypes.data_as(dp)))
        return s, q, b, bq

    def counters(self) -> dict:
        c = _Counters()
        lib().orc_get_counters(self.h, C.byref(c))
        return {f: int(getattr(c, f)) for f in COUNTER_FIELDS}

    def reset_counters(self):
        lib().orc_reset_counters(self.h)
