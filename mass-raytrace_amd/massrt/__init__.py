"""massrt — ctypes harness over libmassrt.so (include/massrt.h).

Python is only the test/bench driver: the product is the C ABI library (C++
host scene builder + gfx950 HIP kernels). There is no CPU fallback — creating a
`Context` without a GPU raises.

Mirrors of the reference surface (file:line under /root/reference/src):
  Builder.builtin(name)     Scene::generate + World::build_bvh (scenes.rs:25-33, main.rs:107-112)
  Context.render            render() sample loop + Image::merge (main.rs:150-295, 629-638)
  Context.trace_rays        World::intersect (world.rs:131-144) on explicit rays
"""
from __future__ import annotations

import ctypes as C
import os
import weakref
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
# MASSRT_LIB=dbg selects the bounds-checked debug build (make DEBUG=1); a path
# ending in .so selects that build (experiments)
_SEL = os.environ.get("MASSRT_LIB", "")
LIB_PATH = (Path(_SEL) if _SEL.endswith(".so") else
            _HERE / ("libmassrt_dbg.so" if _SEL == "dbg" else "libmassrt.so"))
REPO = _HERE.parent.parent

# ---- constants (massrt.h) --------------------------------------------------
ABI_VERSION = 9  # MRT_ABI_VERSION this binding was written for
REF_NONE, REF_NODE, REF_SPHERE, REF_TRIANGLE, REF_INSTANCE, REF_MODEL, REF_VOLUME = range(7)
MAT_NONE, MAT_LAMBERTIAN, MAT_METAL, MAT_DIELECTRIC, MAT_DIFFUSE_LIGHT, MAT_SPECULAR, MAT_ISOTROPHIC, MAT_MIX = range(8)
WRAP_MIRROR, WRAP_REPEAT, WRAP_CLAMP = range(3)
BG_SOLID, BG_SKY, BG_SKYSPHERE, BG_CUBEMAP = range(4)
SURF_SOLID, SURF_TEXTURE, SURF_YCBCR, SURF_BLEND, SURF_FALLBACK = range(5)
BLEND_LIGHTEN, BLEND_DARKEN, BLEND_ADDITION, BLEND_SUBTRACTION = range(4)
NO_MATERIAL = 0xFFFFFFFF
RENDER_COUNTERS = 1
RENDER_TIME_KERNELS = 2
RENDER_SIMPLE_TRACE = 4  # debug: one-ray-per-thread closest hit (bisection aid)
RENDER_FUSED = 8  # one persistent k_render instead of the k_trace/k_shade loop (same results)
MAX_DEPTH = 50  # main.rs:37
ASPECT_RATIO = np.float32(16.0) / np.float32(9.0)  # main.rs:39 (f32)


def ref_kind(r: int) -> int:
    return int(r) >> 28


def ref_index(r: int) -> int:
    return int(r) & 0x0FFFFFFF


class MrtNode(C.Structure):
    _fields_ = [("min", C.c_float * 3), ("max", C.c_float * 3), ("left", C.c_uint32), ("right", C.c_uint32)]


class MrtSphere(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("radius", C.c_float), ("material", C.c_uint32)]


class MrtTriangle(C.Structure):
    _fields_ = [
        ("a", C.c_float * 3), ("b", C.c_float * 3), ("c", C.c_float * 3),
        ("na", C.c_float * 3), ("nb", C.c_float * 3), ("nc", C.c_float * 3),
        ("uva", C.c_float * 2), ("uvb", C.c_float * 2), ("uvc", C.c_float * 2),
        ("tangent", C.c_float * 3), ("bitangent", C.c_float * 3),
        ("material", C.c_uint32), ("flags", C.c_uint32),
    ]


class MrtInstance(C.Structure):
    _fields_ = [("fwd", C.c_float * 16), ("inv", C.c_float * 16), ("blas_root", C.c_uint32), ("material", C.c_uint32)]


class MrtModel(C.Structure):
    _fields_ = [("blas_root", C.c_uint32), ("material", C.c_uint32)]


class MrtMaterial(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("surface", C.c_uint32), ("param", C.c_float), ("emit", C.c_float * 3),
                ("left", C.c_uint32), ("right", C.c_uint32)]


class MrtSurface(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("texture", C.c_uint32), ("color", C.c_float * 4),
                ("a", C.c_uint32), ("b", C.c_uint32), ("mode", C.c_uint32)]


class MrtTexture(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("wrap", C.c_uint32), ("rgba", C.POINTER(C.c_uint8))]


class MrtBackground(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("surface", C.c_uint32), ("color", C.c_float * 3),
                ("faces", C.c_uint32 * 6), ("transform", C.c_float * 16)]


class MrtSceneDesc(C.Structure):
    _fields_ = [
        ("nodes", C.POINTER(MrtNode)), ("n_nodes", C.c_uint32),
        ("roots", C.POINTER(C.c_uint32)), ("n_roots", C.c_uint32),
        ("spheres", C.POINTER(MrtSphere)), ("n_spheres", C.c_uint32),
        ("triangles", C.POINTER(MrtTriangle)), ("n_triangles", C.c_uint32),
        ("instances", C.POINTER(MrtInstance)), ("n_instances", C.c_uint32),
        ("models", C.POINTER(MrtModel)), ("n_models", C.c_uint32),
        ("materials", C.POINTER(MrtMaterial)), ("n_materials", C.c_uint32),
        ("surfaces", C.POINTER(MrtSurface)), ("n_surfaces", C.c_uint32),
        ("textures", C.POINTER(MrtTexture)), ("n_textures", C.c_uint32),
        ("background", MrtBackground),
        ("volumes", C.c_void_p), ("n_volumes", C.c_uint32),
    ]


class MrtCamera(C.Structure):
    _fields_ = [
        ("origin", C.c_float * 3), ("lower_left_corner", C.c_float * 3), ("horizontal", C.c_float * 3),
        ("vertical", C.c_float * 3), ("u", C.c_float * 3), ("v", C.c_float * 3), ("lens_radius", C.c_float),
    ]

    def fields(self) -> np.ndarray:
        return np.array(list(self.origin) + list(self.lower_left_corner) + list(self.horizontal)
                        + list(self.vertical) + list(self.u) + list(self.v) + [self.lens_radius], dtype=np.float32)


class MrtRenderArgs(C.Structure):
    _fields_ = [
        ("width", C.c_uint32), ("height", C.c_uint32), ("spp_begin", C.c_uint32), ("spp_count", C.c_uint32),
        ("seed", C.c_uint64), ("max_depth", C.c_uint32), ("shard_index", C.c_uint32), ("shard_count", C.c_uint32),
        ("flags", C.c_uint32),
    ]


class MrtHit(C.Structure):
    _fields_ = [("prim", C.c_uint32), ("container", C.c_uint32), ("t", C.c_float), ("front_face", C.c_uint32)]


COUNTER_FIELDS = ["samples", "segments", "node_visits", "sphere_tests", "triangle_tests", "instance_entries",
                  "model_entries", "closest_hits", "texel_taps", "bounces"]


class MrtKernelStats(C.Structure):
    _fields_ = [("trace_ms", C.c_double), ("shade_ms", C.c_double), ("other_ms", C.c_double),
                ("trace_launches", C.c_uint64), ("shade_launches", C.c_uint64), ("iterations", C.c_uint64),
                ("finish_ms", C.c_double), ("finish_launches", C.c_uint64)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


class MrtTuning(C.Structure):
    _fields_ = [("queues", C.c_uint32), ("trace_refill", C.c_uint32), ("trace_box_min", C.c_uint32),
                ("trace_chunk", C.c_uint32), ("shade_waves", C.c_uint32), ("pool_paths", C.c_uint64),
                ("results_max", C.c_uint64), ("traversal", C.c_uint32),
                ("shade_bin", C.c_uint32)]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


GATHER_AUTO, GATHER_PEER, GATHER_RCCL = 0, 1, 2
TRAVERSAL_AUTO, TRAVERSAL_REFERENCE, TRAVERSAL_NEAR_FIRST = -1, 0, 1


def parse_options(text: str, what: str = "options") -> dict:
    """"queues=1,treelet_kb=16" -> {"queues": 1, "treelet_kb": 16}; a malformed
    item raises ValueError naming it."""
    out = {}
    for item in filter(None, (x.strip() for x in text.split(","))):
        k, eq, v = item.partition("=")
        try:
            if not eq or not k.strip():
                raise ValueError
            out[k.strip()] = int(v, 0)
        except ValueError:
            raise ValueError(f"{what}: item {item!r} is not NAME=INTEGER") from None
    return out


def env_options(env=None) -> dict:
    """MASSRT_OPTIONS ("queues=1,treelet_kb=16") parsed: the harness's way for
    tools/ scripts to A/B a knob through bench.py, which passes the result as
    Context(options=...). Neither the library nor Context reads the
    environment; options reach a context only through mrt_set_option."""
    return parse_options((os.environ if env is None else env).get("MASSRT_OPTIONS", ""), "MASSRT_OPTIONS")


# scheduling counters of the persistent k_trace (no reference counterpart)
SCHED_FIELDS = ["wave_slots", "lane_steps", "box_exact", "shaded", "vnf_fallbacks", "shade_waves", "shade_kinds",
                "shade_materials"]


class MrtCounters(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in COUNTER_FIELDS + SCHED_FIELDS]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f in COUNTER_FIELDS + SCHED_FIELDS}


# symbols the header declares (checked by the CPU test-suite)
EXPORTED_SYMBOLS = [
    "mrt_create", "mrt_destroy", "mrt_last_error", "mrt_global_last_error", "mrt_abi_version",
    "mrt_upload_scene", "mrt_set_camera", "mrt_render", "mrt_render_device", "mrt_trace_rays",
    "mrt_get_counters", "mrt_reset_counters", "mrt_scene_device_bytes", "mrt_get_kernel_stats",
    "mrt_reset_kernel_stats", "mrt_selftest_division", "mrt_selftest_slab", "mrt_debug_status", "mrt_debug_build",
    "mrt_builder_new", "mrt_builder_free", "mrt_builder_builtin", "mrt_builder_rand_f32", "mrt_builder_solid",
    "mrt_builder_texture_png", "mrt_builder_texture_rgba", "mrt_builder_material", "mrt_builder_mix", "mrt_builder_add_volume",
    "mrt_builder_background_cubemap", "mrt_builder_ycbcr", "mrt_builder_blend", "mrt_builder_fallback",
    "mrt_builder_background",
    "mrt_builder_add_sphere", "mrt_builder_add_triangle", "mrt_builder_model", "mrt_builder_model_from_ply",
    "mrt_builder_add_instance", "mrt_builder_camera", "mrt_builder_build_bvh", "mrt_builder_desc",
    "mrt_builder_build_bvh_device", "mrt_builder_builtin_device", "mrt_builder_last_build_ms",
    "mrt_builder_last_error", "mrt_load_ply", "mrt_load_stl", "mrt_load_obj",
    "mrt_tonemap_device", "mrt_tonemap", "mrt_write_png", "mrt_display_gamma_thresholds",
    "mrt_prepass_device", "mrt_prepass",
    "mrt_shard_pixels", "mrt_shard_pack_device", "mrt_shard_unpack_device",
    "mrt_create_multi", "mrt_context_devices", "mrt_image_create", "mrt_image_destroy", "mrt_image_clear",
    "mrt_image_render", "mrt_image_prepass", "mrt_image_read", "mrt_image_tonemap", "mrt_image_gather_stats",
    "mrt_build_info", "mrt_set_option", "mrt_get_option", "mrt_get_tuning", "mrt_context_transport", "mrt_image_gather",
    "mrt_debug_rccl_library", "mrt_debug_transport", "mrt_image_device_stats",
]

_lib = None


def lib() -> C.CDLL:
    """Load libmassrt.so (built by __graft_entry__.build() / make)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(str(LIB_PATH))
    P, U32, U64, F, I, I64 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_float, C.c_int, C.c_int64
    fp = C.POINTER(C.c_float)
    sig = {
        "mrt_create": (I, [I, C.POINTER(P)]),
        "mrt_destroy": (I, [P]),
        "mrt_last_error": (C.c_char_p, [P]),
        "mrt_global_last_error": (C.c_char_p, []),
        "mrt_builder_last_error": (C.c_char_p, []),
        "mrt_abi_version": (I, []),
        "mrt_upload_scene": (I, [P, C.POINTER(MrtSceneDesc)]),
        "mrt_set_camera": (I, [P, C.POINTER(MrtCamera)]),
        "mrt_render": (I, [P, C.POINTER(MrtRenderArgs), fp, C.POINTER(C.c_uint32)]),
        "mrt_render_device": (I, [P, C.POINTER(MrtRenderArgs), P, P, P]),
        "mrt_trace_rays": (I, [P, fp, U32, F, F, C.POINTER(MrtHit)]),
        "mrt_get_counters": (I, [P, C.POINTER(MrtCounters)]),
        "mrt_reset_counters": (I, [P]),
        "mrt_get_kernel_stats": (I, [P, C.POINTER(MrtKernelStats)]),
        "mrt_reset_kernel_stats": (I, [P]),
        "mrt_selftest_division": (I, [P, U64, U64, C.POINTER(C.c_uint64)]),
        "mrt_selftest_slab": (I, [P, U64, U64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "mrt_debug_status": (I, [P, C.POINTER(C.c_uint32)]),
        "mrt_debug_build": (I, []),
        "mrt_scene_device_bytes": (I, [P, C.POINTER(C.c_uint64)]),
        "mrt_builder_new": (I, [U64, C.POINTER(P)]),
        "mrt_builder_free": (I, [P]),
        "mrt_builder_builtin": (I, [P, C.c_char_p, F, C.c_char_p]),
        "mrt_builder_rand_f32": (F, [P]),
        "mrt_builder_solid": (I, [P, F, F, F, F]),
        "mrt_builder_texture_png": (I, [P, C.c_char_p, U32]),
        "mrt_builder_texture_rgba": (I, [P, C.POINTER(C.c_uint8), U32, U32, U32]),
        "mrt_builder_material": (I, [P, U32, U32, F, F, F, F]),
        "mrt_builder_background": (I, [P, U32, U32, F, F, F]),
        "mrt_builder_mix": (I, [P, F, U32, U32]),
        "mrt_builder_add_volume": (I, [P, fp, F, F, fp]),
        "mrt_builder_background_cubemap": (I, [P, C.POINTER(C.c_uint32), fp]),
        "mrt_builder_ycbcr": (I, [P, U32, U32]),
        "mrt_builder_blend": (I, [P, U32, U32, U32]),
        "mrt_builder_fallback": (I, [P, F, F, F, F, U32]),
        "mrt_builder_add_sphere": (I, [P, U32, F, F, F, F]),
        "mrt_builder_add_triangle": (I, [P, U32, fp]),
        "mrt_builder_model": (I, [P, U32, U32, fp, U32, I, I]),
        "mrt_builder_model_from_ply": (I, [P, C.c_char_p, U32, U32, I]),
        "mrt_builder_add_instance": (I, [P, I, fp, fp, fp, U32]),
        "mrt_builder_camera": (I, [P, F, fp, fp, fp, F, F, F]),
        "mrt_builder_build_bvh": (I, [P]),
        "mrt_builder_build_bvh_device": (I, [P, P]),
        "mrt_builder_builtin_device": (I, [P, C.c_char_p, F, C.c_char_p, P]),
        "mrt_builder_last_build_ms": (I, [P, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
        "mrt_builder_desc": (I, [P, C.POINTER(MrtSceneDesc), C.POINTER(MrtCamera)]),
        "mrt_load_ply": (I64, [C.c_char_p, fp, U64]),
        "mrt_load_stl": (I64, [C.c_char_p, fp, U64]),
        "mrt_load_obj": (I64, [C.c_char_p, fp, U64]),
        "mrt_tonemap_device": (I, [P, U32, U32, P, P, U32, U32, P, P]),
        "mrt_tonemap": (I, [P, U32, U32, fp, C.POINTER(C.c_uint32), U32, U32, C.POINTER(C.c_uint8)]),
        "mrt_write_png": (I, [C.c_char_p, U32, U32, C.POINTER(C.c_uint8)]),
        "mrt_display_gamma_thresholds": (I, [C.POINTER(C.c_uint32)]),
        "mrt_prepass_device": (I, [P, U32, U32, U64, P, P, P]),
        "mrt_prepass": (I, [P, U32, U32, U64, fp, fp]),
        "mrt_shard_pixels": (I, [U32, U32, U32, U32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
        "mrt_shard_pack_device": (I, [P, U32, U32, U32, U32, P, P, P, P]),
        "mrt_shard_unpack_device": (I, [P, U32, U32, U32, U32, P, P, P, P]),
        "mrt_create_multi": (I, [I, C.POINTER(C.c_int), C.POINTER(P)]),
        "mrt_context_devices": (I, [P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "mrt_image_create": (I, [P, U32, U32, C.POINTER(P)]),
        "mrt_image_destroy": (I, [P]),
        "mrt_image_clear": (I, [P]),
        "mrt_image_render": (I, [P, U64, U32, U32, U32, U32]),
        "mrt_image_prepass": (I, [P, U64]),
        "mrt_image_read": (I, [P, fp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
        "mrt_image_tonemap": (I, [P, U32, C.POINTER(C.c_uint8)]),
        "mrt_image_gather_stats": (I, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_double)]),
        "mrt_build_info": (C.c_char_p, []),
        "mrt_set_option": (I, [P, C.c_char_p, I64]),
        "mrt_get_option": (I, [P, C.c_char_p, C.POINTER(I64)]),
        "mrt_get_tuning": (I, [P, C.POINTER(MrtTuning)]),
        "mrt_context_transport": (C.c_char_p, [P]),
        "mrt_debug_rccl_library": (C.c_int, [C.c_char_p]),
        "mrt_image_device_stats": (C.c_int, [P, C.c_int, C.POINTER(C.c_double)]),
        "mrt_debug_transport": (C.c_int, [C.c_int, C.POINTER(C.c_int), C.c_char_p, C.c_uint32]),
        "mrt_image_gather": (I, [P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


class MassrtError(RuntimeError):
    pass


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _f3(v) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(v, dtype=np.float32).reshape(3))


def _check_builder(rc: int) -> int:
    if rc < 0:
        raise MassrtError(lib().mrt_builder_last_error().decode())
    return rc


class Builder:
    """Host scene builder (C++ mirror of World/Model/Instance/...)."""

    def __init__(self, rng_seed: int = 1):
        h = C.c_void_p()
        if lib().mrt_builder_new(rng_seed, C.byref(h)) != 0:
            raise MassrtError("mrt_builder_new failed")
        self.h = h
        self._keep = []

    def close(self):
        if self.h:
            lib().mrt_builder_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def builtin(self, name: str, aspect: float = float(ASPECT_RATIO), asset_dir: str | os.PathLike = ""):
        rc = lib().mrt_builder_builtin(self.h, name.encode(), aspect, str(asset_dir).encode())
        if rc != 0:
            raise MassrtError(lib().mrt_builder_last_error().decode())
        return self

    def builtin_device(self, name: str, ctx: "Context", aspect: float = float(ASPECT_RATIO),
                       asset_dir: str | os.PathLike = ""):
        """builtin() with World::build_bvh done on ctx's GPU (same tree)."""
        rc = lib().mrt_builder_builtin_device(self.h, name.encode(), aspect, str(asset_dir).encode(), ctx.h)
        if rc != 0:
            raise MassrtError(lib().mrt_builder_last_error().decode())
        return self

    def build_bvh_device(self, ctx: "Context"):
        if lib().mrt_builder_build_bvh_device(self.h, ctx.h) != 0:
            raise MassrtError(lib().mrt_builder_last_error().decode())

    def last_build_ms(self):
        h, d = C.c_double(), C.c_double()
        lib().mrt_builder_last_build_ms(self.h, C.byref(h), C.byref(d))
        return h.value, d.value

    def rand_f32(self) -> float:
        return lib().mrt_builder_rand_f32(self.h)

    def solid(self, r, g, b, a=1.0) -> int:
        return _check_builder(lib().mrt_builder_solid(self.h, r, g, b, a))

    def texture_rgba(self, rgba: np.ndarray, wrap: int = WRAP_REPEAT) -> int:
        rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
        h, w = rgba.shape[:2]
        return _check_builder(lib().mrt_builder_texture_rgba(self.h, rgba.ctypes.data_as(C.POINTER(C.c_uint8)), w, h, wrap))

    def texture_png(self, path, wrap: int = WRAP_REPEAT) -> int:
        return _check_builder(lib().mrt_builder_texture_png(self.h, str(path).encode(), wrap))

    def material(self, kind, surface=0, param=0.0, emit=(0.0, 0.0, 0.0)) -> int:
        return _check_builder(lib().mrt_builder_material(self.h, kind, surface, param, *emit))

    def mix(self, ratio, left, right) -> int:
        """Mix::new(ratio, left, right) (material.rs:391-426)."""
        return _check_builder(lib().mrt_builder_mix(self.h, ratio, left, right))

    def background(self, kind, surface=0, color=(0.0, 0.0, 0.0)):
        _check_builder(lib().mrt_builder_background(self.h, kind, surface, *color))

    def background_cubemap(self, faces, rotation=(0.0, 0.0, 0.0)):
        """CubeMap::new(x_pos, x_neg, y_pos, y_neg, z_pos, z_neg, rotation) (material.rs:91-190)."""
        f = np.ascontiguousarray(faces, dtype=np.uint32).reshape(6)
        _check_builder(lib().mrt_builder_background_cubemap(self.h, f.ctypes.data_as(C.POINTER(C.c_uint32)),
                                                            _fptr(_f3(rotation))))

    def ycbcr(self, luma, chroma) -> int:
        """YCbCrTexture over two texture surfaces (texture.rs:207-250)."""
        return _check_builder(lib().mrt_builder_ycbcr(self.h, luma, chroma))

    def blend(self, mode, left, right) -> int:
        """TextureBlend::new(mode, left, right) (texture.rs:303-334)."""
        return _check_builder(lib().mrt_builder_blend(self.h, mode, left, right))

    def fallback(self, color, surface) -> int:
        """SolidColorFallback::new(color, surface) (texture.rs:336-357)."""
        return _check_builder(lib().mrt_builder_fallback(self.h, *[float(c) for c in color], surface))

    def add_sphere(self, material, center, radius):
        _check_builder(lib().mrt_builder_add_sphere(self.h, material, *[float(c) for c in center], radius))

    def add_volume(self, center, radius, density, albedo) -> int:
        """World::add(Volume::new(Sphere(center, radius), density, albedo)) (geom.rs:595-653)."""
        return _check_builder(lib().mrt_builder_add_volume(self.h, _fptr(_f3(center)), float(radius), float(density),
                                                           _fptr(_f3(albedo))))

    def add_triangle(self, material, abc):
        a = np.ascontiguousarray(np.asarray(abc, dtype=np.float32).reshape(9))
        _check_builder(lib().mrt_builder_add_triangle(self.h, material, _fptr(a)))

    def model(self, tri_material, tris: np.ndarray, override=NO_MATERIAL, add_to_world=False, shading=False) -> int:
        t = np.ascontiguousarray(tris, dtype=np.float32)
        n = t.shape[0]
        return _check_builder(lib().mrt_builder_model(self.h, tri_material, override, _fptr(t), n, int(shading),
                                                      int(add_to_world)))

    def model_from_ply(self, path, tri_material, override=NO_MATERIAL, add_to_world=False) -> int:
        return _check_builder(lib().mrt_builder_model_from_ply(self.h, str(path).encode(), tri_material, override,
                                                               int(add_to_world)))

    def add_instance(self, model, translation, rotation, scale, material=NO_MATERIAL):
        t, r, s = _f3(translation), _f3(rotation), _f3(scale)
        _check_builder(lib().mrt_builder_add_instance(self.h, model, _fptr(t), _fptr(r), _fptr(s), material))

    def camera(self, vfov, look_from, look_at, view_up=(0, 1, 0), aspect=float(ASPECT_RATIO), aperture=0.0,
               focus=None):
        f, a, u = _f3(look_from), _f3(look_at), _f3(view_up)
        if focus is None:
            d = (f - a).astype(np.float32)
            focus = float(np.sqrt(np.float32(d[0] * d[0] + d[1] * d[1]) + np.float32(d[2] * d[2])))
        _check_builder(lib().mrt_builder_camera(self.h, vfov, _fptr(f), _fptr(a), _fptr(u), aspect, aperture, focus))

    def build_bvh(self):
        if lib().mrt_builder_build_bvh(self.h) != 0:
            raise MassrtError(lib().mrt_builder_last_error().decode())

    def desc(self):
        d, cam = MrtSceneDesc(), MrtCamera()
        if lib().mrt_builder_desc(self.h, C.byref(d), C.byref(cam)) != 0:
            raise MassrtError(lib().mrt_builder_last_error().decode())
        return d, cam

    def desc_only(self) -> MrtSceneDesc:
        d = MrtSceneDesc()
        if lib().mrt_builder_desc(self.h, C.byref(d), None) != 0:
            raise MassrtError(lib().mrt_builder_last_error().decode())
        return d


def preorder(desc: MrtSceneDesc):
    """Preorder listing of the world tree in the oracle's format:
    list of (kind, id) with kind 6 = end of node, plus boxes of nodes."""
    out, boxes = [], []

    def walk(ref):
        stack = [("ref", ref)]
        while stack:
            tag, r = stack.pop()
            if tag == "end":
                out.append((6, 0))
                boxes.append(None)
                continue
            k, i = ref_kind(r), ref_index(r)
            if k == REF_NODE:
                n = desc.nodes[i]
                out.append((REF_NODE, 0))
                boxes.append(tuple(n.min) + tuple(n.max))
                stack.append(("end", 0))
                if ref_kind(n.right) != REF_NONE:
                    stack.append(("ref", n.right))
                stack.append(("ref", n.left))
            else:
                out.append((k, i))
                boxes.append(None)

    for r in range(desc.n_roots):
        walk(desc.roots[r])
    return out, boxes


def debug_transport(devices, rccl_library: str | None = None) -> str:
    """The gather transport mrt_create_multi would pick for `devices`
    (mrt_debug_transport; opens RCCL from `rccl_library`, default
    librccl.so.1, creates no communicators: no GPU needed)."""
    L = lib()
    L.mrt_debug_rccl_library((rccl_library or "").encode())
    try:
        ids = (C.c_int * len(devices))(*devices)
        buf = C.create_string_buffer(512)
        rc = L.mrt_debug_transport(len(devices), ids, buf, 512)
        if rc != 0:
            raise MassrtError(f"mrt_debug_transport failed ({rc}): {L.mrt_global_last_error().decode()}")
        return buf.value.decode()
    finally:
        L.mrt_debug_rccl_library(b"")


def build_info() -> str:
    """"src <hash>": the source hash the loaded library was built from (tools/src_hash.py)."""
    return lib().mrt_build_info().decode()


class Context:
    """One GPU context (mrt_ctx), or one over several devices (devices=[...],
    mrt_create_multi). Raises if no HIP device is present."""

    def __init__(self, device: int = 0, devices=None, options=None):
        h = C.c_void_p()
        if devices is not None:
            ids = (C.c_int * len(devices))(*devices)
            rc = lib().mrt_create_multi(len(devices), ids, C.byref(h))
            what = "mrt_create_multi"
        else:
            rc = lib().mrt_create(device, C.byref(h))
            what = "mrt_create"
        if rc != 0:
            raise MassrtError(f"{what} failed ({rc}): {lib().mrt_global_last_error().decode()}")
        self.h = h
        self._images = weakref.WeakSet()  # closed before the context (massrt.h: images first)
        for k, v in (options or {}).items():
            self.set_option(k, v)

    def set_option(self, name: str, value: int):
        """mrt_set_option (massrt.h lists the names); -1 = the per-scene rule where allowed."""
        self._check(lib().mrt_set_option(self.h, name.encode(), int(value)))

    def get_option(self, name: str) -> int:
        v = C.c_int64()
        self._check(lib().mrt_get_option(self.h, name.encode(), C.byref(v)))
        return int(v.value)

    def tuning(self) -> dict:
        """The loop's tuning in effect (after the per-scene rules of the last upload)."""
        t = MrtTuning()
        self._check(lib().mrt_get_tuning(self.h, C.byref(t)))
        return t.as_dict()

    def transport(self) -> str:
        """Gather transport of a multi-device context: "rccl", "peer", "peer (...)" or "none"."""
        return lib().mrt_context_transport(self.h).decode()

    def devices(self) -> list:
        n = C.c_int()
        self._check(lib().mrt_context_devices(self.h, C.byref(n), None))
        ids = (C.c_int * n.value)()
        self._check(lib().mrt_context_devices(self.h, C.byref(n), ids))
        return list(ids)

    def _check(self, rc):
        if rc != 0:
            raise MassrtError(lib().mrt_last_error(self.h).decode())

    def close(self):
        if self.h:
            for img in list(self._images):  # an image must not outlive its context
                img.close()
            rc = lib().mrt_destroy(self.h)
            if rc != 0:
                raise MassrtError(lib().mrt_global_last_error().decode())
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, builder: Builder):
        d, cam = builder.desc()
        self._check(lib().mrt_upload_scene(self.h, C.byref(d)))
        self._check(lib().mrt_set_camera(self.h, C.byref(cam)))

    def upload_desc(self, desc: MrtSceneDesc):
        self._check(lib().mrt_upload_scene(self.h, C.byref(desc)))

    def set_camera(self, cam: MrtCamera):
        self._check(lib().mrt_set_camera(self.h, C.byref(cam)))

    def scene_bytes(self) -> int:
        v = C.c_uint64()
        self._check(lib().mrt_scene_device_bytes(self.h, C.byref(v)))
        return int(v.value)

    @staticmethod
    def args(width, height, spp_begin=0, spp_count=1, seed=1, max_depth=MAX_DEPTH, shard_index=0, shard_count=1,
             counters=False, time_kernels=False, flags=0) -> MrtRenderArgs:
        flags |= (RENDER_COUNTERS if counters else 0) | (RENDER_TIME_KERNELS if time_kernels else 0)
        return MrtRenderArgs(width, height, spp_begin, spp_count, seed, max_depth, shard_index, shard_count, flags)

    def render(self, width, height, spp_begin=0, spp_count=1, seed=1, max_depth=MAX_DEPTH, shard_index=0,
               shard_count=1, counters=False, accum=None, flags=0):
        """Returns (rgb float32 [H*W*3], bounces uint32 [H*W]) accumulated in sample order."""
        if accum is None:
            rgb = np.zeros(width * height * 3, dtype=np.float32)
            b = np.zeros(width * height, dtype=np.uint32)
        else:
            rgb, b = accum
        a = self.args(width, height, spp_begin, spp_count, seed, max_depth, shard_index, shard_count, counters,
                      flags=flags)
        self._check(lib().mrt_render(self.h, C.byref(a), _fptr(rgb), b.ctypes.data_as(C.POINTER(C.c_uint32))))
        return rgb, b

    def render_device(self, args: MrtRenderArgs, d_rgb: int, d_bounces: int, stream: int | None = None):
        self._check(lib().mrt_render_device(self.h, C.byref(args), C.c_void_p(d_rgb), C.c_void_p(d_bounces),
                                            C.c_void_p(stream or 0)))

    def trace_rays(self, rays: np.ndarray, t_min=0.001, t_max=float("inf")):
        r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        n = r.shape[0]
        out = (MrtHit * max(n, 1))()
        self._check(lib().mrt_trace_rays(self.h, _fptr(r), n, t_min, t_max, out))
        a = np.frombuffer(out, dtype=np.uint32).reshape(-1, 4)[:n].copy()
        return a  # columns: prim, container, t bits, front_face

    def counters(self) -> dict:
        c = MrtCounters()
        self._check(lib().mrt_get_counters(self.h, C.byref(c)))
        return c.as_dict()

    def reset_counters(self):
        self._check(lib().mrt_reset_counters(self.h))

    def kernel_stats(self) -> dict:
        k = MrtKernelStats()
        self._check(lib().mrt_get_kernel_stats(self.h, C.byref(k)))
        return k.as_dict()

    def selftest_division(self, n: int, seed: int = 1) -> int:
        m = C.c_uint64()
        self._check(lib().mrt_selftest_division(self.h, n, seed, C.byref(m)))
        return int(m.value)

    def tonemap(self, width, height, rgb, bounces, passes, mode=0) -> np.ndarray:
        """Image::to_rgb_bytes + dump's row flip on the GPU: (H, W, 3) uint8, top row first."""
        rgb = np.ascontiguousarray(rgb, dtype=np.float32).reshape(-1)
        b = np.ascontiguousarray(bounces, dtype=np.uint32).reshape(-1)
        out = np.empty(width * height * 3, dtype=np.uint8)
        self._check(lib().mrt_tonemap(self.h, width, height, _fptr(rgb), b.ctypes.data_as(C.POINTER(C.c_uint32)),
                                      passes, mode, out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out.reshape(height, width, 3)

    def prepass(self, width, height, seed=1):
        """Camera::albedo_normal pre-pass: (albedo, normal) float32 [H*W*3] each."""
        a = np.empty(width * height * 3, dtype=np.float32)
        n = np.empty(width * height * 3, dtype=np.float32)
        self._check(lib().mrt_prepass(self.h, width, height, seed, _fptr(a), _fptr(n)))
        return a, n

    def tonemap_device(self, width, height, d_rgb: int, d_bounces: int, passes: int, mode: int, d_out: int,
                       stream: int | None = None):
        self._check(lib().mrt_tonemap_device(self.h, width, height, C.c_void_p(d_rgb), C.c_void_p(d_bounces), passes,
                                             mode, C.c_void_p(d_out), C.c_void_p(stream or 0)))

    def selftest_slab(self, n: int, seed: int = 1):
        """(mismatches, near_ties) of the early slab decision vs the exact test."""
        m, t = C.c_uint64(), C.c_uint64()
        self._check(lib().mrt_selftest_slab(self.h, n, seed, C.byref(m), C.byref(t)))
        return int(m.value), int(t.value)

    def debug_status(self):
        out = (C.c_uint32 * 4)()
        self._check(lib().mrt_debug_status(self.h, out))
        return list(out)

    def reset_kernel_stats(self):
        self._check(lib().mrt_reset_kernel_stats(self.h))

    def shard_pack_device(self, width, height, shard_index, shard_count, d_rgb: int, d_bounces: int, d_slab: int,
                          stream: int | None = None):
        """This shard's pixels of the accumulation buffers -> slab (16 B per pixel)."""
        self._check(lib().mrt_shard_pack_device(self.h, width, height, shard_index, shard_count, C.c_void_p(d_rgb),
                                                C.c_void_p(d_bounces), C.c_void_p(d_slab), C.c_void_p(stream or 0)))

    def shard_unpack_device(self, width, height, shard_index, shard_count, d_slab: int, d_rgb: int, d_bounces: int,
                            stream: int | None = None):
        """Slab -> this shard's pixels of the accumulation buffers (overwritten)."""
        self._check(lib().mrt_shard_unpack_device(self.h, width, height, shard_index, shard_count, C.c_void_p(d_slab),
                                                  C.c_void_p(d_rgb), C.c_void_p(d_bounces), C.c_void_p(stream or 0)))


def shard_pixels(width: int, height: int, shard_index: int, shard_count: int) -> np.ndarray:
    """Pixel indices (p = y*W + x) shard `shard_index` of `shard_count` owns, in slab order (host only)."""
    n = C.c_uint32()
    rc = lib().mrt_shard_pixels(width, height, shard_index, shard_count, None, C.byref(n))
    if rc != 0:
        raise MassrtError(lib().mrt_global_last_error().decode())
    out = np.empty(max(n.value, 1), dtype=np.uint32)
    rc = lib().mrt_shard_pixels(width, height, shard_index, shard_count, out.ctypes.data_as(C.POINTER(C.c_uint32)),
                                C.byref(n))
    if rc != 0:
        raise MassrtError(lib().mrt_global_last_error().decode())
    return out[: n.value]


DISPLAY_DEFAULT, DISPLAY_DEPTH, DISPLAY_ALBEDO, DISPLAY_NORMAL = 0, 1, 2, 3


def gamma_thresholds() -> np.ndarray:
    t = np.zeros(256, dtype=np.uint32)
    lib().mrt_display_gamma_thresholds(t.ctypes.data_as(C.POINTER(C.c_uint32)))
    return t


def write_png(path, rgb8: np.ndarray):
    """RGB8 (H, W, 3), top row first -> PNG (host code in libmassrt)."""
    a = np.ascontiguousarray(rgb8, dtype=np.uint8)
    h, w = a.shape[0], a.shape[1]
    if lib().mrt_write_png(str(path).encode(), w, h, a.ctypes.data_as(C.POINTER(C.c_uint8))) != 0:
        raise MassrtError(lib().mrt_builder_last_error().decode())


def load_ply(path) -> np.ndarray:
    n = lib().mrt_load_ply(str(path).encode(), None, 0)
    if n < 0:
        raise MassrtError(lib().mrt_builder_last_error().decode())
    out = np.zeros((n, 9), dtype=np.float32)
    lib().mrt_load_ply(str(path).encode(), _fptr(out), n)
    return out


def load_stl(path) -> np.ndarray:
    n = lib().mrt_load_stl(str(path).encode(), None, 0)
    if n < 0:
        raise MassrtError(lib().mrt_builder_last_error().decode())
    out = np.zeros((n, 9), dtype=np.float32)
    lib().mrt_load_stl(str(path).encode(), _fptr(out), n)
    return out


def load_obj(path) -> np.ndarray:
    n = lib().mrt_load_obj(str(path).encode(), None, 0)
    if n < 0:
        raise MassrtError(lib().mrt_builder_last_error().decode())
    out = np.zeros((n, 24), dtype=np.float32)
    lib().mrt_load_obj(str(path).encode(), _fptr(out), n)
    return out


class Image:
    """The reference's Image (main.rs:598-638) in HBM (mrt_image): colour and
    depth sums plus the pass count stay on the context's device(s); render()
    adds passes without a host round trip, read()/tonemap() cross PCIe."""

    def __init__(self, ctx: Context, width: int, height: int):
        h = C.c_void_p()
        rc = lib().mrt_image_create(ctx.h, width, height, C.byref(h))
        if rc != 0:
            raise MassrtError(lib().mrt_last_error(ctx.h).decode())
        self.h, self.ctx, self.width, self.height = h, ctx, width, height
        ctx._images.add(self)

    def _check(self, rc):
        if rc != 0:
            raise MassrtError(lib().mrt_last_error(self.ctx.h).decode())

    def close(self):
        if self.h:
            lib().mrt_image_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def clear(self):
        """Image::clear (main.rs:749-758)."""
        self._check(lib().mrt_image_clear(self.h))

    def render(self, seed: int, spp_begin: int, passes: int, max_depth: int = MAX_DEPTH, counters=False,
               time_kernels=False):
        """`passes` 1-spp passes merged: samples [spp_begin, spp_begin + passes) of every pixel."""
        flags = (RENDER_COUNTERS if counters else 0) | (RENDER_TIME_KERNELS if time_kernels else 0)
        self._check(lib().mrt_image_render(self.h, seed, spp_begin, passes, max_depth, flags))

    def prepass(self, seed: int = 1):
        """Camera::albedo_normal pre-pass into the image (main.rs:162-222)."""
        self._check(lib().mrt_image_prepass(self.h, seed))

    @property
    def passes(self) -> int:
        p = C.c_uint32()
        self._check(lib().mrt_image_read(self.h, None, None, C.byref(p)))
        return int(p.value)

    def read(self):
        """(rgb float32 [H*W*3], bounces uint32 [H*W], passes)."""
        n = self.width * self.height
        rgb = np.empty(3 * n, dtype=np.float32)
        b = np.empty(n, dtype=np.uint32)
        p = C.c_uint32()
        self._check(lib().mrt_image_read(self.h, _fptr(rgb), b.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(p)))
        return rgb, b, int(p.value)

    def gather(self):
        """Image::merge at the end of a frame: the devices' tiles onto devices[0]
        (on the device, no host copy); returns once every device's work has ended."""
        self._check(lib().mrt_image_gather(self.h))

    def tonemap(self, mode: int = 0) -> np.ndarray:
        """Image::to_rgb_bytes + dump's row flip: (H, W, 3) uint8, top row first."""
        out = np.empty(self.width * self.height * 3, dtype=np.uint8)
        self._check(lib().mrt_image_tonemap(self.h, mode, out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out.reshape(self.height, self.width, 3)

    def gather_stats(self):
        """(bytes moved between devices by this image's gathers, their wall ms)."""
        b, ms = C.c_uint64(), C.c_double()
        self._check(lib().mrt_image_gather_stats(self.h, C.byref(b), C.byref(ms)))
        return int(b.value), float(ms.value)

    def device_stats(self) -> list:
        """Per-device render ms so far (HIP events around each device's share of every render)."""
        n = len(self.ctx.devices())
        out = (C.c_double * n)()
        self._check(lib().mrt_image_device_stats(self.h, n, out))
        return [float(x) for x in out]


# ---- render(): the drop-in pass loop (mirror of bindings/rust/src/lib.rs) ---

class SampleStreams:
    """Where a frame's samples come from (lib.rs SampleStreams). The
    reference's render threads draw from thread-local fastrand streams seeded
    afresh for every render() call (main.rs:167-250), so frames never share
    samples; here sample s of pixel p is keyed (seed, p, s) and the sample
    index keeps counting across frames (the seed moves on before it wraps)."""

    def __init__(self, seed: int = 1, next_sample: int = 0):
        self.seed, self.next_sample = seed, next_sample

    def take(self, n: int):
        if self.next_sample + n > 0xFFFFFFFF:
            self.seed = (self.seed + 1) & 0xFFFFFFFFFFFFFFFF
            self.next_sample = 0
        first = self.next_sample
        self.next_sample += n
        return self.seed, first


def default_workers() -> int:
    """render()'s thread count: num_cpus - 2, at least 1 (main.rs:159-160)."""
    return max(1, (os.cpu_count() or 1) - 2)


def render(image, streams: SampleStreams, frame_limit=None, workers=None, batch=256, max_depth=MAX_DEPTH,
           prepass=True, update=None, keep_going=None) -> int:
    """render(image, event_proxy, world, camera, frame_limit) (main.rs:150-295)
    on the GPU, exactly as bindings/rust/src/lib.rs `render` does it:
    pre-pass (main.rs:162-222), Image::clear (main.rs:233), then `workers`
    render threads x `frame_limit` whole 1-spp passes each (None: until
    keep_going() is false), one merge per pass (main.rs:243-280), run `batch`
    passes per mrt_image_render call; update(image, passes) after every batch
    (UserEvent::Update, main.rs:274-278); keep_going() before every batch
    (QUICK_PASS, main.rs:224-231, 282-284). Returns the passes rendered."""
    workers = default_workers() if workers is None else max(1, int(workers))
    if prepass:
        image.prepass(streams.seed)
    image.clear()
    total = None if frame_limit is None else int(frame_limit) * workers
    batch = max(1, int(batch))
    done = 0
    while total is None or done < total:
        if keep_going is not None and not keep_going():
            break
        k = batch if total is None else min(batch, total - done)
        seed, first = streams.take(k)
        image.render(seed, first, k, max_depth)
        done += k
        if update is not None:
            update(image, image.passes)
    return done
