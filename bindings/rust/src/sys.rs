//! Raw FFI of include/massrt.h, MRT_ABI_VERSION 9.
//!
//! Every struct is `#[repr(C)]` with the header's field order and types;
//! tests/test_rust_binding.py parses this file and checks each struct's
//! size and field offsets against gcc's view of the header, and every
//! `extern "C"` signature against the header's prototypes.
#![allow(non_camel_case_types, dead_code)]

use std::os::raw::{c_char, c_void};

pub const MRT_ABI_VERSION: i32 = 9;

pub const MRT_OK: i32 = 0;
pub const MRT_ERR_INVALID: i32 = 1;
pub const MRT_ERR_HIP: i32 = 2;
pub const MRT_ERR_IO: i32 = 3;
pub const MRT_ERR_STATE: i32 = 4;
pub const MRT_ERR_NOMEM: i32 = 5;

// child references of the boundary BVH: kind << 28 | index (geom.rs:103-107)
pub const MRT_REF_NONE: u32 = 0;
pub const MRT_REF_NODE: u32 = 1;
pub const MRT_REF_SPHERE: u32 = 2;
pub const MRT_REF_TRIANGLE: u32 = 3;
pub const MRT_REF_INSTANCE: u32 = 4;
pub const MRT_REF_MODEL: u32 = 5;
pub const MRT_REF_VOLUME: u32 = 6;
pub const fn mrt_ref(kind: u32, index: u32) -> u32 {
    (kind << 28) | (index & 0x0FFF_FFFF)
}
pub const MRT_NO_MATERIAL: u32 = 0xFFFF_FFFF;
pub const MRT_TRI_HAS_UV: u32 = 1;

pub const MRT_MAT_NONE: u32 = 0;
pub const MRT_MAT_LAMBERTIAN: u32 = 1;
pub const MRT_MAT_METAL: u32 = 2;
pub const MRT_MAT_DIELECTRIC: u32 = 3;
pub const MRT_MAT_DIFFUSE_LIGHT: u32 = 4;
pub const MRT_MAT_SPECULAR: u32 = 5;
pub const MRT_MAT_ISOTROPHIC: u32 = 6;
pub const MRT_MAT_MIX: u32 = 7;

pub const MRT_SURF_SOLID: u32 = 0;
pub const MRT_SURF_TEXTURE: u32 = 1;
pub const MRT_SURF_YCBCR: u32 = 2;
pub const MRT_SURF_BLEND: u32 = 3;
pub const MRT_SURF_FALLBACK: u32 = 4;
pub const MRT_BLEND_LIGHTEN: u32 = 0;
pub const MRT_BLEND_DARKEN: u32 = 1;
pub const MRT_BLEND_ADDITION: u32 = 2;
pub const MRT_BLEND_SUBTRACTION: u32 = 3;

pub const MRT_WRAP_MIRROR: u32 = 0;
pub const MRT_WRAP_REPEAT: u32 = 1;
pub const MRT_WRAP_CLAMP: u32 = 2;

pub const MRT_BG_SOLID: u32 = 0;
pub const MRT_BG_SKY: u32 = 1;
pub const MRT_BG_SKYSPHERE: u32 = 2;
pub const MRT_BG_CUBEMAP: u32 = 3;

pub const MRT_TILE: u32 = 8;
pub const MRT_RENDER_COUNTERS: u32 = 1;
pub const MRT_RENDER_TIME_KERNELS: u32 = 2;
pub const MRT_RENDER_SIMPLE_TRACE: u32 = 4;
pub const MRT_RENDER_FUSED: u32 = 8;

pub const MRT_DISPLAY_DEFAULT: u32 = 0;
pub const MRT_DISPLAY_DEPTH: u32 = 1;
pub const MRT_DISPLAY_ALBEDO: u32 = 2;
pub const MRT_DISPLAY_NORMAL: u32 = 3;

// ---- flat scene description (the reference tree) -------------------------

/// BvhNode: BoundingBox + two child references (geom.rs:103-107,207-211).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_node {
    pub min: [f32; 3],
    pub max: [f32; 3],
    pub left: u32,
    pub right: u32,
}

/// Sphere (geom.rs:40-54).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_sphere {
    pub center: [f32; 3],
    pub radius: f32,
    pub material: u32,
}

/// Triangle (geom.rs:427-446).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_triangle {
    pub a: [f32; 3],
    pub b: [f32; 3],
    pub c: [f32; 3],
    pub na: [f32; 3],
    pub nb: [f32; 3],
    pub nc: [f32; 3],
    pub uva: [f32; 2],
    pub uvb: [f32; 2],
    pub uvc: [f32; 2],
    pub tangent: [f32; 3],
    pub bitangent: [f32; 3],
    pub material: u32,
    pub flags: u32,
}

/// Instance: transform / inv_transform (column-major M4) of a shared BLAS (geom.rs:335-345).
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct mrt_instance {
    pub fwd: [f32; 16],
    pub inv: [f32; 16],
    pub blas_root: u32,
    pub material: u32,
}

/// Model: owns its BLAS, optional material override (geom.rs:275-279).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_model {
    pub blas_root: u32,
    pub material: u32,
}

/// Material (material.rs:15-27 implementors), flattened.
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_material {
    pub kind: u32,
    pub surface: u32,
    pub param: f32,
    pub emit: [f32; 3],
    pub left: u32,
    pub right: u32,
}

/// Surface (texture.rs:12-17 implementors), flattened.
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_surface {
    pub kind: u32,
    pub texture: u32,
    pub color: [f32; 4],
    pub a: u32,
    pub b: u32,
    pub mode: u32,
}

/// RGBA8 texture, row 0 first (texture.rs:30-69).
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct mrt_texture {
    pub width: u32,
    pub height: u32,
    pub wrap: u32,
    pub rgba: *const u8,
}

/// Background (material.rs:29-190).
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct mrt_background {
    pub kind: u32,
    pub surface: u32,
    pub color: [f32; 3],
    pub faces: [u32; 6],
    pub transform: [f32; 16],
}

/// Volume<Sphere> with its Isotrophic material (geom.rs:594-660).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_volume {
    pub center: [f32; 3],
    pub radius: f32,
    pub density: f32,
    pub material: u32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct mrt_scene_desc {
    pub nodes: *const mrt_node,
    pub n_nodes: u32,
    pub roots: *const u32,
    pub n_roots: u32,
    pub spheres: *const mrt_sphere,
    pub n_spheres: u32,
    pub triangles: *const mrt_triangle,
    pub n_triangles: u32,
    pub instances: *const mrt_instance,
    pub n_instances: u32,
    pub models: *const mrt_model,
    pub n_models: u32,
    pub materials: *const mrt_material,
    pub n_materials: u32,
    pub surfaces: *const mrt_surface,
    pub n_surfaces: u32,
    pub textures: *const mrt_texture,
    pub n_textures: u32,
    pub background: mrt_background,
    pub volumes: *const mrt_volume,
    pub n_volumes: u32,
}

/// Camera fields precomputed by Camera::new (world.rs:5-51).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_camera {
    pub origin: [f32; 3],
    pub lower_left_corner: [f32; 3],
    pub horizontal: [f32; 3],
    pub vertical: [f32; 3],
    pub u: [f32; 3],
    pub v: [f32; 3],
    pub lens_radius: f32,
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_render_args {
    pub width: u32,
    pub height: u32,
    pub spp_begin: u32,
    pub spp_count: u32,
    pub seed: u64,
    pub max_depth: u32,
    pub shard_index: u32,
    pub shard_count: u32,
    pub flags: u32,
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_hit {
    pub prim: u32,
    pub container: u32,
    pub t: f32,
    pub front_face: u32,
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_counters {
    pub samples: u64,
    pub segments: u64,
    pub node_visits: u64,
    pub sphere_tests: u64,
    pub triangle_tests: u64,
    pub instance_entries: u64,
    pub model_entries: u64,
    pub closest_hits: u64,
    pub texel_taps: u64,
    pub bounces: u64,
    pub wave_slots: u64,
    pub lane_steps: u64,
    pub box_exact: u64,
    pub shaded: u64,
    pub vnf_fallbacks: u64,
    pub shade_waves: u64,
    pub shade_kinds: u64,
    pub shade_materials: u64,
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_kernel_stats {
    pub trace_ms: f64,
    pub shade_ms: f64,
    pub other_ms: f64,
    pub trace_launches: u64,
    pub shade_launches: u64,
    pub iterations: u64,
    pub finish_ms: f64,
    pub finish_launches: u64,
}

/// Context options (ABI v8): the gather transport of a multi-device context.
pub const MRT_GATHER_AUTO: i64 = 0;
pub const MRT_GATHER_PEER: i64 = 1;
pub const MRT_GATHER_RCCL: i64 = 2;

/// The tuning in effect after the per-scene rules (mrt_get_tuning).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct mrt_tuning {
    pub queues: u32,
    pub trace_refill: u32,
    pub trace_box_min: u32,
    pub trace_chunk: u32,
    pub shade_waves: u32,
    pub pool_paths: u64,
    pub results_max: u64,
    pub traversal: u32,
    pub shade_bin: u32,
}

/// Context option "traversal" (ABI v8).
pub const MRT_TRAVERSAL_AUTO: i64 = -1;
pub const MRT_TRAVERSAL_REFERENCE: i64 = 0;
pub const MRT_TRAVERSAL_NEAR_FIRST: i64 = 1;

/// Opaque handles.
#[repr(C)]
pub struct mrt_ctx {
    _private: [u8; 0],
}
#[repr(C)]
pub struct mrt_builder {
    _private: [u8; 0],
}
#[repr(C)]
pub struct mrt_image {
    _private: [u8; 0],
}

extern "C" {
    // ---- device context
    pub fn mrt_create(device: i32, out: *mut *mut mrt_ctx) -> i32;
    pub fn mrt_destroy(ctx: *mut mrt_ctx) -> i32;
    pub fn mrt_last_error(ctx: *const mrt_ctx) -> *const c_char;
    pub fn mrt_global_last_error() -> *const c_char;
    pub fn mrt_abi_version() -> i32;
    pub fn mrt_upload_scene(ctx: *mut mrt_ctx, scene: *const mrt_scene_desc) -> i32;
    pub fn mrt_set_camera(ctx: *mut mrt_ctx, camera: *const mrt_camera) -> i32;
    pub fn mrt_render(ctx: *mut mrt_ctx, args: *const mrt_render_args, accum_rgb: *mut f32, accum_bounces: *mut u32)
        -> i32;
    pub fn mrt_render_device(ctx: *mut mrt_ctx, args: *const mrt_render_args, d_accum_rgb: *mut f32,
                             d_accum_bounces: *mut u32, hip_stream: *mut c_void) -> i32;
    pub fn mrt_trace_rays(ctx: *mut mrt_ctx, rays: *const f32, n: u32, t_min: f32, t_max: f32, out: *mut mrt_hit)
        -> i32;
    pub fn mrt_get_counters(ctx: *mut mrt_ctx, out: *mut mrt_counters) -> i32;
    pub fn mrt_reset_counters(ctx: *mut mrt_ctx) -> i32;
    pub fn mrt_get_kernel_stats(ctx: *mut mrt_ctx, out: *mut mrt_kernel_stats) -> i32;
    pub fn mrt_selftest_division(ctx: *mut mrt_ctx, n: u64, seed: u64, mismatches: *mut u64) -> i32;
    pub fn mrt_selftest_slab(ctx: *mut mrt_ctx, n: u64, seed: u64, mismatches: *mut u64, near_ties: *mut u64) -> i32;
    pub fn mrt_debug_status(ctx: *mut mrt_ctx, out4: *mut u32) -> i32;
    pub fn mrt_debug_build() -> i32;
    pub fn mrt_reset_kernel_stats(ctx: *mut mrt_ctx) -> i32;
    pub fn mrt_scene_device_bytes(ctx: *mut mrt_ctx, out: *mut u64) -> i32;
    pub fn mrt_set_option(ctx: *mut mrt_ctx, name: *const c_char, value: i64) -> i32;
    pub fn mrt_get_option(ctx: *mut mrt_ctx, name: *const c_char, value: *mut i64) -> i32;
    pub fn mrt_get_tuning(ctx: *mut mrt_ctx, out: *mut mrt_tuning) -> i32;

    // ---- multi-GPU tile exchange (Image::merge, main.rs:629-638)
    pub fn mrt_shard_pixels(width: u32, height: u32, shard_index: u32, shard_count: u32, pixels: *mut u32,
                            count: *mut u32) -> i32;
    pub fn mrt_shard_pack_device(ctx: *mut mrt_ctx, width: u32, height: u32, shard_index: u32, shard_count: u32,
                                 d_accum_rgb: *const f32, d_accum_bounces: *const u32, d_slab: *mut c_void,
                                 hip_stream: *mut c_void) -> i32;
    pub fn mrt_shard_unpack_device(ctx: *mut mrt_ctx, width: u32, height: u32, shard_index: u32, shard_count: u32,
                                   d_slab: *const c_void, d_accum_rgb: *mut f32, d_accum_bounces: *mut u32,
                                   hip_stream: *mut c_void) -> i32;

    // ---- one context over several devices (ABI v7)
    pub fn mrt_create_multi(n_devices: i32, devices: *const i32, out: *mut *mut mrt_ctx) -> i32;
    pub fn mrt_context_devices(ctx: *mut mrt_ctx, n_devices: *mut i32, devices: *mut i32) -> i32;
    pub fn mrt_context_transport(ctx: *const mrt_ctx) -> *const c_char;
    pub fn mrt_debug_rccl_library(name: *const c_char) -> i32;
    pub fn mrt_debug_transport(n_devices: i32, devices: *const i32, buf: *mut c_char, len: u32) -> i32;

    // ---- device-resident Image (main.rs:598-638, ABI v7)
    pub fn mrt_image_create(ctx: *mut mrt_ctx, width: u32, height: u32, out: *mut *mut mrt_image) -> i32;
    pub fn mrt_image_destroy(img: *mut mrt_image) -> i32;
    pub fn mrt_image_clear(img: *mut mrt_image) -> i32;
    pub fn mrt_image_render(img: *mut mrt_image, seed: u64, spp_begin: u32, passes: u32, max_depth: u32, flags: u32)
        -> i32;
    pub fn mrt_image_prepass(img: *mut mrt_image, seed: u64) -> i32;
    pub fn mrt_image_read(img: *mut mrt_image, rgb: *mut f32, bounces: *mut u32, passes: *mut u32) -> i32;
    pub fn mrt_image_gather(img: *mut mrt_image) -> i32;
    pub fn mrt_image_tonemap(img: *mut mrt_image, mode: u32, rgb8: *mut u8) -> i32;
    pub fn mrt_image_gather_stats(img: *mut mrt_image, bytes: *mut u64, ms: *mut f64) -> i32;
    pub fn mrt_image_device_stats(img: *mut mrt_image, n_devices: i32, render_ms: *mut f64) -> i32;

    // ---- build identity (ABI v7)
    pub fn mrt_build_info() -> *const c_char;

    // ---- host scene builder (C++ mirror of the reference trait surface)
    pub fn mrt_builder_new(rng_seed: u64, out: *mut *mut mrt_builder) -> i32;
    pub fn mrt_builder_free(b: *mut mrt_builder) -> i32;
    pub fn mrt_builder_last_error() -> *const c_char;
    pub fn mrt_builder_builtin(b: *mut mrt_builder, name: *const c_char, aspect_ratio: f32, asset_dir: *const c_char)
        -> i32;
    pub fn mrt_builder_rand_f32(b: *mut mrt_builder) -> f32;
    pub fn mrt_builder_solid(b: *mut mrt_builder, r: f32, g: f32, bl: f32, a: f32) -> i32;
    pub fn mrt_builder_texture_png(b: *mut mrt_builder, path: *const c_char, wrap: u32) -> i32;
    pub fn mrt_builder_texture_rgba(b: *mut mrt_builder, rgba: *const u8, w: u32, h: u32, wrap: u32) -> i32;
    pub fn mrt_builder_material(b: *mut mrt_builder, kind: u32, surface: u32, param: f32, er: f32, eg: f32, eb: f32)
        -> i32;
    pub fn mrt_builder_add_volume(b: *mut mrt_builder, center: *const f32, radius: f32, density: f32,
                                  albedo: *const f32) -> i32;
    pub fn mrt_builder_mix(b: *mut mrt_builder, ratio: f32, left: u32, right: u32) -> i32;
    pub fn mrt_builder_background(b: *mut mrt_builder, kind: u32, surface: u32, r: f32, g: f32, bl: f32) -> i32;
    pub fn mrt_builder_background_cubemap(b: *mut mrt_builder, faces: *const u32, rotation: *const f32) -> i32;
    pub fn mrt_builder_ycbcr(b: *mut mrt_builder, luma: u32, chroma: u32) -> i32;
    pub fn mrt_builder_blend(b: *mut mrt_builder, mode: u32, left: u32, right: u32) -> i32;
    pub fn mrt_builder_fallback(b: *mut mrt_builder, r: f32, g: f32, bl: f32, a: f32, surface: u32) -> i32;
    pub fn mrt_builder_add_sphere(b: *mut mrt_builder, material: u32, cx: f32, cy: f32, cz: f32, radius: f32) -> i32;
    pub fn mrt_builder_add_triangle(b: *mut mrt_builder, material: u32, abc: *const f32) -> i32;
    pub fn mrt_builder_model(b: *mut mrt_builder, tri_material: u32, override_material: u32, tris: *const f32,
                             n: u32, with_shading: i32, add_to_world: i32) -> i32;
    pub fn mrt_builder_model_from_ply(b: *mut mrt_builder, path: *const c_char, tri_material: u32,
                                      override_material: u32, add_to_world: i32) -> i32;
    pub fn mrt_builder_add_instance(b: *mut mrt_builder, model: i32, translation: *const f32, rotation: *const f32,
                                    scale: *const f32, material: u32) -> i32;
    pub fn mrt_builder_camera(b: *mut mrt_builder, vfov: f32, look_from: *const f32, look_at: *const f32,
                              view_up: *const f32, aspect: f32, aperture: f32, focus_distance: f32) -> i32;
    pub fn mrt_builder_build_bvh(b: *mut mrt_builder) -> i32;
    pub fn mrt_builder_build_bvh_device(b: *mut mrt_builder, ctx: *mut mrt_ctx) -> i32;
    pub fn mrt_builder_builtin_device(b: *mut mrt_builder, name: *const c_char, aspect_ratio: f32,
                                      asset_dir: *const c_char, ctx: *mut mrt_ctx) -> i32;
    pub fn mrt_builder_last_build_ms(b: *mut mrt_builder, host_ms: *mut f64, device_ms: *mut f64) -> i32;
    pub fn mrt_builder_desc(b: *mut mrt_builder, desc: *mut mrt_scene_desc, camera: *mut mrt_camera) -> i32;

    // ---- display / export (main.rs:640-722, 760-783)
    pub fn mrt_tonemap_device(ctx: *mut mrt_ctx, width: u32, height: u32, d_accum_rgb: *const f32,
                              d_accum_bounces: *const u32, passes: u32, mode: u32, d_rgb8: *mut u8,
                              hip_stream: *mut c_void) -> i32;
    pub fn mrt_tonemap(ctx: *mut mrt_ctx, width: u32, height: u32, accum_rgb: *const f32, accum_bounces: *const u32,
                       passes: u32, mode: u32, rgb8: *mut u8) -> i32;
    pub fn mrt_prepass_device(ctx: *mut mrt_ctx, width: u32, height: u32, seed: u64, d_albedo: *mut f32,
                              d_normal: *mut f32, hip_stream: *mut c_void) -> i32;
    pub fn mrt_prepass(ctx: *mut mrt_ctx, width: u32, height: u32, seed: u64, albedo: *mut f32, normal: *mut f32)
        -> i32;
    pub fn mrt_display_gamma_thresholds(out256: *mut u32) -> i32;
    pub fn mrt_write_png(path: *const c_char, width: u32, height: u32, rgb8: *const u8) -> i32;

    // ---- loaders (ply_loader.rs, obj_loader.rs, stl_loader.rs)
    pub fn mrt_load_ply(path: *const c_char, out: *mut f32, cap: u64) -> i64;
    pub fn mrt_load_stl(path: *const c_char, out: *mut f32, cap: u64) -> i64;
    pub fn mrt_load_obj(path: *const c_char, out: *mut f32, cap: u64) -> i64;
}
