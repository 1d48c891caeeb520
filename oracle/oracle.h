// oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's
// path-tracing hot path (nickmass/mass-raytrace, Rust) used as the parity
// checker and the CPU baseline. Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load it; the product (libmassrt.so) never
// links or calls it.
//
// Parity status: the reference has no tests, golden vectors or fixtures other
// than cube.ply, and it cannot be built here (Rust toolchain
// and 215 crates absent). This restatement is therefore pinned only by
// cube.ply, hand-derived known answers (analytic sphere/triangle hits, BVH
// node counts, furnace scenes) and the fastrand algorithm as published:
// PARITY UNPINNED against the reference binary itself.
//
// Structure follows the reference on purpose (and unlike the product):
// heap-allocated objects behind virtual `intersect`, recursive left-first
// BvhNode traversal, recursive Camera::trace with post-order radiance fold.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

typedef struct {
  uint64_t samples, segments, node_visits, sphere_tests, triangle_tests, instance_entries, model_entries,
      closest_hits, texel_taps, bounces, alpha_taps;
} orc_counters;

typedef struct {
  uint32_t prim, container;
  float t;
  uint32_t front_face;
} orc_hit;

const char* orc_last_error(void);

// scene construction ---------------------------------------------------------
orc_scene* orc_new(uint64_t rng_seed);
void orc_free(orc_scene* s);
int orc_builtin(orc_scene* s, const char* name, float aspect, const char* asset_dir);
float orc_rand_f32(orc_scene* s);
int orc_solid(orc_scene* s, float r, float g, float b, float a);
int orc_texture_rgba(orc_scene* s, const uint8_t* rgba, uint32_t w, uint32_t h, uint32_t wrap);
int orc_texture_png(orc_scene* s, const char* path, uint32_t wrap);
int orc_material(orc_scene* s, uint32_t kind, uint32_t surface, float param, float er, float eg, float eb);
// Mix::new(ratio, left, right) (material.rs:391-426); kinds 5 Specular
// (param = refraction index, surface) and 6 Isotrophic (albedo = er,eg,eb) go
// through orc_material.
int orc_mix(orc_scene* s, float ratio, uint32_t left, uint32_t right);
int orc_background(orc_scene* s, uint32_t kind, uint32_t surface, float r, float g, float b);
// texture.rs:207-357 composite surfaces; each returns the new surface index
int orc_ycbcr(orc_scene* s, uint32_t luma, uint32_t chroma);
int orc_blend(orc_scene* s, uint32_t mode, uint32_t left, uint32_t right);
int orc_fallback(orc_scene* s, float r, float g, float b, float a, uint32_t surface);
// material.rs:91-190 CubeMap(x_pos, x_neg, y_pos, y_neg, z_pos, z_neg, rotation)
int orc_background_cubemap(orc_scene* s, const uint32_t* faces, const float* rotation);
int orc_add_sphere(orc_scene* s, uint32_t material, float cx, float cy, float cz, float radius);
// geom.rs:595-653 Volume over a Sphere target with an Isotrophic(albedo) material
int orc_add_volume(orc_scene* s, float cx, float cy, float cz, float radius, float density, float ar, float ag,
                   float ab);
int orc_add_triangle(orc_scene* s, uint32_t material, const float* abc);
int orc_model(orc_scene* s, uint32_t tri_material, uint32_t override_material, const float* tris, uint32_t n,
              int with_shading, int add_to_world);
int orc_model_from_ply(orc_scene* s, const char* path, uint32_t tri_material, uint32_t override_material,
                       int add_to_world);
int orc_add_instance(orc_scene* s, int model, const float* t, const float* r, const float* sc, uint32_t material);
int orc_camera(orc_scene* s, float vfov, const float* from, const float* at, const float* up, float aspect,
               float aperture, float focus);
int orc_build_bvh(orc_scene* s);
// camera fields: origin, llc, horizontal, vertical, u, v (18 floats) + lens radius
int orc_camera_fields(orc_scene* s, float* out19);

// preorder listing of the world tree: per element {kind, index} (kind: 1 node,
// 2 sphere, 3 triangle, 4 instance, 5 model, 6 end-of-node) and for nodes the
// 6 box floats. Returns element count (call with NULL to size).
int64_t orc_export_preorder(orc_scene* s, uint32_t* kinds_ids, float* boxes, uint64_t cap);
// same for the BLAS of model `m` (index in creation order of models/instances' BLAS)
int64_t orc_blas_count(orc_scene* s);
int64_t orc_export_blas(orc_scene* s, int64_t blas, uint32_t* kinds_ids, float* boxes, uint64_t cap);

// hot path ---------------------------------------------------------------------
int orc_trace_rays(orc_scene* s, const float* rays, uint32_t n, float tmin, float tmax, orc_hit* out);
// Deterministic render: samples [spp_begin, spp_begin+spp_count) of every pixel
// of the shard added in sample order (same contract as mrt_render).
int orc_render(orc_scene* s, uint32_t W, uint32_t H, uint32_t spp_begin, uint32_t spp_count, uint64_t seed,
               uint32_t max_depth, uint32_t shard_index, uint32_t shard_count, int threads, float* accum_rgb,
               uint32_t* accum_bounces);
// Same, for an explicit list of pixel indices (p = y*W + x); out_rgb n*3, out_b n (added to).
int orc_render_pixels(orc_scene* s, uint32_t W, uint32_t H, const uint32_t* pixels, uint32_t n, uint32_t spp_begin,
                      uint32_t spp_count, uint64_t seed, uint32_t max_depth, int threads, float* out_rgb,
                      uint32_t* out_b);
// Reference-mode CPU baseline (main.rs:159-290): `threads` workers, each
// rendering whole 1-spp frames into a private buffer merged under a mutex,
// for `passes_per_thread` passes. Only rows row_begin, row_begin + row_step,
// ... < row_end are rendered (a stratified sample of the frame for timing).
// Returns wall seconds (< 0 on error).
double orc_bench_reference_mode(orc_scene* s, uint32_t W, uint32_t H, uint32_t passes_per_thread, uint64_t seed,
                                uint32_t max_depth, int threads, float* accum_rgb, uint32_t* accum_bounces,
                                uint32_t row_begin, uint32_t row_end, uint32_t row_step);
// The reference's RNG semantics (statistical check): each
// of `workers` render threads owns ONE fastrand wyrand stream (the reference
// seeds it from the clock and thread id, main.rs:245-250 + fastrand; here
// splitmix64(seed ^ worker << 32)) and renders `passes` whole 1-spp passes in
// the reference's loop order (main.rs:253-264), every draw — jitter u, v,
// Camera::ray's disk, scatter, Volume / alpha draws — taken from that one
// stream in call order (math.rs:244-246). Adds per-pixel sums and sums of
// squares of the radiance (W*H*3 doubles each) and of the bounce counts (W*H).
int orc_render_refrng(orc_scene* s, uint32_t W, uint32_t H, uint32_t passes, uint64_t seed, uint32_t max_depth,
                      uint32_t workers, int threads, double* sum, double* sumsq, double* bsum, double* bsumsq);
void orc_wyrand(uint64_t seed, uint32_t n, uint64_t* out_u64, float* out_f32);
void orc_path_rng(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, uint64_t* out_u64, float* out_f32);
// Image::to_rgb_bytes (main.rs:640-722) + dump's row flip (main.rs:760-767):
// accumulated colour sums and bounce counts of `passes` merged passes ->
// RGB8, top row first. mode 0 Default (gamma 1/2.2), 1 Depth, 2 Albedo and
// 3 Normal (accum_rgb = the pre-pass buffer; passes ignored).
int orc_tonemap(uint32_t W, uint32_t H, const float* accum_rgb, const uint32_t* accum_bounces, uint32_t passes,
                uint32_t mode, uint8_t* out_rgb8);
// Camera::albedo_normal pre-pass (world.rs:81-92, main.rs:181-222): one ray per
// pixel through (x/(W-1), y/(H-1)); albedo/normal W*H*3 (row y = pixel row y).
// Per-pixel RNG: the path stream keyed (seed, pixel, 0xFFFFFFFF).
int orc_prepass(orc_scene* s, uint32_t W, uint32_t H, uint64_t seed, int threads, float* albedo, float* normal);
// Exhaustive check of the byte a Default-mode component takes, over every
// f32 in [0, 1] (bit patterns 0..0x3F800000): returns the number of x whose
// byte differs from the count of thresholds <= x in `thresholds[1..255]`
// (the device's method) and writes the thresholds it derived (256 words).
uint64_t orc_tonemap_check(uint32_t* thresholds, int threads);
void orc_get_counters(orc_scene* s, orc_counters* out);
void orc_reset_counters(orc_scene* s);
void orc_set_counting(orc_scene* s, int on);

#ifdef __cplusplus
}
#endif
