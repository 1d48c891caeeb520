/*
 * massrt.h — C ABI of the MI355X (gfx950) path-tracing hot path.
 *
 * Drop-in boundary for the reference's per-pixel-per-sample render loop:
 *   fn render(image, event_proxy, world: World<B>, camera: Camera, frame_limit)
 *   (/root/reference/src/main.rs:150-295)
 * Everything the reference does below that call — Camera::ray
 * (world.rs:53-63), Camera::trace (world.rs:65-79), World::intersect
 * (world.rs:131-144), BvhNode/BoundingBox/Sphere/Triangle/Instance/Model
 * intersect (geom.rs:56-425,503-593), Material scatter/emit
 * (material.rs:192-329,385-389), Background (material.rs:39-89), Surface
 * (texture.rs:117-194,277-299) and the per-pass ImageBuffer::set /
 * Image::merge accumulation (main.rs:253-265,577-596,629-638) — runs on the
 * GPU behind these entry points.
 *
 * Rules of the ABI:
 *  - every function returns an int status: MRT_OK (0) or an MRT_ERR_* code;
 *    the message is in mrt_last_error(ctx) (or mrt_global_last_error() for
 *    calls without a context). No C++ exception or panic crosses the ABI.
 *  - handles are opaque; calls on one context must be serialized by the caller.
 *  - plain C types only (pointers + sizes). Host buffers are caller-owned.
 *    Device memory for the scene is owned by the context.
 *  - a context drives one GPU (mrt_create) or several (mrt_create_multi, one
 *    process); multi-process multi-GPU = one process (rank) per GPU, each
 *    rendering its shard of framebuffer tiles (mrt_render_args.shard_*).
 *  - tuning comes from the caller (mrt_set_option), never from the process
 *    environment.
 *
 * The reference's Rust side would bind these with `extern "C"` (see
 * INTEGRATION.md); the C++ host in this repo (mass-raytrace_amd/csrc/host)
 * mirrors the reference's Scene/World/Camera/Intersect/Material surface and
 * produces mrt_scene_desc through the mrt_builder_* entry points below.
 */
#ifndef MASSRT_H
#define MASSRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MRT_ABI_VERSION 9

/* ---- status codes ------------------------------------------------------ */
#define MRT_OK 0
#define MRT_ERR_INVALID 1  /* bad argument / malformed scene */
#define MRT_ERR_HIP 2      /* HIP runtime failure (no GPU, kernel fault...) */
#define MRT_ERR_IO 3       /* loader could not read/parse a file */
#define MRT_ERR_STATE 4    /* call out of order (e.g. render before upload) */
#define MRT_ERR_NOMEM 5

/* ---- child references of the boundary BVH ------------------------------
 * A BvhNode child (geom.rs:103-107: Option<Box<dyn Intersect>>) is encoded as
 * kind<<28 | index. MRT_REF_NONE is the `None` right child of a 1-item node
 * (geom.rs:120-121). */
#define MRT_REF_KIND_SHIFT 28u
#define MRT_REF_INDEX_MASK 0x0FFFFFFFu
#define MRT_REF_NONE 0u
#define MRT_REF_NODE 1u     /* BvhNode            geom.rs:185-205 */
#define MRT_REF_SPHERE 2u   /* Sphere             geom.rs:56-101  */
#define MRT_REF_TRIANGLE 3u /* Triangle           geom.rs:503-593 */
#define MRT_REF_INSTANCE 4u /* Instance (of BLAS) geom.rs:403-425 */
#define MRT_REF_MODEL 5u    /* Model (owns BLAS)  geom.rs:317-333 */
#define MRT_REF_VOLUME 6u   /* Volume<Sphere>     geom.rs:594-660 (world level only) */
#define MRT_REF(kind, idx) ((((uint32_t)(kind)) << MRT_REF_KIND_SHIFT) | ((uint32_t)(idx)&MRT_REF_INDEX_MASK))
#define MRT_REF_KIND(r) (((uint32_t)(r)) >> MRT_REF_KIND_SHIFT)
#define MRT_REF_INDEX(r) (((uint32_t)(r)) & MRT_REF_INDEX_MASK)
#define MRT_NO_MATERIAL 0xFFFFFFFFu

/* ---- flat scene description (the reference tree, not our GPU layout) --- */
typedef struct {
  float min[3], max[3]; /* BoundingBox   geom.rs:207-211 */
  uint32_t left, right; /* MRT_REF(...)  geom.rs:104-105 */
} mrt_node;

typedef struct {
  float center[3];
  float radius; /* negative radius flips normals (geom.rs:78) */
  uint32_t material;
} mrt_sphere;

#define MRT_TRI_HAS_UV 1u /* Triangle::uvs is Some (with_norms_and_uvs) */
typedef struct {
  float a[3], b[3], c[3];                  /* vertex_a/b/c     geom.rs:436-438 */
  float na[3], nb[3], nc[3];               /* normal_a/b/c     geom.rs:441-443 */
  float uva[2], uvb[2], uvc[2];            /* UV               geom.rs:428-432 */
  float tangent[3], bitangent[3];          /* geom.rs:444-445 */
  uint32_t material;                       /* per-triangle material */
  uint32_t flags;                          /* MRT_TRI_HAS_UV */
} mrt_triangle;

typedef struct {
  float fwd[16];      /* column-major M4 (generic.rs:71-77): transform     */
  float inv[16];      /*                                   inv_transform   */
  uint32_t blas_root; /* MRT_REF_NODE index of the shared Arc<BvhNode>      */
  uint32_t material;  /* override (with_material) or MRT_NO_MATERIAL        */
} mrt_instance;

typedef struct {
  uint32_t blas_root; /* MRT_REF_NODE index */
  uint32_t material;  /* Model::with_material override or MRT_NO_MATERIAL */
} mrt_model;

#define MRT_MAT_NONE 0u          /* impl Material for ()  material.rs:385-389 */
#define MRT_MAT_LAMBERTIAN 1u    /* material.rs:192-225 */
#define MRT_MAT_METAL 2u         /* material.rs:248-284 (param = fuzz, clamped) */
#define MRT_MAT_DIELECTRIC 3u    /* material.rs:286-329 (param = refraction index) */
#define MRT_MAT_DIFFUSE_LIGHT 4u /* material.rs:227-246 (emit) */
#define MRT_MAT_SPECULAR 5u      /* material.rs:331-378 (param = refraction index; surface of the inner Lambertian) */
#define MRT_MAT_ISOTROPHIC 6u    /* material.rs:428-445 (emit[] holds the albedo) */
#define MRT_MAT_MIX 7u           /* material.rs:391-426 (param = ratio; left, right = material indices < own) */
typedef struct {
  uint32_t kind;
  uint32_t surface; /* index into surfaces (Lambertian/Metal/Specular) */
  float param;
  float emit[3];
  uint32_t left, right; /* Mix only */
} mrt_material;

#define MRT_SURF_SOLID 0u    /* SolidColor         texture.rs:179-194 */
#define MRT_SURF_TEXTURE 1u  /* Texture            texture.rs:117-149 */
#define MRT_SURF_YCBCR 2u    /* YCbCrTexture       texture.rs:207-250: texture = luma, a = chroma texture */
#define MRT_SURF_BLEND 3u    /* TextureBlend       texture.rs:303-334: mode, a = left, b = right surface */
#define MRT_SURF_FALLBACK 4u /* SolidColorFallback texture.rs:336-357: color, a = surface */
/* BlendMode (texture.rs:252-267) */
#define MRT_BLEND_LIGHTEN 0u
#define MRT_BLEND_DARKEN 1u
#define MRT_BLEND_ADDITION 2u
#define MRT_BLEND_SUBTRACTION 3u
/* Composite surfaces (BLEND, FALLBACK) reference surfaces with lower
 * indices, so the table is acyclic; evaluating one may hold at most 4
 * operands at once (e.g. Blend(Texture, YCbCr) holds 3). */
typedef struct {
  uint32_t kind;
  uint32_t texture;
  float color[4];
  uint32_t a, b, mode;
} mrt_surface;

#define MRT_WRAP_MIRROR 0u /* unimplemented in the reference (texture.rs:280-282) */
#define MRT_WRAP_REPEAT 1u
#define MRT_WRAP_CLAMP 2u
typedef struct {
  uint32_t width, height, wrap;
  const uint8_t* rgba; /* width*height*4 bytes, row 0 first (texture.rs:113) */
} mrt_texture;

#define MRT_BG_SOLID 0u     /* SolidBackground material.rs:39-53 */
#define MRT_BG_SKY 1u       /* SkyBackground   material.rs:55-63 */
#define MRT_BG_SKYSPHERE 2u /* SkySphere       material.rs:65-89 */
#define MRT_BG_CUBEMAP 3u   /* CubeMap         material.rs:91-190 */
typedef struct {
  uint32_t kind;
  uint32_t surface;
  float color[3];
  /* CubeMap: x_pos, x_neg, y_pos, y_neg, z_pos, z_neg surfaces and the
   * direction transform (column-major 4x4, CubeMap::new material.rs:102-118) */
  uint32_t faces[6];
  float transform[16];
} mrt_background;

/* Volume::new(Sphere::new((), center, radius), density, albedo): a constant-
 * density medium in a sphere (the reference's only Volume target, eve.rs:41);
 * `material` is its Isotrophic(albedo) (material.rs:428-445). Its
 * intersection draws from the path RNG (geom.rs:640). */
typedef struct {
  float center[3];
  float radius;
  float density;
  uint32_t material;
} mrt_volume;

typedef struct {
  const mrt_node* nodes;
  uint32_t n_nodes;
  const uint32_t* roots; /* World::objects in order (world.rs:97,131-144) */
  uint32_t n_roots;
  const mrt_sphere* spheres;
  uint32_t n_spheres;
  const mrt_triangle* triangles;
  uint32_t n_triangles;
  const mrt_instance* instances;
  uint32_t n_instances;
  const mrt_model* models;
  uint32_t n_models;
  const mrt_material* materials;
  uint32_t n_materials;
  const mrt_surface* surfaces;
  uint32_t n_surfaces;
  const mrt_texture* textures;
  uint32_t n_textures;
  mrt_background background;
  const mrt_volume* volumes;
  uint32_t n_volumes;
} mrt_scene_desc;

/* Camera fields precomputed by Camera::new (world.rs:5-51). */
typedef struct {
  float origin[3];
  float lower_left_corner[3];
  float horizontal[3];
  float vertical[3];
  float u[3];
  float v[3];
  float lens_radius;
} mrt_camera;

/* One render call = samples [spp_begin, spp_begin+spp_count) of every pixel
 * in this shard, ADDED in sample order into the accumulation buffers:
 *   accum_rgb[3*p+c] += color_c, accum_bounces[p] += MAX_DEPTH-depth
 * with p = y*width + x and y = 0 the BOTTOM row (main.rs:258-263,592-595,
 * 629-638). Per-(pixel,sample) RNG: xoroshiro128** seeded by splitmix64 of
 * (seed, p, sample) — results do not depend on the shard split. */
#define MRT_TILE 8u /* framebuffer tiles are MRT_TILE x MRT_TILE pixels */
typedef struct {
  uint32_t width, height;
  uint32_t spp_begin, spp_count;
  uint64_t seed;
  uint32_t max_depth;   /* MAX_DEPTH = 50 in the reference (main.rs:37) */
  uint32_t shard_index; /* tiles t with t % shard_count == shard_index */
  uint32_t shard_count; /* 0 or 1 = whole frame */
  uint32_t flags;       /* MRT_RENDER_* */
} mrt_render_args;
#define MRT_RENDER_COUNTERS 1u     /* collect traversal counters (slower) */
#define MRT_RENDER_TIME_KERNELS 2u /* time every k_trace/k_shade launch with HIP events */
#define MRT_RENDER_SIMPLE_TRACE 4u /* debug: one-ray-per-thread closest hit instead of the persistent k_trace */
#define MRT_RENDER_FUSED 8u        /* one persistent k_render (trace + shade per lane) instead of the
                                      k_trace/k_shade wavefront loop; same results, slower at 108 VGPRs */

/* Closest hit of one ray (parity entry point). */
typedef struct {
  uint32_t prim;      /* MRT_REF(kind, index) of the primitive hit, or NONE */
  uint32_t container; /* MRT_REF(INSTANCE|MODEL, index) or NONE */
  float t;
  uint32_t front_face;
} mrt_hit;

/* Algorithmic work counters (SURVEY §8d bytes model). */
typedef struct {
  uint64_t samples;
  uint64_t segments;        /* World::intersect calls */
  uint64_t node_visits;     /* BoundingBox::hit calls */
  uint64_t sphere_tests;
  uint64_t triangle_tests;
  uint64_t instance_entries;
  uint64_t model_entries;
  uint64_t closest_hits;
  uint64_t texel_taps;      /* bilinear taps: shading and alpha tests */
  uint64_t bounces;
  /* scheduling efficiency of the persistent k_trace (not reference quantities):
   * wave_slots = loop iterations x 64 lanes, lane_steps = box/primitive steps
   * executed; lane_steps / wave_slots = SIMD lane utilisation */
  uint64_t wave_slots;
  uint64_t lane_steps;
  /* box tests the early slab decision left to the exact slab test (ABI v6) */
  uint64_t box_exact;
  /* paths k_shade advanced (one per traced segment shaded by the wavefront
     loop; the drain hand-off's fused launches shade the rest; ABI v7) */
  uint64_t shaded;
  /* near-first walks whose hit the reference's walk would not reach: walked
     again the reference's way (ABI v8) */
  uint64_t vnf_fallbacks;
  /* shading coherence of the counting k_shade (ABI v9): waves with work, and
     summed over them the distinct material kinds (a miss: one more) and the
     distinct material indices among their lanes */
  uint64_t shade_waves;
  uint64_t shade_kinds;
  uint64_t shade_materials;
} mrt_counters;

/* Kernel timing accumulated by renders flagged MRT_RENDER_TIME_KERNELS
 * (HIP events on the stream the kernels run on). */
typedef struct {
  double trace_ms, shade_ms, other_ms;
  uint64_t trace_launches, shade_launches, iterations;
  /* the drain hand-off: fused k_render launches that finished a queue's last
   * paths (trace + shade of every remaining bounce; ABI v6) */
  double finish_ms;
  uint64_t finish_launches;
} mrt_kernel_stats;

typedef struct mrt_ctx mrt_ctx;

/* ---- device context ---------------------------------------------------- */
int mrt_create(int device, mrt_ctx** out);
int mrt_destroy(mrt_ctx* ctx);
const char* mrt_last_error(const mrt_ctx* ctx);
const char* mrt_global_last_error(void);
int mrt_abi_version(void);

int mrt_upload_scene(mrt_ctx* ctx, const mrt_scene_desc* scene);
int mrt_set_camera(mrt_ctx* ctx, const mrt_camera* camera);
/* host buffers: accum_rgb = width*height*3 floats, accum_bounces = width*height */
int mrt_render(mrt_ctx* ctx, const mrt_render_args* args, float* accum_rgb, uint32_t* accum_bounces);
/* device buffers, enqueued on `hip_stream` (hipStream_t; NULL = the null stream, ordered
 * with the caller's default-stream work) */
int mrt_render_device(mrt_ctx* ctx, const mrt_render_args* args, float* d_accum_rgb,
                      uint32_t* d_accum_bounces, void* hip_stream);
/* rays: n x {ox,oy,oz,dx,dy,dz} host floats; out: n hits. Draws during the
 * traversal (Volume, Mix alpha tests) use ray i's stream keyed
 * (seed 0, i, sample 0xFFFFFFFE). */
int mrt_trace_rays(mrt_ctx* ctx, const float* rays, uint32_t n, float t_min, float t_max, mrt_hit* out);
int mrt_get_counters(mrt_ctx* ctx, mrt_counters* out);
int mrt_reset_counters(mrt_ctx* ctx);
int mrt_get_kernel_stats(mrt_ctx* ctx, mrt_kernel_stats* out);
/* Self-test of the device's correctly rounded division (box slab test):
 * n random/structured operand pairs vs IEEE a/b; mismatches must be 0. */
int mrt_selftest_division(mrt_ctx* ctx, uint64_t n, uint64_t seed, uint64_t* mismatches);
/* Self-test of the slab test's early decision (approximate quotients with an
 * error margin, exact fallback near ties) against the exact slab test on n
 * random rays/boxes built to graze each other; mismatches must be 0,
 * near_ties counts the cases the exact fallback decided. */
int mrt_selftest_slab(mrt_ctx* ctx, uint64_t n, uint64_t seed, uint64_t* mismatches, uint64_t* near_ties);
/* Debug builds (-DMRT_DEBUG_BOUNDS, libmassrt_dbg.so) check every scene and
 * path-buffer index on the device and record the first failure here as
 * {check code, index, bound, failure count} instead of faulting.
 * mrt_debug_build() reports whether the loaded library is such a build. */
int mrt_debug_status(mrt_ctx* ctx, uint32_t* out4);
int mrt_debug_build(void);
int mrt_reset_kernel_stats(mrt_ctx* ctx);
/* bytes of device memory held for the scene */
int mrt_scene_device_bytes(mrt_ctx* ctx, uint64_t* out);

/* ---- context options (ABI v8) -------------------------------------------
 * Tuning of the wavefront loop, per context (on a multi-device context: every
 * device). Values are integers; -1 where allowed = the per-scene rule chosen
 * at upload. Unknown names and out-of-range values: MRT_ERR_INVALID.
 *   queues            1..4   path pools on their own streams (default 2)
 *   pool_paths        live paths at most (default 384Mi; capped by free memory)
 *   results_log2      10..31 samples per results slab at most (default 31)
 *   finish_paths      drain hand-off threshold, 0 = never (default 500000)
 *   finish_grid_div   1..64  (default 1)
 *   trace_refill      -1, 1..64  k_trace refill threshold (-1: 32)
 *   trace_box_min     -1, 1..65  k_trace box-run threshold (-1: per scene)
 *   trace_chunk       -1, >= 64  rays per work grab (-1: per scene)
 *   trace_prim_batch  1..64  (default 1)
 *   trace_prim_run    -1, 1..65  near-first k_trace primitive run threshold
 *                     (-1: 32; 65: off)
 *   trace_wgs_per_cu  0..32  persistent-grid workgroups per CU (0: occupancy)
 *   shade_waves       -1, 7, 8  k_shade register budget (-1: per scene)
 *   shade_batch       1..64  fused kernel's shade batch (default 16)
 *   treelet_kb        0..150 LDS treelet per workgroup (default 0; next upload)
 *   trace_block       256, 512, 1024  k_trace workgroup beside a treelet
 *   mem_reserve_mb    device memory a render leaves free (default 4096)
 *   gather            MRT_GATHER_* (multi-device contexts)
 *   traversal         MRT_TRAVERSAL_* (default AUTO: per scene); NEAR_FIRST
 *                     applies to scenes without traversal draws (Volume, Mix
 *                     alpha) and without a treelet, others keep REFERENCE.
 *                     The near-first trees are built at upload for the value
 *                     then in effect (REFERENCE: none; AUTO: where it would
 *                     walk near first): set NEAR_FIRST before uploading
 *   nf_kappa_log2     -40..-8  NEAR_FIRST: rays whose generic-triangle kappa
 *                     (nf_bound.h) exceeds 2^v take the reference walk (-8)
 *   trace_nf_batch    -1, 1..64  NEAR_FIRST: finished walks checked together
 *                     once this many lanes wait (-1: the refill threshold)
 *   shade_bin      -1, 0, 1, 2  k_shade writes each workgroup's surviving
 *                     paths into the next pool grouped by the material kind
 *                     they scattered from and the signs of their direction's
 *                     y and x, so k_trace's waves walk rays that go the same
 *                     way together (1); 2 also splits the whole pool by the
 *                     y sign (up-going paths from the bottom, down-going from
 *                     the top, new camera rays between); -1: 2 under the
 *                     near-first walk, 1 under the reference walk (round 5:
 *                     sphere_grid 974 / 1030 / 1068 Msamples/s at 0 / 1 / 2,
 *                     mesh_ply 1149 / 1151 / 1134); images are identical
 *                     whichever is set
 * Every render sizes its path pool and results slab to the device memory
 * free at that moment minus mem_reserve_mb (several contexts may share a
 * device), shrinking the pool first and then the samples per chunk. */
/* How k_trace finds each closest hit (geom.rs:185-205 BvhNode::intersect):
 * REFERENCE walks the reference's tree left child first (the reference's own
 * sequence of box and primitive tests: bit-exact by construction). NEAR_FIRST
 * walks surface-area-heuristic trees over the same primitives, nearer child
 * first, then checks that the reference's walk reaches the hit it found (its
 * innermost reference ancestors pass BoundingBox::hit) and walks the
 * reference's way where it does not. Its boxes are thickened by a proven
 * bound on how far a primitive's computed hit can lie outside its box (the
 * reference's own f32 Moller-Trumbore and sphere roots, instance transforms;
 * DESIGN.md §4), so it meets every hit that can win and its closest hit is
 * the reference's, t bits and ties included; rays the bound does not cover
 * take the reference's walk. AUTO (the default) picks NEAR_FIRST unless the
 * world is a big instanced one (Menger), where REFERENCE is faster. Round 6
 * (1080p x 1024 spp per step): sphere_grid 1152 vs 968, cube_field 563 vs
 * 422, mesh_ply 1228 vs 1152 Msamples/s (normal cones bound the generic
 * triangles' term per node; wild instances pass their own box test, nf_bound.h
 * NfWild); Menger 26 vs 50 (hence AUTO). Counters (node visits, ...) count
 * the walk taken. */
#define MRT_TRAVERSAL_AUTO (-1)
#define MRT_TRAVERSAL_REFERENCE 0
#define MRT_TRAVERSAL_NEAR_FIRST 1
#define MRT_GATHER_AUTO 0 /* RCCL between distinct devices, peer copies otherwise */
#define MRT_GATHER_PEER 1 /* HIP peer copies */
#define MRT_GATHER_RCCL 2 /* RCCL send/recv (distinct devices only) */
int mrt_set_option(mrt_ctx* ctx, const char* name, int64_t value);
int mrt_get_option(mrt_ctx* ctx, const char* name, int64_t* value);
/* the values in effect after the per-scene rules (devices[0] of a multi-device context) */
typedef struct {
  uint32_t queues, trace_refill, trace_box_min, trace_chunk, shade_waves;
  uint64_t pool_paths, results_max;
  uint32_t traversal; /* the walk k_trace uses for this scene (MRT_TRAVERSAL_*) */
  uint32_t shade_bin; /* 0, 1, 2: the survivor grouping in effect (option shade_bin; ABI v9) */
} mrt_tuning;
int mrt_get_tuning(mrt_ctx* ctx, mrt_tuning* out);

/* ---- multi-GPU tile exchange (Image::merge, main.rs:629-638) ------------
 * A render sharded over N devices (mrt_render_args.shard_index/count) leaves
 * each device's accumulation buffers holding its own tiles only. A shard's
 * SLAB packs exactly those pixels, in the order the shard owns them (tiles
 * t = shard_index, shard_index + shard_count, ... in raster order of 8x8
 * tiles, pixels of a tile in raster order), 16 B per pixel:
 * {r, g, b, bounces as u32 bits}. Gathering every shard's slab to one
 * device (RCCL send/recv or a peer copy) and unpacking them there yields the
 * 1-device image bit for bit: every pixel is summed on one device only.
 * mrt_shard_pixels is host-only (no device); pixels may be NULL to count. */
int mrt_shard_pixels(uint32_t width, uint32_t height, uint32_t shard_index, uint32_t shard_count,
                     uint32_t* pixels, uint32_t* count);
/* d_slab: count*4 words (device), enqueued on `hip_stream` */
int mrt_shard_pack_device(mrt_ctx* ctx, uint32_t width, uint32_t height, uint32_t shard_index, uint32_t shard_count,
                          const float* d_accum_rgb, const uint32_t* d_accum_bounces, void* d_slab, void* hip_stream);
/* overwrites the shard's pixels of the accumulation buffers with the slab */
int mrt_shard_unpack_device(mrt_ctx* ctx, uint32_t width, uint32_t height, uint32_t shard_index,
                            uint32_t shard_count, const void* d_slab, float* d_accum_rgb, uint32_t* d_accum_bounces,
                            void* hip_stream);

/* ---- one context over several devices (ABI v7) --------------
 * render() (main.rs:150-295) spreads its samples over worker threads that all
 * merge into ONE Image (main.rs:629-638). The device counterpart: one context
 * spans n devices (repeats allowed, e.g. {0,0,0} rehearses the exchange on one
 * GPU). Every device holds the scene; a render splits the frame's 8x8 tiles
 * over the devices — device i renders shard (shard_index*n + i) of
 * (shard_count*n), one host thread per device — and the devices' slabs are
 * gathered onto devices[0] (RCCL send/recv over xGMI when the devices are
 * distinct, HIP peer copies otherwise; option "gather" overrides). With
 * distinct devices mrt_create_multi opens RCCL and creates its communicators
 * at once; if that fails the context falls back to peer copies and
 * mrt_context_transport says why. Every pixel is summed on one device only,
 * so the image equals the one-device render bit for bit. mrt_render with
 * host buffers uploads the caller's whole buffers to devices[0] and only
 * their own shard's pixels to the others, and copies the whole frame back:
 * pixels outside this call's shards come back as the caller had them.
 * On such a context mrt_upload_scene, mrt_set_camera and mrt_render (host
 * buffers) use every device; mrt_get/reset_counters and mrt_get/reset_
 * kernel_stats sum over them; every other entry point runs on devices[0]
 * (device pointers then live on devices[0]). */
int mrt_create_multi(int n_devices, const int* devices, mrt_ctx** out);
/* devices the context spans (1 for mrt_create) and their ordinals (may be NULL) */
int mrt_context_devices(mrt_ctx* ctx, int* n_devices, int* devices);
/* the gather transport: "none" (one device), "peer", "rccl", or
 * "peer (...)" with the reason RCCL was not used */
const char* mrt_context_transport(const mrt_ctx* ctx);
/* TEST-ONLY hooks of the transport choice (no GPU needed): the library RCCL
 * is opened from (NULL or "": librccl.so.1) by contexts created after the
 * call (a live context keeps the RCCL it was created with), and the transport
 * mrt_create_multi would pick for these devices — opening RCCL but creating
 * no communicators — written to buf (e.g. "peer (RCCL unavailable: ...)"). */
int mrt_debug_rccl_library(const char* name);
int mrt_debug_transport(int n_devices, const int* devices, char* buf, uint32_t len);

/* ---- device-resident Image (main.rs:598-638, ABI v7) --------------------
 * The reference's Image {pass count, per-pixel (colour sum, depth sum),
 * albedo, normal} kept in HBM: renders add to it on the device(s) without a
 * host round trip, and only a read or a tonemap crosses PCIe — the call
 * pattern of a render() whose passes are batched. On a
 * multi-device context every device keeps the sums of its own tiles and a
 * read gathers them. Calls on one image are serialized by the caller.
 * An image must be destroyed before its context: mrt_destroy returns
 * MRT_ERR_STATE (and destroys nothing) while images of the context exist. */
typedef struct mrt_image mrt_image;
int mrt_image_create(mrt_ctx* ctx, uint32_t width, uint32_t height, mrt_image** out);
int mrt_image_destroy(mrt_image* img);
/* Image::clear (main.rs:749-758): sums, depths and the pass count to 0 */
int mrt_image_clear(mrt_image* img);
/* `passes` 1-spp passes merged (Image::merge x passes, main.rs:253-273):
 * sample s in [spp_begin, spp_begin + passes) of every pixel, keyed (seed,
 * pixel, s) as in mrt_render; the pass count grows by `passes`. flags:
 * MRT_RENDER_COUNTERS / MRT_RENDER_TIME_KERNELS. Enqueued: returns once the
 * work is queued on every device (a read or tonemap waits for it). */
int mrt_image_render(mrt_image* img, uint64_t seed, uint32_t spp_begin, uint32_t passes, uint32_t max_depth,
                     uint32_t flags);
/* Camera::albedo_normal pre-pass into the image (main.rs:162-222; as mrt_prepass) */
int mrt_image_prepass(mrt_image* img, uint64_t seed);
/* sums (W*H*3 f32) and depths (W*H u32) — either may be NULL — and the pass
 * count; with both NULL only the count is returned (no gather, no sync) */
int mrt_image_read(mrt_image* img, float* rgb, uint32_t* bounces, uint32_t* passes);
/* Image::merge of the devices' tiles at the end of a frame: gathers them onto
 * devices[0] (device-resident, no host copy) and waits until every device's
 * queued work has ended */
int mrt_image_gather(mrt_image* img);
/* Image::to_rgb_bytes + dump's row flip (as mrt_tonemap) on devices[0]: W*H*3
 * bytes, top row first. ALBEDO / NORMAL show the pre-pass (zeros before one). */
int mrt_image_tonemap(mrt_image* img, uint32_t mode, uint8_t* rgb8);
/* bytes that crossed between devices in the image's gathers, and their time */
int mrt_image_gather_stats(mrt_image* img, uint64_t* bytes, double* ms);
/* per-device render time so far (ms, HIP events around each device's share
 * of every mrt_image_render; waits for renders still running); render_ms has
 * one entry per device of the context */
int mrt_image_device_stats(mrt_image* img, int n_devices, double* render_ms);

/* ---- build identity (ABI v7) -------------------------------------------
 * hash of the sources the library was built from (csrc/ + include/, as
 * tools/src_hash.py computes it), so a run can prove it loaded HEAD's code */
const char* mrt_build_info(void);

/* ---- host scene builder (C++ mirror of the reference trait surface) -----
 * A builder owns a World under construction plus the scene RNG (fastrand
 * wyrand restatement, seeded like main.rs:86). Model construction and
 * build_bvh draw from it exactly where the reference does (geom.rs:111).
 * Calls returning an index return >= 0 on success and -MRT_ERR_* on error;
 * status calls return MRT_OK or a positive MRT_ERR_*. Message:
 * mrt_builder_last_error() (thread-local). */
typedef struct mrt_builder mrt_builder;
int mrt_builder_new(uint64_t rng_seed, mrt_builder** out);
int mrt_builder_free(mrt_builder* b);
const char* mrt_builder_last_error(void);
/* Scene::generate of a built-in scene, then World::build_bvh (main.rs:107-112).
 * names: "sphere_grid", "cornell", "cube_field", "mesh_ply", "mesh_obj",
 *        "mesh_obj_textured", "menger", "menger_l3"; asset_dir holds cube.ply
 *        and generated assets. */
int mrt_builder_builtin(mrt_builder* b, const char* name, float aspect_ratio, const char* asset_dir);
float mrt_builder_rand_f32(mrt_builder* b); /* f32::rand() on the scene stream */
/* surfaces / materials; each returns an index >= 0 */
int mrt_builder_solid(mrt_builder* b, float r, float g, float bl, float a);
int mrt_builder_texture_png(mrt_builder* b, const char* path, uint32_t wrap);
int mrt_builder_texture_rgba(mrt_builder* b, const uint8_t* rgba, uint32_t w, uint32_t h, uint32_t wrap);
int mrt_builder_material(mrt_builder* b, uint32_t kind, uint32_t surface, float param, float er, float eg, float eb);
/* World::add(Volume::new(Sphere::new((), center, radius), density, albedo));
 * returns the volume index */
int mrt_builder_add_volume(mrt_builder* b, const float* center, float radius, float density, const float* albedo);
/* Mix::new(ratio, left, right): returns the material index */
int mrt_builder_mix(mrt_builder* b, float ratio, uint32_t left, uint32_t right);
int mrt_builder_background(mrt_builder* b, uint32_t kind, uint32_t surface, float r, float g, float bl);
/* CubeMap::new(x_pos, x_neg, y_pos, y_neg, z_pos, z_neg, rotation) — faces are surface indices */
int mrt_builder_background_cubemap(mrt_builder* b, const uint32_t* faces /*6*/, const float* rotation /*3*/);
/* YCbCrTexture::load_png(luma, chroma, _): two texture surfaces -> a new surface index */
int mrt_builder_ycbcr(mrt_builder* b, uint32_t luma, uint32_t chroma);
/* TextureBlend::new(mode, left, right) -> a new surface index */
int mrt_builder_blend(mrt_builder* b, uint32_t mode, uint32_t left, uint32_t right);
/* SolidColorFallback::new(color, surface) -> a new surface index */
int mrt_builder_fallback(mrt_builder* b, float r, float g, float bl, float a, uint32_t surface);
/* world objects (World::add, world.rs:112-115) */
int mrt_builder_add_sphere(mrt_builder* b, uint32_t material, float cx, float cy, float cz, float radius);
int mrt_builder_add_triangle(mrt_builder* b, uint32_t material, const float* abc /*9*/);
/* Model::new / with_material over a triangle list (geom.rs:280-310); draws
 * the BLAS BVH immediately. tris: n x 9 floats (Triangle::new) or, when
 * shading != NULL, n x 24 floats {v,n,uv} x3 (Triangle::with_norms_and_uvs).
 * Returns model handle index. add_to_world: also World::add(model). */
int mrt_builder_model(mrt_builder* b, uint32_t tri_material, uint32_t override_material, const float* tris,
                      uint32_t n, int with_shading, int add_to_world);
int mrt_builder_model_from_ply(mrt_builder* b, const char* path, uint32_t tri_material,
                               uint32_t override_material, int add_to_world);
int mrt_builder_add_instance(mrt_builder* b, int model, const float* translation, const float* rotation,
                             const float* scale, uint32_t material);
int mrt_builder_camera(mrt_builder* b, float vfov, const float* look_from, const float* look_at,
                       const float* view_up, float aspect, float aperture, float focus_distance);
int mrt_builder_build_bvh(mrt_builder* b); /* World::build_bvh (world.rs:117-122) */
/* World::build_bvh with the top-level tree built on ctx's device
 * (csrc/device/build.hip): the same nodes, node numbering
 * and scene-stream draws as mrt_builder_build_bvh (BvhNode::new,
 * geom.rs:110-161). MRT_ERR_INVALID for a NaN sort key in a node of >= 3 items;
 * a failed build leaves the world and the scene stream unchanged. */
int mrt_builder_build_bvh_device(mrt_builder* b, mrt_ctx* ctx);
/* mrt_builder_builtin with the scene's World::build_bvh done on ctx's device */
int mrt_builder_builtin_device(mrt_builder* b, const char* name, float aspect_ratio, const char* asset_dir,
                               mrt_ctx* ctx);
/* wall milliseconds of the builder's last device tree build: host part
 * (node ranges + axis draws + assembly) and device part (upload, sorts,
 * boxes, download) */
int mrt_builder_last_build_ms(mrt_builder* b, double* host_ms, double* device_ms);
/* flatten; pointers stay valid until the builder is freed or modified */
int mrt_builder_desc(mrt_builder* b, mrt_scene_desc* desc, mrt_camera* camera);

/* ---- display / export (main.rs:640-722, 760-783) ----------------------- */
/* Image::to_rgb_bytes + dump's row flip: accumulated colour sums (W*H*3
 * f32) and bounce counts (W*H u32) of `passes` merged 1-spp passes -> RGB8
 * (W*H*3), TOP row first, exactly the bytes dump() hands to the PNG encoder.
 * Default: ((sum/passes)^(1/2.2)).min(1).max(0) * 255 as u8 (the gamma byte
 * is taken from 255 thresholds derived from the host libm powf, so it is the
 * reference's byte for every input); Depth: (count/passes)/(max/passes).
 * passes == 0 gives zeros. _device: device pointers on `hip_stream`. */
#define MRT_DISPLAY_DEFAULT 0u
#define MRT_DISPLAY_DEPTH 1u
#define MRT_DISPLAY_ALBEDO 2u /* accum_rgb = the pre-pass albedo; p.min(1).max(0).powf(1/2.2) (passes ignored) */
#define MRT_DISPLAY_NORMAL 3u /* accum_rgb = the pre-pass normal; (p + 1) / 2 (passes ignored) */
int mrt_tonemap_device(mrt_ctx* ctx, uint32_t width, uint32_t height, const float* d_accum_rgb,
                       const uint32_t* d_accum_bounces, uint32_t passes, uint32_t mode, uint8_t* d_rgb8,
                       void* hip_stream);
int mrt_tonemap(mrt_ctx* ctx, uint32_t width, uint32_t height, const float* accum_rgb, const uint32_t* accum_bounces,
                uint32_t passes, uint32_t mode, uint8_t* rgb8);
/* Camera::albedo_normal pre-pass (world.rs:81-92, main.rs:181-222): one ray
 * per pixel through (x/(W-1), y/(H-1)), no jitter; albedo = the scatter
 * attenuation (emission if the material absorbs, background on a miss),
 * normal = the hit's face-oriented world normal (0 on a miss). W*H*3 f32
 * each, row y = pixel row y (FloatBuffer, main.rs:544-575). The reference
 * draws this pass from thread-local RNG; here pixel p uses the path stream
 * keyed (seed, p, sample 0xFFFFFFFF). _device: device pointers on `hip_stream`. */
int mrt_prepass_device(mrt_ctx* ctx, uint32_t width, uint32_t height, uint64_t seed, float* d_albedo, float* d_normal,
                       void* hip_stream);
int mrt_prepass(mrt_ctx* ctx, uint32_t width, uint32_t height, uint64_t seed, float* albedo, float* normal);
/* The 256 Default-mode thresholds (t[k] = f32 bits of the smallest x in
 * [0, 1] whose byte is >= k), derived from the host libm powf. */
int mrt_display_gamma_thresholds(uint32_t* out256);
/* RGB8 (top row first) -> PNG file (8-bit truecolour, zlib). 0 or MRT_ERR_IO. */
int mrt_write_png(const char* path, uint32_t width, uint32_t height, const uint8_t* rgb8);

/* ---- loaders (host; ply_loader.rs, obj_loader.rs, stl_loader.rs) -------- */
/* returns triangle count (or -MRT_ERR_IO); out (if non-NULL, capacity cap triangles) gets 9 floats per tri */
int64_t mrt_load_ply(const char* path, float* out, uint64_t cap);
int64_t mrt_load_stl(const char* path, float* out, uint64_t cap);
/* OBJ with v/vt/vn: 24 floats per tri {v(3),n(3),uv(2)} x3, uv as read (obj_fns) */
int64_t mrt_load_obj(const char* path, float* out, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* MASSRT_H */
