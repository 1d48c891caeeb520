// path.h — device-side restatement of the reference hot path for gfx950.
//   BoundingBox::hit      geom.rs:218-247
//   Sphere::intersect     geom.rs:56-93
//   Triangle::intersect   geom.rs:504-585 (candidate test; shading deferred)
//   Instance::intersect   geom.rs:403-420
//   BvhNode::intersect    geom.rs:185-205 (via the preorder stream, layout.h)
//   World::intersect      world.rs:131-144
//   Camera::ray           world.rs:53-63
//   Material::scatter/emit material.rs:203-329,385-389
//   Background            material.rs:49-89
//   Texture::get_f        texture.rs:126-148, WrapMode::wrap texture.rs:278-299
// All arithmetic follows mrt_math.h's evaluation order; build with
// -ffp-contract=off and correctly rounded f32 divide/sqrt.
#pragma once
#include <hip/hip_runtime.h>

#include "../mrt_math.h"
#include "../mrt_rng.h"
#include "layout.h"

namespace mrt {

#define MRT_DEV __device__ __forceinline__

constexpr uint32_t kRefNone = 0u;
MRT_DEV uint32_t make_ref(uint32_t kind, uint32_t idx) { return (kind << 28) | idx; }

struct DevCounters {
  unsigned long long samples, segments, node_visits, sphere_tests, triangle_tests, instance_entries,
      model_entries, closest_hits, texel_taps, bounces, wave_slots, lane_steps, box_exact, shaded, vnf_fallbacks,
      shade_waves, shade_kinds, shade_materials;
};

struct LocalCounters {
  uint32_t node_visits = 0, sphere_tests = 0, triangle_tests = 0, instance_entries = 0, model_entries = 0,
           texel_taps = 0, wave_slots = 0, lane_steps = 0, box_exact = 0, vnf_fallbacks = 0, shade_waves = 0,
           shade_kinds = 0, shade_materials = 0;
};

// Bounds checks of every scene-array index, compiled in with
// -DMRT_DEBUG_BOUNDS (libmassrt_dbg.so): a failing index is recorded in
// S.dbg and replaced by 0, so a bad index shows up as a record instead of a
// GPU memory fault.
#ifdef MRT_DEBUG_BOUNDS
MRT_DEV uint32_t mrt_chk(uint32_t* dbg, uint32_t idx, uint32_t bound, uint32_t code) {
  if (idx < bound) return idx;
  if (atomicCAS(dbg, 0u, code) == 0u) {
    dbg[1] = idx;
    dbg[2] = bound;
  }
  atomicAdd(dbg + 3, 1u);
  return 0;
}
#define MRT_IDX(S, idx, bound, code) mrt_chk((S).dbg, (idx), (bound), (code))
#else
#define MRT_IDX(S, idx, bound, code) (idx)
#endif

MRT_DEV float u2f(uint32_t u) { return __uint_as_float(u); }
MRT_DEV V3 ld3(const float* p) { return V3{p[0], p[1], p[2]}; }
// `c ? uv : V2{0, 0}` per component: the conditional on whole aggregates made
// clang select between the addresses of two stack temporaries, which kept
// them in scratch memory (k_shade spilled 44 B per lane)
MRT_DEV V2 uv_or_zero(bool c, V2 uv) { return V2{c ? uv.x : 0.0f, c ? uv.y : 0.0f}; }

// ---- textures -----------------------------------------------------------
MRT_DEV float rust_fract(float x) { return x - truncf(x); }
// `f32 as usize` saturates: NaN and negatives -> 0
MRT_DEV uint32_t f2usize(float f) { return f > 0.0f ? (f < 4294967040.0f ? (uint32_t)f : 0xFFFFFFFFu) : 0u; }

MRT_DEV V4 texel(const DevScene& S, const GpuTexture& t, uint32_t x, uint32_t y) {
  const uint32_t tpr = (t.width + kTexBlockW - 1) / kTexBlockW;  // layout.h: 8x4-texel blocks
  uint32_t v = S.texels[MRT_IDX(S, t.offset + texel_index(tpr, x, y), S.n_texels, 1)];
  return V4{(float)(v & 255u) / 255.0f, (float)((v >> 8) & 255u) / 255.0f, (float)((v >> 16) & 255u) / 255.0f,
            (float)(v >> 24) / 255.0f};
}

MRT_DEV V4 texture_get_f(const DevScene& S, uint32_t tex, V2 uv, LocalCounters& lc) {
  const GpuTexture t = S.textures[MRT_IDX(S, tex, S.n_textures, 2)];
  float x = uv.x, y = uv.y;
  if (t.wrap == MRT_WRAP_REPEAT) {
    x = x < 0.0f ? 1.0f - rust_fract(fabsf(x)) : x;
    y = y < 0.0f ? 1.0f - rust_fract(fabsf(y)) : y;
    x = x > 1.0f ? rust_fract(x) : x;
    y = y > 1.0f ? rust_fract(y) : y;
  } else {
    x = fmaxf(fminf(x, 1.0f), 0.0f);
    y = fmaxf(fminf(y, 1.0f), 0.0f);
  }
  x = x * (float)(t.width - 1);
  y = y * (float)(t.height - 1);
  uint32_t x0 = f2usize(floorf(x)), x1 = f2usize(ceilf(x));
  uint32_t y0 = f2usize(floorf(y)), y1 = f2usize(ceilf(y));
  x0 = x0 < t.width ? x0 : t.width - 1;  // the reference would panic out of range
  x1 = x1 < t.width ? x1 : t.width - 1;
  y0 = y0 < t.height ? y0 : t.height - 1;
  y1 = y1 < t.height ? y1 : t.height - 1;
  float tt = x - (float)x0;
  V4 p0 = texel(S, t, x0, y0) * (1.0f - tt) + texel(S, t, x1, y0) * tt;
  V4 p1 = texel(S, t, x0, y1) * (1.0f - tt) + texel(S, t, x1, y1) * tt;
  tt = y - (float)y0;
  lc.texel_taps += 4;
  return p1 * tt + p0 * (1.0f - tt);
}

// YCbCrTexture::get_f tail (texture.rs:233-249): YUV_TRANSFORM as a point
// transform (generic.rs:105-115), clamp to [0,1], powf(2.2); alpha 1.
MRT_DEV V4 ycbcr(V4 luma, V4 chroma) {
  constexpr float KR = 0.2126f, KG = 0.7152f, KB = 0.0722f;
  const M4 m{V4{1.0f, 1.0f, 1.0f, 0.0f}, V4{0.0f, -(KB / KG) * (2.0f - 2.0f * KB), 2.0f - 2.0f * KB, 0.0f},
             V4{2.0f - 2.0f * KR, -(KR / KG) * (2.0f - 2.0f * KR), 0.0f, 0.0f}, V4{0.0f, 0.0f, 0.0f, 1.0f}};
  V3 c = transform(m, V3{luma.x, chroma.x - 0.5f, chroma.y - 0.5f}, 1.0f);
  c = V3{fmaxf(fminf(c.x, 1.0f), 0.0f), fmaxf(fminf(c.y, 1.0f), 0.0f), fmaxf(fminf(c.z, 1.0f), 0.0f)};
  return V4{powf(c.x, 2.2f), powf(c.y, 2.2f), powf(c.z, 2.2f), 1.0f};
}
MRT_DEV V4 vmin4(V4 a, V4 b) { return V4{fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z), fminf(a.w, b.w)}; }
MRT_DEV V4 vmax4(V4 a, V4 b) { return V4{fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w)}; }

// A composite surface's postfix program (layout.h). The operand stack is
// kSurfStack registers shifted on push/pop (static indices only, so it never
// lives in scratch); only the EXT kernel variants contain this code.
MRT_DEV V4 surface_program(const DevScene& S, uint32_t start, uint32_t len, V2 uv, LocalCounters& lc) {
  static_assert(kSurfStack == 4, "stack shifts below are written for 4 slots");
  V4 s0{}, s1{}, s2{}, s3{};
  for (uint32_t i = 0; i < len; ++i) {
    const GpuSurfOp o = S.surf_ops[MRT_IDX(S, start + i, S.n_surf_ops, 17)];
    const V4 color{o.color[0], o.color[1], o.color[2], o.color[3]};
    if (o.op == MRT_SURF_SOLID || o.op == MRT_SURF_TEXTURE) {  // push
      const V4 v = o.op == MRT_SURF_TEXTURE ? texture_get_f(S, o.tex, uv, lc) : color;
      s3 = s2, s2 = s1, s1 = s0, s0 = v;
    } else if (o.op == MRT_SURF_FALLBACK) {  // SolidColorFallback::get_f (texture.rs:353-356)
      s0 = (color * (1.0f - s0.w)) + (s0 * s0.w);
    } else {  // binary: left = s1, right = s0
      V4 v;
      if (o.op == MRT_SURF_YCBCR) v = ycbcr(s1, s0);
      else if (o.arg == MRT_BLEND_LIGHTEN) v = vmax4(s1, s0);  // BlendMode::blend (texture.rs:260-267)
      else if (o.arg == MRT_BLEND_DARKEN) v = vmin4(s1, s0);
      else if (o.arg == MRT_BLEND_ADDITION) v = vmin4(s1 + s0, V4{1.0f, 1.0f, 1.0f, 1.0f});
      else v = vmax4(s1 - s0, V4{0.0f, 0.0f, 0.0f, 0.0f});
      s0 = v, s1 = s2, s2 = s3;
    }
  }
  return s0;
}

template <bool EXT>
MRT_DEV V4 surface_ref_get_f(const DevScene& S, uint32_t kind, uint32_t index, uint32_t len, const float* color,
                             V2 uv, LocalCounters& lc) {
  if (kind == MRT_SURF_TEXTURE) return texture_get_f(S, index, uv, lc);
  if (EXT && kind == SURF_PROGRAM) return surface_program(S, index, len, uv, lc);
  return V4{color[0], color[1], color[2], color[3]};
}

template <bool EXT>
MRT_DEV V4 surface_get_f(const DevScene& S, const GpuMaterial& m, V2 uv, LocalCounters& lc) {
  return surface_ref_get_f<EXT>(S, m.surf_kind, m.texture, m.surf_len, m.color, uv, lc);
}

// ---- primitive tests -------------------------------------------------------
// Correctly rounded quotient a/b from y = RN(1/b) (computed once per ray,
// rcp_cr: exactly the IEEE 1/b): q0 = a*y can be ~2 ulp off; one FMA residual
// correction makes it faithful and a second rounds it exactly (Markstein's
// theorem: y within 1/2 ulp of 1/b + faithful q => RN(q + (a - bq)y) = RN(a/b),
// absent under/overflow). Results outside [2^-90, 2^90], dividends below
// 2^-100 and divisors outside [2^-60, 2^60] take the plain division. 1 mul + 4 fma instead of the ~10
// instruction v_div_scale/v_rcp/v_div_fmas/v_div_fixup sequence; verified
// bit-exact against `a / b` by mrt_selftest_division.
struct Recip {
  float b, y;
};
MRT_DEV Recip make_recip(float b) {
  Recip r;
  r.b = b;
  r.y = rcp_cr(b);
  return r;
}
// divisor inside the fast path's range
MRT_DEV bool recip_ok(const Recip& r) { return fabsf(r.b) >= 0x1p-60f && fabsf(r.b) <= 0x1p60f; }
// q ~ RN(a/b): exact whenever div_in_range(q, a) and the divisor was `ok`
MRT_DEV float div_fast(float a, const Recip& r) {
  float q = a * r.y;
  float e = fmaf(-q, r.b, a);
  q = fmaf(e, r.y, q);
  e = fmaf(-q, r.b, a);
  return fmaf(e, r.y, q);
}
// fast path valid: quotient in [2^-90, 2^90] and dividend >= 2^-100 (else the
// FMA residual a - q*b can fall into the subnormal range and lose bits)
MRT_DEV bool div_in_range(float q, float a) {
  float aq = fabsf(q);
  return (aq <= 0x1p90f && aq >= 0x1p-90f && fabsf(a) >= 0x1p-100f) || a == 0.0f;
}
MRT_DEV float div_cr(float a, const Recip& r) {
  float q = div_fast(a, r);
  if (!recip_ok(r) || !div_in_range(q, a)) q = a / r.b;
  return q;
}
// Ray in the space being traversed (world, or an instance's object space)
// with what the slab test needs: y = RN(1/d) per axis, the products
// oy = RN(o*y) of the early slab decision, its error margin om, and |d|^2.
struct TRay {
  V3 o, d;
  float yx, yy, yz;
  float oyx, oyy, oyz;  // RN(o.k * y.k)
  // |om| = max(max_k |oy.k| * 2^-20, 2^-120), the early decision's absolute
  // margin term (box_hit_any), or +inf when the early decision does not apply
  // to this ray (outside the early domain below: every box test is exact);
  // its sign bit set: the exact test may NOT use qfast (the ray or the scene
  // is outside the qfast domain below)
  float om;
  Recip a;  // |d|^2 for Sphere::intersect
};
// the early slab decision applies to this ray (early domain below)
MRT_DEV bool tray_fast(const TRay& r) { return fabsf(r.om) != INFINITY; }
// qfast domain: with every box coordinate and ray-origin coordinate in
// {0} U [2^-40, 2^28] (scene bound checked on the host, origin here) each
// nonzero numerator (min - o) is >= 2^-63 and < 2^29; with |d| in
// [2^-20, 2^20] every quotient lies in [2^-83, 2^49] — inside div_fast's
// exact range — so no per-quotient check is needed.
// Early domain (slab_fast): its error bound needs no lower bound on the
// coordinates, only that no product overflows — box and origin coordinates
// finite and within 2^28, |d| in [2^-20, 2^20] — plus an absolute 2^-149 per
// rounding in the subnormal range, which the 2^-120 floor of |om| covers. (A
// mesh vertex at sin(pi) ~ 1e-16 is outside the qfast domain; until round 2's
// split it switched the whole 1M-triangle mesh_ply scene to the exact test.)
MRT_DEV bool coord_ok(float c) {
  float a = fabsf(c);
  return a == 0.0f || (a >= 0x1p-40f && a <= 0x1p28f);
}
MRT_DEV bool orig_ok(float c) { return fabsf(c) <= 0x1p28f; }
MRT_DEV bool dir_ok(float c) {
  float a = fabsf(c);
  return a >= 0x1p-20f && a <= 0x1p20f;
}
// scene_flags (DevScene::fast_ok): bit 0 every box coordinate in the qfast
// domain, bit 1 every box coordinate finite and within 2^28.
MRT_DEV TRay make_tray(V3 o, V3 d, uint32_t scene_flags) {
  TRay r;
  r.o = o;
  r.d = d;
  r.yx = rcp_cr(d.x);
  r.yy = rcp_cr(d.y);
  r.yz = rcp_cr(d.z);
  r.oyx = o.x * r.yx;
  r.oyy = o.y * r.yy;
  r.oyz = o.z * r.yz;
  const float om = fmaxf(fmaxf(fmaxf(fabsf(r.oyx), fabsf(r.oyy)), fabsf(r.oyz)) * 0x1p-20f, 0x1p-120f);
  r.a = make_recip(length_squared(d));
  const bool dok = dir_ok(d.x) && dir_ok(d.y) && dir_ok(d.z);
  const bool qok = (scene_flags & 1u) && coord_ok(o.x) && coord_ok(o.y) && coord_ok(o.z) && dok;
  const bool fast = (scene_flags & 2u) && orig_ok(o.x) && orig_ok(o.y) && orig_ok(o.z) && dok;
  const float m = fast ? om : INFINITY;
  r.om = qok ? m : -m;
  return r;
}
MRT_DEV float qfast(float a, float b, float y) {
  float q = a * y;
  float e = fmaf(-q, b, a);
  q = fmaf(e, y, q);
  e = fmaf(-q, b, a);
  return fmaf(e, y, q);
}

MRT_DEV bool sphere_hit(V3 c, float r, V3 o, V3 d, const Recip& ra, float tmin, float tmax, float& t) {
  V3 oc = o - c;
  float a = ra.b;  // length_squared(d), precomputed per ray
  float half_b = dot(oc, d);
  float cc = length_squared(oc) - (r * r);
  float disc = (half_b * half_b) - (a * cc);
  if (disc < 0.0f) return false;
  float sq = sqrtf(disc);
  float root = div_cr(-half_b - sq, ra);
  if (root < tmin || tmax < root) {
    root = div_cr(-half_b + sq, ra);
    if (root < tmin || tmax < root) return false;
  }
  t = root;
  return true;
}

MRT_DEV bool tri_hit(V3 a, V3 ab, V3 ac, V3 o, V3 d, float tmin, float tmax, float& t) {
  V3 p_vec = cross(d, ac);
  float det = dot(ab, p_vec);
  if (fabsf(det) < 0.000001f) return false;
  float inv_det = rcp_cr(det);  // RN(1 / det), as the reference's 1.0 / det
  V3 t_vec = o - a;
  float u = dot(t_vec, p_vec) * inv_det;
  if (u < 0.0f || u > 1.0f) return false;
  V3 q_vec = cross(t_vec, ab);
  float v = dot(d, q_vec) * inv_det;
  if (v < 0.0f || v + u > 1.0f) return false;
  float tt = dot(ac, q_vec) * inv_det;
  if (tt < tmin || tt > tmax) return false;
  t = tt;
  return true;
}

// The same test without early exits (the near-first leaf step, whose lanes
// are mixed: every lane pays the whole test either way, and the exits cost
// exec-mask juggling): identical arithmetic, the conditions combined at the end.
MRT_DEV bool tri_hit_nb(V3 a, V3 ab, V3 ac, V3 o, V3 d, float tmin, float tmax, float& t) {
  V3 p_vec = cross(d, ac);
  float det = dot(ab, p_vec);
  float inv_det = rcp_cr(det);
  V3 t_vec = o - a;
  float u = dot(t_vec, p_vec) * inv_det;
  V3 q_vec = cross(t_vec, ab);
  float v = dot(d, q_vec) * inv_det;
  float tt = dot(ac, q_vec) * inv_det;
  t = tt;
  return !(fabsf(det) < 0.000001f) && !(u < 0.0f || u > 1.0f) && !(v < 0.0f || v + u > 1.0f) && !(tt < tmin || tt > tmax);
}

struct TriShade {
  V3 a, b, c, na, nb, nc;
  V2 uva, uvb, uvc;
  uint32_t material, flags;
};
MRT_DEV TriShade load_tri(const DevScene& S, uint32_t id) {
  const float4* q = reinterpret_cast<const float4*>(S.tri_shade) + (size_t)MRT_IDX(S, id, S.n_tris, 3) * kTriShadeQuads;
  float4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4], q5 = q[5], q6 = q[6];
  TriShade s;
  s.a = V3{q0.x, q0.y, q0.z};
  s.b = V3{q0.w, q1.x, q1.y};
  s.c = V3{q1.z, q1.w, q2.x};
  s.na = V3{q2.y, q2.z, q2.w};
  s.nb = V3{q3.x, q3.y, q3.z};
  s.nc = V3{q3.w, q4.x, q4.y};
  s.uva = V2{q4.z, q4.w};
  s.uvb = V2{q5.x, q5.y};
  s.uvc = V2{q5.z, q5.w};
  s.material = __float_as_uint(q6.x);
  s.flags = __float_as_uint(q6.y);
  return s;
}

// Area-ratio barycentrics of the accepted point (geom.rs:535-547)
MRT_DEV void tri_bary(const TriShade& s, V3 point, float& a0, float& a1, float& a2) {
  V3 d0 = s.a - point, d1 = s.b - point, d2 = s.c - point;
  float area = length(cross(s.a - s.b, s.a - s.c));
  a0 = length(cross(d1, d2)) / area;
  a1 = length(cross(d2, d0)) / area;
  a2 = length(cross(d0, d1)) / area;
}

// Material::alpha_test of the triangle's OWN material (geom.rs:567-571,
// material.rs:222-224,281-283): surface alpha != 0.
template <bool RNG, bool EXT>
MRT_DEV bool tri_alpha_pass(const DevScene& S, uint32_t id, V3 o, V3 d, float t, PathRng& rng, LocalCounters& lc) {
  TriShade s = load_tri(S, id);
  V3 point = o + d * t;
  float a0, a1, a2;
  tri_bary(s, point, a0, a1, a2);
  V2 uv = (s.uva * a0 + s.uvb * a1) + s.uvc * a2;
  GpuMaterial m = S.materials[MRT_IDX(S, s.material, S.n_materials, 4)];
  // Mix::alpha_test draws to pick a side (material.rs:418-424)
  if (RNG)
    while (m.kind == MRT_MAT_MIX) m = S.materials[MRT_IDX(S, rng.f32() < m.param ? m.left : m.right, S.n_materials, 4)];
  // Lambertian/Metal alpha_test; Specular's forwards to its inner Lambertian
  if (m.kind != MRT_MAT_LAMBERTIAN && m.kind != MRT_MAT_METAL && m.kind != MRT_MAT_SPECULAR) return true;
  return surface_get_f<EXT>(S, m, uv, lc).w != 0.0f;
}

MRT_DEV void load_m12(const float* p, V3& c0, V3& c1, V3& c2, V3& c3) {
  c0 = V3{p[0], p[1], p[2]};
  c1 = V3{p[3], p[4], p[5]};
  c2 = V3{p[6], p[7], p[8]};
  c3 = V3{p[9], p[10], p[11]};
}
// M4::transform (generic.rs:106-115) on the xyz rows: ((c0*x + c1*y) + c2*z) + c3*w
MRT_DEV V3 xform(V3 c0, V3 c1, V3 c2, V3 c3, V3 p, float w) {
  return ((c0 * p.x + c1 * p.y) + c2 * p.z) + c3 * w;
}

struct Hit {
  float t;
  uint32_t prim;       // make_ref(kind, id) or kRefNone
  uint32_t container;  // make_ref(INSTANCE|MODEL, id) or kRefNone
};

// World::intersect over the preorder stream, one record per step so that a
// persistent kernel can interleave many rays per lane (render.hip k_trace).
// Each lane's sequence of box/primitive tests is exactly the reference's
// (left-first recursion with shrinking t_max, geom.rs:185-205); only which
// lanes of a wave are busy at a time differs.
//
// Register budget: the per-lane state is kept small (occupancy is the lever
// for this latency-bound loop). The world ray is not kept: the rays live in
// the pool buffers (ro/rd), and leaving an instance's BLAS reloads it. The
// closest t so far is `best` (Hit.t is filled in by trav_hit()).
struct TravIn {
  const DevScene& S;
  const uint4* slots;      // record stream in global memory (S.slots, or S.slots_tl beside an LDS treelet)
  uint32_t world_begin;    // first record of the world region (an LDS-tagged index beside a treelet)
  const float4* ro;        // ray origins  (xyz) of the pool
  const float4* rd;        // ray directions (xyz)
  float tmin;
  uint4* rng = nullptr;    // the rays' RNG states (traversal draws: Volume, Mix alpha tests)
  float tmax0 = INFINITY;  // the walk's initial t_max (a near-first lane that falls back restarts with it)
  // k_trace (reference walk, no treelet): this lane's 4 x 16 B of LDS, stride
  // `stash_stride` float4s, holding the world ray while the lane is inside an
  // instance's BLAS — leaving it then costs 4 LDS reads instead of 2 pool
  // loads and make_tray's four correctly rounded divisions (nullptr: recompute)
  float4* stash = nullptr;
  uint32_t stash_stride = 0;
};
MRT_DEV void tray_stash(const TravIn& in, const TRay& r) {
  float4* p = in.stash;
  const uint32_t k = in.stash_stride;
  p[0] = make_float4(r.o.x, r.o.y, r.o.z, r.d.x);
  p[k] = make_float4(r.d.y, r.d.z, r.yx, r.yy);
  p[2 * k] = make_float4(r.yz, r.oyx, r.oyy, r.oyz);
  p[3 * k] = make_float4(r.om, r.a.b, r.a.y, 0.0f);
}
MRT_DEV TRay tray_unstash(const TravIn& in) {
  const float4* p = in.stash;
  const uint32_t k = in.stash_stride;
  const float4 a = p[0], b = p[k], c = p[2 * k], e = p[3 * k];
  TRay r;
  r.o = V3{a.x, a.y, a.z};
  r.d = V3{a.w, b.x, b.y};
  r.yx = b.z, r.yy = b.w, r.yz = c.x;
  r.oyx = c.y, r.oyy = c.z, r.oyz = c.w;
  r.om = e.x;
  r.a.b = e.y, r.a.y = e.z;
  return r;
}

// Inside a BLAS, `ret` is the world record after the instance/model record
// that entered it, with kRetInstance set for an instance; the container of a
// hit is recovered from that record when the ray finishes (trav_hit).
constexpr uint32_t kNoRet = 0xFFFFFFFFu;
constexpr uint32_t kRetInstance = 0x80000000u;
constexpr uint32_t kExactModeInit = 0xFFFFu;  // Trav::sp of the reference's walk (= kExactMode below)

struct Trav {
  TRay r;  // ray of the space being traversed (world, or instance object space)
  uint32_t ray;  // pool index of the ray
  uint32_t i, ret;
  float best;
  uint32_t prim, hit_ret;  // closest hit so far: primitive (kRefNone: none) and `ret` when found
  uint4 s0, s1;  // current record (prefetched when i moves)
  PathRng rng;   // the ray's stream, for scenes whose traversal draws (RNG variants only)
  uint32_t sp;   // near-first walk: stack entries in use (kExactMode: the reference's walk)
  float t2;      // near-first walk: the smallest t of the other hits it met (nf_finish)
  NfLine nfl;    // near-first walk: the current space's rounding margin, for t <= cull(best) (nf_bound.h nf_line)
  float nl;      // near-first walk: the current node's hits have t <= nl (its box's exit; +inf: unknown)
  bool done;
#ifdef MRT_DEBUG_BOUNDS
  uint32_t steps;
#endif
};

// LDS treelet (layout.h): records with kLdsTag in their index live in the
// workgroup's LDS copy (mrt_lds), the rest in the global stream. Kernels
// built with LDS=false never see a tagged index.
extern __shared__ uint4 mrt_lds[];
template <bool LDS>
MRT_DEV void rec_load2(const TravIn& in, uint32_t i, uint4& a, uint4& b) {
  if (LDS && (i & kLdsTag)) {
    const uint32_t j = i & kIdxMask;
    a = mrt_lds[MRT_IDX(in.S, j, in.S.n_tlet, 22)];
    b = mrt_lds[MRT_IDX(in.S, j + 1, in.S.n_tlet, 22)];
  } else {
    MRT_IDX(in.S, i + 1, in.S.n_slots, 6);
    const uint4* p = in.slots + MRT_IDX(in.S, i, in.S.n_slots, 5);  // one address, offset:16 for slot 2
    a = p[0];
    b = p[1];
  }
}
template <bool LDS>
MRT_DEV uint4 rec_load1(const TravIn& in, uint32_t i) {
  if (LDS && (i & kLdsTag)) return mrt_lds[MRT_IDX(in.S, i & kIdxMask, in.S.n_tlet, 22)];
  return in.slots[MRT_IDX(in.S, i, in.S.n_slots, 7)];
}

template <bool LDS = false>
MRT_DEV Hit trav_hit(const TravIn& in, const Trav& t) {
  uint32_t container = kRefNone;
  if (t.hit_ret != kNoRet) {
    const uint32_t rec = (t.hit_ret & ~kRetInstance) - 2;  // the instance/model record
    container = make_ref((t.hit_ret & kRetInstance) ? MRT_REF_INSTANCE : MRT_REF_MODEL, rec_load1<LDS>(in, rec).x);
  }
  return Hit{t.best, t.prim, container};
}

// f32 min/max without the canonicalising v_max hipcc inserts before fminf:
// every operand here is an arithmetic result (never a signalling NaN), for
// which v_min/v_max/v_min3/v_max3 are IEEE minNum/maxNum = Rust f32::min/max.
MRT_DEV float vmin1(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
MRT_DEV float vmax1(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
MRT_DEV float vmin3(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
MRT_DEV float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// max(|a|, |b|, c) in one instruction (the abs as source modifiers)
MRT_DEV float vmax3ab(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, |%1|, |%2|, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// BoundingBox::hit (geom.rs:218-247): v_min = (min - o)/d, v_max = (max - o)/d,
// six correctly rounded quotients — qfast in the ray's fast domain (bit-identical
// to IEEE division there), IEEE division otherwise. The per-axis early-outs
// cannot change the result (t0 only grows, t1 only shrinks, NaNs are ignored
// by min/max): one final compare of max(tmin, lo) against min(tmax, hi).
MRT_DEV bool box_hit_exact(V3 mn, V3 mx, const TRay& r, float tmin, float tmax) {
  V3 na = mn - r.o, nb = mx - r.o;
  V3 a{qfast(na.x, r.d.x, r.yx), qfast(na.y, r.d.y, r.yy), qfast(na.z, r.d.z, r.yz)};
  V3 b{qfast(nb.x, r.d.x, r.yx), qfast(nb.y, r.d.y, r.yy), qfast(nb.z, r.d.z, r.yz)};
  if (signbit(r.om)) {  // outside the qfast domain
    a = na / r.d;
    b = nb / r.d;
  }
  float t0 = vmax3(vmin1(a.x, b.x), vmin1(a.y, b.y), vmax1(vmin1(a.z, b.z), tmin));
  float t1 = vmin3(vmax1(a.x, b.x), vmax1(a.y, b.y), vmin1(vmax1(a.z, b.z), tmax));
  return !(t1 < t0);
}

// The same decision, cheaper: in the fast domain a = RN(m*y - RN(o*y)) (one
// FMA per slab plane) is within |Q|*2^-22.4 + |o*y|*2^-23.9 of the correctly
// rounded quotient RN((m - o)/d) — one rounding in y = RN(1/d), one in o*y,
// one in the FMA, half an ulp to the quotient; no under/overflow in the fast
// domain. min/max are 1-Lipschitz and the terms that decide them lie at t0
// (t1), so t0 and t1 carry that bound relative to their own magnitude plus
// max_k |o.k*y.k|*2^-23.9. When t1 - t0 exceeds (|t0|+|t1|)*2^-19 + |om| (|om| >=
// max_k |o.k*y.k|*2^-20, 4x slack on both terms) the comparison of the exact
// values is decided; otherwise — grazing rays, flat boxes, ties — the exact
// test decides. mrt_selftest_slab checks this against box_hit_exact on
// near-tie boxes.
MRT_DEV void slab_fast(V3 mn, V3 mx, const TRay& r, float tmin, float tmax, float& t0, float& t1) {
  const float ax = fmaf(mn.x, r.yx, -r.oyx), ay = fmaf(mn.y, r.yy, -r.oyy), az = fmaf(mn.z, r.yz, -r.oyz);
  const float bx = fmaf(mx.x, r.yx, -r.oyx), by = fmaf(mx.y, r.yy, -r.oyy), bz = fmaf(mx.z, r.yz, -r.oyz);
  t0 = vmax3(vmin1(ax, bx), vmin1(ay, by), vmax1(vmin1(az, bz), tmin));
  t1 = vmin3(vmax1(ax, bx), vmax1(ay, by), vmin1(vmax1(az, bz), tmax));
}
MRT_DEV float slab_margin(const TRay& r, float t0, float t1) {
  return fmaf(fabsf(t0) + fabsf(t1), 0x1p-19f, fabsf(r.om));
}
template <bool COUNT = false>
MRT_DEV bool box_hit_any(V3 mn, V3 mx, const TRay& r, float tmin, float tmax, LocalCounters* lc = nullptr) {
  // no branch on the ray's domain: outside the early domain |om| = +inf makes
  // the margin +inf (or NaN), so neither comparison decides and the exact
  // test runs
  {
    float t0, t1;
    slab_fast(mn, mx, r, tmin, tmax, t0, t1);
    const float m = slab_margin(r, t0, t1);
    const float gap = t1 - t0;
    if (gap > m) return true;
    if (-gap > m) return false;
  }
  if (COUNT) lc->box_exact++;
  return box_hit_exact(mn, mx, r, tmin, tmax);
}

MRT_DEV TRay world_ray(const TravIn& in, uint32_t ray) {
  const float4 o4 = in.ro[ray], d4 = in.rd[ray];
  return make_tray(V3{o4.x, o4.y, o4.z}, V3{d4.x, d4.y, d4.z}, in.S.fast_ok);
}

// Load record t.i. Every region ends in an END record (handled by
// trav_prim: leave the BLAS, or finish), so there is no bounds compare here.
template <bool LDS = false>
MRT_DEV void trav_fetch(const TravIn& in, Trav& t) {
#ifdef MRT_DEBUG_BOUNDS
  if (++t.steps > (1u << 24)) {  // record and stop instead of looping
    MRT_IDX(in.S, 0xFFFFFFF0u, 0u, 5);
    t.done = true;
    t.s1.w = KIND_END;  // a done lane never holds a box record (k_trace's box run)
    return;
  }
#endif
  rec_load2<LDS>(in, t.i, t.s0, t.s1);
}

// The region ended: leave the BLAS back to the world ray (geom.rs:405-409;
// a model shares the world ray, an instance's object-space ray is replaced),
// or finish the ray.
MRT_DEV void trav_end_index(const TravIn& in, Trav& t) {
  if (t.ret == kNoRet) {
    t.done = true;
    return;
  }
  if (t.ret & kRetInstance) t.r = in.stash ? tray_unstash(in) : world_ray(in, t.ray);
  t.i = t.ret & ~kRetInstance;
  t.ret = kNoRet;
}

MRT_DEV void nf_start(const TravIn& in, Trav& t);  // the near-first walk's start (below)

// Start ray `ray` of the pool (World::intersect(ray, in.tmin, tmax)).
template <bool RNG = false, bool LDS = false>
MRT_DEV void trav_init(const TravIn& in, Trav& t, uint32_t ray, float tmax, uint32_t start = 0xFFFFFFFFu) {
  if (RNG) {
    const uint4 q = in.rng[ray];
    t.rng = PathRng{(unsigned long long)q.x | ((unsigned long long)q.y << 32),
                    (unsigned long long)q.z | ((unsigned long long)q.w << 32)};
  }
  t.r = world_ray(in, ray);
  t.ray = ray;
  t.i = start == 0xFFFFFFFFu ? in.world_begin : start;  // the near-first walk starts at its own world tree
  t.sp = start == 0xFFFFFFFFu ? kExactModeInit : 0u;
  t.t2 = INFINITY;
  t.ret = kNoRet;
  t.best = tmax;
  t.prim = kRefNone;
  t.hit_ret = kNoRet;
  t.done = false;
#ifdef MRT_DEBUG_BOUNDS
  t.steps = 0;
#endif
  if (start != 0xFFFFFFFFu) nf_start(in, t);
  trav_fetch<LDS>(in, t);
}

MRT_DEV bool trav_at_box(const Trav& t) { return (int32_t)t.s1.w < 0; }  // kBoxFlag (layout.h)

// The current record is a box: test it and move on.
template <bool COUNT, bool LDS = false>
MRT_DEV void trav_box(const TravIn& in, Trav& t, LocalCounters& lc) {
  if (COUNT) lc.node_visits++;
  V3 mn{u2f(t.s0.x), u2f(t.s0.y), u2f(t.s0.z)}, mx{u2f(t.s0.w), u2f(t.s1.x), u2f(t.s1.y)};
  t.i = box_hit_any<COUNT>(mn, mx, t.r, in.tmin, t.best, &lc) ? (t.s1.w & ~kBoxFlag) : t.s1.z;
  trav_fetch<LDS>(in, t);
}

// trav_box without the fetch of the next record (k_trace's box run loads at
// the top of each step).
template <bool COUNT>
MRT_DEV void trav_box_index(const TravIn& in, Trav& t, LocalCounters& lc) {
  if (COUNT) lc.node_visits++;
  V3 mn{u2f(t.s0.x), u2f(t.s0.y), u2f(t.s0.z)}, mx{u2f(t.s0.w), u2f(t.s1.x), u2f(t.s1.y)};
  t.i = box_hit_any<COUNT>(mn, mx, t.r, in.tmin, t.best, &lc) ? (t.s1.w & ~kBoxFlag) : t.s1.z;
}

// The current record is a primitive, an instance or a model. ALPHA=false is
// the specialisation for scenes without alpha-tested triangles (the alpha
// test's registers would otherwise cost occupancy everywhere).
// The ray's RNG state back to the pool (RNG variants, when the ray is done).
MRT_DEV void trav_store_rng(const TravIn& in, const Trav& t) {
  in.rng[t.ray] = make_uint4((uint32_t)t.rng.s0, (uint32_t)(t.rng.s0 >> 32), (uint32_t)t.rng.s1,
                             (uint32_t)(t.rng.s1 >> 32));
}

// Volume::intersect with a sphere target (geom.rs:609-653): entry and exit of
// the target over the whole line, clipped to [tmin, best], then a distance
// f.ln() * -1/density drawn from the ray's stream; the ln is looked up
// (S.ln_table, upload.h) for the exact value of the host libm.
MRT_DEV bool volume_hit(const DevScene& S, const TravIn& in, Trav& t, uint4 s0, uint32_t vid, float& th) {
  const V3 c{u2f(s0.x), u2f(s0.y), u2f(s0.z)};
  const float rad = u2f(s0.w);
  float te, tx;
  if (!sphere_hit(c, rad, t.r.o, t.r.d, t.r.a, -INFINITY, INFINITY, te)) return false;
  if (!sphere_hit(c, rad, t.r.o, t.r.d, t.r.a, te + 0.0001f, INFINITY, tx)) return false;
  if (te < in.tmin) te = in.tmin;
  if (tx > t.best) tx = t.best;
  if (te >= tx) return false;
  if (te < 0.0f) te = 0.0f;
  const float len = sqrtf(length_squared(t.r.d));
  const float inside = (tx - te) * len;
  const uint32_t m = (uint32_t)(t.rng.next() >> 32) >> 9;  // the draw of f32() (mrt_rng.h)
  const float dist = S.ln_table[MRT_IDX(S, m, 1u << 23, 14)] * S.vol_nid[MRT_IDX(S, vid, S.n_vol, 15)];
  if (dist > inside) return false;
  th = te + dist / len;
  return true;
}

// ALPHA: 0 no alpha tests, 1 alpha tests, 2 alpha tests over EXT surfaces
// trav_prim_index moves to the next record (or finishes the ray) without
// loading it; trav_prim also loads it.
template <bool COUNT, uint32_t ALPHA, bool RNG = false, bool LDS = false>
MRT_DEV void trav_prim_index(const TravIn& in, Trav& t, LocalCounters& lc) {
  const DevScene& S = in.S;
  const uint4 s0 = t.s0, s1 = t.s1;
  const uint32_t kind = s1.w;
  if (kind == KIND_END) {
    trav_end_index(in, t);
    return;
  }
  if (kind == KIND_TRI) {
    if (COUNT) lc.triangle_tests++;
    const uint4 s2 = rec_load1<LDS>(in, t.i + 2);
    V3 a{u2f(s0.x), u2f(s0.y), u2f(s0.z)}, ab{u2f(s0.w), u2f(s1.x), u2f(s1.y)}, ac{u2f(s2.x), u2f(s2.y), u2f(s2.z)};
    float th;
    if (tri_hit(a, ab, ac, t.r.o, t.r.d, in.tmin, t.best, th)) {
      const uint32_t id = s1.z & kTriIdMask;
      if (!ALPHA || !(s1.z & kTriAlpha) || tri_alpha_pass<RNG, ALPHA == 2>(S, id, t.r.o, t.r.d, th, t.rng, lc)) {
        t.best = th;
        t.prim = make_ref(MRT_REF_TRIANGLE, id);
        t.hit_ret = t.ret;
      }
    }
    t.i = s2.w;
  } else if (kind == KIND_SPHERE) {
    if (COUNT) lc.sphere_tests++;
    float th;
    if (sphere_hit(V3{u2f(s0.x), u2f(s0.y), u2f(s0.z)}, u2f(s0.w), t.r.o, t.r.d, t.r.a, in.tmin, t.best, th)) {
      t.best = th;
      t.prim = make_ref(MRT_REF_SPHERE, s1.x);
      t.hit_ret = t.ret;
    }
    t.i = s1.y;
  } else if (RNG && kind == KIND_VOLUME) {
    float th;
    if (volume_hit(S, in, t, s0, s1.x, th)) {
      t.best = th;
      t.prim = make_ref(MRT_REF_VOLUME, s1.x);
      t.hit_ret = t.ret;
    }
    t.i = s1.y;
  } else if (kind == KIND_INST) {
    if (COUNT) lc.instance_entries++;
    V3 c0, c1, c2, c3;
    load_m12(S.inst_inv + (size_t)MRT_IDX(S, s0.x, S.n_inst, 8) * 12, c0, c1, c2, c3);
    // entered from the world region: t.r is the world ray here
    if (in.stash) tray_stash(in, t.r);
    t.r = make_tray(xform(c0, c1, c2, c3, t.r.o, 1.0f), xform(c0, c1, c2, c3, t.r.d, 0.0f), S.fast_ok);
    t.ret = (t.i + 2) | kRetInstance;
    t.i = s0.y;
  } else {  // KIND_MODEL
    if (COUNT) lc.model_entries++;
    t.ret = t.i + 2;
    t.i = s0.y;
  }
}
template <bool COUNT, uint32_t ALPHA, bool RNG = false, bool LDS = false>
MRT_DEV void trav_prim(const TravIn& in, Trav& t, LocalCounters& lc) {
  trav_prim_index<COUNT, ALPHA, RNG, LDS>(in, t, lc);
  if (!t.done) trav_fetch<LDS>(in, t);
}

// ---- verified near-first walk (layout.h, nf_tree.cpp; k_trace<..., NF>) ------
// The lane walks the SAH trees near child first with a stack of record
// indices in LDS (kNfStack entries per lane, stride BLK), finds the closest
// hit with the reference's tie rule, then checks that the reference's
// left-first walk reaches that hit; if not it walks again the reference's
// way (sp = kExactMode: trav_box_index / trav_prim_index on the reference
// stream, the exact kernel's steps). Boxes are culled at cull(best) = best *
// (1 + 2^-10), each thickened by rho (nf_bound.h): a bound, proven for the
// reference's own f32 arithmetic, on how far a primitive's computed hit can
// lie outside its box — so the walk meets every primitive whose computed t is
// at most cull(best). Rays the bound does not cover (a
// generic triangle's kappa above kNfKappaMax) take the reference's walk.
constexpr uint32_t kExactMode = kExactModeInit;
constexpr uint32_t kNfDone = 0xFFFEu;     // Trav::sp: the near-first walk is over, its hit not yet checked
constexpr uint32_t kNfRet = 0x80000000u;  // stack marker: leave the BLAS (back to the world ray)

struct NfStack {
  uint32_t* p;  // this lane's entry 0 (LDS)
  uint32_t stride;
};
MRT_DEV void nf_push(const NfStack& k, Trav& t, uint32_t v) {
  k.p[t.sp * k.stride] = v;
  t.sp += 1;  // the builder bounds the depth (nf_stack_need <= kNfStack)
}
MRT_DEV float nf_cull(float best) { return fmaf(fabsf(best), 0x1p-10f, best); }
// t.nfc: the rounding margin's coefficients (nf_bound.h) of the space being
// walked — set when the walk enters a space; nf_rho_at turns them into how
// far a node's boxes are thickened (trav_box_index_nf)
MRT_DEV void nf_margin(const TravIn& in, Trav& t) {
  const bool obj = t.ret != kNoRet && (t.ret & kRetInstance);
  const NfBound& B = in.S.nfb;
  const NfCoef c = obj ? nf_coef_object(B, t.r.o, t.r.a.b) : nf_coef_world(B, t.r.o, t.r.a.b);
  t.nfl = nf_line(B, c, nf_cull(t.best), obj ? B.ao0 : B.aw0, obj ? B.ao1 : B.aw1, t.r.a.b, t.r.d);
}
// the walk starts at the NF world tree (trav_init): rays its bound does not
// cover take the reference's walk instead
MRT_DEV void nf_start(const TravIn& in, Trav& t) {
  if (nf_ray_ok(in.S.nfb, t.r.a.b)) {
    nf_margin(in, t);
    t.nl = INFINITY;
  } else {
    t.i = in.world_begin;
    t.sp = kExactModeInit;
  }
}
// next record from the stack; false: the walk is over. A return marker
// (leaving a BLAS) sits above world entries only — instances are world
// objects, never nested — so one pop meets at most one: straight-line code,
// the marker's branch taken only by the lanes that leave a BLAS.
MRT_DEV bool nf_pop(const TravIn& in, const NfStack& k, Trav& t) {
  if (t.sp == 0) return false;
  t.sp -= 1;
  t.nl = INFINITY;  // a popped node's exit is not kept (LDS: the stack's words are the walk's occupancy limit)
  uint32_t v = k.p[t.sp * k.stride];
  if (v == kNfRet) {
    const bool inst = (t.ret & kRetInstance) != 0;
    t.ret = kNoRet;
    if (inst) {  // a model shares the world ray (and its margin)
      t.r = world_ray(in, t.ray);
      nf_margin(in, t);
    }
    if (t.sp == 0) return false;
    t.sp -= 1;
    v = k.p[t.sp * k.stride];
  }
  t.i = v;
  return true;
}
MRT_DEV uint32_t vnf_entry(const DevScene& S, uint32_t base, uint32_t id, uint32_t word) {
  return S.vnf_leaf[2 * (size_t)MRT_IDX(S, S.vnf_base[base] + id, S.n_vnf, 23) + word];
}
// the reference's order of primitive occurrence (prim, ret): {world key, BLAS key}
MRT_DEV unsigned long long nf_key(const TravIn& in, uint32_t prim, uint32_t ret) {
  const DevScene& S = in.S;
  const uint32_t kind = prim >> 28, id = prim & 0x0FFFFFFFu;
  if (kind == MRT_REF_SPHERE) return (unsigned long long)vnf_entry(S, VNF_SPHERE, id, 1) << 32;
  const uint32_t k = vnf_entry(S, VNF_TRI, id, 1);
  if (k & kWorldKey) return (unsigned long long)(k & ~kWorldKey) << 32;
  const uint32_t rec = (ret & ~kRetInstance) - 2;  // the NF instance/model record (layout.h)
  const uint32_t cid = in.slots[MRT_IDX(S, rec, S.n_slots, 24)].x;
  const uint32_t wk = vnf_entry(S, (ret & kRetInstance) ? VNF_INST : VNF_MODEL, cid, 1);
  return ((unsigned long long)wk << 32) | k;
}
// does a hit (th, prim, current ret) replace the best so far? (t_max is
// inclusive in the reference: an equal t goes to the later primitive)
MRT_DEV bool nf_better(const TravIn& in, const Trav& t, float th, uint32_t prim) {
  if (th < t.best) return true;
  if (!(th == t.best)) return false;
  if (t.prim == kRefNone) return true;
  return nf_key(in, prim, t.ret) > nf_key(in, t.prim, t.hit_ret);
}
// a hit at th (<= the culling bound): the new best, or one of the other hits (t2)
// (selects; the tie's key comparison, which loads, is the only branch)
MRT_DEV void nf_hit(const TravIn& in, Trav& t, float th, uint32_t prim) {
  bool better = th < t.best;
  if (th == t.best) better = nf_better(in, t, th, prim);
  t.t2 = vmin1(t.t2, better ? t.best : th);
  t.best = better ? th : t.best;
  t.prim = better ? prim : t.prim;
  t.hit_ret = better ? t.ret : t.hit_ret;
  // a nearer bound: a smaller cap (the line stays valid below it)
  t.nfl.rcb = better ? nf_rho_node(t.nfl, nf_cull(th)) : t.nfl.rcb;
}
// the walk is over: k_trace checks the hit once per loop iteration (nf_finish);
// until then the lane holds an END record, never a box (the box-run ballot)
MRT_DEV void nf_over(Trav& t) {
  t.sp = kNfDone;
  t.s1.w = KIND_END;
}

// The reference's box test of reference record `rec` (a box) at t_max = t.
MRT_DEV bool ref_box_hits(const TravIn& in, uint32_t rec, const TRay& r, float t) {
  uint4 a, b;
  rec_load2<false>(in, rec, a, b);
  return box_hit_any(V3{u2f(a.x), u2f(a.y), u2f(a.z)}, V3{u2f(a.w), u2f(b.x), u2f(b.y)}, r, in.tmin, t);
}

// The near-first walk is over: does the reference's left-first walk reach
// the winner? The reference enters an ancestor box B of the winner iff
// BoundingBox::hit(B, t_max) holds for its t_max when it gets there, which is
// the smallest t of the hits it accepted BEFORE B — other hits than the
// winner, so at least tau = min(t2, best * (1 + 2^-10)) (t2: the other hits
// this walk met; any hit it did not meet lies beyond the culling margin).
// BoundingBox::hit is monotone in t_max, so B passing at tau suffices; the
// reference's boxes are nested, so the winner's world parent (world ray) and,
// inside a BLAS, its BLAS parent (that space's ray) stand for all of them.
// Yes: the ray is done (its record set to END for k_trace's box-run ballot).
// No: the reference's walk from the start (kExactMode).
template <bool COUNT>
MRT_DEV void nf_finish(const TravIn& in, Trav& t, LocalCounters& lc) {
  const DevScene& S = in.S;
  bool ok = true;
  const float tau = fminf(t.t2, nf_cull(t.best));
#ifdef MRT_PROBE_NF_NOCHECK  // measurement build only: the winner is not checked (NOT exact)
  if (false) {
#else
  if (t.prim != kRefNone) {
#endif
    const uint32_t kind = t.prim >> 28, id = t.prim & 0x0FFFFFFFu;
    const uint32_t own = vnf_entry(S, kind == MRT_REF_SPHERE ? VNF_SPHERE : VNF_TRI, id, 0);
    if (t.hit_ret == kNoRet) {  // a world object (t.r is the world ray: every BLAS was left)
      if (own != kNoParent) ok = ref_box_hits(in, own, t.r, tau);
    } else {
      const bool inst = (t.hit_ret & kRetInstance) != 0;
      // the NF instance/model record holds its id and its reference world
      // parent (layout.h): one load pair, not id -> vnf_leaf -> parent
      uint4 ra, rb;
      rec_load2<false>(in, (t.hit_ret & ~kRetInstance) - 2, ra, rb);
      const uint32_t cid = ra.x, wpar = rb.x;
      if (wpar != kNoParent) ok = ref_box_hits(in, wpar, t.r, tau);
      if (ok && own != kNoParent) {
        TRay r = t.r;
        if (inst) {
          V3 c0, c1, c2, c3;
          load_m12(S.inst_inv + (size_t)MRT_IDX(S, cid, S.n_inst, 8) * 12, c0, c1, c2, c3);
          r = make_tray(xform(c0, c1, c2, c3, t.r.o, 1.0f), xform(c0, c1, c2, c3, t.r.d, 0.0f), S.fast_ok);
        }
        ok = ref_box_hits(in, own, r, tau);
      }
      if (COUNT) lc.node_visits += 1;
    }
    if (COUNT) lc.node_visits += 1;
  }
  if (ok) {
    t.done = true;
    t.s1.w = KIND_END;  // a done lane holds an END record (k_trace's box-run ballot)
    return;
  }
  if (COUNT) lc.vnf_fallbacks++;
  t.sp = kExactMode;  // the reference's walk (the caller fetches t.i)
  t.i = in.world_begin;
  t.ret = kNoRet;
  t.best = in.tmax0;
  t.prim = kRefNone;
  t.hit_ret = kNoRet;
}

// Both children's boxes of an NF node (layout.h NF NODE) against [tmin,
// tmax], each thickened by rho = nfm (nf_bound.h): hit[c] unless the box is
// certainly missed, ent[c] its entry t. Fast rays: plane t = q * (2^e * y) +
// (o * y - oy) -/+ rho * y — 2^e * y is exact, so the error against (plane -/+
// rho - o_ray) / d adds the node's |o * y - oy -/+ rho * y| term to the early
// decision's margin (box_hit_any; rho carries a 2^-20 excess for the
// rounding of rho * y against rho / d) — and only a certain miss counts as
// one: the walk's boxes may be loose (its hits are checked against the
// reference tree), never tight. Other rays: the exact test on the decoded
// planes moved out by rho and widened by an ulp. A child whose force bit is
// set (kNfForceL/R: a wild instance below, nf_bound.h NfWild) is never culled
// here; the wild instance's own leaf test decides (trav_prim_index_nf).
MRT_DEV void nf_node_test(const uint4& s0, const uint4& s1, const TRay& r, float tmin, float tmax, float nfm, bool hit[2],
                          float ent[2], float ex[2]) {
  const V3 o{u2f(s0.x), u2f(s0.y), u2f(s0.z)};
  const V3 sc{__uint_as_float((s0.w & 0xFFu) << 23), __uint_as_float(((s0.w >> 8) & 0xFFu) << 23),
              __uint_as_float(((s0.w >> 16) & 0xFFu) << 23)};
  const uint32_t qw[3] = {s1.x, s1.y, s1.z};
  auto q = [&](int j) { return (float)((qw[j >> 2] >> (8 * (j & 3))) & 0xFFu); };  // v_cvt_f32_ubyteN
  // both paths leave floats only (entry, entry - exit, margin, exit bound):
  // the hit flags are formed after the merge, so no lane mask is carried
  // across it in vector registers
  float t0[2], dt[2], m[2], xb[2];
  if (tray_fast(r)) {
    const float ax = sc.x * r.yx, ay = sc.y * r.yy, az = sc.z * r.yz;
    const float bx = fmaf(o.x, r.yx, -r.oyx), by = fmaf(o.y, r.yy, -r.oyy), bz = fmaf(o.z, r.yz, -r.oyz);
    const float lbx = fmaf(-nfm, r.yx, bx), lby = fmaf(-nfm, r.yy, by), lbz = fmaf(-nfm, r.yz, bz);
    const float hbx = fmaf(nfm, r.yx, bx), hby = fmaf(nfm, r.yy, by), hbz = fmaf(nfm, r.yz, bz);
    const float mabs = fmaf(vmax3ab(lbx, lby, vmax3ab(lbz, hbx, vmax3ab(hby, hbz, 0.0f))), 0x1p-20f, fabsf(r.om));
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int b = 6 * c;
      const float lx = fmaf(q(b), ax, lbx), ly = fmaf(q(b + 1), ay, lby), lz = fmaf(q(b + 2), az, lbz);
      const float hx = fmaf(q(b + 3), ax, hbx), hy = fmaf(q(b + 4), ay, hby), hz = fmaf(q(b + 5), az, hbz);
      t0[c] = vmax3(vmin1(lx, hx), vmin1(ly, hy), vmax1(vmin1(lz, hz), tmin));
      const float t1 = vmin3(vmax1(lx, hx), vmax1(ly, hy), vmin1(vmax1(lz, hz), tmax));
      m[c] = fmaf(fabsf(t0[c]) + fabsf(t1), 0x1p-19f, mabs);
      dt[c] = t0[c] - t1;
      // every hit in the thickened box has t <= this (m covers t1's error and this rounding)
      xb[c] = fmaf(m[c], 2.0f, t1);
    }
  } else {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int b = 6 * c;
      auto lo = [&](float qq, float s, float org) {
        const float p = fmaf(qq, s, org) - nfm;
        return p - fmaf(fabsf(p), 0x1p-23f, 0x1p-140f);
      };
      auto hi = [&](float qq, float s, float org) {
        const float p = fmaf(qq, s, org) + nfm;
        return p + fmaf(fabsf(p), 0x1p-23f, 0x1p-140f);
      };
      const V3 mn{lo(q(b), sc.x, o.x), lo(q(b + 1), sc.y, o.y), lo(q(b + 2), sc.z, o.z)};
      const V3 mx{hi(q(b + 3), sc.x, o.x), hi(q(b + 4), sc.y, o.y), hi(q(b + 5), sc.z, o.z)};
      const V3 a = (mn - r.o) / r.d, bb = (mx - r.o) / r.d;  // IEEE quotients (the planes may lie outside the qfast domain)
      t0[c] = vmax3(vmin1(a.x, bb.x), vmin1(a.y, bb.y), vmax1(vmin1(a.z, bb.z), tmin));
      const float t1 = vmin3(vmax1(a.x, bb.x), vmax1(a.y, bb.y), vmin1(vmax1(a.z, bb.z), tmax));
      dt[c] = t0[c] - t1;  // > 0 exactly when t1 < t0 (+-inf pairs: NaN, a hit as !(t1 < t0))
      m[c] = 0.0f;
      xb[c] = INFINITY;  // no exit bound from the exact quotients
    }
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const bool force = (s1.w & (kNfForceL << c)) != 0;
    hit[c] = !(dt[c] > m[c]) || force;
    ent[c] = t0[c];
    // a forced child holds a wild instance, whose hits the world margin does
    // not place inside the box: no exit bound below it
    ex[c] = force ? INFINITY : xb[c];
  }
}

// The current record is an NF node: both children's boxes tested (culling at
// best * (1 + 2^-10)); both hit: the nearer next, the other pushed; one: that
// one; none: the stack's next.
template <bool COUNT>
MRT_DEV void trav_box_index_nf(const TravIn& in, const NfStack& k, Trav& t, LocalCounters& lc) {
  if (COUNT) lc.node_visits += 2;
  bool h[2];
  float e[2], x[2];
  // the hits this node must keep have t <= min(cull(best), nl)
  const float cb = nf_cull(t.best);
#ifdef MRT_PROBE_NF_ZERO_RHO  // measurement build only: no rounding margin (NOT exact)
  const float rho = 0.0f;
#elif defined(MRT_PROBE_NF_NOCONE)  // measurement build only: the ray's generic term everywhere (exact, looser)
  const float rho = nf_rho_node(t.nfl, fminf(cb, t.nl));
#else
  // the node's normal cone narrows the generic-triangle term (nf_bound.h
  // nf_cone_rg); scenes without generic triangles (kc == 0) skip it
  // (the cones only while some lane's worst-case generic term is worth it:
  // a wave-uniform choice, either rho is valid)
  const float tn = vmin1(cb, t.nl);
  float rho = nf_rho_node(t.nfl, tn);
  if (in.S.nfb.kc > 0.0f && __builtin_amdgcn_ballot_w64(t.nfl.rg * tn > in.S.nfb.kcmin) != 0)
    rho = nf_rho_cone(t.nfl, tn, t.s0.x, t.s0.y, t.s0.z, t.s0.w, t.r.d);
#endif
  nf_node_test(t.s0, t.s1, t.r, in.tmin, cb, rho, h, e, x);
  const uint32_t base = t.s1.w & kNfIdx, right = base + 2u + ((t.s0.w >> 24) & 1u);  // lsz - 2 in bit 24 (layout.h)
  // selects for the next record and its exit bound, the push and the pop as
  // the only branches (the left child when it is hit and nearer, or alone)
  const bool left = h[0] && (!h[1] || !(e[1] < e[0]));
  t.i = left ? base : right;
  t.nl = left ? x[0] : x[1];
  if (h[0] && h[1]) nf_push(k, t, left ? right : base);
  if (!(h[0] || h[1]) && !nf_pop(in, k, t)) nf_over(t);
}

// A wild instance's leaf record (slot0.w: its WILD entry, layout.h): does the
// world ray meet its world box thickened by its own margin at [tmin,
// cull(best)]? (nf_bound.h NfWild; the nodes above it never cull it)
MRT_DEV bool nf_wild_enter(const TravIn& in, const Trav& t, uint32_t at) {
  const uint4 a = rec_load1<false>(in, at), b = rec_load1<false>(in, at + 1), c = rec_load1<false>(in, at + 2),
              e = rec_load1<false>(in, at + 3);
  const NfWild x{{u2f(a.x), u2f(a.y), u2f(a.z)}, {u2f(a.w), u2f(b.x), u2f(b.y)}, u2f(b.z), u2f(b.w), u2f(c.x), u2f(c.y),
                 {u2f(c.z), u2f(c.w), u2f(e.x)}, u2f(e.y)};
  return nf_wild_hit(x, t.r.o, t.r.d, t.r.a.b, in.tmin, nf_cull(t.best));
}

// The current record is an NF leaf's primitive, instance or model.
template <bool COUNT, uint32_t ALPHA>
MRT_DEV void trav_prim_index_nf(const TravIn& in, const NfStack& k, Trav& t, LocalCounters& lc) {
  const DevScene& S = in.S;
  const uint4 s0 = t.s0, s1 = t.s1;
  const uint32_t kind = s1.w;
  uint32_t next;
  if (kind == KIND_TRI) {
    if (COUNT) lc.triangle_tests++;
    const uint4 s2 = rec_load1<false>(in, t.i + 2);
    V3 a{u2f(s0.x), u2f(s0.y), u2f(s0.z)}, ab{u2f(s0.w), u2f(s1.x), u2f(s1.y)}, ac{u2f(s2.x), u2f(s2.y), u2f(s2.z)};
    float th;
    // tested up to the culling bound: hits beyond `best` are recorded in t2
    if (tri_hit_nb(a, ab, ac, t.r.o, t.r.d, in.tmin, nf_cull(t.best), th)) {
      const uint32_t id = s1.z & kTriIdMask;
      if (!ALPHA || !(s1.z & kTriAlpha) || tri_alpha_pass<false, ALPHA == 2>(S, id, t.r.o, t.r.d, th, t.rng, lc))
        nf_hit(in, t, th, make_ref(MRT_REF_TRIANGLE, id));
    }
    next = s2.w;
  } else if (kind == KIND_SPHERE) {
    if (COUNT) lc.sphere_tests++;
    float th;
    if (sphere_hit(V3{u2f(s0.x), u2f(s0.y), u2f(s0.z)}, u2f(s0.w), t.r.o, t.r.d, t.r.a, in.tmin, nf_cull(t.best), th))
      nf_hit(in, t, th, make_ref(MRT_REF_SPHERE, s1.x));
    next = s1.y;
  } else if (kind == KIND_INST && s0.w != 0 && !nf_wild_enter(in, t, s0.w)) {
    next = s0.z;  // a wild instance the ray passes by (its own box and margin)
  } else {  // KIND_INST / KIND_MODEL: enter its BLAS, come back to the leaf's next record
    if (s0.z != kNfPop) nf_push(k, t, s0.z);
    nf_push(k, t, kNfRet);
    if (kind == KIND_INST) {
      if (COUNT) lc.instance_entries++;
      V3 c0, c1, c2, c3;
      load_m12(S.inst_inv + (size_t)MRT_IDX(S, s0.x, S.n_inst, 8) * 12, c0, c1, c2, c3);
      t.r = make_tray(xform(c0, c1, c2, c3, t.r.o, 1.0f), xform(c0, c1, c2, c3, t.r.d, 0.0f), S.fast_ok);
      t.ret = (t.i + 2) | kRetInstance;
      nf_margin(in, t);  // the object space's margin
    } else {
      if (COUNT) lc.model_entries++;
      t.ret = t.i + 2;
    }
    t.i = s0.y;
    return;
  }
  t.i = next;
  if (next == kNfPop && !nf_pop(in, k, t)) nf_over(t);
}

// Whole traversal of pool ray `ray` (one ray per thread); RNG: the
// traversal's draws come from (and advance) `rng`.
template <bool COUNT, bool RNG = false, bool EXT = false>
MRT_DEV Hit closest_hit(const TravIn& in, uint32_t ray, float tmax, LocalCounters& lc, PathRng& rng) {
  Trav t;
  trav_init(in, t, ray, tmax);
  if (RNG) t.rng = rng;
  while (!t.done) {
    if (trav_at_box(t))
      trav_box<COUNT>(in, t, lc);
    else
      trav_prim<COUNT, EXT ? 2u : 1u, RNG>(in, t, lc);
  }
  if (RNG) rng = t.rng;
  return trav_hit(in, t);
}

// Hit record of the closest hit, computed the way the reference's winning
// intersect computed it (geom.rs:77-91,535-584,405-419,318-326).
struct Surf {
  V3 point, normal;
  V2 uv;
  bool has_uv, front_face;
  uint32_t material;
};

MRT_DEV Surf resolve_hit(const DevScene& S, V3 o, V3 d, const Hit& h) {
  Surf s;
  V3 ro = o, rd = d;
  const uint32_t ckind = h.container >> 28, cidx = h.container & 0x0FFFFFFFu;
  V3 f0, f1, f2, f3;
  if (ckind == MRT_REF_INSTANCE) {
    V3 c0, c1, c2, c3;
    load_m12(S.inst_inv + (size_t)MRT_IDX(S, cidx, S.n_inst, 9) * 12, c0, c1, c2, c3);
    ro = xform(c0, c1, c2, c3, o, 1.0f);
    rd = xform(c0, c1, c2, c3, d, 0.0f);
  }
  const uint32_t pkind = h.prim >> 28, pidx = h.prim & 0x0FFFFFFFu;
  V3 outward;
  s.point = ro + rd * h.t;
  if (pkind == MRT_REF_VOLUME) {  // geom.rs:644-651: fixed normal, front face, no uv
    s.normal = V3{1.0f, 0.0f, 0.0f};
    s.front_face = true;
    s.has_uv = false;
    s.uv = V2{0, 0};
    s.material = S.vol_mat[MRT_IDX(S, pidx, S.n_vol, 16)];
    return s;  // volumes are World objects: no container
  }
  if (pkind == MRT_REF_SPHERE) {
    const uint32_t sp = MRT_IDX(S, pidx, S.n_sph, 10);
    V3 c = ld3(S.sph + (size_t)sp * 4);
    float r = S.sph[(size_t)sp * 4 + 3];
    outward = (s.point - c) / r;
    s.has_uv = false;
    s.uv = V2{0, 0};
    s.material = S.sph_mat[sp];
  } else {
    TriShade t = load_tri(S, pidx);
    float a0, a1, a2;
    tri_bary(t, s.point, a0, a1, a2);
    outward = (t.na * a0 + t.nb * a1) + t.nc * a2;
    s.has_uv = (t.flags & TRI_FLAG_UV) != 0;
    s.uv = uv_or_zero(s.has_uv, (t.uva * a0 + t.uvb * a1) + t.uvc * a2);
    s.material = t.material;
  }
  // Hit::set_face_normal in the intersecting (object) space (geom.rs:17-24)
  s.front_face = dot(rd, outward) < 0.0f;
  s.normal = s.front_face ? outward : -outward;
  if (ckind == MRT_REF_INSTANCE) {
    load_m12(S.inst_fwd + (size_t)MRT_IDX(S, cidx, S.n_inst, 11) * 12, f0, f1, f2, f3);
    s.point = xform(f0, f1, f2, f3, s.point, 1.0f);
    s.normal = unit(xform(f0, f1, f2, f3, s.normal, 0.0f));
    uint32_t m = S.inst_mat[MRT_IDX(S, cidx, S.n_inst, 12)];
    if (m != MRT_NO_MATERIAL) s.material = m;
  } else if (ckind == MRT_REF_MODEL) {
    uint32_t m = S.model_mat[MRT_IDX(S, cidx, S.n_models, 13)];
    if (m != MRT_NO_MATERIAL) s.material = m;
  }
  return s;
}

// ---- sampling (math.rs:262-291) -----------------------------------------------
MRT_DEV V3 random_in_unit_sphere(PathRng& rng) {
  for (;;) {
    float x = rng.f32() * 2.0f - 1.0f;
    float y = rng.f32() * 2.0f - 1.0f;
    float z = rng.f32() * 2.0f - 1.0f;
    V3 v{x, y, z};
    if (length_squared(v) >= 1.0f) continue;
    return v;
  }
}
MRT_DEV V3 random_in_unit_disk(PathRng& rng) {
  for (;;) {
    float x = rng.f32() * 2.0f - 1.0f;
    float y = rng.f32() * 2.0f - 1.0f;
    V3 v{x, y, 0.0f};
    if (length_squared(v) >= 1.0f) continue;
    return v;
  }
}

// Dielectric::reflectance (material.rs:296-299); powi(5) = x*((x*x)*(x*x))
MRT_DEV float reflectance(float cosine, float ref_idx) {
  float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
  r0 = r0 * r0;
  float x = 1.0f - cosine;
  return r0 + (1.0f - r0) * (x * ((x * x) * (x * x)));
}

struct DevCamera {
  V3 origin, llc, horizontal, vertical, u, v;
  float lens_radius;
};

// main.rs:258-260 + Camera::ray (world.rs:53-63)
// Camera::ray (world.rs:53-63) through (u, v)
MRT_DEV void camera_ray_uv(const DevCamera& cam, float u, float v, PathRng& rng, V3& o, V3& d) {
  V3 blur = random_in_unit_disk(rng) * cam.lens_radius;
  V3 offset = cam.u * blur.x + cam.v * blur.y;
  o = cam.origin + offset;
  d = (((cam.llc + (cam.horizontal * u)) + (cam.vertical * v)) - cam.origin) - offset;
}

// the jittered sample ray of pixel (x, y) (main.rs:258-260)
MRT_DEV void camera_ray(const DevCamera& cam, uint32_t x, uint32_t y, uint32_t W, uint32_t H, PathRng& rng, V3& o,
                        V3& d) {
  float u = ((float)x + rng.f32()) / (float)(W - 1);
  float v = ((float)y + rng.f32()) / (float)(H - 1);
  camera_ray_uv(cam, u, v, rng, o, d);
}

template <bool EXT>
MRT_DEV V3 background(const DevScene& S, V3 d, LocalCounters& lc) {
  if (S.bg_kind == MRT_BG_SOLID) return V3{S.bg_color[0], S.bg_color[1], S.bg_color[2]};
  if (S.bg_kind == MRT_BG_SKY) {
    V3 ud = unit(d);
    float t = 0.5f * (ud.y + 1.0f);
    return (fill3(1.0f) * (1.0f - t)) + (V3{0.5f, 0.7f, 1.0f} * t);
  }
  V2 uv{0.0f, 0.0f};
  uint32_t face = 0;
  if (!EXT || S.bg_kind == MRT_BG_SKYSPHERE) {
    V3 p = unit(d);
    float theta = acosf(p.y);
    float phi = atan2f(p.z * -1.0f, p.x) + kPi;
    uv = V2{phi / (2.0f * kPi), theta / kPi};
  } else if (EXT) {  // CubeMap::background (material.rs:122-189); y faces swapped as in the reference
    const float* mf = S.bg_m;
    const M4 m{V4{mf[0], mf[1], mf[2], mf[3]}, V4{mf[4], mf[5], mf[6], mf[7]}, V4{mf[8], mf[9], mf[10], mf[11]},
               V4{mf[12], mf[13], mf[14], mf[15]}};
    V3 p = transform(m, d, 0.0f);
    V3 a{fabsf(p.x), fabsf(p.y), fabsf(p.z)};
    float max_axis = 0.0f, u = 0.0f, v = 0.0f;
    if (a.x >= a.y && a.x >= a.z) {
      if (p.x > 0.0f) face = 0, u = p.z * -1.0f, v = p.y;
      else face = 1, u = p.z, v = p.y;
      max_axis = a.x;
    } else if (a.y >= a.x && a.y >= a.z) {
      if (p.y > 0.0f) face = 3, u = p.x, v = p.z * -1.0f;
      else face = 2, u = p.x, v = p.z;
      max_axis = a.y;
    } else if (a.z >= a.x && a.z >= a.y) {
      if (p.z > 0.0f) face = 4, u = p.x, v = p.y;
      else face = 5, u = p.x * -1.0f, v = p.y;
      max_axis = a.z;
    }
    uv = V2{0.5f * (u / max_axis + 1.0f), 0.5f * (v / max_axis + 1.0f)};
  }
  const GpuSurfRef f = S.bg_faces[face];
  V4 px = surface_ref_get_f<EXT>(S, f.kind, f.index, f.len, f.color, uv, lc);
  return V3{px.x, px.y, px.z};
}

// Hit::emit + Hit::scatter (geom.rs:26-32). Returns true when the path
// continues with (new_o, new_d) and attenuation `atten`.
// Mix::scatter/emit/alpha_test (material.rs:402-424): every call draws once
// to pick a side, recursively; children precede their Mix in the table.
MRT_DEV uint32_t mix_pick(const DevScene& S, uint32_t mi, PathRng& rng) {
  for (;;) {
    const GpuMaterial m = S.materials[MRT_IDX(S, mi, S.n_materials, 4)];
    if (m.kind != MRT_MAT_MIX) return mi;
    mi = rng.f32() < m.param ? m.left : m.right;
  }
}

// Lambertian::scatter (material.rs:203-215)
template <bool EXT>
MRT_DEV void lambertian(const DevScene& S, const GpuMaterial& m, const Surf& s, PathRng& rng, V3& atten, V3& new_d,
                        LocalCounters& lc) {
  V3 dir = s.normal + unit(random_in_unit_sphere(rng));
  if (near_zero(dir)) dir = s.normal;
  V4 c = surface_get_f<EXT>(S, m, uv_or_zero(s.has_uv, s.uv), lc);
  atten = V3{c.x, c.y, c.z};
  new_d = dir;
}

// Hit::emit then Hit::scatter (world.rs:69-70), in that order of RNG draws.
template <bool EXT>
MRT_DEV bool scatter(const DevScene& S, const Surf& s, V3 d, PathRng& rng, V3& emitted, V3& atten, V3& new_d,
                     LocalCounters& lc) {
  emitted = V3{0, 0, 0};
  {
    const GpuMaterial e = S.materials[mix_pick(S, s.material, rng)];
    if (e.kind == MRT_MAT_DIFFUSE_LIGHT) emitted = V3{e.color[0], e.color[1], e.color[2]};
  }
  const GpuMaterial m = S.materials[mix_pick(S, s.material, rng)];
  V2 uv = uv_or_zero(s.has_uv, s.uv);
  switch (m.kind) {
    case MRT_MAT_LAMBERTIAN:
      lambertian<EXT>(S, m, s, rng, atten, new_d, lc);
      return true;
    case MRT_MAT_METAL: {
      V3 reflected = reflect(unit(d), s.normal);
      V3 dir = reflected + (random_in_unit_sphere(rng) * m.param);
      if (dot(dir, s.normal) > 0.0f) {
        V4 c = surface_get_f<EXT>(S, m, uv, lc);
        atten = V3{c.x, c.y, c.z};
        new_d = dir;
        return true;
      }
      return false;
    }
    case MRT_MAT_DIELECTRIC:
    case MRT_MAT_SPECULAR: {  // material.rs:299-328 / 355-377
      float ratio = s.front_face ? 1.0f / m.param : m.param;
      V3 ud = unit(d);
      float cos_theta = fminf(dot(-ud, s.normal), 1.0f);
      float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
      bool cannot_refract = ratio * sin_theta > 1.0f;
      if (cannot_refract || reflectance(cos_theta, ratio) > rng.f32()) {
        new_d = reflect(ud, s.normal);
      } else if (m.kind == MRT_MAT_SPECULAR) {
        lambertian<EXT>(S, m, s, rng, atten, new_d, lc);  // return self.inner.scatter(ray, hit)
        return true;
      } else {
        new_d = refract(ud, s.normal, ratio);
      }
      atten = fill3(1.0f);
      return true;
    }
    case MRT_MAT_ISOTROPHIC:  // material.rs:438-444: direction not normalised
      atten = V3{m.color[0], m.color[1], m.color[2]};
      new_d = random_in_unit_sphere(rng);
      return true;
    default:  // DiffuseLight, ()
      return false;
  }
}

}  // namespace mrt
