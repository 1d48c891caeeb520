// nf_bound.h — how far outside its own box a primitive's COMPUTED hit point
// can lie, as a margin the near-first walk's box tests add (DESIGN.md §4,
// "Why the near-first walk is exact"). Shared by the device walk (path.h), the
// host tree builder that derives the constants (nf_tree.cpp) and the host
// restatement that checks them (tools/slab_check.cpp).
//
// The walk culls a box when the ray's slab interval [t0, t1] misses
// [tmin, cull(best)]. That is safe for a primitive P inside the box if P's
// computed hit X = o + t*d (t: the reference's own f32 arithmetic,
// geom.rs:56-93, 504-533) lies in the box thickened by rho: the slab interval
// of the thickened box contains t. Thickening moves each slab plane by
// rho / d_k = rho * y_k (y = RN(1/d); rho carries a 2^-20 excess for that
// rounding), which the walk's node test adds to the planes. rho depends on the
// distance L = |X - o| <= cull(best) * |d| (and, before any hit, at most a
// cap from a ball holding the primitives of its kind):
//   rho(L) = a0 L_w + a1 |d| L_g + B (+ the spheres' term),  B = b0 + b1 |o|
// (L_w, L_g: L capped by the world's ball and by the ball of the primitives
// whose term grows with |d| — generic triangles, directly or instanced)
// with per-scene constants from nf_tree.cpp; the parts proportional to a
// primitive's own size are padded onto its box on the host instead.
// Deeper in the tree the walk knows more: a node's hits have t <= nl, the
// exit of its (thickened) box computed at its parent, so a node is tested
// with rho at min(cull(best), nl).
#pragma once
#include <math.h>
#include <stdint.h>

#include "../mrt_math.h"

namespace mrt {

struct NfBound {
  // world space: world primitives, model triangles, non-"wild" instances
  float aw0, aw1;        // A = aw0 + aw1 |d|
  float bw0, bw1;        // B = bw0 + bw1 |o|
  float kw1, ko1;        // generic triangles' kappa per unit |d| (world; instances' object spaces via the world |d|)
  float wc[3], wr;       // a ball holding every world box (the L cap of the a0 term)
  float gc[3], gr;       // a ball holding the world boxes of every generic triangle (the a1 term's cap)
  float sc[3], sr;       // a ball holding every world sphere; sr < 0: no spheres
  float s51, s28, s130, s11;  // sphere terms: u 51.2 / r_min, u 27.8, u 130.2, u 11.2 r_max
  // object space of instances (every BLAS an instance enters)
  float ao0, ao1;        // A_o = ao0 + ao1 |d_obj|
  float orad;            // a ball about the origin holding every instanced BLAS's boxes
  float kmax;            // a ray walks near first only while its generic kappa is at most this (<= kNfKappaMax)
};

// The walk is run only when the generic-triangle kappa stays at most
// kNfKappaMax (the host pads assume it) and A at most kNfAMax; otherwise the
// ray takes the reference's walk from the start (always exact).
constexpr float kNfKappaMax = 0x1p-8f;
constexpr float kNfAMax = 0x1p-4f;


// A ray's rho as a function of t (the walk's bound on the t of the hits it
// must still meet: cull(best), or a node's exit): coefficients per ray and
// space, set when the walk enters a space (sqrt there only), evaluated per
// node test (nf_rho_at: a few multiply-adds).
//   rho(t) = min(a t, fc) + b + min(d0, (s51 L' + s130) L'),  L' = dl t + delta
// (the spheres' term; d0 = delta = 0 without spheres and in object space).
struct NfCoef {
  float a, fc, b, d0, dl, delta;
  float ls;  // a sphere hit lies within ls of o (2.5 ds; 0 without spheres)
};

// |v|^2's square root rounded up (the device's v_sqrt_f32 is within an ulp;
// 2^-18 is 64 ulps of slack), for the caps and |d| of the coefficients
MRT_HD float nf_sqrt_up(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_sqrtf(x) * (1.0f + 0x1p-18f);
#else
  return sqrtf(x) * (1.0f + 0x1p-18f);
#endif
}
MRT_HD float nf_len(V3 v) { return nf_sqrt_up((v.x * v.x + v.y * v.y) + v.z * v.z); }

// may this ray (world space, |d|^2 = d2) take the near-first walk?
MRT_HD bool nf_ray_ok(const NfBound& B, float d2) {
  const float dl = nf_sqrt_up(d2);
  return d2 >= 0x1p-100f && B.kw1 * dl <= B.kmax && B.ko1 * dl <= B.kmax && B.aw0 + B.aw1 * dl <= kNfAMax &&
         dl < INFINITY;
}

// The world-space coefficients of a ray (o, |d|^2 = d2): a generic or
// instance hit at t lies within L = |d| t of o and within 2.5 (dist + b) of it
// whatever t (dist: to the far side of the ball of its kind); a sphere hit
// within 2.5 ds. Evaluated in float with every input rounded
// up; nf_rho_at rounds its result up by 2^-16 (covering the rounding of
// this evaluation and of rho * y_k in the node test).
MRT_HD NfCoef nf_coef_world(const NfBound& B, V3 o, float d2) {
  const float dl = nf_sqrt_up(d2);
  const float b = B.bw0 + B.bw1 * nf_len(o);
  const float dw = nf_len(V3{o.x - B.wc[0], o.y - B.wc[1], o.z - B.wc[2]}) + B.wr;
  const float dg = nf_len(V3{o.x - B.gc[0], o.y - B.gc[1], o.z - B.gc[2]}) + B.gr;
  const float ag = B.aw1 * dl;
  NfCoef c{(B.aw0 + ag) * dl, B.aw0 * (2.5f * (dw + b)) + ag * (2.5f * (dg + b)), b, 0.0f, dl, 0.0f, 0.0f};
  if (B.sr >= 0.0f) {
    const float ds = nf_len(V3{o.x - B.sc[0], o.y - B.sc[1], o.z - B.sc[2]}) + B.sr;
    c.d0 = (B.s51 * ds) * ds + B.s28 * ds;  // any sphere hit: |o - c| <= ds
    c.delta = c.d0 + B.s11;
    c.ls = 2.5f * ds;
  }
  return c;
}
// an instance's object-space ray (o, |d|^2 = d2): its BLAS within orad of the origin
MRT_HD NfCoef nf_coef_object(const NfBound& B, V3 o, float d2) {
  const float dl = nf_sqrt_up(d2);
  const float A = B.ao0 + B.ao1 * dl;
  return NfCoef{A * dl, A * (1.25f * (nf_len(o) + 2.0f * B.orad)), 0.0f, 0.0f, dl, 0.0f, 0.0f};
}
// rho for the hits at t or before (t = +inf: every hit)
MRT_HD float nf_rho_at(const NfBound& B, const NfCoef& c, float t) {
  const float l = fmaf(c.dl, t, c.delta);
  const float s = fminf(c.d0, fmaf(B.s51, l, B.s130) * l);
  return ((fminf(c.a * t, c.fc) + c.b) + s) * (1.0f + 0x1p-16f);
}

// The per-node form for a walk culling at cb: rho(t) <= min(rho(cb), ra t + rb)
// for t <= cb (rho is monotone in t; the line drops the caps and takes the
// spheres' slope at min(cb |d|, ls), beyond which no sphere hit lies), so a
// node whose hits have t <= nl costs one fma and one min (nf_rho_node).
struct NfLine {
  float rcb, ra, rb;
};
MRT_HD NfLine nf_line(const NfBound& B, const NfCoef& c, float cb) {
  const float k = fmaf(B.s51, fminf(c.dl * cb, c.ls) + c.delta, B.s130);  // the spheres' slope per unit L
  constexpr float up = 1.0f + 0x1p-16f;
  return NfLine{nf_rho_at(B, c, cb), fmaf(k, c.dl, c.a) * up, fmaf(k, c.delta, c.b) * up};
}
// (a nearer cull bound cb' < cb keeps the line and caps it at nf_rho_node(l, cb'))
MRT_HD float nf_rho_node(const NfLine& l, float t) { return fminf(l.rcb, fmaf(l.ra, t, l.rb)); }

}  // namespace mrt
