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
  // normal cones (round 6, nf_cone_rg below): the generic term per unit t is
  // at most kc |d|^2 2^k / (|d . c| - |d| chi) over a node whose generic
  // triangles' normals lie in the cone (c, chi) and whose |c| M <= 2^(k+6);
  // 0: the scene's trees carry no cones (no generic triangles)
  float kc;
  // a node's cone is evaluated only while some lane of the wave has a generic
  // term rg t above this (2^-6 of the median generic triangle's extent): a
  // bounce ray's short reach leaves the worst-case term small (path.h
  // trav_box_index_nf; either value is a valid rho)
  float kcmin;
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
// min of two arithmetic results (never a signalling NaN): on the device one
// v_min_f32 — fminf would first canonicalise each operand (v_max x, x), a
// per-node cost of the margin
MRT_HD float nf_min(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return fminf(a, b);
#endif
}

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
// The slope is kept in two parts, ra = ra0 + rg: rg is the generic
// triangles' term (gen |d|^2, gen = aw1 or ao1), which a node's normal cone
// may lower (nf_cone_rg); kd, dl and s128 are the ray's constants for that.
struct NfLine {
  float rcb, ra0, rg, rb;
  float kd;    // kc |d|^2 (rounded up)
  float dl;    // |d| (rounded up)
  float s128;  // 128 (d.x + d.y + d.z): the bias of the cone's stored components
};
// the line of a space whose margin per unit L is a0 + gen |d| (world: aw0,
// aw1; an instance's object space: ao0, ao1 — nf_coef_world / _object)
MRT_HD NfLine nf_line(const NfBound& B, const NfCoef& c, float cb, float a0, float gen, float d2, V3 d) {
  const float k = fmaf(B.s51, fminf(c.dl * cb, c.ls) + c.delta, B.s130);  // the spheres' slope per unit L
  constexpr float up = 1.0f + 0x1p-16f;
  return NfLine{nf_rho_at(B, c, cb), fmaf(k, c.dl, a0 * c.dl) * up, (gen * c.dl) * c.dl * up,
                fmaf(k, c.delta, c.b) * up, B.kc * d2 * up, c.dl, 128.0f * ((d.x + d.y) + d.z)};
}
// (a nearer cull bound cb' < cb keeps the line and caps it at nf_rho_node(l, cb'))
MRT_HD float nf_rho_node(const NfLine& l, float t) { return nf_min(l.rcb, fmaf(l.ra0 + l.rg, t, l.rb)); }

// ---- normal cones (round 6; DESIGN.md §4 "Normal cones") ----
// The generic-triangle term comes from Moller-Trumbore's cancellation, which
// the reference bounds only by its absolute |det| >= 1e-6 test (geom.rs:511):
// priced that way, every ray pays for the worst direction and rho grows to
// ~3e-3 L for camera rays of the 1M-triangle mesh. But det = -d . N (N = ab x
// ac), so over a node whose triangles' normals lie in a cone about an integer
// vector c (|c| n_i within chord delta of c, each n_i up to sign):
//   |det_i| >= |ab_i||ac_i| (|d . c| - |d| chi) / (|c| m_i),  m_i = |ab||ac|/|N|
// where chi = |c| delta + 7.3u |c| M (the computed det's own error, M =
// max m_i) + 3000u (this evaluation's rounding) — so the term
// 24u |d| |ab||ac| / |det| <= 24u |c| M |d| / (|d . c| - |d| chi), and per
// unit t the node's generic slope is at most kd 2^k / (|d . c| - |d| chi)
// with |c| M <= 2^(k+6) (kc = 24.01u / (1 - kNfKappaMax), rounded up with the
// slack of rcp, ldexp and these roundings). Where the cone says nothing
// (a ray within the cone's grazing band: G <= 0) the node keeps rg.
// The node record carries c + 128 in the low byte of each origin word (an
// origin is any float at or below the children's minimum: nf_tree.cpp picks
// one with that byte) and, in bits 25-31 of slot0.w, j (chi = 2^(j - 3);
// j = 15: no cone) and k.
constexpr uint32_t kNfConeNone = 15u;  // j of a node without a cone (chi = 2^12 > any |c|)
MRT_HD float nf_cone_rg(const NfLine& l, uint32_t ox, uint32_t oy, uint32_t oz, uint32_t w, V3 d) {
  const float cx = (float)(ox & 0xFFu), cy = (float)(oy & 0xFFu), cz = (float)(oz & 0xFFu);  // c + 128
  const float dc = fabsf(fmaf(d.z, cz, fmaf(d.y, cy, fmaf(d.x, cx, -l.s128))));
  const uint32_t code = w >> 25;
  const float G = fmaf(-l.dl, ldexpf(1.0f, (int)(code & 15u) - 3), dc);
#if defined(__HIP_DEVICE_COMPILE__)
  const float rcp = __builtin_amdgcn_rcpf(fmaxf(G, 0x1p-100f));  // within an ulp: kc's slack
#else
  const float rcp = 1.0f / fmaxf(G, 0x1p-100f);
#endif
  return nf_min(l.rg, ldexpf(l.kd, (int)(code >> 4)) * rcp);
}
// rho of a node (record words o.x, o.y, o.z, w) for hits at t or before
MRT_HD float nf_rho_cone(const NfLine& l, float t, uint32_t ox, uint32_t oy, uint32_t oz, uint32_t w, V3 d) {
  return nf_min(l.rcb, fmaf(l.ra0 + nf_cone_rg(l, ox, oy, oz, w, d), t, l.rb));
}

// ---- wild instances (round 6; DESIGN.md §4 "Wild instances") ----
// An instance whose rounding terms would dominate the world margin — a thin
// light box (cond = |F||G| ~ 1.4e4: A ~ 0.047 per unit L), a 1000x floor (an
// absolute term ~4e-4) — or any instance of a world with few of them
// (kNfWildFew) stays out of the world margin (aw*, bw*). The nodes above it
// never cull it (kNfForceL/R); its leaf record points at a WILD entry (layout.h)
// holding its world box and its own instance term (nf_tree.cpp inst_term, the
// bound of every instance): its hits lie within
//   rho_x(t) = A min(|d| t, 2.5 (|o - c| + r + b)) + b,  A = a0 + a1 |d|,  b = b0 + b1 |o|
// of that box ((c, r): a ball holding the box; a hit X has L = |X - o| <=
// |o - c| + r + A L + b, so L <= 2.5 (...) while A <= 0.6), so the walk enters
// it only if the ray meets the box thickened by rho_x(cull(best)) — after the
// rest of the world has set `best`, a floor behind the mesh or a light the ray
// passes far from costs one box test instead of a transform and a BLAS walk.
// A > 0.6 (no cap) or no finite value: +inf (entered).
struct NfWild {
  float mn[3], mx[3];  // the instance's world box (nf_tree.cpp object_box)
  float a0, a1, b0, b1;
  float c[3], r;
};
MRT_HD float nf_rho_wild(const NfWild& x, V3 o, float d2, float t) {
  const float dl = nf_sqrt_up(d2);
  const float A = x.a0 + x.a1 * dl;
  if (!(A <= 0.6f)) return INFINITY;
  const float b = x.b0 + x.b1 * nf_len(o);
  const float dist = nf_len(V3{o.x - x.c[0], o.y - x.c[1], o.z - x.c[2]}) + x.r;
  const float r = fmaf(A, fminf(dl * t, 2.5f * (dist + b)), b) * (1.0f + 0x1p-16f);
  return r <= 0x1p100f ? r : INFINITY;  // NaN (an infinite origin) or huge: entered
}
// Does the ray (o, d) meet the wild box thickened by rho = nf_rho_wild(x, o,
// |d|^2, tmax) at some t in [tmin, tmax]? Planes moved out by rho and by an
// ulp (the rounding of plane -/+ rho), IEEE quotients (plane - o) / d, each
// entry lowered and exit raised by 2^-21 relative (the subtraction's and the
// division's roundings, 2.01u, with slack) plus 2^-140 (underflow); a
// direction component of zero: the slab holds all t or none. False only for
// a certain miss.
MRT_HD bool nf_wild_hit(const NfWild& x, V3 o, V3 d, float d2, float tmin, float tmax) {
  const float rho = nf_rho_wild(x, o, d2, tmax);
  if (!(rho < INFINITY)) return true;
  float t0 = tmin, t1 = tmax;
  const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
  for (int k = 0; k < 3; ++k) {
    float pl = x.mn[k] - rho, ph = x.mx[k] + rho;
    pl -= fmaf(fabsf(pl), 0x1p-23f, 0x1p-140f);
    ph += fmaf(fabsf(ph), 0x1p-23f, 0x1p-140f);
    float en, ex;
    if (dd[k] == 0.0f) {
      const bool in = pl <= oo[k] && oo[k] <= ph;
      en = in ? -INFINITY : INFINITY;
      ex = in ? INFINITY : -INFINITY;
    } else {
      const float a = (pl - oo[k]) / dd[k], b = (ph - oo[k]) / dd[k];
      en = fminf(a, b);
      ex = fmaxf(a, b);
      en -= fmaf(fabsf(en), 0x1p-21f, 0x1p-140f);
      ex += fmaf(fabsf(ex), 0x1p-21f, 0x1p-140f);
    }
    t0 = fmaxf(t0, en);
    t1 = fminf(t1, ex);
  }
  return !(t1 < t0);
}

}  // namespace mrt
