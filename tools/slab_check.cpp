// slab_check — host-side restatement of k_trace's early slab decision
// (path.h make_tray / slab_fast / box_hit_any), run over the record stream of
// a built-in scene on camera rays and one-bounce rays, no GPU needed: every
// box the early decision settles must get the exact BoundingBox::hit answer
// (IEEE quotients, geom.rs:218-247), and the fraction left to the exact test
// is reported. Round 2 used it to find that mesh_ply's vertices at ~1e-16
// (sin(pi)) had switched the whole scene to the exact test.
//   g++ -O2 -std=c++17 -ffp-contract=off -o tools/slab_check tools/slab_check.cpp -Lmass-raytrace_amd/massrt
//       -lmassrt -Wl,-rpath,$PWD/mass-raytrace_amd/massrt && tools/slab_check mesh_ply 20000 assets
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "../mass-raytrace_amd/csrc/device/upload.h"

using namespace mrt;

namespace {

float f(uint32_t u) {
  float x;
  memcpy(&x, &u, 4);
  return x;
}
struct V {
  float x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
float dot(V a, V b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }

struct Ray {
  V o, d;
  float y[3], oy[3], om;
  bool fast;
};
bool dir_ok(float c) {
  float a = fabsf(c);
  return a >= 0x1p-20f && a <= 0x1p20f;
}
Ray make_ray(V o, V d, bool scene_fast) {
  Ray r{o, d, {}, {}, 0, false};
  const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
  float m = 0;
  for (int k = 0; k < 3; ++k) {
    r.y[k] = 1.0f / dd[k];
    r.oy[k] = oo[k] * r.y[k];
    m = std::max(m, fabsf(r.oy[k]));
  }
  r.om = std::max(m * 0x1p-20f, 0x1p-120f);
  // early-decision domain (path.h make_tray): finite origin within 2^28, |d| in [2^-20, 2^20]
  auto o_ok = [](float c) { return fabsf(c) <= 0x1p28f; };
  r.fast = scene_fast && o_ok(o.x) && o_ok(o.y) && o_ok(o.z) && dir_ok(d.x) && dir_ok(d.y) && dir_ok(d.z);
  return r;
}
// BoundingBox::hit with IEEE quotients (fminf/fmaxf = minNum/maxNum, as v_min/v_max)
bool box_exact(const float mn[3], const float mx[3], const Ray& r, float tmin, float tmax) {
  const float oo[3] = {r.o.x, r.o.y, r.o.z}, dd[3] = {r.d.x, r.d.y, r.d.z};
  float t0 = tmin, t1 = tmax;
  float a[3], b[3];
  for (int k = 0; k < 3; ++k) a[k] = (mn[k] - oo[k]) / dd[k], b[k] = (mx[k] - oo[k]) / dd[k];
  t0 = fmaxf(fmaxf(fminf(a[0], b[0]), fminf(a[1], b[1])), fmaxf(fminf(a[2], b[2]), tmin));
  t1 = fminf(fminf(fmaxf(a[0], b[0]), fmaxf(a[1], b[1])), fminf(fmaxf(a[2], b[2]), tmax));
  return !(t1 < t0);
}
float margin(const Ray& r, float t0, float t1) { return std::fma(fabsf(t0) + fabsf(t1), 0x1p-19f, r.om); }

struct Stats {
  uint64_t boxes = 0, undecided = 0, wrong = 0;
  uint64_t loads = 0;  // 16-B record loads (k_trace's vector-memory instructions per lane step)
  uint64_t entries = 0;  // instance entries (each: a transform, the object margin, the world ray back)
  uint64_t wild_skips = 0;  // wild instances passed by on their own box test
  uint64_t prims = 0;       // primitive tests
};
// path.h box_hit_any's early decision: 1 hit, 0 miss, -1 left to the exact test
int early_decide(const float mn[3], const float mx[3], const Ray& r, float tmin, float best) {
  if (!r.fast) return -1;
  float a[3], b[3];
  for (int k = 0; k < 3; ++k) a[k] = std::fma(mn[k], r.y[k], -r.oy[k]), b[k] = std::fma(mx[k], r.y[k], -r.oy[k]);
  const float t0 = fmaxf(fmaxf(fminf(a[0], b[0]), fminf(a[1], b[1])), fmaxf(fminf(a[2], b[2]), tmin));
  const float t1 = fminf(fminf(fmaxf(a[0], b[0]), fmaxf(a[1], b[1])), fminf(fmaxf(a[2], b[2]), best));
  const float m = margin(r, t0, t1), gap = t1 - t0;
  return gap > m ? 1 : (-gap > m ? 0 : -1);
}

bool sphere_hit(V c, float rad, V o, V d, float tmin, float tmax, float& t) {
  V oc = sub(o, c);
  float a = dot(d, d), hb = dot(oc, d), cc = dot(oc, oc) - rad * rad, disc = hb * hb - a * cc;
  if (disc < 0.0f) return false;
  float sq = sqrtf(disc), root = (-hb - sq) / a;
  if (root < tmin || tmax < root) {
    root = (-hb + sq) / a;
    if (root < tmin || tmax < root) return false;
  }
  t = root;
  return true;
}
bool tri_hit(V a, V ab, V ac, V o, V d, float tmin, float tmax, float& t) {
  V p = cross(d, ac);
  float det = dot(ab, p);
  if (fabsf(det) < 0.000001f) return false;
  float inv = 1.0f / det;
  V tv = sub(o, a);
  float u = dot(tv, p) * inv;
  if (u < 0.0f || u > 1.0f) return false;
  V qv = cross(tv, ab);
  float v = dot(d, qv) * inv;
  if (v < 0.0f || v + u > 1.0f) return false;
  float tt = dot(ac, qv) * inv;
  if (tt < tmin || tt > tmax) return false;
  t = tt;
  return true;
}
V xf(const float* m, V p, float w) {  // c0.xyz c1.xyz c2.xyz c3.xyz
  return {((m[0] * p.x + m[3] * p.y) + m[6] * p.z) + m[9] * w, ((m[1] * p.x + m[4] * p.y) + m[7] * p.z) + m[10] * w,
          ((m[2] * p.x + m[5] * p.y) + m[8] * p.z) + m[11] * w};
}

struct Result {
  uint32_t prim, container;
  float t;
};
const float kTmin = 0.001f;

// `bound` checks (nf_bound.h): every primitive test of the
// reference walk is repeated with t_max = inf; an accepted hit X = o + t d
// (exact, in double) must lie within rho(L = t |d|) of the primitive's NF leaf
// box in its own space, and an instance's hit within the world rho of the
// instance's world box (unless it is wild: never culled)
struct BoundCheck {
  uint64_t checks = 0, outside = 0, over = 0, wild_checks = 0;
  double worst = 0, worst_cap = 0, worst_wild = 0;  // max dist / rho, max L / L_cap, the wild margin's max dist / rho
};
BoundCheck* g_bc = nullptr;
// instance id -> its WILD entry's first slot (nf_bound.h NfWild; 0: not wild)
std::unordered_map<uint32_t, uint32_t> g_wild_entry;
NfWild wild_entry(const HostScene& s, uint32_t at) {
  const uint32_t* e = s.slots.data() + 4 * (size_t)at;
  auto fl = [&](int i) { float v; memcpy(&v, &e[i], 4); return v; };
  return NfWild{{fl(0), fl(1), fl(2)}, {fl(3), fl(4), fl(5)}, fl(6), fl(7), fl(8), fl(9), {fl(10), fl(11), fl(12)}, fl(13)};
}

// NF tree parents (normal cones, round 6): every node a primitive's test
// passes through on the near-first walk thickens its boxes by that node's
// rho, so each must cover the hit: leaf_parent[vnf slot] is the NF node
// holding the primitive's leaf, nf_parent the node above a node (~0: a root)
std::unordered_map<uint32_t, uint32_t> g_nf_parent;
std::vector<uint32_t> g_leaf_parent;
uint32_t nf_vslot(const HostScene& s, const uint32_t* a) {
  switch (a[7]) {
    case KIND_TRI: return s.vnf_base[VNF_TRI] + (a[6] & kTriIdMask);
    case KIND_SPHERE: return s.vnf_base[VNF_SPHERE] + a[4];
    case KIND_INST: return s.vnf_base[VNF_INST] + a[0];
    default: return s.vnf_base[VNF_MODEL] + a[0];
  }
}
void map_nf_tree(const HostScene& s, uint32_t root, std::vector<uint8_t>& seen_blas) {
  const uint32_t* w = s.slots.data();
  std::vector<std::pair<uint32_t, uint32_t>> st{{root, ~0u}};
  while (!st.empty()) {
    const auto [i, par] = st.back();
    st.pop_back();
    const uint32_t* a = w + 4 * (size_t)i;
    if (a[7] & kBoxFlag) {
      g_nf_parent[i] = par;
      const uint32_t base = a[7] & kNfIdx;
      st.push_back({base, i});
      st.push_back({base + 2 + ((a[3] >> 24) & 1u), i});
      continue;
    }
    for (uint32_t r = i;;) {
      const uint32_t* b = w + 4 * (size_t)r;
      g_leaf_parent[nf_vslot(s, b)] = par;
      uint32_t next;
      if (b[7] == KIND_TRI) {
        next = b[11];
      } else if (b[7] == KIND_SPHERE) {
        next = b[5];
      } else {
        if (b[7] == KIND_INST && b[3] != 0) g_wild_entry[b[0]] = b[3];
        if (!seen_blas[b[1]]) {
          seen_blas[b[1]] = 1;
          map_nf_tree(s, b[1], seen_blas);
        }
        next = b[2];
      }
      if (next == kNfPop) break;
      r = next;
    }
  }
}
// the smallest rho over the NF nodes a hit's primitive (vnf slot) sits below,
// each with its normal cone (path.h trav_box_index_nf), at the hit's t
float cone_rho_min(const HostScene& s, uint32_t vslot, V o, V d, float t, bool obj) {
  const mrt::V3 oo{o.x, o.y, o.z}, dd{d.x, d.y, d.z};
  const float d2 = (d.x * d.x + d.y * d.y) + d.z * d.z;
  const NfBound& B = s.nfb;
  const NfCoef c = obj ? nf_coef_object(B, oo, d2) : nf_coef_world(B, oo, d2);
  const NfLine l = nf_line(B, c, t, obj ? B.ao0 : B.aw0, obj ? B.ao1 : B.aw1, d2, dd);
  float rho = nf_rho_at(B, c, t);
  if (!(B.kc > 0) || vslot >= g_leaf_parent.size()) return rho;
  const uint32_t* w = s.slots.data();
  for (uint32_t n = g_leaf_parent[vslot]; n != ~0u; n = g_nf_parent[n]) {
    const uint32_t* a = w + 4 * (size_t)n;
    rho = std::min(rho, nf_rho_cone(l, t, a[0], a[1], a[2], a[3], dd));
  }
  return rho;
}
double box_dist(const float* b, double x, double y, double z) {
  const double p[3] = {x, y, z};
  double m = 0;
  for (int k = 0; k < 3; ++k) m = std::max(m, std::max((double)b[k] - p[k], p[k] - (double)b[3 + k]));
  return m;
}
void check_hit(const HostScene& s, const float* box, V o, V d, float t, bool obj, uint32_t vslot = ~0u) {
  if (!box || std::isnan(box[0])) return;
  const double x = (double)o.x + (double)t * d.x, y = (double)o.y + (double)t * d.y, z = (double)o.z + (double)t * d.z;
  const mrt::V3 oo{o.x, o.y, o.z};
  const NfCoef c = obj ? nf_coef_object(s.nfb, oo, dot(d, d)) : nf_coef_world(s.nfb, oo, dot(d, d));
  // the rho of every NF node above the primitive, narrowed by its cone
  const float rho = vslot == ~0u ? nf_rho_at(s.nfb, c, t) : cone_rho_min(s, vslot, o, d, t, obj);
  const float cap = nf_rho_at(s.nfb, c, INFINITY);
  const double dist = box_dist(box, x, y, z);

  g_bc->checks++;
  if (dist > 0) g_bc->outside++;
  const double ratio = dist / (double)rho;
  if (ratio > 1) {
    if (g_bc->over < 5)
      fprintf(stderr, "bound exceeded: dist %.3e rho %.3e (%s space) t %a\n", dist, (double)rho, obj ? "object" : "world", t);
    g_bc->over++;
  }
  g_bc->worst = std::max(g_bc->worst, ratio);
  // the cap: rho at the capped L must still cover this hit
  if (dist > cap) g_bc->over++;
}
// a wild instance's hit in world space against its world box, within the wild margin
void check_hit_wild(const HostScene& s, uint32_t inst, V o, V d, float t) {
  auto it = g_wild_entry.find(inst);
  if (it == g_wild_entry.end()) return;  // no entry (an infinite box): always entered
  const NfWild e = wild_entry(s, it->second);
  const float box[6] = {e.mn[0], e.mn[1], e.mn[2], e.mx[0], e.mx[1], e.mx[2]};
  const double x = (double)o.x + (double)t * d.x, y = (double)o.y + (double)t * d.y, z = (double)o.z + (double)t * d.z;
  const mrt::V3 oo{o.x, o.y, o.z};
  const float rho = nf_rho_wild(e, oo, dot(d, d), t), cap = nf_rho_wild(e, oo, dot(d, d), INFINITY);
  const double dist = box_dist(box, x, y, z);
  g_bc->checks++;
  g_bc->wild_checks++;
  if (dist > 0) g_bc->outside++;
  const double ratio = dist / (double)rho;
  if (ratio > 1 || dist > cap) {
    if (g_bc->over < 5) fprintf(stderr, "wild bound exceeded: dist %.3e rho %.3e t %a\n", dist, (double)rho, t);
    g_bc->over++;
  }
  g_bc->worst = std::max(g_bc->worst, ratio);
  g_bc->worst_wild = std::max(g_bc->worst_wild, ratio);
}
const float* leaf_box(const HostScene& s, uint32_t base, uint32_t id) {
  if (s.nf_leaf_box.empty()) return nullptr;
  return &s.nf_leaf_box[6 * (size_t)(s.vnf_base[base] + id)];
}

// plain stream (layout.h): exact box tests
Result walk_plain(const HostScene& s, V o, V d, Stats* st = nullptr) {
  const uint32_t* w = s.slots.data();
  Ray wr = make_ray(o, d, s.early_ok), r = wr;
  uint32_t i = s.world_begin, ret = ~0u, hit_ret = ~0u;
  float best = INFINITY;
  uint32_t prim = 0;
  for (;;) {
    const uint32_t* a = w + 4 * (size_t)i;
    const uint32_t k = a[7];
    if (k & kBoxFlag) {
      float mn[3] = {f(a[0]), f(a[1]), f(a[2])}, mx[3] = {f(a[3]), f(a[4]), f(a[5])};
      const bool truth = box_exact(mn, mx, r, kTmin, best);
      if (st) {
        st->boxes++;
        st->loads += 2;
        const int dec = early_decide(mn, mx, r, kTmin, best);
        if (dec < 0) st->undecided++;
        else if ((dec != 0) != truth) st->wrong++;
      }
      i = truth ? (k & ~kBoxFlag) : a[6];
    } else if (k == KIND_END) {
      if (st) st->loads += 2;
      if (ret == ~0u) break;
      if (ret & 0x80000000u) r = wr;
      i = ret & 0x7FFFFFFFu;
      ret = ~0u;
    } else if (k == KIND_SPHERE) {
      float t;
      if (st) st->loads += 2;
      if (sphere_hit({f(a[0]), f(a[1]), f(a[2])}, f(a[3]), r.o, r.d, kTmin, best, t))
        best = t, prim = MRT_REF(MRT_REF_SPHERE, a[4]), hit_ret = ret;
      if (g_bc && sphere_hit({f(a[0]), f(a[1]), f(a[2])}, f(a[3]), r.o, r.d, kTmin, INFINITY, t))
        check_hit(s, leaf_box(s, VNF_SPHERE, a[4]), r.o, r.d, t, false);  // spheres are world objects
      i = a[5];  // next (layout.h)
    } else if (k == KIND_TRI) {
      float t;
      if (st) st->loads += 3;
      if (tri_hit({f(a[0]), f(a[1]), f(a[2])}, {f(a[3]), f(a[4]), f(a[5])}, {f(a[8]), f(a[9]), f(a[10])}, r.o, r.d,
                  kTmin, best, t))
        best = t, prim = MRT_REF(MRT_REF_TRIANGLE, a[6] & kTriIdMask), hit_ret = ret;
      if (g_bc && tri_hit({f(a[0]), f(a[1]), f(a[2])}, {f(a[3]), f(a[4]), f(a[5])}, {f(a[8]), f(a[9]), f(a[10])}, r.o,
                          r.d, kTmin, INFINITY, t)) {
        const bool inst = ret != ~0u && (ret & 0x80000000u);
        check_hit(s, leaf_box(s, VNF_TRI, a[6] & kTriIdMask), r.o, r.d, t, inst, s.vnf_base[VNF_TRI] + (a[6] & kTriIdMask));
        if (inst) {  // the same hit in world space against the instance's world box
          const uint32_t cid = w[4 * (size_t)((ret & 0x7FFFFFFFu) - 2)];
          if (s.nf_inst_wild.empty() || !s.nf_inst_wild[cid])
            check_hit(s, leaf_box(s, VNF_INST, cid), wr.o, wr.d, t, false);
          else  // a wild instance: its world box within the wild margin (nf_bound.h nf_rho_wild)
            check_hit_wild(s, cid, wr.o, wr.d, t);
        } else if (ret != ~0u) {  // a model's triangle: its world box too
          const uint32_t cid = w[4 * (size_t)(ret - 2)];
          check_hit(s, leaf_box(s, VNF_MODEL, cid), wr.o, wr.d, t, false);
        }
      }
      i = a[11];  // next (layout.h)
    } else if (k == KIND_INST) {
      const float* m = &s.inst_inv[12 * (size_t)a[0]];
      if (st) st->loads += 5, st->entries++;
      r = make_ray(xf(m, wr.o, 1.0f), xf(m, wr.d, 0.0f), s.early_ok);
      ret = (i + 2) | 0x80000000u;
      i = a[1];
    } else if (k == KIND_MODEL) {
      if (st) st->loads += 2;
      ret = i + 2;
      i = a[1];
    } else {
      fprintf(stderr, "plain: unsupported kind %u\n", k);
      exit(2);
    }
  }
  uint32_t cont = 0;
  if (hit_ret != ~0u) {
    const uint32_t rec = (hit_ret & 0x7FFFFFFFu) - 2;
    cont = MRT_REF((hit_ret & 0x80000000u) ? MRT_REF_INSTANCE : MRT_REF_MODEL, w[4 * (size_t)rec]);
  }
  return {prim, cont, best};
}

// path.h nf_node_test: both children's boxes of an NF node (layout.h) at
// once, from the planes' 8-bit steps. Fast rays: t = q * (2^e * y) +
// (o * y - oy) per plane with the early decision's margin plus the node's
// |o * y - oy| term — "miss" only when certain, anything else a hit
// (conservative: the walk's hits are checked, its boxes never need to be
// exact); other rays: the exact test on the decoded planes widened by an ulp.
void node_test(const uint32_t* a, const Ray& r, float tmin, float tmax, float nfm, bool hit[2], float ent[2],
               float ex[2]) {
  const float o[3] = {f(a[0]), f(a[1]), f(a[2])};
  uint8_t q[12];
  for (int j = 0; j < 3; ++j)
    for (int b = 0; b < 4; ++b) q[4 * j + b] = (uint8_t)(a[4 + j] >> (8 * b));
  float sc[3], A[3], B[3], BL[3], BH[3], mb = 0.0f;
  for (int k = 0; k < 3; ++k) {
    sc[k] = f(((a[3] >> (8 * k)) & 0xFFu) << 23);
    A[k] = sc[k] * r.y[k];
    B[k] = std::fma(o[k], r.y[k], -r.oy[k]);
    BL[k] = std::fma(-nfm, r.y[k], B[k]);
    BH[k] = std::fma(nfm, r.y[k], B[k]);
    mb = std::max(mb, std::max(fabsf(BL[k]), fabsf(BH[k])));
  }
  const float mabs = std::fma(mb, 0x1p-20f, r.om);
  for (int c = 0; c < 2; ++c) {
    const uint8_t* lo = q + 6 * c;
    const uint8_t* hi = q + 6 * c + 3;
    if (r.fast) {
      float tl[3], th[3];
      for (int k = 0; k < 3; ++k) tl[k] = std::fma((float)lo[k], A[k], BL[k]), th[k] = std::fma((float)hi[k], A[k], BH[k]);
      const float t0 = fmaxf(fmaxf(fminf(tl[0], th[0]), fminf(tl[1], th[1])), fmaxf(fminf(tl[2], th[2]), tmin));
      const float t1 = fminf(fminf(fmaxf(tl[0], th[0]), fmaxf(tl[1], th[1])), fminf(fmaxf(tl[2], th[2]), tmax));
      const float m = std::fma(fabsf(t0) + fabsf(t1), 0x1p-19f, mabs);
      const bool force = (a[7] & (kNfForceL << c)) != 0;
      hit[c] = !(t0 - t1 > m) || force;
      ent[c] = t0;
      ex[c] = force ? INFINITY : std::fma(m, 2.0f, t1);  // a wild instance's hits: no exit bound
    } else {
      float mn[3], mx[3];
      for (int k = 0; k < 3; ++k) {
        const float pl = std::fma((float)lo[k], sc[k], o[k]) - nfm, ph = std::fma((float)hi[k], sc[k], o[k]) + nfm;
        mn[k] = pl - std::fma(fabsf(pl), 0x1p-23f, 0x1p-140f);
        mx[k] = ph + std::fma(fabsf(ph), 0x1p-23f, 0x1p-140f);
      }
      hit[c] = box_exact(mn, mx, r, tmin, tmax) || (a[7] & (kNfForceL << c));
      ent[c] = 0.0f;
      ex[c] = INFINITY;
    }
  }
}

// The verified near-first walk (layout.h; path.h trav_*_nf, nf_finish)
// restated on the host: the NF trees near child first with a stack, the
// reference's tie rule by order keys, the reachability check of the winner
// on the reference stream, the reference's walk where it fails.
uint64_t nf_key(const HostScene& s, uint32_t prim, uint32_t ret) {
  const uint32_t* w = s.slots.data();
  const uint32_t kind = prim >> 28, id = prim & 0x0FFFFFFFu;
  auto entry = [&](uint32_t base, uint32_t i, int word) { return s.vnf_leaf[2 * (size_t)(s.vnf_base[base] + i) + word]; };
  if (kind == MRT_REF_SPHERE) return (uint64_t)entry(VNF_SPHERE, id, 1) << 32;
  const uint32_t k = entry(VNF_TRI, id, 1);
  if (k & kWorldKey) return (uint64_t)(k & ~kWorldKey) << 32;
  const uint32_t cid = w[4 * (size_t)((ret & 0x7FFFFFFFu) - 2)];
  return ((uint64_t)entry((ret & 0x80000000u) ? VNF_INST : VNF_MODEL, cid, 1) << 32) | k;
}
Result walk_nf(const HostScene& s, V o, V d, Stats* st, uint64_t* fallbacks, uint64_t* starts_ref = nullptr) {
  const uint32_t* w = s.slots.data();
  const Ray wr = make_ray(o, d, s.early_ok);
  if (!nf_ray_ok(s.nfb, dot(d, d))) {  // path.h nf_start: the bound does not cover this ray
    if (starts_ref) ++*starts_ref;
    return walk_plain(s, o, d, st);
  }
  Ray r = wr;
  uint32_t i = s.nf_world, ret = ~0u, hit_ret = ~0u, prim = 0;
  float best = INFINITY, t2 = INFINITY, nl = INFINITY;
  NfCoef nfc{};
  NfLine nfl{};
  std::vector<uint32_t> stack;
  std::vector<float> stack_nl;
  auto cull = [&]() { return std::fma(fabsf(best), 0x1p-10f, best); };
  auto margin = [&]() {  // path.h nf_margin
    const bool obj = ret != ~0u && (ret & 0x80000000u);
    const mrt::V3 oo{r.o.x, r.o.y, r.o.z};
    nfc = obj ? nf_coef_object(s.nfb, oo, dot(r.d, r.d)) : nf_coef_world(s.nfb, oo, dot(r.d, r.d));
    nfl = nf_line(s.nfb, nfc, cull(), obj ? s.nfb.ao0 : s.nfb.aw0, obj ? s.nfb.ao1 : s.nfb.aw1, dot(r.d, r.d),
                  mrt::V3{r.d.x, r.d.y, r.d.z});
  };
  margin();
  auto pop = [&]() {
    while (!stack.empty()) {
      const uint32_t v = stack.back();
      stack.pop_back();
      nl = INFINITY;
      stack_nl.pop_back();
      if (v != 0x80000000u) {
        i = v;
        return true;
      }
      const bool inst = (ret & 0x80000000u) != 0;
      ret = ~0u;
      if (inst) {
        r = wr;
        if (st) st->loads += 2;
        margin();
      }
    }
    return false;
  };
  auto better = [&](float t, uint32_t pr) {
    if (t < best) return true;
    if (!(t == best)) return false;
    if (prim == 0) return true;
    return nf_key(s, pr, ret) > nf_key(s, prim, hit_ret);
  };
  auto hit = [&](float t, uint32_t pr) {
    if (t <= best && better(t, pr)) {
      t2 = fminf(t2, best);
      best = t, prim = pr, hit_ret = ret;
      nfl.rcb = nf_rho_node(nfl, cull());
    } else {
      t2 = fminf(t2, t);
    }
  };
  for (;;) {
    const uint32_t* a = w + 4 * (size_t)i;
    const uint32_t k = a[7];
    if (k & kBoxFlag) {  // a node: both children's boxes, the nearer hit child first
      if (st) st->boxes += 2, st->loads += 2;
      bool h[2];
      float e[2], x[2];
      const float tn = fminf(cull(), nl);
      // the cone while this ray's worst-case generic term is worth it (path.h: while some lane's is)
      const float rho = s.nfb.kc > 0 && nfl.rg * tn > s.nfb.kcmin
                            ? nf_rho_cone(nfl, tn, a[0], a[1], a[2], a[3], mrt::V3{r.d.x, r.d.y, r.d.z})
                            : nf_rho_node(nfl, tn);
      node_test(a, r, kTmin, cull(), getenv("SLAB_NO_CONE") ? nf_rho_node(nfl, tn) : rho, h, e, x);
      const uint32_t base = k & kNfIdx, right = base + 2 + ((a[3] >> 24) & 1u);
      if (h[0] && h[1]) {
        const bool lf = !(e[1] < e[0]);
        stack.push_back(lf ? right : base);
        stack_nl.push_back(lf ? x[1] : x[0]);
        if (stack.size() > kNfStack) {
          fprintf(stderr, "nf: stack overflow\n");
          exit(3);
        }
        i = lf ? base : right;
        nl = getenv("SLAB_NO_NL") ? INFINITY : (lf ? x[0] : x[1]);
      } else if (h[0] || h[1]) {
        i = h[0] ? base : right;
        nl = getenv("SLAB_NO_NL") ? INFINITY : (h[0] ? x[0] : x[1]);
      } else if (!pop()) {
        break;
      }
      continue;
    }
    uint32_t next;
    if (k == KIND_TRI) {
      float t;
      const uint32_t pr = MRT_REF(MRT_REF_TRIANGLE, a[6] & kTriIdMask);
      if (st) st->loads += 3, st->prims++;
      if (tri_hit({f(a[0]), f(a[1]), f(a[2])}, {f(a[3]), f(a[4]), f(a[5])}, {f(a[8]), f(a[9]), f(a[10])}, r.o, r.d,
                  kTmin, cull(), t))
        hit(t, pr);
      next = a[11];
    } else if (k == KIND_SPHERE) {
      float t;
      const uint32_t pr = MRT_REF(MRT_REF_SPHERE, a[4]);
      if (st) st->loads += 2, st->prims++;
      if (sphere_hit({f(a[0]), f(a[1]), f(a[2])}, f(a[3]), r.o, r.d, kTmin, cull(), t)) hit(t, pr);
      next = a[5];
    } else if (k == KIND_INST && a[3] != 0 &&
               !nf_wild_hit(wild_entry(s, a[3]), mrt::V3{r.o.x, r.o.y, r.o.z}, mrt::V3{r.d.x, r.d.y, r.d.z}, dot(r.d, r.d),
                            kTmin, cull())) {
      if (st) st->loads += 4, st->wild_skips++;  // path.h nf_wild_enter: the WILD entry, then the leaf's next
      next = a[2];
    } else if (k == KIND_INST || k == KIND_MODEL) {
      if (st) st->loads += k == KIND_INST ? 5 : 2;
      if (st && k == KIND_INST) st->entries++;
      if (a[2] != kNfPop) stack.push_back(a[2]), stack_nl.push_back(nl);
      stack.push_back(0x80000000u);
      stack_nl.push_back(nl);
      if (k == KIND_INST) {
        const float* m = &s.inst_inv[12 * (size_t)a[0]];
        r = make_ray(xf(m, wr.o, 1.0f), xf(m, wr.d, 0.0f), s.early_ok);
        ret = (i + 2) | 0x80000000u;
        margin();
      } else {
        ret = i + 2;
      }
      i = a[1];
      continue;
    } else {
      fprintf(stderr, "nf: unsupported kind %u at %u\n", k, i);
      exit(2);
    }
    if (next != kNfPop) {
      i = next;
    } else if (!pop()) {
      break;
    }
  }
  // the check: the winner's innermost reference ancestors pass at
  // tau = min(t2, best * (1 + 2^-10)), a lower bound of the reference's t_max there
  bool ok = true;
  const float tau = fminf(t2, cull());
  auto box_at = [&](uint32_t rec, const Ray& rr) {
    const uint32_t* b = w + 4 * (size_t)rec;
    float mn[3] = {f(b[0]), f(b[1]), f(b[2])}, mx[3] = {f(b[3]), f(b[4]), f(b[5])};
    if (st) st->boxes++, st->loads += 2;
    return box_exact(mn, mx, rr, kTmin, tau);
  };
  if (prim) {
    const uint32_t kind = prim >> 28, id = prim & 0x0FFFFFFFu;
    const uint32_t own = s.vnf_leaf[2 * (size_t)(s.vnf_base[kind == MRT_REF_SPHERE ? VNF_SPHERE : VNF_TRI] + id)];
    if (hit_ret == ~0u) {
      if (own != kNoParent) ok = box_at(own, wr);
    } else {
      const bool inst = (hit_ret & 0x80000000u) != 0;
      const uint32_t cid = w[4 * (size_t)((hit_ret & 0x7FFFFFFFu) - 2)];
      const uint32_t wpar = s.vnf_leaf[2 * (size_t)(s.vnf_base[inst ? VNF_INST : VNF_MODEL] + cid)];
      if (wpar != kNoParent) ok = box_at(wpar, wr);
      if (ok && own != kNoParent) {
        Ray rr = wr;
        if (inst) {
          const float* m = &s.inst_inv[12 * (size_t)cid];
          rr = make_ray(xf(m, wr.o, 1.0f), xf(m, wr.d, 0.0f), s.early_ok);
        }
        ok = box_at(own, rr);
      }
    }
  }
  if (ok) {
    uint32_t cont = 0;
    if (hit_ret != ~0u) {
      const uint32_t rec = (hit_ret & 0x7FFFFFFFu) - 2;
      cont = MRT_REF((hit_ret & 0x80000000u) ? MRT_REF_INSTANCE : MRT_REF_MODEL, w[4 * (size_t)rec]);
    }
    return {prim, cont, best};
  }
  ++*fallbacks;
  return walk_plain(s, o, d, st);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) return 1;
  const int n = argc > 2 ? atoi(argv[2]) : 20000;
  mrt_builder* b = nullptr;
  mrt_builder_new(1, &b);
  if (mrt_builder_builtin(b, argv[1], 16.0f / 9.0f, argc > 3 ? argv[3] : "tests/golden") != 0) {
    printf("%s: %s\n", argv[1], mrt_global_last_error());
    return 1;
  }
  mrt_builder_build_bvh(b);
  mrt_scene_desc d;
  mrt_camera cam;
  mrt_builder_desc(b, &d, &cam);
  HostScene s;
  s.keep_nf_boxes = true;  // the bound checks' leaf boxes
  s.nf_build = kNfBuildAlways;  // the trees even where the per-scene rule would walk the reference's way
  std::string err;
  if (!build_host_scene(d, s, err)) {
    printf("%s\n", err.c_str());
    return 1;
  }
  // `layout` mode: the same rays through the plain preorder stream (build_host_scene(..., false))
  // and the default layout (BLAS regions with siblings together) must find the
  // same closest hits, t bits included, after the same number of box tests
  HostScene dfs;
  const bool layout = argc > 4 && !strcmp(argv[4], "layout");
  // `nf` mode: the verified near-first walk must find the reference's closest
  // hits (primitive, container, t bits) on every ray
  const bool nf = argc > 4 && (!strcmp(argv[4], "nf") || !strcmp(argv[4], "graze") || !strcmp(argv[4], "tangent"));
  // `graze` mode: rays nearly parallel to a triangle of the scene (angle
  // 10^U(-8,-1.5) rad to its plane, through a random point of it, from 0.5-60
  // units back; through an instance's transform half the time) — where
  // Moller-Trumbore's t is least accurate, the near-first walk's culling
  // margin is tested hardest
  const bool graze = argc > 4 && !strcmp(argv[4], "graze");
  // `tangent` mode: rays nearly tangent to a sphere (offset 10^U(-7,-1) of its
  // radius from the tangent line) from 1-400 radii away — where the sphere
  // test's disc cancels
  const bool tangent = argc > 4 && !strcmp(argv[4], "tangent");
  const bool stress = graze || tangent;
  if (getenv("SLAB_ZERO_RHO")) {  // experiment: the walk without its rounding margins (not exact)
    const float wr = s.nfb.wr;
    s.nfb = NfBound{};
    s.nfb.sr = -1.0f;
    s.nfb.wr = wr;
  }
  if (getenv("SLAB_GEN_SCALE")) s.nfb.aw1 *= atof(getenv("SLAB_GEN_SCALE"));
  if (nf && s.nf_ok) {
    const NfBound& B = s.nfb;
    printf("%-14s bound: aw0 %.3g aw1 %.3g bw0 %.3g bw1 %.3g kw1 %.3g ko1 %.3g ao0 %.3g ao1 %.3g orad %.3g | world ball r %.3g"
           " generic r %.3g | spheres r %.3g s51 %.3g s11 %.3g\n", argv[1], B.aw0, B.aw1, B.bw0, B.bw1, B.kw1, B.ko1, B.ao0, B.ao1, B.orad,
           B.wr, B.gr, B.sr, B.s51, B.s11);
  }
  if (nf && !s.nf_ok) {
    printf("%-14s nf: no near-first trees (%s)\n", argv[1], s.nf_note.c_str());
    return 0;
  }
  if (nf && s.nf_ok) {  // NF parents for the cone-narrowed bound checks
    g_leaf_parent.assign(s.vnf_leaf.size() / 2, ~0u);
    std::vector<uint8_t> seen(s.slots.size() / 4, 0);
    map_nf_tree(s, s.nf_world, seen);
    printf("%-14s nf cones: %u of %u nodes carry one, kc %.3g\n", argv[1], s.nf_cones, s.nf_boxes, (double)s.nfb.kc);
    for (const auto& [inst, at] : g_wild_entry) {
      const NfWild e = wild_entry(s, at);
      printf("%-14s wild instance %u: box (%.4g %.4g %.4g)-(%.4g %.4g %.4g) a0 %.3g a1 %.3g b0 %.3g b1 %.3g r %.3g\n", argv[1],
             inst, e.mn[0], e.mn[1], e.mn[2], e.mx[0], e.mx[1], e.mx[2], e.a0, e.a1, e.b0, e.b1, e.r);
    }
  }
  uint64_t nf_bad = 0, nf_fallbacks = 0, nf_starts_ref = 0, nf_even = 0, nf_odd = 0;
  BoundCheck bc;
  if (nf) g_bc = &bc;
  std::vector<uint32_t> nf_per_ray, ref_per_ray;  // box tests per ray: the tail a persistent wave waits on
  Stats nf_st;
  if (layout) {
    if (!build_host_scene(d, dfs, err, false)) return 1;
  }
  uint64_t layout_bad = 0;
  std::mt19937 g(7);
  std::uniform_real_distribution<float> u(0.0f, 1.0f);
  Stats st;
  uint64_t hits = 0, fast = 0;
  const V o{cam.origin[0], cam.origin[1], cam.origin[2]};
  V cam_d{0, 0, -1};
  for (int k = 0; k < n; ++k) {
    V ro, rd;
    if (tangent) {
      if (!d.n_spheres) break;
      const mrt_sphere& sp = d.spheres[std::min<uint32_t>(d.n_spheres - 1, (uint32_t)(u(g) * d.n_spheres))];
      const float rad = fabsf(sp.radius);
      V w{u(g) * 2 - 1, u(g) * 2 - 1, u(g) * 2 - 1};
      const float wl = sqrtf(dot(w, w));
      if (!(wl > 0.1f)) continue;
      w = {w.x / wl, w.y / wl, w.z / wl};  // from the centre towards the tangent point
      V t1 = cross(w, fabsf(w.x) < 0.9f ? V{1, 0, 0} : V{0, 1, 0});
      const float tl = sqrtf(dot(t1, t1));
      t1 = {t1.x / tl, t1.y / tl, t1.z / tl};
      const float off = rad * (1.0f + (u(g) < 0.5f ? -1.0f : 1.0f) * powf(10.0f, -7.0f + 6.0f * u(g)));
      const V p{sp.center[0] + w.x * off, sp.center[1] + w.y * off, sp.center[2] + w.z * off};
      const float sc = 0.5f + 1.5f * u(g), back = rad * powf(10.0f, 2.6f * u(g));
      rd = {t1.x * sc, t1.y * sc, t1.z * sc};
      ro = {p.x - rd.x * back / sc, p.y - rd.y * back / sc, p.z - rd.z * back / sc};
    } else if (graze) {
      const mrt_triangle& tr = d.triangles[std::min<uint32_t>(d.n_triangles - 1, (uint32_t)(u(g) * d.n_triangles))];
      const float* m = nullptr;
      if (d.n_instances && u(g) < 0.5f)
        m = d.instances[std::min<uint32_t>(d.n_instances - 1, (uint32_t)(u(g) * d.n_instances))].fwd;
      auto xw = [&](const float* v, float w) -> V {
        if (!m) return {v[0] * w + (1 - w) * v[0], v[1], v[2]};
        return {m[0] * v[0] + m[4] * v[1] + m[8] * v[2] + m[12] * w, m[1] * v[0] + m[5] * v[1] + m[9] * v[2] + m[13] * w,
                m[2] * v[0] + m[6] * v[1] + m[10] * v[2] + m[14] * w};
      };
      const V A = xw(tr.a, 1), B = xw(tr.b, 1), C = xw(tr.c, 1);
      float b1 = u(g), b2 = u(g);
      if (b1 + b2 > 1) b1 = 1 - b1, b2 = 1 - b2;
      const V p{A.x + (B.x - A.x) * b1 + (C.x - A.x) * b2, A.y + (B.y - A.y) * b1 + (C.y - A.y) * b2,
                A.z + (B.z - A.z) * b1 + (C.z - A.z) * b2};
      V nn = cross(sub(B, A), sub(C, A));
      const double nl = sqrt((double)dot(nn, nn));
      if (!(nl > 0)) continue;
      nn = {(float)(nn.x / nl), (float)(nn.y / nl), (float)(nn.z / nl)};
      V t1 = cross(nn, fabsf(nn.x) < 0.9f ? V{1, 0, 0} : V{0, 1, 0});
      const float tl = sqrtf(dot(t1, t1));
      t1 = {t1.x / tl, t1.y / tl, t1.z / tl};
      const V t2 = cross(nn, t1);
      const float phi = 6.2831853f * u(g), th = powf(10.0f, -8.0f + 6.5f * u(g)) * (u(g) < 0.5f ? -1.0f : 1.0f);
      const float sc = 0.5f + 1.5f * u(g), back = 0.5f + 59.5f * u(g);
      const float ct = cosf(th), st_ = sinf(th);
      rd = {sc * (ct * (cosf(phi) * t1.x + sinf(phi) * t2.x) + st_ * nn.x),
            sc * (ct * (cosf(phi) * t1.y + sinf(phi) * t2.y) + st_ * nn.y),
            sc * (ct * (cosf(phi) * t1.z + sinf(phi) * t2.z) + st_ * nn.z)};
      ro = {p.x - rd.x * back, p.y - rd.y * back, p.z - rd.z * back};
    } else if (k % 2 == 0) {  // camera ray
      const float s1 = u(g), t1 = u(g);
      rd = {((cam.lower_left_corner[0] + cam.horizontal[0] * s1) + cam.vertical[0] * t1) - o.x,
            ((cam.lower_left_corner[1] + cam.horizontal[1] * s1) + cam.vertical[1] * t1) - o.y,
            ((cam.lower_left_corner[2] + cam.horizontal[2] * s1) + cam.vertical[2] * t1) - o.z};
      ro = o;
      cam_d = rd;
    } else {  // from the first hit of the previous camera ray, random direction (a bounce)
      const Result h = walk_plain(s, o, cam_d);
      if (h.prim == 0) continue;
      ro = {o.x + cam_d.x * h.t, o.y + cam_d.y * h.t, o.z + cam_d.z * h.t};
      rd = {u(g) * 2 - 1, u(g) * 2 - 1, u(g) * 2 - 1};
    }
    fast += make_ray(ro, rd, s.early_ok).fast;
    const uint64_t boxes0 = st.boxes;
    const Result r = walk_plain(s, ro, rd, &st);
    hits += r.prim != 0;
    if (nf) {
      const uint64_t nb0 = nf_st.boxes;
      BoundCheck* keep = g_bc;
      g_bc = nullptr;  // the reference walk inside walk_nf's fallback is not checked twice
      const Result q = walk_nf(s, ro, rd, &nf_st, &nf_fallbacks, &nf_starts_ref);
      g_bc = keep;
      nf_per_ray.push_back(uint32_t(nf_st.boxes - nb0));
      (k % 2 ? nf_odd : nf_even) += nf_st.boxes - nb0;
      ref_per_ray.push_back(uint32_t(st.boxes - boxes0));
      uint32_t tb, qb;
      memcpy(&tb, &r.t, 4);
      memcpy(&qb, &q.t, 4);
      const bool bad = r.prim != q.prim || r.container != q.container || (r.prim && tb != qb);
      if (bad && nf_bad < 5)
        fprintf(stderr, "nf differs: ref prim %08x cont %08x t %a | nf prim %08x cont %08x t %a\n", r.prim, r.container,
                r.t, q.prim, q.container, q.t);
      nf_bad += bad;
    }
    if (layout) {
      Stats sd;
      const Result q = walk_plain(dfs, ro, rd, &sd);
      uint32_t tb, qb;
      memcpy(&tb, &r.t, 4);
      memcpy(&qb, &q.t, 4);
      layout_bad += r.prim != q.prim || r.container != q.container || tb != qb || sd.boxes != st.boxes - boxes0;
    }
  }
  if (nf) {
    printf("%-14s nf: %llu of %d rays differ from the reference walk; box tests %.1f vs %.1f per ray (x%.2f), "
           "record loads %.1f vs %.1f (x%.2f), %llu fallbacks (%.2f%%), stack need %u\n",
           argv[1], (unsigned long long)nf_bad, n, (double)nf_st.boxes / n, (double)st.boxes / n,
           (double)st.boxes / std::max<uint64_t>(nf_st.boxes, 1), (double)nf_st.loads / n, (double)st.loads / n,
           (double)st.loads / std::max<uint64_t>(nf_st.loads, 1), (unsigned long long)nf_fallbacks,
           100.0 * nf_fallbacks / n, s.nf_stack_need);
    auto tail = [](std::vector<uint32_t> v, double q) {
      if (v.empty()) return 0u;
      std::sort(v.begin(), v.end());
      return v[std::min<size_t>(v.size() - 1, size_t(q * v.size()))];
    };
    printf("%-14s nf tail: box tests per ray p99 %u / p99.9 %u / max %u (reference walk %u / %u / %u)\n", argv[1],
           tail(nf_per_ray, 0.99), tail(nf_per_ray, 0.999), tail(nf_per_ray, 1.0), tail(ref_per_ray, 0.99),
           tail(ref_per_ray, 0.999), tail(ref_per_ray, 1.0));
    printf("%-14s nf bound: %llu accepted hits checked, %llu outside their box, worst dist/rho %.3g, %llu over; "
           "%llu rays start on the reference walk (%.2f%%), %u wild instances\n",
           argv[1], (unsigned long long)bc.checks, (unsigned long long)bc.outside, bc.worst,
           (unsigned long long)bc.over, (unsigned long long)nf_starts_ref, 100.0 * nf_starts_ref / n, s.nf_wild);
    printf("%-14s nf box tests per ray: even rays %.1f, odd rays %.1f; instance entries per ray %.3f\n", argv[1],
           2.0 * nf_even / n, 2.0 * nf_odd / n, (double)nf_st.entries / n);
    printf("%-14s nf wild instances passed by per ray %.3f; primitive tests per ray %.2f; cost estimate %.0f VALU/ray "
           "(58 per box test, 45 per primitive test, 500 per instance entry)\n", argv[1], (double)nf_st.wild_skips / n,
           (double)nf_st.prims / n, (58.0 * nf_st.boxes + 45.0 * nf_st.prims + 500.0 * nf_st.entries) / n);
    printf("%-14s reference walk: instance entries per ray %.3f\n", argv[1], (double)st.entries / n);
    printf("%-14s nf wild: %llu hits of wild instances checked, worst dist/rho %.3g\n", argv[1],
           (unsigned long long)bc.wild_checks, bc.worst_wild);
    if (bc.over) return 1;
    if (nf_bad) return 1;
  }
  if (layout) {
    printf("%-14s layout: %llu of %d rays differ between the sibling layout and the preorder stream; stream %zu vs %zu slots\n",
           argv[1], (unsigned long long)layout_bad, n, s.slots.size() / 4, dfs.slots.size() / 4);
    if (layout_bad) return 1;
  }
  printf("%-14s rays %d (early domain %llu) hits %llu  boxes %llu  left to the exact test %.5f  wrong %llu\n", argv[1],
         n, (unsigned long long)fast, (unsigned long long)hits, (unsigned long long)st.boxes,
         (double)st.undecided / std::max<uint64_t>(st.boxes, 1), (unsigned long long)st.wrong);
  mrt_builder_free(b);
  return st.wrong ? 1 : 0;
}
