// nf_tree.cpp — the verified near-first trees (layout.h "verified near-first
// trees"): surface-area-heuristic BVHs over the scene's objects, appended to
// the record stream, plus each leaf object's reference parent box and order
// key for the check that the reference's left-first walk reaches the winner.
//
// Why (tools/order_check.cpp): the
// reference's tree (random-axis median splits, geom.rs:110-161) walked left
// child first (geom.rs:185-205) costs 80-96 box tests per ray on the BASELINE
// scenes; the same primitives under an SAH tree walked near child first cost
// 2.3-3.4x fewer. The closest hit the reference returns is, whenever its
// left-first walk reaches it, the smallest t with ties going to the later
// primitive of its order — which a near-first walk of any tree finds — and
// whether it reaches it is a property of the winner's ancestor boxes alone.
#include <math.h>
#include <cmath>
#include <string.h>

#include <algorithm>
#include <unordered_map>

#include "upload.h"

namespace mrt {

namespace {

float u2f(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}
uint32_t f2u(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

// ---- the reference stream (layout.h) ----
uint32_t kind_of(const std::vector<uint32_t>& w, uint32_t i) { return w[4 * (i + 1) + 3]; }
bool is_box(const std::vector<uint32_t>& w, uint32_t i) { return (kind_of(w, i) & kBoxFlag) != 0; }
uint32_t skip_of(const std::vector<uint32_t>& w, uint32_t i) { return w[4 * (i + 1) + 2]; }
uint32_t next_of(const std::vector<uint32_t>& w, uint32_t i) {
  switch (kind_of(w, i)) {
    case KIND_TRI: return w[4 * (i + 2) + 3];
    case KIND_SPHERE:
    case KIND_VOLUME: return w[4 * (i + 1) + 1];
    default: return i + 2;  // instance / model: the record after it
  }
}
// the items of a level: from `first` along successors until `end` (a skip
// target) or an END record
void level(const std::vector<uint32_t>& w, uint32_t first, uint32_t end, std::vector<uint32_t>& out) {
  out.clear();
  for (uint32_t c = first; c != end && kind_of(w, c) != KIND_END; c = is_box(w, c) ? skip_of(w, c) : next_of(w, c))
    out.push_back(c);
}

struct Box {
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const Box& b) {
    for (int k = 0; k < 3; ++k) mn[k] = fminf(mn[k], b.mn[k]), mx[k] = fmaxf(mx[k], b.mx[k]);
  }
  void grow(float x, float y, float z) {
    const float p[3] = {x, y, z};
    for (int k = 0; k < 3; ++k) mn[k] = fminf(mn[k], p[k]), mx[k] = fmaxf(mx[k], p[k]);
  }
  double area() const {
    const double dx = (double)mx[0] - mn[0], dy = (double)mx[1] - mn[1], dz = (double)mx[2] - mn[2];
    return dx < 0 ? 0.0 : 2.0 * (dx * dy + dy * dz + dz * dx);
  }
  float c(int k) const { return 0.5f * mn[k] + 0.5f * mx[k]; }
};

// Outward padding of an NF box plane (culling must never drop what the
// object's own test would hit): relative 2^-22 (two ulps) plus rel_extra,
// at least 2^-39, and never into (0, 2^-40) — the slab test's fast domain
// (path.h coord_ok) stays intact.
float pad(float v, float dir, float rel_extra) {
  if (!(fabsf(v) < INFINITY)) return v;
  float p = v + dir * fmaxf(fabsf(v) * (0x1p-22f + rel_extra), 0x1p-39f);
  const float a = fabsf(p);
  if (a > 0.0f && a < 0x1p-40f) p = ((p > 0.0f) == (dir > 0.0f)) ? dir * 0x1p-40f : 0.0f;
  return p;
}
void pad_box(Box& b, float rel_extra) {
  for (int k = 0; k < 3; ++k) b.mn[k] = pad(b.mn[k], -1.0f, rel_extra), b.mx[k] = pad(b.mx[k], 1.0f, rel_extra);
}

// ---- the rounding bounds (nf_bound.h; DESIGN.md §4 "Why the near-first walk
// is exact"): u = 2^-24, gamma_n = n u / (1 - n u) ----
constexpr double kU = 0x1p-24;
double gam(int n) { return n * kU / (1.0 - n * kU); }
// a float at or below / above v
float f_down(double v) {
  float f = (float)v;
  if ((double)f > v) f = nextafterf(f, -INFINITY);
  return f;
}
float f_up(double v) {
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, INFINITY);
  return f;
}
double norm3(const double v[3]) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

// A triangle's bound on how far its computed hit X = o + t d can lie from the
// triangle (Triangle::intersect, geom.rs:504-533, as path.h tri_hit computes
// it): |X - tri| <= a(|d|) L + pad with L = |X - o| and a(|d|) = a0 + a1 |d|;
// pad (proportional to the triangle's size) is added to its box on the host.
// k1: generic kappa per unit |d| (the walk requires k1 |d| <= kNfKappaMax).
struct TriBound {
  double a0 = 0, a1 = 0, k1 = 0, pad = 0;
};
TriBound tri_bound(const float ab[3], const float ac[3]) {
  const double u = kU;
  const double dab[3] = {ab[0], ab[1], ab[2]}, dac[3] = {ac[0], ac[1], ac[2]};
  const double S = norm3(dab) + norm3(dac), M2 = norm3(dab) * norm3(dac);
  // axis-structured: ab_k == ac_k == 0 — the plane x_k = const; every product
  // with those zeros is exact, det = d_k n_k up to the two in-plane products'
  // roundings, and the residual's terms all carry d_k or (o - a)_k
  for (int k = 0; k < 3; ++k) {
    if (!(ab[k] == 0.0f && ac[k] == 0.0f)) continue;
    const int j = (k + 1) % 3, l = (k + 2) % 3;  // n_k = ab_j ac_l - ab_l ac_j (cross, mrt_math.h)
    const double p1 = dab[j] * dac[l], p2 = dab[l] * dac[j];  // exact
    const double nk = std::fabs(p1 - p2), n1 = std::fabs(p1) + std::fabs(p2);
    if (!(nk > 0)) break;  // degenerate: the generic bound
    const double sl = n1 / nk, sigma = M2 / nk;
    const double beta = 1.0 - 3.01 * u * sl;
    if (beta < 0.5) break;
    const double lambda = (1.0 + 3.01 * u * sl) / ((1.0 - 3.01 * u * sl) * (1.0 - gam(2)));
    const double kap = u + 19.01 * u * sigma / beta;
    if (kap > (double)kNfKappaMax) break;
    TriBound b;
    b.a0 = (kap + 16.0 * u * sigma * lambda / beta + 2.01 * u) / (1.0 - kap);
    b.pad = ((1.0001 * kap + 2.01 * u) / (1.0 - kap) + 3.01 * u) * S;
    return b;
  }
  // generic: |det| >= 0.000001f (the reference's own test) bounds the
  // cancellation: kappa = u + c_g M2 |d|, c_g = 1.0001 * 24u / 0.000001f
  const double km = 1.01 * (double)kNfKappaMax, cg = 1.0001 * 24.0 * u * 1.0000001e6;
  TriBound b;
  b.a0 = 3.01 * u / (1.0 - km);
  b.a1 = cg * M2 / (1.0 - km);
  b.k1 = cg * M2;
  b.pad = ((1.0001 * km + 2.01 * u) / (1.0 - km) + 3.01 * u) * S;
  return b;
}

// ---- binned SAH over items ----
struct Item {
  Box b;
  uint32_t rec;       // the item's record in the reference stream
  bool wild = false;  // an instance under the wild margin (nf_bound.h nf_rho_wild): its path's nodes are flagged
};
struct Node {
  Box b;
  int32_t l = -1, r = -1;
  uint32_t first = 0, count = 0, axis = 0;
  uint32_t force = 0;  // kNfForceL / kNfForceR: that child's subtree holds a wild instance
  uint32_t lo = 0, hi = 0;  // the subtree's items [lo, hi) (build partitions them in place)
  // normal cone of the subtree's generic triangles (nf_bound.h nf_cone_rg):
  // c + 128 per axis, and the code {j (4 bits), k (3 bits)}
  uint8_t cb[3] = {128, 128, 128};
  uint8_t code = kNfConeNone | 7u << 4;
};
struct Tree {
  std::vector<Node> nodes;
  std::vector<Item> items;
  uint32_t depth = 0;  // internal nodes on the longest root-leaf path (stack entries the walk may push)

  // internal levels a balanced tree over cnt items needs (leaves of <= 4)
  static uint32_t min_levels(uint32_t cnt) {
    uint32_t lv = 0;
    for (uint32_t leaves = (cnt + 3) / 4; leaves > 1; leaves = (leaves + 1) / 2) ++lv;
    return lv;
  }
  uint32_t max_depth = ~0u;  // cap on internal levels: below it, median splits where SAH would go deeper

  int32_t build(uint32_t b, uint32_t e, uint32_t internal_depth) {
    Node n;
    Box cb;
    for (uint32_t i = b; i < e; ++i) {
      n.b.grow(items[i].b);
      const float c[3] = {items[i].b.c(0), items[i].b.c(1), items[i].b.c(2)};
      cb.grow(c[0], c[1], c[2]);
    }
    const int32_t id = (int32_t)nodes.size();
    n.lo = b, n.hi = e;
    nodes.push_back(n);
    const uint32_t cnt = e - b;
    constexpr uint32_t kLeaf = 4;
    constexpr int NB = 16;
    double best = (double)cnt * n.b.area();  // leaf cost (one test per item)
    int bk = -1, bs = -1;
    // at the depth cap's edge the subtree is split at the median (balanced)
    const bool capped = max_depth != ~0u && internal_depth + min_levels(cnt) >= max_depth;
    if (cnt > 1 && !capped) {
      for (int k = 0; k < 3; ++k) {
        const float lo = cb.mn[k], ext = cb.mx[k] - cb.mn[k];
        if (!(ext > 0.0f) || !(ext < INFINITY)) continue;
        Box bins[NB];
        uint32_t nb[NB] = {};
        for (uint32_t i = b; i < e; ++i) {
          const int j = std::min(NB - 1, std::max(0, (int)((items[i].b.c(k) - lo) / ext * NB)));
          bins[j].grow(items[i].b);
          nb[j]++;
        }
        Box right[NB];
        uint32_t nr[NB] = {};
        for (int j = NB - 1; j > 0; --j) {
          right[j] = bins[j];
          nr[j] = nb[j];
          if (j + 1 < NB) right[j].grow(right[j + 1]), nr[j] += nr[j + 1];
        }
        Box left;
        uint32_t nl = 0;
        for (int sp = 1; sp < NB; ++sp) {
          left.grow(bins[sp - 1]);
          nl += nb[sp - 1];
          if (!nl || !nr[sp]) continue;
          const double cost = 0.5 * n.b.area() + left.area() * nl + right[sp].area() * nr[sp];
          if (cost < best) best = cost, bk = k, bs = sp;
        }
      }
    }
    if (cnt <= kLeaf && (bk < 0 || capped)) {
      nodes[id].first = b, nodes[id].count = cnt;
      return id;
    }
    uint32_t mid = b + cnt / 2;
    int axis = 0;
    if (bk >= 0) {
      const float lo = cb.mn[bk], ext = cb.mx[bk] - cb.mn[bk];
      auto it = std::partition(items.begin() + b, items.begin() + e, [&](const Item& x) {
        return std::min(NB - 1, std::max(0, (int)((x.b.c(bk) - lo) / ext * NB))) < bs;
      });
      mid = (uint32_t)(it - items.begin());
      axis = bk;
    }
    if (bk < 0 || mid == b || mid == e) {  // no useful split: the median along the longest extent
      int k = 0;
      for (int q = 1; q < 3; ++q)
        if (cb.mx[q] - cb.mn[q] > cb.mx[k] - cb.mn[k]) k = q;
      mid = b + cnt / 2;
      std::nth_element(items.begin() + b, items.begin() + mid, items.begin() + e,
                       [&](const Item& x, const Item& y) { return x.b.c(k) < y.b.c(k); });
      axis = k;
    }
    depth = std::max(depth, internal_depth + 1);
    const int32_t l = build(b, mid, internal_depth + 1), r = build(mid, e, internal_depth + 1);
    nodes[id].l = l, nodes[id].r = r, nodes[id].axis = (uint32_t)axis;
    return id;
  }
  // every node flags its child whose subtree holds a wild item (the nodes on
  // the path from the root to each wild leaf thicken their boxes by the wild
  // margin too); returns whether node n's subtree holds one
  bool mark_forced(int32_t n) {
    Node& x = nodes[n];
    if (x.l < 0) {
      for (uint32_t i = 0; i < x.count; ++i)
        if (items[x.first + i].wild) return true;
      return false;
    }
    const bool wl = mark_forced(x.l), wr = mark_forced(x.r);
    nodes[n].force = (wl ? kNfForceL : 0u) | (wr ? kNfForceR : 0u);
    return wl || wr;
  }
};

struct Builder {
  const mrt_scene_desc& d;
  HostScene& s;
  std::string& err;
  std::vector<uint32_t>& w;  // s.slots
  // BLAS: reference region begin -> NF root record (patched into instance/model records)
  std::unordered_map<uint32_t, uint32_t> blas_root;
  std::vector<std::pair<uint32_t, uint32_t>> patches;  // (NF instance/model record, reference BLAS begin)

  uint32_t n_slots() const { return (uint32_t)(w.size() / 4); }
  uint32_t push(uint32_t a, uint32_t b, uint32_t c, uint32_t dd) {
    const uint32_t i = n_slots();
    w.push_back(a), w.push_back(b), w.push_back(c), w.push_back(dd);
    return i;
  }

  // Quantized frame of a node over its children's boxes a, b (layout.h NF
  // NODE): origin = the union's min, per axis the smallest step 2^e with
  // 254 steps covering the union (one step of slack for the rounding of the
  // double arithmetic below, whose error is < 2^-40 of a step); planes rounded
  // outward. false: a box is not finite (or past the exponent range).
  // The origin of axis k is the largest float at or below the children's
  // minimum whose low mantissa byte is cb[k] (the node's cone component,
  // nf_bound.h): the planes are quantized from that exact float, so the byte
  // costs at most 2^-15 of |origin| of range, never tightness.
  static float origin_with_byte(float v, uint8_t byte) {
    if (!(fabsf(v) >= 0x1p-100f)) v = fminf(v, -0x1p-100f);  // zero or tiny: a normal origin below it
    uint32_t u = f2u(v), c = (u & ~0xFFu) | byte;
    if (u2f(c) > v) c = v > 0.0f ? c - 0x100u : c + 0x100u;  // one step of 256 ulps further down
    return u2f(c);
  }
  static bool quantize(const Box& a, const Box& b, const uint8_t cb[3], uint32_t o[3], uint32_t& ew, uint32_t q[3]) {
    uint8_t bytes[12];
    ew = 0;
    for (int k = 0; k < 3; ++k) {
      const float mn = fminf(a.mn[k], b.mn[k]);
      const double hi = std::max((double)a.mx[k], (double)b.mx[k]);
      if (!(fabsf(mn) < INFINITY) || !(fabs(hi) < INFINITY)) return false;
      const float org = origin_with_byte(mn, cb[k]);
      if (!(fabsf(org) < INFINITY) || !(org <= mn) || (f2u(org) & 0xFFu) != cb[k]) return false;
      const double ext = hi - (double)org;
      int e = kNfExpMin;
      while (std::ldexp(254.0, e) < ext) ++e;
      if (e > 127) return false;
      const double step = std::ldexp(1.0, e);
      auto lo_q = [&](float v) {
        return (uint8_t)std::max(0.0, std::floor(((double)v - org) / step - 0x1p-30));
      };
      auto hi_q = [&](float v) {
        return (uint8_t)std::min(255.0, std::ceil(((double)v - org) / step + 0x1p-30));
      };
      o[k] = f2u(org);
      ew |= (uint32_t)(e + 127) << (8 * k);
      bytes[k] = lo_q(a.mn[k]);
      bytes[3 + k] = hi_q(a.mx[k]);
      bytes[6 + k] = lo_q(b.mn[k]);
      bytes[9 + k] = hi_q(b.mx[k]);
    }
    for (int j = 0; j < 3; ++j)
      q[j] = bytes[4 * j] | (uint32_t)bytes[4 * j + 1] << 8 | (uint32_t)bytes[4 * j + 2] << 16 |
             (uint32_t)bytes[4 * j + 3] << 24;
    return true;
  }

  uint32_t rec_slots(uint32_t r) const { return kind_of(w, r) == KIND_TRI ? 3u : 2u; }
  // slots of the record a child of a node starts with (a node, or its leaf's first object)
  uint32_t child_slots(const Tree& t, const Node& c) const { return c.l < 0 ? rec_slots(t.items[c.first].rec) : 2u; }

  // writes leaf n's objects: the first at `at` (reserved), the rest appended
  void emit_leaf(const Tree& t, const Node& n, uint32_t at) {
    uint32_t pos = at;
    for (uint32_t k = 0; k < n.count; ++k) {
      const uint32_t r = t.items[n.first + k].rec;
      if (k > 0) {
        pos = n_slots();
        for (uint32_t z = 0; z < 4 * rec_slots(r); ++z) w.push_back(0);
      }
      const uint32_t next = k + 1 == n.count ? kNfPop : std::max(n_slots(), pos + rec_slots(r));
      copy_record(r, pos, next);
    }
  }
  // node n's record at `at` (reserved): its children's records follow as a
  // pair, then their subtrees (left first)
  bool emit_node(const Tree& t, const Node& n, uint32_t at) {
    const Node& L = t.nodes[n.l];
    const Node& R = t.nodes[n.r];
    const uint32_t lsz = child_slots(t, L), rsz = child_slots(t, R), base = n_slots();
    for (uint32_t z = 0; z < 4 * (lsz + rsz); ++z) w.push_back(0);
    uint32_t o[3], ew, q[3];
    if (!quantize(L.b, R.b, n.cb, o, ew, q)) return false;
    if (lsz < 2 || lsz > 3) return false;  // a node (2 slots) or a leaf's first record (2 or 3)
    uint32_t* rec = &w[4 * (size_t)at];
    rec[0] = o[0], rec[1] = o[1], rec[2] = o[2], rec[3] = ew | (lsz - 2) << 24 | (uint32_t)n.code << 25;
    rec[4] = q[0], rec[5] = q[1], rec[6] = q[2], rec[7] = kBoxFlag | n.force | base;
    s.nf_boxes++;
    for (const auto& [c, pos] : {std::pair<const Node*, uint32_t>{&L, base}, {&R, base + lsz}}) {
      if (c->l < 0)
        emit_leaf(t, *c, pos);
      else if (!emit_node(t, *c, pos))
        return false;
    }
    return true;
  }
  // emits tree t; returns its root record (a node, or a leaf's first object),
  // ~0u when a box cannot be quantized
  uint32_t emit(const Tree& t) {
    const Node& root = t.nodes[0];
    const uint32_t at = n_slots();
    const uint32_t sz = child_slots(t, root);
    for (uint32_t z = 0; z < 4 * sz; ++z) w.push_back(0);
    if (root.l < 0) {
      emit_leaf(t, root, at);
      return at;
    }
    return emit_node(t, root, at) ? at : ~0u;
  }
  // reference record `r` copied to slot `at` with the leaf's successor `next`
  void copy_record(uint32_t r, uint32_t at, uint32_t next) {
    const uint32_t k = kind_of(w, r);
    for (uint32_t q = 0; q < 4 * rec_slots(r); ++q) w[4 * (size_t)at + q] = w[4 * (size_t)r + q];
    switch (k) {
      case KIND_TRI: w[4 * (at + 2) + 3] = next; break;
      case KIND_SPHERE: w[4 * (at + 1) + 1] = next; break;
      case KIND_INST:
      case KIND_MODEL:
        w[4 * at + 2] = next;
        w[4 * (at + 1)] = s.vnf_leaf[2 * (size_t)vnf_slot(r)];  // its reference world parent (path.h nf_finish)
        patches.push_back({at, w[4 * r + 1]});  // the reference BLAS region it enters
        if (wild_term.count(r)) wild_at.push_back({at, r});
        break;
      default: break;
    }
  }

  // reference parents and keys of the objects of a region (left-first order)
  bool ref_order(uint32_t first, bool world, std::vector<uint32_t>& objects) {
    std::vector<uint32_t> kids, top;
    level(w, first, ~0u, top);
    struct F {
      uint32_t rec, parent;
    };
    std::vector<F> st;
    for (size_t k = top.size(); k-- > 0;) st.push_back({top[k], kNoParent});
    uint32_t key = 0;
    while (!st.empty()) {
      const F f = st.back();
      st.pop_back();
      if (is_box(w, f.rec)) {
        level(w, kind_of(w, f.rec) & ~kBoxFlag, skip_of(w, f.rec), kids);
        for (size_t k = kids.size(); k-- > 0;) st.push_back({kids[k], f.rec});
        continue;
      }
      const uint32_t kd = kind_of(w, f.rec);
      uint32_t slot;
      switch (kd) {
        case KIND_SPHERE: slot = s.vnf_base[VNF_SPHERE] + w[4 * (f.rec + 1)]; break;
        case KIND_TRI: slot = s.vnf_base[VNF_TRI] + (w[4 * (f.rec + 1) + 2] & kTriIdMask); break;
        case KIND_INST: slot = s.vnf_base[VNF_INST] + w[4 * f.rec]; break;
        case KIND_MODEL: slot = s.vnf_base[VNF_MODEL] + w[4 * f.rec]; break;
        default:
          s.nf_note = "a volume in the world";
          return false;
      }
      if (s.vnf_leaf[2 * slot] != 0xFFFFFFFEu) {
        s.nf_note = "an object referenced twice";
        return false;
      }
      s.vnf_leaf[2 * slot] = f.parent;
      s.vnf_leaf[2 * slot + 1] = (world && kd == KIND_TRI ? kWorldKey : 0u) | key++;
      if (key >= kWorldKey) {
        s.nf_note = "more than 2^31 objects in a region";
        return false;
      }
      objects.push_back(f.rec);
    }
    return true;
  }

  // ---- boxes and bounds (nf_bound.h) ----
  std::unordered_map<uint32_t, size_t> region_of;  // reference BLAS region begin -> blas_regions index
  std::vector<Box> blas_box;                       // each BLAS's NF root box (object space, padded)
  std::vector<TriBound> blas_bound;                // each BLAS's worst triangle bound (max of a0, a1, k1)
  TriBound world_tri;                              // world triangles and model BLAS triangles
  double r_min = INFINITY, r_max = 0;
  Box sph_box;                                     // the world spheres' union
  struct InstTerm {
    double w0, w1, b0, b1, ko;
  };
  // wild instances: reference record -> (world box, instance term), and their
  // NF leaf records (slot0.w patched to their WILD entry)
  std::unordered_map<uint32_t, std::pair<Box, InstTerm>> wild_term;
  std::vector<float> gen_extent;  // each generic triangle's largest box extent (the cones' threshold, NfBound::kcmin)
  std::vector<std::pair<uint32_t, uint32_t>> wild_at;  // (NF instance record, reference record)

  static void grow_bound(TriBound& m, const TriBound& b) {
    m.a0 = std::max(m.a0, b.a0), m.a1 = std::max(m.a1, b.a1), m.k1 = std::max(m.k1, b.k1);
  }
  static void pad_abs(Box& b, double p) {
    for (int k = 0; k < 3; ++k) b.mn[k] = f_down((double)b.mn[k] - p), b.mx[k] = f_up((double)b.mx[k] + p);
  }

  // A leaf object's NF box: its geometry, every hit it can return within
  // the size-proportional pads of its bound (the distance-proportional part
  // is the walk's margin, nf_bound.h).
  Box object_box(uint32_t r, TriBound* tb) {
    Box b;
    const uint32_t* q = &w[4 * (size_t)r];
    switch (kind_of(w, r)) {
      case KIND_SPHERE: {
        // the ball, plus the bound's terms proportional to the radius (90.2u |r|)
        const double rad = std::fabs((double)u2f(q[3])) * (1.0 + 0x1p-17);
        for (int k = 0; k < 3; ++k) b.mn[k] = f_down(u2f(q[k]) - rad), b.mx[k] = f_up(u2f(q[k]) + rad);
        pad_box(b, 0.0f);
        break;
      }
      case KIND_TRI: {
        const mrt_triangle& t = d.triangles[q[6] & kTriIdMask];
        b.grow(t.a[0], t.a[1], t.a[2]);
        b.grow(t.b[0], t.b[1], t.b[2]);
        b.grow(t.c[0], t.c[1], t.c[2]);
        const float ab[3] = {u2f(q[3]), u2f(q[4]), u2f(q[5])}, ac[3] = {u2f(q[8]), u2f(q[9]), u2f(q[10])};
        const TriBound tbd = tri_bound(ab, ac);
        if (tb) grow_bound(*tb, tbd);
        if (tbd.a1 > 0) gen_extent.push_back(std::max(b.mx[0] - b.mn[0], std::max(b.mx[1] - b.mn[1], b.mx[2] - b.mn[2])));
        pad_box(b, 0.0f);
        pad_abs(b, tbd.pad);
        break;
      }
      case KIND_INST:
      case KIND_MODEL: {
        auto it = region_of.find(q[1]);  // the reference BLAS region it enters
        if (it == region_of.end()) {
          b.grow(-INFINITY, -INFINITY, -INFINITY);
          b.grow(INFINITY, INFINITY, INFINITY);
          break;
        }
        const Box& ob = blas_box[it->second];
        if (kind_of(w, r) == KIND_MODEL) {
          b = ob;
          break;
        }
        // the hull of the transformed corners, in double (each product of
        // two floats exact, the sum's rounding added) and rounded outward
        const float* f = d.instances[q[0]].fwd;  // column-major 4x4 (M4::transform)
        for (int c = 0; c < 8; ++c) {
          const double x = c & 1 ? ob.mx[0] : ob.mn[0], y = c & 2 ? ob.mx[1] : ob.mn[1], z = c & 4 ? ob.mx[2] : ob.mn[2];
          for (int k = 0; k < 3; ++k) {
            const double t0 = (double)f[k] * x, t1 = (double)f[4 + k] * y, t2 = (double)f[8 + k] * z, t3 = f[12 + k];
            const double v = ((t0 + t1) + t2) + t3;
            const double e = 0x1p-50 * (std::fabs(t0) + std::fabs(t1) + std::fabs(t2) + std::fabs(t3));
            b.mn[k] = std::min(b.mn[k], f_down(v - e)), b.mx[k] = std::max(b.mx[k], f_up(v + e));
          }
        }
        break;
      }
      default:
        break;
    }
    return b;
  }

  // The world-space terms an instance's object-space rounding contributes
  // (DESIGN.md §4): F = fwd, G = inv (the stored f32 matrices), the object
  // ray RN(G o), RN(G d) and the hit mapped back by F.
  InstTerm inst_term(uint32_t id, const TriBound& ob) const {
    const float* F = d.instances[id].fwd;
    const float* G = d.instances[id].inv;
    double nf = 0, ng = 0, psi = 0, gt = 0, ft = 0;
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        nf += (double)F[4 * c + r] * F[4 * c + r];
        ng += (double)G[4 * c + r] * G[4 * c + r];
        double m = 0;  // (F_L G_L)_rc
        for (int k = 0; k < 3; ++k) m += (double)F[4 * k + r] * G[4 * c + k];
        m -= r == c ? 1.0 : 0.0;
        psi += m * m;
      }
    nf = std::sqrt(nf), ng = std::sqrt(ng), psi = std::sqrt(psi) + 0x1p-48 * nf * ng;
    double pt = 0;
    for (int r = 0; r < 3; ++r) {
      double v = F[12 + r];
      for (int k = 0; k < 3; ++k) v += (double)F[4 * k + r] * G[12 + k];
      pt += v * v;
      gt += (double)G[12 + r] * G[12 + r];
      ft += (double)F[12 + r] * F[12 + r];
    }
    pt = std::sqrt(pt) + 0x1p-48 * (nf * std::sqrt(gt) + std::sqrt(ft));
    gt = std::sqrt(gt);
    const double cond = nf * ng, g3 = gam(3), g4 = gam(4);
    InstTerm m;
    m.w0 = cond * (1 + g3) * ob.a0 + psi + g3 * cond;
    m.w1 = cond * (1 + g3) * (1 + g3) * ob.a1 * ng;
    m.b1 = psi + g4 * cond;
    m.b0 = pt + g4 * nf * gt;
    m.ko = ob.k1 * ng * (1 + g3);
    return m;
  }
  // a wild instance: its terms would dominate the world margin; the walk
  // never culls it (and its subtree) instead
  static bool wild(const InstTerm& m) { return m.w0 > 0x1p-14 || m.w1 > 0x1p-14 || m.b1 > 0x1p-14; }

  // vnf_leaf slot of a leaf object's record
  uint32_t vnf_slot(uint32_t r) const {
    const uint32_t* q = &w[4 * (size_t)r];
    switch (kind_of(w, r)) {
      case KIND_SPHERE: return s.vnf_base[VNF_SPHERE] + q[4];
      case KIND_TRI: return s.vnf_base[VNF_TRI] + (q[6] & kTriIdMask);
      case KIND_INST: return s.vnf_base[VNF_INST] + q[0];
      default: return s.vnf_base[VNF_MODEL] + q[0];
    }
  }
  void keep_box(uint32_t r, const Box& b) {
    if (!s.keep_nf_boxes) return;
    float* p = &s.nf_leaf_box[6 * (size_t)vnf_slot(r)];
    for (int k = 0; k < 3; ++k) p[k] = b.mn[k], p[3 + k] = b.mx[k];
  }

  // Normal cones of every internal node of tree t (nf_bound.h nf_cone_rg):
  // over the node's generic triangles, an integer axis c (components within
  // +-127, stored as c + 128) near the mean of their normals (each up to
  // sign), the chord chi of the widest normal from it (in |c| units, plus the
  // computed determinant's error and the evaluation's rounding), and the
  // exponent k with |c| M <= 2^(k+6). A node holding an instance or model
  // whose BLAS has generic triangles (their world-space rounding is the
  // instance term, not a cone's) or a cone wider than a hemisphere's chord
  // gets none: the node keeps the ray's generic term.
  void fit_cones(Tree& t) {
    struct N {
      double n[3], m;
      int kind;  // 0 none, 1 generic triangle, 2 poison (generic instance / model)
    };
    std::vector<N> it(t.items.size());
    for (size_t i = 0; i < t.items.size(); ++i) {
      const uint32_t r = t.items[i].rec;
      N& x = it[i];
      x.kind = 0;
      const uint32_t kd = kind_of(w, r);
      if (kd == KIND_TRI) {
        const float ab[3] = {u2f(w[4 * (size_t)r + 3]), u2f(w[4 * (size_t)r + 4]), u2f(w[4 * (size_t)r + 5])};
        const float ac[3] = {u2f(w[4 * (size_t)r + 8]), u2f(w[4 * (size_t)r + 9]), u2f(w[4 * (size_t)r + 10])};
        if (!(tri_bound(ab, ac).a1 > 0)) continue;
        // N = ab x ac: each product of two floats exact in double, one rounding per component
        const double nn[3] = {(double)ab[1] * ac[2] - (double)ab[2] * ac[1], (double)ab[2] * ac[0] - (double)ab[0] * ac[2],
                              (double)ab[0] * ac[1] - (double)ab[1] * ac[0]};
        const double ln = norm3(nn);
        const double dab[3] = {ab[0], ab[1], ab[2]}, dac[3] = {ac[0], ac[1], ac[2]};
        x.kind = 2;  // a degenerate generic triangle: no cone can bound it
        if (!(ln > 0) || !(ln < INFINITY)) continue;
        x.kind = 1;
        for (int k = 0; k < 3; ++k) x.n[k] = nn[k] / ln;
        x.m = norm3(dab) * norm3(dac) / ln * (1.0 + 1e-9);
      } else if (kd == KIND_INST || kd == KIND_MODEL) {
        auto rg = region_of.find(w[4 * (size_t)r + 1]);
        if (rg != region_of.end() && blas_bound[rg->second].a1 > 0) x.kind = 2;
      }
    }
    const double u = kU;
    for (Node& nd : t.nodes) {
      if (nd.l < 0) continue;
      nd.cb[0] = nd.cb[1] = nd.cb[2] = 128;
      nd.code = (uint8_t)(kNfConeNone | 7u << 4);
      bool poison = false, any = false;
      double ax[3] = {0, 0, 0};
      for (uint32_t i = nd.lo; i < nd.hi && !poison; ++i) {
        if (it[i].kind == 2) poison = true;
        if (it[i].kind != 1) continue;
        if (!any) ax[0] = it[i].n[0], ax[1] = it[i].n[1], ax[2] = it[i].n[2], any = true;
      }
      if (poison) continue;
      if (!any) {  // no generic triangle below: any cone is valid; the narrowest slope is k = 0
        nd.cb[0] = 255, nd.code = 0;  // c = (127, 0, 0), chi = 1/8
        continue;
      }
      for (int pass = 0; pass < 2; ++pass) {  // the mean of the normals aligned to the current axis
        double sm[3] = {0, 0, 0};
        for (uint32_t i = nd.lo; i < nd.hi; ++i) {
          if (it[i].kind != 1) continue;
          const double* n = it[i].n;
          const double sg = n[0] * ax[0] + n[1] * ax[1] + n[2] * ax[2] < 0 ? -1.0 : 1.0;
          for (int k = 0; k < 3; ++k) sm[k] += sg * n[k];
        }
        const double l = norm3(sm);
        if (!(l > 0)) break;
        for (int k = 0; k < 3; ++k) ax[k] = sm[k] / l;
      }
      const double mx = std::max(std::fabs(ax[0]), std::max(std::fabs(ax[1]), std::fabs(ax[2])));
      if (!(mx > 0)) continue;
      int c[3];
      for (int k = 0; k < 3; ++k) c[k] = (int)std::lround(127.0 * ax[k] / mx);
      const double dc[3] = {(double)c[0], (double)c[1], (double)c[2]};
      const double lc = norm3(dc);
      double chord = 0, M = 0;
      for (uint32_t i = nd.lo; i < nd.hi; ++i) {
        if (it[i].kind != 1) continue;
        const double* n = it[i].n;
        double dm = 0, dp = 0;
        for (int k = 0; k < 3; ++k) {
          const double q = dc[k] / lc;
          dm += (n[k] - q) * (n[k] - q), dp += (n[k] + q) * (n[k] + q);
        }
        chord = std::max(chord, std::sqrt(std::min(dm, dp)));
        M = std::max(M, it[i].m);
      }
      if (!(chord < 1.0)) continue;  // wider than 60 degrees: the grazing band is most of the sphere
      const double chi = lc * chord * (1.0 + 1e-9) + 7.3 * u * lc * M + 3000.0 * u;
      int j = 3 + (int)std::ceil(std::log2(chi));
      while (std::ldexp(1.0, j - 3) < chi) ++j;
      j = std::max(j, 0);
      int kk = std::max(0, (int)std::ceil(std::log2(lc * M)) - 6);
      while (std::ldexp(1.0, kk + 6) < lc * M) ++kk;
      if (j >= (int)kNfConeNone || kk > 7) continue;
      for (int k = 0; k < 3; ++k) nd.cb[k] = (uint8_t)(c[k] + 128);
      nd.code = (uint8_t)(j | kk << 4);
      s.nf_cones++;
    }
  }

  // the per-scene rule's verdict before building (render.hip apply_options):
  // the reference walk for a generic-triangle term or a big instanced world
  // (round 6: generic triangles no longer decline it — the normal cones and
  // the wild instances' own tests made mesh_ply's near-first walk the faster)
  bool auto_declines() const { return d.n_instances > 1000 && (size_t)n_slots() * 16 > ((size_t)16 << 20); }

  bool run() {
    s.nf_ok = false;
    s.nf_first_slot = n_slots();
    if (s.trav_rng) return (s.nf_note = "the traversal draws random numbers (Volume, Mix alpha)", true);
    if (s.nf_build == kNfBuildNever) return (s.nf_note = "not built (option traversal = REFERENCE at upload)", true);
    if (s.nf_build == kNfBuildAuto && auto_declines())
      return (s.nf_note = "not built: the per-scene rule walks the reference's way (a big instanced world; "
                          "option traversal = NEAR_FIRST at upload builds them)", true);
    s.vnf_base[VNF_SPHERE] = 0;
    s.vnf_base[VNF_TRI] = d.n_spheres;
    s.vnf_base[VNF_INST] = d.n_spheres + d.n_triangles;
    s.vnf_base[VNF_MODEL] = d.n_spheres + d.n_triangles + d.n_instances;
    s.vnf_leaf.assign(2 * ((size_t)d.n_spheres + d.n_triangles + d.n_instances + d.n_models), 0xFFFFFFFEu);
    std::vector<uint32_t> world_objs;
    if (!ref_order(s.world_begin, true, world_objs)) return true;
    if (world_objs.empty()) return (s.nf_note = "an empty world", true);
    std::vector<std::vector<uint32_t>> blas_objs(s.blas_regions.size());
    if (s.keep_nf_boxes) {
      s.nf_leaf_box.assign(3 * s.vnf_leaf.size(), NAN);
      s.nf_inst_wild.assign(d.n_instances, 0);
    }
    for (size_t k = 0; k < s.blas_regions.size(); ++k) {
      region_of[s.blas_regions[k].begin] = k;
      if (!ref_order(s.blas_regions[k].begin, false, blas_objs[k])) return true;
    }
    // which BLAS regions models / instances enter (world objects)
    std::vector<uint8_t> by_model(s.blas_regions.size(), 0), by_inst(s.blas_regions.size(), 0);
    for (uint32_t r : world_objs) {
      const uint32_t kd = kind_of(w, r);
      if (kd != KIND_INST && kd != KIND_MODEL) continue;
      auto it = region_of.find(w[4 * (size_t)r + 1]);
      if (it != region_of.end()) (kd == KIND_MODEL ? by_model : by_inst)[it->second] = 1;
    }
    // trees; stack entries the walk may need: a far child per internal level
    // of the world tree, an instance's successor and its return marker, a far
    // child per BLAS level — kept within kNfStack by capping the depth (median
    // splits at the cap's edge): the BLAS trees first, leaving the world tree
    // at least the levels a balanced tree over its objects needs (and one for
    // the wild instances' subtree)
    const uint32_t has_blas = s.blas_regions.empty() ? 0 : 2;
    std::vector<Tree> blas(s.blas_regions.size());
    blas_box.assign(s.blas_regions.size(), Box{});
    blas_bound.assign(s.blas_regions.size(), TriBound{});
    uint32_t blas_depth = 0;
    const uint32_t world_min = Tree::min_levels((uint32_t)world_objs.size());
    if (world_min + has_blas > kNfStack) return (s.nf_note = "too many world objects for the walk's stack", true);
    for (size_t k = 0; k < blas.size(); ++k) {
      for (uint32_t r : blas_objs[k]) {
        blas[k].items.push_back({object_box(r, &blas_bound[k]), r});
        keep_box(r, blas[k].items.back().b);
      }
      if (blas[k].items.empty()) continue;
      blas[k].max_depth = kNfStack - 2 - world_min;
      blas[k].build(0, (uint32_t)blas[k].items.size(), 0);
      blas_depth = std::max(blas_depth, blas[k].depth);
      blas_box[k] = blas[k].nodes[0].b;
      if (by_model[k]) grow_bound(world_tri, blas_bound[k]);
    }
    // the world's items: wild instances first
    Tree world;
    NfBound& B = s.nfb;
    B = NfBound{};
    double aw0 = 0, aw1 = 0, bw0 = 0, bw1 = 0, ko1 = 0, ao0 = 0, ao1 = 0, orad = 0;
    std::vector<Item> wild_items, items;
    Box gen_box;  // the world boxes of generic triangles (world, model or instanced): the a1 term's ball
    // in a world of few instances, one whose absolute term exceeds 2^-14 (a
    // 1000x floor's 4.6e-4: the rounding of its object-space origin, scaled
    // back) is wild too (round 6): that term would thicken every node of the
    // primitives' trees (mesh_ply's 1M triangles of 0.01), while a wild
    // instance costs one box test of its own where the walk reaches it
    uint32_t n_world_inst = 0;
    for (uint32_t r : world_objs) n_world_inst += kind_of(w, r) == KIND_INST;
    const bool few = n_world_inst <= kNfWildFew;
    for (uint32_t r : world_objs) {
      const uint32_t kd = kind_of(w, r);
      TriBound tb;
      const Box b = object_box(r, kd == KIND_TRI ? &tb : nullptr);
      keep_box(r, b);
      if (kd == KIND_TRI) grow_bound(world_tri, tb);
      bool generic = tb.a1 > 0;
      if (kd == KIND_INST || kd == KIND_MODEL) {
        auto it = region_of.find(w[4 * (size_t)r + 1]);
        generic = it != region_of.end() && blas_bound[it->second].a1 > 0;
      }
      if (kd == KIND_SPHERE) {
        const double rad = std::fabs((double)u2f(w[4 * (size_t)r + 3]));
        r_min = std::min(r_min, rad), r_max = std::max(r_max, rad);
        Box sb;
        for (int k = 0; k < 3; ++k) sb.mn[k] = f_down(u2f(w[4 * (size_t)r + k]) - rad), sb.mx[k] = f_up(u2f(w[4 * (size_t)r + k]) + rad);
        sph_box.grow(sb);
      }
      if (kd == KIND_INST) {
        auto it = region_of.find(w[4 * (size_t)r + 1]);
        const TriBound ob = it == region_of.end() ? TriBound{} : blas_bound[it->second];
        const InstTerm m = inst_term(w[4 * (size_t)r], ob);
        ko1 = std::max(ko1, m.ko);
        if (it != region_of.end()) {
          const Box& bb = blas_box[it->second];
          for (int c = 0; c < 8; ++c) {
            const double x = c & 1 ? bb.mx[0] : bb.mn[0], y = c & 2 ? bb.mx[1] : bb.mn[1], z = c & 4 ? bb.mx[2] : bb.mn[2];
            orad = std::max(orad, std::sqrt(x * x + y * y + z * z));
          }
          ao0 = std::max(ao0, ob.a0), ao1 = std::max(ao1, ob.a1);
        }
        if (wild(m) || (few && m.b0 > 0x1p-14)) {
          wild_items.push_back({b, r, true});
          wild_term[r] = {b, m};
          s.nf_wild++;
          if (s.keep_nf_boxes) s.nf_inst_wild[w[4 * (size_t)r]] = 1;
          continue;
        }
        aw0 = std::max(aw0, m.w0), aw1 = std::max(aw1, m.w1), bw0 = std::max(bw0, m.b0), bw1 = std::max(bw1, m.b1);
      }
      if (generic) gen_box.grow(b);
      items.push_back({b, r});
    }
    aw0 = std::max(aw0, world_tri.a0), aw1 = std::max(aw1, world_tri.a1);
    if (r_min < 0x1p-60) return (s.nf_note = "a sphere too small for the walk's rounding bound", true);
    world.items = items;
    world.items.insert(world.items.end(), wild_items.begin(), wild_items.end());
    world.max_depth = kNfStack - (has_blas ? 2 + blas_depth : 0);
    world.build(0, (uint32_t)world.items.size(), 0);
    if (!wild_items.empty()) world.mark_forced(0);
    if (aw1 > 0 || ao1 > 0)  // generic triangles somewhere: every tree's nodes get their cones
      for (Tree* t : [&] {
             std::vector<Tree*> v{&world};
             for (Tree& b : blas) v.push_back(&b);
             return v;
           }())
        fit_cones(*t);
    s.nf_stack_need = world.depth + (has_blas ? 2 + blas_depth : 0);
    if (s.nf_stack_need > kNfStack) return (s.nf_note = "trees deeper than the walk's stack", true);
    // the constants (rounded up) of nf_bound.h
    auto ball = [](const Box& b, float c[3], float& rr) {
      double r2 = 0;
      for (int k = 0; k < 3; ++k) {
        const double m = 0.5 * ((double)b.mn[k] + (double)b.mx[k]);
        c[k] = (float)m;
        const double e = std::max(std::fabs((double)b.mx[k] - c[k]), std::fabs(c[k] - (double)b.mn[k]));
        r2 += e * e;
      }
      rr = f_up(std::sqrt(r2) * (1 + 0x1p-40));
    };
    // the a0 term's cap: a ball over the objects the world margin covers (the
    // wild ones have their own)
    Box wb;
    for (const Item& it : items) wb.grow(it.b);
    if (items.empty()) wb = world.nodes[0].b;
    for (int k = 0; k < 3; ++k)
      if (!(std::fabs(wb.mn[k]) < INFINITY && std::fabs(wb.mx[k]) < INFINITY))
        return (s.nf_note = "a box the node format cannot hold (not finite)", true);
    ball(wb, B.wc, B.wr);
    if (aw1 > 0) ball(gen_box, B.gc, B.gr);
    B.aw0 = f_up(aw0), B.aw1 = f_up(aw1), B.bw0 = f_up(bw0 + 0x1p-90), B.bw1 = f_up(bw1);
    B.kw1 = f_up(world_tri.k1), B.ko1 = f_up(ko1);
    B.ao0 = f_up(ao0), B.ao1 = f_up(ao1), B.orad = f_up(orad);
    B.kmax = kNfKappaMax;
    // the cones' slope constant (nf_bound.h nf_cone_rg): 1.0001 * 24u * 2^6 /
    // (1 - kappa max), with 2^-17 for rcp (an ulp), the kd product and d2's
    // roundings, and G's
    B.kc = (aw1 > 0 || ao1 > 0) ? f_up(1.0001 * 24.0 * kU * 64.0 / (1.0 - 1.01 * (double)kNfKappaMax) * (1.0 + 0x1p-17))
                                : 0.0f;
    B.kcmin = 0.0f;
    if (!gen_extent.empty()) {
      std::nth_element(gen_extent.begin(), gen_extent.begin() + gen_extent.size() / 2, gen_extent.end());
      B.kcmin = std::ldexp(gen_extent[gen_extent.size() / 2], -6);
    }
    if (r_max > 0) {
      ball(sph_box, B.sc, B.sr);
      B.s51 = f_up(51.2 * kU / r_min), B.s28 = f_up(27.8 * kU), B.s130 = f_up(130.2 * kU), B.s11 = f_up(11.2 * kU * r_max);
    } else {
      B.sr = -1.0f;
    }
    s.nf_world = emit(world);
    if (s.nf_world == ~0u) return (s.nf_note = "a box the node format cannot hold (not finite)", true);
    for (size_t k = 0; k < blas.size(); ++k) {
      if (blas[k].items.empty()) continue;
      const uint32_t root = emit(blas[k]);
      if (root == ~0u) return (s.nf_note = "a box the node format cannot hold (not finite)", true);
      blas_root[s.blas_regions[k].begin] = root;
    }
    // each wild instance's WILD entry (layout.h, nf_bound.h NfWild): its
    // world box, its own instance term, a ball holding the box
    for (auto& [at, r] : wild_at) {
      const auto& [b, m] = wild_term.at(r);
      bool finite = true;
      for (int k = 0; k < 3; ++k) finite = finite && std::fabs(b.mn[k]) < INFINITY && std::fabs(b.mx[k]) < INFINITY;
      if (!finite) continue;  // no entry: the instance is entered whenever its forced path is walked
      float c[3], rr;
      ball(b, c, rr);
      const uint32_t e = push(f2u(b.mn[0]), f2u(b.mn[1]), f2u(b.mn[2]), f2u(b.mx[0]));
      push(f2u(b.mx[1]), f2u(b.mx[2]), f2u(f_up(m.w0)), f2u(f_up(m.w1)));
      push(f2u(f_up(m.b0 + 0x1p-90)), f2u(f_up(m.b1)), f2u(c[0]), f2u(c[1]));
      push(f2u(c[2]), f2u(rr), 0, 0);
      w[4 * (size_t)at + 3] = e;
    }
    for (auto& [rec, ref_blas] : patches) {
      auto it = blas_root.find(ref_blas);
      if (it == blas_root.end()) return (s.nf_note = "an instance of an empty BLAS", true);
      w[4 * rec + 1] = it->second;
    }
    if (n_slots() > kNfIdx) return (s.nf_note = "record stream past 2^28 slots", true);
    s.nf_ok = true;
    return true;
  }
};

}  // namespace

bool build_nf_trees(const mrt_scene_desc& d, HostScene& s, std::string& err) {
  Builder b{d, s, err, s.slots, {}, {}};
  const size_t keep = s.slots.size();
  const bool ok = b.run();
  if (!s.nf_ok) {  // no NF trees: drop whatever was appended
    s.slots.resize(keep);
    s.nf_boxes = 0;
    s.nf_wild = 0;
    s.nf_cones = 0;
    s.vnf_leaf.clear();
  }
  return ok;
}

}  // namespace mrt
