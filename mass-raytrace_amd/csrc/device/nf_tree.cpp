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

// NF triangle boxes are thickened by this fraction of the triangle's extent
// (object_box): grazing rays, whose computed t can undercut the plane far
// more than the culling margin, then meet the box before the plane
constexpr float kTriThick = 0x1p-6f;

// ---- binned SAH over items ----
struct Item {
  Box b;
  uint32_t rec;  // the item's record in the reference stream
};
struct Node {
  Box b;
  int32_t l = -1, r = -1;
  uint32_t first = 0, count = 0, axis = 0;
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
  static bool quantize(const Box& a, const Box& b, uint32_t o[3], uint32_t& ew, uint32_t q[3]) {
    uint8_t bytes[12];
    ew = 0;
    for (int k = 0; k < 3; ++k) {
      const float org = fminf(a.mn[k], b.mn[k]);
      const double hi = std::max((double)a.mx[k], (double)b.mx[k]);
      if (!(fabsf(org) < INFINITY) || !(fabs(hi) < INFINITY)) return false;
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
    if (!quantize(L.b, R.b, o, ew, q)) return false;
    uint32_t* rec = &w[4 * (size_t)at];
    rec[0] = o[0], rec[1] = o[1], rec[2] = o[2], rec[3] = ew | lsz << 24;
    rec[4] = q[0], rec[5] = q[1], rec[6] = q[2], rec[7] = kBoxFlag | base;
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
        patches.push_back({at, w[4 * r + 1]});  // the reference BLAS region it enters
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

  Box object_box(uint32_t r) {
    Box b;
    const uint32_t* q = &w[4 * (size_t)r];
    switch (kind_of(w, r)) {
      case KIND_SPHERE: {
        const float rad = fabsf(u2f(q[3]));
        for (int k = 0; k < 3; ++k) b.mn[k] = u2f(q[k]) - rad, b.mx[k] = u2f(q[k]) + rad;
        pad_box(b, 0x1p-20f);  // the rounded c +- r, and the sphere test's own rounding
        break;
      }
      case KIND_TRI: {
        const mrt_triangle& t = d.triangles[q[6] & kTriIdMask];
        b.grow(t.a[0], t.a[1], t.a[2]);
        b.grow(t.b[0], t.b[1], t.b[2]);
        b.grow(t.c[0], t.c[1], t.c[2]);
        pad_box(b, 0.0f);
        // a slab of kTriThick x the triangle's extent on every side: a ray
        // grazing the triangle at angle a enters the box h / sin(a) before
        // the plane, while Moller-Trumbore's t can undercut the plane by
        // ~dist * eps / sin(a) — the sin(a) cancels, so hits within
        // ext * kTriThick / (c * eps) of the ray origin (~10^5 x the
        // triangle's extent) can never be culled
        {
          float ext = 0.0f;
          for (int k = 0; k < 3; ++k) ext = fmaxf(ext, b.mx[k] - b.mn[k]);
          for (int k = 0; k < 3; ++k) b.mn[k] -= ext * kTriThick, b.mx[k] += ext * kTriThick;
        }
        break;
      }
      case KIND_INST:
      case KIND_MODEL: {
        const uint32_t blas = q[1];  // the reference BLAS root record (a box)
        Box ob;
        if (is_box(w, blas)) {
          const uint32_t* p = &w[4 * (size_t)blas];
          ob.grow(u2f(p[0]), u2f(p[1]), u2f(p[2]));
          ob.grow(u2f(p[3]), u2f(p[4]), u2f(p[5]));
        } else {
          ob.grow(-INFINITY, -INFINITY, -INFINITY);
          ob.grow(INFINITY, INFINITY, INFINITY);
        }
        if (kind_of(w, r) == KIND_MODEL) {
          b = ob;
          pad_box(b, 0.0f);
          break;
        }
        const float* f = d.instances[q[0]].fwd;  // column-major 4x4 (M4::transform)
        for (int c = 0; c < 8; ++c) {
          const float x = c & 1 ? ob.mx[0] : ob.mn[0], y = c & 2 ? ob.mx[1] : ob.mn[1], z = c & 4 ? ob.mx[2] : ob.mn[2];
          b.grow(((f[0] * x + f[4] * y) + f[8] * z) + f[12], ((f[1] * x + f[5] * y) + f[9] * z) + f[13],
                 ((f[2] * x + f[6] * y) + f[10] * z) + f[14]);
        }
        // the object-space walk runs on the inverse-transformed ray: its
        // rounding moves hits by a few ulps of the transform's magnitudes
        float mag = 0.0f;
        for (int k = 0; k < 3; ++k) mag = fmaxf(mag, fmaxf(fabsf(b.mn[k]), fabsf(b.mx[k])));
        pad_box(b, 0x1p-16f);
        for (int k = 0; k < 3; ++k) b.mn[k] -= mag * 0x1p-18f, b.mx[k] += mag * 0x1p-18f;
        break;
      }
      default:
        break;
    }
    return b;
  }

  bool run() {
    s.nf_ok = false;
    s.nf_first_slot = n_slots();
    if (s.trav_rng) return (s.nf_note = "the traversal draws random numbers (Volume, Mix alpha)", true);
    s.vnf_base[VNF_SPHERE] = 0;
    s.vnf_base[VNF_TRI] = d.n_spheres;
    s.vnf_base[VNF_INST] = d.n_spheres + d.n_triangles;
    s.vnf_base[VNF_MODEL] = d.n_spheres + d.n_triangles + d.n_instances;
    s.vnf_leaf.assign(2 * ((size_t)d.n_spheres + d.n_triangles + d.n_instances + d.n_models), 0xFFFFFFFEu);
    std::vector<uint32_t> world_objs;
    if (!ref_order(s.world_begin, true, world_objs)) return true;
    if (world_objs.empty()) return (s.nf_note = "an empty world", true);
    std::vector<std::vector<uint32_t>> blas_objs(s.blas_regions.size());
    for (size_t k = 0; k < s.blas_regions.size(); ++k)
      if (!ref_order(s.blas_regions[k].begin, false, blas_objs[k])) return true;
    // trees; stack entries the walk may need: a far child per internal level
    // of the world tree, an instance's successor and its return marker, a far
    // child per BLAS level — kept within kNfStack by capping the depth (median
    // splits at the cap's edge): the BLAS trees first, leaving the world tree
    // at least the levels a balanced tree over its objects needs
    Tree world;
    for (uint32_t r : world_objs) world.items.push_back({object_box(r), r});
    const uint32_t has_blas = s.blas_regions.empty() ? 0 : 2;
    std::vector<Tree> blas(s.blas_regions.size());
    uint32_t blas_depth = 0;
    const uint32_t world_min = Tree::min_levels((uint32_t)world.items.size());
    if (world_min + has_blas > kNfStack) return (s.nf_note = "too many world objects for the walk's stack", true);
    for (size_t k = 0; k < blas.size(); ++k) {
      for (uint32_t r : blas_objs[k]) blas[k].items.push_back({object_box(r), r});
      if (blas[k].items.empty()) continue;
      blas[k].max_depth = kNfStack - 2 - world_min;
      blas[k].build(0, (uint32_t)blas[k].items.size(), 0);
      blas_depth = std::max(blas_depth, blas[k].depth);
    }
    world.max_depth = kNfStack - (has_blas ? 2 + blas_depth : 0);
    world.build(0, (uint32_t)world.items.size(), 0);
    s.nf_stack_need = world.depth + (has_blas ? 2 + blas_depth : 0);
    if (s.nf_stack_need > kNfStack) return (s.nf_note = "trees deeper than the walk's stack", true);
    s.nf_world = emit(world);
    if (s.nf_world == ~0u) return (s.nf_note = "a box the node format cannot hold (not finite)", true);
    for (size_t k = 0; k < blas.size(); ++k) {
      if (blas[k].items.empty()) continue;
      const uint32_t root = emit(blas[k]);
      if (root == ~0u) return (s.nf_note = "a box the node format cannot hold (not finite)", true);
      blas_root[s.blas_regions[k].begin] = root;
    }
    for (auto& [rec, ref_blas] : patches) {
      auto it = blas_root.find(ref_blas);
      if (it == blas_root.end()) return (err = "NF: an instance of an empty BLAS", false);
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
    s.vnf_leaf.clear();
  }
  return ok;
}

}  // namespace mrt
