// order_check — the price of the reference's traversal order, measured on
// the host. For rays of a built-in scene it runs
//   ref : BvhNode::intersect as the reference does it (geom.rs:185-205):
//         left subtree first, right subtree with t_max shrunk to the left
//         hit, BoundingBox::hit (geom.rs:218-247) with IEEE quotients;
//   nf  : a near-first traversal of the SAME tree and the same box and
//         primitive arithmetic: at a node both child boxes are tested, the
//         nearer (smaller entry) is visited first, a box is culled once its
//         entry passes the closest hit so far, ties go to the later
//         primitive in the reference's order (t_max is inclusive);
//   nf+ : nf whose culling keeps a relative margin (an entry beyond
//         best * (1 + 2^-k) culls), then a check that the reference would
//         reach nf's answer: every ancestor box of the winning primitive
//         must pass BoundingBox::hit at the winning t — if not, the ray falls
//         back to ref (counted).
// It reports box tests per ray for each and how many rays' closest hits
// (primitive, container, t bits) differ from ref. No GPU; the arithmetic is
// the GPU kernels' (bit-identical to the oracle).
//   g++ -O2 -std=c++17 -ffp-contract=off -o /tmp/order_check tools/order_check.cpp \
//       -Lmass-raytrace_amd/massrt -lmassrt -Wl,-rpath,$PWD/mass-raytrace_amd/massrt
//   /tmp/order_check sphere_grid 200000 tests/golden [margin_log2]
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include "../include/massrt.h"

namespace {

struct V {
  float x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
float dot(V a, V b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
uint32_t bits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

struct Ray {
  V o, d;
};
// BoundingBox::hit (geom.rs:218-247): IEEE quotients, Rust min/max = fminf/fmaxf
bool box_hit(const mrt_node& n, const Ray& r, float tmin, float tmax, float* entry = nullptr) {
  const float oo[3] = {r.o.x, r.o.y, r.o.z}, dd[3] = {r.d.x, r.d.y, r.d.z};
  float a[3], b[3];
  for (int k = 0; k < 3; ++k) a[k] = (n.min[k] - oo[k]) / dd[k], b[k] = (n.max[k] - oo[k]) / dd[k];
  const float e = fmaxf(fmaxf(fminf(a[0], b[0]), fminf(a[1], b[1])), fminf(a[2], b[2]));
  const float t0 = fmaxf(e, tmin);
  const float t1 = fminf(fminf(fmaxf(a[0], b[0]), fmaxf(a[1], b[1])), fminf(fmaxf(a[2], b[2]), tmax));
  if (entry) *entry = t0;
  return !(t1 < t0);
}
bool sphere_hit(const mrt_sphere& s, const Ray& r, float tmin, float tmax, float& t) {
  const V c{s.center[0], s.center[1], s.center[2]};
  V oc = sub(r.o, c);
  float a = dot(r.d, r.d), hb = dot(oc, r.d), cc = dot(oc, oc) - s.radius * s.radius, disc = hb * hb - a * cc;
  if (disc < 0.0f) return false;
  float sq = sqrtf(disc), root = (-hb - sq) / a;
  if (root < tmin || tmax < root) {
    root = (-hb + sq) / a;
    if (root < tmin || tmax < root) return false;
  }
  t = root;
  return true;
}
bool tri_hit(const mrt_triangle& tr, const Ray& r, float tmin, float tmax, float& t) {
  const V a{tr.a[0], tr.a[1], tr.a[2]}, b{tr.b[0], tr.b[1], tr.b[2]}, c{tr.c[0], tr.c[1], tr.c[2]};
  const V ab = sub(b, a), ac = sub(c, a);
  V p = cross(r.d, ac);
  float det = dot(ab, p);
  if (fabsf(det) < 0.000001f) return false;
  float inv = 1.0f / det;
  V tv = sub(r.o, a);
  float u = dot(tv, p) * inv;
  if (u < 0.0f || u > 1.0f) return false;
  V qv = cross(tv, ab);
  float v = dot(r.d, qv) * inv;
  if (v < 0.0f || v + u > 1.0f) return false;
  float tt = dot(ac, qv) * inv;
  if (tt < tmin || tt > tmax) return false;
  t = tt;
  return true;
}
// M4::transform (generic.rs:106-115), column-major 4x4
V xf(const float* m, V p, float w) {
  return {((m[0] * p.x + m[4] * p.y) + m[8] * p.z) + m[12] * w, ((m[1] * p.x + m[5] * p.y) + m[9] * p.z) + m[13] * w,
          ((m[2] * p.x + m[6] * p.y) + m[10] * p.z) + m[14] * w};
}

const float kTmin = 0.001f;
uint32_t kind(uint32_t r) { return MRT_REF_KIND(r); }
uint32_t idx(uint32_t r) { return MRT_REF_INDEX(r); }

struct Hit {
  float t = INFINITY;
  uint32_t prim = 0, container = 0;
  uint64_t key = 0;  // the primitive occurrence's position in the reference's (left-first) order
};

struct Scene {
  const mrt_scene_desc& d;
  std::vector<uint64_t> leaves;  // leaf occurrences under each node (instances count as 1 in the world tree)
  std::vector<uint64_t> blas_leaves;
  explicit Scene(const mrt_scene_desc& dd) : d(dd), leaves(dd.n_nodes, 0) {
    // nodes are numbered with children after parents? not guaranteed: memoised DFS
    std::vector<uint8_t> done(d.n_nodes, 0);
    for (uint32_t i = 0; i < d.n_nodes; ++i) count(i, done);
  }
  uint64_t count_ref(uint32_t r, std::vector<uint8_t>& done) {
    if (kind(r) == MRT_REF_NONE) return 0;
    if (kind(r) == MRT_REF_NODE) return count(idx(r), done);
    return 1;
  }
  uint64_t count(uint32_t i, std::vector<uint8_t>& done) {
    if (done[i]) return leaves[i];
    // iterative post-order to avoid deep recursion
    std::vector<std::pair<uint32_t, int>> st{{i, 0}};
    while (!st.empty()) {
      auto& [n, s] = st.back();
      if (done[n]) {
        st.pop_back();
        continue;
      }
      const mrt_node& nd = d.nodes[n];
      bool pushed = false;
      for (uint32_t c : {nd.left, nd.right})
        if (kind(c) == MRT_REF_NODE && !done[idx(c)]) {
          st.push_back({idx(c), 0});
          pushed = true;
        }
      if (pushed) continue;
      uint64_t k = 0;
      for (uint32_t c : {nd.left, nd.right}) k += kind(c) == MRT_REF_NODE ? leaves[idx(c)] : (kind(c) ? 1 : 0);
      leaves[n] = k;
      done[n] = 1;
      st.pop_back();
    }
    return leaves[i];
  }
};

struct Stats {
  uint64_t boxes = 0, prims = 0;
};

// the parent node of every reference tree node and leaf occurrence needed by
// the reachability check: world parent of each world leaf, BLAS parent of
// each triangle (per BLAS root)
struct Parents {
  std::vector<uint32_t> sphere, inst, model;  // world parent node of world leaves
  std::vector<uint32_t> tri;                   // BLAS parent node of each triangle
  explicit Parents(const mrt_scene_desc& d)
      : sphere(d.n_spheres, ~0u), inst(d.n_instances, ~0u), model(d.n_models, ~0u), tri(d.n_triangles, ~0u) {
    for (uint32_t i = 0; i < d.n_nodes; ++i)
      for (uint32_t c : {d.nodes[i].left, d.nodes[i].right}) {
        switch (kind(c)) {
          case MRT_REF_SPHERE: sphere[idx(c)] = i; break;
          case MRT_REF_INSTANCE: inst[idx(c)] = i; break;
          case MRT_REF_MODEL: model[idx(c)] = i; break;
          case MRT_REF_TRIANGLE: tri[idx(c)] = i; break;
          default: break;
        }
      }
  }
};

// ---- the reference: left-first recursion with the shrinking inclusive t_max
struct RefWalk {
  const Scene& S;
  Stats& st;
  Hit h;
  uint32_t container = 0;
  uint64_t base = 0;  // key of the current BLAS occurrence
  void prim(uint32_t r, const Ray& ray, uint64_t key) {
    float t;
    st.prims++;
    if (kind(r) == MRT_REF_SPHERE) {
      if (sphere_hit(S.d.spheres[idx(r)], ray, kTmin, h.t, t)) h = Hit{t, r, container, key};
    } else if (kind(r) == MRT_REF_TRIANGLE) {
      if (tri_hit(S.d.triangles[idx(r)], ray, kTmin, h.t, t)) h = Hit{t, r, container, key};
    }
  }
  bool blas = false;
  void walk(uint32_t r, const Ray& ray, uint64_t key) {
    switch (kind(r)) {
      case MRT_REF_NONE:
        return;
      case MRT_REF_NODE: {
        const mrt_node& n = S.d.nodes[idx(r)];
        st.boxes++;
        if (!box_hit(n, ray, kTmin, h.t)) return;
        walk(n.left, ray, key);
        walk(n.right, ray, key + (kind(n.left) == MRT_REF_NODE ? S.leaves[idx(n.left)] : 1));
        return;
      }
      case MRT_REF_INSTANCE: {
        const mrt_instance& in = S.d.instances[idx(r)];
        const Ray o{xf(in.inv, ray.o, 1.0f), xf(in.inv, ray.d, 0.0f)};
        const uint32_t save = container;
        container = r, blas = true;
        walk(MRT_REF(MRT_REF_NODE, in.blas_root), o, key << 24);  // BLAS keys below the world leaf's
        container = save, blas = false;
        return;
      }
      case MRT_REF_MODEL: {
        const uint32_t save = container;
        container = r, blas = true;
        walk(MRT_REF(MRT_REF_NODE, S.d.models[idx(r)].blas_root), ray, key << 24);
        container = save, blas = false;
        return;
      }
      default:
        prim(r, ray, blas ? key : key << 24);
    }
  }
};

// ---- near-first: a stack of (ref, ray space, key, entry) --------------------
struct Item {
  uint32_t ref;
  int32_t slot;    // object ray slot (inst_rays) or -1: the world ray
  int32_t inst;    // instance index of that ray space, or -1
  uint32_t container;
  uint64_t key;    // key of the subtree's first leaf: world leaf index (world), full key (BLAS)
  bool blas;
  float entry;
  uint32_t depth;
};
struct NearFirst {
  const Scene& S;
  Stats& st;
  float margin;  // relative culling margin (0: exact entry <= best)
  Hit h;
  std::vector<Item> stack;
  std::vector<Ray> inst_rays;  // object rays of the instances entered
  // the ancestors (node, instance space) of the current item, and of the winner
  std::vector<std::pair<uint32_t, int32_t>> path, best_path;

  float cull_at() const { return h.t == INFINITY ? INFINITY : h.t + fabsf(h.t) * margin; }
  void accept(uint32_t r, float t, uint32_t container, uint64_t key, uint32_t depth) {
    if (t < h.t || (t == h.t && key > h.key)) {
      h = Hit{t, r, container, key};
      best_path.assign(path.begin(), path.begin() + depth);
    }
  }
  void run(uint32_t root, const Ray& world) {
    stack.clear();
    inst_rays.clear();
    path.clear();
    stack.push_back({root, -1, -1, 0, 0, false, -INFINITY, 0});
    while (!stack.empty()) {
      const Item it = stack.back();
      stack.pop_back();
      if (it.entry > cull_at()) continue;
      const Ray ray = it.slot >= 0 ? inst_rays[it.slot] : world;
      path.resize(it.depth);
      if (kind(it.ref) != MRT_REF_NODE) {
        leaf(it, it.ref, it.key, ray, it.depth);
        continue;
      }
      const mrt_node& n = S.d.nodes[idx(it.ref)];
      path.push_back({idx(it.ref), it.inst});
      Item ch[2];
      int nch = 0;
      const uint64_t kr = it.key + (kind(n.left) == MRT_REF_NODE ? S.leaves[idx(n.left)] : 1);
      for (int c = 0; c < 2; ++c) {
        const uint32_t cr = c ? n.right : n.left;
        const uint64_t ck = c ? kr : it.key;
        if (kind(cr) == MRT_REF_NONE) continue;
        if (kind(cr) == MRT_REF_NODE) {
          float e;
          st.boxes++;
          if (!box_hit(S.d.nodes[idx(cr)], ray, kTmin, cull_at(), &e)) continue;
          Item x = it;
          x.ref = cr, x.key = ck, x.entry = e, x.depth = it.depth + 1;
          ch[nch++] = x;
        } else {
          leaf(it, cr, ck, ray, it.depth + 1);
        }
      }
      if (nch == 2 && ch[1].entry < ch[0].entry) std::swap(ch[0], ch[1]);
      for (int c = nch - 1; c >= 0; --c) stack.push_back(ch[c]);
    }
  }
  // a non-node child of the current item's space: test it, or enter its BLAS
  void leaf(const Item& it, uint32_t r, uint64_t key, const Ray& ray, uint32_t depth) {
    float t;
    const uint64_t full = it.blas ? key : key << 24;
    switch (kind(r)) {
      case MRT_REF_SPHERE:
        st.prims++;
        if (sphere_hit(S.d.spheres[idx(r)], ray, kTmin, cull_at(), t)) accept(r, t, it.container, full, depth);
        return;
      case MRT_REF_TRIANGLE:
        st.prims++;
        if (tri_hit(S.d.triangles[idx(r)], ray, kTmin, cull_at(), t)) accept(r, t, it.container, full, depth);
        return;
      case MRT_REF_INSTANCE: {
        const mrt_instance& in = S.d.instances[idx(r)];
        inst_rays.push_back(Ray{xf(in.inv, ray.o, 1.0f), xf(in.inv, ray.d, 0.0f)});
        float e;
        st.boxes++;
        if (!box_hit(S.d.nodes[in.blas_root], inst_rays.back(), kTmin, cull_at(), &e)) return;
        stack.push_back({MRT_REF(MRT_REF_NODE, in.blas_root), (int32_t)inst_rays.size() - 1, (int32_t)idx(r), r,
                         key << 24, true, e, depth});
        return;
      }
      case MRT_REF_MODEL: {
        const uint32_t root = S.d.models[idx(r)].blas_root;
        float e;
        st.boxes++;
        if (!box_hit(S.d.nodes[root], ray, kTmin, cull_at(), &e)) return;
        stack.push_back({MRT_REF(MRT_REF_NODE, root), it.slot, it.inst, r, key << 24, true, e, depth});
        return;
      }
      default:
        return;
    }
  }
};

// ---- a surface-area-heuristic BVH over the same primitives ---------------------
// (the experiment's "better tree": binned SAH, 2-wide, leaves of <= 4 items)
struct Box3 {
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const Box3& b) {
    for (int k = 0; k < 3; ++k) mn[k] = fminf(mn[k], b.mn[k]), mx[k] = fmaxf(mx[k], b.mx[k]);
  }
  float area() const {
    const float dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
    return dx < 0 ? 0 : 2 * (dx * dy + dy * dz + dz * dx);
  }
  float c(int k) const { return 0.5f * (mn[k] + mx[k]); }
};
struct SItem {
  Box3 b;
  uint32_t ref;
  uint64_t key;  // leaf occurrence key in the reference's order (world leaf index, or BLAS-local index)
};
struct SNode {
  mrt_node box;        // box as an mrt_node (for box_hit)
  int32_t l = -1, r = -1;  // children (internal)
  uint32_t first = 0, count = 0;  // items (leaf)
  int axis = 0;        // split axis: l holds the lower centroids
};
struct SahTree {
  std::vector<SNode> nodes;
  std::vector<SItem> items;
  int32_t build(uint32_t b, uint32_t e) {
    SNode n;
    Box3 bb, cb;
    for (uint32_t i = b; i < e; ++i) {
      bb.grow(items[i].b);
      Box3 c;
      for (int k = 0; k < 3; ++k) c.mn[k] = c.mx[k] = items[i].b.c(k);
      cb.grow(c);
    }
    for (int k = 0; k < 3; ++k) n.box.min[k] = bb.mn[k], n.box.max[k] = bb.mx[k];
    const int32_t id = (int32_t)nodes.size();
    nodes.push_back(n);
    const uint32_t cnt = e - b;
    if (cnt <= 4) {
      nodes[id].first = b, nodes[id].count = cnt;
      return id;
    }
    constexpr int NB = 16;
    float best = INFINITY;
    int bk = -1, bs = -1;
    for (int k = 0; k < 3; ++k) {
      const float lo = cb.mn[k], ext = cb.mx[k] - cb.mn[k];
      if (!(ext > 0)) continue;
      Box3 bins[NB];
      uint32_t cntb[NB] = {};
      for (uint32_t i = b; i < e; ++i) {
        int j = std::min(NB - 1, (int)((items[i].b.c(k) - lo) / ext * NB));
        bins[j].grow(items[i].b);
        cntb[j]++;
      }
      for (int sp = 1; sp < NB; ++sp) {
        Box3 L, R;
        uint32_t nl = 0, nr = 0;
        for (int j = 0; j < sp; ++j) L.grow(bins[j]), nl += cntb[j];
        for (int j = sp; j < NB; ++j) R.grow(bins[j]), nr += cntb[j];
        if (!nl || !nr) continue;
        const float cost = L.area() * nl + R.area() * nr;
        if (cost < best) best = cost, bk = k, bs = sp;
      }
    }
    uint32_t mid;
    if (bk < 0) {
      mid = b + cnt / 2;
    } else {
      const float lo = cb.mn[bk], ext = cb.mx[bk] - cb.mn[bk];
      auto it = std::partition(items.begin() + b, items.begin() + e, [&](const SItem& x) {
        return std::min(NB - 1, (int)((x.b.c(bk) - lo) / ext * NB)) < bs;
      });
      mid = (uint32_t)(it - items.begin());
      if (mid == b || mid == e) mid = b + cnt / 2;
    }
    const int32_t l = build(b, mid), r = build(mid, e);
    nodes[id].l = l, nodes[id].r = r, nodes[id].axis = bk < 0 ? 0 : bk;
    return id;
  }
};

Box3 box_of_node(const mrt_node& n) {
  Box3 b;
  for (int k = 0; k < 3; ++k) b.mn[k] = n.min[k], b.mx[k] = n.max[k];
  return b;
}

struct SahScene {
  const Scene& S;
  SahTree tlas;
  std::vector<int32_t> blas_of_root;     // reference BLAS root node -> index into blas
  std::vector<SahTree> blas;
  explicit SahScene(const Scene& sc) : S(sc), blas_of_root(sc.d.n_nodes, -1) {
    // world leaves in the reference's order, with their keys
    collect(S.d.roots[0], 0, tlas.items, false);
    tlas.build(0, (uint32_t)tlas.items.size());
  }
  void collect(uint32_t r, uint64_t key, std::vector<SItem>& out, bool in_blas) {
    std::vector<std::pair<uint32_t, uint64_t>> st{{r, key}};
    while (!st.empty()) {
      auto [x, k] = st.back();
      st.pop_back();
      switch (kind(x)) {
        case MRT_REF_NONE:
          break;
        case MRT_REF_NODE: {
          const mrt_node& n = S.d.nodes[idx(x)];
          const uint64_t kr = k + (kind(n.left) == MRT_REF_NODE ? S.leaves[idx(n.left)] : 1);
          st.push_back({n.right, kr});
          st.push_back({n.left, k});
          break;
        }
        case MRT_REF_SPHERE: {
          const mrt_sphere& sp = S.d.spheres[idx(x)];
          SItem it;
          for (int q = 0; q < 3; ++q)
            it.b.mn[q] = sp.center[q] - fabsf(sp.radius), it.b.mx[q] = sp.center[q] + fabsf(sp.radius);
          it.ref = x, it.key = k;
          out.push_back(it);
          break;
        }
        case MRT_REF_TRIANGLE: {
          const mrt_triangle& t = S.d.triangles[idx(x)];
          SItem it;
          for (int q = 0; q < 3; ++q)
            it.b.mn[q] = fminf(fminf(t.a[q], t.b[q]), t.c[q]), it.b.mx[q] = fmaxf(fmaxf(t.a[q], t.b[q]), t.c[q]);
          it.ref = x, it.key = k;
          out.push_back(it);
          break;
        }
        case MRT_REF_INSTANCE: {
          const mrt_instance& in = S.d.instances[idx(x)];
          ensure_blas(in.blas_root);
          const Box3 ob = box_of_node(S.d.nodes[in.blas_root]);
          SItem it;
          for (int c = 0; c < 8; ++c) {
            const V p{c & 1 ? ob.mx[0] : ob.mn[0], c & 2 ? ob.mx[1] : ob.mn[1], c & 4 ? ob.mx[2] : ob.mn[2]};
            const V w = xf(in.fwd, p, 1.0f);
            Box3 pb;
            pb.mn[0] = pb.mx[0] = w.x, pb.mn[1] = pb.mx[1] = w.y, pb.mn[2] = pb.mx[2] = w.z;
            it.b.grow(pb);
          }
          it.ref = x, it.key = k;
          out.push_back(it);
          break;
        }
        case MRT_REF_MODEL: {
          const uint32_t root = S.d.models[idx(x)].blas_root;
          ensure_blas(root);
          SItem it;
          it.b = box_of_node(S.d.nodes[root]);
          it.ref = x, it.key = k;
          out.push_back(it);
          break;
        }
        default:
          break;
      }
    }
    (void)in_blas;
  }
  void ensure_blas(uint32_t root) {
    if (blas_of_root[root] >= 0) return;
    SahTree t;
    collect(MRT_REF(MRT_REF_NODE, root), 0, t.items, true);
    t.build(0, (uint32_t)t.items.size());
    blas_of_root[root] = (int32_t)blas.size();
    blas.push_back(std::move(t));
  }
};

// near-first over the SAH trees, exact culling (entry <= best), reference tie keys
struct SahWalk {
  const SahScene& Z;
  Stats& st;
  Hit h;
  struct It {
    const SahTree* t;
    int32_t node;
    Ray ray;
    uint32_t container;
    uint64_t base;  // world key << 24 for BLAS items, 0 in the TLAS
    bool blas;
    float entry;
  };
  std::vector<It> stack;
  float margin = 0.0f;
  float cull() const { return h.t == INFINITY ? INFINITY : h.t + fabsf(h.t) * margin; }
  void run(const Ray& world) {
    stack.clear();
    float e;
    st.boxes++;
    if (!box_hit(Z.tlas.nodes[0].box, world, kTmin, cull(), &e)) return;
    stack.push_back({&Z.tlas, 0, world, 0, 0, false, e});
    while (!stack.empty()) {
      const It it = stack.back();
      stack.pop_back();
      if (it.entry > cull()) continue;
      const SNode& n = it.t->nodes[it.node];
      if (n.l < 0) {
        for (uint32_t i = n.first; i < n.first + n.count; ++i) item(it, it.t->items[i]);
        continue;
      }
      It ch[2];
      int nc = 0;
      for (int32_t c : {n.l, n.r}) {
        st.boxes++;
        if (!box_hit(it.t->nodes[c].box, it.ray, kTmin, cull(), &e)) continue;
        It x = it;
        x.node = c, x.entry = e;
        ch[nc++] = x;
      }
      if (nc == 2 && ch[1].entry < ch[0].entry) std::swap(ch[0], ch[1]);
      for (int c = nc - 1; c >= 0; --c) stack.push_back(ch[c]);
    }
  }
  void accept(uint32_t r, float t, uint32_t container, uint64_t key) {
    if (t < h.t || (t == h.t && key > h.key)) h = Hit{t, r, container, key};
  }
  void item(const It& it, const SItem& x) {
    float t, e;
    const uint64_t key = it.blas ? it.base + x.key : x.key << 24;
    switch (kind(x.ref)) {
      case MRT_REF_SPHERE:
        st.prims++;
        if (sphere_hit(Z.S.d.spheres[idx(x.ref)], it.ray, kTmin, cull(), t)) accept(x.ref, t, it.container, key);
        return;
      case MRT_REF_TRIANGLE:
        st.prims++;
        if (tri_hit(Z.S.d.triangles[idx(x.ref)], it.ray, kTmin, cull(), t)) accept(x.ref, t, it.container, key);
        return;
      case MRT_REF_INSTANCE: {
        const mrt_instance& in = Z.S.d.instances[idx(x.ref)];
        const SahTree* bt = &Z.blas[Z.blas_of_root[in.blas_root]];
        const Ray o{xf(in.inv, it.ray.o, 1.0f), xf(in.inv, it.ray.d, 0.0f)};
        st.boxes++;
        if (!box_hit(bt->nodes[0].box, o, kTmin, cull(), &e)) return;
        stack.push_back({bt, 0, o, x.ref, x.key << 24, true, e});
        return;
      }
      case MRT_REF_MODEL: {
        const SahTree* bt = &Z.blas[Z.blas_of_root[Z.S.d.models[idx(x.ref)].blas_root]];
        st.boxes++;
        if (!box_hit(bt->nodes[0].box, it.ray, kTmin, cull(), &e)) return;
        stack.push_back({bt, 0, it.ray, x.ref, x.key << 24, true, e});
        return;
      }
      default:
        return;
    }
  }
};

// the GPU-friendly variant: a preorder (stackless, skip-pointer) walk of the
// SAH trees whose child order is chosen per ray octant (the near child along
// the node's split axis first) — the k_trace record-stream machinery with one
// stream per octant; one box test per visited node, culling at the best t
struct OctWalk {
  const SahScene& Z;
  Stats& st;
  Hit h;
  void run(const Ray& world) { node(&Z.tlas, 0, world, 0, 0, false); }
  void accept(uint32_t r, float t, uint32_t container, uint64_t key) {
    if (t < h.t || (t == h.t && key > h.key)) h = Hit{t, r, container, key};
  }
  void node(const SahTree* T, int32_t ni, const Ray& ray, uint32_t container, uint64_t base, bool blas) {
    const SNode& n = T->nodes[ni];
    st.boxes++;
    if (!box_hit(n.box, ray, kTmin, h.t)) return;
    if (n.l < 0) {
      for (uint32_t i = n.first; i < n.first + n.count; ++i) item(T->items[i], ray, container, base, blas);
      return;
    }
    const float dk = n.axis == 0 ? ray.d.x : (n.axis == 1 ? ray.d.y : ray.d.z);
    const int32_t a = dk >= 0 ? n.l : n.r, b = dk >= 0 ? n.r : n.l;
    node(T, a, ray, container, base, blas);
    node(T, b, ray, container, base, blas);
  }
  void item(const SItem& x, const Ray& ray, uint32_t container, uint64_t base, bool blas) {
    float t;
    const uint64_t key = blas ? base + x.key : x.key << 24;
    switch (kind(x.ref)) {
      case MRT_REF_SPHERE:
        st.prims++;
        if (sphere_hit(Z.S.d.spheres[idx(x.ref)], ray, kTmin, h.t, t)) accept(x.ref, t, container, key);
        return;
      case MRT_REF_TRIANGLE:
        st.prims++;
        if (tri_hit(Z.S.d.triangles[idx(x.ref)], ray, kTmin, h.t, t)) accept(x.ref, t, container, key);
        return;
      case MRT_REF_INSTANCE: {
        const mrt_instance& in = Z.S.d.instances[idx(x.ref)];
        const Ray o{xf(in.inv, ray.o, 1.0f), xf(in.inv, ray.d, 0.0f)};
        node(&Z.blas[Z.blas_of_root[in.blas_root]], 0, o, x.ref, x.key << 24, true);
        return;
      }
      case MRT_REF_MODEL:
        node(&Z.blas[Z.blas_of_root[Z.S.d.models[idx(x.ref)].blas_root]], 0, ray, x.ref, x.key << 24, true);
        return;
      default:
        return;
    }
  }
};

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) return 1;
  const int n = argc > 2 ? atoi(argv[2]) : 20000;
  const int mlog = argc > 4 ? atoi(argv[4]) : 10;
  mrt_builder* b = nullptr;
  mrt_builder_new(1, &b);
  if (mrt_builder_builtin(b, argv[1], 16.0f / 9.0f, argc > 3 ? argv[3] : "tests/golden") != 0) {
    printf("%s: %s\n", argv[1], mrt_builder_last_error());
    return 1;
  }
  mrt_scene_desc d;
  mrt_camera cam;
  mrt_builder_desc(b, &d, &cam);
  if (d.n_roots != 1 || kind(d.roots[0]) != MRT_REF_NODE) {
    printf("%s: expects one root node after build_bvh\n", argv[1]);
    return 1;
  }
  Scene S(d);
  SahScene Z(S);
  Parents P(d);
  Stats ss, so;
  uint64_t diff_sah = 0, diff_oct = 0;
  constexpr int NM = 4;
  const int margins[NM] = {23, 20, 16, 10};
  Stats sv[NM];
  uint64_t fb[NM] = {}, dv[NM] = {};
  std::mt19937 g(7);
  std::uniform_real_distribution<float> u(0.0f, 1.0f);
  Stats sr, sn, sm;
  uint64_t rays = 0, diff_nf = 0, diff_nfm = 0, fallback = 0, diff_key_only = 0;
  const V o{cam.origin[0], cam.origin[1], cam.origin[2]};
  const float margin = ldexpf(1.0f, -mlog);
  for (int k = 0; k < n; ++k) {
    Ray ray;
    const float s1 = u(g), t1 = u(g);
    const V cd{((cam.lower_left_corner[0] + cam.horizontal[0] * s1) + cam.vertical[0] * t1) - o.x,
               ((cam.lower_left_corner[1] + cam.horizontal[1] * s1) + cam.vertical[1] * t1) - o.y,
               ((cam.lower_left_corner[2] + cam.horizontal[2] * s1) + cam.vertical[2] * t1) - o.z};
    if (k % 2 == 0) {
      ray = {o, cd};
    } else {  // a bounce: from the camera ray's hit, random direction
      Stats tmp;
      RefWalk w{S, tmp};
      w.walk(d.roots[0], Ray{o, cd}, 0);
      if (w.h.prim == 0) continue;
      ray = {{o.x + cd.x * w.h.t, o.y + cd.y * w.h.t, o.z + cd.z * w.h.t}, {u(g) * 2 - 1, u(g) * 2 - 1, u(g) * 2 - 1}};
    }
    ++rays;
    RefWalk w{S, sr};
    w.walk(d.roots[0], ray, 0);
    NearFirst nf{S, sn, 0.0f};
    nf.run(d.roots[0], ray);
    const bool same = nf.h.prim == w.h.prim && nf.h.container == w.h.container && bits(nf.h.t) == bits(w.h.t);
    diff_nf += !same;
    diff_key_only += same && nf.h.key != w.h.key;
    NearFirst nm{S, sm, margin};
    nm.run(d.roots[0], ray);
    // reachability check: would the reference's traversal reach nm's winner?
    // (every ancestor box passes BoundingBox::hit at the winning t)
    bool reach = true;
    if (nm.h.prim) {
      for (auto& [node, inst] : nm.best_path) {
        Ray rr = ray;
        if (inst >= 0) {
          const mrt_instance& in = d.instances[inst];
          rr = Ray{xf(in.inv, ray.o, 1.0f), xf(in.inv, ray.d, 0.0f)};
        }
        sm.boxes++;
        if (!box_hit(d.nodes[node], rr, kTmin, nm.h.t)) reach = false;
      }
    }
    Hit got = nm.h;
    if (!reach) {
      ++fallback;
      RefWalk w2{S, sm};
      w2.walk(d.roots[0], ray, 0);
      got = w2.h;
    }
    diff_nfm += !(got.prim == w.h.prim && got.container == w.h.container && bits(got.t) == bits(w.h.t));
    OctWalk ow{Z, so};
    ow.run(ray);
    diff_oct += !(ow.h.prim == w.h.prim && ow.h.container == w.h.container && bits(ow.h.t) == bits(w.h.t));
    SahWalk sw{Z, ss};
    sw.run(ray);
    diff_sah += !(sw.h.prim == w.h.prim && sw.h.container == w.h.container && bits(sw.h.t) == bits(w.h.t));
    // SAH + near-first with the culling margin, then the strict reachability
    // check on the winner's two innermost reference ancestors (world parent,
    // BLAS parent: nested boxes, so these imply the outer ones), else ref
    for (int mi = 0; mi < NM; ++mi) {
      SahWalk v{Z, sv[mi]};
      v.margin = ldexpf(1.0f, -margins[mi]);
      v.run(ray);
      Hit gotv = v.h;
      bool ok = true;
      if (v.h.prim) {
        const uint32_t pk = kind(v.h.prim), pi = idx(v.h.prim);
        Ray rr = ray;
        uint32_t wp = ~0u, bp = ~0u;
        if (pk == MRT_REF_SPHERE) wp = P.sphere[pi];
        if (pk == MRT_REF_TRIANGLE) bp = P.tri[pi];
        if (kind(v.h.container) == MRT_REF_INSTANCE) {
          const mrt_instance& in = d.instances[idx(v.h.container)];
          wp = P.inst[idx(v.h.container)];
          rr = Ray{xf(in.inv, ray.o, 1.0f), xf(in.inv, ray.d, 0.0f)};
        } else if (kind(v.h.container) == MRT_REF_MODEL) {
          wp = P.model[idx(v.h.container)];
        } else if (pk == MRT_REF_TRIANGLE) {  // a world-level triangle
          wp = bp, bp = ~0u;
        }
        if (wp != ~0u) sv[mi].boxes++, ok = ok && box_hit(d.nodes[wp], ray, kTmin, v.h.t);
        if (bp != ~0u) sv[mi].boxes++, ok = ok && box_hit(d.nodes[bp], rr, kTmin, v.h.t);
      }
      if (!ok) {
        fb[mi]++;
        RefWalk w3{S, sv[mi]};
        w3.walk(d.roots[0], ray, 0);
        gotv = w3.h;
      }
      dv[mi] += !(gotv.prim == w.h.prim && gotv.container == w.h.container && bits(gotv.t) == bits(w.h.t));
    }
  }
  const double R = (double)std::max<uint64_t>(rays, 1);
  printf("%-12s rays %llu  ref %.1f boxes/ray  nf %.1f (x%.2f, %llu differ, %llu same hit other key)  "
         "nf+2^-%d %.1f (x%.2f incl. checks/fallbacks, %llu fallbacks, %llu differ)\n",
         argv[1], (unsigned long long)rays, sr.boxes / R, sn.boxes / R, (double)sr.boxes / std::max<uint64_t>(sn.boxes, 1),
         (unsigned long long)diff_nf, (unsigned long long)diff_key_only, mlog, sm.boxes / R,
         (double)sr.boxes / std::max<uint64_t>(sm.boxes, 1), (unsigned long long)fallback, (unsigned long long)diff_nfm);
  {
    auto depth = [](const SahTree& t) {
      std::vector<std::pair<int32_t, int>> st{{0, 1}};
      int m = 0;
      while (!st.empty()) {
        auto [n, dd] = st.back();
        st.pop_back();
        m = std::max(m, dd);
        if (t.nodes[n].l >= 0) st.push_back({t.nodes[n].l, dd + 1}), st.push_back({t.nodes[n].r, dd + 1});
      }
      return m;
    };
    int bm = 0;
    for (auto& t : Z.blas) bm = std::max(bm, depth(t));
    printf("%-12s sah depth: tlas %d, deepest blas %d\n", argv[1], depth(Z.tlas), bm);
  }
  printf("%-12s sah+nf %.1f boxes/ray (x%.2f vs ref), prims %.1f vs %.1f, %llu differ (no margin, no check)\n", argv[1],
         ss.boxes / R, (double)sr.boxes / std::max<uint64_t>(ss.boxes, 1), ss.prims / R, sr.prims / R,
         (unsigned long long)diff_sah);
  const double R2 = (double)std::max<uint64_t>(rays, 1);
  printf("%-12s sah octant-ordered stackless %.1f boxes/ray (x%.2f vs ref), %llu differ (no check)\n", argv[1],
         so.boxes / R2, (double)sr.boxes / std::max<uint64_t>(so.boxes, 1), (unsigned long long)diff_oct);
  for (int mi = 0; mi < NM; ++mi)
    printf("%-12s sah+nf margin 2^-%d + check: %.1f boxes/ray incl. fallbacks (x%.2f vs ref), %llu fallbacks (%.2f%%), "
           "%llu differ\n", argv[1], margins[mi], sv[mi].boxes / R, (double)sr.boxes / std::max<uint64_t>(sv[mi].boxes, 1),
           (unsigned long long)fb[mi], 100.0 * fb[mi] / R, (unsigned long long)dv[mi]);
  mrt_builder_free(b);
  return 0;
}
