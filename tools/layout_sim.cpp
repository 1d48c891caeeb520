// layout_sim — cache model of record-stream layouts for k_trace.
//
// Builds a scene's record stream with the library's own builder and
// linearisation (mrt_builder_builtin + mrt::build_host_scene), traces a set
// of camera rays and one-bounce rays through it (the reference's left-first
// order over the preorder stream, plain float slab test — locality only, not
// parity), and replays the record fetches under several layouts of the same
// records through a model of the cache hierarchy:
//   L1: one CU, 32 KiB, 128-B lines, LRU; the CU's 8 resident waves x 64 rays
//       advance one record per ray per round (SIMT lockstep, interleaved)
//   L2: one XCD, 4 MiB, 128-B lines, LRU, fed by the L1 misses of 32 CUs
// and reports per ray segment: records, distinct 128-B lines, L1 and L2 hit rates.
//
//   g++ -O2 -std=c++17 -I mass-raytrace_amd/csrc tools/layout_sim.cpp \
//       -Lmass-raytrace_amd/massrt -lmassrt -Wl,-rpath,$PWD/mass-raytrace_amd/massrt -o /tmp/layout_sim
//   /tmp/layout_sim mesh_ply assets [rays]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <list>
#include <queue>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "../include/massrt.h"
#include "device/upload.h"

using namespace mrt;

static float f(uint32_t u) {
  float x;
  memcpy(&x, &u, 4);
  return x;
}

struct Stream {
  const std::vector<uint32_t>& w;
  uint32_t kind(uint32_t i) const { return w[4 * (i + 1) + 3]; }
  bool box(uint32_t i) const { return (kind(i) & kBoxFlag) != 0; }
  uint32_t size(uint32_t i) const { return box(i) ? 2 : (kind(i) == KIND_TRI ? 3 : 2); }
  uint32_t hit(uint32_t i) const { return kind(i) & ~kBoxFlag; }
  uint32_t skip(uint32_t i) const { return w[4 * (i + 1) + 2]; }
  uint32_t next(uint32_t i) const {
    const uint32_t k = kind(i);
    return k == KIND_TRI ? w[4 * (i + 2) + 3] : (k == KIND_INST || k == KIND_MODEL) ? i + 2 : w[4 * (i + 1) + 1];
  }
};

struct Ray {
  float o[3], d[3];
};

// closest hit over the region starting at `begin` (no instances: BLAS/world of
// boxes and triangles/spheres), recording every record index fetched
static float trace(const Stream& s, uint32_t begin, const Ray& r, std::vector<uint32_t>* seq, float* nrm) {
  float best = INFINITY;
  uint32_t i = begin;
  for (;;) {
    if (seq) seq->push_back(i);
    const uint32_t k = s.kind(i);
    if (k == KIND_END) break;
    const uint32_t* a = &s.w[4 * i];
    if (s.box(i)) {
      float mn[3] = {f(a[0]), f(a[1]), f(a[2])}, mx[3] = {f(a[3]), f(a[4]), f(a[5])};
      float t0 = 0.001f, t1 = best;
      for (int c = 0; c < 3; ++c) {
        float inv = 1.0f / r.d[c];
        float ta = (mn[c] - r.o[c]) * inv, tb = (mx[c] - r.o[c]) * inv;
        if (inv < 0) std::swap(ta, tb);
        t0 = ta > t0 ? ta : t0;
        t1 = tb < t1 ? tb : t1;
      }
      i = (t1 >= t0) ? s.hit(i) : s.skip(i);
      continue;
    }
    if (k == KIND_TRI) {
      float A[3] = {f(a[0]), f(a[1]), f(a[2])}, e1[3] = {f(a[3]), f(a[4]), f(a[5])}, e2[3] = {f(a[8]), f(a[9]), f(a[10])};
      float p[3] = {r.d[1] * e2[2] - r.d[2] * e2[1], r.d[2] * e2[0] - r.d[0] * e2[2], r.d[0] * e2[1] - r.d[1] * e2[0]};
      float det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
      if (fabsf(det) > 1e-12f) {
        float id = 1.0f / det, tv[3] = {r.o[0] - A[0], r.o[1] - A[1], r.o[2] - A[2]};
        float u = (tv[0] * p[0] + tv[1] * p[1] + tv[2] * p[2]) * id;
        float q[3] = {tv[1] * e1[2] - tv[2] * e1[1], tv[2] * e1[0] - tv[0] * e1[2], tv[0] * e1[1] - tv[1] * e1[0]};
        float v = (r.d[0] * q[0] + r.d[1] * q[1] + r.d[2] * q[2]) * id;
        float t = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * id;
        if (u >= 0 && v >= 0 && u + v <= 1 && t > 0.001f && t < best) {
          best = t;
          if (nrm) {
            nrm[0] = e1[1] * e2[2] - e1[2] * e2[1], nrm[1] = e1[2] * e2[0] - e1[0] * e2[2], nrm[2] = e1[0] * e2[1] - e1[1] * e2[0];
          }
        }
      }
    }
    i = s.next(i);
  }
  return best;
}

struct LRU {
  size_t cap;
  std::list<uint64_t> order;
  std::unordered_map<uint64_t, std::list<uint64_t>::iterator> where;
  uint64_t hits = 0, misses = 0;
  explicit LRU(size_t lines) : cap(lines) {}
  bool access(uint64_t line) {
    auto it = where.find(line);
    if (it != where.end()) {
      order.splice(order.begin(), order, it->second);
      ++hits;
      return true;
    }
    ++misses;
    order.push_front(line);
    where[line] = order.begin();
    if (order.size() > cap) {
      where.erase(order.back());
      order.pop_back();
    }
    return false;
  }
};

// tree of the region: children of each box record
struct Tree {
  std::vector<uint32_t> recs;                    // every record of the region, stream order
  std::unordered_map<uint32_t, std::vector<uint32_t>> kids;  // box -> children (records)
};

static Tree parse(const Stream& s, uint32_t begin) {
  Tree t;
  uint32_t i = begin;
  while (s.kind(i) != KIND_END) {
    t.recs.push_back(i);
    if (s.box(i)) {
      std::vector<uint32_t> k;
      uint32_t c = s.hit(i), end = s.skip(i);
      while (c < end) {
        k.push_back(c);
        c = s.box(c) ? s.skip(c) : s.next(c);
      }
      t.kids[i] = k;
    }
    i += s.size(i);
  }
  t.recs.push_back(i);  // END
  return t;
}

// address (bytes) of every record under a layout: a permutation of records,
// packed in that order, each record padded to `align` bytes
using Layout = std::unordered_map<uint32_t, uint64_t>;
static Layout pack(const Stream& s, const std::vector<uint32_t>& order, uint32_t align) {
  Layout L;
  uint64_t a = 0;
  for (uint32_t r : order) {
    a = (a + align - 1) / align * align;
    L[r] = a;
    a += 16 * s.size(r);
  }
  return L;
}

// packed in order, every sibling group (a node's children) starting on a
// `galign`-byte boundary, triangles padded to `tri` bytes
static Layout pack_groups(const Stream& s, const Tree& t, const std::vector<uint32_t>& order, uint32_t galign,
                          uint32_t tri, uint32_t prim_galign = 0) {
  std::unordered_map<uint32_t, bool> first;  // first record of a sibling group
  for (auto& kv : t.kids) first[kv.second.front()] = true;
  Layout L;
  uint64_t a = 0;
  for (uint32_t r : order) {
    const uint32_t ga = (prim_galign && !s.box(r)) ? prim_galign : galign;
    if (first.count(r)) a = (a + ga - 1) / ga * ga;
    L[r] = a;
    a += (s.kind(r) == KIND_TRI) ? tri : 16 * s.size(r);
  }
  return L;
}

// leaves (a box whose children are all primitives) keep their primitives right after them
static void leaf_unit(const Stream& s, const Tree& t, uint32_t b, std::vector<uint32_t>& out) {
  out.push_back(b);
  for (uint32_t c : t.kids.at(b))
    if (!s.box(c)) out.push_back(c);
}

// sibling pairs: a node's children placed together, pairs allocated in DFS order
static std::vector<uint32_t> sibling_order(const Stream& s, const Tree& t, uint32_t root) {
  std::vector<uint32_t> out{root};
  std::vector<uint32_t> st{root};
  while (!st.empty()) {
    uint32_t b = st.back();
    st.pop_back();
    auto it = t.kids.find(b);
    if (it == t.kids.end()) continue;
    for (uint32_t c : it->second) out.push_back(c);  // the children (boxes and primitives) together
    for (auto c = it->second.rbegin(); c != it->second.rend(); ++c)
      if (s.box(*c)) st.push_back(*c);
  }
  return out;
}

// sibling groups, but the groups of the top `levels` levels in BFS order
// (a contiguous hot treelet), then the remaining groups in DFS order
static std::vector<uint32_t> sibling_bfs_top(const Stream& s, const Tree& t, uint32_t root, int levels) {
  std::vector<uint32_t> out{root};
  std::vector<uint32_t> frontier{root}, deep;
  for (int l = 0; l < levels && !frontier.empty(); ++l) {
    std::vector<uint32_t> next;
    for (uint32_t b : frontier) {
      auto it = t.kids.find(b);
      if (it == t.kids.end()) continue;
      for (uint32_t c : it->second) out.push_back(c);
      for (uint32_t c : it->second)
        if (s.box(c)) next.push_back(c);
    }
    frontier = next;
  }
  std::vector<uint32_t> st(frontier.rbegin(), frontier.rend());
  while (!st.empty()) {
    uint32_t b = st.back();
    st.pop_back();
    auto it = t.kids.find(b);
    if (it == t.kids.end()) continue;
    for (uint32_t c : it->second) out.push_back(c);
    for (auto c = it->second.rbegin(); c != it->second.rend(); ++c)
      if (s.box(*c)) st.push_back(*c);
  }
  return out;
}

// hot treelet first: the `hot` boxes of largest surface area (a rooted
// treelet), BFS order, then every other record in stream order
static std::vector<uint32_t> hot_first(const Stream& s, const Tree& t, uint32_t root, size_t hot) {
  auto area = [&](uint32_t i) {
    const uint32_t* a = &s.w[4 * i];
    double dx = f(a[3]) - f(a[0]), dy = f(a[4]) - f(a[1]), dz = f(a[5]) - f(a[2]);
    return dx * dy + dy * dz + dz * dx;
  };
  std::vector<uint32_t> out;
  std::unordered_map<uint32_t, bool> in;
  std::priority_queue<std::pair<double, uint32_t>> pq;
  pq.push({area(root), root});
  while (!pq.empty() && out.size() < hot) {
    uint32_t b = pq.top().second;
    pq.pop();
    out.push_back(b);
    in[b] = true;
    for (uint32_t c : t.kids.at(b))
      if (s.box(c)) pq.push({area(c), c});
  }
  for (uint32_t r : t.recs)
    if (!in.count(r)) out.push_back(r);
  return out;
}

// subtree clusters: BFS blocks of `depth` levels, blocks emitted in DFS order
static std::vector<uint32_t> clustered(const Stream& s, const Tree& t, uint32_t root, int depth) {
  std::vector<uint32_t> out;
  std::vector<uint32_t> roots{root};
  while (!roots.empty()) {
    uint32_t r = roots.back();
    roots.pop_back();
    std::vector<uint32_t> level{r}, next_roots;
    for (int d = 0; d < depth && !level.empty(); ++d) {
      std::vector<uint32_t> nl;
      for (uint32_t b : level) {
        out.push_back(b);
        auto it = t.kids.find(b);
        if (it == t.kids.end()) continue;
        for (uint32_t c : it->second) {
          if (!s.box(c))
            out.push_back(c);
          else if (d + 1 < depth)
            nl.push_back(c);
          else
            next_roots.push_back(c);
        }
      }
      level = nl;
    }
    for (auto it = next_roots.rbegin(); it != next_roots.rend(); ++it) roots.push_back(*it);
  }
  return out;
}

int main(int argc, char** argv) {
  const char* scene = argc > 1 ? argv[1] : "mesh_ply";
  const char* assets = argc > 2 ? argv[2] : "assets";
  const int nrays = argc > 3 ? atoi(argv[3]) : 200000;
  setenv("MRT_LAYOUT", "dfs", 1);  // the preorder stream: the layouts below are made from it
  mrt_builder* b = nullptr;
  mrt_builder_new(1, &b);
  if (mrt_builder_builtin(b, scene, 16.0f / 9.0f, assets) != MRT_OK) {
    fprintf(stderr, "%s\n", mrt_builder_last_error());
    return 1;
  }
  mrt_scene_desc d;
  mrt_camera cam;
  mrt_builder_desc(b, &d, &cam);
  HostScene hs;
  std::string err;
  if (!build_host_scene(d, hs, err)) {
    fprintf(stderr, "%s\n", err.c_str());
    return 1;
  }
  Stream s{hs.slots};
  // the region to study: the largest BLAS (mesh_ply: the 1M-triangle model), or the world
  uint32_t begin = hs.world_begin;
  size_t best_len = hs.world_end - hs.world_begin;
  for (auto& r : hs.blas_regions)
    if (r.end - r.begin > best_len) best_len = r.end - r.begin, begin = r.begin;
  Tree t = parse(s, begin);
  printf("%s: region at %u, %zu records, %zu boxes\n", scene, begin, t.recs.size(), t.kids.size());

  // rays: 1080p camera rays at jittered pixels in tile order + one diffuse bounce each
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  std::vector<Ray> rays;
  std::vector<std::vector<uint32_t>> seqs;
  const int W = 1920, H = 1080;
  const int n_primary = nrays / 2;
  // a block of adjacent pixels per group of 64 rays (the pool is in 8x8-tile order)
  for (int k = 0; (int)rays.size() < n_primary; ++k) {
    int tx = (int)(U(rng) * (W / 8)), ty = (int)(U(rng) * (H / 8));
    for (int j = 0; j < 64; ++j) {
      float u = (tx * 8 + j % 8 + U(rng)) / (W - 1), v = (ty * 8 + j / 8 + U(rng)) / (H - 1);
      Ray r;
      for (int c = 0; c < 3; ++c) {
        r.o[c] = cam.origin[c];
        r.d[c] = cam.lower_left_corner[c] + cam.horizontal[c] * u + cam.vertical[c] * v - cam.origin[c];
      }
      rays.push_back(r);
    }
  }
  std::vector<Ray> bounce;
  for (const Ray& r : rays) {
    float n[3];
    float th = trace(s, begin, r, nullptr, n);
    if (!std::isfinite(th)) continue;
    float len = sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    for (float& x : n) x /= len;
    if (n[0] * r.d[0] + n[1] * r.d[1] + n[2] * r.d[2] > 0) for (float& x : n) x = -x;
    float v[3];
    do {
      for (float& x : v) x = 2 * U(rng) - 1;
    } while (v[0] * v[0] + v[1] * v[1] + v[2] * v[2] >= 1);
    Ray q;
    for (int c = 0; c < 3; ++c) q.o[c] = r.o[c] + r.d[c] * th, q.d[c] = n[c] + v[c];
    bounce.push_back(q);
  }
  rays.insert(rays.end(), bounce.begin(), bounce.end());
  seqs.resize(rays.size());
  size_t total = 0;
  for (size_t k = 0; k < rays.size(); ++k) {
    trace(s, begin, rays[k], &seqs[k], nullptr);
    total += seqs[k].size();
  }
  printf("%zu rays (%d primary), %.1f records per ray\n", rays.size(), n_primary, (double)total / rays.size());

  struct Cand {
    std::string name;
    Layout L;
  };
  std::vector<Cand> cands;
  cands.push_back({"dfs (current)", pack(s, t.recs, 16)});
  cands.push_back({"dfs, 32-B aligned", pack(s, t.recs, 32)});
  cands.push_back({"sibling pairs", pack(s, sibling_order(s, t, begin), 16)});
  cands.push_back({"sibling pairs, 32-B", pack(s, sibling_order(s, t, begin), 32)});
  cands.push_back({"sibling pairs, groups 64-B", pack_groups(s, t, sibling_order(s, t, begin), 64, 48)});
  cands.push_back({"sibling pairs, grp 64, tri 64", pack_groups(s, t, sibling_order(s, t, begin), 64, 64)});
  cands.push_back({"sib, box grp 64, prim grp 16", pack_groups(s, t, sibling_order(s, t, begin), 64, 48, 16)});
  cands.push_back({"sib, box grp 64, prim grp 32", pack_groups(s, t, sibling_order(s, t, begin), 64, 48, 32)});
  for (int lv : {6, 10, 14})
    cands.push_back({"sib 64/32, BFS top " + std::to_string(lv), pack_groups(s, t, sibling_bfs_top(s, t, begin, lv), 64, 48, 32)});
  cands.push_back({"sibling pairs, grp 128, tri 64", pack_groups(s, t, sibling_order(s, t, begin), 128, 64)});
  for (size_t hot : {1024, 16384, 131072}) cands.push_back({"hot " + std::to_string(hot) + " first", pack(s, hot_first(s, t, begin, hot), 16)});
  for (int dep : {2, 3, 4}) cands.push_back({"clusters depth " + std::to_string(dep), pack(s, clustered(s, t, begin, dep), 16)});
  for (int dep : {3}) cands.push_back({"clusters depth 3, 32-B", pack(s, clustered(s, t, begin, dep), 32)});

  const int kWaveRays = 64, kWavesPerCU = 8, kCUs = 32;
  for (auto& c : cands) {
    // lines per ray
    double lines = 0;
    for (auto& q : seqs) {
      std::vector<uint64_t> ls;
      for (uint32_t r : q) {
        uint64_t a = c.L[r], e = a + 16 * s.size(r) - 1;
        for (uint64_t l = a / 128; l <= e / 128; ++l) ls.push_back(l);
      }
      std::sort(ls.begin(), ls.end());
      lines += std::unique(ls.begin(), ls.end()) - ls.begin();
    }
    // caches: CUs take consecutive groups of 512 rays; rays advance in lockstep rounds
    LRU l2(4 * 1024 * 1024 / 128);
    uint64_t l1h = 0, l1m = 0, acc = 0;
    const size_t per_cu = (size_t)kWaveRays * kWavesPerCU;
    for (size_t base = 0; base < seqs.size(); base += per_cu * kCUs) {
      std::vector<LRU> l1(kCUs, LRU(32 * 1024 / 128));
      size_t longest = 0;
      for (size_t k = base; k < std::min(seqs.size(), base + per_cu * kCUs); ++k) longest = std::max(longest, seqs[k].size());
      for (size_t step = 0; step < longest; ++step)
        for (int cu = 0; cu < kCUs; ++cu)
          for (size_t j = 0; j < per_cu; ++j) {
            size_t k = base + cu * per_cu + j;
            if (k >= seqs.size() || step >= seqs[k].size()) continue;
            uint32_t r = seqs[k][step];
            uint64_t a = c.L[r], e = a + 16 * s.size(r) - 1;
            for (uint64_t l = a / 128; l <= e / 128; ++l) {
              ++acc;
              if (l1[cu].access(l)) continue;
              l2.access(l);
            }
          }
      for (auto& x : l1) l1h += x.hits, l1m += x.misses;
    }
    printf("%-26s lines/ray %6.2f  line accesses/ray %6.2f  L1 hit %.3f  L2 hit %.3f  L2 misses/ray %.2f\n",
           c.name.c_str(), lines / seqs.size(), (double)acc / seqs.size(), (double)l1h / (l1h + l1m),
           (double)l2.hits / (l2.hits + l2.misses), (double)l2.misses / seqs.size());
  }
  return 0;
}
