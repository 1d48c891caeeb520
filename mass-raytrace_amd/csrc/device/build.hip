// build.hip — the reference's BvhNode tree (geom.rs:110-161) built on the GPU
// (see build.h). Host: node ranges and axes in preorder. Device, per tree
// level: one stable LSD radix sort of (range start << 32 | orderable
// bbox.min[axis]) keys carrying the item order, so every node's items end up
// in exactly the order the reference's recursive stable sorts leave them;
// then node boxes bottom-up with the host's f32 min/max.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <functional>
#include <unordered_map>
#include <string>

#include "build.h"

namespace massrt {
namespace {

#define BUILD_CHECK(x)                                                                                   \
  do {                                                                                                   \
    hipError_t e_ = (x);                                                                                 \
    if (e_ != hipSuccess) throw Error(MRT_ERR_HIP, std::string("device BVH build: ") + hipGetErrorString(e_)); \
  } while (0)

constexpr uint32_t kBuildBlock = 256;

struct Seg {  // a node with >= 2 items at the level being sorted
  uint32_t lo, cnt, axis, pad;
};
struct NodeRange {
  uint32_t lo, cnt, left_p, right_p;  // preorder indices of node children (cnt >= 3)
};

// f32 -> u32 with the order of `<` (only is_less is consulted by the
// reference's sort_by, so -0 and +0 are one key)
__device__ __forceinline__ uint32_t order_key(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7FFFFFFFu) == 0) u = 0;  // -0 == +0
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Sort keys of one level: items inside a node being split get (node start,
// key of bbox.min[axis]); every other position keeps its place (key = its
// own position, which no node start inside another range can equal).
__global__ __launch_bounds__(kBuildBlock) void k_level_keys(const Seg* segs, uint32_t n_segs, const uint32_t* perm,
                                                            const float* bmin, uint32_t n, unsigned long long* keys,
                                                            uint32_t* nan_flag) {
  const uint32_t i = blockIdx.x * kBuildBlock + threadIdx.x;
  if (i >= n) return;
  // last segment with lo <= i
  uint32_t a = 0, b = n_segs;
  while (a < b) {
    const uint32_t m = (a + b) / 2;
    if (segs[m].lo <= i)
      a = m + 1;
    else
      b = m;
  }
  unsigned long long key = (unsigned long long)i << 32;
  if (a > 0) {
    const Seg s = segs[a - 1];
    if (i < s.lo + s.cnt) {
      const float f = bmin[(size_t)s.axis * n + perm[i]];
      uint32_t k = order_key(f);
      if (s.cnt == 2) {
        // 2 items: the reference compares once, `a < b` with a = the last
        // item (geom.rs:123-129); a NaN makes it false, so the first item
        // goes left — equal keys keep that order in the stable sort
        const float g = bmin[(size_t)s.axis * n + perm[i == s.lo ? i + 1 : s.lo]];
        if (f != f || g != g) k = 0;
      } else if (f != f) {
        atomicOr(nan_flag, 1u);  // >= 3 items: no order over NaN keys
      }
      key = ((unsigned long long)s.lo << 32) | k;
    }
  }
  keys[i] = key;
}

// glibc fminf/fmaxf on x86-64 (minss/maxss after the NaN checks): equal
// operands (-0, +0) give the second one — the host's BoundingBox::join.
__device__ __forceinline__ float host_fmin(float x, float y) {
  if (x != x) return y;
  if (y != y) return x;
  return x < y ? x : y;
}
__device__ __forceinline__ float host_fmax(float x, float y) {
  if (x != x) return y;
  if (y != y) return x;
  return x > y ? x : y;
}

// Node boxes of one level (deepest level first): 1 item: its box; 2 items:
// join of the two (left = first after the sort); more: join of the children.
__global__ __launch_bounds__(kBuildBlock) void k_level_boxes(const uint32_t* level_nodes, uint32_t count,
                                                             const NodeRange* nodes, const uint32_t* perm,
                                                             const float* bmin, const float* bmax, uint32_t n,
                                                             float* nbox, uint32_t T) {
  const uint32_t k = blockIdx.x * kBuildBlock + threadIdx.x;
  if (k >= count) return;
  const uint32_t p = level_nodes[k];
  const NodeRange r = nodes[p];
  float lo[3], hi[3];
  if (r.cnt <= 2) {
    const uint32_t a = perm[r.lo];
    for (int c = 0; c < 3; ++c) lo[c] = bmin[(size_t)c * n + a], hi[c] = bmax[(size_t)c * n + a];
    if (r.cnt == 2) {
      const uint32_t b = perm[r.lo + 1];
      for (int c = 0; c < 3; ++c) {
        lo[c] = host_fmin(lo[c], bmin[(size_t)c * n + b]);
        hi[c] = host_fmax(hi[c], bmax[(size_t)c * n + b]);
      }
    }
  } else {
    for (int c = 0; c < 3; ++c) {
      lo[c] = host_fmin(nbox[(size_t)c * T + r.left_p], nbox[(size_t)c * T + r.right_p]);
      hi[c] = host_fmax(nbox[(size_t)(3 + c) * T + r.left_p], nbox[(size_t)(3 + c) * T + r.right_p]);
    }
  }
  for (int c = 0; c < 3; ++c) nbox[(size_t)c * T + p] = lo[c], nbox[(size_t)(3 + c) * T + p] = hi[c];
}

// Nodes in preorder from index `base` (World::bvh_new layout): the boxes of
// k_level_boxes and the children — item refs for 1- and 2-item nodes (the
// sorted order), node refs otherwise. Written straight into the node array
// the host copies back (no per-node host pass over randomly ordered items).
__global__ __launch_bounds__(kBuildBlock) void k_assemble(const NodeRange* nodes, uint32_t T, const float* nbox,
                                                          const uint32_t* perm, const uint32_t* item_ref,
                                                          uint32_t base, mrt_node* out) {
  const uint32_t p = blockIdx.x * kBuildBlock + threadIdx.x;
  if (p >= T) return;
  const NodeRange r = nodes[p];
  mrt_node d;
  for (int c = 0; c < 3; ++c) d.min[c] = nbox[(size_t)c * T + p], d.max[c] = nbox[(size_t)(3 + c) * T + p];
  if (r.cnt <= 2) {
    d.left = item_ref[perm[r.lo]];
    d.right = r.cnt == 2 ? item_ref[perm[r.lo + 1]] : MRT_REF(MRT_REF_NONE, 0);
  } else {
    d.left = MRT_REF(MRT_REF_NODE, base + r.left_p);
    d.right = MRT_REF(MRT_REF_NODE, base + r.right_p);
  }
  out[p] = d;
}

// the identity item order (on the device: no n*4-byte pageable copy)
__global__ __launch_bounds__(kBuildBlock) void k_iota(uint32_t* perm, uint32_t n) {
  const uint32_t i = blockIdx.x * kBuildBlock + threadIdx.x;
  if (i < n) perm[i] = i;
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  explicit DevBuf(size_t n) {
    if (n) BUILD_CHECK(hipMalloc(&p, n * sizeof(T)));
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
};

uint32_t grid_for(size_t n) { return (uint32_t)((n + kBuildBlock - 1) / kBuildBlock); }

}  // namespace

void device_build_tree(int device, const std::vector<Item>& items, mrt::WyRand& rng, std::vector<mrt_node>& nodes,
                       BoundingBox& root_box, DeviceBuildStats* stats) {
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  const size_t n = items.size();
  if (n == 0) throw Error(MRT_ERR_INVALID, "BvhNode::new over an empty item list (the reference recurses forever)");
  if (n >= (1ull << 31)) throw Error(MRT_ERR_INVALID, "device BVH build: too many items");
  // ---- host: node ranges level by level (the tree's shape depends on the
  // item count alone: n >= 3 splits at n/2), numbered in preorder — a node's
  // left child is p + 1, its right child p + 1 + size(left subtree) — and
  // one axis draw per node in preorder (bvh_new order, geom.rs:111).
  std::unordered_map<uint32_t, uint32_t> memo;
  std::function<uint32_t(uint32_t)> tree_size = [&](uint32_t c) -> uint32_t {
    if (c <= 2) return 1u;
    auto it = memo.find(c);
    if (it != memo.end()) return it->second;
    const uint32_t v = 1u + tree_size(c / 2) + tree_size(c - c / 2);
    memo.emplace(c, v);
    return v;
  };
  const uint32_t T = tree_size((uint32_t)n);
  std::vector<NodeRange> range(T);
  std::vector<uint8_t> axis(T);
  for (uint32_t p = 0; p < T; ++p) axis[p] = (uint8_t)rng.axis();  // fastrand::u8(0..3) per node, in preorder
  struct Frame {
    uint32_t p, lo, cnt;
  };
  std::vector<std::vector<Seg>> segs;
  std::vector<uint32_t> level_off{0}, level_nodes;
  level_nodes.reserve(T);
  std::vector<Frame> cur{{0u, 0u, (uint32_t)n}}, next;
  while (!cur.empty()) {  // one tree level, in ascending lo (= ascending preorder index)
    segs.emplace_back();
    next.clear();
    for (const Frame& f : cur) {
      NodeRange& r = range[f.p];
      r = NodeRange{f.lo, f.cnt, ~0u, ~0u};
      level_nodes.push_back(f.p);
      if (f.cnt >= 2) segs.back().push_back(Seg{f.lo, f.cnt, axis[f.p], 0});
      if (f.cnt >= 3) {
        const uint32_t half = f.cnt / 2;
        r.left_p = f.p + 1;
        r.right_p = f.p + 1 + tree_size(half);
        next.push_back(Frame{r.left_p, f.lo, half});
        next.push_back(Frame{r.right_p, f.lo + half, f.cnt - half});
      }
    }
    level_off.push_back((uint32_t)level_nodes.size());
    std::swap(cur, next);
  }
  const uint32_t L = (uint32_t)segs.size();
  if (level_nodes.size() != T) throw Error(MRT_ERR_INVALID, "device BVH build: node count mismatch (internal)");
  const auto t1 = clock::now();

  // ---- device
  BUILD_CHECK(hipSetDevice(device));
  hipStream_t st;
  BUILD_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamDestroy(s); }
  } sg{st};
  std::vector<float> hb(6 * n);
  std::vector<uint32_t> href(n);
  for (size_t i = 0; i < n; ++i) {
    const BoundingBox& b = items[i].box;
    hb[0 * n + i] = b.minimum.x, hb[1 * n + i] = b.minimum.y, hb[2 * n + i] = b.minimum.z;
    hb[3 * n + i] = b.maximum.x, hb[4 * n + i] = b.maximum.y, hb[5 * n + i] = b.maximum.z;
    href[i] = items[i].ref;
  }
  size_t total_segs = 0;
  for (auto& s : segs) total_segs += s.size();
  DevBuf<float> d_box(6 * n), d_nbox(6 * (size_t)T);
  DevBuf<uint32_t> d_perm(n), d_perm2(n), d_level_nodes(T), d_nan(1);
  DevBuf<unsigned long long> d_keys(n), d_keys2(n);
  DevBuf<Seg> d_segs(total_segs ? total_segs : 1);
  DevBuf<NodeRange> d_range(T);
  DevBuf<uint32_t> d_ref(n);
  DevBuf<mrt_node> d_out(T);
  BUILD_CHECK(hipMemcpyAsync(d_box.p, hb.data(), hb.size() * 4, hipMemcpyHostToDevice, st));
  BUILD_CHECK(hipMemcpyAsync(d_ref.p, href.data(), n * 4, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n)), dim3(kBuildBlock), 0, st, d_perm.p, (uint32_t)n);
  BUILD_CHECK(hipGetLastError());
  BUILD_CHECK(hipMemcpyAsync(d_range.p, range.data(), (size_t)T * sizeof(NodeRange), hipMemcpyHostToDevice, st));
  BUILD_CHECK(hipMemcpyAsync(d_level_nodes.p, level_nodes.data(), (size_t)T * 4, hipMemcpyHostToDevice, st));
  BUILD_CHECK(hipMemsetAsync(d_nan.p, 0, 4, st));
  std::vector<size_t> seg_off(L + 1, 0);
  for (uint32_t l = 0; l < L; ++l) {
    seg_off[l + 1] = seg_off[l] + segs[l].size();
    if (!segs[l].empty())
      BUILD_CHECK(hipMemcpyAsync(d_segs.p + seg_off[l], segs[l].data(), segs[l].size() * sizeof(Seg),
                                 hipMemcpyHostToDevice, st));
  }
  uint32_t pos_bits = 1;
  while ((1ull << pos_bits) < n) ++pos_bits;
  const int end_bit = 32 + (int)pos_bits;
  size_t temp_bytes = 0;
  BUILD_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, d_keys.p, d_keys2.p, d_perm.p, d_perm2.p,
                                                 (int)n, 0, end_bit, st));
  DevBuf<char> d_temp(temp_bytes ? temp_bytes : 1);
  uint32_t* perm = d_perm.p;
  uint32_t* perm_alt = d_perm2.p;
  for (uint32_t l = 0; l < L; ++l) {
    if (segs[l].empty()) continue;
    hipLaunchKernelGGL(k_level_keys, dim3(grid_for(n)), dim3(kBuildBlock), 0, st, d_segs.p + seg_off[l],
                       (uint32_t)segs[l].size(), perm, d_box.p, (uint32_t)n, d_keys.p, d_nan.p);
    BUILD_CHECK(hipGetLastError());
    BUILD_CHECK(hipcub::DeviceRadixSort::SortPairs(d_temp.p, temp_bytes, d_keys.p, d_keys2.p, perm, perm_alt, (int)n,
                                                   0, end_bit, st));
    std::swap(perm, perm_alt);
  }
  for (uint32_t l = L; l-- > 0;) {
    const uint32_t cnt = level_off[l + 1] - level_off[l];
    hipLaunchKernelGGL(k_level_boxes, dim3(grid_for(cnt)), dim3(kBuildBlock), 0, st, d_level_nodes.p + level_off[l],
                       cnt, d_range.p, perm, d_box.p, d_box.p + 3 * n, (uint32_t)n, d_nbox.p, T);
    BUILD_CHECK(hipGetLastError());
  }
  // ---- nodes in preorder from the first free index (World::bvh_new layout),
  // assembled on the device and copied straight into the node array
  const uint32_t base = (uint32_t)nodes.size();
  hipLaunchKernelGGL(k_assemble, dim3(grid_for(T)), dim3(kBuildBlock), 0, st, d_range.p, T, d_nbox.p, perm, d_ref.p,
                     base, d_out.p);
  BUILD_CHECK(hipGetLastError());
  uint32_t nan_flag = 0;
  BUILD_CHECK(hipMemcpyAsync(&nan_flag, d_nan.p, 4, hipMemcpyDeviceToHost, st));
  BUILD_CHECK(hipStreamSynchronize(st));
  if (nan_flag)
    throw Error(MRT_ERR_INVALID, "device BVH build: a NaN bounding-box key (the reference's sort order is undefined)");
  nodes.resize(base + (size_t)T);
  try {
    BUILD_CHECK(hipMemcpyAsync(nodes.data() + base, d_out.p, (size_t)T * sizeof(mrt_node), hipMemcpyDeviceToHost, st));
    BUILD_CHECK(hipStreamSynchronize(st));
  } catch (...) {
    nodes.resize(base);  // the node array is unchanged by a failed build
    throw;
  }
  const auto t2 = clock::now();
  root_box.minimum = V3{nodes[base].min[0], nodes[base].min[1], nodes[base].min[2]};
  root_box.maximum = V3{nodes[base].max[0], nodes[base].max[1], nodes[base].max[2]};
  if (stats) {
    stats->host_ms = std::chrono::duration<double, std::milli>(t1 - t0).count() +
                     std::chrono::duration<double, std::milli>(clock::now() - t2).count();
    stats->device_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
    stats->levels = L;
  }
}

}  // namespace massrt
