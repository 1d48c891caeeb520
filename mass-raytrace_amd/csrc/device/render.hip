// render.hip — the wavefront path-tracing integrator for gfx950 and the
// device half of the C ABI (include/massrt.h).
//
// Replaces render()'s per-thread pixel loop (main.rs:235-290): each sample
// (one camera path, main.rs:257-263) becomes a path slot in a pool of SoA
// HBM buffers, advanced one segment per iteration by two kernels:
//   k_trace : closest hit of every active ray (World::intersect)      [k2]
//   k_shade : emit/scatter/background, path termination and wave
//             ballot/prefix-sum compaction of the survivors           [k3,k4]
//   k_reserve + k_refill : new camera rays (Camera::ray) for the free
//             slots behind the survivors                              [k1]
// Finished samples are written to a per-(pixel,sample) result slab and folded
// into the caller's accumulation buffers in sample order by k_accumulate [k5]
// (Image::merge, main.rs:629-638), so the sums do not depend on scheduling
// or on how tiles are sharded across GPUs.
#include <hip/hip_runtime.h>
#include <string.h>

#include <array>
#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../../include/massrt.h"
#include "../host/display.h"
#include "frames.h"
#include "path.h"
#include "upload.h"

using namespace mrt;

namespace {

struct HipError {
  std::string msg;
};
#define HIP_CHECK(x)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) throw HipError{std::string(#x) + ": " + hipGetErrorString(e_)}; \
  } while (0)

struct ApiError {
  int code;
  std::string msg;
};

constexpr int kBlock = 256;

// XCD groups: workgroups are dealt round-robin over the 8 XCDs, so
// blockIdx.x % 8 names the workgroups that share one XCD's L2.
constexpr uint32_t kGroups = 8;
struct Ctrl {
  uint32_t active[2];
  uint32_t next_work;
  uint32_t shade_short;  // nonzero: a k_shade grid did not cover its live pool (host bound wrong; reported)
  // shade_bin 2: the survivors of the first half of the keys counted from the
  // bottom of the next pool (low word) and of the second half from its top
  // (high word), in one 64-bit word so that a workgroup reserves both with
  // ONE atomic (two, one per word, doubled k_shade's solo time: every
  // workgroup's atomics go to this one line)
  unsigned long long surv[2];
  // refill (k_reserve -> k_refill): work items [gen_base, gen_base + gen_count)
  // go to pool slots [gen_slot, gen_slot + gen_count), behind the survivors
  uint32_t gen_slot, gen_count, gen_base;
  // shade_bin 2: k_reserve closes the gap between the pool's two ends that
  // the refill leaves: k_refill moves gen_move paths from gen_move_src.. to
  // gen_move_dst..
  uint32_t gen_move, gen_move_src, gen_move_dst;
  uint32_t pad_[18];
  // persistent k_trace work counters (zeroed by k_shade), one 128-B line per
  // XCD group: group g takes its rays from the g-th eighth of the pool
  uint32_t group_next[kGroups * 32];
};

// SoA path state, 5 x 16 B per slot:
//   ro  = {o.x, o.y, o.z, work index g}    rd  = {d.x, d.y, d.z, bounces k}
//   thr = {T.x, T.y, T.z, kHoldsL or 0}    rad = {L.x, L.y, L.z, -}
//   rng = xoroshiro128** {s0.lo, s0.hi, s1.lo, s1.hi}
// rad is read and written only while thr.w says the path holds radiance
// (some component of L has nonzero bits): a path gains L only where a hit
// both emits and scatters (a Mix of DiffuseLight and a scattering material)
// — most paths end where they first gain it — so the slot's rad is
// otherwise stale and L is +0.
constexpr uint32_t kHoldsL = 1u;
__device__ __forceinline__ bool holds_l(const float4& thr) { return __float_as_uint(thr.w) != 0u; }
__device__ __forceinline__ bool nonzero_bits(float x, float y, float z) {
  return (__float_as_uint(x) | __float_as_uint(y) | __float_as_uint(z)) != 0u;
}
struct PathBufs {
  float4* ro;
  float4* rd;
  float4* thr;
  float4* rad;
  uint4* rng;
};

struct RenderParams {
  uint32_t W, H;
  unsigned long long seed;
  uint32_t max_depth;
  uint32_t n_pix;        // pixels in this shard
  uint32_t G;            // work items in this chunk = n_pix * spp
  uint32_t spp;          // samples per pixel in this chunk
  uint32_t sample_base;  // absolute sample index of chunk sample 0
  uint32_t pool_cap;     // path slots per buffer
  const uint32_t* pixlist;
  uint32_t shade_bin;    // k_shade: survivors grouped by material kind and direction in the next pool (option shade_bin)
};

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t lane_rank(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

constexpr uint32_t kWaves = kBlock / 64;
// k_shade's workgroup: its survivors are grouped (option shade_bin) within
// one workgroup, so the size sets the grouping's scope
#ifndef MRT_SHADE_BLOCK
#define MRT_SHADE_BLOCK 256
#endif
constexpr int kShadeBlock = MRT_SHADE_BLOCK;

// Workgroup-wide reservation of `count` (this wave's share) consecutive
// slots from *counter: one atomic per workgroup; returns this wave's first
// slot. Every thread of the workgroup must call it.
template <uint32_t NW = kWaves>
__device__ __forceinline__ uint32_t wg_reserve(uint32_t* counter, uint32_t count, uint32_t wave, uint32_t* s_cnt,
                                               uint32_t& s_base) {
  if (lane_id() == 0) s_cnt[wave] = count;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t total = 0;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) total += s_cnt[w];
    s_base = total ? atomicAdd(counter, total) : 0u;
  }
  __syncthreads();
  uint32_t base = s_base;
  for (uint32_t w = 0; w < wave; ++w) base += s_cnt[w];
  __syncthreads();  // s_cnt/s_base are reused by the next call
  return base;
}

// wg_reserve for the alive lanes, the workgroup's survivors ordered by `key`
// (< kOutKeys): a lane's rank within its key comes from an LDS atomic (so
// the order within a key is arbitrary — paths are independent, the images
// do not depend on it), the keys' offsets from one wave's scan of the
// histogram. k_shade uses it to group the next pool's rays by the material
// kind they scattered from and the signs of their direction's y and x
// (option shade_bin): k_trace's waves then walk rays that go the same way
// together (round 5, profiles/r5_shade_bin/: kind only 1003 / 514, octant
// 1018 / 526, kind x octant 1022 / 528, y sign only 1038 / 531, kind x y x x
// 1035 / 535 Msamples/s on sphere_grid / cube_field, none 974 / 504). Every
// thread of the workgroup must call it.
constexpr uint32_t kOutKeys = 64;  // one wave scans the histogram (k_shade's keys use 32)
// hi != nullptr (shade_bin 2): keys >= 32 take slots counted down from the
// top of the pool (cap - 1, cap - 2, ...) instead: both counts go to *hi
// (low word: from the bottom, high word: from the top, one atomic; *counter
// is unused), the next pool then holds the two halves at its two ends, and
// k_reserve/k_refill put the new camera rays between them.
__device__ __forceinline__ uint32_t wg_reserve_keyed(uint32_t* counter, bool alive, uint32_t key, uint32_t* s_hist,
                                                     unsigned long long* hi = nullptr, uint32_t cap = 0) {
  if (threadIdx.x < kOutKeys) s_hist[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t rank = alive ? atomicAdd(&s_hist[key], 1u) : 0u;
  __syncthreads();
  if (threadIdx.x < kOutKeys) {  // wave 0: exclusive scan of the 64 counts
    const uint32_t c = s_hist[threadIdx.x];
    uint32_t v = c;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t u = __shfl_up(v, d, 64);
      if (lane_id() >= d) v += u;
    }
    const uint32_t total = __shfl(v, 63, 64);
    const uint32_t tlo = hi ? __shfl(v, 31, 64) : total, thi = total - tlo;
    uint32_t b = 0, bh = 0;
    if (threadIdx.x == 0) {
      if (hi) {
        const unsigned long long r = total ? atomicAdd(hi, ((unsigned long long)thi << 32) | tlo) : 0ull;
        b = (uint32_t)r;
        bh = (uint32_t)(r >> 32);
      } else {
        b = total ? atomicAdd(counter, total) : 0u;
      }
    }
    b = __shfl(b, 0, 64);
    bh = __shfl(bh, 0, 64);
    s_hist[threadIdx.x] = hi && threadIdx.x >= 32 ? cap - 1u - bh - (v - c - tlo) : b + v - c;
  }
  __syncthreads();
  const uint32_t slot = hi && key >= 32 ? s_hist[key] - rank : s_hist[key] + rank;
  __syncthreads();  // s_hist is reused by the next call
  return slot;
}

__device__ void flush_counters(DevCounters* c, const LocalCounters& lc, uint32_t segs, uint32_t hits,
                               uint32_t samples, uint32_t bounces, uint32_t shaded = 0) {
  uint32_t v[18] = {samples,         segs,           lc.node_visits, lc.sphere_tests,   lc.triangle_tests, lc.instance_entries,
                    lc.model_entries, hits,           lc.texel_taps,  bounces,           lc.wave_slots,     lc.lane_steps,
                    lc.box_exact,     shaded,         lc.vnf_fallbacks, lc.shade_waves, lc.shade_kinds,    lc.shade_materials};
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(c);
#pragma unroll
  for (int k = 0; k < 18; ++k) {
    uint32_t s = wave_sum(v[k]);
    if (lane_id() == 0 && s) atomicAdd(dst + k, (unsigned long long)s);
  }
}

__device__ __forceinline__ void gen_work(const DevCamera& cam, const RenderParams& rp, uint32_t g, float4& ro,
                                         float4& rd, uint4& rs) {
  // work items run sample-minor: the samples of one pixel are consecutive
  // (camera rays of a wave nearly equal), and the results slab is laid out
  // the same way, g = pixel * spp + sample
  uint32_t lp = g / rp.spp;
  uint32_t s_local = g - lp * rp.spp;
  uint32_t p = rp.pixlist[lp];  // lp < n_pix by construction (g < G)
  uint32_t y = p / rp.W, x = p - y * rp.W;
  PathRng rng = path_rng(rp.seed, p, rp.sample_base + s_local);
  V3 o, d;
  camera_ray(cam, x, y, rp.W, rp.H, rng, o, d);
  ro = make_float4(o.x, o.y, o.z, __uint_as_float(g));
  rd = make_float4(d.x, d.y, d.z, __uint_as_float(0u));
  rs = make_uint4((uint32_t)rng.s0, (uint32_t)(rng.s0 >> 32), (uint32_t)rng.s1, (uint32_t)(rng.s1 >> 32));
}

// Initial pool: work items [base, base + n0) into slots [0, n0).
__global__ __launch_bounds__(kBlock) void k_generate(DevCamera cam, RenderParams rp, PathBufs out, uint32_t base,
                                                     uint32_t n0) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n0) return;
  float4 ro, rd;
  uint4 rs;
  gen_work(cam, rp, base + i, ro, rd, rs);
  out.ro[i] = ro;
  out.rd[i] = rd;
  out.thr[i] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);  // L = 0: rad not written
  out.rng[i] = rs;
}

// Lagged status read of a queue (host loop, one per batch): the fields the
// host needs, written by one wave straight into pinned host memory. A
// hipMemcpyAsync to pinned memory ran as a 1024-thread blit kernel, which
// waited for a CU with 16 free wave slots while both queues' kernels held
// the chip (12-46 ms per read in the kernel trace, the queue's stream stalled
// behind it); one wave finds a slot at once.
struct HostStatus {
  uint32_t active0, active1, shade_short, work;
};
__global__ void k_status(const Ctrl* ctrl, const uint32_t* work, HostStatus* out) {
  if (threadIdx.x != 0) return;
  HostStatus h;
  h.active0 = ctrl->active[0];
  h.active1 = ctrl->active[1];
  h.shade_short = ctrl->shade_short;
  h.work = *work;
  *out = h;
  __threadfence_system();
}

// Refill after k_shade compacted the survivors of pool `cur` into the next
// pool (ctrl->active[cur ^ 1] of them): reserve work items for the free slots
// behind them from the shared work counter. One thread; the counter is only
// advanced while it is below G, so it passes G by at most a pool per queue.
__global__ void k_reserve(Ctrl* ctrl, uint32_t cur, uint32_t* work, uint32_t G, uint32_t cap) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const unsigned long long sv = ctrl->surv[cur ^ 1];  // 0 unless shade_bin 2
  const uint32_t lo = ctrl->active[cur ^ 1] + (uint32_t)sv, hi = (uint32_t)(sv >> 32), n = lo + hi;
  const uint32_t want = n < cap ? cap - n : 0u;
  uint32_t m = 0, base = G;
  if (want && __hip_atomic_load(work, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < G) {
    base = atomicAdd(work, want);
    m = base < G ? (G - base < want ? G - base : want) : 0u;
  }
  ctrl->gen_slot = lo;
  ctrl->gen_count = m;
  ctrl->gen_base = base;
  // the top block [cap - hi, cap) closes onto the refill's end lo + m: its
  // paths at or past the new end E move into the free slots below E
  const uint32_t E = n + m, g = cap - E;
  const uint32_t mv = g < hi ? g : hi;
  ctrl->gen_move = mv;
  ctrl->gen_move_src = cap - mv;
  ctrl->gen_move_dst = lo + m;
  ctrl->active[cur ^ 1] = E;
  ctrl->surv[cur ^ 1] = 0;
}

// ... and generate them (camera rays of consecutive work items, i.e. pixel
// order): the next k_trace finds the new paths together behind the
// survivors instead of scattered among them one per finished slot.
__global__ __launch_bounds__(kBlock) void k_refill(DevCamera cam, RenderParams rp, PathBufs out, const Ctrl* ctrl) {
  const uint32_t m = ctrl->gen_count, slot = ctrl->gen_slot, base = ctrl->gen_base;
  const uint32_t mv = ctrl->gen_move, src = ctrl->gen_move_src, dst = ctrl->gen_move_dst;
  for (uint32_t j = blockIdx.x * kBlock + threadIdx.x; j < mv; j += gridDim.x * kBlock) {
    // sources [cap - mv, cap) and destinations [lo + m, lo + m + mv) are disjoint
    const uint32_t a = src + j, b = dst + j;
    const float4 thr = out.thr[a];
    out.ro[b] = out.ro[a];
    out.rd[b] = out.rd[a];
    out.thr[b] = thr;
    if (holds_l(thr)) out.rad[b] = out.rad[a];
    out.rng[b] = out.rng[a];
  }
  for (uint32_t j = blockIdx.x * kBlock + threadIdx.x; j < m; j += gridDim.x * kBlock) {
    float4 ro, rd;
    uint4 rs;
    gen_work(cam, rp, base + j, ro, rd, rs);
    const uint32_t i = slot + j;
    out.ro[i] = ro;
    out.rd[i] = rd;
    out.thr[i] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);  // L = 0: rad not written
    out.rng[i] = rs;
  }
}

// Persistent closest-hit kernel: a fixed grid of waves pulls chunks of rays
// from a counter; inside a wave a lane whose ray has finished takes the next
// ray of the wave's chunk as soon as enough lanes are idle, so the SIMD keeps
// issuing for busy lanes instead of waiting for the wave's slowest ray.
constexpr float kTmin = 0.001f;          // World::intersect(ray, 0.001, INFINITY) (main.rs trace)
// Scheduling knobs of the persistent loop (kernel arguments so that they can
// be tuned without a rebuild: options "trace_refill", "trace_chunk", ...).
// samples per results slab at most (16 B each, one slab per queue set):
// mrt_ctx::results_max, 2^31 = 32 GiB by default (option "results_log2")
constexpr uint64_t kResultsMaxLimit = 1ull << 31;

struct TraceTune {
  uint32_t chunk = 128;     // rays per atomic grab
  uint32_t refill = 32;      // refill once this many lanes idle
  uint32_t prim_batch = 1;   // run the primitive branch once this many lanes wait at one
  uint32_t box_min = 24;     // inner box loop while this many lanes are at a box (65: off)
  uint32_t shade_batch = 16; // k_render: shade once this many lanes finished a segment
  uint32_t nf_batch = 32;    // near-first walk: check the hits once this many lanes' walks are over
  uint32_t prim_run = 32;    // primitive steps alone while this many lanes are at a primitive (65: off)
};

// LDS=true: the scene's treelet (layout.h, upload.cpp build_treelet) is first
// copied into the workgroup's LDS; records with an LDS-tagged index are then
// read there (ds_read_b128) instead of through L1/L2 — the top of the trees,
// which every ray visits, and small instanced BLAS whole. BLK threads per
// workgroup share one copy.
constexpr size_t kTraceLdsMaxBytes = 160 * 1024;
constexpr uint32_t kIdle = 0xFFFFFFFFu;  // Trav.ray of a lane without a ray
constexpr uint32_t kStashQuads = 4;      // float4s per lane of the world-ray stash (TravIn::stash)

// RNG: the scene's traversal draws random numbers (Volume, Mix alpha tests):
// each ray carries its path stream through the traversal and stores it back.
// (R > 1 would interleave R rays per lane — software ILP; measured slower at
// its 84 VGPRs, so only R = 1 is instantiated.)
// NF: the verified near-first walk (path.h trav_*_nf): the SAH trees walked
// near child first with a per-lane stack in LDS (kNfStack x BLK words of
// dynamic shared memory), the winner checked against the reference tree,
// rays that fail the check walked again the reference's way.
template <bool COUNT, bool LDS, uint32_t ALPHA, bool RNG, int BLK, bool NF = false>
__global__ __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(NF ? (COUNT ? 1 : 5) : (ALPHA == 0 && !RNG && !COUNT ? 8 : 1)))) void k_trace(DevScene S, PathBufs in, uint4* hits, Ctrl* ctrl, uint32_t cur,
                                                  DevCounters* cnt, float tmin, float tmax, TraceTune tune) {
  static_assert(!NF || (!LDS && !RNG), "the near-first walk has no treelet and no traversal draws");
  constexpr int R = 1;
  const uint32_t n = ctrl->active[cur];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ctrl->active[cur ^ 1] = 0;
    ctrl->surv[cur ^ 1] = 0;
  }
  if (n == 0) return;  // uniform: every workgroup reads the same n
  if (LDS) {
    for (uint32_t k = threadIdx.x; k < S.n_tlet; k += BLK) mrt_lds[k] = reinterpret_cast<const uint4*>(S.tlet)[k];
    __syncthreads();
  }
  TravIn tin_{S, reinterpret_cast<const uint4*>(LDS ? S.slots_tl : S.slots), LDS ? S.tl_world_begin : S.world_begin,
              in.ro, in.rd, tmin, in.rng, tmax};
  if (!LDS && !NF) {  // the reference walk without a treelet: LDS holds the world-ray stash (TravIn::stash)
    tin_.stash = reinterpret_cast<float4*>(mrt_lds) + threadIdx.x;
    tin_.stash_stride = (uint32_t)BLK;
  }
  const TravIn& tin = tin_;
  const NfStack stk{reinterpret_cast<uint32_t*>(mrt_lds) + threadIdx.x, (uint32_t)BLK};
  LocalCounters lc;
  uint32_t seg = 0, nh = 0;
  uint32_t pool = 0, pool_end = 0;  // wave-uniform chunk [pool, pool_end)
  bool drained = false;             // wave-uniform: every group's share is taken
  // XCD-aware ray ranges: the pool is roughly in pixel order (camera rays in
  // tile order, survivors compacted in order), so giving each XCD group a
  // contiguous eighth keeps an XCD's rays — and the scene parts they touch —
  // together in that XCD's L2. A group whose eighth is taken helps the next.
  uint32_t grp = blockIdx.x % kGroups, visited = 0;  // wave-uniform
  Trav t[R];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    t[q] = Trav{};  // fully initialised: idle lanes must not carry undefined state
    t[q].done = true;
    t[q].ray = kIdle;
  }
  for (;;) {
    unsigned long long idle[R];
    uint32_t n_idle = 0;
#pragma unroll
    for (int q = 0; q < R; ++q) {
      idle[q] = __ballot(t[q].ray == kIdle);
      n_idle += (uint32_t)__popcll(idle[q]);
    }
    if (n_idle >= tune.refill * R || n_idle == 64u * R) {
      while (pool == pool_end && !drained) {  // grab the next chunk (wave-uniform)
        const uint32_t lo = (uint32_t)((uint64_t)n * grp / kGroups), hi = (uint32_t)((uint64_t)n * (grp + 1) / kGroups);
        uint32_t b = 0;
        if (lane_id() == 0) b = atomicAdd(&ctrl->group_next[grp * 32], tune.chunk);
        b = __shfl(b, 0, 64);
        if (b < hi - lo) {
          pool = lo + b;
          pool_end = hi - pool > tune.chunk ? pool + tune.chunk : hi;
        } else if (++visited == kGroups) {
          drained = true;
        } else {
          grp = (grp + 1) % kGroups;
        }
      }
      const uint32_t avail = pool_end - pool;
      uint32_t off = 0;
      unsigned long long live = 0;
#pragma unroll
      for (int q = 0; q < R; ++q) {
        if (t[q].ray == kIdle) {
          const uint32_t r = off + lane_rank(idle[q]);
          if (r < avail) trav_init<RNG, LDS>(tin, t[q], MRT_IDX(S, pool + r, n, 20), tmax, NF ? S.nf_world : 0xFFFFFFFFu);
        }
        off += (uint32_t)__popcll(idle[q]);
        live |= __ballot(t[q].ray != kIdle);
      }
      pool += n_idle < avail ? n_idle : avail;
      if (live == 0) break;  // chunk source exhausted
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
      // box run: keep stepping boxes with little per-step overhead while at
      // least tune.box_min lanes are at one (lanes reaching a primitive wait)
      // Two steps per loop iteration: with one, the compiler carried the
      // record just loaded into the loop-header registers with 8 v_mov per
      // step; unrolled, the two steps alternate register sets and the copies
      // are gone (sphere_grid 671 -> 703, cube_field 254 -> 266, mesh_ply
      // 740 -> 749 Msamples/s, same box).
      auto box_step = [&]() {  // false: too few lanes at a box
        // a done lane holds an END record (or an idle lane's zeros), never a
        // box, so the record's flag alone decides (no done mask in the ballot)
        const bool run_box = trav_at_box(t[q]);
        const unsigned long long bm = __builtin_amdgcn_ballot_w64(run_box);
        if ((uint32_t)__popcll(bm) < tune.box_min) return false;
        if (run_box) {
          if (NF && t[q].sp != kExactMode)
            trav_box_index_nf<COUNT>(tin, stk, t[q], lc);
          else
            trav_box_index<COUNT>(tin, t[q], lc);
        }
        if (run_box && (!NF || t[q].sp != kNfDone)) trav_fetch<LDS>(tin, t[q]);
        if (COUNT) {
          lc.wave_slots += lane_id() == 0 ? 64u : 0u;
          lc.lane_steps += run_box ? 1u : 0u;
        }
        return true;
      };
      while (box_step() && box_step()) {
      }
      // idle lanes hold a done Trav; a near-first lane whose walk is over
      // waits for the check below.
      // One step per busy lane (a box, or a primitive once enough lanes wait
      // at one or no lane is at a box), then ONE record fetch for every lane
      // that moved: the address unit costs per wave instruction, so the box
      // and primitive lanes share the load pair instead of issuing one each.
      // Primitive run (the box run's mirror): while at least tune.prim_run
      // lanes are at a primitive, they step alone (a leaf's primitives one
      // after another) instead of paying the box branch beside each step —
      // the same code with the box lanes masked off, so nothing is inlined twice
      for (;;) {
        const bool busy = !t[q].done && (!NF || t[q].sp != kNfDone);
        const bool at_box = busy && trav_at_box(t[q]);
        const unsigned long long box_mask = __ballot(at_box);
        const unsigned long long prim_mask = __ballot(busy && !at_box);
        // (the near-first walk only: the reference walk's k_trace, compiled
        // with this loop, lost 14% — 971 -> 832 on sphere_grid at any
        // threshold, profiles/r6_primrun/ — so there it folds to one step)
        const bool prim_run = NF && (uint32_t)__popcll(prim_mask) >= tune.prim_run;  // wave-uniform
        const bool box_go = at_box && !prim_run;
        const bool prim_go = (__popcll(prim_mask) >= tune.prim_batch || box_mask == 0) && busy && !at_box;
        if (box_go) {
          if (NF && t[q].sp != kExactMode)
            trav_box_index_nf<COUNT>(tin, stk, t[q], lc);
          else
            trav_box_index<COUNT>(tin, t[q], lc);
        }
        if (prim_go) {
          if (NF && t[q].sp != kExactMode)
            trav_prim_index_nf<COUNT, ALPHA>(tin, stk, t[q], lc);
          else
            trav_prim_index<COUNT, ALPHA, RNG, LDS>(tin, t[q], lc);
        }
        if ((box_go || prim_go) && !t[q].done && (!NF || t[q].sp != kNfDone)) trav_fetch<LDS>(tin, t[q]);
        if (COUNT) {
          lc.wave_slots += lane_id() == 0 ? 64u : 0u;
          lc.lane_steps += (box_go || prim_go) ? 1u : 0u;
        }
        if (!prim_run) break;
      }
      // near-first walks that are over: check their hits (done, or the
      // reference's walk from the start) — batched: the check is a few
      // hundred wave instructions, so finished lanes wait (holding an END
      // record) until tune.nf_batch of them can share one pass, or until no
      // lane is walking any more
      if (NF) {
        const bool over = t[q].sp == kNfDone;
        const unsigned long long om = __builtin_amdgcn_ballot_w64(over);
        if (om != 0 && ((uint32_t)__popcll(om) >= tune.nf_batch ||
                        __builtin_amdgcn_ballot_w64(!t[q].done && !over) == 0) && over) {
          nf_finish<COUNT>(tin, t[q], lc);
          if (!t[q].done) trav_fetch<LDS>(tin, t[q]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
      if (t[q].ray != kIdle && t[q].done) {
        if (RNG) trav_store_rng(tin, t[q]);
        const Hit h = trav_hit<LDS>(tin, t[q]);
        hits[t[q].ray] = make_uint4(__float_as_uint(h.t), h.prim, h.container, 0u);
        seg += 1;
        nh += t[q].prim != kRefNone;
        t[q].ray = kIdle;
      }
    }
  }
  if (COUNT) flush_counters(cnt, lc, seg, nh, 0, 0);
}

// Debug/bisection variant (MRT_RENDER_SIMPLE_TRACE): one ray per thread,
// the whole traversal in closest_hit.
template <bool RNG>
__global__ __launch_bounds__(kBlock) void k_trace_simple(DevScene S, PathBufs in, uint4* hits, Ctrl* ctrl,
                                                         uint32_t cur, DevCounters* cnt) {
  const uint32_t n = ctrl->active[cur];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ctrl->active[cur ^ 1] = 0;
    ctrl->surv[cur ^ 1] = 0;
  }
  LocalCounters lc;
  uint32_t seg = 0, nh = 0;
  const TravIn tin{S, reinterpret_cast<const uint4*>(S.slots), S.world_begin, in.ro, in.rd, kTmin, in.rng};
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    PathRng rng{0, 0};
    if (RNG) {
      const uint4 q = in.rng[i];
      rng = PathRng{(unsigned long long)q.x | ((unsigned long long)q.y << 32),
                    (unsigned long long)q.z | ((unsigned long long)q.w << 32)};
    }
    Hit h = closest_hit<true, RNG>(tin, i, INFINITY, lc, rng);
    if (RNG)
      in.rng[i] = make_uint4((uint32_t)rng.s0, (uint32_t)(rng.s0 >> 32), (uint32_t)rng.s1, (uint32_t)(rng.s1 >> 32));
    hits[i] = make_uint4(__float_as_uint(h.t), h.prim, h.container, 0u);
    seg += 1;
    nh += h.prim != kRefNone;
  }
  flush_counters(cnt, lc, seg, nh, 0, 0);
}

// One level of main.rs trace() after World::intersect returned `h` for the
// ray (o, d): adds T * emitted (hit) or T * background (miss) to L; on a
// scatter that continues (and depth left) moves (o, d) to the scattered ray,
// multiplies T by the attenuation and returns true.
// (mat: the hit's material index, kShadeMiss for a miss: the counting
// k_shade's coherence counters)
constexpr uint32_t kShadeMiss = 0xFFFFFFFEu, kShadeIdle = 0xFFFFFFFFu;
template <bool EXT>
MRT_DEV bool shade_step(const DevScene& S, uint32_t max_depth, const Hit& h, V3& o, V3& d, V3& T, V3& L, uint32_t& k,
                        PathRng& rng, LocalCounters& lc, uint32_t& nbounce, uint32_t& mat) {
  if (h.prim == kRefNone) {
    mat = kShadeMiss;
    L = L + T * background<EXT>(S, d, lc);
    return false;
  }
  Surf s = resolve_hit(S, o, d, h);
  mat = s.material;
  V3 emitted, atten, nd;
  bool cont = scatter<EXT>(S, s, d, rng, emitted, atten, nd, lc);
  L = L + T * emitted;
  if (!cont) return false;
  T = T * atten;
  k += 1;
  nbounce += 1;
  o = s.point;
  d = nd;
  return k < max_depth;  // trace(depth 0) returns (0, 0)
}

// How coherent a k_shade wave's shading is (counting launches only; SURVEY
// §7 step 7 asks whether sorting rays by material would pay): per wave with
// work, the distinct material kinds among its lanes (a miss counts as one
// more kind: the background branch) — the branches the wave executes one
// after another — and the distinct material indices (the material records
// it gathers). A material-sorted pool could bring both to ~1.
MRT_DEV void shade_coherence(const DevScene& S, uint32_t mat, LocalCounters& lc) {
  const unsigned long long act = __ballot(mat != kShadeIdle);
  if (act == 0) return;
  const uint32_t kind = mat == kShadeIdle ? 0xFFu : mat == kShadeMiss ? 16u : S.materials[MRT_IDX(S, mat, S.n_materials, 4)].kind;
  uint32_t nk = 0, nm = 0;
  for (uint32_t kk = 0; kk <= 16; ++kk) nk += __ballot(kind == kk) != 0;
  for (unsigned long long rem = act; rem;) {
    const uint32_t m0 = __shfl(mat, __ffsll((long long)rem) - 1, 64);
    rem &= ~__ballot(mat == m0);
    ++nm;
  }
  if (lane_id() == 0) {
    lc.shade_waves += 1;
    lc.shade_kinds += nk;
    lc.shade_materials += nm;
  }
}

// k_shade only shades and compacts: new camera rays go in behind the
// survivors (k_reserve + k_refill). (Round 3's in-place regeneration of
// finished slots is profiles/r3_experiments/ab_branches.patch.)
// WPE: waves per SIMD the register budget is sized for (8: 64 VGPRs, 32 B of
// scratch; 7: 71 VGPRs, none). With 8, k_shade takes more of the CU beside
// the other queue's k_trace; a world whose records stream from the Infinity
// Cache runs better with 7 (mesh_ply 948.6 -> 969.0, 6: 962.9 Msamples/s),
// an L2-resident one with 8 (sphere_grid 808.8, 7: 778.1, 6: 761.0;
// profiles/r3_tune2/wpe.txt).
template <bool COUNT, bool EXT, int WPE>
__global__ __launch_bounds__(kShadeBlock, WPE) void k_shade(DevScene S, RenderParams rp, PathBufs in, PathBufs out,
                                                  const uint4* hits, Ctrl* ctrl, uint32_t cur, float4* results,
                                                  DevCounters* cnt) {
  const uint32_t n = ctrl->active[cur];
  if (blockIdx.x == 0 && threadIdx.x < kGroups) ctrl->group_next[threadIdx.x * 32] = 0;  // next k_trace
  // one workgroup per 256 live paths: the host sizes the grid from a bound on
  // the live count (shade_grid), so a drain launch does not dispatch a
  // workgroup per 256 slots of the whole pool. A bound that fell short is
  // reported to the host, never dropped silently. (A grid-stride loop here
  // made the kernel spill 80 B instead of 44 and cost 3.5% of the frame.)
  if (blockIdx.x == 0 && threadIdx.x == 0 && n > gridDim.x * kShadeBlock) ctrl->shade_short = n;
  LocalCounters lc;
  uint32_t nbounce = 0, nsample = 0, nshaded = 0;
  __shared__ uint32_t s_cnt[kShadeBlock / 64], s_base, s_hist[kOutKeys];
  const uint32_t wave = threadIdx.x / 64;
  {
    const uint32_t base = blockIdx.x * kShadeBlock;
    if (base >= n) return;
    const uint32_t i = base + threadIdx.x;
    bool alive = false;
    float4 ro{}, rd{}, thr{}, rad{};
    uint4 rs{};
    uint32_t mat = kShadeIdle;
    if (i < n) {
      nshaded += 1;
      ro = in.ro[i];
      rd = in.rd[i];
      thr = in.thr[i];
      if (holds_l(thr)) rad = in.rad[i];
      rs = in.rng[i];
      const uint4 hv = hits[i];
      Hit h{__uint_as_float(hv.x), hv.y, hv.z};
      V3 o{ro.x, ro.y, ro.z}, d{rd.x, rd.y, rd.z}, T{thr.x, thr.y, thr.z}, L{rad.x, rad.y, rad.z};
      uint32_t g = __float_as_uint(ro.w), k = __float_as_uint(rd.w);
      PathRng rng{(unsigned long long)rs.x | ((unsigned long long)rs.y << 32),
                  (unsigned long long)rs.z | ((unsigned long long)rs.w << 32)};
      const bool cont = shade_step<EXT>(S, rp.max_depth, h, o, d, T, L, k, rng, lc, nbounce, mat);
      if (cont) {
        alive = true;
        ro = make_float4(o.x, o.y, o.z, __uint_as_float(g));
        rd = make_float4(d.x, d.y, d.z, __uint_as_float(k));
        thr = make_float4(T.x, T.y, T.z, __uint_as_float(nonzero_bits(L.x, L.y, L.z) ? kHoldsL : 0u));
        rad = make_float4(L.x, L.y, L.z, 0.0f);
        rs = make_uint4((uint32_t)rng.s0, (uint32_t)(rng.s0 >> 32), (uint32_t)rng.s1, (uint32_t)(rng.s1 >> 32));
      } else {
#ifndef MRT_PROBE_NO_RESULTS  // probe build (tools/shade_probe.sh): k_shade's HBM writes without the scattered results stores
        results[MRT_IDX(S, g, rp.G, 21)] = make_float4(L.x, L.y, L.z, __uint_as_float(k));
#endif
        nsample += 1;
      }
    }
    if (COUNT) shade_coherence(S, mat, lc);
    // compact the survivors into the next pool: one atomic per workgroup
    // (same-address atomics from every wave serialise in L2)
    uint32_t slot;
    if (rp.shade_bin) {  // survivors grouped by the material kind they scattered from (wg_reserve_keyed)
      // key: the material kind scattered from and the signs of the new ray's y and x
      const uint32_t kind = alive ? (S.materials[MRT_IDX(S, mat, S.n_materials, 4)].kind & 7u) : 0u;
      if (rp.shade_bin == 2) {  // y sign: the two ends of the pool; kind and x, z signs within
        const uint32_t key = (rd.y < 0.0f ? 32u : 0u) + kind * 4u + (rd.x < 0.0f ? 2u : 0u) + (rd.z < 0.0f ? 1u : 0u);
        slot = wg_reserve_keyed(&ctrl->active[cur ^ 1], alive, key, s_hist, &ctrl->surv[cur ^ 1], rp.pool_cap);
      } else {
        const uint32_t key = kind * 4u + (rd.y < 0.0f ? 2u : 0u) + (rd.x < 0.0f ? 1u : 0u);
        slot = wg_reserve_keyed(&ctrl->active[cur ^ 1], alive, key, s_hist);
      }
    } else {
      const unsigned long long alive_mask = __ballot(alive);
      slot = wg_reserve<kShadeBlock / 64>(&ctrl->active[cur ^ 1], (uint32_t)__popcll(alive_mask), wave, s_cnt, s_base) +
             lane_rank(alive_mask);
    }
    if (alive) {
      uint32_t pos = MRT_IDX(S, slot, rp.pool_cap, 22);
      out.ro[pos] = ro;
      out.rd[pos] = rd;
      out.thr[pos] = thr;
      if (holds_l(thr)) out.rad[pos] = rad;
      out.rng[pos] = rs;
    }
  }
  if (COUNT) flush_counters(cnt, lc, 0, 0, nsample, nbounce, nshaded);
}

// The whole path loop in one persistent kernel: every lane owns a path
// (work item g = pixel*spp + sample, gen_work), steps its closest-hit traversal like
// k_trace, and when a segment ends shades it in place (shade_step) and
// continues with the scattered ray — no pool buffers, no per-bounce launch
// and no per-launch tail. Finished paths write results[g] (accumulated in
// sample order by k_accumulate, so the image is independent of scheduling);
// idle lanes take new work items from ctrl->next_work. slot_ro/slot_rd hold
// each lane's current world ray (re-read when leaving an instance and when
// shading, instead of keeping it in registers).
//
// ADOPT (the wavefront loop's drain, "finish"): instead of new work items the
// lanes adopt the paths of a wavefront pool (`pool`, ctrl->active[cur] of
// them, handed out by ctrl->next_work) in the state k_shade left them — the
// next ray to trace, T, L, bounces, RNG — and run each to its end. The
// wavefront loop switches to it once its work counter is exhausted and few
// paths remain: every per-bounce k_trace launch lasts at least as long as its
// slowest ray (mesh_ply: ~2 ms), so a pool draining over ~50 bounces pays that
// floor ~50 times, while here a lane moves on to its path's next segment as
// soon as its own segment ends.
template <bool COUNT, bool ALPHA, bool ADOPT>
__global__ __launch_bounds__(kBlock) void k_render(DevScene S, DevCamera cam, RenderParams rp, float4* slot_ro,
                                                   float4* slot_rd, Ctrl* ctrl, float4* results, DevCounters* cnt,
                                                   TraceTune tune, PathBufs pool, uint32_t cur) {
  const uint32_t slot = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t n_src = ADOPT ? ctrl->active[cur] : rp.G;  // uniform
  const TravIn tin{S, reinterpret_cast<const uint4*>(S.slots), S.world_begin, slot_ro, slot_rd, kTmin};
  LocalCounters lc;
  uint32_t seg = 0, nh = 0, nsamples = 0, nbounces = 0;
  Trav t{};
  t.done = true;
  t.ray = slot;
  uint32_t g = kIdle, k = 0;
  V3 T{0, 0, 0}, L{0, 0, 0};
  PathRng rng{0, 0};
  bool drained = false;  // wave-uniform: the work counter passed G
  for (;;) {
    const unsigned long long idle = __ballot(g == kIdle);
    const uint32_t n_idle = (uint32_t)__popcll(idle);
    if (!drained && (n_idle >= tune.refill || n_idle == 64)) {
      uint32_t b = 0;
      if (lane_id() == 0) b = atomicAdd(&ctrl->next_work, n_idle);
      b = __shfl(b, 0, 64);
      drained = b + n_idle >= n_src;
      if (g == kIdle) {
        const uint32_t w = b + lane_rank(idle);
        if (w < n_src) {
          float4 ro, rd;
          uint4 rs;
          if (ADOPT) {  // a wavefront path: {o, g} {d, bounces} T L rng (PathBufs)
            ro = pool.ro[w];
            rd = pool.rd[w];
            const float4 tv = pool.thr[w];
            const float4 lv = holds_l(tv) ? pool.rad[w] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            rs = pool.rng[w];
            g = __float_as_uint(ro.w);
            k = __float_as_uint(rd.w);
            T = V3{tv.x, tv.y, tv.z};
            L = V3{lv.x, lv.y, lv.z};
          } else {
            gen_work(cam, rp, w, ro, rd, rs);
            g = w;
            k = 0;
            T = V3{1.0f, 1.0f, 1.0f};
            L = V3{0.0f, 0.0f, 0.0f};
          }
          rng = PathRng{(unsigned long long)rs.x | ((unsigned long long)rs.y << 32),
                        (unsigned long long)rs.z | ((unsigned long long)rs.w << 32)};
          slot_ro[slot] = ro;
          slot_rd[slot] = rd;
          trav_init(tin, t, slot, INFINITY);
        }
      }
    }
    if (drained && __ballot(g != kIdle) == 0) break;
    // one traversal step (as k_trace)
    const bool busy = g != kIdle && !t.done;
    const bool at_box = busy && trav_at_box(t);
    const unsigned long long box_mask = __ballot(at_box);
    const unsigned long long prim_mask = __ballot(busy && !at_box);
    if (at_box) trav_box<COUNT>(tin, t, lc);
    if ((__popcll(prim_mask) >= tune.prim_batch || box_mask == 0) && busy && !at_box)
      trav_prim<COUNT, ALPHA>(tin, t, lc);
    // shade finished segments once enough lanes wait (or nothing else runs)
    const bool ready = g != kIdle && t.done;
    const unsigned long long ready_mask = __ballot(ready);
    if (ready_mask != 0 && ((uint32_t)__popcll(ready_mask) >= tune.shade_batch || (box_mask | prim_mask) == 0)) {
      if (ready) {
        const Hit h = trav_hit(tin, t);
        seg += 1;
        nh += h.prim != kRefNone;
        const float4 o4 = slot_ro[slot], d4 = slot_rd[slot];
        V3 o{o4.x, o4.y, o4.z}, d{d4.x, d4.y, d4.z};
        uint32_t mat;
        if (shade_step<false>(S, rp.max_depth, h, o, d, T, L, k, rng, lc, nbounces, mat)) {
          slot_ro[slot] = make_float4(o.x, o.y, o.z, 0.0f);
          slot_rd[slot] = make_float4(d.x, d.y, d.z, 0.0f);
          trav_init(tin, t, slot, INFINITY);
        } else {
          results[MRT_IDX(S, g, rp.G, 21)] = make_float4(L.x, L.y, L.z, __uint_as_float(k));
          nsamples += 1;
          g = kIdle;
        }
      }
    }
  }
  if (COUNT) flush_counters(cnt, lc, seg, nh, nsamples, nbounces);
}

// Image::merge in sample order: acc = ((acc + s0) + s1) + ...
// A workgroup sums kAccPix pixels: blocks of kAccS samples of all of them
// are staged through LDS with coalesced loads (a pixel's samples are
// contiguous in the pixel-major slab), then each of the first kAccPix
// threads adds its pixel's samples in sample order — the same sequence of
// float additions as one thread walking its pixel's samples, so the sums are
// bit-identical, at HBM rate instead of one 16-KiB-strided line per lane.
constexpr uint32_t kAccPix = 64, kAccS = 16, kAccPad = kAccS + 1;  // +1 quad per row: no bank-aligned rows
__global__ __launch_bounds__(kBlock) void k_accumulate(const float4* results, uint32_t n_pix, uint32_t n_samples,
                                                       const uint32_t* pixlist, float* accum_rgb,
                                                       uint32_t* accum_bounces) {
  __shared__ float4 tile[kAccPix * kAccPad];
  const uint32_t lp0 = blockIdx.x * kAccPix;
  const uint32_t n_here = n_pix - lp0 < kAccPix ? n_pix - lp0 : kAccPix;
  const uint32_t j = threadIdx.x;  // the pixel this thread sums (j < n_here)
  float r = 0.0f, g = 0.0f, b = 0.0f;
  uint32_t k = 0, p = 0;
  if (j < n_here) {
    p = pixlist[lp0 + j];
    r = accum_rgb[3 * (size_t)p], g = accum_rgb[3 * (size_t)p + 1], b = accum_rgb[3 * (size_t)p + 2];
    k = accum_bounces[p];
  }
  for (uint32_t s0 = 0; s0 < n_samples; s0 += kAccS) {
    const uint32_t sb = n_samples - s0 < kAccS ? n_samples - s0 : kAccS;
    for (uint32_t e = threadIdx.x; e < kAccPix * kAccS; e += kBlock) {
      const uint32_t px = e / kAccS, sx = e % kAccS;
      if (px < n_here && sx < sb) tile[px * kAccPad + sx] = results[(size_t)(lp0 + px) * n_samples + s0 + sx];
    }
    __syncthreads();
    if (j < n_here) {
      for (uint32_t sx = 0; sx < sb; ++sx) {
        const float4 q = tile[j * kAccPad + sx];
        r = r + q.x;
        g = g + q.y;
        b = b + q.z;
        k += __float_as_uint(q.w);
      }
    }
    __syncthreads();
  }
  if (j < n_here) {
    accum_rgb[3 * (size_t)p] = r;
    accum_rgb[3 * (size_t)p + 1] = g;
    accum_rgb[3 * (size_t)p + 2] = b;
    accum_bounces[p] = k;
  }
}

// mrt_trace_rays: arbitrary rays go through the product k_trace. In: rays
// (6 floats each) -> pool slots; out: hit records -> mrt_hit with front_face.
__global__ __launch_bounds__(kBlock) void k_rays_in(const float* rays, uint32_t n, PathBufs out) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const float* r = rays + 6 * (size_t)i;
  out.ro[i] = make_float4(r[0], r[1], r[2], __uint_as_float(i));
  out.rd[i] = make_float4(r[3], r[4], r[5], __uint_as_float(0u));
  const PathRng g = path_rng(0, i, 0xFFFFFFFEu);  // traversal draws of mrt_trace_rays (massrt.h)
  out.rng[i] = make_uint4((uint32_t)g.s0, (uint32_t)(g.s0 >> 32), (uint32_t)g.s1, (uint32_t)(g.s1 >> 32));
}

__global__ __launch_bounds__(kBlock) void k_rays_out(DevScene S, PathBufs in, const uint4* hits, uint32_t n,
                                                     uint4* out) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const float4 o4 = in.ro[i], d4 = in.rd[i];
  const uint4 hv = hits[i];
  Hit h{__uint_as_float(hv.x), hv.y, hv.z};
  uint32_t front = 0;
  if (h.prim != kRefNone)
    front = resolve_hit(S, V3{o4.x, o4.y, o4.z}, V3{d4.x, d4.y, d4.z}, h).front_face ? 1u : 0u;
  out[i] = make_uint4(h.prim, h.container, __float_as_uint(h.prim != kRefNone ? h.t : 0.0f), front);
}

// div_cr (path.h) against the IEEE division on random bit patterns plus
// structured operands (all-ones / power-of-two mantissas, range edges).
__global__ __launch_bounds__(kBlock) void k_selftest_division(unsigned long long n, unsigned long long seed,
                                                              unsigned long long* mismatches) {
  unsigned long long bad = 0;
  const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
  for (unsigned long long i = blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    uint64_t x = seed ^ (i * 0x9E3779B97F4A7C15ull);
    unsigned long long r1 = splitmix64_next(x), r2 = splitmix64_next(x);
    uint32_t ua = (uint32_t)r1, ub = (uint32_t)(r1 >> 32);
    switch (r2 & 7) {
      case 0:  // all-ones divisor mantissa
        ub |= 0x007FFFFFu;
        break;
      case 1:  // power-of-two divisor
        ub &= 0xFF800000u;
        break;
      case 2:  // all-ones dividend mantissa
        ua |= 0x007FFFFFu;
        break;
      case 3:  // scene-like magnitudes: exponents near 1
        ua = (ua & 0x807FFFFFu) | ((120u + ((uint32_t)(r2 >> 8) % 20u)) << 23);
        ub = (ub & 0x807FFFFFu) | ((110u + ((uint32_t)(r2 >> 16) % 30u)) << 23);
        break;
      case 4:  // quotient near 1 ulp ties: a = b * small integer
        ub = (ub & 0x807FFFFFu) | (127u << 23);
        {
          float fa = __uint_as_float(ub) * (float)((r2 >> 8) & 0xFFFF);
          ua = __float_as_uint(fa) ^ (uint32_t)((r2 >> 32) & 3);
        }
        break;
      default:
        break;
    }
    float a = __uint_as_float(ua), b = __uint_as_float(ub);
    float q;
    if ((r2 & 7) >= 5) {
      // the slab test's fast domain (path.h TRay::fast): a = m - o with m, o in
      // {0} U [2^-40, 2^28], |b| in [2^-20, 2^20]; q = qfast(a, b, RN(1/b))
      auto coord = [](uint32_t bits, uint32_t sel) {
        uint32_t e = 87u + (sel % 68u);  // 2^-40 .. 2^27
        float v = __uint_as_float((bits & 0x807FFFFFu) | (e << 23));
        return (sel & 15u) == 0 ? 0.0f : v;
      };
      float m = coord(ua, (uint32_t)(r2 >> 8)), o = coord(ub, (uint32_t)(r2 >> 24));
      if ((r2 >> 40) & 1) o = m;  // zero numerators
      if (((r2 >> 42) & 3) == 0 && m != 0.0f)  // cancellation: o a few ulps from m
        o = __uint_as_float(__float_as_uint(m) + (uint32_t)((r2 >> 44) & 7));
      a = m - o;
      uint32_t eb = 107u + ((uint32_t)(r2 >> 48) % 40u);  // 2^-20 .. 2^19
      b = __uint_as_float((ub & 0x807FFFFFu) | (eb << 23));
      q = qfast(a, b, 1.0f / b);
    } else {
      q = div_cr(a, make_recip(b));
    }
    float ref = a / b;
    uint32_t uq = __float_as_uint(q), ur = __float_as_uint(ref);
    bool same = uq == ur || (q != q && ref != ref) || (q == 0.0f && ref == 0.0f);
    bad += same ? 0 : 1;
  }
  bad = (unsigned long long)wave_sum((uint32_t)bad);
  if (lane_id() == 0 && bad) atomicAdd(mismatches, bad);
}


// ---- display (main.rs:640-722, 760-767) ----------------------------------
// Rust f32::min/max (the non-NaN operand wins) and saturating `as u8`.
__device__ __forceinline__ float rs_min(float a, float b) { return a != a ? b : (b != b ? a : (a < b ? a : b)); }
__device__ __forceinline__ float rs_max(float a, float b) { return a != a ? b : (b != b ? a : (a > b ? a : b)); }
__device__ __forceinline__ uint32_t rs_u8(float v) { return !(v > 0.0f) ? 0u : (v >= 255.0f ? 255u : (uint32_t)v); }

// Default-mode byte of x = sum/passes: the count of thresholds <= x for x in
// [0, 1] (-0.0 counts as 0); NaN or negative x -> NaN.powf -> .min(1.0) = 1.0
// -> 255; -inf.powf = +inf and x > 1 -> 255.
// t: host/display.h's table, t[k] = bits of the smallest x in [0,1] whose byte is >= k
__device__ __forceinline__ uint32_t gamma_byte(const uint32_t* t, float x) {
  if (!(x >= 0.0f) || x > 1.0f) return 255u;
  const uint32_t u = __float_as_uint(x) & 0x7FFFFFFFu;  // -0.0 -> powf gives +0 -> byte 0
  uint32_t lo = 0;  // largest k with t[k] <= u (t[0] = 0 <= u)
#pragma unroll
  for (uint32_t step = 128; step > 0; step >>= 1)
    if (t[lo + step] <= u) lo += step;  // lo + step <= 255
  return lo;
}

__global__ __launch_bounds__(kBlock) void k_max_u32(const uint32_t* v, uint32_t n, uint32_t* out) {
  uint32_t m = 0;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) m = v[i] > m ? v[i] : m;
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = __shfl_xor(m, off, 64);
    m = o > m ? o : m;
  }
  if (lane_id() == 0) atomicMax(out, m);
}

// Tile-slab exchange (mrt_shard_*): slab k = the shard's k-th pixel.
__global__ __launch_bounds__(kBlock) void k_shard_pack(const uint32_t* pixlist, uint32_t n, const float* rgb,
                                                       const uint32_t* b, uint4* slab) {
  const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  const uint32_t p = pixlist[k];
  slab[k] = make_uint4(__float_as_uint(rgb[3 * (size_t)p]), __float_as_uint(rgb[3 * (size_t)p + 1]),
                       __float_as_uint(rgb[3 * (size_t)p + 2]), b[p]);
}
__global__ __launch_bounds__(kBlock) void k_shard_unpack(const uint32_t* pixlist, uint32_t n, const uint4* slab,
                                                         float* rgb, uint32_t* b) {
  const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  const uint32_t p = pixlist[k];
  const uint4 v = slab[k];
  rgb[3 * (size_t)p] = __uint_as_float(v.x);
  rgb[3 * (size_t)p + 1] = __uint_as_float(v.y);
  rgb[3 * (size_t)p + 2] = __uint_as_float(v.z);
  b[p] = v.w;
}

// Camera::albedo_normal for pixel p (one ray, no jitter). The rays go through
// ray_ro/ray_rd so that the traversal can re-read them (TravIn).
template <bool RNG, bool EXT>
__global__ __launch_bounds__(kBlock) void k_prepass(DevScene S, DevCamera cam, uint32_t W, uint32_t H,
                                                    unsigned long long seed, float4* ray_ro, float4* ray_rd,
                                                    float* albedo, float* normal) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= W * H) return;
  const uint32_t y = p / W, x = p - y * W;
  PathRng rng = path_rng(seed, p, 0xFFFFFFFFu);
  V3 o, d;
  camera_ray_uv(cam, (float)x / (float)(W - 1), (float)y / (float)(H - 1), rng, o, d);
  ray_ro[p] = make_float4(o.x, o.y, o.z, 0.0f);
  ray_rd[p] = make_float4(d.x, d.y, d.z, 0.0f);
  const TravIn tin{S, reinterpret_cast<const uint4*>(S.slots), S.world_begin, ray_ro, ray_rd, kTmin};
  LocalCounters lc;
  const Hit h = closest_hit<false, RNG, EXT>(tin, p, INFINITY, lc, rng);
  V3 a{0.0f, 0.0f, 0.0f}, n{0.0f, 0.0f, 0.0f};
  if (h.prim != kRefNone) {
    Surf s = resolve_hit(S, o, d, h);
    V3 emitted, atten, nd;
    a = scatter<EXT>(S, s, d, rng, emitted, atten, nd, lc) ? atten : emitted;
    n = s.normal;
  } else {
    a = background<EXT>(S, d, lc);
  }
  albedo[3 * (size_t)p] = a.x, albedo[3 * (size_t)p + 1] = a.y, albedo[3 * (size_t)p + 2] = a.z;
  normal[3 * (size_t)p] = n.x, normal[3 * (size_t)p + 1] = n.y, normal[3 * (size_t)p + 2] = n.z;
}

// One thread per pixel; writes the pixel's 3 bytes at the flipped row.
__global__ __launch_bounds__(kBlock) void k_tonemap(uint32_t W, uint32_t H, const float* rgb, const uint32_t* b,
                                                    uint32_t passes, uint32_t mode, const uint32_t* max_count,
                                                    const uint32_t* g, uint8_t* out) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= W * H) return;
  const uint32_t y = p / W, x = p - y * W;
  uint8_t* dst = out + ((size_t)(H - 1 - y) * W + x) * 3;
  if (mode == MRT_DISPLAY_ALBEDO || mode == MRT_DISPLAY_NORMAL) {  // main.rs:689-718
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = rgb[3 * (size_t)p + c];
      if (mode == MRT_DISPLAY_NORMAL) {
        dst[c] = (uint8_t)rs_u8(((v + 1.0f) / 2.0f) * 255.0f);
      } else {  // p.min(1).max(0).powf(1/2.2): NaN -> 1 -> 255, <= 0 -> 0
        const float q = rs_max(rs_min(v, 1.0f), 0.0f);
        dst[c] = (uint8_t)(q >= 1.0f ? 255u : gamma_byte(g, q));
      }
    }
    return;
  }
  if (passes == 0) {
    dst[0] = dst[1] = dst[2] = 0;
    return;
  }
  const float scale = 1.0f / (float)passes;
  if (mode == MRT_DISPLAY_DEPTH) {
    const uint32_t m = *max_count;
    const float max_depth = (float)(m > 1u ? m : 1u) * scale;
    const float d = rs_min(rs_max(((float)b[p] * scale) / max_depth, 0.0f), 1.0f);
    dst[0] = dst[1] = dst[2] = (uint8_t)rs_u8(d * 255.0f);
  } else {
    dst[0] = (uint8_t)gamma_byte(g, scale * rgb[3 * (size_t)p]);
    dst[1] = (uint8_t)gamma_byte(g, scale * rgb[3 * (size_t)p + 1]);
    dst[2] = (uint8_t)gamma_byte(g, scale * rgb[3 * (size_t)p + 2]);
  }
}

// box_hit_any (early decision + exact fallback) against box_hit_exact on
// rays in the fast domain and boxes whose faces pass within a few ulps of a
// point of the ray (entry/exit ties), flat boxes, and t_max near the faces.
__global__ __launch_bounds__(kBlock) void k_selftest_slab(unsigned long long n, unsigned long long seed,
                                                          unsigned long long* out) {
  unsigned long long bad = 0, ties = 0;
  const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
  for (unsigned long long i = blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    uint64_t x = seed ^ (i * 0xD1B54A32D192ED03ull);
    auto rnd = [&]() { return splitmix64_next(x); };
    auto coord = [&](uint64_t r) {  // {0} U [2^-40, 2^27], random sign
      uint32_t e = 87u + (uint32_t)((r >> 32) % 68u);
      float v = __uint_as_float(((uint32_t)r & 0x807FFFFFu) | (e << 23));
      return ((r >> 60) & 15u) == 0 ? 0.0f : v;
    };
    auto dir = [&](uint64_t r) {  // |d| in [2^-20, 2^19]
      uint32_t e = 107u + (uint32_t)((r >> 32) % 40u);
      return __uint_as_float(((uint32_t)r & 0x807FFFFFu) | (e << 23));
    };
    auto nudge = [](float v, int k) { return __uint_as_float(__float_as_uint(v) + k); };
    V3 o{coord(rnd()), coord(rnd()), coord(rnd())};
    const uint64_t sc = rnd();
    if (sc & 1) {  // scene-like magnitudes
      o = V3{(float)((int)(sc >> 8 & 255) - 128) * 0.37f, (float)((int)(sc >> 16 & 255) - 128) * 0.11f,
             (float)((int)(sc >> 24 & 255) - 128) * 0.23f};
    }
    V3 d{dir(rnd()), dir(rnd()), dir(rnd())};
    const float t = __uint_as_float((uint32_t)(((uint64_t)100u + (rnd() % 37u)) << 23) | ((uint32_t)rnd() & 0x7FFFFFu));
    const V3 p = o + d * t;
    float mn[3], mx[3];
    const float pv[3] = {p.x, p.y, p.z};
    for (int k = 0; k < 3; ++k) {
      const uint64_t r = rnd();
      const int a = (int)(r & 7), b = (int)((r >> 3) & 7);
      const float lo = (r >> 6 & 3) == 0 ? pv[k] - fabsf(pv[k]) * 0.25f - 0.5f : nudge(pv[k], -a);
      const float hi = (r >> 8 & 3) == 0 ? pv[k] + fabsf(pv[k]) * 0.25f + 0.5f : nudge(pv[k], b);
      mn[k] = fminf(lo, hi);
      mx[k] = fmaxf(lo, hi);
      if ((r >> 10 & 7) == 0) mx[k] = mn[k];  // flat box
    }
    // every 8th case: some box minima replaced by a tiny nonzero coordinate
    // (~1e-16, a mesh vertex at sin(pi)): outside the qfast domain, inside the
    // early decision's; the exact test then divides
    if ((sc >> 40 & 7) == 0)
      for (int k = 0; k < 3; ++k)
        if (rnd() & 1) mn[k] = fminf(mx[k], __uint_as_float((__float_as_uint(mn[k]) & 0x80000000u) | 0x25100000u));
    bool ok = true, early = true;
    for (int k = 0; k < 3; ++k) ok = ok && coord_ok(mn[k]) && coord_ok(mx[k]);
    for (int k = 0; k < 3; ++k) early = early && orig_ok(mn[k]) && orig_ok(mx[k]);
    if (!early) continue;
    const TRay ray = make_tray(o, d, ok ? 3u : 2u);
    if (!tray_fast(ray)) continue;
    const uint64_t rt = rnd();
    const float tmin = (rt & 3) == 0 ? nudge(t, -(int)(rt >> 2 & 3)) : 0.001f;
    const float tmax = (rt >> 4 & 3) == 0 ? INFINITY : ((rt >> 4 & 3) == 1 ? nudge(t, (int)(rt >> 6 & 7) - 3) : t * 2.0f);
    const V3 bmn{mn[0], mn[1], mn[2]}, bmx{mx[0], mx[1], mx[2]};
    const bool e = box_hit_exact(bmn, bmx, ray, tmin, tmax);
    const bool f = box_hit_any(bmn, bmx, ray, tmin, tmax);
    bad += e != f;
    // count how often the exact fallback had to decide
    float t0, t1;
    slab_fast(bmn, bmx, ray, tmin, tmax, t0, t1);
    const float m = slab_margin(ray, t0, t1);
    ties += !(t1 - t0 > m) && !(t0 - t1 > m);
  }
  bad = (unsigned long long)wave_sum((uint32_t)bad);
  ties = (unsigned long long)wave_sum((uint32_t)ties);
  if (lane_id() == 0 && (bad || ties)) {
    atomicAdd(out, bad);
    atomicAdd(out + 1, ties);
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// One independent path pool driven on its own stream. Several queues share
// the work counter and run concurrently, so one queue's k_trace tail (the
// last long rays on few lanes) overlaps the other queues' kernels instead of
// idling the GPU.
constexpr int kMaxQueues = 4;

// Context options (mrt_set_option / mrt_get_option, massrt.h): the tuning
// knobs of the loop, set by the caller per context — never read from the
// process environment. -1 (where allowed) = the per-scene rule chosen at
// upload (apply_options). Measurements behind each default: DESIGN.md §4.
enum OptId {
  OPT_QUEUES,            // path pools on their own streams (2: one's tail overlaps the other's kernels)
  OPT_POOL_PATHS,        // live paths at most over all queues (384M: 66 GiB)
  OPT_RESULTS_LOG2,      // samples per results slab at most, log2 (31: a 1080p x 1024-spp frame in one chunk)
  OPT_FINISH_PATHS,      // drain hand-off threshold (fused adopt-mode launch); 0 = never
  OPT_FINISH_GRID_DIV,   // the hand-off launch takes 1/div of its occupancy grid
  OPT_TRACE_REFILL,      // k_trace: refill a wave once this many lanes are idle (-1: 32)
  OPT_TRACE_BOX_MIN,     // k_trace: box run while this many lanes are at a box (-1: 16 instanced / 32 big / 24)
  OPT_TRACE_CHUNK,       // k_trace: rays per work grab (-1: 128 big or instanced / 512)
  OPT_TRACE_PRIM_BATCH,  // k_trace: primitive step once this many lanes wait at one
  OPT_TRACE_WGS_PER_CU,  // persistent grids: workgroups per CU (0: occupancy, 3/4 of it beside other queues)
  OPT_SHADE_WAVES,       // k_shade register budget, waves per SIMD: 7 or 8 (-1: 7 for big non-instanced worlds)
  OPT_SHADE_BATCH,       // k_render: shade once this many lanes finished a segment
  OPT_TREELET_KB,        // LDS treelet per workgroup, KiB (0: none); applies at the next upload
  OPT_TRACE_BLOCK,       // k_trace workgroup size beside a treelet: 256, 512 or 1024
  OPT_MEM_RESERVE_MB,    // device memory a render leaves free when it sizes the pool and results slab
  OPT_TRAVERSAL,         // 0: the reference's left-first walk; 1: the verified near-first walk; -1: per scene (MRT_TRAVERSAL_*)
  OPT_TRACE_NF_BATCH,    // near-first walk: lanes whose walks are over wait for this many to check their hits together (-1: = refill)
  OPT_NF_KAPPA_LOG2,     // near-first walk: rays whose generic-triangle kappa exceeds 2^v take the reference walk (-8: every ray the bound covers)
  OPT_SHADE_BIN,         // k_shade: group each workgroup's survivors by material kind and direction signs (1), and split the pool by y sign (2); -1: per scene
  OPT_TRACE_PRIM_RUN,    // k_trace: primitive run while this many lanes are at a primitive (65: off; -1: 32 near-first / off)
  kNumOpts
};
struct OptDef {
  const char* name;
  int64_t def, lo, hi;
};
constexpr OptDef kOptDefs[kNumOpts] = {
    {"queues", 2, 1, kMaxQueues},
    {"pool_paths", (int64_t)384 << 20, 1 << 16, 1 << 30},
    {"results_log2", 31, 10, 31},
    {"finish_paths", 500000, 0, 1 << 30},
    {"finish_grid_div", 1, 1, 64},
    {"trace_refill", -1, -1, 64},
    {"trace_box_min", -1, -1, 65},
    {"trace_chunk", -1, -1, 1 << 20},
    {"trace_prim_batch", 1, 1, 64},
    {"trace_wgs_per_cu", 0, 0, 32},
    {"shade_waves", -1, -1, 8},
    {"shade_batch", 16, 1, 64},
    {"treelet_kb", 0, 0, 150},
    {"trace_block", 256, 256, 1024},
    {"mem_reserve_mb", 4096, 0, 1 << 20},
    {"traversal", -1, -1, 1},
    {"trace_nf_batch", -1, -1, 64},
    {"nf_kappa_log2", -8, -40, -8},
    {"shade_bin", -1, -1, 2},
    {"trace_prim_run", -1, -1, 65},
};
int opt_find(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < kNumOpts; ++i)
    if (!strcmp(kOptDefs[i].name, name)) return i;
  return -1;
}
struct Queue {
  hipStream_t stream = nullptr;
  PathBufs bufs[2]{};
  uint4* hits = nullptr;
  size_t cap = 0;
  Ctrl* ctrl = nullptr;        // device
  HostStatus* h_stat = nullptr;  // pinned coherent, 2 slots, written by k_status (lagged status reads)
  HostStatus* d_stat = nullptr;  // the same memory as the device addresses it
  hipEvent_t ev[2]{};
  hipEvent_t join = nullptr;
};

struct mrt_ctx {
  int device = 0;
  MultiDev* multi = nullptr;  // a context over several devices (frames.hip): the rest is unused
  std::atomic<int> images{0};  // live mrt_image objects created on this handle (any thread)
  hipStream_t stream = nullptr;
  std::string err;
  // scene
  void* scene_mem = nullptr;
  size_t scene_bytes = 0;
  DevScene S{};
  bool has_scene = false;
  DevCamera cam{};
  bool has_camera = false;
  // render state
  size_t pool_cap = 0;  // paths over all queues
  void* pool_mem = nullptr;
  Queue q[kMaxQueues];
  int64_t opt[kNumOpts];       // mrt_set_option values (kOptDefs); derived fields below (apply_options)
  bool scene_big = false;      // the record stream is past half the chip's L2 (per-scene rules)
  uint32_t scene_instances = 0;
  int n_queues = 2;            // option "queues"
  uint32_t* work = nullptr;    // shared work counter of the wavefront loop (word 1: tonemap max count)
  uint32_t* gamma_d = nullptr; // display: gamma byte thresholds (256 words)
  hipEvent_t fork = nullptr;
  float4* results = nullptr;  // the results slab (results_cap samples)
  size_t results_cap = 0;
  // acc_done: recorded on the caller's stream after the accumulate that read
  // the results slab (and after any other caller-stream work on the shared
  // buffers, mark_ctx_busy); the next render's queues fork after it.
  // (Round 2's two alternating queue sets, measured 5-12% slower, are in
  // profiles/r3_experiments/ab_branches.patch.)
  hipEvent_t acc_done = nullptr;
  hipEvent_t set_fork = nullptr;
  // kernel-timing marks resolved lazily (mrt_get_kernel_stats): a timed
  // render does not wait for its set's drain
  std::vector<std::array<hipEvent_t, 3>> pend_marks;
  std::vector<std::array<hipEvent_t, 2>> pend_fin;
  DevCounters* d_cnt = nullptr;
  uint32_t* dbg = nullptr;  // MRT_DEBUG_BOUNDS record (4 words)
  uint32_t trace_grid = 1024;  // k_trace_simple workgroups
  std::map<std::pair<const void*, size_t>, uint32_t> grids;  // persistent grid per (kernel, LDS bytes)
  bool scene_alpha = true;  // the scene has alpha-tested triangles
  bool scene_rng = false;   // the traversal draws random numbers (Volume, Mix alpha tests)
  bool scene_ext = false;   // composite surfaces or a CubeMap background (the EXT kernel variants)
  TraceTune tune;
  // k_render: per-lane current world ray; event pair timing one launch
  float4* slot_ro = nullptr;
  float4* slot_rd = nullptr;
  size_t slots_cap = 0;
  hipEvent_t tev[2] = {nullptr, nullptr};
  // Live paths per iteration (MRT_POOL_PATHS overrides). Large on purpose:
  // every k_trace launch ends with a tail of long rays on few lanes, so the
  // more rays a launch carries the smaller that tail's share (measured on
  // SphereGrid 1080p: 2M paths 186, 16M 377, 64M 434 Msamples/s; round 3,
  // 256-spp steps: 64M 674, 128M 716, 256M 762, 384M 777, 544M 770). 384M
  // paths hold 66 GiB of HBM (176 B each); a render allocates
  // min(samples per chunk, pool_paths).
  size_t pool_paths = (size_t)384 << 20;
  int cus = 1;
  bool trace_lds = false;          // the scene has an LDS treelet (set per scene)
  int shade_wpe = 8;               // k_shade register budget: 8 or 7 waves/SIMD (option "shade_waves")
  uint32_t tl_boxes = 0;           // box records in the treelet
  bool scene_nf = false;           // the scene has verified near-first trees (nf_tree.cpp)
  std::string nf_note;             // why it has none
  bool use_nf = false;             // k_trace walks them (option "traversal", the scene, no treelet)
  int shade_bin = 0;                        // k_shade groups its survivors by material kind and direction (option "shade_bin")
  // LDS treelet: off by default. Measured: it removes the
  // global load of a step only when every lane of the wave is in the copy,
  // and the TA cost is per wave instruction, not per lane — 256/16 KB and
  // 1024/78 KB were 1% and 1-4% slower than no treelet.
  int trace_block = 256;           // k_trace workgroup size with a treelet (option "trace_block")
  uint32_t treelet_kb = 0;         // treelet budget per workgroup (option "treelet_kb"; 0 = none)
  // a queue whose work is exhausted hands its last <= finish_paths paths to
  // one fused k_render launch (adopt mode) instead of per-bounce launches
  // (MRT_FINISH_PATHS; 0 = never). 500k measured best (profiles/r2_experiments/
  // finish_sweep.txt): mesh_ply 545 -> 678, sphere_grid 638 -> 642 Msamples/s
  uint32_t finish_paths = 500000;
  uint32_t refill_grid = 2048;  // k_refill workgroups (grid-stride; cus * 8)
  uint64_t results_max = kResultsMaxLimit;  // samples per results slab (option "results_log2")
  uint32_t finish_grid_div = 1;  // the finish launch takes 1/div of its occupancy grid (option "finish_grid_div")
  uint32_t wgs_per_cu = 0;       // option "trace_wgs_per_cu" (0: occupancy)
  size_t mem_reserve = (size_t)4096 << 20;  // option "mem_reserve_mb"

  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, std::pair<uint32_t*, uint32_t>> pixlists;
  // host-buffer render staging
  float* d_acc_rgb = nullptr;
  uint32_t* d_acc_b = nullptr;
  size_t acc_cap = 0;
  // kernel timing
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  mrt_kernel_stats kstats{};
  // device ray buffer for mrt_trace_rays
  float* d_rays = nullptr;
  uint4* d_rhits = nullptr;
  size_t rays_cap = 0;
};

static thread_local std::string g_last_error;

static int massrt_ctx_device_of(const mrt_ctx* c) { return c->device; }

mrt_ctx* ctx_wrap_multi(MultiDev* m) {
  mrt_ctx* c = new mrt_ctx();
  c->multi = m;
  c->device = massrt_ctx_device_of(multi_dev(m, 0));
  return c;
}
MultiDev* ctx_multi(const mrt_ctx* c) { return c ? c->multi : nullptr; }
void ctx_images(mrt_ctx* c, int delta) {
  if (c) c->images += delta;
}
void ctx_set_error(mrt_ctx* c, const std::string& msg) {
  if (c)
    c->err = msg;
  else
    g_last_error = msg;
}

namespace {
// A multi-device handle (mrt_create_multi): entry points that act on one
// device run on device 0; scene and camera go to every device.
template <typename F>
int on_dev0(mrt_ctx* c, F&& f) {
  mrt_ctx* d = multi_dev(c->multi, 0);
  const int rc = f(d);
  c->err = d->err;
  return rc;
}
template <typename F>
int on_each(mrt_ctx* c, F&& f) {
  for (int i = 0; i < multi_count(c->multi); ++i) {
    mrt_ctx* d = multi_dev(c->multi, i);
    const int rc = f(d);
    if (rc != MRT_OK) {
      c->err = d->err;
      return rc;
    }
  }
  c->err.clear();
  return MRT_OK;
}
}  // namespace
#define MRT_DEV0(c, call) \
  if ((c) && (c)->multi) return on_dev0((c), [&](mrt_ctx* c) { return call; })
#define MRT_EACH(c, call) \
  if ((c) && (c)->multi) return on_each((c), [&](mrt_ctx* c) { return call; })

namespace {

void set_device(mrt_ctx* c) { HIP_CHECK(hipSetDevice(c->device)); }

// Derived fields from the options; options left at -1 take the per-scene
// rules (scene_big / scene_instances, set at upload):
//  * box run / refill (profiles/r2_tune, r3_tune.txt): refill 32
//    except 12 for a big instanced world (Menger 50.0 -> 53.0 at 64 spp per
//    step, 57.4 -> 58.8 at 256 with 16; mesh_ply keeps 32: 1148.7 vs 1125.9
//    at 24; profiles/r5_nf_probe/summary.txt); box run while >= 16 lanes are at a box for an
//    instance-heavy world (cube_field 266 -> 275, Menger 37.3 -> 44.1
//    Msamples/s), >= 32 for another stream past half the chip's L2 (its
//    record round trips go to the Infinity Cache; mesh_ply 749 -> 775), else
//    >= 24 (sphere_grid);
//  * rays per grab (profiles/r3_tune2/): an L2-resident world without many
//    instances runs longer stretches of neighbouring rays per wave
//    (sphere_grid 762.8 / 775.0 / 780.3 / 780.6 at 128 / 256 / 512 / 1024),
//    while big or instanced worlds keep 128 (mesh_ply 897.4 -> 841.4 at 1024:
//    its waves end on longer tails);
//  * k_shade at 7 waves/SIMD for a big non-instanced world (mesh_ply 948.6
//    -> 969.0), else 8 (sphere_grid 808.8, 7: 778.1; profiles/r3_tune2/wpe.txt).
//  The near-first walk (round 4, profiles/r4_nf/tune.txt) has rules of its
//  own: refill 40 except for a big non-instanced world (sphere_grid 1106.9
//  -> 1137.4, cube_field 608.6 -> 614.6; mesh_ply 1581.6 -> 1528.7 keeps 32)
//  (round 6: a big solid world grabs 256, mesh_ply 1274 -> 1290; profiles/r6_knobs/)
//  and box run >= 20 lanes without many instances (round 6, profiles/r6_knobs/:
//  mesh_ply 1213 -> 1252 from 28, sphere_grid 1155 -> 1164 from 24), 512 rays per grab except there (cube_field
//  556.2 -> 580.2 with shade 7; mesh_ply keeps 128: 1386.7 vs 1372.7), and
//  k_shade at 7 waves/SIMD everywhere (sphere_grid 983.3 -> 992.9).
void apply_options(mrt_ctx* c) {
  const int64_t* o = c->opt;
  const bool inst = c->scene_instances > 1000, big = c->scene_big;
  c->treelet_kb = (uint32_t)o[OPT_TREELET_KB];
  // traversal -1 (per scene): the near-first walk unless the world is a big
  // instanced one (Menger 25.7 / 45.9 at trace_nf_batch 64 vs 50.0;
  // profiles/r5_walk_ab/). Round 5 also declined a margin with the generic-
  // triangle term (mesh_ply 548 vs 1148: |det| >= 1e-6 priced for every
  // ray); the normal cones and the wild instances' own tests turned that
  // around (mesh_ply 1228 vs 1152, profiles/r6_wild/)
  const bool nf_rule = !(inst && big);
  c->use_nf = (o[OPT_TRAVERSAL] == MRT_TRAVERSAL_NEAR_FIRST || (o[OPT_TRAVERSAL] < 0 && nf_rule)) && c->scene_nf &&
              !c->trace_lds && !c->scene_rng;
  const bool nf = c->use_nf, big_solid = big && !inst;
  c->n_queues = (int)o[OPT_QUEUES];
  c->pool_paths = (size_t)o[OPT_POOL_PATHS];
  c->results_max = 1ull << o[OPT_RESULTS_LOG2];
  c->finish_paths = (uint32_t)o[OPT_FINISH_PATHS];
  c->finish_grid_div = (uint32_t)o[OPT_FINISH_GRID_DIV];
  c->tune.refill = o[OPT_TRACE_REFILL] >= 0 ? (uint32_t)std::max<int64_t>(1, o[OPT_TRACE_REFILL])
                                            : ((nf && !big_solid) ? 40u : (inst && big) ? 12u : 32u);
  c->tune.box_min = o[OPT_TRACE_BOX_MIN] >= 0 ? (uint32_t)std::max<int64_t>(1, o[OPT_TRACE_BOX_MIN])
                                              : (inst ? 16u : (nf ? 20u : (big ? 32u : 24u)));
  c->tune.chunk = o[OPT_TRACE_CHUNK] >= 0 ? (uint32_t)o[OPT_TRACE_CHUNK]
                                          : (nf ? (big_solid ? 256u : 512u) : ((big || inst) ? 128u : 512u));
  c->tune.prim_batch = (uint32_t)o[OPT_TRACE_PRIM_BATCH];
  // primitive run (round 6, profiles/r6_primrun/): near-first walk 32
  // (mesh_ply 1365 -> 1392, sphere_grid 1206 -> 1229, cube_field 592 -> 605);
  // the reference walk's kernel has no primitive run (k_trace)
  c->tune.prim_run = o[OPT_TRACE_PRIM_RUN] > 0 ? (uint32_t)o[OPT_TRACE_PRIM_RUN] : (nf ? 32u : 65u);
  c->tune.nf_batch = o[OPT_TRACE_NF_BATCH] > 0 ? (uint32_t)o[OPT_TRACE_NF_BATCH] : c->tune.refill;
  c->tune.shade_batch = (uint32_t)o[OPT_SHADE_BATCH];
  c->shade_wpe = o[OPT_SHADE_WAVES] >= 0 ? (int)o[OPT_SHADE_WAVES] : ((nf || big_solid) ? 7 : 8);
  c->trace_block = (int)o[OPT_TRACE_BLOCK];
  c->mem_reserve = (size_t)o[OPT_MEM_RESERVE_MB] << 20;
  if (c->wgs_per_cu != (uint32_t)o[OPT_TRACE_WGS_PER_CU]) c->grids.clear();
  c->wgs_per_cu = (uint32_t)o[OPT_TRACE_WGS_PER_CU];
  c->S.nfb.kmax = ldexpf(1.0f, (int)o[OPT_NF_KAPPA_LOG2]);
  // survivors grouped by material kind and direction signs (round 5,
  // profiles/r5_shade_bin/): sphere_grid 974 -> 1035, cube_field 504 -> 535
  // Msamples/s (k_trace lane utilisation 0.731 -> 0.774: a wave walks rays
  // that go the same way); mesh_ply, C5, Menger within noise. The pool-wide
  // y-sign split (2) on top, its two counts in one 64-bit atomic per
  // workgroup: sphere_grid 1035 -> 1086, cube_field 538 -> 558 (utilisation
  // 0.774 -> 0.798), mesh_ply 1150 -> 1152, C5 1137 -> 1132
  // (profiles/r5_surv64/; with two 32-bit atomics mesh_ply lost 1151 -> 1134,
  // profiles/r5_shade_block/) — 2 where the near-first walk runs, else 1
  c->shade_bin = o[OPT_SHADE_BIN] >= 0 ? (int)o[OPT_SHADE_BIN] : (nf ? 2 : 1);
}

// Validates and stores option `id`; the caller re-derives (apply_options).
void set_option(mrt_ctx* c, int id, int64_t v) {
  const OptDef& d = kOptDefs[id];
  if (v < d.lo || v > d.hi)
    throw ApiError{MRT_ERR_INVALID, std::string("option ") + d.name + " out of range [" + std::to_string(d.lo) + ", " +
                                        std::to_string(d.hi) + "]"};
  if (id == OPT_TRACE_BLOCK && v != 256 && v != 512 && v != 1024)
    throw ApiError{MRT_ERR_INVALID, "option trace_block must be 256, 512 or 1024"};
  if (id == OPT_SHADE_WAVES && v != -1 && v != 7 && v != 8)
    throw ApiError{MRT_ERR_INVALID, "option shade_waves must be 7, 8 or -1 (per scene)"};
  if (id == OPT_TRACE_NF_BATCH && v == 0) throw ApiError{MRT_ERR_INVALID, "option trace_nf_batch must be 1..64 or -1"};
  if (id == OPT_TRACE_PRIM_RUN && v == 0) throw ApiError{MRT_ERR_INVALID, "option trace_prim_run must be 1..65 or -1"};
  if (id == OPT_TRACE_CHUNK && v != -1 && v < 64) throw ApiError{MRT_ERR_INVALID, "option trace_chunk must be >= 64 or -1"};
  if (id == OPT_QUEUES && v != c->opt[id] && c->pool_mem) {  // the pool is split per queue: reallocated at the next render
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipFree(c->pool_mem));
    c->pool_mem = nullptr;
    c->pool_cap = 0;
    c->grids.clear();  // k_trace's grid share depends on the queue count
  }
  c->opt[id] = v;
}

template <typename F>
int guarded(mrt_ctx* c, F&& f) {
  if (!c) {
    g_last_error = "null context";
    return MRT_ERR_INVALID;
  }
  try {
    set_device(c);
    f();
    c->err.clear();
    return MRT_OK;
  } catch (const ApiError& e) {
    c->err = e.msg;
    return e.code;
  } catch (const HipError& e) {
    c->err = e.msg;
    return MRT_ERR_HIP;
  } catch (const std::bad_alloc&) {
    c->err = "out of host memory";
    return MRT_ERR_NOMEM;
  } catch (const std::exception& e) {
    c->err = e.what();
    return MRT_ERR_INVALID;
  }
}

template <typename T>
size_t align_up(size_t x) {
  return (x + 255) & ~(size_t)255;
}

// The persistent closest-hit kernel over pool buffer `in`, specialised on
// the scene (record stream in LDS when it fits; alpha test compiled in only
// when the scene has alpha-textured triangles).
// `st` waits for the wavefront queues' last render (their buffers are reused).
void wait_queues(mrt_ctx* c, hipStream_t st) {
  for (Queue& q : c->q)
    if (q.join) HIP_CHECK(hipStreamWaitEvent(st, q.join, 0));
}

// Occupancy-sized persistent grid for kernel f with `smem` dynamic LDS.
// `shared`: the kernel runs beside the other queues' kernels (k_trace with
// several queues) — it takes 3/4 of the occupancy, so another queue's trace
// and shade launches find room on every CU instead of queueing behind a
// grid that holds the whole GPU until its last ray (sphere_grid, 2 queues:
// 8 WGs/CU 585, 6 WGs/CU 618 Msamples/s).
uint32_t persistent_grid(mrt_ctx* c, const void* f, size_t smem, bool shared = false, int block = kBlock,
                         int share_num = 3, int share_den = 4) {
  auto key = std::make_pair(f, smem);
  auto it = c->grids.find(key);
  if (it != c->grids.end()) return it->second;
  if (smem > 0) HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTraceLdsMaxBytes));
  int per_cu = 0;
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, block, smem));
  if (shared) per_cu = std::max(1, per_cu * share_num / share_den);
  if (c->wgs_per_cu) per_cu = (int)c->wgs_per_cu;
  const uint32_t g = (uint32_t)c->cus * (uint32_t)std::max(1, per_cu);
  c->grids[key] = g;
  return g;
}

template <bool LDS, uint32_t ALPHA, bool RNG, int BLK>
void launch_trace_b(mrt_ctx* c, hipStream_t st, const Queue& q, const PathBufs& in, uint32_t cur, bool count,
                    float tmin, float tmax) {
  // no treelet: 4 x 16 B per lane for the world-ray stash (TravIn::stash)
  const size_t smem = LDS ? (size_t)c->S.n_tlet * 16 : (size_t)kStashQuads * BLK * 16;
  const void* f = count ? (const void*)k_trace<true, LDS, ALPHA, RNG, BLK> : (const void*)k_trace<false, LDS, ALPHA, RNG, BLK>;
  const uint32_t grid = persistent_grid(c, f, smem, c->n_queues > 1, BLK);
  if (count)
    hipLaunchKernelGGL((k_trace<true, LDS, ALPHA, RNG, BLK>), dim3(grid), dim3(BLK), smem, st, c->S, in, q.hits,
                       q.ctrl, cur, c->d_cnt, tmin, tmax, c->tune);
  else
    hipLaunchKernelGGL((k_trace<false, LDS, ALPHA, RNG, BLK>), dim3(grid), dim3(BLK), smem, st, c->S, in, q.hits,
                       q.ctrl, cur, c->d_cnt, tmin, tmax, c->tune);
}

template <bool LDS, uint32_t ALPHA, bool RNG>
void launch_trace_r(mrt_ctx* c, hipStream_t st, const Queue& q, const PathBufs& in, uint32_t cur, bool count,
                    float tmin, float tmax) {
  if (!LDS)
    launch_trace_b<false, ALPHA, RNG, kBlock>(c, st, q, in, cur, count, tmin, tmax);
  else if (c->trace_block == 1024)
    launch_trace_b<true, ALPHA, RNG, 1024>(c, st, q, in, cur, count, tmin, tmax);
  else if (c->trace_block == 512)
    launch_trace_b<true, ALPHA, RNG, 512>(c, st, q, in, cur, count, tmin, tmax);
  else
    launch_trace_b<true, ALPHA, RNG, kBlock>(c, st, q, in, cur, count, tmin, tmax);
}

template <bool LDS, uint32_t ALPHA>
void launch_trace_v(mrt_ctx* c, hipStream_t st, const Queue& q, const PathBufs& in, uint32_t cur, bool count,
                    float tmin, float tmax) {
  if (c->scene_rng)
    launch_trace_r<LDS, ALPHA, true>(c, st, q, in, cur, count, tmin, tmax);
  else
    launch_trace_r<LDS, ALPHA, false>(c, st, q, in, cur, count, tmin, tmax);
}

// The verified near-first walk (option "traversal" 1; scenes with NF trees,
// no treelet, no traversal draws): its stack takes kNfStack words of LDS per lane.
template <uint32_t ALPHA>
void launch_trace_nf(mrt_ctx* c, hipStream_t st, const Queue& q, const PathBufs& in, uint32_t cur, bool count,
                     float tmin, float tmax) {
  const size_t smem = (size_t)kNfStack * kBlock * 4;
  const void* f = count ? (const void*)k_trace<true, false, ALPHA, false, kBlock, true>
                        : (const void*)k_trace<false, false, ALPHA, false, kBlock, true>;
  // kNfStack KiB of LDS per workgroup allow 6 waves per SIMD, its registers
  // (<= 128 VGPRs: the rounding margins' state and code, round 5, would
  // spill at 80) at least 4. Beside another queue the walk takes 3 WG/CU: its
  // vector-memory unit is the shared limit, so more of its waves buy nothing
  // while k_shade beside it gains (profiles/r4_nf/tune.txt §6: 4 -> 3 WG/CU
  // +0.8%, 2 WG/CU -14%)
  const uint32_t grid = persistent_grid(c, f, smem, c->n_queues > 1, kBlock, 1, 1);
  const uint32_t nf_cap = 3u * (uint32_t)c->cus;
  if (c->n_queues > 1 && !c->wgs_per_cu && grid > nf_cap) c->grids[std::make_pair(f, smem)] = nf_cap;
  const uint32_t g = c->grids[std::make_pair(f, smem)];
  if (count)
    hipLaunchKernelGGL((k_trace<true, false, ALPHA, false, kBlock, true>), dim3(g), dim3(kBlock), smem, st, c->S, in,
                       q.hits, q.ctrl, cur, c->d_cnt, tmin, tmax, c->tune);
  else
    hipLaunchKernelGGL((k_trace<false, false, ALPHA, false, kBlock, true>), dim3(g), dim3(kBlock), smem, st, c->S, in,
                       q.hits, q.ctrl, cur, c->d_cnt, tmin, tmax, c->tune);
}

void launch_trace(mrt_ctx* c, hipStream_t st, const Queue& q, const PathBufs& in, uint32_t cur, bool count,
                  float tmin, float tmax) {
  // alpha tests: none / plain surfaces / composite surfaces (EXT)
  const uint32_t alpha = c->scene_alpha ? (c->scene_ext ? 2u : 1u) : 0u;
  if (c->use_nf) {
    if (alpha == 2)
      launch_trace_nf<2>(c, st, q, in, cur, count, tmin, tmax);
    else if (alpha == 1)
      launch_trace_nf<1>(c, st, q, in, cur, count, tmin, tmax);
    else
      launch_trace_nf<0>(c, st, q, in, cur, count, tmin, tmax);
  } else if (c->trace_lds) {
    if (alpha == 2)
      launch_trace_v<true, 2>(c, st, q, in, cur, count, tmin, tmax);
    else if (alpha == 1)
      launch_trace_v<true, 1>(c, st, q, in, cur, count, tmin, tmax);
    else
      launch_trace_v<true, 0>(c, st, q, in, cur, count, tmin, tmax);
  } else {
    if (alpha == 2)
      launch_trace_v<false, 2>(c, st, q, in, cur, count, tmin, tmax);
    else if (alpha == 1)
      launch_trace_v<false, 1>(c, st, q, in, cur, count, tmin, tmax);
    else
      launch_trace_v<false, 0>(c, st, q, in, cur, count, tmin, tmax);
  }
  HIP_CHECK(hipGetLastError());
}

// k_shade's grid for a pool known to hold at most `bound` live paths: one
// workgroup per 256 of them.
// While the work counter has items left the pool refills to capacity; once
// it is exhausted the live count only falls, so the last status the host
// read bounds every later launch — a drain launch then dispatches a few
// workgroups instead of one per 256 slots of the whole pool.
uint32_t shade_grid(const Queue& q, size_t bound) {
  const size_t n = std::min(q.cap, bound);
  return (uint32_t)std::max<size_t>(1, (n + kShadeBlock - 1) / kShadeBlock);
}

// device bytes of a pool of P paths over the context's queues: two state
// sets (5 x 16 B each) + the hit record per path, 256-B aligned sections
constexpr size_t kPathBytes = 16 * (2 * 5 + 1);
size_t pool_bytes(const mrt_ctx* c, size_t P) {
  const size_t K = (size_t)c->n_queues, per_q = (P + K - 1) / K;
  return (kPathBytes * per_q + 4096) * K;
}

// P paths over the context's queues.
void ensure_pool(mrt_ctx* c, size_t P) {
  if (P <= c->pool_cap) return;
  HIP_CHECK(hipDeviceSynchronize());  // the queues may still be draining into the old pool
  if (c->pool_mem) HIP_CHECK(hipFree(c->pool_mem));
  c->pool_mem = nullptr;
  c->pool_cap = 0;
  const int K = c->n_queues;
  const size_t per_q = (P + K - 1) / K;
  HIP_CHECK(hipMalloc(&c->pool_mem, pool_bytes(c, P)));
  char* p = (char*)c->pool_mem;
  auto take = [&](size_t bytes) {
    char* r = p;
    p += (bytes + 255) & ~(size_t)255;
    return r;
  };
  for (int k = 0; k < K; ++k) {
    Queue& q = c->q[k];
    for (int b = 0; b < 2; ++b) {
      q.bufs[b].ro = (float4*)take(16 * per_q);
      q.bufs[b].rd = (float4*)take(16 * per_q);
      q.bufs[b].thr = (float4*)take(16 * per_q);
      q.bufs[b].rad = (float4*)take(16 * per_q);
      q.bufs[b].rng = (uint4*)take(16 * per_q);
    }
    q.hits = (uint4*)take(16 * per_q);
    q.cap = per_q;
  }
  c->pool_cap = per_q * K;
}

// n samples in the results slab.
void ensure_results(mrt_ctx* c, size_t n) {
  if (n <= c->results_cap) return;
  HIP_CHECK(hipDeviceSynchronize());  // the queues may still write or accumulate the old slab
  if (c->results) HIP_CHECK(hipFree(c->results));
  c->results = nullptr;
  c->results_cap = 0;
  HIP_CHECK(hipMalloc(&c->results, 16 * n));
  c->results_cap = n;
}

// Sizes a render's path pool and results slab to the device:
// they must fit the memory free now minus mem_reserve, since several
// contexts may share one device (a multi-device context over {0,0,0}, ranks
// rehearsed on one GPU) and the defaults alone ask for ~98 GiB. When either
// buffer has to grow both are released and planned afresh: the pool shrinks
// first (its size barely matters from 128M paths on), down to
// kPoolFloor paths, then the samples per results chunk (more chunks, the
// same image: chunks accumulate in sample order). The planning of the
// contexts of a process is serialised, so each sees the others' buffers.
constexpr size_t kPoolFloor = (size_t)64 << 20;
std::mutex g_alloc_mutex;
void plan_buffers(mrt_ctx* c, uint32_t n_pix, uint32_t& spp_chunk, bool need_pool) {
  std::lock_guard<std::mutex> lock(g_alloc_mutex);
  size_t P = need_pool ? std::min<size_t>((size_t)n_pix * spp_chunk, c->pool_paths) : 0;
  if (P <= c->pool_cap && (size_t)n_pix * spp_chunk <= c->results_cap) return;
  HIP_CHECK(hipDeviceSynchronize());  // the queues may still use the old buffers
  if (c->pool_mem) HIP_CHECK(hipFree(c->pool_mem));
  c->pool_mem = nullptr;
  c->pool_cap = 0;
  if (c->results) HIP_CHECK(hipFree(c->results));
  c->results = nullptr;
  c->results_cap = 0;
  size_t free_b = 0, total_b = 0;
  HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
  const size_t budget = free_b > c->mem_reserve ? free_b - c->mem_reserve : 0;
  for (;;) {
    const size_t need = (P ? pool_bytes(c, P) : 0) + (size_t)n_pix * spp_chunk * 16;
    if (need <= budget) break;
    if (P > kPoolFloor) {
      P = std::max(kPoolFloor, P / 2);
    } else if (spp_chunk > 1) {
      spp_chunk = spp_chunk / 2;
      if (P) P = std::min<size_t>(P, (size_t)n_pix * spp_chunk);
    } else {
      throw ApiError{MRT_ERR_NOMEM, "device memory: " + std::to_string(free_b >> 20) + " MiB free, mem_reserve_mb " +
                                        std::to_string(c->mem_reserve >> 20) + ": not even one sample per pixel fits"};
    }
  }
  if (P) ensure_pool(c, P);
  ensure_results(c, (size_t)n_pix * spp_chunk);
}

void ensure_slots(mrt_ctx* c, size_t n) {
  if (n <= c->slots_cap) return;
  if (c->slot_ro) HIP_CHECK(hipDeviceSynchronize());  // a queue set's drain may still use them
  if (c->slot_ro) HIP_CHECK(hipFree(c->slot_ro));
  c->slot_ro = nullptr;
  c->slot_rd = nullptr;
  HIP_CHECK(hipMalloc(&c->slot_ro, 32 * n));
  c->slot_rd = c->slot_ro + n;
  c->slots_cap = n;
}

// MRT_TILE x MRT_TILE tiles in raster order; shard si of sc owns t % sc == si;
// pixels of a tile in raster order, y = 0 the bottom row (main.rs:253-263)
std::vector<uint32_t> shard_pixel_list(uint32_t W, uint32_t H, uint32_t si, uint32_t sc) {
  uint32_t tx = (W + MRT_TILE - 1) / MRT_TILE, ty = (H + MRT_TILE - 1) / MRT_TILE;
  std::vector<uint32_t> list;
  for (uint32_t t = si; t < tx * ty; t += sc) {
    uint32_t bx = (t % tx) * MRT_TILE, by = (t / tx) * MRT_TILE;
    for (uint32_t py = 0; py < MRT_TILE; ++py)
      for (uint32_t px = 0; px < MRT_TILE; ++px) {
        uint32_t x = bx + px, y = by + py;
        if (x < W && y < H) list.push_back(y * W + x);
      }
  }
  return list;
}

std::pair<uint32_t*, uint32_t> pixlist(mrt_ctx* c, uint32_t W, uint32_t H, uint32_t si, uint32_t sc) {
  auto key = std::make_tuple(W, H, si, sc);
  auto it = c->pixlists.find(key);
  if (it != c->pixlists.end()) return it->second;
  const std::vector<uint32_t> list = shard_pixel_list(W, H, si, sc);
  uint32_t* d = nullptr;
  if (!list.empty()) {
    HIP_CHECK(hipMalloc(&d, list.size() * 4));
    HIP_CHECK(hipMemcpy(d, list.data(), list.size() * 4, hipMemcpyHostToDevice));
  }
  auto v = std::make_pair(d, (uint32_t)list.size());
  c->pixlists[key] = v;
  return v;
}


template <bool ALPHA>
void launch_render_v(mrt_ctx* c, hipStream_t st, const RenderParams& rp, bool count) {
  const void* f = count ? (const void*)k_render<true, ALPHA, false> : (const void*)k_render<false, ALPHA, false>;
  const uint32_t grid = persistent_grid(c, f, 0);
  ensure_slots(c, (size_t)grid * kBlock);
  const PathBufs none{};
  if (count)
    hipLaunchKernelGGL((k_render<true, ALPHA, false>), dim3(grid), dim3(kBlock), 0, st, c->S, c->cam, rp, c->slot_ro,
                       c->slot_rd, c->q[0].ctrl, c->results, c->d_cnt, c->tune, none, 0u);
  else
    hipLaunchKernelGGL((k_render<false, ALPHA, false>), dim3(grid), dim3(kBlock), 0, st, c->S, c->cam, rp, c->slot_ro,
                       c->slot_rd, c->q[0].ctrl, c->results, c->d_cnt, c->tune, none, 0u);
  HIP_CHECK(hipGetLastError());
}

// Finish queue qi's pool bufs[cur] (ctrl->active[cur] paths) with the fused
// kernel in adopt mode; each queue uses its own range of lane-ray slots.
template <bool ALPHA>
void launch_finish_v(mrt_ctx* c, int qi, uint32_t cur, const RenderParams& rp, bool count, float4* res) {
  Queue& q = c->q[qi];
  const void* f = count ? (const void*)k_render<true, ALPHA, true> : (const void*)k_render<false, ALPHA, true>;
  const uint32_t full = persistent_grid(c, f, 0, c->n_queues > 1);
  const size_t lanes = (size_t)full * kBlock;
  const uint32_t grid = std::max<uint32_t>(c->cus, full / c->finish_grid_div);
  ensure_slots(c, lanes * kMaxQueues);
  float4* sro = c->slot_ro + lanes * qi;
  float4* srd = c->slot_rd + lanes * qi;
  HIP_CHECK(hipMemsetAsync(&q.ctrl->next_work, 0, 4, q.stream));
  if (count)
    hipLaunchKernelGGL((k_render<true, ALPHA, true>), dim3(grid), dim3(kBlock), 0, q.stream, c->S, c->cam, rp, sro, srd,
                       q.ctrl, res, c->d_cnt, c->tune, q.bufs[cur], cur);
  else
    hipLaunchKernelGGL((k_render<false, ALPHA, true>), dim3(grid), dim3(kBlock), 0, q.stream, c->S, c->cam, rp, sro,
                       srd, q.ctrl, res, c->d_cnt, c->tune, q.bufs[cur], cur);
  HIP_CHECK(hipGetLastError());
}

// Work enqueued on a caller's stream `st` that writes the context's shared
// buffers (q[0].ctrl, the results slab, the lane-ray slots): the next
// wavefront render forks its queues after acc_done, so recording it here
// orders that render after this work too.
void mark_ctx_busy(mrt_ctx* c, hipStream_t st) { HIP_CHECK(hipEventRecord(c->acc_done, st)); }

// The fused path loop: one k_render launch + one k_accumulate per chunk.
void render_fused(mrt_ctx* c, const mrt_render_args* a, const uint32_t* pixlist_d, uint32_t n_pix, uint32_t spp_chunk,
                  float* d_rgb, uint32_t* d_b, hipStream_t st) {
  const bool count = (a->flags & MRT_RENDER_COUNTERS) != 0;
  const bool timing = (a->flags & MRT_RENDER_TIME_KERNELS) != 0;
  plan_buffers(c, n_pix, spp_chunk, false);
  wait_queues(c, st);
  for (uint32_t done = 0; done < a->spp_count; done += spp_chunk) {
    const uint32_t cs = std::min(spp_chunk, a->spp_count - done);
    if (a->max_depth == 0) continue;  // trace(ray, 0) returns (0, 0): nothing to add
    RenderParams rp;
    rp.W = a->width;
    rp.H = a->height;
    rp.seed = a->seed;
    rp.max_depth = a->max_depth;
    rp.n_pix = n_pix;
    rp.G = n_pix * cs;
    rp.spp = cs;
    rp.sample_base = a->spp_begin + done;
    rp.pixlist = pixlist_d;
    rp.pool_cap = 0;
    Ctrl init{{0, 0}, 0, 0};
    HIP_CHECK(hipMemcpyAsync(c->q[0].ctrl, &init, sizeof(Ctrl), hipMemcpyHostToDevice, st));
    if (timing) HIP_CHECK(hipEventRecord(c->tev[0], st));
    if (c->scene_alpha)
      launch_render_v<true>(c, st, rp, count);
    else
      launch_render_v<false>(c, st, rp, count);
    if (timing) {
      HIP_CHECK(hipEventRecord(c->tev[1], st));
      HIP_CHECK(hipEventSynchronize(c->tev[1]));
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, c->tev[0], c->tev[1]));
      c->kstats.trace_ms += ms;
      c->kstats.trace_launches++;
      c->kstats.iterations++;
    }
    hipLaunchKernelGGL(k_accumulate, dim3((n_pix + kAccPix - 1) / kAccPix), dim3(kBlock), 0, st, (const float4*)c->results,
                       n_pix, cs, pixlist_d, d_rgb, d_b);
    HIP_CHECK(hipGetLastError());
  }
  mark_ctx_busy(c, st);
}

void resolve_kernel_timing(mrt_ctx* c);
// pending kernel-timing marks resolved at the start of a timed render once
// this many accumulated (a caller that never reads the stats)
constexpr size_t kMaxPendingMarks = 1u << 14;

void render_device(mrt_ctx* c, const mrt_render_args* a, float* d_rgb, uint32_t* d_b, hipStream_t st) {
  if (!a) throw ApiError{MRT_ERR_INVALID, "null render args"};
  if (!c->has_scene) throw ApiError{MRT_ERR_STATE, "no scene uploaded"};
  if (!c->has_camera) throw ApiError{MRT_ERR_STATE, "no camera set"};
  if (a->width == 0 || a->height == 0) throw ApiError{MRT_ERR_INVALID, "empty image"};
  if ((uint64_t)a->width * a->height >= (1ull << 32)) throw ApiError{MRT_ERR_INVALID, "image too large"};
  uint32_t sc = a->shard_count ? a->shard_count : 1;
  if (a->shard_index >= sc) throw ApiError{MRT_ERR_INVALID, "shard_index >= shard_count"};
  if (a->spp_count == 0) return;
  if ((uint64_t)a->spp_begin + a->spp_count > 0xFFFFFFFFull) throw ApiError{MRT_ERR_INVALID, "sample index overflow"};
  auto pl = pixlist(c, a->width, a->height, a->shard_index, sc);
  const uint32_t n_pix = pl.second;
  if (n_pix == 0) return;
  const bool count = (a->flags & MRT_RENDER_COUNTERS) != 0;
  // results slab <= c->results_max samples (16 B each); pool <= c->pool_paths
  uint32_t spp_chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(a->spp_count, c->results_max / n_pix));
  if ((a->flags & MRT_RENDER_SIMPLE_TRACE) && c->scene_ext)
    throw ApiError{MRT_ERR_INVALID, "MRT_RENDER_SIMPLE_TRACE does not support composite surfaces or CubeMap backgrounds"};
  if ((a->flags & MRT_RENDER_FUSED) && !(a->flags & MRT_RENDER_SIMPLE_TRACE)) {
    if (c->scene_rng)
      throw ApiError{MRT_ERR_INVALID, "MRT_RENDER_FUSED does not support scenes whose traversal draws (Volume, Mix alpha)"};
    if (c->scene_ext)
      throw ApiError{MRT_ERR_INVALID, "MRT_RENDER_FUSED does not support composite surfaces or CubeMap backgrounds"};
    render_fused(c, a, pl.first, n_pix, spp_chunk, d_rgb, d_b, st);
    return;
  }
  plan_buffers(c, n_pix, spp_chunk, true);
  const int K = c->n_queues;
  const bool timing = (a->flags & MRT_RENDER_TIME_KERNELS) != 0;
  if (timing && c->pend_marks.size() + c->pend_fin.size() > kMaxPendingMarks) resolve_kernel_timing(c);
  // the drain hand-off (launch_finish_v): the fused kernel has no traversal
  // draws or composite surfaces; its lane-ray slots are allocated here, before
  // any queue runs (ensure_slots reallocates)
  const bool can_finish = !c->scene_rng && !c->scene_ext && !(a->flags & MRT_RENDER_SIMPLE_TRACE);
  const uint32_t finish_paths = can_finish ? c->finish_paths : 0u;
  if (finish_paths) {
    const void* f = c->scene_alpha ? (count ? (const void*)k_render<true, true, true> : (const void*)k_render<false, true, true>)
                                   : (count ? (const void*)k_render<true, false, true> : (const void*)k_render<false, false, true>);
    ensure_slots(c, (size_t)persistent_grid(c, f, 0, K > 1) * kBlock * kMaxQueues);
  }
  auto next_event = [&]() {
    if (c->ev_used == c->ev_pool.size()) {
      hipEvent_t e;
      HIP_CHECK(hipEventCreate(&e));
      c->ev_pool.push_back(e);
    }
    return c->ev_pool[c->ev_used++];
  };
  for (uint32_t done = 0; done < a->spp_count; done += spp_chunk) {
    uint32_t cs = std::min(spp_chunk, a->spp_count - done);
    RenderParams rp;
    rp.W = a->width;
    rp.H = a->height;
    rp.seed = a->seed;
    rp.max_depth = a->max_depth;
    rp.n_pix = n_pix;
    rp.G = n_pix * cs;
    rp.spp = cs;
    rp.sample_base = a->spp_begin + done;
    rp.pixlist = pl.first;
    rp.pool_cap = (uint32_t)c->q[0].cap;
    rp.shade_bin = (uint32_t)c->shade_bin;
    if (a->max_depth == 0) {
      // trace(ray, 0) returns (0, 0) for every sample: nothing to add
      continue;
    }
    // the queues, their shared work counter and the results slab
    uint32_t* work = c->work;
    float4* res = c->results;
    // fork: the queues start after the accumulate that last read the slab
    // (acc_done, on the caller's stream; the kernels read nothing else the
    // caller's stream writes)
    const uint32_t n0 = (uint32_t)std::min<size_t>(rp.G, c->pool_cap);
    HIP_CHECK(hipStreamWaitEvent(c->q[0].stream, c->acc_done, 0));
    HIP_CHECK(hipMemcpyAsync(work, &n0, 4, hipMemcpyHostToDevice, c->q[0].stream));
    HIP_CHECK(hipEventRecord(c->set_fork, c->q[0].stream));
    uint32_t base = 0;
    for (int k = 0; k < K; ++k) {
      Queue& q = c->q[k];
      const uint32_t nk = (uint32_t)(((uint64_t)n0 * (k + 1)) / K) - base;  // <= q.cap
      if (k) HIP_CHECK(hipStreamWaitEvent(q.stream, c->set_fork, 0));
      Ctrl init{{nk, 0}, 0, 0};
      HIP_CHECK(hipMemcpyAsync(q.ctrl, &init, sizeof(Ctrl), hipMemcpyHostToDevice, q.stream));
      if (nk) {
        hipLaunchKernelGGL(k_generate, dim3((nk + kBlock - 1) / kBlock), dim3(kBlock), 0, q.stream, c->cam, rp,
                           q.bufs[0], base, nk);
        HIP_CHECK(hipGetLastError());
      }
      base += nk;
    }
    std::vector<std::array<hipEvent_t, 3>> marks;
    std::vector<std::array<hipEvent_t, 2>> fin_marks;
    const int kBatch = 4;  // even: a status read sees the live pool in active[0]
    struct Loop {
      uint32_t it = 0;
      int slot = 0;
      bool pending = false, finished = false;
      size_t bound = ~(size_t)0;  // live paths at most (shade_grid)
      bool exhausted = false;     // the work counter was seen at or past G: no refill
    } st_[kMaxQueues];
    int open = K;
    // an internal error in the middle of a chunk: every queue's kernels end
    // before the error returns, so the next render does not fork onto pools
    // and a results slab that this chunk's launches still write
    auto fail_chunk = [&](const std::string& msg) {
      for (int k = 0; k < K; ++k) (void)hipStreamSynchronize(c->q[k].stream);
      throw ApiError{MRT_ERR_HIP, msg};
    };
    auto* shade = c->shade_wpe == 7
                      ? (count ? (c->scene_ext ? k_shade<true, true, 7> : k_shade<true, false, 7>)
                               : (c->scene_ext ? k_shade<false, true, 7> : k_shade<false, false, 7>))
                      : (count ? (c->scene_ext ? k_shade<true, true, 8> : k_shade<true, false, 8>)
                               : (c->scene_ext ? k_shade<false, true, 8> : k_shade<false, false, 8>));
    while (open > 0) {
      for (int k = 0; k < K; ++k) {
        Queue& q = c->q[k];
        Loop& L = st_[k];
        if (L.finished) continue;
        for (int b = 0; b < kBatch; ++b, ++L.it) {
          const uint32_t cur = L.it & 1;
          std::array<hipEvent_t, 3> m{};
          if (timing) {
            m[0] = next_event();
            HIP_CHECK(hipEventRecord(m[0], q.stream));
          }
          if (a->flags & MRT_RENDER_SIMPLE_TRACE)
            if (c->scene_rng)
              hipLaunchKernelGGL(k_trace_simple<true>, dim3(c->trace_grid), dim3(kBlock), 0, q.stream, c->S,
                                 q.bufs[cur], q.hits, q.ctrl, cur, c->d_cnt);
            else
              hipLaunchKernelGGL(k_trace_simple<false>, dim3(c->trace_grid), dim3(kBlock), 0, q.stream, c->S,
                                 q.bufs[cur], q.hits, q.ctrl, cur, c->d_cnt);
          else
            launch_trace(c, q.stream, q, q.bufs[cur], cur, count, kTmin, INFINITY);
          HIP_CHECK(hipGetLastError());
          if (timing) {
            m[1] = next_event();
            HIP_CHECK(hipEventRecord(m[1], q.stream));
          }
          hipLaunchKernelGGL(shade, dim3(shade_grid(q, L.bound)), dim3(kShadeBlock), 0, q.stream, c->S, rp, q.bufs[cur],
                             q.bufs[cur ^ 1], (const uint4*)q.hits, q.ctrl, cur, res, c->d_cnt);
          HIP_CHECK(hipGetLastError());
          if (!L.exhausted || rp.shade_bin == 2) {  // new paths behind the survivors (shade_bin 2: and the pool's ends joined)
            hipLaunchKernelGGL(k_reserve, dim3(1), dim3(64), 0, q.stream, q.ctrl, cur, work, rp.G, rp.pool_cap);
            hipLaunchKernelGGL(k_refill, dim3(c->refill_grid), dim3(kBlock), 0, q.stream, c->cam, rp, q.bufs[cur ^ 1],
                               (const Ctrl*)q.ctrl);
            HIP_CHECK(hipGetLastError());
          }
          if (timing) {
            m[2] = next_event();
            HIP_CHECK(hipEventRecord(m[2], q.stream));
            marks.push_back(m);
          }
        }
        hipLaunchKernelGGL(k_status, dim3(1), dim3(64), 0, q.stream, (const Ctrl*)q.ctrl, (const uint32_t*)work,
                           q.d_stat + L.slot);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipEventRecord(q.ev[L.slot], q.stream));
        if (L.pending) {  // the previous batch's status (one batch stays in flight)
          HIP_CHECK(hipEventSynchronize(q.ev[L.slot ^ 1]));
          const volatile HostStatus& v = q.h_stat[L.slot ^ 1];  // written by the GPU
          const HostStatus s{v.active0, v.active1, v.shade_short, v.work};
          if (s.shade_short)
            fail_chunk("internal: a k_shade grid was smaller than its live pool (" + std::to_string(s.shade_short) +
                       " paths)");
          if (s.work >= rp.G) {
            L.bound = std::min<size_t>(L.bound, s.active0);
            L.exhausted = true;
          }
          if (s.work >= rp.G && s.active0 <= finish_paths) {
            // no new work: the paths left (at most as many as that status
            // showed) finish in one fused launch after the batch just queued
            if (s.active0 > 0) {
              std::array<hipEvent_t, 2> fm{};
              if (timing) {
                fm[0] = next_event();
                HIP_CHECK(hipEventRecord(fm[0], q.stream));
              }
              if (c->scene_alpha)
                launch_finish_v<true>(c, k, L.it & 1, rp, count, res);
              else
                launch_finish_v<false>(c, k, L.it & 1, rp, count, res);
              if (timing) {
                fm[1] = next_event();
                HIP_CHECK(hipEventRecord(fm[1], q.stream));
                fin_marks.push_back(fm);
              }
            }
            L.finished = true;
            --open;
          }
        }
        L.pending = true;
        L.slot ^= 1;
        if (L.it > 64u * 1024u) fail_chunk("render did not converge");
      }
    }
    // join: `st` continues after every queue (which may still be running its
    // drain: the host does not wait)
    for (int k = 0; k < K; ++k) {
      HIP_CHECK(hipEventRecord(c->q[k].join, c->q[k].stream));
      HIP_CHECK(hipStreamWaitEvent(st, c->q[k].join, 0));
    }
    if (timing) {  // resolved by mrt_get_kernel_stats (resolve_kernel_timing)
      c->pend_marks.insert(c->pend_marks.end(), marks.begin(), marks.end());
      c->pend_fin.insert(c->pend_fin.end(), fin_marks.begin(), fin_marks.end());
    }
    hipLaunchKernelGGL(k_accumulate, dim3((n_pix + kAccPix - 1) / kAccPix), dim3(kBlock), 0, st, (const float4*)res,
                       n_pix, cs, (const uint32_t*)pl.first, d_rgb, d_b);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipEventRecord(c->acc_done, st));  // the slab is free again after this
  }
}

// Kernel timing of renders flagged MRT_RENDER_TIME_KERNELS, resolved when the
// stats are read (a timed render does not wait for its queue set's drain).
void resolve_kernel_timing(mrt_ctx* c) {
  if (c->pend_marks.empty() && c->pend_fin.empty()) return;
  for (auto& m : c->pend_marks) {
    float t0 = 0, t1 = 0;
    HIP_CHECK(hipEventSynchronize(m[2]));
    HIP_CHECK(hipEventElapsedTime(&t0, m[0], m[1]));
    HIP_CHECK(hipEventElapsedTime(&t1, m[1], m[2]));
    c->kstats.trace_ms += t0;
    c->kstats.shade_ms += t1;
    c->kstats.trace_launches++;
    c->kstats.shade_launches++;
    c->kstats.iterations++;
  }
  for (auto& m : c->pend_fin) {
    float t = 0;
    HIP_CHECK(hipEventSynchronize(m[1]));
    HIP_CHECK(hipEventElapsedTime(&t, m[0], m[1]));
    c->kstats.finish_ms += t;
    c->kstats.finish_launches++;
  }
  c->pend_marks.clear();
  c->pend_fin.clear();
  c->ev_used = 0;
}

}  // namespace

extern "C" {

int mrt_abi_version(void) { return MRT_ABI_VERSION; }
const char* mrt_global_last_error(void) { return g_last_error.c_str(); }
const char* mrt_last_error(const mrt_ctx* c) { return c ? c->err.c_str() : g_last_error.c_str(); }

int mrt_create(int device, mrt_ctx** out) {
  if (!out) {
    g_last_error = "null output pointer";
    return MRT_ERR_INVALID;
  }
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    g_last_error = "no HIP device available (the massrt hot path has no CPU fallback)";
    return MRT_ERR_HIP;
  }
  if (device < 0 || device >= n) {
    g_last_error = "device ordinal out of range";
    return MRT_ERR_INVALID;
  }
  mrt_ctx* c = new mrt_ctx();
  c->device = device;
  int rc = guarded(c, [&] {
    HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (int i = 0; i < kNumOpts; ++i) c->opt[i] = kOptDefs[i].def;
    apply_options(c);
    for (int k = 0; k < kMaxQueues; ++k) {
      Queue& q = c->q[k];
      HIP_CHECK(hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking));
      HIP_CHECK(hipMalloc(&q.ctrl, sizeof(Ctrl)));
      HIP_CHECK(hipHostMalloc(&q.h_stat, 2 * sizeof(HostStatus), hipHostMallocCoherent | hipHostMallocMapped));
      memset(q.h_stat, 0, 2 * sizeof(HostStatus));
      HIP_CHECK(hipHostGetDevicePointer((void**)&q.d_stat, q.h_stat, 0));
      HIP_CHECK(hipEventCreateWithFlags(&q.ev[0], hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&q.ev[1], hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&q.join, hipEventDisableTiming));
    }
    HIP_CHECK(hipMalloc(&c->work, 256));
    HIP_CHECK(hipMemset(c->work, 0, 256));
    HIP_CHECK(hipEventCreateWithFlags(&c->fork, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&c->acc_done, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&c->set_fork, hipEventDisableTiming));
    HIP_CHECK(hipMalloc(&c->d_cnt, sizeof(DevCounters)));
    HIP_CHECK(hipMemset(c->d_cnt, 0, sizeof(DevCounters)));
    HIP_CHECK(hipMalloc(&c->dbg, 16));
    HIP_CHECK(hipMemset(c->dbg, 0, 16));
    HIP_CHECK(hipEventCreate(&c->tev[0]));
    HIP_CHECK(hipEventCreate(&c->tev[1]));
    int cus = 0;
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    c->cus = std::max(1, cus);
    c->trace_grid = (uint32_t)c->cus * 4;  // k_trace_simple (debug)
    c->refill_grid = (uint32_t)c->cus * 8;
  });
  if (rc != MRT_OK) {
    g_last_error = c->err;
    mrt_destroy(c);
    return rc;
  }
  *out = c;
  return MRT_OK;
}

}  // extern "C"

int massrt_ctx_device(const mrt_ctx* c) { return c ? c->device : -1; }  // device 0's for a multi-device context

extern "C" {

int mrt_destroy(mrt_ctx* c) {
  if (!c) return MRT_OK;
  if (c->images > 0) {  // an image holds the per-device contexts (massrt.h)
    c->err = "mrt_destroy: " + std::to_string(c->images.load()) + " image(s) of this context still exist";
    g_last_error = c->err;
    return MRT_ERR_STATE;
  }
  if (c->multi) {
    multi_free(c->multi);
    delete c;
    return MRT_OK;
  }
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  for (Queue& q : c->q)
    if (q.stream) hipStreamSynchronize(q.stream);
  hipFree(c->scene_mem);
  hipFree(c->pool_mem);
  hipFree(c->results);
  if (c->acc_done) hipEventDestroy(c->acc_done);
  if (c->set_fork) hipEventDestroy(c->set_fork);
  hipFree(c->work);
  hipFree(c->gamma_d);
  for (Queue& q : c->q) {
    hipFree(q.ctrl);
    if (q.h_stat) hipHostFree(q.h_stat);
    for (hipEvent_t e : {q.ev[0], q.ev[1], q.join})
      if (e) hipEventDestroy(e);
    if (q.stream) hipStreamDestroy(q.stream);
  }
  if (c->fork) hipEventDestroy(c->fork);
  hipFree(c->d_cnt);
  hipFree(c->dbg);
  hipFree(c->d_acc_rgb);
  hipFree(c->d_acc_b);
  hipFree(c->d_rays);
  hipFree(c->d_rhits);
  hipFree(c->slot_ro);
  for (auto& kv : c->pixlists) hipFree(kv.second.first);
  if (c->tev[0]) hipEventDestroy(c->tev[0]);
  if (c->tev[1]) hipEventDestroy(c->tev[1]);
  for (hipEvent_t e : c->ev_pool) hipEventDestroy(e);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
  return MRT_OK;
}

int mrt_upload_scene(mrt_ctx* c, const mrt_scene_desc* d) {
  MRT_EACH(c, mrt_upload_scene(c, d));
  return guarded(c, [&] {
    if (!d) throw ApiError{MRT_ERR_INVALID, "null scene"};
    HostScene hs;
    std::string err;
    // NF trees per the option in effect at upload (upload.h nf_build)
    hs.nf_build = c->opt[OPT_TRAVERSAL] == MRT_TRAVERSAL_REFERENCE ? kNfBuildNever
                  : c->opt[OPT_TRAVERSAL] == MRT_TRAVERSAL_NEAR_FIRST ? kNfBuildAlways : kNfBuildAuto;
    if (!build_host_scene(*d, hs, err)) throw ApiError{MRT_ERR_INVALID, err};
    build_treelet(hs, (uint32_t)((size_t)c->treelet_kb * 1024 / 16));
    // one allocation, 256-B aligned sections
    size_t off = 0;
    auto sec = [&](size_t bytes) {
      size_t o = off;
      off += (bytes + 255) & ~(size_t)255;
      return o;
    };
    size_t o_slots = sec(hs.slots.size() * 4), o_stl = sec(hs.slots_tl.size() * 4), o_tlet = sec(hs.tlet.size() * 4),
           o_inv = sec(hs.inst_inv.size() * 4),
           o_fwd = sec(hs.inst_fwd.size() * 4), o_imat = sec(hs.inst_mat.size() * 4),
           o_mmat = sec(hs.model_mat.size() * 4), o_sph = sec(hs.sph.size() * 4), o_smat = sec(hs.sph_mat.size() * 4),
           o_tri = sec(hs.tri_shade.size() * 4), o_mat = sec(hs.materials.size() * sizeof(GpuMaterial)),
           o_tex = sec(hs.textures.size() * sizeof(GpuTexture)), o_texel = sec(hs.texels.size() * 4),
           o_vnid = sec(hs.vol_nid.size() * 4), o_vmat = sec(hs.vol_mat.size() * 4);
    const std::vector<float>& ln_table = hs.ln_table;
    const size_t o_ln = sec(ln_table.size() * 4);
    const size_t o_sops = sec(hs.surf_ops.size() * sizeof(GpuSurfOp));
    const size_t o_bgf = sec(hs.bg_faces.size() * sizeof(GpuSurfRef));
    const size_t o_bgm = sec(sizeof(hs.bg_m));
    const size_t o_vnf = sec(hs.vnf_leaf.size() * 4);
    if (c->scene_mem) HIP_CHECK(hipFree(c->scene_mem));
    c->scene_mem = nullptr;
    c->has_scene = false;
    HIP_CHECK(hipMalloc(&c->scene_mem, off + 256));
    char* base = (char*)c->scene_mem;
    auto up = [&](size_t o, const void* src, size_t bytes) {
      if (bytes) HIP_CHECK(hipMemcpy(base + o, src, bytes, hipMemcpyHostToDevice));
    };
    up(o_slots, hs.slots.data(), hs.slots.size() * 4);
    up(o_stl, hs.slots_tl.data(), hs.slots_tl.size() * 4);
    up(o_tlet, hs.tlet.data(), hs.tlet.size() * 4);
    up(o_vnid, hs.vol_nid.data(), hs.vol_nid.size() * 4);
    up(o_vmat, hs.vol_mat.data(), hs.vol_mat.size() * 4);
    up(o_ln, ln_table.data(), ln_table.size() * 4);
    up(o_inv, hs.inst_inv.data(), hs.inst_inv.size() * 4);
    up(o_fwd, hs.inst_fwd.data(), hs.inst_fwd.size() * 4);
    up(o_imat, hs.inst_mat.data(), hs.inst_mat.size() * 4);
    up(o_mmat, hs.model_mat.data(), hs.model_mat.size() * 4);
    up(o_sph, hs.sph.data(), hs.sph.size() * 4);
    up(o_smat, hs.sph_mat.data(), hs.sph_mat.size() * 4);
    up(o_tri, hs.tri_shade.data(), hs.tri_shade.size() * 4);
    up(o_mat, hs.materials.data(), hs.materials.size() * sizeof(GpuMaterial));
    up(o_tex, hs.textures.data(), hs.textures.size() * sizeof(GpuTexture));
    up(o_texel, hs.texels.data(), hs.texels.size() * 4);
    up(o_sops, hs.surf_ops.data(), hs.surf_ops.size() * sizeof(GpuSurfOp));
    up(o_bgf, hs.bg_faces.data(), hs.bg_faces.size() * sizeof(GpuSurfRef));
    up(o_bgm, hs.bg_m, sizeof(hs.bg_m));
    up(o_vnf, hs.vnf_leaf.data(), hs.vnf_leaf.size() * 4);
    DevScene S{};
    S.slots = (const uint32_t*)(base + o_slots);
    S.slots_tl = (const uint32_t*)(base + o_stl);
    S.tlet = (const uint32_t*)(base + o_tlet);
    S.n_tlet = (uint32_t)(hs.tlet.size() / 4);
    S.tl_world_begin = hs.tl_world_begin;
    S.world_begin = hs.world_begin;
    S.world_end = hs.world_end;
    S.inst_inv = (const float*)(base + o_inv);
    S.inst_fwd = (const float*)(base + o_fwd);
    S.inst_mat = (const uint32_t*)(base + o_imat);
    S.model_mat = (const uint32_t*)(base + o_mmat);
    S.sph = (const float*)(base + o_sph);
    S.sph_mat = (const uint32_t*)(base + o_smat);
    S.tri_shade = (const float*)(base + o_tri);
    S.materials = (const GpuMaterial*)(base + o_mat);
    S.textures = (const GpuTexture*)(base + o_tex);
    S.texels = (const uint32_t*)(base + o_texel);
    S.fast_ok = (hs.fast_ok ? 1u : 0u) | (hs.early_ok ? 2u : 0u);
    S.vol_nid = (const float*)(base + o_vnid);
    S.vol_mat = (const uint32_t*)(base + o_vmat);
    S.ln_table = ln_table.empty() ? nullptr : (const float*)(base + o_ln);
    S.n_vol = (uint32_t)hs.vol_nid.size();
    S.n_slots = (uint32_t)(hs.slots.size() / 4);
    S.n_tris = (uint32_t)(hs.tri_shade.size() / (kTriShadeQuads * 4));
    S.n_sph = (uint32_t)hs.sph_mat.size();
    S.n_inst = (uint32_t)hs.inst_mat.size();
    S.n_models = (uint32_t)hs.model_mat.size();
    S.n_materials = (uint32_t)hs.materials.size();
    S.n_textures = (uint32_t)hs.textures.size();
    S.n_texels = (uint32_t)hs.texels.size();
    S.dbg = c->dbg;
    S.bg_kind = hs.bg_kind;
    for (int k = 0; k < 4; ++k) S.bg_color[k] = hs.bg_color[k];
    S.surf_ops = (const GpuSurfOp*)(base + o_sops);
    S.n_surf_ops = (uint32_t)hs.surf_ops.size();
    S.bg_faces = (const GpuSurfRef*)(base + o_bgf);
    S.bg_m = (const float*)(base + o_bgm);
    S.nf_ok = hs.nf_ok ? 1u : 0u;
    S.nf_world = hs.nf_world;
    S.vnf_leaf = (const uint32_t*)(base + o_vnf);
    for (int k = 0; k < 4; ++k) S.vnf_base[k] = hs.vnf_base[k];
    S.n_vnf = (uint32_t)(hs.vnf_leaf.size() / 2);
    S.nfb = hs.nfb;
    c->S = S;
    c->scene_bytes = off;
    c->trace_lds = S.n_tlet > 0;
    // the reference stream's size decides the per-scene rules (the NF trees follow it)
    c->scene_big = (size_t)hs.nf_first_slot * 16 > ((size_t)16 << 20);
    c->scene_instances = S.n_inst;
    c->tl_boxes = hs.tl_boxes;
    c->scene_alpha = hs.has_alpha;
    c->scene_rng = hs.trav_rng;
    c->scene_ext = !hs.surf_ops.empty() || hs.bg_kind == MRT_BG_CUBEMAP;
    c->scene_nf = hs.nf_ok;
    c->nf_note = hs.nf_ok ? "" : hs.nf_note;
    apply_options(c);  // the per-scene rules of the options left at -1
    c->has_scene = true;
  });
}

int mrt_set_option(mrt_ctx* c, const char* name, int64_t value) {
  if (c && c->multi && name && !strcmp(name, "gather")) return multi_set_gather(c->multi, value, c->err);
  MRT_EACH(c, mrt_set_option(c, name, value));
  return guarded(c, [&] {
    if (name && !strcmp(name, "gather")) {
      if (value != MRT_GATHER_AUTO && value != MRT_GATHER_PEER)
        throw ApiError{MRT_ERR_INVALID, "option gather: a one-device context has no RCCL transport"};
      return;  // nothing to gather on one device
    }
    const int id = opt_find(name);
    if (id < 0) throw ApiError{MRT_ERR_INVALID, std::string("unknown option ") + (name ? name : "(null)")};
    set_option(c, id, value);
    apply_options(c);
  });
}

int mrt_get_option(mrt_ctx* c, const char* name, int64_t* value) {
  if (c && c->multi && name && value && !strcmp(name, "gather")) {
    *value = multi_gather(c->multi);
    return MRT_OK;
  }
  MRT_DEV0(c, mrt_get_option(c, name, value));
  return guarded(c, [&] {
    if (!value) throw ApiError{MRT_ERR_INVALID, "null output"};
    if (name && !strcmp(name, "gather")) {
      *value = MRT_GATHER_AUTO;
      return;
    }
    const int id = opt_find(name);
    if (id < 0) throw ApiError{MRT_ERR_INVALID, std::string("unknown option ") + (name ? name : "(null)")};
    *value = c->opt[id];
  });
}

int mrt_get_tuning(mrt_ctx* c, mrt_tuning* out) {
  MRT_DEV0(c, mrt_get_tuning(c, out));
  return guarded(c, [&] {
    if (!out) throw ApiError{MRT_ERR_INVALID, "null output"};
    out->queues = (uint32_t)c->n_queues;
    out->trace_refill = c->tune.refill;
    out->trace_box_min = c->tune.box_min;
    out->trace_chunk = c->tune.chunk;
    out->shade_waves = (uint32_t)c->shade_wpe;
    out->pool_paths = c->pool_paths;
    out->results_max = c->results_max;
    out->traversal = c->use_nf ? MRT_TRAVERSAL_NEAR_FIRST : MRT_TRAVERSAL_REFERENCE;
    out->shade_bin = (uint32_t)c->shade_bin;
  });
}

int mrt_scene_device_bytes(mrt_ctx* c, uint64_t* out) {
  MRT_DEV0(c, mrt_scene_device_bytes(c, out));
  return guarded(c, [&] {
    if (!out) throw ApiError{MRT_ERR_INVALID, "null output"};
    *out = c->scene_bytes;
  });
}

int mrt_set_camera(mrt_ctx* c, const mrt_camera* cam) {
  MRT_EACH(c, mrt_set_camera(c, cam));
  return guarded(c, [&] {
    if (!cam) throw ApiError{MRT_ERR_INVALID, "null camera"};
    DevCamera d;
    d.origin = V3{cam->origin[0], cam->origin[1], cam->origin[2]};
    d.llc = V3{cam->lower_left_corner[0], cam->lower_left_corner[1], cam->lower_left_corner[2]};
    d.horizontal = V3{cam->horizontal[0], cam->horizontal[1], cam->horizontal[2]};
    d.vertical = V3{cam->vertical[0], cam->vertical[1], cam->vertical[2]};
    d.u = V3{cam->u[0], cam->u[1], cam->u[2]};
    d.v = V3{cam->v[0], cam->v[1], cam->v[2]};
    d.lens_radius = cam->lens_radius;
    c->cam = d;
    c->has_camera = true;
  });
}

int mrt_render_device(mrt_ctx* c, const mrt_render_args* a, float* d_rgb, uint32_t* d_b, void* stream) {
  MRT_DEV0(c, mrt_render_device(c, a, d_rgb, d_b, stream));
  return guarded(c, [&] {
    if (!d_rgb || !d_b) throw ApiError{MRT_ERR_INVALID, "null accumulation buffer"};
    render_device(c, a, d_rgb, d_b, (hipStream_t)stream);  // NULL: the null stream
  });
}

int mrt_render(mrt_ctx* c, const mrt_render_args* a, float* rgb, uint32_t* bounces) {
  if (c && c->multi) return multi_render(c->multi, a, rgb, bounces, c->err);
  return guarded(c, [&] {
    if (!a || !rgb || !bounces) throw ApiError{MRT_ERR_INVALID, "null argument"};
    size_t np = (size_t)a->width * a->height;
    if (np > c->acc_cap) {
      hipFree(c->d_acc_rgb);
      hipFree(c->d_acc_b);
      c->d_acc_rgb = nullptr;
      c->d_acc_b = nullptr;
      HIP_CHECK(hipMalloc(&c->d_acc_rgb, np * 12));
      HIP_CHECK(hipMalloc(&c->d_acc_b, np * 4));
      c->acc_cap = np;
    }
    HIP_CHECK(hipMemcpyAsync(c->d_acc_rgb, rgb, np * 12, hipMemcpyHostToDevice, c->stream));
    HIP_CHECK(hipMemcpyAsync(c->d_acc_b, bounces, np * 4, hipMemcpyHostToDevice, c->stream));
    render_device(c, a, c->d_acc_rgb, c->d_acc_b, c->stream);
    HIP_CHECK(hipMemcpyAsync(rgb, c->d_acc_rgb, np * 12, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(hipMemcpyAsync(bounces, c->d_acc_b, np * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(hipStreamSynchronize(c->stream));
  });
}

int mrt_trace_rays(mrt_ctx* c, const float* rays, uint32_t n, float t_min, float t_max, mrt_hit* out) {
  MRT_DEV0(c, mrt_trace_rays(c, rays, n, t_min, t_max, out));
  return guarded(c, [&] {
    if (!c->has_scene) throw ApiError{MRT_ERR_STATE, "no scene uploaded"};
    if (n == 0) return;
    if (!rays || !out) throw ApiError{MRT_ERR_INVALID, "null argument"};
    if (n > c->rays_cap) {
      hipFree(c->d_rays);
      hipFree(c->d_rhits);
      c->d_rays = nullptr;
      c->d_rhits = nullptr;
      HIP_CHECK(hipMalloc(&c->d_rays, (size_t)n * 24));
      HIP_CHECK(hipMalloc(&c->d_rhits, (size_t)n * 16));
      c->rays_cap = n;
    }
    HIP_CHECK(hipMemcpyAsync(c->d_rays, rays, (size_t)n * 24, hipMemcpyHostToDevice, c->stream));
    wait_queues(c, c->stream);
    ensure_pool(c, (size_t)n * c->n_queues);  // all rays go to queue 0
    const Queue& q = c->q[0];
    const uint32_t g = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_rays_in, dim3(g), dim3(kBlock), 0, c->stream, (const float*)c->d_rays, n, q.bufs[0]);
    HIP_CHECK(hipGetLastError());
    Ctrl init{{n, 0}, n, 0};
    HIP_CHECK(hipMemcpyAsync(q.ctrl, &init, sizeof(Ctrl), hipMemcpyHostToDevice, c->stream));
    launch_trace(c, c->stream, q, q.bufs[0], 0u, true, t_min, t_max);
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_rays_out, dim3(g), dim3(kBlock), 0, c->stream, c->S, q.bufs[0], (const uint4*)q.hits, n,
                       c->d_rhits);
    HIP_CHECK(hipGetLastError());
    std::vector<uint4> h(n);
    HIP_CHECK(hipMemcpyAsync(h.data(), c->d_rhits, (size_t)n * 16, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(hipStreamSynchronize(c->stream));
    for (uint32_t i = 0; i < n; ++i) {
      out[i].prim = h[i].x;
      out[i].container = h[i].y;
      memcpy(&out[i].t, &h[i].z, 4);
      out[i].front_face = h[i].w;
    }
  });
}

int mrt_get_counters(mrt_ctx* c, mrt_counters* out) {
  if (c && c->multi && out) {  // summed over the devices
    mrt_counters sum{};
    const int rc = on_each(c, [&](mrt_ctx* d) {
      mrt_counters x{};
      const int r = mrt_get_counters(d, &x);
      const uint64_t* px = reinterpret_cast<const uint64_t*>(&x);
      uint64_t* ps = reinterpret_cast<uint64_t*>(&sum);
      for (size_t k = 0; k < sizeof(x) / 8; ++k) ps[k] += px[k];
      return r;
    });
    *out = sum;
    return rc;
  }
  return guarded(c, [&] {
    if (!out) throw ApiError{MRT_ERR_INVALID, "null output"};
    HIP_CHECK(hipStreamSynchronize(c->stream));
    HIP_CHECK(hipDeviceSynchronize());
    DevCounters h;
    HIP_CHECK(hipMemcpy(&h, c->d_cnt, sizeof(h), hipMemcpyDeviceToHost));
    out->samples = h.samples;
    out->segments = h.segments;
    out->node_visits = h.node_visits;
    out->sphere_tests = h.sphere_tests;
    out->triangle_tests = h.triangle_tests;
    out->instance_entries = h.instance_entries;
    out->model_entries = h.model_entries;
    out->closest_hits = h.closest_hits;
    out->texel_taps = h.texel_taps;
    out->bounces = h.bounces;
    out->wave_slots = h.wave_slots;
    out->lane_steps = h.lane_steps;
    out->box_exact = h.box_exact;
    out->shaded = h.shaded;
    out->vnf_fallbacks = h.vnf_fallbacks;
    out->shade_waves = h.shade_waves;
    out->shade_kinds = h.shade_kinds;
    out->shade_materials = h.shade_materials;
  });
}

int mrt_get_kernel_stats(mrt_ctx* c, mrt_kernel_stats* out) {
  if (c && c->multi && out) {  // summed over the devices
    mrt_kernel_stats sum{};
    const int rc = on_each(c, [&](mrt_ctx* d) {
      mrt_kernel_stats x{};
      const int r = mrt_get_kernel_stats(d, &x);
      sum.trace_ms += x.trace_ms, sum.shade_ms += x.shade_ms, sum.other_ms += x.other_ms;
      sum.trace_launches += x.trace_launches, sum.shade_launches += x.shade_launches;
      sum.iterations += x.iterations, sum.finish_ms += x.finish_ms, sum.finish_launches += x.finish_launches;
      return r;
    });
    *out = sum;
    return rc;
  }
  return guarded(c, [&] {
    if (!out) throw ApiError{MRT_ERR_INVALID, "null output"};
    resolve_kernel_timing(c);
    *out = c->kstats;
  });
}

int mrt_reset_kernel_stats(mrt_ctx* c) {
  MRT_EACH(c, mrt_reset_kernel_stats(c));
  return guarded(c, [&] {
    resolve_kernel_timing(c);
    c->kstats = mrt_kernel_stats{};
  });
}

int mrt_selftest_division(mrt_ctx* c, uint64_t n, uint64_t seed, uint64_t* mismatches) {
  MRT_DEV0(c, mrt_selftest_division(c, n, seed, mismatches));
  return guarded(c, [&] {
    if (!mismatches) throw ApiError{MRT_ERR_INVALID, "null output"};
    unsigned long long* d = nullptr;
    HIP_CHECK(hipMalloc(&d, 8));
    HIP_CHECK(hipMemsetAsync(d, 0, 8, c->stream));
    hipLaunchKernelGGL(k_selftest_division, dim3(4096), dim3(kBlock), 0, c->stream, (unsigned long long)n,
                       (unsigned long long)seed, d);
    HIP_CHECK(hipGetLastError());
    unsigned long long h = 0;
    HIP_CHECK(hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(hipStreamSynchronize(c->stream));
    HIP_CHECK(hipFree(d));
    *mismatches = h;
  });
}

int mrt_tonemap_device(mrt_ctx* c, uint32_t W, uint32_t H, const float* d_rgb, const uint32_t* d_b, uint32_t passes,
                       uint32_t mode, uint8_t* d_out, void* stream) {
  MRT_DEV0(c, mrt_tonemap_device(c, W, H, d_rgb, d_b, passes, mode, d_out, stream));
  return guarded(c, [&] {
    if (W == 0 || H == 0 || (uint64_t)W * H >= (1ull << 32)) throw ApiError{MRT_ERR_INVALID, "bad image size"};
    if (mode > MRT_DISPLAY_NORMAL) throw ApiError{MRT_ERR_INVALID, "bad display mode"};
    const bool aux = mode == MRT_DISPLAY_ALBEDO || mode == MRT_DISPLAY_NORMAL;
    if (!d_out || (aux && !d_rgb) ||
        (passes && ((mode == MRT_DISPLAY_DEFAULT && !d_rgb) || (mode == MRT_DISPLAY_DEPTH && !d_b))))
      throw ApiError{MRT_ERR_INVALID, "null buffer"};
    hipStream_t st = (hipStream_t)stream;  // NULL: the null stream (ordered with the caller's default-stream work)
    const uint32_t n = W * H;
    if (!c->gamma_d) {
      HIP_CHECK(hipMalloc(&c->gamma_d, 256 * 4));
      HIP_CHECK(hipMemcpy(c->gamma_d, mrt::gamma_thresholds().data(), 256 * 4, hipMemcpyHostToDevice));
    }
    HIP_CHECK(hipMemsetAsync(c->work + 1, 0, 4, st));  // word 1 of the work line: max count
    if (mode == MRT_DISPLAY_DEPTH && passes) {
      hipLaunchKernelGGL(k_max_u32, dim3(std::min<uint32_t>((n + kBlock - 1) / kBlock, 4096u)), dim3(kBlock), 0, st,
                         d_b, n, c->work + 1);
      HIP_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(k_tonemap, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, W, H, d_rgb, d_b, passes,
                       mode, (const uint32_t*)(c->work + 1), (const uint32_t*)c->gamma_d, d_out);
    HIP_CHECK(hipGetLastError());
  });
}

int mrt_tonemap(mrt_ctx* c, uint32_t W, uint32_t H, const float* rgb, const uint32_t* b, uint32_t passes,
                uint32_t mode, uint8_t* out) {
  MRT_DEV0(c, mrt_tonemap(c, W, H, rgb, b, passes, mode, out));
  return guarded(c, [&] {
    if (W == 0 || H == 0 || (uint64_t)W * H >= (1ull << 32)) throw ApiError{MRT_ERR_INVALID, "bad image size"};
    if (!out || !rgb || !b) throw ApiError{MRT_ERR_INVALID, "null buffer"};
    const size_t n = (size_t)W * H;
    void* mem = nullptr;
    HIP_CHECK(hipMalloc(&mem, n * 12 + n * 4 + n * 3 + 256));
    float* d_rgb = (float*)mem;
    uint32_t* d_b = (uint32_t*)(d_rgb + 3 * n);
    uint8_t* d_out = (uint8_t*)(d_b + n);
    HIP_CHECK(hipMemcpyAsync(d_rgb, rgb, n * 12, hipMemcpyHostToDevice, c->stream));
    HIP_CHECK(hipMemcpyAsync(d_b, b, n * 4, hipMemcpyHostToDevice, c->stream));
    int rc = mrt_tonemap_device(c, W, H, d_rgb, d_b, passes, mode, d_out, c->stream);
    if (rc != MRT_OK) {
      hipFree(mem);
      throw ApiError{rc, c->err};
    }
    HIP_CHECK(hipMemcpyAsync(out, d_out, n * 3, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(hipStreamSynchronize(c->stream));
    HIP_CHECK(hipFree(mem));
  });
}

int mrt_prepass_device(mrt_ctx* c, uint32_t W, uint32_t H, uint64_t seed, float* d_albedo, float* d_normal,
                       void* stream) {
  MRT_DEV0(c, mrt_prepass_device(c, W, H, seed, d_albedo, d_normal, stream));
  return guarded(c, [&] {
    if (!c->has_scene) throw ApiError{MRT_ERR_STATE, "no scene uploaded"};
    if (!c->has_camera) throw ApiError{MRT_ERR_STATE, "no camera set"};
    if (W == 0 || H == 0 || (uint64_t)W * H >= (1ull << 32)) throw ApiError{MRT_ERR_INVALID, "bad image size"};
    if (!d_albedo || !d_normal) throw ApiError{MRT_ERR_INVALID, "null buffer"};
    hipStream_t st = (hipStream_t)stream;  // NULL: the null stream (ordered with the caller's default-stream work)
    wait_queues(c, st);
    const uint32_t n = W * H;
    ensure_slots(c, n);  // the pre-pass rays
    auto* prepass = c->scene_rng ? (c->scene_ext ? k_prepass<true, true> : k_prepass<true, false>)
                                 : (c->scene_ext ? k_prepass<false, true> : k_prepass<false, false>);
    hipLaunchKernelGGL(prepass, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, c->S, c->cam, W, H,
                       (unsigned long long)seed, c->slot_ro, c->slot_rd, d_albedo, d_normal);
    HIP_CHECK(hipGetLastError());
    mark_ctx_busy(c, st);  // the pre-pass rays live in slot_ro/slot_rd, which the drain hand-off reuses
  });
}

int mrt_prepass(mrt_ctx* c, uint32_t W, uint32_t H, uint64_t seed, float* albedo, float* normal) {
  MRT_DEV0(c, mrt_prepass(c, W, H, seed, albedo, normal));
  return guarded(c, [&] {
    if (W == 0 || H == 0 || (uint64_t)W * H >= (1ull << 32)) throw ApiError{MRT_ERR_INVALID, "bad image size"};
    if (!albedo || !normal) throw ApiError{MRT_ERR_INVALID, "null buffer"};
    const size_t n = (size_t)W * H;
    float* d = nullptr;
    HIP_CHECK(hipMalloc(&d, n * 24));
    int rc = mrt_prepass_device(c, W, H, seed, d, d + 3 * n, c->stream);
    if (rc != MRT_OK) {
      hipFree(d);
      throw ApiError{rc, c->err};
    }
    HIP_CHECK(hipMemcpyAsync(albedo, d, n * 12, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(hipMemcpyAsync(normal, d + 3 * n, n * 12, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(hipStreamSynchronize(c->stream));
    HIP_CHECK(hipFree(d));
  });
}

int mrt_selftest_slab(mrt_ctx* c, uint64_t n, uint64_t seed, uint64_t* mismatches, uint64_t* near_ties) {
  MRT_DEV0(c, mrt_selftest_slab(c, n, seed, mismatches, near_ties));
  return guarded(c, [&] {
    if (!mismatches || !near_ties) throw ApiError{MRT_ERR_INVALID, "null output"};
    unsigned long long* d = nullptr;
    HIP_CHECK(hipMalloc(&d, 16));
    HIP_CHECK(hipMemsetAsync(d, 0, 16, c->stream));
    hipLaunchKernelGGL(k_selftest_slab, dim3(4096), dim3(kBlock), 0, c->stream, (unsigned long long)n,
                       (unsigned long long)seed, d);
    HIP_CHECK(hipGetLastError());
    unsigned long long h[2] = {0, 0};
    HIP_CHECK(hipMemcpyAsync(h, d, 16, hipMemcpyDeviceToHost, c->stream));
    HIP_CHECK(hipStreamSynchronize(c->stream));
    HIP_CHECK(hipFree(d));
    *mismatches = h[0];
    *near_ties = h[1];
  });
}

int mrt_debug_status(mrt_ctx* c, uint32_t* out4) {
  MRT_DEV0(c, mrt_debug_status(c, out4));
  return guarded(c, [&] {
    if (!out4) throw ApiError{MRT_ERR_INVALID, "null output"};
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpy(out4, c->dbg, 16, hipMemcpyDeviceToHost));
  });
}

int mrt_debug_build(void) {
#ifdef MRT_DEBUG_BOUNDS
  return 1;
#else
  return 0;
#endif
}

int mrt_shard_pixels(uint32_t W, uint32_t H, uint32_t si, uint32_t sc, uint32_t* pixels, uint32_t* count) {
  try {
    if (!count) throw ApiError{MRT_ERR_INVALID, "null count"};
    if (W == 0 || H == 0 || (uint64_t)W * H >= (1ull << 32)) throw ApiError{MRT_ERR_INVALID, "bad image size"};
    if (sc == 0) sc = 1;
    if (si >= sc) throw ApiError{MRT_ERR_INVALID, "shard_index >= shard_count"};
    const std::vector<uint32_t> list = shard_pixel_list(W, H, si, sc);
    *count = (uint32_t)list.size();
    if (pixels && !list.empty()) memcpy(pixels, list.data(), list.size() * 4);
    return MRT_OK;
  } catch (const ApiError& e) {
    g_last_error = e.msg;
    return e.code;
  } catch (const std::bad_alloc&) {
    g_last_error = "out of host memory";
    return MRT_ERR_NOMEM;
  }
}

static int shard_exchange(mrt_ctx* c, uint32_t W, uint32_t H, uint32_t si, uint32_t sc, const void* src_rgb,
                          const void* src_b, const void* slab, float* dst_rgb, uint32_t* dst_b, void* stream,
                          bool pack) {
  return guarded(c, [&] {
    if (W == 0 || H == 0 || (uint64_t)W * H >= (1ull << 32)) throw ApiError{MRT_ERR_INVALID, "bad image size"};
    if (sc == 0) sc = 1;
    if (si >= sc) throw ApiError{MRT_ERR_INVALID, "shard_index >= shard_count"};
    if (!slab || (pack && (!src_rgb || !src_b)) || (!pack && (!dst_rgb || !dst_b)))
      throw ApiError{MRT_ERR_INVALID, "null buffer"};
    hipStream_t st = (hipStream_t)stream;  // NULL: the null stream (ordered with the caller's default-stream work)
    auto pl = pixlist(c, W, H, si, sc);
    if (pl.second == 0) return;
    const dim3 grid((pl.second + kBlock - 1) / kBlock);
    if (pack)
      hipLaunchKernelGGL(k_shard_pack, grid, dim3(kBlock), 0, st, pl.first, pl.second, (const float*)src_rgb,
                         (const uint32_t*)src_b, (uint4*)slab);
    else
      hipLaunchKernelGGL(k_shard_unpack, grid, dim3(kBlock), 0, st, pl.first, pl.second, (const uint4*)slab, dst_rgb,
                         dst_b);
    HIP_CHECK(hipGetLastError());
  });
}

int mrt_shard_pack_device(mrt_ctx* c, uint32_t W, uint32_t H, uint32_t si, uint32_t sc, const float* d_rgb,
                          const uint32_t* d_b, void* d_slab, void* stream) {
  MRT_DEV0(c, mrt_shard_pack_device(c, W, H, si, sc, d_rgb, d_b, d_slab, stream));
  return shard_exchange(c, W, H, si, sc, d_rgb, d_b, d_slab, nullptr, nullptr, stream, true);
}

int mrt_shard_unpack_device(mrt_ctx* c, uint32_t W, uint32_t H, uint32_t si, uint32_t sc, const void* d_slab,
                            float* d_rgb, uint32_t* d_b, void* stream) {
  MRT_DEV0(c, mrt_shard_unpack_device(c, W, H, si, sc, d_slab, d_rgb, d_b, stream));
  return shard_exchange(c, W, H, si, sc, nullptr, nullptr, d_slab, d_rgb, d_b, stream, false);
}

int mrt_reset_counters(mrt_ctx* c) {
  MRT_EACH(c, mrt_reset_counters(c));
  return guarded(c, [&] {
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemset(c->d_cnt, 0, sizeof(DevCounters)));
  });
}

}  // extern "C"
