// frames.hip — one context over several devices, and the device-resident
// Image (include/massrt.h, ABI v7).
//
// The reference's render() (main.rs:150-295) runs num_cpus-2 worker threads
// that each render whole 1-spp passes and merge them into ONE Image
// (main.rs:629-638). Here the workers are devices: a frame's 8x8 tiles are
// split over the devices of a context (device i renders shard si + i*sc of
// sc*n, one host thread per device, each through the single-device path of
// render.hip), every device keeps the sums of its own tiles in its own HBM,
// and a read gathers the devices' tile slabs onto the first device — RCCL
// send/recv over xGMI between distinct devices, HIP peer copies otherwise —
// where they are unpacked. Every pixel is summed on one device only, in
// sample order, so the image equals the one-device render bit for bit.
//
// This file uses only the public single-device entry points on the
// per-device contexts (mrt_render_device, mrt_shard_pack/unpack_device,
// mrt_prepass_device, mrt_tonemap_device); render.hip routes the entry
// points of a multi-device handle here (frames.h).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "frames.h"

int massrt_ctx_device(const mrt_ctx* ctx);  // render.hip

namespace {

struct Fail {
  int code;
  std::string msg;
};

#define HIPF(x)                                                                                 \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) throw Fail{MRT_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)}; \
  } while (0)
#define MRTF(ctx, x)                                \
  do {                                              \
    int r_ = (x);                                   \
    if (r_ != MRT_OK) throw Fail{r_, mrt_last_error(ctx)}; \
  } while (0)
// RCCL is opened on first use (dlopen), not linked: a process that never
// gathers over RCCL (one device, peer copies, every test on a 1-GPU box)
// does not load it next to the HIP runtime its host (e.g. torch) brings.
struct Rccl {
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

// the library RCCL is opened from (mrt_debug_rccl_library: a test points it
// at a missing file to take the peer-copy fallback on a machine that has RCCL).
// One table per library name, loaded once and never overwritten: a context
// keeps the table it was created with (MultiDev::R), so the test hook never
// changes the function pointers a live context is calling through.
std::string g_rccl_name = "librccl.so.1";
std::map<std::string, std::unique_ptr<Rccl>> g_rccl_tables;
std::mutex g_rccl_mu;
const Rccl& rccl() {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  std::unique_ptr<Rccl>& slot = g_rccl_tables[g_rccl_name];
  if (!slot) {
    slot.reset(new Rccl{});
    Rccl& r = *slot;
    void* h = dlopen(g_rccl_name.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h && g_rccl_name == "librccl.so.1") h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (h) {
      r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
      r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
      r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
      r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
      r.send = (decltype(r.send))dlsym(h, "ncclSend");
      r.recv = (decltype(r.recv))dlsym(h, "ncclRecv");
      r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    }
  }
  const Rccl& r = *slot;
  if (!r.comm_init_all || !r.group_start || !r.group_end || !r.send || !r.recv || !r.error_string)
    throw Fail{MRT_ERR_HIP, "RCCL (" + g_rccl_name + ") is not available"};
  return r;
}

#define NCCLF(x)                                                                                     \
  do {                                                                                               \
    ncclResult_t r_ = (x);                                                                           \
    if (r_ != ncclSuccess) throw Fail{MRT_ERR_HIP, std::string(#x) + ": " + m->R->error_string(r_)}; \
  } while (0)

bool valid_size(uint32_t W, uint32_t H) { return W && H && (uint64_t)W * H < (1ull << 32); }

// One device's part of a frame: the accumulation buffers (full frame size;
// only this device's tiles are written), its tile slab and, on device 0, the
// buffer its slab is received into.
struct DevFrame {
  mrt_ctx* ctx = nullptr;
  int device = 0;
  hipStream_t st = nullptr;
  hipEvent_t ev = nullptr;
  float* rgb = nullptr;
  uint32_t* b = nullptr;
  void* slab = nullptr;
  uint32_t count = 0;  // pixels of this device's shard
  std::vector<uint32_t> pix;  // their indices, in slab order (host; mrt_render's per-shard upload)
  void* recv = nullptr;  // on device 0
  // timing events around this device's renders not yet added to render_ms
  // (mrt_image_device_stats collects them; a render never waits for them)
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  double render_ms = 0;  // this device's render time so far (HIP events)
  // past kMaxPending pairs (a caller that never reads the stats, e.g. the
  // drop-in render() loop) the finished ones are folded into render_ms, so
  // the list stays bounded without making a render wait (the caller's device
  // is current)
  static constexpr size_t kMaxPending = 64;
  void fold_finished() {
    if (pending.size() < kMaxPending) return;
    size_t keep = 0;
    for (size_t k = 0; k < pending.size(); ++k) {
      auto& e = pending[k];
      float ms = 0;
      if (hipEventQuery(e.second) == hipSuccess && hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess) {
        render_ms += ms;
        hipEventDestroy(e.first), hipEventDestroy(e.second);
      } else {
        pending[keep++] = e;
      }
    }
    pending.resize(keep);
  }
};

// A frame over the devices of a context: device i owns shard si + i*sc of sc*n.
struct Frame {
  std::vector<DevFrame> d;
  MultiDev* m = nullptr;  // transport (null: one device)
  uint32_t W = 0, H = 0, si = 0, sc = 1;
  uint64_t gather_bytes = 0;
  double gather_ms = 0;

  uint32_t shard(size_t i) const { return si + (uint32_t)i * sc; }
  uint32_t shards() const { return sc * (uint32_t)d.size(); }
  size_t npix() const { return (size_t)W * H; }

  void setup(MultiDev* mm, const std::vector<mrt_ctx*>& ctxs, uint32_t w, uint32_t h, uint32_t s_i, uint32_t s_c) {
    release();
    m = ctxs.size() > 1 ? mm : nullptr;
    W = w, H = h, si = s_i, sc = s_c ? s_c : 1;
    d.resize(ctxs.size());
    for (size_t i = 0; i < d.size(); ++i) {
      DevFrame& f = d[i];
      f.ctx = ctxs[i];
      f.device = massrt_ctx_device(f.ctx);
      HIPF(hipSetDevice(f.device));
      HIPF(hipStreamCreateWithFlags(&f.st, hipStreamNonBlocking));
      HIPF(hipEventCreateWithFlags(&f.ev, hipEventDisableTiming));
      HIPF(hipMalloc(&f.rgb, npix() * 12));
      HIPF(hipMalloc(&f.b, npix() * 4));
      if (d.size() > 1) {
        MRTF(f.ctx, mrt_shard_pixels(W, H, shard(i), shards(), nullptr, &f.count));
        f.pix.resize(f.count);
        if (f.count) MRTF(f.ctx, mrt_shard_pixels(W, H, shard(i), shards(), f.pix.data(), &f.count));
        HIPF(hipMalloc(&f.slab, (size_t)f.count * 16 + 16));
      }
    }
    HIPF(hipSetDevice(d[0].device));
    for (size_t i = 1; i < d.size(); ++i) HIPF(hipMalloc(&d[i].recv, (size_t)d[i].count * 16 + 16));
    clear();
  }

  void clear() {
    for (DevFrame& f : d) {
      HIPF(hipSetDevice(f.device));
      HIPF(hipMemsetAsync(f.rgb, 0, npix() * 12, f.st));
      HIPF(hipMemsetAsync(f.b, 0, npix() * 4, f.st));
    }
  }

  void release() {
    for (DevFrame& f : d) {
      hipSetDevice(f.device);
      if (f.st) hipStreamSynchronize(f.st);
    }
    for (DevFrame& f : d) {
      hipSetDevice(f.device);
      hipFree(f.rgb), hipFree(f.b), hipFree(f.slab);
      if (f.ev) hipEventDestroy(f.ev);
      for (auto& e : f.pending) hipEventDestroy(e.first), hipEventDestroy(e.second);
      if (f.st) hipStreamDestroy(f.st);
    }
    if (!d.empty()) {
      hipSetDevice(d[0].device);
      for (DevFrame& f : d) hipFree(f.recv);
    }
    d.clear();
  }

  ~Frame() { release(); }

  // every device renders its shard of `a` (a.shard_* ignored), concurrently;
  // events around each device's render time it (collect_times)
  void render(const mrt_render_args& a0) {
    auto one = [&](size_t i, mrt_render_args a) {
      DevFrame& f = d[i];
      HIPF(hipSetDevice(f.device));
      f.fold_finished();
      hipEvent_t e0 = nullptr, e1 = nullptr;
      HIPF(hipEventCreate(&e0));
      HIPF(hipEventCreate(&e1));
      f.pending.push_back({e0, e1});
      HIPF(hipEventRecord(e0, f.st));
      MRTF(f.ctx, mrt_render_device(f.ctx, &a, f.rgb, f.b, f.st));
      HIPF(hipSetDevice(f.device));
      HIPF(hipEventRecord(e1, f.st));
    };
    if (d.size() == 1) {
      mrt_render_args a = a0;
      a.shard_index = si, a.shard_count = sc;
      one(0, a);
      return;
    }
    std::vector<Fail> fails(d.size(), Fail{MRT_OK, ""});
    std::vector<std::thread> th;
    for (size_t i = 0; i < d.size(); ++i)
      th.emplace_back([&, i] {
        mrt_render_args a = a0;
        a.shard_index = shard(i), a.shard_count = shards();
        try {
          one(i, a);
        } catch (const Fail& e) {
          fails[i] = e;
        }
      });
    for (auto& t : th) t.join();
    for (const Fail& f : fails)
      if (f.code != MRT_OK) throw f;
  }

  // the other devices' tiles onto device 0's buffers (pack, send, unpack)
  void gather();

  // adds every finished render's event time to its device's render_ms
  // (waits for renders still running)
  void collect_times() {
    for (DevFrame& f : d) {
      HIPF(hipSetDevice(f.device));
      for (auto& e : f.pending) {
        HIPF(hipEventSynchronize(e.second));
        float ms = 0;
        HIPF(hipEventElapsedTime(&ms, e.first, e.second));
        f.render_ms += ms;
        hipEventDestroy(e.first), hipEventDestroy(e.second);
      }
      f.pending.clear();
    }
  }
};

}  // namespace

// ---------------------------------------------------------------------------
struct MultiDev {
  std::vector<mrt_ctx*> devs;
  std::vector<int> ids;
  bool distinct = false;          // no device repeats (RCCL has one rank per device)
  bool rccl = false;              // the gather uses RCCL (else peer copies)
  int64_t mode = MRT_GATHER_AUTO;
  std::string transport = "peer";
  std::vector<ncclComm_t> comms;  // created with the context (distinct devices)
  const Rccl* R = nullptr;        // the RCCL table the communicators were created with
  Frame* scratch = nullptr;       // mrt_render's frame (host buffers)
};

namespace {

void ensure_comms(MultiDev* m) {
  if (!m->comms.empty()) return;
  m->comms.resize(m->ids.size());
  const Rccl& R = m->R ? *m->R : rccl();
  m->R = &R;
  const ncclResult_t r = R.comm_init_all(m->comms.data(), (int)m->ids.size(), m->ids.data());
  if (r != ncclSuccess) {
    m->comms.clear();
    throw Fail{MRT_ERR_HIP, std::string("ncclCommInitAll: ") + R.error_string(r)};
  }
}

void Frame::gather() {
  if (d.size() < 2) return;
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t i = 1; i < d.size(); ++i)
    if (d[i].count) MRTF(d[i].ctx, mrt_shard_pack_device(d[i].ctx, W, H, shard(i), shards(), d[i].rgb, d[i].b, d[i].slab, d[i].st));
  uint64_t bytes = 0;
  if (m && m->rccl) {
    ensure_comms(m);
    const Rccl& R = *m->R;
    NCCLF(R.group_start());
    for (size_t i = 1; i < d.size(); ++i) {
      if (!d[i].count) continue;
      NCCLF(R.send(d[i].slab, (size_t)d[i].count * 4, ncclUint32, 0, m->comms[i], d[i].st));
      NCCLF(R.recv(d[i].recv, (size_t)d[i].count * 4, ncclUint32, (int)i, m->comms[0], d[0].st));
      bytes += (uint64_t)d[i].count * 16;
    }
    NCCLF(R.group_end());
  } else {
    for (size_t i = 1; i < d.size(); ++i) {
      if (!d[i].count) continue;
      HIPF(hipSetDevice(d[i].device));
      HIPF(hipEventRecord(d[i].ev, d[i].st));
      HIPF(hipSetDevice(d[0].device));
      HIPF(hipStreamWaitEvent(d[0].st, d[i].ev, 0));
      HIPF(hipMemcpyPeerAsync(d[i].recv, d[0].device, d[i].slab, d[i].device, (size_t)d[i].count * 16, d[0].st));
      bytes += (uint64_t)d[i].count * 16;
    }
  }
  for (size_t i = 1; i < d.size(); ++i)
    if (d[i].count)
      MRTF(d[0].ctx, mrt_shard_unpack_device(d[0].ctx, W, H, shard(i), shards(), d[i].recv, d[0].rgb, d[0].b, d[0].st));
  HIPF(hipSetDevice(d[0].device));
  HIPF(hipStreamSynchronize(d[0].st));
  gather_bytes += bytes;
  gather_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// The gather transport of n devices (distinct: no repeats): "none" for one,
// "peer" for repeated devices (a rehearsal on one GPU), else RCCL if
// init_rccl() (open RCCL, create the communicators) succeeds, and peer copies
// with the reason otherwise. mrt_create_multi and mrt_debug_transport share it.
template <typename Init>
std::string choose_transport(int n, bool distinct, Init&& init_rccl, bool& use_rccl) {
  use_rccl = false;
  if (n == 1) return "none";
  if (!distinct) return "peer";
  try {
    init_rccl();
    use_rccl = true;
    return "rccl";
  } catch (const Fail& e) {
    return "peer (RCCL unavailable: " + e.msg + ")";
  }
}

std::vector<mrt_ctx*> devices_of(mrt_ctx* ctx) {
  MultiDev* m = ctx_multi(ctx);
  return m ? m->devs : std::vector<mrt_ctx*>{ctx};
}

template <typename F>
int guard(mrt_ctx* ctx, F&& f) {
  try {
    f();
    return MRT_OK;
  } catch (const Fail& e) {
    ctx_set_error(ctx, e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    ctx_set_error(ctx, "out of host memory");
    return MRT_ERR_NOMEM;
  } catch (const std::exception& e) {
    ctx_set_error(ctx, e.what());
    return MRT_ERR_INVALID;
  }
}

}  // namespace

// ---- render.hip's side of a multi-device handle (frames.h) -----------------
int multi_count(const MultiDev* m) { return (int)m->devs.size(); }
mrt_ctx* multi_dev(const MultiDev* m, int i) { return m->devs[(size_t)i]; }

void multi_free(MultiDev* m) {
  if (!m) return;
  delete m->scratch;
  if (!m->comms.empty() && m->R && m->R->comm_destroy)
    for (ncclComm_t c : m->comms) m->R->comm_destroy(c);
  for (mrt_ctx* c : m->devs) mrt_destroy(c);
  delete m;
}

int multi_render(MultiDev* m, const mrt_render_args* a, float* rgb, uint32_t* bounces, std::string& err) {
  try {
    if (!a || !rgb || !bounces) throw Fail{MRT_ERR_INVALID, "null argument"};
    if (!valid_size(a->width, a->height)) throw Fail{MRT_ERR_INVALID, "bad image size"};
    const uint32_t sc = a->shard_count ? a->shard_count : 1;
    if (a->shard_index >= sc) throw Fail{MRT_ERR_INVALID, "shard_index >= shard_count"};
    if (!m->scratch) m->scratch = new Frame();
    Frame& f = *m->scratch;
    if (f.d.empty() || f.W != a->width || f.H != a->height || f.si != a->shard_index || f.sc != sc)
      f.setup(m, m->devs, a->width, a->height, a->shard_index, sc);
    const size_t n = f.npix();
    // Device 0 starts from the caller's whole buffers: after the gather it
    // holds every device's shards, and every other pixel of the frame (the
    // other processes' shards when shard_count > 1) stays as the caller had
    // it, so the copy back below returns the caller's sums there unchanged.
    // Devices 1.. start from the caller's sums of their own shard's pixels
    // only (what they add to), packed on the host into their slab.
    {
      std::vector<Fail> fails(f.d.size(), Fail{MRT_OK, ""});
      std::vector<std::thread> th;
      for (size_t i = 0; i < f.d.size(); ++i)
        th.emplace_back([&, i] {
          try {
            DevFrame& d = f.d[i];
            HIPF(hipSetDevice(d.device));
            if (i == 0) {
              HIPF(hipMemcpyAsync(d.rgb, rgb, n * 12, hipMemcpyHostToDevice, d.st));
              HIPF(hipMemcpyAsync(d.b, bounces, n * 4, hipMemcpyHostToDevice, d.st));
              HIPF(hipStreamSynchronize(d.st));
              return;
            }
            if (!d.count) return;
            std::vector<uint32_t> slab((size_t)d.count * 4);
            for (uint32_t k = 0; k < d.count; ++k) {
              const uint32_t p = d.pix[k];
              memcpy(&slab[4 * (size_t)k], rgb + 3 * (size_t)p, 12);
              slab[4 * (size_t)k + 3] = bounces[p];
            }
            HIPF(hipMemcpyAsync(d.slab, slab.data(), slab.size() * 4, hipMemcpyHostToDevice, d.st));
            MRTF(d.ctx, mrt_shard_unpack_device(d.ctx, f.W, f.H, f.shard(i), f.shards(), d.slab, d.rgb, d.b, d.st));
            HIPF(hipStreamSynchronize(d.st));  // the host slab goes out of scope
          } catch (const Fail& e) {
            fails[i] = e;
          }
        });
      for (auto& t : th) t.join();
      for (const Fail& e : fails)
        if (e.code != MRT_OK) throw e;
    }
    f.render(*a);
    f.gather();
    HIPF(hipSetDevice(f.d[0].device));
    HIPF(hipMemcpyAsync(rgb, f.d[0].rgb, n * 12, hipMemcpyDeviceToHost, f.d[0].st));
    HIPF(hipMemcpyAsync(bounces, f.d[0].b, n * 4, hipMemcpyDeviceToHost, f.d[0].st));
    HIPF(hipStreamSynchronize(f.d[0].st));
    return MRT_OK;
  } catch (const Fail& e) {
    err = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    err = e.what();
    return MRT_ERR_INVALID;
  }
}

int multi_set_gather(MultiDev* m, int64_t mode, std::string& err) {
  if (mode != MRT_GATHER_AUTO && mode != MRT_GATHER_PEER && mode != MRT_GATHER_RCCL) {
    err = "option gather must be MRT_GATHER_AUTO, _PEER or _RCCL";
    return MRT_ERR_INVALID;
  }
  if (mode == MRT_GATHER_RCCL && !m->distinct) {
    err = "option gather: RCCL needs distinct devices (one rank per device)";
    return MRT_ERR_INVALID;
  }
  if (mode != MRT_GATHER_PEER && m->distinct && m->devs.size() > 1) {
    try {
      ensure_comms(m);
    } catch (const Fail& e) {
      if (mode == MRT_GATHER_RCCL) {
        err = e.msg;
        return MRT_ERR_HIP;
      }
      m->comms.clear();
      m->rccl = false;
      m->mode = mode;
      m->transport = "peer (RCCL unavailable: " + e.msg + ")";
      err.clear();
      return MRT_OK;
    }
    m->rccl = true;
    m->transport = "rccl";
  } else if (m->devs.size() > 1) {
    m->rccl = false;
    m->transport = "peer";
  }
  m->mode = mode;
  err.clear();
  return MRT_OK;
}
int64_t multi_gather(const MultiDev* m) { return m->mode; }
const char* multi_transport(const MultiDev* m) { return m->transport.c_str(); }

// ---- the device-resident Image ----------------------------------------------
struct mrt_image {
  mrt_ctx* ctx = nullptr;  // the handle it was created on (counts it: ctx_images)
  Frame f;
  uint32_t passes = 0;
  bool gathered = true;  // device 0's buffers hold every device's tiles
  float* aux = nullptr;  // device 0: albedo then normal (W*H*3 each), zero before a pre-pass
  uint8_t* rgb8 = nullptr;  // device 0: display bytes
};

extern "C" {

int mrt_create_multi(int n, const int* devices, mrt_ctx** out) {
  if (!out || !devices || n < 1) {
    ctx_set_error(nullptr, "mrt_create_multi: need n >= 1 devices and an output pointer");
    return MRT_ERR_INVALID;
  }
  *out = nullptr;
  MultiDev* m = new MultiDev();
  m->ids.assign(devices, devices + n);
  for (int i = 0; i < n; ++i) {
    mrt_ctx* c = nullptr;
    const int rc = mrt_create(devices[i], &c);
    if (rc != MRT_OK) {  // mrt_create left its message in the global error
      const std::string msg = mrt_global_last_error();
      multi_free(m);
      ctx_set_error(nullptr, msg);
      return rc;
    }
    m->devs.push_back(c);
  }
  std::vector<int> sorted = m->ids;
  std::sort(sorted.begin(), sorted.end());
  m->distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  // xGMI peer access from device 0 to the others and back (peer copies and
  // RCCL's P2P transport); already-enabled is fine
  for (int i = 1; i < n; ++i) {
    if (devices[i] == devices[0]) continue;
    hipSetDevice(devices[0]);
    hipDeviceEnablePeerAccess(devices[i], 0);
    hipSetDevice(devices[i]);
    hipDeviceEnablePeerAccess(devices[0], 0);
  }
  (void)hipGetLastError();
  // RCCL between distinct devices: opened and its communicators created
  // now, so a missing or failing RCCL shows here and not after a render;
  // the context then gathers with peer copies and says why
  m->transport = choose_transport(n, m->distinct, [&] { ensure_comms(m); }, m->rccl);
  if (!m->rccl) m->comms.clear();
  *out = ctx_wrap_multi(m);
  return MRT_OK;
}

int mrt_debug_rccl_library(const char* name) {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  g_rccl_name = name && *name ? name : "librccl.so.1";
  return MRT_OK;
}

int mrt_debug_transport(int n, const int* devices, char* buf, uint32_t len) {
  if (n < 1 || !devices || !buf || !len) {
    ctx_set_error(nullptr, "mrt_debug_transport: need n >= 1 devices and a buffer");
    return MRT_ERR_INVALID;
  }
  std::vector<int> sorted(devices, devices + n);
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  bool use = false;
  // the loader only (no communicators: this runs without GPUs)
  const std::string t = choose_transport(n, distinct, [] { rccl(); }, use);
  snprintf(buf, len, "%s", t.c_str());
  return MRT_OK;
}

const char* mrt_context_transport(const mrt_ctx* ctx) {
  MultiDev* m = ctx_multi(ctx);
  return m ? m->transport.c_str() : "none";
}

int mrt_context_devices(mrt_ctx* ctx, int* n, int* devices) {
  if (!ctx || !n) {
    ctx_set_error(ctx, "null argument");
    return MRT_ERR_INVALID;
  }
  if (MultiDev* m = ctx_multi(ctx)) {
    *n = (int)m->ids.size();
    if (devices) std::copy(m->ids.begin(), m->ids.end(), devices);
  } else {
    *n = 1;
    if (devices) devices[0] = massrt_ctx_device(ctx);
  }
  return MRT_OK;
}

int mrt_image_create(mrt_ctx* ctx, uint32_t W, uint32_t H, mrt_image** out) {
  if (!ctx || !out) {
    ctx_set_error(ctx, "null argument");
    return MRT_ERR_INVALID;
  }
  *out = nullptr;
  auto img = std::make_unique<mrt_image>();
  img->ctx = ctx;
  const int rc = guard(ctx, [&] {
    if (!valid_size(W, H)) throw Fail{MRT_ERR_INVALID, "bad image size"};
    img->f.setup(ctx_multi(ctx), devices_of(ctx), W, H, 0, 1);
    HIPF(hipSetDevice(img->f.d[0].device));
    HIPF(hipStreamSynchronize(img->f.d[0].st));
  });
  if (rc == MRT_OK) {
    ctx_images(ctx, +1);
    *out = img.release();
  }
  return rc;
}

int mrt_image_destroy(mrt_image* img) {
  if (!img) return MRT_OK;
  if (!img->f.d.empty()) {
    hipSetDevice(img->f.d[0].device);
    if (img->f.d[0].st) hipStreamSynchronize(img->f.d[0].st);
    hipFree(img->aux);
    hipFree(img->rgb8);
  }
  ctx_images(img->ctx, -1);
  delete img;
  return MRT_OK;
}

int mrt_image_clear(mrt_image* img) {
  if (!img) return MRT_ERR_INVALID;
  return guard(img->ctx, [&] {
    img->f.clear();
    img->passes = 0;
    img->gathered = true;
  });
}

int mrt_image_render(mrt_image* img, uint64_t seed, uint32_t spp_begin, uint32_t passes, uint32_t max_depth,
                     uint32_t flags) {
  if (!img) return MRT_ERR_INVALID;
  return guard(img->ctx, [&] {
    if ((uint64_t)spp_begin + passes > 0xFFFFFFFFull) throw Fail{MRT_ERR_INVALID, "sample index overflow"};
    if ((uint64_t)img->passes + passes > 0xFFFFFFFFull) throw Fail{MRT_ERR_INVALID, "pass count overflow"};
    if (flags & ~(uint32_t)(MRT_RENDER_COUNTERS | MRT_RENDER_TIME_KERNELS))
      throw Fail{MRT_ERR_INVALID, "mrt_image_render takes MRT_RENDER_COUNTERS / MRT_RENDER_TIME_KERNELS only"};
    if (!passes) return;
    mrt_render_args a{img->f.W, img->f.H, spp_begin, passes, seed, max_depth, 0, 1, flags};
    img->f.render(a);
    img->passes += passes;
    img->gathered = img->f.d.size() == 1;
  });
}

int mrt_image_prepass(mrt_image* img, uint64_t seed) {
  if (!img) return MRT_ERR_INVALID;
  return guard(img->ctx, [&] {
    DevFrame& d0 = img->f.d[0];
    const size_t n = img->f.npix();
    HIPF(hipSetDevice(d0.device));
    if (!img->aux) HIPF(hipMalloc(&img->aux, n * 24));
    MRTF(d0.ctx, mrt_prepass_device(d0.ctx, img->f.W, img->f.H, seed, img->aux, img->aux + 3 * n, d0.st));
  });
}

int mrt_image_read(mrt_image* img, float* rgb, uint32_t* bounces, uint32_t* passes) {
  if (!img) return MRT_ERR_INVALID;
  if (!rgb && !bounces) {  // the pass count alone: no gather, no sync
    if (passes) *passes = img->passes;
    return MRT_OK;
  }
  return guard(img->ctx, [&] {
    if (!img->gathered) {
      img->f.gather();
      img->gathered = true;
    }
    DevFrame& d0 = img->f.d[0];
    const size_t n = img->f.npix();
    HIPF(hipSetDevice(d0.device));
    if (rgb) HIPF(hipMemcpyAsync(rgb, d0.rgb, n * 12, hipMemcpyDeviceToHost, d0.st));
    if (bounces) HIPF(hipMemcpyAsync(bounces, d0.b, n * 4, hipMemcpyDeviceToHost, d0.st));
    HIPF(hipStreamSynchronize(d0.st));
    if (passes) *passes = img->passes;
  });
}

int mrt_image_gather(mrt_image* img) {
  if (!img) return MRT_ERR_INVALID;
  return guard(img->ctx, [&] {
    if (!img->gathered) {
      img->f.gather();
      img->gathered = true;
    }
    for (DevFrame& d : img->f.d) {  // every device's queued work has ended
      HIPF(hipSetDevice(d.device));
      HIPF(hipStreamSynchronize(d.st));
    }
  });
}

int mrt_image_tonemap(mrt_image* img, uint32_t mode, uint8_t* out) {
  if (!img) return MRT_ERR_INVALID;
  return guard(img->ctx, [&] {
    if (!out) throw Fail{MRT_ERR_INVALID, "null output"};
    if (mode > MRT_DISPLAY_NORMAL) throw Fail{MRT_ERR_INVALID, "bad display mode"};
    const bool aux = mode == MRT_DISPLAY_ALBEDO || mode == MRT_DISPLAY_NORMAL;
    DevFrame& d0 = img->f.d[0];
    const size_t n = img->f.npix();
    if (!aux && !img->gathered) {
      img->f.gather();
      img->gathered = true;
    }
    HIPF(hipSetDevice(d0.device));
    if (!img->rgb8) HIPF(hipMalloc(&img->rgb8, n * 3));
    if (aux && !img->aux) {  // Image::to_rgb_bytes: no buffer yet -> zeros
      HIPF(hipMemsetAsync(img->rgb8, 0, n * 3, d0.st));
    } else {
      const float* src = aux ? img->aux + (mode == MRT_DISPLAY_NORMAL ? 3 * n : 0) : d0.rgb;
      MRTF(d0.ctx, mrt_tonemap_device(d0.ctx, img->f.W, img->f.H, src, d0.b, img->passes, mode, img->rgb8, d0.st));
    }
    HIPF(hipMemcpyAsync(out, img->rgb8, n * 3, hipMemcpyDeviceToHost, d0.st));
    HIPF(hipStreamSynchronize(d0.st));
  });
}

int mrt_image_gather_stats(mrt_image* img, uint64_t* bytes, double* ms) {
  if (!img) return MRT_ERR_INVALID;
  if (bytes) *bytes = img->f.gather_bytes;
  if (ms) *ms = img->f.gather_ms;
  return MRT_OK;
}

int mrt_image_device_stats(mrt_image* img, int n, double* render_ms) {
  if (!img) return MRT_ERR_INVALID;
  return guard(img->ctx, [&] {
    if (!render_ms || n < (int)img->f.d.size()) throw Fail{MRT_ERR_INVALID, "render_ms needs one entry per device"};
    img->f.collect_times();
    for (size_t i = 0; i < img->f.d.size(); ++i) render_ms[i] = img->f.d[i].render_ms;
  });
}

}  // extern "C"
