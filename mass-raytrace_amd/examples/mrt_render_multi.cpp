// mrt_render_multi — render() (main.rs:150-295) over several GPUs from ONE
// process, for a C / Rust caller that has no torch.distributed: one thread
// and one mrt_ctx per device, each rendering its shard of 8x8 tiles
// (mrt_render_args.shard_index/count) into its own device frame; every
// device packs its pixels into a slab (mrt_shard_pack_device) and the slabs
// are gathered to the first device — RCCL send/recv over xGMI
// (ncclCommInitAll over the device list) or HIP peer copies — where each is
// unpacked into the frame (mrt_shard_unpack_device). That is Image::merge
// (main.rs:629-638) with every pixel summed on exactly one device, so the
// image equals the one-device render bit for bit.
//
//   mrt_render_multi <scene> <W> <H> <passes> <out.png> <asset_dir> <devices> [rccl|peer] [raw_out]
//     devices: comma list, e.g. 0,1,2,3 (repeats allowed with `peer`, e.g.
//     0,0 to rehearse the exchange on one GPU; RCCL needs distinct devices)
//     raw_out: also write the accumulated float sums and u32 bounce counts
//
// Prints: scene, size, passes, devices, render seconds, gather seconds, Msamples/s.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/massrt.h"

#define HIPOK(x)                                                                            \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                          \
      std::exit(1);                                                                         \
    }                                                                                       \
  } while (0)
#define NCCLOK(x)                                                                           \
  do {                                                                                      \
    ncclResult_t r_ = (x);                                                                  \
    if (r_ != ncclSuccess) {                                                                \
      std::fprintf(stderr, "%s: %s\n", #x, ncclGetErrorString(r_));                         \
      std::exit(1);                                                                         \
    }                                                                                       \
  } while (0)

static void die(const char* what, mrt_ctx* ctx) {
  std::fprintf(stderr, "%s failed: %s\n", what, ctx ? mrt_last_error(ctx) : mrt_global_last_error());
  std::exit(1);
}

struct Shard {
  int device = 0;
  mrt_ctx* ctx = nullptr;
  hipStream_t stream = nullptr;
  float* rgb = nullptr;      // device frame W*H*3 (this shard's tiles)
  uint32_t* bounces = nullptr;
  void* slab = nullptr;      // this shard's pixels, 16 B each (padded to the largest shard)
  uint32_t count = 0;
};

int main(int argc, char** argv) {
  if (argc < 8) {
    std::fprintf(stderr, "usage: %s <scene> <W> <H> <passes> <out.png> <asset_dir> <devices> [rccl|peer] [raw_out]\n",
                 argv[0]);
    return 2;
  }
  const std::string scene = argv[1];
  const uint32_t W = (uint32_t)std::atoi(argv[2]), H = (uint32_t)std::atoi(argv[3]);
  const uint32_t passes = (uint32_t)std::atoi(argv[4]);
  const std::string out = argv[5], assets = argv[6];
  std::vector<int> devs;
  {
    std::stringstream ss(argv[7]);
    for (std::string tok; std::getline(ss, tok, ',');) devs.push_back(std::atoi(tok.c_str()));
  }
  const std::string transport = argc > 8 ? argv[8] : "rccl";
  const std::string raw = argc > 9 ? argv[9] : "";
  const uint32_t N = (uint32_t)devs.size();
  if (N == 0 || (transport != "rccl" && transport != "peer")) return 2;

  // Scene::generate + World::build_bvh once on the host (fastrand seed 1, main.rs:86);
  // every device gets the same description (the scene is replicated).
  mrt_builder* b = nullptr;
  if (mrt_builder_new(1, &b) != MRT_OK) die("mrt_builder_new", nullptr);
  if (mrt_builder_builtin(b, scene.c_str(), 16.0f / 9.0f, assets.c_str()) < 0) {
    std::fprintf(stderr, "scene: %s\n", mrt_builder_last_error());
    return 1;
  }
  mrt_scene_desc desc;
  mrt_camera cam;
  if (mrt_builder_desc(b, &desc, &cam) != MRT_OK) die("mrt_builder_desc", nullptr);

  const size_t n = (size_t)W * H;
  std::vector<Shard> sh(N);
  uint32_t cap = 0;
  for (uint32_t r = 0; r < N; ++r) {
    if (mrt_shard_pixels(W, H, r, N, nullptr, &sh[r].count) != MRT_OK) die("mrt_shard_pixels", nullptr);
    cap = sh[r].count > cap ? sh[r].count : cap;
  }
  for (uint32_t r = 0; r < N; ++r) {
    Shard& s = sh[r];
    s.device = devs[r];
    HIPOK(hipSetDevice(s.device));
    if (mrt_create(s.device, &s.ctx) != MRT_OK) die("mrt_create", nullptr);
    if (mrt_upload_scene(s.ctx, &desc) != MRT_OK) die("mrt_upload_scene", s.ctx);
    if (mrt_set_camera(s.ctx, &cam) != MRT_OK) die("mrt_set_camera", s.ctx);
    HIPOK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    HIPOK(hipMalloc(&s.rgb, n * 12));
    HIPOK(hipMalloc(&s.bounces, n * 4));
    HIPOK(hipMalloc(&s.slab, (size_t)cap * 16 + 16));
    HIPOK(hipMemset(s.rgb, 0, n * 12));
    HIPOK(hipMemset(s.bounces, 0, n * 4));
  }
  mrt_builder_free(b);

  // root (shard 0's device) receives every slab
  std::vector<void*> recv(N, nullptr);
  HIPOK(hipSetDevice(sh[0].device));
  for (uint32_t r = 0; r < N; ++r) HIPOK(hipMalloc(&recv[r], (size_t)cap * 16 + 16));
  std::vector<ncclComm_t> comms;
  if (transport == "rccl" && N > 1) {
    comms.resize(N);
    NCCLOK(ncclCommInitAll(comms.data(), (int)N, devs.data()));
  }

  // render: each device its tiles, all passes (main.rs:235-290), concurrently
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> threads;
  for (uint32_t r = 0; r < N; ++r)
    threads.emplace_back([&, r] {
      Shard& s = sh[r];
      HIPOK(hipSetDevice(s.device));
      mrt_render_args a{W, H, 0, passes, 1, 50, r, N, 0};
      if (mrt_render_device(s.ctx, &a, s.rgb, s.bounces, s.stream) != MRT_OK) die("mrt_render_device", s.ctx);
      if (mrt_shard_pack_device(s.ctx, W, H, r, N, s.rgb, s.bounces, s.slab, s.stream) != MRT_OK)
        die("mrt_shard_pack_device", s.ctx);
      HIPOK(hipStreamSynchronize(s.stream));
    });
  for (auto& t : threads) t.join();
  const auto t1 = std::chrono::steady_clock::now();

  // gather the slabs onto the root
  if (!comms.empty()) {
    NCCLOK(ncclGroupStart());
    for (uint32_t r = 0; r < N; ++r) {
      NCCLOK(ncclSend(sh[r].slab, (size_t)sh[r].count * 4, ncclFloat, 0, comms[r], sh[r].stream));
      NCCLOK(ncclRecv(recv[r], (size_t)sh[r].count * 4, ncclFloat, (int)r, comms[0], sh[0].stream));
    }
    NCCLOK(ncclGroupEnd());
    for (uint32_t r = 0; r < N; ++r) HIPOK(hipStreamSynchronize(sh[r].stream));
  } else {
    HIPOK(hipSetDevice(sh[0].device));
    for (uint32_t r = 0; r < N; ++r)
      HIPOK(hipMemcpyPeerAsync(recv[r], sh[0].device, sh[r].slab, sh[r].device, (size_t)sh[r].count * 16,
                               sh[0].stream));
    HIPOK(hipStreamSynchronize(sh[0].stream));
  }
  // the root's frame: every shard's pixels unpacked into a zeroed image
  HIPOK(hipSetDevice(sh[0].device));
  float* frame_rgb = nullptr;
  uint32_t* frame_b = nullptr;
  HIPOK(hipMalloc(&frame_rgb, n * 12));
  HIPOK(hipMalloc(&frame_b, n * 4));
  HIPOK(hipMemsetAsync(frame_rgb, 0, n * 12, sh[0].stream));
  HIPOK(hipMemsetAsync(frame_b, 0, n * 4, sh[0].stream));
  for (uint32_t r = 0; r < N; ++r)
    if (mrt_shard_unpack_device(sh[0].ctx, W, H, r, N, recv[r], frame_rgb, frame_b, sh[0].stream) != MRT_OK)
      die("mrt_shard_unpack_device", sh[0].ctx);
  HIPOK(hipStreamSynchronize(sh[0].stream));
  const auto t2 = std::chrono::steady_clock::now();

  std::vector<float> rgb(n * 3);
  std::vector<uint32_t> bounces(n);
  std::vector<uint8_t> bytes(n * 3);
  HIPOK(hipMemcpy(rgb.data(), frame_rgb, n * 12, hipMemcpyDeviceToHost));
  HIPOK(hipMemcpy(bounces.data(), frame_b, n * 4, hipMemcpyDeviceToHost));
  if (mrt_tonemap(sh[0].ctx, W, H, rgb.data(), bounces.data(), passes, MRT_DISPLAY_DEFAULT, bytes.data()) != MRT_OK)
    die("mrt_tonemap", sh[0].ctx);
  if (mrt_write_png(out.c_str(), W, H, bytes.data()) != MRT_OK) die("mrt_write_png", nullptr);
  if (!raw.empty()) {
    FILE* f = std::fopen(raw.c_str(), "wb");
    if (!f || std::fwrite(rgb.data(), 4, rgb.size(), f) != rgb.size() ||
        std::fwrite(bounces.data(), 4, bounces.size(), f) != bounces.size()) {
      std::fprintf(stderr, "cannot write %s\n", raw.c_str());
      return 1;
    }
    std::fclose(f);
  }
  const double rs = std::chrono::duration<double>(t1 - t0).count(), gs = std::chrono::duration<double>(t2 - t1).count();
  std::printf("%s %ux%u passes=%u devices=%u transport=%s render_s=%.3f gather_s=%.4f msamples_per_s=%.1f\n",
              scene.c_str(), W, H, passes, N, transport.c_str(), rs, gs, (double)n * passes / rs / 1e6);
  for (auto& c : comms) ncclCommDestroy(c);
  for (uint32_t r = 0; r < N; ++r) {
    hipSetDevice(sh[r].device);
    hipFree(sh[r].rgb), hipFree(sh[r].bounces), hipFree(sh[r].slab);
    hipStreamDestroy(sh[r].stream);
    mrt_destroy(sh[r].ctx);
  }
  hipSetDevice(sh[0].device);
  for (void* p : recv) hipFree(p);
  hipFree(frame_rgb), hipFree(frame_b);
  return 0;
}
