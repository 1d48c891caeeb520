// mrt_render_multi — render() (main.rs:150-295) over several GPUs from ONE
// process through the C ABI, as a C or Rust caller would: one context over
// the device list (mrt_create_multi), one device-resident Image
// (mrt_image_*), `passes` 1-spp passes, then the gathered sums and the PNG.
// The library splits the tiles over the devices and gathers them onto the
// first device (RCCL between distinct devices, peer copies otherwise).
//
//   mrt_render_multi <scene> <W> <H> <passes> <out.png> <asset_dir> <devices> [rccl|peer] [raw_out]
//     devices: comma list, e.g. 0,1,2,3 (repeats allowed with `peer`, e.g.
//     0,0 to rehearse the exchange on one GPU; RCCL needs distinct devices)
//     raw_out: also write the accumulated float sums and u32 bounce counts
//
// Prints: scene, size, passes, devices, render seconds, gather bytes/ms, Msamples/s.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/massrt.h"

static void die(const char* what, mrt_ctx* ctx) {
  std::fprintf(stderr, "%s failed: %s\n", what, ctx ? mrt_last_error(ctx) : mrt_global_last_error());
  std::exit(1);
}

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
  if (devs.empty() || (transport != "rccl" && transport != "peer")) return 2;
  setenv("MRT_GATHER", transport.c_str(), 1);  // read by mrt_create_multi

  // Scene::generate + World::build_bvh once on the host (fastrand seed 1, main.rs:86)
  mrt_builder* b = nullptr;
  if (mrt_builder_new(1, &b) != MRT_OK) die("mrt_builder_new", nullptr);
  if (mrt_builder_builtin(b, scene.c_str(), 16.0f / 9.0f, assets.c_str()) != MRT_OK) {
    std::fprintf(stderr, "scene: %s\n", mrt_builder_last_error());
    return 1;
  }
  mrt_scene_desc desc;
  mrt_camera cam;
  if (mrt_builder_desc(b, &desc, &cam) != MRT_OK) die("mrt_builder_desc", nullptr);

  mrt_ctx* ctx = nullptr;
  if (mrt_create_multi((int)devs.size(), devs.data(), &ctx) != MRT_OK) die("mrt_create_multi", nullptr);
  if (mrt_upload_scene(ctx, &desc) != MRT_OK) die("mrt_upload_scene", ctx);
  if (mrt_set_camera(ctx, &cam) != MRT_OK) die("mrt_set_camera", ctx);
  mrt_builder_free(b);
  mrt_image* img = nullptr;
  if (mrt_image_create(ctx, W, H, &img) != MRT_OK) die("mrt_image_create", ctx);

  const auto t0 = std::chrono::steady_clock::now();
  if (mrt_image_render(img, 1, 0, passes, 50, 0) != MRT_OK) die("mrt_image_render", ctx);
  const size_t n = (size_t)W * H;
  std::vector<float> rgb(n * 3);
  std::vector<uint32_t> bounces(n);
  uint32_t got = 0;
  if (mrt_image_read(img, rgb.data(), bounces.data(), &got) != MRT_OK) die("mrt_image_read", ctx);
  const auto t1 = std::chrono::steady_clock::now();
  std::vector<uint8_t> bytes(n * 3);
  if (mrt_image_tonemap(img, MRT_DISPLAY_DEFAULT, bytes.data()) != MRT_OK) die("mrt_image_tonemap", ctx);
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
  uint64_t gb = 0;
  double gms = 0;
  mrt_image_gather_stats(img, &gb, &gms);
  const double rs = std::chrono::duration<double>(t1 - t0).count();
  std::printf("%s %ux%u passes=%u devices=%zu transport=%s render_s=%.3f gather_bytes=%llu gather_ms=%.3f "
              "msamples_per_s=%.1f\n",
              scene.c_str(), W, H, got, devs.size(), transport.c_str(), rs, (unsigned long long)gb, gms,
              (double)n * passes / rs / 1e6);
  mrt_image_destroy(img);
  mrt_destroy(ctx);
  return 0;
}
