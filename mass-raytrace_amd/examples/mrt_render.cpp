// mrt_render — the C++ driver in the role of the reference's render()
// (main.rs:150-295) + export (main.rs:760-783), written against the C ABI
// only (include/massrt.h): build a built-in Scene, pre-pass, render N
// passes of 1 spp into the accumulation buffers, tonemap, write PNGs.
//
//   mrt_render <scene> <width> <height> <passes> <out.png> [asset_dir] [device]
//
// Prints one line: scene, size, passes, render seconds, Msamples/s.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/massrt.h"

static int fail(const char* what, mrt_ctx* ctx) {
  std::fprintf(stderr, "%s failed: %s\n", what, ctx ? mrt_last_error(ctx) : mrt_global_last_error());
  return 1;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s <scene> <width> <height> <passes> <out.png> [asset_dir] [device]\n", argv[0]);
    return 2;
  }
  const std::string scene = argv[1];
  const uint32_t W = (uint32_t)std::atoi(argv[2]), H = (uint32_t)std::atoi(argv[3]);
  const uint32_t passes = (uint32_t)std::atoi(argv[4]);
  const std::string out = argv[5];
  const std::string assets = argc > 6 ? argv[6] : "";
  const int device = argc > 7 ? std::atoi(argv[7]) : 0;

  // Scene::generate + World::build_bvh (scenes.rs, world.rs:117-122); fastrand seed 1 (main.rs:86)
  mrt_builder* b = nullptr;
  if (mrt_builder_new(1, &b) != MRT_OK) return fail("mrt_builder_new", nullptr);
  if (mrt_builder_builtin(b, scene.c_str(), 16.0f / 9.0f, assets.c_str()) < 0) {
    std::fprintf(stderr, "scene: %s\n", mrt_builder_last_error());
    return 1;
  }
  mrt_scene_desc desc;
  mrt_camera cam;
  if (mrt_builder_desc(b, &desc, &cam) != MRT_OK) {
    std::fprintf(stderr, "desc: %s\n", mrt_builder_last_error());
    return 1;
  }
  mrt_ctx* ctx = nullptr;
  if (mrt_create(device, &ctx) != MRT_OK) return fail("mrt_create", nullptr);
  if (mrt_upload_scene(ctx, &desc) != MRT_OK) return fail("mrt_upload_scene", ctx);
  if (mrt_set_camera(ctx, &cam) != MRT_OK) return fail("mrt_set_camera", ctx);
  mrt_builder_free(b);

  const size_t n = (size_t)W * H;
  std::vector<float> albedo(n * 3), normal(n * 3), rgb(n * 3, 0.0f);
  std::vector<uint32_t> bounces(n, 0);
  std::vector<uint8_t> bytes(n * 3);
  // pre-render pass (main.rs:162-222)
  if (mrt_prepass(ctx, W, H, 1, albedo.data(), normal.data()) != MRT_OK) return fail("mrt_prepass", ctx);
  // passes (main.rs:235-290): each pass is one sample of every pixel, merged in order
  const auto t0 = std::chrono::steady_clock::now();
  mrt_render_args a{W, H, 0, passes, 1, 50, 0, 1, 0};
  if (mrt_render(ctx, &a, rgb.data(), bounces.data()) != MRT_OK) return fail("mrt_render", ctx);
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  // export (main.rs:760-783): Default view, plus the auxiliary views next to it
  const char* names[4] = {"", "_depth", "_albedo", "_normal"};
  for (uint32_t mode = MRT_DISPLAY_DEFAULT; mode <= MRT_DISPLAY_NORMAL; ++mode) {
    const float* src = mode == MRT_DISPLAY_ALBEDO ? albedo.data() : mode == MRT_DISPLAY_NORMAL ? normal.data() : rgb.data();
    if (mrt_tonemap(ctx, W, H, src, bounces.data(), passes, mode, bytes.data()) != MRT_OK) return fail("mrt_tonemap", ctx);
    std::string path = out;
    if (mode) {
      const size_t dot = path.rfind('.');
      path = (dot == std::string::npos ? path : path.substr(0, dot)) + names[mode] + ".png";
    }
    if (mrt_write_png(path.c_str(), W, H, bytes.data()) != MRT_OK) {
      std::fprintf(stderr, "png: %s\n", mrt_builder_last_error());
      return 1;
    }
  }
  std::printf("%s %ux%u passes=%u render_s=%.3f msamples_per_s=%.1f\n", scene.c_str(), W, H, passes, secs,
              (double)n * passes / secs / 1e6);
  mrt_destroy(ctx);
  return 0;
}
