// capi.cpp — C ABI of the host scene builder and loaders (include/massrt.h).
// Mirrors what the reference's worker does before render(): Scene::generate
// (scenes.rs:25-33) and World::build_bvh (main.rs:107-112), and hands the
// reference-topology tree to the device half as an mrt_scene_desc.
#include <string.h>

#include "../device/build.h"
#include "display.h"
#include "world.h"

// device ordinal of a context (render.hip), -1 for a null context
int massrt_ctx_device(const mrt_ctx* ctx);

using namespace massrt;

struct mrt_builder {
  std::unique_ptr<World> world;
  DeviceBuildStats build_stats;
  Camera camera;
  bool has_camera = false;
  std::vector<Model> models;
  std::vector<Material> materials;
  std::vector<Surface> surfaces;
  std::string err;
};

static thread_local std::string g_builder_error;

namespace {

template <typename F>
int guard(mrt_builder* b, F&& f) {
  if (!b) {
    g_builder_error = "null builder";
    return MRT_ERR_INVALID;
  }
  try {
    return f();
  } catch (const Error& e) {
    b->err = e.what();
    g_builder_error = b->err;
    return -e.code;
  } catch (const std::exception& e) {
    b->err = e.what();
    g_builder_error = b->err;
    return -MRT_ERR_INVALID;
  }
}

V3 v3p(const float* p) { return V3{p[0], p[1], p[2]}; }

}  // namespace

extern "C" {

const char* mrt_builder_last_error(void) { return g_builder_error.c_str(); }

int mrt_builder_new(uint64_t rng_seed, mrt_builder** out) {
  if (!out) return MRT_ERR_INVALID;
  mrt_builder* b = new mrt_builder();
  b->world = std::make_unique<World>(SolidBackground(V3{0, 0, 0}), rng_seed);
  *out = b;
  return MRT_OK;
}

int mrt_builder_free(mrt_builder* b) {
  delete b;
  return MRT_OK;
}

int mrt_builder_builtin(mrt_builder* b, const char* name, float aspect, const char* asset_dir) {
  int rc = guard(b, [&] {
    uint64_t seed = b->world->rng.state;
    SceneResult r = generate_builtin(name ? name : "", aspect, asset_dir ? asset_dir : "", seed);
    b->world = std::move(r.world);
    b->camera = r.camera;
    b->has_camera = true;
    return 0;
  });
  return rc < 0 ? -rc : rc;
}

float mrt_builder_rand_f32(mrt_builder* b) { return b ? b->world->rand_f32() : 0.0f; }

int mrt_builder_solid(mrt_builder* b, float r, float g, float bl, float a) {
  return guard(b, [&] {
    b->surfaces.push_back(SolidColor(V4{r, g, bl, a}));
    return (int)b->surfaces.size() - 1;
  });
}

int mrt_builder_texture_png(mrt_builder* b, const char* path, uint32_t wrap) {
  return guard(b, [&] {
    b->surfaces.push_back(TextureSurface(Texture::load_png(path ? path : "", (WrapMode)wrap)));
    return (int)b->surfaces.size() - 1;
  });
}

int mrt_builder_texture_rgba(mrt_builder* b, const uint8_t* rgba, uint32_t w, uint32_t h, uint32_t wrap) {
  return guard(b, [&] {
    if (!rgba || !w || !h) throw Error(MRT_ERR_INVALID, "empty texture");
    b->surfaces.push_back(TextureSurface(Texture::load_bytes(rgba, w, h, (WrapMode)wrap)));
    return (int)b->surfaces.size() - 1;
  });
}

int mrt_builder_material(mrt_builder* b, uint32_t kind, uint32_t surface, float param, float er, float eg, float eb) {
  return guard(b, [&] {
    Surface s;
    if (kind == MRT_MAT_LAMBERTIAN || kind == MRT_MAT_METAL || kind == MRT_MAT_SPECULAR) {
      if (surface >= b->surfaces.size()) throw Error(MRT_ERR_INVALID, "surface index out of range");
      s = b->surfaces[surface];
    }
    Material m;
    switch (kind) {
      case MRT_MAT_NONE:
        m = NoMaterial();
        break;
      case MRT_MAT_LAMBERTIAN:
        m = Lambertian(s);
        break;
      case MRT_MAT_METAL:
        m = Metal(param, s);
        break;
      case MRT_MAT_DIELECTRIC:
        m = Dielectric(param);
        break;
      case MRT_MAT_DIFFUSE_LIGHT:
        m = DiffuseLight(V3{er, eg, eb});
        break;
      case MRT_MAT_SPECULAR:
        m = Specular(param, s);
        break;
      case MRT_MAT_ISOTROPHIC:
        m = Isotrophic(V3{er, eg, eb});
        break;
      default:
        throw Error(MRT_ERR_INVALID, "bad material kind");
    }
    b->materials.push_back(m);
    return (int)b->materials.size() - 1;
  });
}

int mrt_builder_mix(mrt_builder* b, float ratio, uint32_t left, uint32_t right) {
  return guard(b, [&] {
    if (left >= b->materials.size() || right >= b->materials.size())
      throw Error(MRT_ERR_INVALID, "material index out of range");
    b->materials.push_back(Mix(ratio, b->materials[left], b->materials[right]));
    return (int)b->materials.size() - 1;
  });
}

static const Surface& surf_at(mrt_builder* b, uint32_t i) {
  if (i >= b->surfaces.size()) throw Error(MRT_ERR_INVALID, "surface index out of range");
  return b->surfaces[i];
}

int mrt_builder_ycbcr(mrt_builder* b, uint32_t luma, uint32_t chroma) {
  return guard(b, [&] {
    const Surface &l = surf_at(b, luma), &c = surf_at(b, chroma);
    if (l.kind != MRT_SURF_TEXTURE || c.kind != MRT_SURF_TEXTURE)
      throw Error(MRT_ERR_INVALID, "YCbCr planes must be texture surfaces");
    b->surfaces.push_back(YCbCrTexture(l.texture, c.texture));
    return (int)b->surfaces.size() - 1;
  });
}

int mrt_builder_blend(mrt_builder* b, uint32_t mode, uint32_t left, uint32_t right) {
  return guard(b, [&] {
    if (mode > MRT_BLEND_SUBTRACTION) throw Error(MRT_ERR_INVALID, "bad blend mode");
    b->surfaces.push_back(TextureBlend(mode, surf_at(b, left), surf_at(b, right)));
    return (int)b->surfaces.size() - 1;
  });
}

int mrt_builder_fallback(mrt_builder* b, float r, float g, float bl, float a, uint32_t surface) {
  return guard(b, [&] {
    b->surfaces.push_back(SolidColorFallback(V4{r, g, bl, a}, surf_at(b, surface)));
    return (int)b->surfaces.size() - 1;
  });
}

int mrt_builder_background_cubemap(mrt_builder* b, const uint32_t* faces, const float* rotation) {
  return guard(b, [&] {
    if (!faces || !rotation) throw Error(MRT_ERR_INVALID, "null argument");
    Surface f[6];
    for (int k = 0; k < 6; ++k) f[k] = surf_at(b, faces[k]);
    b->world->set_background(CubeMap(f, V3{rotation[0], rotation[1], rotation[2]}));
    return 0;
  });
}

static const Material& mat_at(mrt_builder* b, uint32_t i) {
  if (i >= b->materials.size()) throw Error(MRT_ERR_INVALID, "material index out of range");
  return b->materials[i];
}

int mrt_builder_background(mrt_builder* b, uint32_t kind, uint32_t surface, float r, float g, float bl) {
  return guard(b, [&] {
    if (kind == MRT_BG_SOLID)
      b->world->set_background(SolidBackground(V3{r, g, bl}));
    else if (kind == MRT_BG_SKY)
      b->world->set_background(SkyBackground());
    else if (kind == MRT_BG_SKYSPHERE) {
      if (surface >= b->surfaces.size()) throw Error(MRT_ERR_INVALID, "surface index out of range");
      b->world->set_background(SkySphere(b->surfaces[surface]));
    } else
      throw Error(MRT_ERR_INVALID, "bad background kind");
    return 0;
  });
}

int mrt_builder_add_sphere(mrt_builder* b, uint32_t material, float cx, float cy, float cz, float radius) {
  return guard(b, [&] {
    b->world->add(Sphere(mat_at(b, material), V3{cx, cy, cz}, radius));
    return 0;
  });
}

int mrt_builder_add_volume(mrt_builder* b, const float* center, float radius, float density, const float* albedo) {
  return guard(b, [&] {
    if (!center || !albedo) throw Error(MRT_ERR_INVALID, "null argument");
    return (int)b->world->add(VolumeDesc{v3p(center), radius, density, v3p(albedo)});
  });
}

int mrt_builder_add_triangle(mrt_builder* b, uint32_t material, const float* abc) {
  return guard(b, [&] {
    if (!abc) throw Error(MRT_ERR_INVALID, "null vertices");
    b->world->add(Triangle::make(mat_at(b, material), v3p(abc), v3p(abc + 3), v3p(abc + 6)));
    return 0;
  });
}

static int finish_model(mrt_builder* b, std::vector<Triangle> tris, uint32_t override_material, int add_to_world) {
  Model m = override_material == MRT_NO_MATERIAL
                ? b->world->model(std::move(tris))
                : b->world->model_with_material(mat_at(b, override_material), std::move(tris));
  if (add_to_world) b->world->add(m);
  b->models.push_back(m);
  return (int)b->models.size() - 1;
}

int mrt_builder_model(mrt_builder* b, uint32_t tri_material, uint32_t override_material, const float* tris,
                      uint32_t n, int with_shading, int add_to_world) {
  return guard(b, [&] {
    if (!tris || n == 0) throw Error(MRT_ERR_INVALID, "empty triangle list");
    const Material& tm = mat_at(b, tri_material);
    std::vector<Triangle> v;
    v.reserve(n);
    for (uint32_t i = 0; i < n; ++i) {
      if (with_shading) {
        const float* t = tris + 24 * (size_t)i;
        v.push_back(Triangle::with_norms_and_uvs(tm, v3p(t), v3p(t + 3), V2{t[6], t[7]}, v3p(t + 8), v3p(t + 11),
                                                 V2{t[14], t[15]}, v3p(t + 16), v3p(t + 19), V2{t[22], t[23]}));
      } else {
        const float* t = tris + 9 * (size_t)i;
        v.push_back(Triangle::make(tm, v3p(t), v3p(t + 3), v3p(t + 6)));
      }
    }
    return finish_model(b, std::move(v), override_material, add_to_world);
  });
}

int mrt_builder_model_from_ply(mrt_builder* b, const char* path, uint32_t tri_material, uint32_t override_material,
                               int add_to_world) {
  return guard(b, [&] {
    const Material& tm = mat_at(b, tri_material);
    std::vector<Triangle> v;
    for (auto& f : load_ply(path ? path : "")) v.push_back(Triangle::make(tm, f[0], f[1], f[2]));
    return finish_model(b, std::move(v), override_material, add_to_world);
  });
}

int mrt_builder_add_instance(mrt_builder* b, int model, const float* translation, const float* rotation,
                             const float* scale, uint32_t material) {
  return guard(b, [&] {
    if (model < 0 || (size_t)model >= b->models.size()) throw Error(MRT_ERR_INVALID, "model index out of range");
    if (!translation || !rotation || !scale) throw Error(MRT_ERR_INVALID, "null transform");
    InstanceDesc d = b->models[model].instance(v3p(translation), v3p(rotation), v3p(scale));
    if (material != MRT_NO_MATERIAL) d = d.with_material(mat_at(b, material));
    b->world->add(d);
    return 0;
  });
}

int mrt_builder_camera(mrt_builder* b, float vfov, const float* from, const float* at, const float* up, float aspect,
                       float aperture, float focus) {
  return guard(b, [&] {
    if (!from || !at || !up) throw Error(MRT_ERR_INVALID, "null camera vector");
    b->camera = Camera::make(vfov, v3p(from), v3p(at), v3p(up), aspect, aperture, focus);
    b->has_camera = true;
    return 0;
  });
}

static TreeBuilder device_builder(mrt_builder* b, mrt_ctx* ctx) {
  const int device = massrt_ctx_device(ctx);
  if (device < 0) throw Error(MRT_ERR_INVALID, "null device context");
  return [b, device](const std::vector<Item>& items, mrt::WyRand& rng, std::vector<mrt_node>& nodes,
                     BoundingBox& root_box) { device_build_tree(device, items, rng, nodes, root_box, &b->build_stats); };
}

int mrt_builder_build_bvh_device(mrt_builder* b, mrt_ctx* ctx) {
  int rc = guard(b, [&] {
    b->world->build_bvh(device_builder(b, ctx));
    return 0;
  });
  return rc < 0 ? -rc : rc;
}

int mrt_builder_builtin_device(mrt_builder* b, const char* name, float aspect, const char* asset_dir, mrt_ctx* ctx) {
  int rc = guard(b, [&] {
    const TreeBuilder tb = device_builder(b, ctx);
    uint64_t seed = b->world->rng.state;
    SceneResult r = generate_builtin(name ? name : "", aspect, asset_dir ? asset_dir : "", seed, &tb);
    b->world = std::move(r.world);
    b->camera = r.camera;
    b->has_camera = true;
    return 0;
  });
  return rc < 0 ? -rc : rc;
}

int mrt_builder_last_build_ms(mrt_builder* b, double* host_ms, double* device_ms) {
  int rc = guard(b, [&] {
    if (host_ms) *host_ms = b->build_stats.host_ms;
    if (device_ms) *device_ms = b->build_stats.device_ms;
    return 0;
  });
  return rc < 0 ? -rc : rc;
}

int mrt_builder_build_bvh(mrt_builder* b) {
  int rc = guard(b, [&] {
    b->world->build_bvh();
    return 0;
  });
  return rc < 0 ? -rc : rc;
}

int mrt_builder_desc(mrt_builder* b, mrt_scene_desc* desc, mrt_camera* camera) {
  int rc = guard(b, [&] {
    if (desc) *desc = b->world->desc();
    if (camera) {
      if (!b->has_camera) throw Error(MRT_ERR_STATE, "no camera");
      *camera = b->camera.to_abi();
    }
    return 0;
  });
  return rc < 0 ? -rc : rc;
}

static int64_t copy_tris(const std::vector<std::array<V3, 3>>& f, float* out, uint64_t cap) {
  if (out) {
    uint64_t n = std::min<uint64_t>(cap, f.size());
    for (uint64_t i = 0; i < n; ++i)
      for (int k = 0; k < 3; ++k) {
        out[9 * i + 3 * k] = f[i][k].x;
        out[9 * i + 3 * k + 1] = f[i][k].y;
        out[9 * i + 3 * k + 2] = f[i][k].z;
      }
  }
  return (int64_t)f.size();
}

int mrt_display_gamma_thresholds(uint32_t* out256) {
  if (!out256) return MRT_ERR_INVALID;
  const auto& t = mrt::gamma_thresholds();
  for (int k = 0; k < 256; ++k) out256[k] = t[k];
  return MRT_OK;
}

int mrt_write_png(const char* path, uint32_t width, uint32_t height, const uint8_t* rgb8) {
  std::string err;
  if (!path || !mrt::write_png_rgb8(path, width, height, rgb8, err)) {
    g_builder_error = path ? err : "null path";
    return MRT_ERR_IO;
  }
  return MRT_OK;
}

int64_t mrt_load_ply(const char* path, float* out, uint64_t cap) {
  try {
    return copy_tris(load_ply(path ? path : ""), out, cap);
  } catch (const std::exception& e) {
    g_builder_error = e.what();
    return -MRT_ERR_IO;
  }
}

int64_t mrt_load_stl(const char* path, float* out, uint64_t cap) {
  try {
    return copy_tris(load_stl_binary(path ? path : ""), out, cap);
  } catch (const std::exception& e) {
    g_builder_error = e.what();
    return -MRT_ERR_IO;
  }
}

int64_t mrt_load_obj(const char* path, float* out, uint64_t cap) {
  try {
    ObjResult r = load_obj(path ? path : "");
    if (out) {
      uint64_t n = std::min<uint64_t>(cap, r.faces.size());
      for (uint64_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
          const ObjCorner& c = r.faces[i].c[k];
          float* o = out + 24 * i + 8 * k;
          o[0] = c.v.x, o[1] = c.v.y, o[2] = c.v.z, o[3] = c.n.x, o[4] = c.n.y, o[5] = c.n.z, o[6] = c.uv.x,
          o[7] = c.uv.y;
        }
    }
    return (int64_t)r.faces.size();
  } catch (const std::exception& e) {
    g_builder_error = e.what();
    return -MRT_ERR_IO;
  }
}

}  // extern "C"
