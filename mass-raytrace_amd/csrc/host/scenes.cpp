// scenes.cpp — built-in scenes written against the host trait-surface mirror.
//   sphere_grid  = SphereGrid::generate   /root/reference/src/scenes/sphere_grid.rs:23-94
//   cornell      = CornellBox::generate   scenes/cornell.rs:20-99
//   cube_field   = BASELINE config 3: 10,000 cube.ply instances (lucy.rs:52-77 pattern)
//   mesh_ply     = BASELINE config 4: synthetic 1M-triangle binary PLY + 2 area lights
//   mesh_obj     = config 4 through obj_loader (v/vt/vn, obj_fns + Lambertian(SolidColor))
//   mesh_obj_textured = config 5: OBJ mesh + Lambertian(Texture) + SkySphere(Texture)
//   menger       = Menger::generate       scenes/menger.rs:20-105 (20^5 = 3.2M cube
//                  instances); menger_l3 = the same with the
//                  three innermost levels only (8,000 cubes, for quick tests)
// The scene RNG is the world's wyrand stream (fastrand::seed(1), main.rs:86);
// draws happen in the same statement order as the Rust scenes.
#include <stdio.h>

#include <functional>

#include "world.h"

namespace massrt {

using namespace mrt;

namespace {

std::string join_path(const std::string& dir, const std::string& name) {
  if (dir.empty()) return name;
  return dir.back() == '/' ? dir + name : dir + "/" + name;
}

std::vector<Triangle> ply_triangles(const std::string& path) {
  std::vector<Triangle> tris;
  for (auto& f : load_ply(path)) tris.push_back(Triangle::make(NoMaterial(), f[0], f[1], f[2]));
  return tris;
}

SceneResult sphere_grid(float aspect, const std::string& assets, uint64_t seed) {
  SceneResult r;
  r.world = std::make_unique<World>(SolidBackground(V3{0, 0, 0}), seed);
  World& world = *r.world;
  Material white = Lambertian(SolidColor(V4{1, 1, 1, 1}));
  Model cube = world.model(ply_triangles(join_path(assets, "cube.ply")));
  InstanceDesc ground = cube.instance(V3{0, -1000, 0}, V3{0, 0, 0}, fill3(1000)).with_material(white);
  world.add(ground);
  const float rr = 1.0f;
  const float d = rr * 2.0f;
  const float a = sqrtf(d * d - rr * rr);
  const int dim = 50;
  for (int i = -dim; i < dim; ++i) {
    for (int j = -dim; j < dim; ++j) {
      float off = (j % 2 == 0) ? rr : 0.0f;
      float x = ((float)i * d) + off;
      float z = (float)j * a;
      float y = rr;
      float radius = rr - 0.05f;
      if (i == 0 && j == 0) {
        world.add(Sphere(DiffuseLight(fill3(3.0f)), V3{x, y, z}, radius));
      } else if ((i == -1 && j == 0) || (i == 1 && j == 0) || (i == 1 && j == -1) || (i == 0 && j == -1) ||
                 (i == 1 && j == 1) || (i == 0 && j == 1)) {
        world.add(Sphere(Dielectric(1.8f), V3{x, y, z}, radius));
      } else {
        float cx = world.rand_f32();
        float cy = world.rand_f32();
        float cz = world.rand_f32();
        world.add(Sphere(Metal(0.0f, SolidColor(V4{cx, cy, cz, 1.0f})), V3{x, y, z}, radius));
      }
    }
  }
  V3 look_from{6, 8, 5}, look_at{0, 0, 0};
  r.camera = Camera::make(40.0f, look_from, look_at, V3{0, 1, 0}, aspect, 0.0f, length(look_from - look_at));
  return r;
}

SceneResult cornell(float aspect, const std::string& assets, uint64_t seed) {
  SceneResult r;
  r.world = std::make_unique<World>(SolidBackground(V3{0, 0, 0}), seed);
  World& world = *r.world;
  Material red = Lambertian(SolidColor(V4{1, 0, 0, 1}));
  Material green = Lambertian(SolidColor(V4{0, 1, 0, 1}));
  Material white = Lambertian(SolidColor(V4{1, 1, 1, 1}));
  Material light = DiffuseLight(fill3(8.0f));
  Material glass = Dielectric(1.3f);
  Model cube = world.model(ply_triangles(join_path(assets, "cube.ply")));
  world.add(cube.instance(V3{-10, 5, 0}, V3{0, 0, 0}, fill3(5)).with_material(red));
  world.add(cube.instance(V3{10, 5, 0}, V3{0, 0, 0}, fill3(5)).with_material(green));
  world.add(cube.instance(V3{0, 15, 0}, V3{0, 0, 0}, fill3(5)).with_material(white));
  world.add(cube.instance(V3{0, 5, -10}, V3{0, 0, 0}, fill3(5)).with_material(white));
  world.add(cube.instance(V3{0, -5, -0.0f}, V3{0, 0, 0}, fill3(5)).with_material(white));
  world.add(Sphere(glass, V3{1.75f, 2.0f, 2.25f}, 2.0f));
  world.add(cube.instance(V3{0, 10.0f - 0.00011f, 0}, V3{0, 0, 0}, V3{1.0f, 0.0001f, 1.0f}).with_material(light));
  world.add(cube.instance(V3{-2, 3, -1}, V3{0, -0.05f, 0}, V3{1.75f, 3.1f, 1.75f}).with_material(white));
  V3 look_from{0, 5, 20}, look_at{0, 5, 0};
  r.camera = Camera::make(37.0f, look_from, look_at, V3{0, 1, 0}, aspect, 0.0f, length(look_from - look_at));
  return r;
}

// Config 3: cube.ply instanced on a 100x100 grid (spacing 3), Lucy-style
// per-instance materials and yaw; ground cube + sun sphere from lucy.rs.
SceneResult cube_field(float aspect, const std::string& assets, uint64_t seed) {
  SceneResult r;
  r.world = std::make_unique<World>(SolidBackground(V3{0, 0, 0}), seed);
  World& world = *r.world;
  Model cube = world.model(ply_triangles(join_path(assets, "cube.ply")));
  Material white = Lambertian(SolidColor(V4{1, 1, 1, 1}));
  world.add(cube.instance(V3{0, -1000, 0}, V3{0, 0, 0}, fill3(1000)).with_material(white));
  int k = 0;
  for (int x = -50; x < 50; ++x) {
    for (int z = -50; z < 50; ++z, ++k) {
      Material m;
      if (k % 3 == 0) {
        float cr = 1.0f - (world.rand_f32() * 0.5f);
        float cg = 1.0f - (world.rand_f32() * 0.5f);
        float cb = 1.0f - (world.rand_f32() * 0.5f);
        m = Lambertian(SolidColor(V4{cr, cg, cb, 1.0f}));
      } else if (k % 3 == 1) {
        float cr = world.rand_f32(), cg = world.rand_f32(), cb = world.rand_f32();
        m = Metal(0.3f, SolidColor(V4{cr, cg, cb, 1.0f}));
      } else {
        m = Dielectric(1.5f);
      }
      float yaw = world.rand_f32();
      world.add(cube.instance(V3{(float)x * 3.0f, 1.0f, (float)z * 3.0f}, V3{0, yaw, 0}, fill3(1.0f)).with_material(m));
    }
  }
  world.add(Sphere(DiffuseLight(V3{4, 4, 5} * 10.0f), V3{10000, 4000, 4800}, 1500));
  V3 look_from{6, 8, 5}, look_at{0, 0, 0};
  r.camera = Camera::make(40.0f, look_from, look_at, V3{0, 1, 0}, aspect, 0.0f, length(look_from - look_at));
  return r;
}

// Shared frame of the synthetic-mesh scenes: ground cube, two thin
// DiffuseLight(8) cube instances (cornell.rs:65-72 pattern), camera.
void mesh_frame(World& world, Model& cube, bool lights) {
  Material white = Lambertian(SolidColor(V4{1, 1, 1, 1}));
  world.add(cube.instance(V3{0, -1001, 0}, V3{0, 0, 0}, fill3(1000)).with_material(white));
  if (lights) {
    Material light = DiffuseLight(fill3(8.0f));
    world.add(cube.instance(V3{-2.5f, 4.0f, 0.0f}, V3{0, 0, 0}, V3{1.0f, 0.0001f, 1.0f}).with_material(light));
    world.add(cube.instance(V3{2.5f, 4.0f, 1.0f}, V3{0, 0, 0}, V3{1.0f, 0.0001f, 1.0f}).with_material(light));
  }
}

Camera mesh_camera(float aspect) {
  V3 look_from{0.0f, 3.2f, 6.5f}, look_at{0.0f, -0.2f, 0.0f};
  return Camera::make(40.0f, look_from, look_at, V3{0, 1, 0}, aspect, 0.0f, length(look_from - look_at));
}

SceneResult mesh_ply(float aspect, const std::string& assets, uint64_t seed) {
  SceneResult r;
  r.world = std::make_unique<World>(SolidBackground(V3{0, 0, 0}), seed);
  World& world = *r.world;
  Model cube = world.model(ply_triangles(join_path(assets, "cube.ply")));
  Model mesh = world.model_with_material(Lambertian(SolidColor(V4{0.8f, 0.6f, 0.4f, 1.0f})),
                                         ply_triangles(join_path(assets, "mesh_1m.ply")));
  world.add(mesh);
  mesh_frame(world, cube, true);
  r.camera = mesh_camera(aspect);
  return r;
}

SceneResult mesh_obj(float aspect, const std::string& assets, uint64_t seed, bool textured) {
  SceneResult r;
  Background bg = SolidBackground(V3{0, 0, 0});
  SharedTexture albedo;
  if (textured) {
    bg = SkySphere(TextureSurface(Texture::load_png(join_path(assets, "env_4096x2048.png"), WrapMode::Repeat)));
    albedo = Texture::load_png(join_path(assets, "albedo_2048.png"), WrapMode::Repeat);
  }
  r.world = std::make_unique<World>(bg, seed);
  World& world = *r.world;
  Model cube = world.model(ply_triangles(join_path(assets, "cube.ply")));
  Material mat = textured ? Lambertian(TextureSurface(albedo)) : Lambertian(SolidColor(V4{0.8f, 0.6f, 0.4f, 1.0f}));
  ObjResult obj = load_obj(join_path(assets, "mesh_1m.obj"));
  std::vector<Triangle> tris;
  tris.reserve(obj.faces.size());
  for (const ObjFace& f : obj.faces)  // obj_fns(V3::new, V3::new, V2::new, with_norms_and_uvs)
    tris.push_back(Triangle::with_norms_and_uvs(mat, f.c[0].v, f.c[0].n, f.c[0].uv, f.c[1].v, f.c[1].n, f.c[1].uv,
                                                f.c[2].v, f.c[2].n, f.c[2].uv));
  Model mesh = world.model(std::move(tris));
  world.add(mesh);
  mesh_frame(world, cube, !textured);
  r.camera = mesh_camera(aspect);
  return r;
}

// eve::environment (eve.rs:342-364): a CubeMap whose faces are
// TextureBlend(Addition, stars, YCbCrTexture(luma, chroma)); the stars tile is
// one shared texture. The PNGs are tools/gen_assets.py stand-ins.
Background environment(const std::string& assets, const std::string& name, V3 rotation) {
  SharedTexture stars = Texture::load_png(join_path(assets, "environments/stars01_tile2.png"), WrapMode::Repeat);
  Surface faces[6];
  for (int i = 0; i < 6; ++i) {
    std::string base = join_path(assets, "environments/" + name + "/" + std::to_string(i));
    Surface nebula = YCbCrTexture(Texture::load_png(base + ".png", WrapMode::Repeat),
                                  Texture::load_png(base + "_chroma.png", WrapMode::Repeat));
    faces[i] = TextureBlend(MRT_BLEND_ADDITION, TextureSurface(stars), nebula);
  }
  return CubeMap(faces, rotation);
}

// menger.rs:117-138
const int MENGER_CUBE_SIDES[20][3] = {{0, 1, 1},   {1, 0, 1},   {1, 1, 0},  {0, -1, -1}, {-1, 0, -1},
                                      {-1, -1, 0}, {0, -1, 1},  {-1, 0, 1}, {-1, 1, 0},  {0, 1, -1},
                                      {1, 0, -1},  {1, -1, 0},  {-1, -1, 1}, {-1, 1, -1}, {1, -1, -1},
                                      {-1, 1, 1},  {1, -1, 1},  {1, 1, -1},  {1, 1, 1},   {-1, -1, -1}};

// menger_gen (menger.rs:69-115): the five nested loops, level k offset by
// sides * dims * 3^k (f32: (V3 * dims) * powi), innermost added last.
void menger_gen(World& world, const std::string& assets, int levels) {
  const float dims = 2.0f;
  Material material = Lambertian(SolidColor(V4{1, 1, 1, 1}));
  Model cube = world.model(ply_triangles(join_path(assets, "cube.ply")));
  float pw[5] = {1.0f, 3.0f, 9.0f, 27.0f, 81.0f};  // (3.0f32).powi(k), exact
  std::function<void(int, V3)> level = [&](int k, V3 base) {
    for (const auto& s : MENGER_CUBE_SIDES) {
      V3 xyz = ((V3{(float)s[0], (float)s[1], (float)s[2]} * dims) * pw[k]) + base;
      if (k == 0)
        world.add(cube.instance(xyz, V3{0, 0, 0}, fill3(1.0f)).with_material(material));
      else
        level(k - 1, xyz);
    }
  };
  // the outermost loop has no `+ xyz`; adding V3 zero is exact
  level(levels - 1, V3{0, 0, 0});
}

SceneResult menger(float aspect, const std::string& assets, uint64_t seed, int levels) {
  SceneResult r;
  r.world = std::make_unique<World>(environment(assets, "j02", V3{0.4f, 0.2f, 0.1f}), seed);
  World& world = *r.world;
  Model cube = world.model(ply_triangles(join_path(assets, "cube.ply")));
  Material foggy = Metal(0.7f, SolidColor(V4{0.5f, 0.5f, 0.5f, 1.0f}));
  menger_gen(world, assets, levels);
  world.add(cube.instance(V3{0, -244, 0}, V3{0, 0, 0}, V3{500000, 1, 500000}).with_material(foggy));
  V3 look_from{2680, 140, 2000}, look_at{0, 0, 0};
  r.camera = Camera::make(15.0f, look_from, look_at, V3{0, 1, 0}, aspect, 0.0f, length(look_from - look_at));
  return r;
}

}  // namespace

SceneResult generate_builtin(const std::string& name, float aspect, const std::string& assets, uint64_t seed,
                             const TreeBuilder* top_level) {
  SceneResult r;
  if (name == "sphere_grid")
    r = sphere_grid(aspect, assets, seed);
  else if (name == "cornell")
    r = cornell(aspect, assets, seed);
  else if (name == "cube_field")
    r = cube_field(aspect, assets, seed);
  else if (name == "mesh_ply")
    r = mesh_ply(aspect, assets, seed);
  else if (name == "mesh_obj")
    r = mesh_obj(aspect, assets, seed, false);
  else if (name == "mesh_obj_textured")
    r = mesh_obj(aspect, assets, seed, true);
  else if (name == "menger")
    r = menger(aspect, assets, seed, 5);
  else if (name == "menger_l3")
    r = menger(aspect, assets, seed, 3);
  else
    throw Error(MRT_ERR_INVALID, "unknown built-in scene '" + name + "'");
  if (top_level)
    r.world->build_bvh(*top_level);  // the same tree, built on the device (build.hip)
  else
    r.world->build_bvh();  // main.rs:112
  return r;
}

}  // namespace massrt
