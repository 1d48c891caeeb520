// world.h — C++ host mirror of the reference's scene-building surface.
//
// The reference (Rust) builds scenes through these types; this header keeps
// their names, constructor arguments and RNG consumption so the scenes of
// scenes.rs can be written against it unchanged in spirit:
//   Scene trait            scenes.rs:25-33
//   World::{new,add,build_bvh}  world.rs:95-122
//   Camera::new            world.rs:15-51
//   Sphere::new            geom.rs:46-54
//   BvhNode::new           geom.rs:109-161 (random axis, stable sort, median)
//   Model::{new,with_material,instance}  geom.rs:275-315
//   Instance::{new,with_material}        geom.rs:343-401
//   Triangle::{new,with_norms_and_uvs}   geom.rs:448-496
//   Lambertian/Metal/Dielectric/DiffuseLight/() material.rs:192-329,385-389
//   SolidBackground/SkyBackground/SkySphere     material.rs:39-89
//   SolidColor/Texture/WrapMode                 texture.rs:19-194,270-300
//
// Unlike the reference, objects are not heap-allocated `Box<dyn Intersect>`:
// the world stores typed arrays and the BVH is built over lightweight
// {reference, bounding box} items, producing the mrt_node tree that the
// C ABI (include/massrt.h) consumes. Intersection itself happens on the GPU.
#pragma once
#include <array>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../../include/massrt.h"
#include "../mrt_math.h"
#include "../mrt_rng.h"

namespace massrt {

using mrt::M4;
using mrt::V2;
using mrt::V3;
using mrt::V4;

using mrt::host_cosf;
using mrt::host_sinf;
using mrt::host_tanf;

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// ---- textures / surfaces ------------------------------------------------
enum class WrapMode : uint32_t { Mirror = MRT_WRAP_MIRROR, Repeat = MRT_WRAP_REPEAT, Clamp = MRT_WRAP_CLAMP };

struct Texture {  // texture.rs:21-27 (RGBA8 kept; decoded c/255.0 on use)
  uint32_t width = 0, height = 0;
  WrapMode wrapping = WrapMode::Repeat;
  std::vector<uint8_t> rgba;
  static std::shared_ptr<Texture> load_png(const std::string& path, WrapMode wrapping);  // texture.rs:30-69
  static std::shared_ptr<Texture> load_bytes(const uint8_t* bytes, uint32_t w, uint32_t h,
                                             WrapMode wrapping);  // texture.rs:71-102
};
using SharedTexture = std::shared_ptr<Texture>;

// SolidColor(V4), a shared Texture, or a composite over them (texture.rs:197-357)
struct Surface {
  uint32_t kind = MRT_SURF_SOLID;
  V4 color{1, 1, 1, 1};    // SolidColor / SolidColorFallback colour
  SharedTexture texture;   // Texture, YCbCr luma
  SharedTexture chroma;    // YCbCr chroma
  uint32_t mode = 0;       // TextureBlend mode
  std::shared_ptr<const Surface> left, right;  // TextureBlend operands; Fallback's surface in `left`
};
inline Surface SolidColor(V4 c) {
  Surface s;
  s.kind = MRT_SURF_SOLID;
  s.color = c;
  return s;
}
inline Surface TextureSurface(SharedTexture t) {
  Surface s;
  s.kind = MRT_SURF_TEXTURE;
  s.texture = std::move(t);
  return s;
}

inline Surface YCbCrTexture(SharedTexture luma, SharedTexture chroma) {  // texture.rs:212-223
  Surface s;
  s.kind = MRT_SURF_YCBCR;
  s.texture = std::move(luma);
  s.chroma = std::move(chroma);
  return s;
}
inline Surface TextureBlend(uint32_t mode, Surface l, Surface r) {  // texture.rs:309-317
  Surface s;
  s.kind = MRT_SURF_BLEND;
  s.mode = mode;
  s.left = std::make_shared<const Surface>(std::move(l));
  s.right = std::make_shared<const Surface>(std::move(r));
  return s;
}
inline Surface SolidColorFallback(V4 color, Surface inner) {  // texture.rs:341-345
  Surface s;
  s.kind = MRT_SURF_FALLBACK;
  s.color = color;
  s.left = std::make_shared<const Surface>(std::move(inner));
  return s;
}

// ---- materials (value types, like the Rust generics) ---------------------
struct Material {
  uint32_t kind = MRT_MAT_NONE;
  Surface surface;
  float param = 0.0f;
  V3 emit{0, 0, 0};                             // DiffuseLight emission / Isotrophic albedo
  std::shared_ptr<const Material> left, right;  // Mix
};
inline Material NoMaterial() { return Material{}; }  // impl Material for ()
inline Material Lambertian(Surface s) {
  Material m;
  m.kind = MRT_MAT_LAMBERTIAN;
  m.surface = std::move(s);
  return m;
}
inline Material Metal(float fuzz, Surface s) {  // material.rs:255-258
  Material m;
  m.kind = MRT_MAT_METAL;
  m.param = fuzz < 1.0f ? fuzz : 1.0f;
  m.surface = std::move(s);
  return m;
}
inline Material Dielectric(float refraction_index) {
  Material m;
  m.kind = MRT_MAT_DIELECTRIC;
  m.param = refraction_index;
  return m;
}
inline Material Specular(float refraction_index, Surface s) {  // material.rs:338-345
  Material m;
  m.kind = MRT_MAT_SPECULAR;
  m.param = refraction_index;
  m.surface = std::move(s);
  return m;
}
inline Material Isotrophic(V3 albedo) {  // material.rs:432-436
  Material m;
  m.kind = MRT_MAT_ISOTROPHIC;
  m.emit = albedo;
  return m;
}
inline Material Mix(float ratio, Material l, Material r) {  // material.rs:396-400
  Material m;
  m.kind = MRT_MAT_MIX;
  m.param = ratio;
  m.left = std::make_shared<const Material>(std::move(l));
  m.right = std::make_shared<const Material>(std::move(r));
  return m;
}
inline Material DiffuseLight(V3 emit) {
  Material m;
  m.kind = MRT_MAT_DIFFUSE_LIGHT;
  m.emit = emit;
  return m;
}

struct Background {
  uint32_t kind = MRT_BG_SOLID;
  V3 color{0, 0, 0};
  Surface surface;
  Surface faces[6];  // CubeMap x_pos, x_neg, y_pos, y_neg, z_pos, z_neg
  M4 transform{};    // CubeMap direction transform
};
inline Background SolidBackground(V3 c) {
  Background b;
  b.kind = MRT_BG_SOLID;
  b.color = c;
  return b;
}
inline Background SkyBackground() {
  Background b;
  b.kind = MRT_BG_SKY;
  return b;
}
inline Background SkySphere(Surface s) {
  Background b;
  b.kind = MRT_BG_SKYSPHERE;
  b.surface = std::move(s);
  return b;
}

// CubeMap::new (material.rs:102-118): note the reference builds all three
// factors with rotate_x.
inline Background CubeMap(const Surface faces[6], V3 rotation) {
  Background b;
  b.kind = MRT_BG_CUBEMAP;
  for (int k = 0; k < 6; ++k) b.faces[k] = faces[k];
  b.transform = mrt::m4_mul(mrt::m4_mul(mrt::m4_rotate_x(rotation.x), mrt::m4_rotate_x(rotation.y)),
                            mrt::m4_rotate_x(rotation.z));
  return b;
}

// ---- geometry -------------------------------------------------------------
struct BoundingBox {  // geom.rs:207-273
  V3 minimum, maximum;
  BoundingBox join(const BoundingBox& o) const {
    return BoundingBox{mrt::vmin(minimum, o.minimum), mrt::vmax(maximum, o.maximum)};
  }
  V3 corner(int i) const {  // geom.rs:256-272 order
    return V3{(i & 1) == 0 ? maximum.x : minimum.x, (i & 2) == 0 ? maximum.y : minimum.y,
              (i & 4) == 0 ? maximum.z : minimum.z};
  }
};

struct Triangle {  // geom.rs:434-446
  V3 vertex_a, vertex_b, vertex_c;
  bool has_uv = false;
  V2 uv_a{0, 0}, uv_b{0, 0}, uv_c{0, 0};
  Material material;
  V3 normal_a, normal_b, normal_c;
  V3 tangent{0, 0, 0}, bitangent{0, 0, 0};
  static Triangle make(Material m, V3 a, V3 b, V3 c);  // Triangle::new
  static Triangle with_norms_and_uvs(Material m, V3 a, V3 na, V2 uva, V3 b, V3 nb, V2 uvb, V3 c, V3 nc,
                                     V2 uvc);
  BoundingBox bounding_box() const {  // geom.rs:587-592
    return BoundingBox{mrt::vmin(mrt::vmin(vertex_a, vertex_b), vertex_c),
                       mrt::vmax(mrt::vmax(vertex_a, vertex_b), vertex_c)};
  }
};

class World;

// An item of a BvhNode: a reference into the world's arrays + its box.
struct Item {
  uint32_t ref;
  BoundingBox box;
};

struct InstanceDesc {  // Instance<M> (geom.rs:335-341)
  uint32_t blas_root = 0;
  M4 transform, inv_transform;
  BoundingBox box;
  bool has_material = false;
  Material material;
  InstanceDesc with_material(Material m) const {
    InstanceDesc d = *this;
    d.has_material = true;
    d.material = std::move(m);
    return d;
  }
};

// Model: a BLAS over triangles, shared by its instances (Arc<BvhNode>).
struct Model {
  World* world = nullptr;
  uint32_t blas_root = 0;  // node index
  BoundingBox box;
  bool has_material = false;
  Material material;
  uint32_t id = 0xFFFFFFFFu;  // index in world models once added/exported
  // Model::instance (geom.rs:312-314)
  InstanceDesc instance(V3 translation, V3 rotation, V3 scale) const;
};

struct SphereDesc {
  V3 center;
  float radius;
  Material material;
};
inline SphereDesc Sphere(Material m, V3 center, float radius) { return SphereDesc{center, radius, std::move(m)}; }

// Volume::new(Sphere::new((), center, radius), density, albedo) (geom.rs:594-607)
struct VolumeDesc {
  V3 center;
  float radius;
  float density;
  V3 albedo;
};

struct Camera {  // world.rs:5-51
  V3 origin, lower_left_corner, horizontal, vertical, u, v;
  float lens_radius = 0;
  static Camera make(float vertical_fov, V3 look_from, V3 look_at, V3 view_up, float aspect_ratio,
                     float aperture, float focus_distance);
  mrt_camera to_abi() const;
};

// World<B>: background + object list; owns the typed arrays behind every
// reference, including all BLAS nodes of models created against it.
// Builds the tree over a World's objects somewhere else (the device builder,
// csrc/device/build.hip): appends to `nodes` exactly what World::bvh_new
// would (preorder numbering from nodes.size(), one rng.axis() per node) and
// returns the root's box.
using TreeBuilder =
    std::function<void(const std::vector<Item>& items, mrt::WyRand& rng, std::vector<mrt_node>& nodes, BoundingBox& root_box)>;

class World {
 public:
  explicit World(Background bg, uint64_t rng_seed = 1) : background_(std::move(bg)) { rng.state = rng_seed; }

  mrt::WyRand rng;  // fastrand thread-local stream (main.rs:86 seeds it with 1)
  float rand_f32() { return rng.f32(); }

  void add(const SphereDesc& s);
  void add(const Triangle& t);
  void add(const InstanceDesc& inst);
  void add(Model& m);  // World::add(model)
  uint32_t add(const VolumeDesc& v);
  // Model::new / Model::with_material: builds the BLAS now (consumes RNG)
  Model model(std::vector<Triangle> triangles);
  Model model_with_material(Material m, std::vector<Triangle> triangles);
  void build_bvh();  // world.rs:117-122
  void build_bvh(const TreeBuilder& builder);  // the same tree, built by `builder`

  void set_background(Background bg) { background_ = std::move(bg); }
  // flatten into the C ABI description (pointers valid until modified)
  const mrt_scene_desc& desc();

  size_t n_objects() const { return objects_.size(); }
  size_t n_nodes() const { return nodes_.size(); }

 private:
  uint32_t bvh_new(std::vector<Item>& items, size_t lo, size_t hi, BoundingBox* out_box);
  uint32_t intern_material(const Material& m);
  uint32_t intern_surface(const Surface& s);
  uint32_t intern_texture(const SharedTexture& t);

  Background background_;
  std::vector<Item> objects_;
  std::vector<mrt_node> nodes_;
  std::vector<mrt_sphere> spheres_;
  std::vector<mrt_triangle> triangles_;
  std::vector<mrt_instance> instances_;
  std::vector<mrt_model> models_;
  std::vector<mrt_volume> volumes_;
  std::vector<mrt_material> materials_;
  std::vector<mrt_surface> surfaces_;
  std::vector<mrt_texture> textures_;
  std::vector<SharedTexture> texture_refs_;
  std::unordered_map<std::string, uint32_t> material_index_, surface_index_;
  std::unordered_map<const Texture*, uint32_t> texture_index_;
  std::vector<uint32_t> roots_;
  mrt_scene_desc desc_{};
};

// ---- loaders (ply_loader.rs, stl_loader.rs, obj_loader.rs) ---------------
struct ObjCorner {
  V3 v, n;
  V2 uv;
};
// PlyLoader::load(path, V3::new, face_fn) — triangles only (ply_loader.rs:396)
std::vector<std::array<V3, 3>> load_ply(const std::string& path);
// PlyLoader::load with a vertex_fn remap (e.g. Lucy's (y,z,x), lucy.rs:33-38)
std::vector<std::array<V3, 3>> load_ply(const std::string& path, const std::function<V3(float, float, float)>& vertex_fn);
std::vector<std::array<V3, 3>> load_stl_binary(const std::string& path);
// ObjLoader::load with obj_fns (identity vertex/normal/uv fns)
struct ObjFace {
  ObjCorner c[3];
  std::string material;
};
struct ObjResult {
  std::vector<ObjFace> faces;
  std::string material_library;  // resolved path ("" if none)
};
ObjResult load_obj(const std::string& path);
// PNG -> RGBA8 (image::io::Reader + to_rgba8, texture.rs:36-39)
bool decode_png(const std::string& path, std::vector<uint8_t>& rgba, uint32_t& w, uint32_t& h, std::string& err);

// ---- scenes -----------------------------------------------------------------
struct SceneResult {
  std::unique_ptr<World> world;
  Camera camera;
};
// Scene::generate + World::build_bvh for a built-in scene.
SceneResult generate_builtin(const std::string& name, float aspect_ratio, const std::string& asset_dir,
                             uint64_t seed, const TreeBuilder* top_level = nullptr);

}  // namespace massrt
