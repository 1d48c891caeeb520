// world.cpp — host scene construction: Triangle/Camera/Instance constructors,
// the reference-topology BVH builder and flattening to mrt_scene_desc.
#include "world.h"

#include <math.h>
#include <string.h>

#include <algorithm>

namespace mrt {
__attribute__((noinline)) float host_sinf(float x) { return sinf(x); }
__attribute__((noinline)) float host_cosf(float x) { return cosf(x); }
__attribute__((noinline)) float host_tanf(float x) { return tanf(x); }
}  // namespace mrt

namespace massrt {

using namespace mrt;

// Triangle::new (geom.rs:449-466): flat normal unit(ab x ac) on all corners.
Triangle Triangle::make(Material m, V3 a, V3 b, V3 c) {
  Triangle t;
  V3 ab = b - a, ac = c - a;
  V3 n = unit(cross(ab, ac));
  t.vertex_a = a;
  t.vertex_b = b;
  t.vertex_c = c;
  t.material = std::move(m);
  t.normal_a = t.normal_b = t.normal_c = n;
  return t;
}

// Triangle::with_norms_and_uvs (geom.rs:468-496).
Triangle Triangle::with_norms_and_uvs(Material m, V3 a, V3 na, V2 uva, V3 b, V3 nb, V2 uvb, V3 c, V3 nc,
                                      V2 uvc) {
  Triangle t;
  V3 ab = b - a, ac = c - a;
  V2 uv_ab = uvb - uva, uv_ac = uvc - uva;
  float r = fmaxf(fminf(1.0f / (uv_ab.x * uv_ac.y - uv_ab.y * uv_ac.x), 1.0f), -1.0f);
  t.tangent = (ab * uv_ac.y - ac * uv_ab.y) * r;
  t.bitangent = (ac * uv_ab.x - ab * uv_ac.x) * r;
  t.vertex_a = a;
  t.vertex_b = b;
  t.vertex_c = c;
  t.has_uv = true;
  t.uv_a = uva;
  t.uv_b = uvb;
  t.uv_c = uvc;
  t.material = std::move(m);
  t.normal_a = na;
  t.normal_b = nb;
  t.normal_c = nc;
  return t;
}

// Camera::new (world.rs:16-51).
Camera Camera::make(float vertical_fov, V3 look_from, V3 look_at, V3 view_up, float aspect_ratio, float aperture,
                    float focus_distance) {
  float vertical_fov_rads = vertical_fov * kPi / 180.0f;
  float half_height = host_tanf(vertical_fov_rads / 2.0f);
  float viewport_height = half_height * 2.0f;
  float viewport_width = aspect_ratio * viewport_height;
  V3 w = unit(look_from - look_at);
  V3 u = unit(cross(view_up, w));
  V3 v = cross(w, u);
  Camera cam;
  cam.origin = look_from;
  cam.horizontal = (u * viewport_width) * focus_distance;
  cam.vertical = (v * viewport_height) * focus_distance;
  cam.lower_left_corner = ((cam.origin - (cam.horizontal / 2.0f)) - (cam.vertical / 2.0f)) - (w * focus_distance);
  cam.u = u;
  cam.v = v;
  cam.lens_radius = aperture / 2.0f;
  return cam;
}

mrt_camera Camera::to_abi() const {
  mrt_camera c;
  auto put = [](float* d, V3 s) {
    d[0] = s.x;
    d[1] = s.y;
    d[2] = s.z;
  };
  put(c.origin, origin);
  put(c.lower_left_corner, lower_left_corner);
  put(c.horizontal, horizontal);
  put(c.vertical, vertical);
  put(c.u, u);
  put(c.v, v);
  c.lens_radius = lens_radius;
  return c;
}

// Instance::new (geom.rs:344-390).
InstanceDesc Model::instance(V3 translation, V3 rotation, V3 scale) const {
  V3 inv_translation_v = translation * -1.0f;
  V3 inv_rotation_v = rotation * -1.0f;
  V3 inv_scale_v = sdiv(1.0f, scale);
  M4 t = m4_translation(translation), it = m4_translation(inv_translation_v);
  M4 rx = m4_rotate_x(rotation.x), ry = m4_rotate_y(rotation.y), rz = m4_rotate_z(rotation.z);
  M4 irx = m4_rotate_x(inv_rotation_v.x), iry = m4_rotate_y(inv_rotation_v.y), irz = m4_rotate_z(inv_rotation_v.z);
  M4 rot = m4_mul(m4_mul(rx, ry), rz);
  M4 inv_rot = m4_mul(m4_mul(irz, iry), irx);
  M4 s = m4_scale(scale), is = m4_scale(inv_scale_v);
  InstanceDesc d;
  d.blas_root = blas_root;
  d.transform = m4_mul(m4_mul(t, rot), s);
  d.inv_transform = m4_mul(m4_mul(is, inv_rot), it);
  V3 mn = fill3(INFINITY), mx = fill3(-INFINITY);
  for (int i = 0; i < 8; ++i) {
    V3 c = transform_point(d.transform, box.corner(i));
    mn = vmin(mn, c);
    mx = vmax(mx, c);
  }
  d.box = BoundingBox{mn, mx};
  return d;
}

static void put3(float* d, V3 s) {
  d[0] = s.x;
  d[1] = s.y;
  d[2] = s.z;
}
static void put_m4(float* d, const M4& m) {
  const V4* cols[4] = {&m.c0, &m.c1, &m.c2, &m.c3};
  for (int i = 0; i < 4; ++i) {
    d[4 * i + 0] = cols[i]->x;
    d[4 * i + 1] = cols[i]->y;
    d[4 * i + 2] = cols[i]->z;
    d[4 * i + 3] = cols[i]->w;
  }
}

uint32_t World::intern_texture(const SharedTexture& t) {
  auto it = texture_index_.find(t.get());
  if (it != texture_index_.end()) return it->second;
  uint32_t idx = (uint32_t)textures_.size();
  mrt_texture d;
  d.width = t->width;
  d.height = t->height;
  d.wrap = (uint32_t)t->wrapping;
  d.rgba = t->rgba.data();
  textures_.push_back(d);
  texture_refs_.push_back(t);
  texture_index_[t.get()] = idx;
  return idx;
}

uint32_t World::intern_surface(const Surface& s) {
  mrt_surface d{};
  d.kind = s.kind;
  switch (s.kind) {  // operands first: their indices are lower than this one's
    case MRT_SURF_TEXTURE:
      d.texture = intern_texture(s.texture);
      break;
    case MRT_SURF_YCBCR:
      d.texture = intern_texture(s.texture);
      d.a = intern_texture(s.chroma);
      break;
    case MRT_SURF_BLEND:
      d.mode = s.mode;
      d.a = intern_surface(*s.left);
      d.b = intern_surface(*s.right);
      break;
    case MRT_SURF_FALLBACK:
      d.a = intern_surface(*s.left);
      break;
  }
  d.color[0] = s.color.x;
  d.color[1] = s.color.y;
  d.color[2] = s.color.z;
  d.color[3] = s.color.w;
  std::string key((const char*)&d, sizeof(d));
  auto it = surface_index_.find(key);
  if (it != surface_index_.end()) return it->second;
  uint32_t idx = (uint32_t)surfaces_.size();
  surfaces_.push_back(d);
  surface_index_[key] = idx;
  return idx;
}

uint32_t World::intern_material(const Material& m) {
  mrt_material d{};
  d.kind = m.kind;
  d.surface = (m.kind == MRT_MAT_LAMBERTIAN || m.kind == MRT_MAT_METAL || m.kind == MRT_MAT_SPECULAR)
                  ? intern_surface(m.surface)
                  : 0;
  d.param = m.param;
  put3(d.emit, m.emit);
  if (m.kind == MRT_MAT_MIX) {  // children first: their indices are lower than this one's
    d.left = intern_material(*m.left);
    d.right = intern_material(*m.right);
  }
  std::string key((const char*)&d, sizeof(d));
  auto it = material_index_.find(key);
  if (it != material_index_.end()) return it->second;
  uint32_t idx = (uint32_t)materials_.size();
  materials_.push_back(d);
  material_index_[key] = idx;
  return idx;
}

static float axis_key(const Item& it, uint32_t axis) {
  return axis == 0 ? it.box.minimum.x : (axis == 1 ? it.box.minimum.y : it.box.minimum.z);
}

// BvhNode::new (geom.rs:110-161). One axis draw per call — including 1- and
// 2-item calls — before recursing into the left half first.
uint32_t World::bvh_new(std::vector<Item>& items, size_t lo, size_t hi, BoundingBox* out_box) {
  const size_t n = hi - lo;
  if (n == 0) throw Error(MRT_ERR_INVALID, "BvhNode::new over an empty item list (the reference recurses forever)");
  uint32_t axis = rng.axis();
  uint32_t idx = (uint32_t)nodes_.size();
  nodes_.push_back(mrt_node{});
  uint32_t left = MRT_REF(MRT_REF_NONE, 0), right = MRT_REF(MRT_REF_NONE, 0);
  BoundingBox lb{}, rb{};
  bool has_right = false;
  if (n == 1) {
    left = items[lo].ref;
    lb = items[lo].box;
  } else if (n == 2) {
    // a = items.pop() (the last), b = items.pop() (the first)
    const Item& a = items[lo + 1];
    const Item& b = items[lo];
    if (axis_key(a, axis) < axis_key(b, axis)) {
      left = a.ref, lb = a.box, right = b.ref, rb = b.box;
    } else {
      left = b.ref, lb = b.box, right = a.ref, rb = a.box;
    }
    has_right = true;
  } else {
    // sort_by with is_less = key(a) < key(b): stable; only is_less matters
    std::stable_sort(items.begin() + lo, items.begin() + hi,
                     [axis](const Item& x, const Item& y) { return axis_key(x, axis) < axis_key(y, axis); });
    size_t mid = lo + n / 2;
    uint32_t l = bvh_new(items, lo, mid, &lb);
    uint32_t r = bvh_new(items, mid, hi, &rb);
    left = MRT_REF(MRT_REF_NODE, l);
    right = MRT_REF(MRT_REF_NODE, r);
    has_right = true;
  }
  BoundingBox box = has_right ? lb.join(rb) : lb;
  mrt_node& nd = nodes_[idx];
  put3(nd.min, box.minimum);
  put3(nd.max, box.maximum);
  nd.left = left;
  nd.right = right;
  *out_box = box;
  return idx;
}

void World::add(const SphereDesc& s) {
  uint32_t idx = (uint32_t)spheres_.size();
  mrt_sphere d;
  put3(d.center, s.center);
  d.radius = s.radius;
  d.material = intern_material(s.material);
  spheres_.push_back(d);
  float r = fabsf(s.radius);  // geom.rs:95-100
  objects_.push_back(Item{MRT_REF(MRT_REF_SPHERE, idx), BoundingBox{s.center - fill3(r), s.center + fill3(r)}});
}

uint32_t World::add(const VolumeDesc& v) {
  uint32_t idx = (uint32_t)volumes_.size();
  mrt_volume d;
  put3(d.center, v.center);
  d.radius = v.radius;
  d.density = v.density;
  d.material = intern_material(Isotrophic(v.albedo));
  volumes_.push_back(d);
  float r = fabsf(v.radius);  // Volume::bounding_box = the target's (geom.rs:656-658)
  objects_.push_back(Item{MRT_REF(MRT_REF_VOLUME, idx), BoundingBox{v.center - fill3(r), v.center + fill3(r)}});
  return idx;
}

static mrt_triangle to_abi(const Triangle& t, uint32_t material) {
  mrt_triangle d{};
  put3(d.a, t.vertex_a);
  put3(d.b, t.vertex_b);
  put3(d.c, t.vertex_c);
  put3(d.na, t.normal_a);
  put3(d.nb, t.normal_b);
  put3(d.nc, t.normal_c);
  d.uva[0] = t.uv_a.x, d.uva[1] = t.uv_a.y;
  d.uvb[0] = t.uv_b.x, d.uvb[1] = t.uv_b.y;
  d.uvc[0] = t.uv_c.x, d.uvc[1] = t.uv_c.y;
  put3(d.tangent, t.tangent);
  put3(d.bitangent, t.bitangent);
  d.material = material;
  d.flags = t.has_uv ? MRT_TRI_HAS_UV : 0;
  return d;
}

void World::add(const Triangle& t) {
  uint32_t idx = (uint32_t)triangles_.size();
  triangles_.push_back(to_abi(t, intern_material(t.material)));
  objects_.push_back(Item{MRT_REF(MRT_REF_TRIANGLE, idx), t.bounding_box()});
}

void World::add(const InstanceDesc& inst) {
  uint32_t idx = (uint32_t)instances_.size();
  mrt_instance d{};
  put_m4(d.fwd, inst.transform);
  put_m4(d.inv, inst.inv_transform);
  d.blas_root = inst.blas_root;
  d.material = inst.has_material ? intern_material(inst.material) : MRT_NO_MATERIAL;
  instances_.push_back(d);
  objects_.push_back(Item{MRT_REF(MRT_REF_INSTANCE, idx), inst.box});
}

void World::add(Model& m) {
  uint32_t idx = (uint32_t)models_.size();
  mrt_model d{};
  d.blas_root = m.blas_root;
  d.material = m.has_material ? intern_material(m.material) : MRT_NO_MATERIAL;
  models_.push_back(d);
  m.id = idx;
  objects_.push_back(Item{MRT_REF(MRT_REF_MODEL, idx), m.box});
}

Model World::model(std::vector<Triangle> triangles) {
  if (triangles.empty()) throw Error(MRT_ERR_INVALID, "Model::new with no triangles");
  std::vector<Item> items;
  items.reserve(triangles.size());
  for (const Triangle& t : triangles) {
    uint32_t idx = (uint32_t)triangles_.size();
    triangles_.push_back(to_abi(t, intern_material(t.material)));
    items.push_back(Item{MRT_REF(MRT_REF_TRIANGLE, idx), t.bounding_box()});
  }
  Model m;
  m.world = this;
  m.blas_root = bvh_new(items, 0, items.size(), &m.box);
  return m;
}

Model World::model_with_material(Material mat, std::vector<Triangle> triangles) {
  Model m = model(std::move(triangles));
  m.has_material = true;
  m.material = std::move(mat);
  return m;
}

// World::build_bvh (world.rs:117-122): every object under one BvhNode.
void World::build_bvh() {
  std::vector<Item> items = std::move(objects_);
  objects_.clear();
  BoundingBox box;
  uint32_t root = bvh_new(items, 0, items.size(), &box);
  objects_.push_back(Item{MRT_REF(MRT_REF_NODE, root), box});
}

void World::build_bvh(const TreeBuilder& builder) {
  std::vector<Item> items = std::move(objects_);
  objects_.clear();
  const uint32_t root = (uint32_t)nodes_.size();
  const mrt::WyRand saved_rng = rng;  // the builder draws every axis before its device work can fail
  BoundingBox box;
  try {
    builder(items, rng, nodes_, box);
  } catch (...) {
    // the world is unchanged by a failed build: objects, nodes and the scene
    // stream (so a host build after it draws the reference's axes)
    objects_ = std::move(items);
    nodes_.resize(root);
    rng = saved_rng;
    throw;
  }
  objects_.push_back(Item{MRT_REF(MRT_REF_NODE, root), box});
}

const mrt_scene_desc& World::desc() {
  roots_.clear();
  for (const Item& it : objects_) roots_.push_back(it.ref);
  mrt_background bg{};
  bg.kind = background_.kind;
  put3(bg.color, background_.color);
  bg.surface = background_.kind == MRT_BG_SKYSPHERE ? intern_surface(background_.surface) : 0;
  if (background_.kind == MRT_BG_CUBEMAP) {
    for (int k = 0; k < 6; ++k) bg.faces[k] = intern_surface(background_.faces[k]);
    const M4& m = background_.transform;
    const V4 cols[4] = {m.c0, m.c1, m.c2, m.c3};
    for (int c = 0; c < 4; ++c) {
      bg.transform[4 * c + 0] = cols[c].x, bg.transform[4 * c + 1] = cols[c].y;
      bg.transform[4 * c + 2] = cols[c].z, bg.transform[4 * c + 3] = cols[c].w;
    }
  }
  desc_.nodes = nodes_.data();
  desc_.n_nodes = (uint32_t)nodes_.size();
  desc_.roots = roots_.data();
  desc_.n_roots = (uint32_t)roots_.size();
  desc_.spheres = spheres_.data();
  desc_.n_spheres = (uint32_t)spheres_.size();
  desc_.triangles = triangles_.data();
  desc_.n_triangles = (uint32_t)triangles_.size();
  desc_.instances = instances_.data();
  desc_.n_instances = (uint32_t)instances_.size();
  desc_.models = models_.data();
  desc_.n_models = (uint32_t)models_.size();
  desc_.materials = materials_.data();
  desc_.n_materials = (uint32_t)materials_.size();
  desc_.surfaces = surfaces_.data();
  desc_.n_surfaces = (uint32_t)surfaces_.size();
  desc_.textures = textures_.data();
  desc_.n_textures = (uint32_t)textures_.size();
  desc_.background = bg;
  desc_.volumes = volumes_.data();
  desc_.n_volumes = (uint32_t)volumes_.size();
  return desc_;
}

}  // namespace massrt
