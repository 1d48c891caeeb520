// upload.cpp — linearise the reference BVH into the preorder slot stream.
#include "upload.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <queue>
#include <stdexcept>
#include <unordered_map>

namespace mrt {

namespace {

uint32_t fbits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

// Surfaces -> GpuSurfRef; composites become postfix programs (layout.h).
struct SurfResolver {
  const mrt_scene_desc& d;
  HostScene& s;
  std::string& err;
  std::unordered_map<uint32_t, GpuSurfRef> memo;
  std::vector<int8_t> tex_zero_alpha;  // per texture: some texel has alpha 0 (-1 = not yet scanned)
  static constexpr uint32_t kMaxOps = 256;

  bool fail(const char* m) {
    err = m;
    return false;
  }
  // Appends surface i's program; `depth` = operand stack slots it needs.
  bool emit(uint32_t i, uint32_t& depth) {
    const mrt_surface& sf = d.surfaces[i];
    GpuSurfOp op{};
    op.op = sf.kind;
    for (int k = 0; k < 4; ++k) op.color[k] = sf.color[k];
    switch (sf.kind) {
      case MRT_SURF_SOLID:
        depth = 1;
        break;
      case MRT_SURF_TEXTURE:
        if (sf.texture >= d.n_textures) return fail("surface texture out of range");
        op.tex = sf.texture;
        depth = 1;
        break;
      case MRT_SURF_YCBCR: {
        if (sf.texture >= d.n_textures || sf.a >= d.n_textures) return fail("YCbCr texture out of range");
        GpuSurfOp t{};
        t.op = MRT_SURF_TEXTURE;
        t.tex = sf.texture;
        s.surf_ops.push_back(t);
        t.tex = sf.a;
        s.surf_ops.push_back(t);
        depth = 2;
        break;
      }
      case MRT_SURF_BLEND: {
        if (sf.a >= i || sf.b >= i) return fail("blend operands must precede the blend in the surface table");
        if (sf.mode > MRT_BLEND_SUBTRACTION) return fail("bad blend mode");
        uint32_t dl, dr;
        if (!emit(sf.a, dl) || !emit(sf.b, dr)) return false;
        op.arg = sf.mode;
        depth = dl > dr + 1 ? dl : dr + 1;
        break;
      }
      case MRT_SURF_FALLBACK:
        if (sf.a >= i) return fail("fallback surface must precede it in the surface table");
        if (!emit(sf.a, depth)) return false;
        break;
      default:
        return fail("bad surface kind");
    }
    s.surf_ops.push_back(op);
    return true;
  }
  bool resolve(uint32_t i, GpuSurfRef& out) {
    if (i >= d.n_surfaces) return fail("surface index out of range");
    auto it = memo.find(i);
    if (it != memo.end()) return (out = it->second, true);
    const mrt_surface& sf = d.surfaces[i];
    GpuSurfRef r{};
    for (int k = 0; k < 4; ++k) r.color[k] = sf.color[k];
    if (sf.kind == MRT_SURF_SOLID || sf.kind == MRT_SURF_TEXTURE) {
      r.kind = sf.kind;
      r.index = sf.kind == MRT_SURF_TEXTURE ? sf.texture : 0;
      if (sf.kind == MRT_SURF_TEXTURE && sf.texture >= d.n_textures) return fail("surface texture out of range");
    } else {
      uint32_t start = (uint32_t)s.surf_ops.size(), depth = 0;
      if (!emit(i, depth)) return false;
      if (depth > kSurfStack) return fail("composite surface nested too deeply (operand stack > 4)");
      if (s.surf_ops.size() - start > kMaxOps) return fail("composite surface program too long");
      r.kind = SURF_PROGRAM;
      r.index = start;
      r.len = (uint32_t)s.surf_ops.size() - start;
    }
    memo[i] = r;
    out = r;
    return true;
  }
  bool texture_has_zero_alpha(uint32_t t) {
    if (t >= d.n_textures) return false;
    if (tex_zero_alpha.empty()) tex_zero_alpha.assign(d.n_textures, -1);
    int8_t& z = tex_zero_alpha[t];
    if (z < 0) {
      const mrt_texture& tx = d.textures[t];
      z = 0;
      for (size_t k = 0; k < (size_t)tx.width * tx.height; ++k)
        if (tx.rgba[4 * k + 3] == 0) {
          z = 1;
          break;
        }
    }
    return z == 1;
  }
  // Can get_f(uv).w be 0 somewhere? (conservative: true means "run the alpha test")
  bool may_zero_alpha(uint32_t i) {
    if (i >= d.n_surfaces) return false;
    const mrt_surface& sf = d.surfaces[i];
    switch (sf.kind) {
      case MRT_SURF_SOLID:
        return sf.color[3] == 0.0f;
      case MRT_SURF_TEXTURE:
        return texture_has_zero_alpha(sf.texture);
      case MRT_SURF_YCBCR:
        return false;  // alpha is 1 (texture.rs:247)
      case MRT_SURF_BLEND:
        if (sf.a >= i || sf.b >= i) return false;
        if (sf.mode == MRT_BLEND_DARKEN) return may_zero_alpha(sf.a) || may_zero_alpha(sf.b);
        if (sf.mode == MRT_BLEND_SUBTRACTION) return true;
        return may_zero_alpha(sf.a) && may_zero_alpha(sf.b);  // max / min(l+r, 1) of non-negative alphas
      default:
        return true;
    }
  }
};

struct Emitter {
  const mrt_scene_desc& d;
  HostScene& s;
  std::string& err;
  // instance/model records whose BLAS range is patched after the BLAS regions
  std::vector<std::pair<uint32_t, uint32_t>> jump_patches;  // (slot index, blas root node)

  uint32_t n_slots() const { return (uint32_t)(s.slots.size() / 4); }
  uint32_t push_slot(uint32_t a, uint32_t b, uint32_t c, uint32_t w) {
    uint32_t i = n_slots();
    s.slots.push_back(a), s.slots.push_back(b), s.slots.push_back(c), s.slots.push_back(w);
    return i;
  }

  // END record closing a region (world or BLAS): a box skip or the last
  // primitive of the region lands on it, so the device never compares the
  // record index against the region's end.
  void push_end() {
    s.rec_starts.push_back(n_slots());
    push_slot(0, 0, 0, 0);
    push_slot(0, 0, 0, KIND_END);
  }

  bool emit_prim(uint32_t ref, bool in_blas) {
    uint32_t kind = MRT_REF_KIND(ref), idx = MRT_REF_INDEX(ref);
    s.rec_starts.push_back(n_slots());  // (a failed emission aborts the whole build)
    switch (kind) {
      case MRT_REF_SPHERE: {
        if (idx >= d.n_spheres) return fail("sphere index out of range");
        const mrt_sphere& sp = d.spheres[idx];
        const uint32_t at = push_slot(fbits(sp.center[0]), fbits(sp.center[1]), fbits(sp.center[2]), fbits(sp.radius));
        push_slot(idx, at + 2, 0, KIND_SPHERE);  // next: the following record
        s.n_prim_records++;
        return true;
      }
      case MRT_REF_TRIANGLE: {
        if (idx >= d.n_triangles) return fail("triangle index out of range");
        const mrt_triangle& t = d.triangles[idx];
        float ab[3], ac[3];
        for (int k = 0; k < 3; ++k) ab[k] = t.b[k] - t.a[k], ac[k] = t.c[k] - t.a[k];
        if (idx > kTriIdMask) return fail("triangle index too large");
        uint32_t id = idx;
        if (needs_alpha(t)) {
          id |= kTriAlpha;
          s.has_alpha = true;
        }
        const uint32_t at = push_slot(fbits(t.a[0]), fbits(t.a[1]), fbits(t.a[2]), fbits(ab[0]));
        push_slot(fbits(ab[1]), fbits(ab[2]), id, KIND_TRI);
        push_slot(fbits(ac[0]), fbits(ac[1]), fbits(ac[2]), at + 3);  // next: the following record
        s.n_prim_records++;
        return true;
      }
      case MRT_REF_VOLUME: {
        if (idx >= d.n_volumes) return fail("volume index out of range");
        if (in_blas) return fail("a Volume must be a World object (not inside a model)");
        const mrt_volume& v = d.volumes[idx];
        const uint32_t at = push_slot(fbits(v.center[0]), fbits(v.center[1]), fbits(v.center[2]), fbits(v.radius));
        push_slot(idx, at + 2, 0, KIND_VOLUME);
        s.n_prim_records++;
        s.trav_rng = true;
        return true;
      }
      case MRT_REF_INSTANCE:
      case MRT_REF_MODEL: {
        if (in_blas) return fail("instances/models cannot be nested inside a BLAS");
        uint32_t root;
        if (kind == MRT_REF_INSTANCE) {
          if (idx >= d.n_instances) return fail("instance index out of range");
          root = d.instances[idx].blas_root;
        } else {
          if (idx >= d.n_models) return fail("model index out of range");
          root = d.models[idx].blas_root;
        }
        if (root >= d.n_nodes) return fail("BLAS root out of range");
        uint32_t at = push_slot(idx, 0, 0, 0);
        push_slot(0, 0, 0, kind == MRT_REF_INSTANCE ? KIND_INST : KIND_MODEL);
        jump_patches.push_back({at, root});
        s.n_prim_records++;
        return true;
      }
      default:
        return fail("bad child reference kind");
    }
  }

  // Triangle::intersect runs alpha_test only with uvs; it can reject only if
  // the triangle's own material's surface can have a zero alpha.
  SurfResolver* surfaces = nullptr;
  bool mix_alpha = false;              // a uv triangle's alpha test draws random numbers
  bool needs_alpha(const mrt_triangle& t) {
    if (!(t.flags & MRT_TRI_HAS_UV) || t.material >= d.n_materials) return false;
    const mrt_material& m = d.materials[t.material];
    if (m.kind == MRT_MAT_MIX) {  // Mix::alpha_test draws from the path RNG (material.rs:418-424)
      mix_alpha = true;
      return true;
    }
    if (m.kind != MRT_MAT_LAMBERTIAN && m.kind != MRT_MAT_METAL && m.kind != MRT_MAT_SPECULAR) return false;
    return surfaces->may_zero_alpha(m.surface);
  }

  bool fail(const char* m) {
    err = m;
    return false;
  }

  // Preorder emission of the subtree under `ref` with an explicit stack.
  bool emit_tree(uint32_t ref, bool in_blas) {
    struct Frame {
      uint32_t ref;
      uint32_t box_slot;  // != ~0: close (patch skip of) this box
    };
    std::vector<Frame> stack;
    stack.push_back({ref, ~0u});
    uint32_t depth_guard = 0;
    while (!stack.empty()) {
      Frame f = stack.back();
      stack.pop_back();
      if (f.box_slot != ~0u) {
        s.slots[4 * (f.box_slot + 1) + 2] = n_slots();  // skip = first slot after subtree
        continue;
      }
      if (MRT_REF_KIND(f.ref) != MRT_REF_NODE) {
        if (!emit_prim(f.ref, in_blas)) return false;
        continue;
      }
      uint32_t idx = MRT_REF_INDEX(f.ref);
      if (idx >= d.n_nodes) return fail("node index out of range");
      if (++depth_guard > 4 * d.n_nodes + 16) return fail("BVH is not a tree (cycle)");
      const mrt_node& n = d.nodes[idx];
      for (int k = 0; k < 3; ++k) {
        float c[2] = {n.min[k], n.max[k]};
        for (float v : c) {
          float a = fabsf(v);
          if (!(a == 0.0f || (a >= 0x1p-40f && a <= 0x1p28f))) s.fast_ok = 0;
          if (!(a <= 0x1p28f)) s.early_ok = 0;  // NaN and inf too
        }
      }
      s.rec_starts.push_back(n_slots());
      uint32_t at = push_slot(fbits(n.min[0]), fbits(n.min[1]), fbits(n.min[2]), fbits(n.max[0]));
      push_slot(fbits(n.max[1]), fbits(n.max[2]), 0, kBoxFlag | (at + 2));  // hit: the first child, next
      s.n_box_records++;
      stack.push_back({0, at});  // closes after both children
      if (MRT_REF_KIND(n.right) != MRT_REF_NONE) stack.push_back({n.right, ~0u});
      if (MRT_REF_KIND(n.left) == MRT_REF_NONE) return fail("BvhNode without a left child");
      stack.push_back({n.left, ~0u});
      if (stack.size() > s.max_depth) s.max_depth = (uint32_t)stack.size();
    }
    return true;
  }
};

// ---- record helpers (layout.h) ----
uint32_t rec_kind(const std::vector<uint32_t>& w, uint32_t i) { return w[4 * (i + 1) + 3]; }
bool rec_is_box(const std::vector<uint32_t>& w, uint32_t i) { return (rec_kind(w, i) & kBoxFlag) != 0; }
uint32_t rec_slots(const std::vector<uint32_t>& w, uint32_t i) {
  const uint32_t k = rec_kind(w, i);
  return (k & kBoxFlag) ? 2 : (k == KIND_TRI ? 3 : 2);
}
// the record the traversal reaches after primitive / instance record i
uint32_t rec_next(const std::vector<uint32_t>& w, uint32_t i) {
  switch (rec_kind(w, i)) {
    case KIND_TRI: return w[4 * (i + 2) + 3];
    case KIND_SPHERE:
    case KIND_VOLUME: return w[4 * (i + 1) + 1];
    default: return i + 2;  // instance / model: the record after it
  }
}
// children of box record i, in order (the first is its hit index; a child's
// successor at its level: a box's skip, a primitive's next)
void box_children(const std::vector<uint32_t>& w, uint32_t i, std::vector<uint32_t>& out) {
  out.clear();
  const uint32_t end = w[4 * (i + 1) + 2];
  for (uint32_t c = rec_kind(w, i) & ~kBoxFlag; c != end; c = rec_is_box(w, c) ? w[4 * (c + 1) + 2] : rec_next(w, c))
    out.push_back(c);
}

// Regions laid out with siblings together (round 3): the
// region's top-level items first, then every box's children as one group,
// the groups in depth-first order of their parents; a group holding a box
// starts on a 64-byte boundary, a group of primitives on 32 B; the END
// record last. The traversal's sequence of records is unchanged (successors
// are explicit); what changes is which records share a cache line: a box
// and its sibling sit in one 64-B half-line, so a ray that tests both
// fetches one line, where the preorder stream put the sibling after the whole
// left subtree. tools/layout_sim.cpp, mesh_ply: 64 -> 39 distinct 128-B lines
// per ray, L2 misses 1.67 -> 1.21 per ray (model; measured on the GPU:
// mesh_ply k_trace 9.40 -> 8.95 ms, 681 -> 716 Msamples/s).
// The world region keeps its preorder layout: an instance or model record
// returns to the record after it (its return index is also the handle of the
// hit's container, path.h trav_hit). Placing each instance right before its
// preorder successor instead was measured (round 3): sphere_grid and
// cube_field unchanged, Menger 38.1 -> 31.4 Msamples/s (the instance pairs of
// its leaves end up beside their successors' groups, not their parents').
struct Relayout {
  const std::vector<uint32_t>& w;
  std::vector<uint32_t>& out;
  std::vector<uint32_t>& remap;
  uint32_t at = 0;

  void place(uint32_t r) {
    remap[r] = at;
    at += rec_slots(w, r);
  }
  void group(const std::vector<uint32_t>& g, uint32_t align) {
    at = (at + align - 1) / align * align;
    for (uint32_t r : g) place(r);
  }

  // records [begin .. end_rec] (end_rec: the region's END record) of a region
  // without instance / model records
  void region(uint32_t begin, uint32_t end_rec) {
    std::vector<uint32_t> top, kids;
    for (uint32_t j = begin; j != end_rec; j = rec_is_box(w, j) ? w[4 * (j + 1) + 2] : rec_next(w, j)) top.push_back(j);
    std::vector<uint32_t> stack(top.rbegin(), top.rend());
    std::vector<uint32_t> boxes;  // DFS order
    while (!stack.empty()) {
      const uint32_t r = stack.back();
      stack.pop_back();
      if (rec_kind(w, r) == KIND_INST || rec_kind(w, r) == KIND_MODEL)
        throw std::logic_error("relayout: an instance inside a relaid region");
      if (!rec_is_box(w, r)) continue;
      boxes.push_back(r);
      box_children(w, r, kids);
      for (size_t k = kids.size(); k-- > 0;) stack.push_back(kids[k]);
    }
    at = (at + 7) & ~7u;  // the region on a 128-B line
    group(top, 4);
    for (uint32_t b : boxes) {
      box_children(w, b, kids);
      bool any_box = false;
      for (uint32_t c : kids) any_box |= rec_is_box(w, c);
      group(kids, any_box ? 4 : 2);
    }
    at = (at + 1) & ~1u;
    place(end_rec);
  }

  // copy every placed record of `recs` with its successor indices remapped
  void emit(const std::vector<uint32_t>& recs) {
    out.resize(4 * (size_t)at, 0u);
    for (uint32_t o : recs) {
      const uint32_t n = remap[o], sl = rec_slots(w, o);
      std::copy(w.begin() + 4 * (size_t)o, w.begin() + 4 * (size_t)(o + sl), out.begin() + 4 * (size_t)n);
      uint32_t* rec = &out[4 * (size_t)n];
      const uint32_t k = rec_kind(w, o);
      if (k & kBoxFlag) {
        rec[6] = remap[rec[6]];
        rec[7] = kBoxFlag | remap[rec[7] & ~kBoxFlag];
      } else if (k == KIND_TRI) {
        rec[11] = remap[rec[11]];
      } else if (k == KIND_SPHERE || k == KIND_VOLUME) {
        rec[5] = remap[rec[5]];
      }
    }
  }
};

void relayout(HostScene& s) {
  const std::vector<uint32_t>& w = s.slots;
  std::vector<uint32_t> out, remap(w.size() / 4, ~0u);
  Relayout L{w, out, remap, 0};
  // the world region (emitted first) as it is
  uint32_t wend = s.world_end + 2;
  for (uint32_t i : s.rec_starts)
    if (i < wend) L.place(i);
  for (const BlasRegion& r : s.blas_regions) L.region(r.begin, r.end);
  for (uint32_t i : s.rec_starts)
    if (remap[i] == ~0u) throw std::logic_error("relayout: a record was not placed");
  L.emit(s.rec_starts);
  for (uint32_t i : s.rec_starts) {  // instance / model records: their BLAS ranges
    const uint32_t k = rec_kind(w, i);
    if (k == KIND_INST || k == KIND_MODEL) {
      uint32_t* rec = &out[4 * (size_t)remap[i]];
      rec[1] = remap[rec[1]];
      rec[2] = remap[rec[2]];
      if (remap[i + 2] != remap[i] + 2) throw std::logic_error("relayout: an instance moved away from its successor");
    }
  }
  s.world_begin = remap[s.world_begin];
  s.world_end = remap[s.world_end];
  for (BlasRegion& r : s.blas_regions) r.begin = remap[r.begin], r.end = remap[r.end];
  for (uint32_t& i : s.rec_starts) i = remap[i];
  std::sort(s.rec_starts.begin(), s.rec_starts.end());
  s.slots.swap(out);
}

void put_m4_12(std::vector<float>& dst, const float* m16) {
  // column-major 4x4 -> c0.xyz c1.xyz c2.xyz c3.xyz
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 3; ++r) dst.push_back(m16[4 * c + r]);
}

}  // namespace

bool build_host_scene(const mrt_scene_desc& d, HostScene& s, std::string& err, bool sibling_layout) {
  const bool keep = s.keep_nf_boxes;
  const int nf_build = s.nf_build;
  s = HostScene{};
  s.keep_nf_boxes = keep;
  s.nf_build = nf_build;
  SurfResolver surf{d, s, err, {}, {}};
  Emitter e{d, s, err, {}, &surf};
  // materials
  for (uint32_t i = 0; i < d.n_materials; ++i) {
    const mrt_material& m = d.materials[i];
    GpuMaterial g{};
    g.kind = m.kind;
    g.param = m.param;
    if (m.kind > MRT_MAT_MIX) return (err = "bad material kind", false);
    if (m.kind == MRT_MAT_LAMBERTIAN || m.kind == MRT_MAT_METAL || m.kind == MRT_MAT_SPECULAR) {
      if (m.surface >= d.n_surfaces) return (err = "material surface out of range", false);
      GpuSurfRef r;
      if (!surf.resolve(m.surface, r)) return false;
      g.surf_kind = r.kind;
      g.texture = r.index;
      g.surf_len = r.len;
      for (int k = 0; k < 4; ++k) g.color[k] = r.color[k];
    } else if (m.kind == MRT_MAT_DIFFUSE_LIGHT || m.kind == MRT_MAT_ISOTROPHIC) {
      for (int k = 0; k < 3; ++k) g.color[k] = m.emit[k];  // emission / albedo
    } else if (m.kind == MRT_MAT_MIX) {
      // children strictly below: the device's pick loop always terminates
      if (m.left >= i || m.right >= i) return (err = "Mix children must precede the Mix in the material table", false);
      g.left = m.left;
      g.right = m.right;
    }
    s.materials.push_back(g);
  }
  // textures
  for (uint32_t i = 0; i < d.n_textures; ++i) {
    const mrt_texture& t = d.textures[i];
    if (t.wrap == MRT_WRAP_MIRROR) return (err = "WrapMode::Mirror is unimplemented (texture.rs:280-282)", false);
    if (t.wrap != MRT_WRAP_REPEAT && t.wrap != MRT_WRAP_CLAMP) return (err = "bad wrap mode", false);
    if (t.width == 0 || t.height == 0 || !t.rgba) return (err = "empty texture", false);
    // 8x4-texel blocks, one 128-B L2 line each (layout.h GpuTexture): a
    // bilinear tap's 2x2 footprint touches 1.41 lines on average instead of
    // the 2.06 of row-major rows
    const uint32_t tpr = (t.width + kTexBlockW - 1) / kTexBlockW, rows = (t.height + kTexBlockH - 1) / kTexBlockH;
    const size_t n = (size_t)tpr * rows * kTexBlockW * kTexBlockH, base = s.texels.size();
    if (base + n > 0xFFFFFFFFull) return (err = "textures past 2^32 texels", false);
    GpuTexture g{t.width, t.height, t.wrap, (uint32_t)base};
    s.textures.push_back(g);
    s.texels.resize(base + n, 0u);
    for (uint32_t y = 0; y < t.height; ++y)
      for (uint32_t x = 0; x < t.width; ++x) {
        uint32_t v;
        memcpy(&v, t.rgba + 4 * ((size_t)y * t.width + x), 4);
        s.texels[base + texel_index(tpr, x, y)] = v;
      }
  }
  auto check_mat = [&](uint32_t m, bool allow_none) {
    return (allow_none && m == MRT_NO_MATERIAL) || m < d.n_materials;
  };
  // spheres
  for (uint32_t i = 0; i < d.n_spheres; ++i) {
    const mrt_sphere& sp = d.spheres[i];
    if (!check_mat(sp.material, false)) return (err = "sphere material out of range", false);
    for (int k = 0; k < 3; ++k) s.sph.push_back(sp.center[k]);
    s.sph.push_back(sp.radius);
    s.sph_mat.push_back(sp.material);
  }
  // triangles (shading records)
  s.tri_shade.reserve((size_t)d.n_triangles * kTriShadeQuads * 4);
  for (uint32_t i = 0; i < d.n_triangles; ++i) {
    const mrt_triangle& t = d.triangles[i];
    if (!check_mat(t.material, false)) return (err = "triangle material out of range", false);
    float q[28] = {t.a[0],   t.a[1],   t.a[2],   t.b[0],   t.b[1],   t.b[2],   t.c[0],
                   t.c[1],   t.c[2],   t.na[0],  t.na[1],  t.na[2],  t.nb[0],  t.nb[1],
                   t.nb[2],  t.nc[0],  t.nc[1],  t.nc[2],  t.uva[0], t.uva[1], t.uvb[0],
                   t.uvb[1], t.uvc[0], t.uvc[1], 0,        0,        0,        0};
    uint32_t flags = (t.flags & MRT_TRI_HAS_UV) ? TRI_FLAG_UV : 0;
    memcpy(&q[24], &t.material, 4);
    memcpy(&q[25], &flags, 4);
    s.tri_shade.insert(s.tri_shade.end(), q, q + 28);
  }
  // volumes (geom.rs:602-607: neg_inv_density = -1.0 / density)
  for (uint32_t i = 0; i < d.n_volumes; ++i) {
    const mrt_volume& v = d.volumes[i];
    if (!check_mat(v.material, false)) return (err = "volume material out of range", false);
    s.vol_nid.push_back(-1.0f / v.density);
    s.vol_mat.push_back(v.material);
  }
  if (d.n_volumes) {
    s.ln_table.resize((size_t)1 << 23);
    for (uint32_t m = 0; m < (1u << 23); ++m) s.ln_table[m] = logf((float)m * 0x1p-23f);
  }
  // instances / models
  for (uint32_t i = 0; i < d.n_instances; ++i) {
    const mrt_instance& in = d.instances[i];
    if (!check_mat(in.material, true)) return (err = "instance material out of range", false);
    put_m4_12(s.inst_inv, in.inv);
    put_m4_12(s.inst_fwd, in.fwd);
    s.inst_mat.push_back(in.material);
  }
  for (uint32_t i = 0; i < d.n_models; ++i) {
    if (!check_mat(d.models[i].material, true)) return (err = "model material out of range", false);
    s.model_mat.push_back(d.models[i].material);
  }
  // background
  s.bg_kind = d.background.kind;
  for (int k = 0; k < 3; ++k) s.bg_color[k] = d.background.color[k];
  if (d.background.kind == MRT_BG_SKYSPHERE || d.background.kind == MRT_BG_CUBEMAP) {
    const bool cube = d.background.kind == MRT_BG_CUBEMAP;
    for (int k = 0; k < (cube ? 6 : 1); ++k) {
      GpuSurfRef r;
      if (!surf.resolve(cube ? d.background.faces[k] : d.background.surface, r)) return false;
      s.bg_faces.push_back(r);
    }
    if (cube) memcpy(s.bg_m, d.background.transform, sizeof(s.bg_m));
  } else if (d.background.kind > MRT_BG_CUBEMAP) {
    return (err = "bad background kind", false);
  }
  // world region: World::objects in order
  s.world_begin = 0;
  for (uint32_t r = 0; r < d.n_roots; ++r)
    if (!e.emit_tree(d.roots[r], false)) return false;
  s.world_end = e.n_slots();
  e.push_end();
  // BLAS regions, one per distinct root, emitted once and shared
  std::unordered_map<uint32_t, size_t> blas;  // BLAS root node -> s.blas_regions index
  for (auto& p : e.jump_patches) {
    auto it = blas.find(p.second);
    if (it == blas.end()) {
      uint32_t b = e.n_slots();
      if (!e.emit_tree(MRT_REF(MRT_REF_NODE, p.second), true)) return false;
      s.blas_regions.push_back({b, e.n_slots(), 0, false});
      it = blas.emplace(p.second, s.blas_regions.size() - 1).first;
      e.push_end();
    }
    BlasRegion& r = s.blas_regions[it->second];
    r.refs++;
    if (s.slots[4 * (p.first + 1) + 3] == KIND_MODEL) r.model = true;
    s.slots[4 * p.first + 1] = r.begin;
    s.slots[4 * p.first + 2] = r.end;
  }
  if (e.mix_alpha) s.trav_rng = true;
  if (sibling_layout) relayout(s);  // false: the plain preorder stream (tools/slab_check.cpp layout check)
  if (!build_nf_trees(d, s, err)) return false;  // appended after the reference stream (layout.h)
  if (s.slots.size() / 4 >= kLdsTag) return (err = "scene too large (record stream >= 2^30 slots)", false);
  return true;
}

// ---- LDS treelet -----------------------------------------------------------

namespace {

double box_area(const std::vector<uint32_t>& w, uint32_t i) {
  float v[6];
  memcpy(v, &w[4 * i], 16);
  memcpy(v + 4, &w[4 * (i + 1)], 8);
  const double dx = (double)v[3] - v[0], dy = (double)v[4] - v[1], dz = (double)v[5] - v[2];
  const double a = 2.0 * (dx * dy + dy * dz + dz * dx);
  return a == a ? a : 1e300;  // NaN/inf boxes: treat as always visited
}

}  // namespace

void build_treelet(HostScene& s, uint32_t budget) {
  const std::vector<uint32_t>& w = s.slots;
  const uint32_t n = (uint32_t)(w.size() / 4);
  s.tlet.clear();
  s.slots_tl.clear();
  s.tl_world_begin = s.world_begin;
  s.tl_boxes = 0;
  if (budget < 2 || n == 0) return;
  std::vector<uint8_t> staged(n, 0);  // record starts chosen for the LDS copy
  uint32_t used = 0;
  auto stage_range = [&](uint32_t b, uint32_t e) {  // every record of [b, e)
    for (auto it = std::lower_bound(s.rec_starts.begin(), s.rec_starts.end(), b);
         it != s.rec_starts.end() && *it < e; ++it) {
      staged[*it] = 1;
      used += rec_slots(w, *it);
    }
  };
  if (n <= budget) {
    stage_range(0, n);  // small scene: the whole stream
  } else {
    // 1. small BLAS regions whole (each instance/model entry then runs in LDS),
    //    the most referenced first, within a quarter of the budget
    std::vector<size_t> order(s.blas_regions.size());
    for (size_t k = 0; k < order.size(); ++k) order[k] = k;
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) {
      const BlasRegion &x = s.blas_regions[a], &y = s.blas_regions[b];
      return x.refs != y.refs ? x.refs > y.refs : (x.end - x.begin) < (y.end - y.begin);
    });
    std::vector<uint8_t> whole(s.blas_regions.size(), 0);
    for (size_t k : order) {
      const BlasRegion& r = s.blas_regions[k];
      const uint32_t size = r.end + 2 - r.begin;  // + its END record
      if (size <= budget / 8 && used + size <= budget / 4) {
        stage_range(r.begin, r.end + 2);
        whole[k] = 1;
      }
    }
    // 2. boxes by surface area (the probability that a ray meets them), from
    //    the world roots and the roots of model BLAS (same space): a child's
    //    area never exceeds its parent's, so the chosen set is a rooted treelet
    std::priority_queue<std::pair<double, uint32_t>> pq;
    std::vector<uint32_t> kids;
    auto push_children = [&](uint32_t i) {
      box_children(w, i, kids);
      for (uint32_t j : kids)
        if (rec_is_box(w, j) && !staged[j]) pq.push({box_area(w, j), j});
    };
    for (uint32_t j = s.world_begin; j < n && w[4 * (j + 1) + 3] != KIND_END;
         j = rec_is_box(w, j) ? w[4 * (j + 1) + 2] : rec_next(w, j))
      if (rec_is_box(w, j)) pq.push({box_area(w, j), j});
    for (size_t k = 0; k < s.blas_regions.size(); ++k)
      if (!whole[k] && s.blas_regions[k].model && rec_is_box(w, s.blas_regions[k].begin))
        pq.push({box_area(w, s.blas_regions[k].begin), s.blas_regions[k].begin});
    while (!pq.empty() && used + 2 <= budget) {
      const uint32_t i = pq.top().second;
      pq.pop();
      staged[i] = 1;
      used += 2;
      push_children(i);
    }
  }
  // LDS image: the chosen records in stream order (whole regions stay together)
  std::vector<uint32_t> lds_at(n, ~0u);
  uint32_t at = 0;
  for (uint32_t i : s.rec_starts)
    if (staged[i]) {
      lds_at[i] = at;
      at += rec_slots(w, i);
      if (rec_is_box(w, i)) s.tl_boxes++;
    }
  for (uint32_t i : s.rec_starts)  // an instance/model returns to the record after it: that one too
    if (staged[i] && (rec_kind(w, i) == KIND_INST || rec_kind(w, i) == KIND_MODEL) &&
        !(i + 2 < n && staged[i + 2] && lds_at[i + 2] == lds_at[i] + 2))
      throw std::logic_error("treelet: a copied instance's successor is not copied after it");
  auto R = [&](uint32_t g) { return g < n && lds_at[g] != ~0u ? (kLdsTag | lds_at[g]) : g; };
  auto rewrite = [&](uint32_t* rec) {  // rec: one record's slots (4 words each)
    if (rec[7] & kBoxFlag) {
      rec[6] = R(rec[6]);
      rec[7] = kBoxFlag | R(rec[7] & ~kBoxFlag);
    } else if (rec[7] == KIND_INST || rec[7] == KIND_MODEL) {
      rec[1] = R(rec[1]);
    } else if (rec[7] == KIND_TRI) {
      rec[11] = R(rec[11]);
    } else if (rec[7] == KIND_SPHERE || rec[7] == KIND_VOLUME) {
      rec[5] = R(rec[5]);
    }
  };
  s.slots_tl = w;
  for (uint32_t i : s.rec_starts) {
    rewrite(&s.slots_tl[4 * i]);
    if (staged[i]) {
      const size_t at = s.tlet.size();
      s.tlet.insert(s.tlet.end(), w.begin() + 4 * (size_t)i, w.begin() + 4 * (size_t)(i + rec_slots(w, i)));
      rewrite(&s.tlet[at]);
    }
  }
  s.tl_world_begin = R(s.world_begin);
}

}  // namespace mrt
