// upload.h — mrt_scene_desc (reference tree) -> HBM layout (layout.h).
#pragma once
#include <string>
#include <vector>

#include "../../../include/massrt.h"
#include "layout.h"

namespace mrt {

// A BLAS region of the stream: records [begin, end) plus the END record at end.
struct BlasRegion {
  uint32_t begin, end, refs;  // refs: instance/model records entering it
  bool model;                 // entered by a model (world space) at least once
};

struct HostScene {
  std::vector<uint32_t> slots;  // 4 words per slot
  std::vector<uint32_t> rec_starts;  // first slot of every record, ascending (padding slots are not records)
  uint32_t world_begin = 0, world_end = 0;
  std::vector<float> inst_inv, inst_fwd;
  std::vector<uint32_t> inst_mat, model_mat;
  std::vector<float> sph;
  std::vector<uint32_t> sph_mat;
  std::vector<float> tri_shade;
  std::vector<GpuMaterial> materials;
  std::vector<GpuTexture> textures;
  std::vector<uint32_t> texels;
  uint32_t fast_ok = 1;   // every box coordinate in {0} U [2^-40, 2^28]: the exact slab test may use qfast
  uint32_t early_ok = 1;  // every box coordinate finite and within 2^28: the early slab decision applies
  bool has_alpha = false;  // some triangle carries TRI_FLAG_ALPHA
  bool trav_rng = false;   // the traversal draws random numbers (Volume, Mix alpha tests)
  std::vector<float> vol_nid;
  std::vector<uint32_t> vol_mat;
  // Volume draws f = m * 2^-23 (m < 2^23, mrt_rng.h) and takes f.ln()
  // (geom.rs:640): the device looks up the host libm logf of every such f
  // instead of computing it, so the distance is the reference's to the bit
  // (32 MiB, built only when the scene has volumes).
  std::vector<float> ln_table;
  std::vector<GpuSurfOp> surf_ops;
  uint32_t bg_kind = 0;
  float bg_color[4] = {0, 0, 0, 0};
  std::vector<GpuSurfRef> bg_faces;  // SkySphere 1, CubeMap 6
  float bg_m[16] = {0};
  std::vector<BlasRegion> blas_regions;
  // LDS treelet (build_treelet): image (4 words per slot), rewritten stream, world entry
  std::vector<uint32_t> tlet, slots_tl;
  uint32_t tl_world_begin = 0, tl_boxes = 0;
  // statistics
  uint32_t n_box_records = 0, n_prim_records = 0, max_depth = 0;
  // verified near-first trees (nf_tree.cpp): appended to `slots` after the
  // reference stream (not in rec_starts: the treelet and relayout never see them)
  bool nf_ok = false;
  uint32_t nf_world = 0, nf_boxes = 0, nf_stack_need = 0, nf_first_slot = 0;
  std::vector<uint32_t> vnf_leaf;  // {parent, key} pairs
  uint32_t vnf_base[4] = {0, 0, 0, 0};
  std::string nf_note;  // why a scene has no NF trees
  NfBound nfb{};         // the walk's rounding margins (nf_bound.h, nf_tree.cpp)
  uint32_t nf_wild = 0;  // instances the world margin does not cover: never culled
  uint32_t nf_cones = 0;  // NF nodes carrying a normal cone (nf_bound.h nf_cone_rg)
  // tools/slab_check: set before building to keep every leaf object's NF box
  // (6 floats per vnf_leaf slot: mn xyz, mx xyz) and which instances are wild
  bool keep_nf_boxes = false;
  // which NF trees to build (set before build_host_scene; the option
  // "traversal" at upload): kNfBuildAuto builds them unless the per-scene
  // rule would walk the reference's way anyway (a generic-triangle term, or a
  // big instanced world), kNfBuildNever skips them, kNfBuildAlways builds them
  int nf_build = 2;
  std::vector<float> nf_leaf_box;
  std::vector<uint8_t> nf_inst_wild;
};

enum { kNfBuildNever = 0, kNfBuildAlways = 1, kNfBuildAuto = 2 };

// Builds the verified near-first trees of a linearised scene (after
// build_host_scene; layout.h). A scene whose traversal draws random numbers,
// or whose trees would need more than kNfStack stack entries, gets none
// (nf_ok false, nf_note says why). Returns false only on an internal error.
bool build_nf_trees(const mrt_scene_desc& d, HostScene& s, std::string& err);

// Validates the description and linearises it. Returns false with `err` set.
// sibling_layout=false keeps every region in plain preorder (the layout
// before round 2; tools/slab_check.cpp checks both walk alike)
bool build_host_scene(const mrt_scene_desc& d, HostScene& out, std::string& err, bool sibling_layout = true);

// Chooses the records copied into LDS by every k_trace workgroup (at most
// `budget` 16-byte slots): the whole stream when it fits; else the small BLAS
// regions whole (most referenced first, within budget/4) and then boxes of the
// world tree and of model BLAS in decreasing surface area — a rooted treelet.
// Fills s.tlet (the LDS image), s.slots_tl (the stream with its indices
// rewritten to reach the copies) and s.tl_world_begin. budget 0: no treelet.
void build_treelet(HostScene& s, uint32_t budget);

}  // namespace mrt
