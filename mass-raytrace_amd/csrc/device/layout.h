// layout.h — the scene as it lives in HBM (built by upload.cpp from an
// mrt_scene_desc, read by the gfx950 kernels).
//
// The reference traverses a binary BvhNode tree recursively, LEFT child first,
// shrinking t_max as hits are found (geom.rs:185-205), and World::intersect
// walks its object list in order (world.rs:131-144). That visiting order is
// fixed (it does not depend on the ray), so the tree is linearised here in
// that exact depth-first preorder with a skip index per box ("threaded BVH"):
//   box hit  -> next record (first child)      box miss -> skip (past subtree)
//   primitive -> next record
// This reproduces the reference's sequence of box and primitive tests — and
// therefore its closest hit, ties included — with no traversal stack.
// Instances/models jump into a shared BLAS region and return (one level).
//
// Records are made of 16-byte slots (uint4); the kind is slot1.w, and a box
// says it is one by bit 31 there (kBoxFlag), the rest of that word being the
// index its box-hit step goes to (its first child). Boxes, spheres, triangles
// and volumes name their successors explicitly (hit / skip / next), so a
// region's records may sit in any order (round 3: BLAS regions are laid out
// with siblings together, upload.cpp relayout_blas); instances and models
// return to the record right after them:
//   BOX    2 slots  {min.x,min.y,min.z,max.x} {max.y,max.z,skip,kBoxFlag|hit}
//   SPHERE 2 slots  {cx,cy,cz,r}              {sphere_id,next,0,SPHERE}
//   TRI    3 slots  {a.x,a.y,a.z,ab.x}        {ab.y,ab.z,tri_id|alpha,TRI} {ac.x,ac.y,ac.z,next}
//   INST   2 slots  {inst_id,blas_begin,blas_end,0} {0,0,0,INST}
//   MODEL  2 slots  {model_id,blas_begin,blas_end,0} {0,0,0,MODEL}
//   VOLUME 2 slots  {cx,cy,cz,r}              {volume_id,next,0,VOLUME}  (sphere target)
//   END    2 slots  {0,0,0,0}                 {0,0,0,END}   closes every region
// Slots between records (alignment padding) are zero and never reached.
// ab = b - a and ac = c - a are precomputed on the host with the same IEEE
// subtraction Triangle::intersect performs (geom.rs:505-506).
#pragma once
#include <stdint.h>

#include "nf_bound.h"

namespace mrt {

enum : uint32_t { KIND_BOX = 1, KIND_SPHERE = 2, KIND_TRI = 3, KIND_INST = 4, KIND_MODEL = 5, KIND_VOLUME = 6 };
constexpr uint32_t kBoxFlag = 0x80000000u;  // slot1.w of a box: kBoxFlag | hit index
// LDS treelet (upload.cpp build_treelet): the most visited records are copied
// into every k_trace workgroup's LDS. An index with kLdsTag names slot
// (index & kIdxMask) of that copy; box hit/skip indices and instance/model
// BLAS entries are rewritten to reach the copies, in the copy itself and in a
// rewritten global stream (slots_tl) the LDS kernels read instead of slots.
// Whole regions are copied contiguously, so a primitive's implicit "next
// record" stays inside the copy; other primitives are never copied.
constexpr uint32_t kLdsTag = 0x40000000u;
constexpr uint32_t kIdxMask = 0x3FFFFFFFu;
// the region being traversed has ended (record after its last one; path.h)
constexpr uint32_t KIND_END = 0;
enum : uint32_t { TRI_FLAG_ALPHA = 1u, TRI_FLAG_UV = 2u };  // tri_shade flags
// a TRI record's slot1.z: the triangle id, bit 31 = the triangle is alpha-tested
constexpr uint32_t kTriAlpha = 0x80000000u;
constexpr uint32_t kTriIdMask = 0x0FFFFFFFu;

// ---- verified near-first trees (round 4, nf_tree.cpp, path.h trav_*_nf) ----
// A second set of trees over the same primitives, appended to the slot
// array after the reference stream: a surface-area-heuristic BVH over the
// world's objects (spheres, instances, models, world triangles) and one per
// BLAS, walked nearer child first (by entry distance) with a per-lane stack
// (k_trace's NF variant).
// The walk finds the closest hit with the reference's tie rule (the later
// primitive in the reference's left-first order wins, keys below), then the
// winner is checked against the REFERENCE tree (its two innermost reference
// ancestors must pass BoundingBox::hit at the winning t — nested boxes, so the
// outer ones do too — i.e. the reference's left-first walk reaches it); a ray
// that fails the check is traced again the reference's way.
//   NF NODE 2 slots {o.x,o.y,o.z,ex|ey<<8|ez<<16|lsz<<24} {qa,qb,qc,kBoxFlag|base}
//           an inner node holding BOTH children's boxes, each plane 8 bits in
//           the node's frame: plane = o.k + q * 2^(e.k - 127) (real value;
//           lo planes rounded down, hi planes up — conservative, which is all
//           the walk needs: its hits are checked against the reference tree,
//           never its boxes). q bytes, low first: qa = {L.lo.x, L.lo.y, L.lo.z,
//           L.hi.x}, qb = {L.hi.y, L.hi.z, R.lo.x, R.lo.y}, qc = {R.lo.z,
//           R.hi.x, R.hi.y, R.hi.z}. The children are the records at `base`
//           (left, lsz slots) and base + lsz (right): a node, or a leaf's first
//           primitive. One 32-B record decides two boxes (the reference
//           stream's box record decides one): half the vector loads per box.
//   SPHERE / TRI as in the reference stream, `next` = the leaf's following
//           record or kNfPop (continue with the stack)
//   INST / MODEL {id, nf_blas_root, next, wild} {parent, 0, 0, INST|MODEL}
//           wild: a wild instance's WILD entry (nf_bound.h NfWild), else 0;
//           parent: its reference world parent box (vnf_leaf's, for nf_finish)
constexpr uint32_t kNfIdx = 0x0FFFFFFFu;  // index bits of an NF node's children base
// an NF node's slot1.w: its left / right child's subtree holds a "wild"
// instance, whose rounding the world margin does not cover (nf_tree.cpp): the
// node's boxes are thickened by the wild margin too (nf_bound.h nf_rho_wild)
constexpr uint32_t kNfForceL = 0x10000000u, kNfForceR = 0x20000000u;
constexpr uint32_t kNfPop = 0x0FFFFFFFu;  // "next" of a leaf's last record: pop the stack
constexpr int kNfExpMin = -100;            // smallest plane step 2^e (products with 1/d stay normal)
constexpr uint32_t kNfStack = 24u;         // stack entries per lane (LDS): the trees' depth is capped to fit
constexpr uint32_t kNfWildFew = 16u;       // a world of at most this many instances may leave big absolute terms out of its margin (nf_tree.cpp)
constexpr uint32_t kNoParent = 0xFFFFFFFFu;
// Verification record of a leaf object (DevScene::vnf_leaf[vnf_base[kind] + id]):
//   {reference parent box record (kNoParent: a root object), order key}
// order key: the object's position among the reference's leaves of its
// region, left-first — the world region for spheres, instances, models and
// world triangles; its BLAS for a model's triangles (kWorldKey set: a world
// triangle, whose key is a world key)
constexpr uint32_t kWorldKey = 0x80000000u;
enum : uint32_t { VNF_SPHERE = 0, VNF_TRI = 1, VNF_INST = 2, VNF_MODEL = 3 };

// Composite surfaces (YCbCrTexture, TextureBlend, SolidColorFallback,
// texture.rs:197-357) run as small postfix programs over a V4 stack:
//   SOLID    push color                TEXTURE  push get_f(tex)
//   YCBCR    pop chroma, luma; push    BLEND    pop right, left; push blend(arg)
//   FALLBACK pop c; push color*(1-c.w) + c*c.w
// A YCbCr node is emitted as TEXTURE luma, TEXTURE chroma, YCBCR, so operands
// are sampled in the reference's order (left before right, luma before chroma).
constexpr uint32_t SURF_PROGRAM = 0xFFu;  // surf_kind of a composite surface reference
constexpr uint32_t kSurfStack = 4;        // deepest operand stack a program may need
struct GpuSurfOp {
  uint32_t op, tex, arg, pad;
  float color[4];
};
// A resolved surface: SOLID (color), TEXTURE (index = texture) or
// SURF_PROGRAM (index = first op, len = op count).
struct GpuSurfRef {
  uint32_t kind, index, len, pad;
  float color[4];
};

// Flattened material: surface resolved in place.
//   q0 = {kind, surf_kind, texture, param bits}
//   q1 = {color/emit rgba as float bits}
//   q2 = {left, right, surf_len, 0}
struct GpuMaterial {
  uint32_t kind, surf_kind, texture;
  float param;     // Metal fuzz, Dielectric/Specular refraction index, Mix ratio
  float color[4];  // SolidColor rgba (Lambertian/Metal/Specular), emit rgb (DiffuseLight), albedo (Isotrophic)
  uint32_t left, right;  // Mix children
  uint32_t surf_len;     // SURF_PROGRAM: op count (texture = first op)
  uint32_t pad1;
};

// RGBA8 texels (decoded c/255.0 exactly as texture.rs:44) in blocks of
// 8 x 4 texels = 128 B, one L2 line (round 6): blocks row-major over the
// texture, texels row-major inside a block, partial blocks zero-padded. A
// bilinear tap (texture.rs:126-148) reads a 2x2 footprint, which row-major
// rows spread over two lines always; in a block it stays in one line unless
// it crosses a block edge (1.41 lines per tap on average).
constexpr uint32_t kTexBlockW = 8, kTexBlockH = 4;
struct GpuTexture {
  uint32_t width, height, wrap;
  uint32_t offset;  // first texel in the texel array (a multiple of 32: line-aligned)
};
// texel (x, y) of a texture whose rows hold tpr = ceil(width / 8) blocks
MRT_HD uint32_t texel_index(uint32_t tpr, uint32_t x, uint32_t y) {
  return (((y >> 2) * tpr + (x >> 3)) << 5) + ((y & 3u) << 3) + (x & 7u);
}

// Per-triangle shading record, 7 x float4 (112 B):
//  0 {a.x a.y a.z b.x} 1 {b.y b.z c.x c.y} 2 {c.z na.x na.y na.z}
//  3 {nb.x nb.y nb.z nc.x} 4 {nc.y nc.z uva.x uva.y} 5 {uvb.x uvb.y uvc.x uvc.y}
//  6 {material, flags, 0, 0}
constexpr uint32_t kTriShadeQuads = 7;

// Kernel-visible scene (plain pointers into one device allocation).
struct DevScene {
  const uint32_t* slots;  // n_slots * 4 words
  uint32_t world_begin, world_end;
  const float* inst_inv;   // 12 floats per instance: c0.xyz c1.xyz c2.xyz c3.xyz
  const float* inst_fwd;   // 12 floats per instance
  const uint32_t* inst_mat;  // override material or 0xFFFFFFFF
  const uint32_t* model_mat;
  const float* sph;        // 4 floats per sphere: cx cy cz r
  const uint32_t* sph_mat;
  const float* tri_shade;  // kTriShadeQuads*4 floats per triangle
  const GpuMaterial* materials;
  const GpuTexture* textures;
  const uint32_t* texels;  // RGBA8 packed little-endian
  uint32_t fast_ok;  // bit 0: every box coordinate in {0} U [2^-40, 2^28] (path.h qfast exact test);
                     // bit 1: every box coordinate finite, |c| <= 2^28 (path.h early slab decision)
  // array sizes (checked only in MRT_DEBUG_BOUNDS builds) and the debug record
  uint32_t n_slots, n_tris, n_sph, n_inst, n_models, n_materials, n_textures, n_texels;
  uint32_t* dbg;  // {first failing check code, index, bound, failures}
  const float* vol_nid;     // Volume: -1/density per volume
  const uint32_t* vol_mat;  // Volume: its Isotrophic material
  const float* ln_table;    // ln(m * 2^-23) for every m < 2^23 (host libm logf), when volumes exist
  uint32_t n_vol;
  const GpuSurfOp* surf_ops;
  uint32_t n_surf_ops;
  uint32_t bg_kind;
  float bg_color[4];
  const GpuSurfRef* bg_faces;  // SkySphere: 1 surface; CubeMap: x_pos x_neg y_pos y_neg z_pos z_neg
  const float* bg_m;           // CubeMap transform, column-major 4x4
  // LDS treelet (n_tlet == 0: none)
  const uint32_t* slots_tl;    // the record stream with indices rewritten to reach the treelet
  const uint32_t* tlet;        // the treelet image copied into LDS (n_tlet slots of 4 words)
  uint32_t n_tlet;
  uint32_t tl_world_begin;     // world entry index beside the treelet (possibly LDS-tagged)
  // verified near-first trees (nf_ok == 0: the scene has none)
  uint32_t nf_ok, nf_world;    // the NF world tree's root record
  const uint32_t* vnf_leaf;    // {reference parent box, order key} pairs per leaf object
  uint32_t vnf_base[4];        // first vnf_leaf entry of spheres, triangles, instances, models
  uint32_t n_vnf;
  NfBound nfb;                 // the walk's rounding margins (nf_bound.h)
};

}  // namespace mrt
