// rt_scene.h -- device scene layout (shared by the host scene compiler and the
// HIP kernels). Everything is a flat array; records are 16-byte aligned so a
// lane fetches a record with dwordx4 loads.
//
// The hittable DAG of the reference (hittable.h, hittable_list.h, bvh_node.h,
// sphere.h, quad.h, triangle.h, volumne.h) is compiled into a stack machine:
// every traversal step pops a 32-bit *entry* whose top 3 bits say what it is.
//
//   QUAD / SPHERE / TRI (i)  a primitive, tested inline where it appears in a list
//   INSTANCE (i)             translate/rotate_* wrappers (hittable.h:67-293): the
//                            ray is re-derived from the world ray through the
//                            instance's transform chain, then its BLAS entry runs
//   VOLUME (i)               volumne::hit (volumne.h:18-46), tested inline
//   NODE (i)                 BVH node: two child boxes, children are entries
//   LIST (pos)               refs[pos], refs[pos+1], ... until END, in order --
//                            hittable_list::hit semantics (closest, later wins ties)
//   SPECIAL: END (in refs), RESTORE(k) (on the stack: back to instance k-1 / world)
#pragma once

#include <stdint.h>

namespace rtd {

enum : uint32_t {
  E_QUAD = 0u,
  E_SPHERE = 1u,
  E_TRI = 2u,
  E_INSTANCE = 3u,
  E_VOLUME = 4u,
  E_NODE = 5u,
  E_LIST = 6u,
  E_SPECIAL = 7u,
};
constexpr uint32_t kTypeShift = 29;
constexpr uint32_t kPayloadMask = (1u << kTypeShift) - 1u;
constexpr uint32_t kEnd = (E_SPECIAL << kTypeShift) | 0u;
constexpr uint32_t kRestoreBase = (E_SPECIAL << kTypeShift) | 1u;  // RESTORE(k) = kRestoreBase + k
constexpr uint32_t kNoHit = 0xFFFFFFFFu;

__host__ __device__ inline uint32_t etype(uint32_t e) { return e >> kTypeShift; }
__host__ __device__ inline uint32_t epay(uint32_t e) { return e & kPayloadMask; }
__host__ __device__ inline uint32_t mk(uint32_t type, uint32_t payload) { return (type << kTypeShift) | payload; }

constexpr int kMaxChain = 4;    // translate/rotate wrappers per instance (composed, outermost first)
constexpr int kStackDepth = 32;  // traversal stack entries per lane (LDS)
constexpr int kMaxBvhDepth = 26; // the builder keeps every BVH within this depth
// Small scenes also get a *linear program*: every top-level item in the reference's
// list order -- primitive entries, INSTANCE(i) ... kInstEnd brackets, VOLUME(i) --
// that all lanes of a wave walk in lock-step (wave-uniform, scalar-loaded records).
constexpr int kLinearMax = 96;
constexpr uint32_t kInstEnd = kRestoreBase;  // back to the world ray

// One linear-program op with the data its test needs inline, so a wave fetches it
// with a single scalar load (64 B for fp32, 128 B for fp64).
//   QUAD, aux = 0        general quad: f = n[3], D, q[3], a[3], b[3] (as Quad)
//   QUAD, aux = 1 + perm axis-aligned quad (perm 0..5 encodes the plane axis A and
//                        the axes U, V of u and v): f = q[A], q[U], q[V], 1/u[U], 1/v[V], u[U], v[V]
//   SPHERE               f = c1[3], r, dc[3]; aux = moving
//   TRI                  f = p0[3], e1[3], e2[3]
//   INSTANCE             the wrapper chain inline: aux = nops | kind_k << (4 + 2k),
//                        f[3k .. 3k+2] = x, y, z of op k (as XOp; at most kMaxChain = 4)
//   VOLUME / kInstEnd    no payload (records in vols)
template <class R>
struct alignas(16) LinRec {
  uint32_t op;
  uint32_t aux;
  R f[14];
};
static_assert(3 * kMaxChain <= 14, "an instance chain must fit one LinRec");

// The *flat program*: a linear program whose ops are all axis-aligned quads, at world level or
// under translate-only instances, is rewritten in world space (translations folded into the
// records) and regrouped by plane axis, so a wave runs three branch-free loops with no per-op
// dispatch. An instance holding exactly the six quads of `box()` (quad.h:91-112) with one
// lambertian material becomes one slab-test record. Both blobs carry it (FlatQuadT<float> /
// <double>): the fp32 kernels use it by default; the fp64 kernels too (round 3), where it agrees
// with the reference-ordered linear program up to rounding (t as (plane - o_A) * (1/d_A) instead
// of a division per quad); RT_TRAV_ORDERED keeps the linear program. Order inside the scene only
// decides exact-t ties.
//   FlatQuadT, group A (plane axis): U < W are the two other axes,
//     alpha = (o_U + t d_U - lo_u) * inv_u, beta = (o_W + t d_W - lo_w) * inv_w (signed inv);
//   nm (both records) = what shade needs of the hit: material | A << 28 | (n_A < 0) << 31, the
//   quad's outward normal being +-e_A exactly (translations leave normals alone).
template <class R>
struct alignas(16) FlatQuadT {
  R plane, lo_u, lo_w, inv_u;
  R inv_w;
  uint32_t e;    // the quad's entry (exclusion state; its record is not read again)
  int32_t inst;  // its instance (translate-only), -1 at world level
  uint32_t nm;
};
using FlatQuad = FlatQuadT<float>;
constexpr uint32_t kNmMat = (1u << 28) - 1u;
//   FlatBoxT: the slab [lo, hi]; face[2k + s] is the entry of the face on plane lo_k (s = 0)
//   or hi_k (s = 1); the compiler gives the faces quad records at an 8-aligned index, face f
//   at base + f, so a ray leaving the box knows the plane it starts on (trace_flat).
template <class R>
struct alignas(16) FlatBoxT {
  R lo[3];
  R hi[3];
  int32_t inst;
  uint32_t mat;
  uint32_t face[6];
  uint32_t neg;  // bit f: face f's outward normal points to -e_k
  uint32_t pad;
};
using FlatBox = FlatBoxT<float>;
static_assert(sizeof(FlatQuadT<float>) == 32 && sizeof(FlatQuadT<double>) == 64, "flat quad records");
static_assert(sizeof(FlatBoxT<float>) == 64 && sizeof(FlatBoxT<double>) == 96, "flat box records");

// quad.h:9-23 precomputed: n = unit(cross(u,v)), D = dot(n, corner),
// a = cross(v, w), b = cross(w, u) with w = cross(u,v)/dot(cross(u,v),cross(u,v)),
// so alpha = dot(p - corner, a) = dot(w, cross(p - corner, v)) and beta = dot(p - corner, b).
template <class R>
struct alignas(16) Quad {
  R n[3];
  R D;
  R q[3];
  int32_t mat;
  R a[3];
  R area;
  R b[3];
  R pad;
};

// sphere.h:7-35. c1 = center (static) / center1 (moving); dc = center2 - center1;
// cn = the `center_` member used for the normal (sphere.h:69): c1 for the static
// constructors, (0,0,0) for the moving one, as in the reference.
template <class R>
struct alignas(16) Sphere {
  R c1[3];
  R r;
  R dc[3];
  int32_t mat;
  R cn[3];
  int32_t moving;
};

// triangle.h:8-40: e1 = p1 - p0, e2 = p2 - p0, n = unit(cross(e1, e2)).
template <class R>
struct alignas(16) Tri {
  R p0[3];
  int32_t mat;
  R e1[3];
  R pad1;
  R e2[3];
  R pad2;
  R n[3];
  R pad3;
};

// One wrapper of a chain, applied world -> object in order (hittable.h:75-82, 125-149, ...).
// kind 0: translate by (x, y, z); kind 1/2/3: rotate about x/y/z with (s, c).
template <class R>
struct alignas(16) XOp {
  R x, y, z;
  int32_t kind;
};

template <class R>
struct alignas(16) Instance {
  XOp<R> op[kMaxChain];
  int32_t nops;
  uint32_t blas;  // entry of the wrapped hittable (object space)
  int32_t pad[2];
};

// volumne.h:9-46: boundary = refs list at `boundary` (object space of chain `inst`,
// -1 = world). neg_inv_density = -1.0 / density (volumne.h:36).
// is_box: the boundary is the six quads of box() (quad.h:91-112) -- [lo, hi] in boundary space --
// and the fp32 kernels find its entry and exit with one slab test instead of twelve quad tests.
template <class R>
struct alignas(16) Volume {
  R neg_inv_density;
  int32_t inst;
  uint32_t boundary;  // LIST entry of the boundary primitives
  int32_t phase_mat;
  R lo[3];
  int32_t is_box;
  R hi[3];
  int32_t pad;
};

template <class R>
struct alignas(16) Node {
  R lo[2][3];
  R hi[2][3];
  uint32_t child[2];
};

// The *wide BVH* (fp32 kernels): a 4-wide tree over world-level primitives, for scenes whose
// world is primitives under lists / bvh_nodes only (no translate/rotate, no volume), e.g. the
// RTOW spheres and glTF triangle meshes. One node is 128 B of structure-of-arrays child boxes,
// read as six 16-byte loads; the primitives sit in leaf order in one stream of 16-byte words
// (no reference indirection), in LDS when the whole tree fits:
//   sphere   [c1.xyz, entry] [dc.xyz, r]
//   triangle [p0.xyz, entry] [e1.xyz, -] [e2.xyz, -]
//   quad     [q.xyz, entry] [n.xyz, D] [a.xyz, -] [b.xyz, -]       (fields of Quad)
// `entry` (as bits) is the primitive's entry in quads/spheres/tris: shading and the
// self-exclusion test use it exactly as for the other traversals.
// child[c]: an inner node's index, or kWLeaf | (count - 1) << kWCountShift | first word;
// unused slots have empty boxes (lo = hi = +inf on every axis: no ray direction hits them).
struct alignas(16) WNode {
  float lox[4], loy[4], loz[4];
  float hix[4], hiy[4], hiz[4];
  uint32_t child[4];
  uint32_t pad[4];
};
// The half-precision node (round 4) for trees in HBM, read by the fp64 rays (RT_WIDE_HALF_F64). A node
// visit of the HBM kernels costs an L1 address-path slot per load instruction whatever its width
// (tools/l1_rates.hip: a random wave64 load costs the same ~39 CU cycles as dword, dwordx2 or dwordx4);
// this node is 5 loads where a WNode visit is 7. Child boxes are fp16 offsets from the node's origin (its
// children's smallest lo corner, a float), rounded outward:
//   lo[2a + h], hi[2a + h]: axis a, children 2h (low half) and 2h + 1 (high half)
//   child[c]: as WNode (an inner node's index, or a leaf code)
// Unused slots hold +inf offsets (no ray direction enters them). Measured on the C4 stand-in: fp64
// 504.0 -> 480.8 ms/frame; fp32 rays, whose node test is VALU-cheaper, lost (310.3 -> 370.0: the fp16
// operands and the per-ray near/far selection cost more issue than the two loads save; eight per-octant
// copies, 373.7; copies padded to one per 128-byte line, 392.5).
struct alignas(16) WNodeH {
  float ox, oy, oz;
  uint32_t pad;
  uint32_t lo[6];
  uint32_t hi[6];
  uint32_t child[4];
};
static_assert(sizeof(WNodeH) == 80, "WNodeH is five 16-byte loads");
constexpr uint32_t kWLeaf = 0x80000000u;
constexpr uint32_t kWCountShift = 25;  // leaf: up to 64 primitives, first word < 2^25
constexpr uint32_t kWFirstMask = (1u << kWCountShift) - 1u;
constexpr int kWLeafMax = 3;         // primitives per leaf (triangles, mixed kinds)
constexpr int kWLeafMaxSpheres = 6;  // sphere-only trees (at most 8: the LDS code's 3-bit count)
constexpr int kWideStackMax = 96;  // stack entries a ray may need in the wide tree (beyond LDS: a spill area)
// top-of-tree nodes ordered first, breadth-first (three levels of a 4-wide tree); the HBM kernels copy the
// first RT_WIDE_TOP_N of them to LDS
constexpr uint32_t kWideTopMax = 85;
// primitive kinds present (SceneHeader::wide_kinds)
enum : uint32_t { WK_SPHERE = 1u, WK_TRI = 2u, WK_QUAD = 4u, WK_MOVING = 8u };

enum : int32_t { M_LAMBERTIAN = 1, M_METAL = 2, M_DIELECTRIC = 3, M_ISOTROPIC = 4, M_DIFFUSE_LIGHT = 5, M_GLOSS = 6 };
enum : int32_t { T_SOLID = 1, T_CHECKER = 2, T_PERLIN = 3, T_VALUE = 4, T_WORLEY = 5, T_VORONOI = 6, T_IMAGE = 7 };
constexpr uint32_t kPerlinPoints = 256;  // noise.h:76 point_count

template <class R>
struct alignas(16) Texture {
  R c0[3];  // solid color / checker odd
  int32_t kind;
  R c1[3];  // checker even
  R scale;  // checker (texture.h:48), perlin (texture.h:87)
  uint32_t data;  // perlin: rand_offset (256 x 3) then perm_x (256); value: n^3 values -- offsets into texdata;
                  // image: byte offset into images
  uint32_t n;     // value noise resolution; image width
  uint32_t h;     // image height
};
// The material's texture is copied inline: shading reads one record per hit.
template <class R>
struct alignas(16) Material {
  int32_t kind;
  int32_t tex;
  R fuzz;  // float in the reference (material.h:96); widened exactly
  R refr;  // float in the reference (material.h:142)
  R smooth, spec;  // gloss: smoothness_ clamped to [0, 1] and specular_prob_ (material.h:147-155)
  R pad[2];
  Texture<R> tx;  // = texs[tex]
};

// The importance-sampling light (camera.h:135 `light`, hittable_list.h:39-50).
enum : int32_t { L_NONE = 0, L_BASE = 1, L_QUAD = 2, L_SPHERE = 3 };
template <class R>
struct alignas(16) Light {
  int32_t kind;
  int32_t aligned;  // L_QUAD: 1 + perm when axis-aligned (af as a LinRec aligned quad), else 0
  int32_t pad[2];
  Quad<R> quad;  // L_QUAD (quad.h:66-78)
  R u[3];
  R pad1;
  R v[3];
  R pad2;
  R center[3];  // L_SPHERE: center_ (sphere.h:76-81)
  R radius;
  R af[8];  // aligned L_QUAD: q[A], q[U], q[V], 1/u[U], 1/v[V], u[U], v[V], 1/area
};

// What the host uploads: offsets into one contiguous device blob.
struct SceneHeader {
  uint32_t root;      // entry of the world
  int32_t background; // texture index or -1
  int32_t has_volumes;
  int32_t num_instances;
  uint64_t off_quads, off_spheres, off_tris, off_instances, off_volumes, off_nodes, off_refs, off_mats, off_texs,
      off_light, off_linear;  // off_linear: LinRec array
  uint64_t off_texdata;       // procedural-texture tables, double in both blobs (noise runs in fp64)
  uint64_t n_texdata;
  int32_t has_cell_noise;     // a worley / voronoi / image texture (EXT kernels)
  int32_t pad2_;
  uint64_t off_images;        // picture-texture pixels (RGB bytes)
  uint64_t n_images;
  uint64_t bytes;
  uint32_t n_linear;  // 0: no linear program (use the BVH traversal)
  uint32_t n_flat_box;          // flat program: boxes
  uint32_t n_flat_quad[3];      // flat program: quads per plane axis
  uint32_t has_flat;            // 1: the flat program replaces the linear program (RT_TRAV_AUTO)
  uint64_t off_flat_quad, off_flat_box;
  uint32_t n_quads, n_spheres, n_tris, n_volumes, n_nodes, n_refs, n_mats, n_texs;
  // wide BVH (fp32 blob only; has_wide = 0: none)
  uint64_t off_wnodes, off_wprims;
  uint32_t n_wnodes, n_wprim_words;
  uint32_t wroot;        // root child code (a node index, or a leaf code for a tiny scene)
  uint32_t wide_stack;   // traversal stack entries a lane can need
  uint32_t wide_kinds;   // WK_* bits
  uint32_t has_wide;
  uint32_t wide_big;     // primitives at the head of the word stream tested before the tree (huge boxes)
  uint32_t has_wnodesh;  // the WNodeH form of the same tree is present (n_wnodes nodes from off_wnodesh)
  uint64_t off_wnodesh;
  // fp32 blob: the fp64 Quad records too (same indices), for the same re-decision in quad_t; 0: none
  uint32_t has_quads64;
  uint64_t off_quads64;
  // what shading can meet (round 5: kernels specialised for lambertian + diffuse_light scenes)
  uint32_t mat_kinds;   // bit M_* of every material kind
  uint32_t tex_kinds;   // bit T_* of every material's texture kind (the background's too)
  int32_t light_kind;   // L_* of the importance-sampling light
  int32_t light_aligned;
  uint32_t wide_top;    // the wide tree's first levels, breadth-first: nodes [0, wide_top) (LDS copy, HBM trees)
};

}  // namespace rtd
