// scene_compile.cpp -- hittable DAG -> device scene (see rt_scene.h).
//
// Semantics kept from the reference:
//  * hittable_list::hit (hittable_list.h:20-31) is an ordered scan where the
//    closest hit wins and, on equal t, the later object wins. Lists that hold a
//    volume (whose hit draws a random number, volumne.h:36) or that are small
//    stay ordered lists; larger volume-free lists and every bvh_node become a
//    SAH BVH of our own (closest hit is independent of the tree except for
//    exact-t ties).
//  * translate / rotate_x/y/z (hittable.h:67-293) become instances holding the
//    whole chain of wrappers from the world down to the object, applied in the
//    reference's order and arithmetic, so object-space hits are bit-identical
//    to the reference's nested calls in the fp64 path.
//  * volumne (volumne.h:9-46) keeps its boundary as an ordered primitive list
//    plus that boundary's wrapper chain.
#include "scene_compile.h"

#include <algorithm>
#include <string>
#include <unordered_map>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <new>
#include <stdexcept>

namespace rtd {
namespace {
// perm -> (A, U, V): the plane axis and the axes of u and v (rt_scene.h LinRec)
constexpr int kPermAxes[6][3] = {{2, 0, 1}, {1, 0, 2}, {2, 1, 0}, {0, 1, 2}, {1, 2, 0}, {0, 2, 1}};

constexpr double kInf = std::numeric_limits<double>::infinity();
constexpr int kSmallList = 8;  // lists up to this size stay ordered lists
constexpr int kLeafMax = 4;

struct Box {
  double lo[3] = {kInf, kInf, kInf};
  double hi[3] = {-kInf, -kInf, -kInf};
  void grow(const double* p) {
    for (int k = 0; k < 3; k++) {
      lo[k] = std::min(lo[k], p[k]);
      hi[k] = std::max(hi[k], p[k]);
    }
  }
  void grow(const Box& b) {
    for (int k = 0; k < 3; k++) {
      lo[k] = std::min(lo[k], b.lo[k]);
      hi[k] = std::max(hi[k], b.hi[k]);
    }
  }
  bool empty() const { return !(lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2]); }
  double area() const {
    if (empty()) return 0;
    double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2 * (dx * dy + dy * dz + dz * dx);
  }
  double center(int k) const { return 0.5 * (lo[k] + hi[k]); }
};

struct Op {  // one wrapper, world -> object direction
  int kind;  // 0 translate, 1/2/3 rotate x/y/z
  double x, y, z;  // translate: offset; rotate: x = sin, y = cos
};

// object -> parent for a point (inverse of one Op), the reference's back-transform
void op_to_parent(const Op& op, double p[3]) {
  if (op.kind == 0) {
    p[0] += op.x;
    p[1] += op.y;
    p[2] += op.z;
    return;
  }
  int a = op.kind == 1 ? 1 : 0, b = op.kind == 3 ? 1 : 2;
  double s = op.x, c = op.y;
  double pa = p[a], pb = p[b];
  p[a] = c * pa + s * pb;
  p[b] = -s * pa + c * pb;
}

Box box_to_parent(const Box& in, const std::vector<Op>& ops) {  // ops outermost first
  if (in.empty()) return in;
  Box out;
  for (int i = 0; i < 8; i++) {
    double p[3] = {(i & 1) ? in.hi[0] : in.lo[0], (i & 2) ? in.hi[1] : in.lo[1], (i & 4) ? in.hi[2] : in.lo[2]};
    for (int k = (int)ops.size() - 1; k >= 0; k--) op_to_parent(ops[(size_t)k], p);
    out.grow(p);
  }
  // rotations are applied in double: widen by a relative margin so the box stays conservative
  for (int k = 0; k < 3; k++) {
    double m = 1e-9 * (std::fabs(out.lo[k]) + std::fabs(out.hi[k])) + 1e-12;
    out.lo[k] -= m;
    out.hi[k] += m;
  }
  return out;
}

inline void v_sub(const double* a, const double* b, double* o) {
  for (int k = 0; k < 3; k++) o[k] = a[k] - b[k];
}
inline void v_cross(const double* a, const double* b, double* o) {  // vec3.h:79-82
  double r0 = a[1] * b[2] - a[2] * b[1], r1 = a[2] * b[0] - a[0] * b[2], r2 = a[0] * b[1] - a[1] * b[0];
  o[0] = r0;
  o[1] = r1;
  o[2] = r2;
}
inline double v_dot(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
inline void v_unit(const double* a, double* o) {  // vec3.h:77: v / v.length()
  double l = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  for (int k = 0; k < 3; k++) o[k] = a[k] / l;
}

struct Item {
  uint32_t entry;
  Box box;
  int need;   // traversal stack entries processing this entry can add
  int depth;  // BVH depth below this entry
  bool volume;
  bool lin_ok = true;         // the item has a linear-program form (see rt_scene.h)
  std::vector<uint32_t> lin;  // its ops in reference order
};

// concatenation of the items' linear programs, in order
void join_lin(Item& dst, const std::vector<Item>& items) {
  dst.lin.clear();
  dst.lin_ok = true;
  for (const Item& m : items) {
    if (!m.lin_ok || dst.lin.size() + m.lin.size() > (size_t)kLinearMax) {
      dst.lin_ok = false;
      dst.lin.clear();
      return;
    }
    dst.lin.insert(dst.lin.end(), m.lin.begin(), m.lin.end());
  }
}

class Compiler {
 public:
  explicit Compiler(const rt_scene_desc* d) : d_(d) {}

  bool run(CompiledScene* out, std::string* err);

 private:
  const rt_scene_desc* d_;
  std::string err_;
  bool ok_ = true;

  std::vector<Quad<double>> quads_;
  std::vector<Sphere<double>> spheres_;
  std::vector<Tri<double>> tris_;
  std::vector<Instance<double>> insts_;
  std::vector<Volume<double>> vols_;
  std::vector<Node<double>> nodes_;
  std::vector<uint32_t> refs_;
  std::vector<Material<double>> mats_;
  std::vector<double> texdata_;  // procedural-texture tables (Texture::data offsets)
  bool cell_noise_ = false;      // a worley / voronoi / image texture (EXT kernels)
  std::vector<uint8_t> images_;  // picture-texture pixels
  std::vector<int32_t> mat_remap_;                    // descriptor material -> mats_ index
  std::unordered_map<std::string, int32_t> mat_index_;  // material record bytes -> mats_ index
  int32_t mat_id(int32_t m) const { return mat_remap_[(size_t)m]; }
  std::vector<Texture<double>> texs_;
  Light<double> light_{};
  int depth_guard_ = 0;

  bool fail(const std::string& m) {
    if (ok_) err_ = m;
    ok_ = false;
    return false;
  }
  const rt_object* obj(int i) {
    if (i < 0 || i >= d_->num_objects) {
      fail("object index " + std::to_string(i) + " out of range");
      return nullptr;
    }
    return &d_->objects[i];
  }
  bool check_mat(int m) {
    if (m < 0 || m >= d_->num_materials) return fail("primitive without a valid material");
    return true;
  }
  static bool is_wrapper(int kind) { return kind >= RT_OBJ_TRANSLATE && kind <= RT_OBJ_ROTATE_Z; }
  static Op op_of(const rt_object& o) {
    if (o.kind == RT_OBJ_TRANSLATE) return {0, o.a[0], o.a[1], o.a[2]};
    return {o.kind - RT_OBJ_ROTATE_X + 1, o.s0, o.s1, 0.0};
  }

  Item prim_item(const rt_object& o);
  void gather(int idx, const std::vector<Op>& chain, std::vector<Item>& out, bool ordered_ctx);
  Item container(std::vector<Item>& items, bool ordered);
  Item list_of(const std::vector<Item>& items);
  Item bvh(std::vector<Item>& items, size_t b, size_t e, int depth);
  int make_instance(const std::vector<Op>& chain, uint32_t blas);
  LinRec<double> lin_record(uint32_t op) const;
  bool flat_program(const std::vector<uint32_t>& lin, std::vector<FlatQuadT<double>>& quads, uint32_t nq[3],
                    std::vector<FlatBoxT<double>>& boxes);
  bool wide_bvh(const std::vector<Item>& prims, CompiledScene* out);
  bool box_of_quads(const std::vector<Item>& prims, double lo[3], double hi[3]) const;
  std::vector<int> aligned_;  // per quad: 1 + perm for axis-aligned quads, 0 otherwise
  std::vector<double> qu_, qv_;  // per quad: u[U], v[V] (aligned quads)
  void light_from(int idx);
};

Item Compiler::prim_item(const rt_object& o) {
  Item it{};
  it.need = 0;
  it.depth = 0;
  it.volume = false;
  if (!check_mat(o.material)) return it;
  if (o.kind == RT_OBJ_QUAD) {  // quad.h:9-23
    Quad<double> q{};
    double n[3], nn;
    v_cross(o.b, o.c, n);
    v_unit(n, q.n);
    q.area = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    for (int k = 0; k < 3; k++) q.q[k] = o.a[k];
    q.D = v_dot(q.n, q.q);
    nn = v_dot(n, n);
    double w[3] = {n[0] / nn, n[1] / nn, n[2] / nn};
    v_cross(o.c, w, q.a);  // alpha = dot(w, cross(p, v)) = dot(p, cross(v, w))
    v_cross(w, o.b, q.b);  // beta  = dot(w, cross(u, p)) = dot(p, cross(w, u))
    q.mat = mat_id(o.material);
    quads_.push_back(q);
    it.entry = mk(E_QUAD, (uint32_t)quads_.size() - 1);
    // axis-aligned: u and v each along one axis, on different axes (then n is exactly +-e_A)
    auto single_axis = [](const double* v) {
      int k = -1;
      for (int j = 0; j < 3; j++)
        if (v[j] != 0.0) {
          if (k >= 0) return -1;
          k = j;
        }
      return k;
    };
    int U = single_axis(o.b), Vv = single_axis(o.c);
    int perm = -1;
    if (U >= 0 && Vv >= 0 && U != Vv) {
      static const int kPerm[3][3] = {{-1, 0, 1}, {2, -1, 3}, {4, 5, -1}};  // (U, V) -> perm
      perm = kPerm[U][Vv];
    }
    aligned_.push_back(perm + 1);
    qu_.push_back(U >= 0 ? o.b[U] : 0.0);
    qv_.push_back(Vv >= 0 ? o.c[Vv] : 0.0);
    double c1[3], c2[3], c3[3];
    for (int k = 0; k < 3; k++) {
      c1[k] = o.a[k] + o.b[k];
      c2[k] = o.a[k] + o.c[k];
      c3[k] = o.a[k] + o.b[k] + o.c[k];
    }
    it.box.grow(o.a);
    it.box.grow(c1);
    it.box.grow(c2);
    it.box.grow(c3);
  } else if (o.kind == RT_OBJ_SPHERE) {  // sphere.h:7-35
    Sphere<double> s{};
    double r = std::fmax(0, o.s0);
    for (int k = 0; k < 3; k++) {
      s.c1[k] = o.a[k];
      s.dc[k] = o.moving ? (o.b[k] - o.a[k]) : 0.0;
      s.cn[k] = o.moving ? 0.0 : o.a[k];
    }
    s.r = r;
    s.mat = mat_id(o.material);
    s.moving = o.moving ? 1 : 0;
    spheres_.push_back(s);
    it.entry = mk(E_SPHERE, (uint32_t)spheres_.size() - 1);
    double lo[3], hi[3];
    for (int k = 0; k < 3; k++) {
      lo[k] = o.a[k] - r;
      hi[k] = o.a[k] + r;
    }
    it.box.grow(lo);
    it.box.grow(hi);
    if (o.moving) {
      for (int k = 0; k < 3; k++) {
        lo[k] = o.b[k] - r;
        hi[k] = o.b[k] + r;
      }
      it.box.grow(lo);
      it.box.grow(hi);
    }
  } else {  // triangle.h:19-25
    Tri<double> t{};
    for (int k = 0; k < 3; k++) t.p0[k] = o.a[k];
    v_sub(o.b, o.a, t.e1);
    v_sub(o.c, o.a, t.e2);
    double n[3];
    v_cross(t.e1, t.e2, n);
    v_unit(n, t.n);
    t.mat = mat_id(o.material);
    tris_.push_back(t);
    it.entry = mk(E_TRI, (uint32_t)tris_.size() - 1);
    it.box.grow(o.a);
    it.box.grow(o.b);
    it.box.grow(o.c);
  }
  it.lin = {it.entry};
  return it;
}

int Compiler::make_instance(const std::vector<Op>& chain, uint32_t blas) {
  if ((int)chain.size() > kMaxChain) {
    fail("more than " + std::to_string(kMaxChain) + " nested translate/rotate wrappers");
    return -1;
  }
  Instance<double> in{};
  in.nops = (int)chain.size();
  for (size_t k = 0; k < chain.size(); k++) in.op[k] = {chain[k].x, chain[k].y, chain[k].z, chain[k].kind};
  in.blas = blas;
  insts_.push_back(in);
  return (int)insts_.size() - 1;
}

Item Compiler::list_of(const std::vector<Item>& items) {
  Item it{};
  it.entry = mk(E_LIST, (uint32_t)refs_.size());
  it.need = 0;
  it.depth = 0;
  it.volume = false;
  for (const Item& m : items) {
    refs_.push_back(m.entry);
    it.box.grow(m.box);
    uint32_t t = etype(m.entry);
    if (t == E_INSTANCE || t == E_NODE || t == E_LIST) it.need = std::max(it.need, std::max(2, 1 + m.need));
    it.depth = std::max(it.depth, m.depth);
    it.volume = it.volume || m.volume;
  }
  refs_.push_back(kEnd);
  join_lin(it, items);
  return it;
}

Item Compiler::bvh(std::vector<Item>& items, size_t b, size_t e, int depth) {
  size_t n = e - b;
  if (n == 1) return items[b];
  Box bounds, cb;
  for (size_t i = b; i < e; i++) {
    bounds.grow(items[i].box);
    double c[3] = {items[i].box.center(0), items[i].box.center(1), items[i].box.center(2)};
    cb.grow(c);
  }
  if (n <= (size_t)kLeafMax && depth > 0) {
    std::vector<Item> leaf(items.begin() + (long)b, items.begin() + (long)e);
    return list_of(leaf);
  }
  // binned SAH over the largest centroid axis
  int axis = 0;
  for (int k = 1; k < 3; k++)
    if (cb.hi[k] - cb.lo[k] > cb.hi[axis] - cb.lo[axis]) axis = k;
  size_t mid = b + n / 2;
  double extent = cb.hi[axis] - cb.lo[axis];
  bool split_found = false;
  if (extent > 0 && depth < kMaxBvhDepth - 4) {
    constexpr int kBins = 16;
    Box bin_box[kBins];
    size_t bin_cnt[kBins] = {};
    auto bin_of = [&](const Item& it) {
      int k = (int)((it.box.center(axis) - cb.lo[axis]) / extent * kBins);
      return std::min(kBins - 1, std::max(0, k));
    };
    for (size_t i = b; i < e; i++) {
      int k = bin_of(items[i]);
      bin_cnt[k]++;
      bin_box[k].grow(items[i].box);
    }
    double best = kInf;
    int best_k = -1;
    for (int s = 1; s < kBins; s++) {
      Box lb, rb;
      size_t lc = 0, rc = 0;
      for (int k = 0; k < s; k++) {
        lb.grow(bin_box[k]);
        lc += bin_cnt[k];
      }
      for (int k = s; k < kBins; k++) {
        rb.grow(bin_box[k]);
        rc += bin_cnt[k];
      }
      if (!lc || !rc) continue;
      double cost = lb.area() * (double)lc + rb.area() * (double)rc;
      if (cost < best) {
        best = cost;
        best_k = s;
      }
    }
    if (best_k > 0) {
      double leaf_cost = bounds.area() * (double)n;
      if (n <= (size_t)kLeafMax && best >= leaf_cost) {
        std::vector<Item> leaf(items.begin() + (long)b, items.begin() + (long)e);
        return list_of(leaf);
      }
      auto it = std::partition(items.begin() + (long)b, items.begin() + (long)e,
                               [&](const Item& x) { return bin_of(x) < best_k; });
      mid = (size_t)(it - items.begin());
      split_found = mid > b && mid < e;
    }
  }
  if (!split_found) {
    mid = b + n / 2;
    std::nth_element(items.begin() + (long)b, items.begin() + (long)mid, items.begin() + (long)e,
                     [&](const Item& x, const Item& y) { return x.box.center(axis) < y.box.center(axis); });
  }
  size_t node_idx = nodes_.size();
  nodes_.emplace_back();
  Item l = bvh(items, b, mid, depth + 1);
  Item r = bvh(items, mid, e, depth + 1);
  Node<double>& nd = nodes_[node_idx];
  for (int k = 0; k < 3; k++) {
    nd.lo[0][k] = l.box.lo[k];
    nd.hi[0][k] = l.box.hi[k];
    nd.lo[1][k] = r.box.lo[k];
    nd.hi[1][k] = r.box.hi[k];
  }
  nd.child[0] = l.entry;
  nd.child[1] = r.entry;
  Item it{};
  it.entry = mk(E_NODE, (uint32_t)node_idx);
  it.box = bounds;
  it.lin_ok = false;  // a BVH's linear form comes from its items in reference order (container())
  it.need = std::max(2, 1 + std::max(l.need, r.need));
  it.depth = 1 + std::max(l.depth, r.depth);
  it.volume = l.volume || r.volume;
  return it;
}

Item Compiler::container(std::vector<Item>& items, bool ordered) {
  if (items.size() == 1) return items[0];
  bool has_volume = false;
  for (auto& i : items) has_volume = has_volume || i.volume;
  if (ordered || has_volume || items.size() <= (size_t)kSmallList) return list_of(items);
  Item lin_src;
  join_lin(lin_src, items);  // reference (gather) order, before the BVH build reorders
  Item it = bvh(items, 0, items.size(), 0);
  it.lin = std::move(lin_src.lin);
  it.lin_ok = lin_src.lin_ok;
  return it;
}

void Compiler::gather(int idx, const std::vector<Op>& chain, std::vector<Item>& out, bool ordered_ctx) {
  if (!ok_) return;
  if (++depth_guard_ > 4096) {
    fail("object graph nesting too deep (cycle?)");
    return;
  }
  const rt_object* o = obj(idx);
  if (!o) return;
  switch (o->kind) {
    case RT_OBJ_QUAD:
    case RT_OBJ_SPHERE:
    case RT_OBJ_TRIANGLE:
      out.push_back(prim_item(*o));
      break;
    case RT_OBJ_LIST:  // spliced in order: closest-hit over nested lists is the same scan
      if (o->first_child < 0 || o->child_count < 0 || o->first_child + o->child_count > d_->num_children) {
        fail("list child range out of bounds");
        break;
      }
      for (int k = 0; k < o->child_count; k++) gather(d_->children[o->first_child + k], chain, out, ordered_ctx);
      break;
    case RT_OBJ_BVH: {
      if (o->first_child < 0 || o->child_count < 0 || o->first_child + o->child_count > d_->num_children) {
        fail("bvh child range out of bounds");
        break;
      }
      std::vector<Item> sub;
      for (int k = 0; k < o->child_count; k++) gather(d_->children[o->first_child + k], chain, sub, false);
      if (!ok_) break;
      if (!ordered_ctx) {
        out.insert(out.end(), sub.begin(), sub.end());
      } else if (!sub.empty()) {
        out.push_back(container(sub, sub.size() <= (size_t)kSmallList));
      }
      break;
    }
    case RT_OBJ_TRANSLATE:
    case RT_OBJ_ROTATE_X:
    case RT_OBJ_ROTATE_Y:
    case RT_OBJ_ROTATE_Z: {
      std::vector<Op> ops;
      const rt_object* w = o;
      while (w && is_wrapper(w->kind)) {
        if ((int)(chain.size() + ops.size()) >= kMaxChain) {
          fail("more than " + std::to_string(kMaxChain) + " nested translate/rotate wrappers (or a cycle)");
          return;
        }
        ops.push_back(op_of(*w));
        w = obj(w->child);
      }
      if (!w) break;
      std::vector<Op> chain2 = chain;
      chain2.insert(chain2.end(), ops.begin(), ops.end());
      std::vector<Item> sub;
      gather((int)(w - d_->objects), chain2, sub, false);
      if (!ok_) break;
      Item blas = sub.empty() ? list_of(sub) : container(sub, false);
      int ii = make_instance(chain2, blas.entry);
      if (ii < 0) break;
      Item it{};
      it.entry = mk(E_INSTANCE, (uint32_t)ii);
      it.box = box_to_parent(blas.box, ops);
      it.need = std::max(2, 1 + blas.need);
      it.depth = blas.depth;
      it.volume = blas.volume;
      it.lin_ok = blas.lin_ok;
      for (uint32_t op : blas.lin)
        if (etype(op) == E_INSTANCE) it.lin_ok = false;  // nested instances: BVH traversal only
      if (it.lin_ok && blas.lin.size() + 2 <= (size_t)kLinearMax) {
        it.lin.push_back(it.entry);
        it.lin.insert(it.lin.end(), blas.lin.begin(), blas.lin.end());
        it.lin.push_back(kInstEnd);
      } else {
        it.lin_ok = false;
      }
      out.push_back(it);
      break;
    }
    case RT_OBJ_VOLUME: {
      if (o->material < 0 || o->material >= d_->num_materials) {
        fail("volume without a phase material");
        break;
      }
      std::vector<Op> ops;
      const rt_object* w = obj(o->child);
      while (w && is_wrapper(w->kind)) {
        if ((int)(chain.size() + ops.size()) >= kMaxChain) {
          fail("more than " + std::to_string(kMaxChain) + " nested translate/rotate wrappers (or a cycle)");
          return;
        }
        ops.push_back(op_of(*w));
        w = obj(w->child);
      }
      if (!w) break;
      std::vector<Op> chain2 = chain;
      chain2.insert(chain2.end(), ops.begin(), ops.end());
      std::vector<Item> prims;
      gather((int)(w - d_->objects), chain2, prims, true);
      if (!ok_) break;
      for (auto& p : prims) {
        uint32_t t = etype(p.entry);
        if (t != E_QUAD && t != E_SPHERE && t != E_TRI) {
          fail("volume boundary must be primitives under one translate/rotate chain");
          return;
        }
      }
      Item bl = list_of(prims);
      Volume<double> v{};
      v.is_box = box_of_quads(prims, v.lo, v.hi) ? 1 : 0;
      v.neg_inv_density = -1.0 / o->s0;
      v.inst = chain2.empty() ? -1 : make_instance(chain2, bl.entry);
      v.boundary = bl.entry;
      v.phase_mat = mat_id(o->material);
      vols_.push_back(v);
      Item it{};
      it.entry = mk(E_VOLUME, (uint32_t)vols_.size() - 1);
      it.box = box_to_parent(bl.box, ops);
      it.need = 0;
      it.depth = 0;
      it.volume = true;
      it.lin = {it.entry};
      out.push_back(it);
      break;
    }
    default:
      fail("unsupported hittable kind " + std::to_string(o->kind));
  }
  --depth_guard_;
}

void Compiler::light_from(int idx) {
  std::memset(&light_, 0, sizeof light_);
  if (idx < 0) {
    light_.kind = L_NONE;
    return;
  }
  const rt_object* o = obj(idx);
  if (!o) return;
  if (o->kind == RT_OBJ_QUAD) {  // quad::pdf_value / random (quad.h:66-78)
    size_t before = quads_.size();
    Item it = prim_item(*o);
    (void)it;
    if (!ok_) return;
    light_.kind = L_QUAD;
    light_.quad = quads_.back();
    if (aligned_.back()) {
      const int* ax = kPermAxes[aligned_.back() - 1];
      light_.aligned = aligned_.back();
      light_.af[0] = light_.quad.q[ax[0]];
      light_.af[1] = light_.quad.q[ax[1]];
      light_.af[2] = light_.quad.q[ax[2]];
      light_.af[3] = 1.0 / qu_.back();
      light_.af[4] = 1.0 / qv_.back();
      light_.af[5] = qu_.back();
      light_.af[6] = qv_.back();
      light_.af[7] = 1.0 / light_.quad.area;  // fp64 light_pdf_aligned
    }
    quads_.resize(before);
    aligned_.resize(before);
    qu_.resize(before);
    qv_.resize(before);
    for (int k = 0; k < 3; k++) {
      light_.u[k] = o->b[k];
      light_.v[k] = o->c[k];
    }
  } else if (o->kind == RT_OBJ_SPHERE) {  // sphere::pdf_value / random (sphere.h:76-81)
    light_.kind = L_SPHERE;
    for (int k = 0; k < 3; k++) light_.center[k] = o->moving ? 0.0 : o->a[k];
    light_.radius = std::fmax(0, o->s0);
  } else {
    light_.kind = L_BASE;  // hittable base class: pdf_value 0, random (1,0,0) (hittable.h:39-41)
  }
}

template <class T>
size_t append(std::vector<unsigned char>& blob, const std::vector<T>& v) {
  size_t off = (blob.size() + 255) & ~size_t(255);
  blob.resize(off + v.size() * sizeof(T));
  if (!v.empty()) std::memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
  return off;
}

inline float down(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
  return std::nextafter(f, -std::numeric_limits<float>::infinity());
}
inline float up(double x) {
  float f = (float)x;
  if ((double)f < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
  return std::nextafter(f, std::numeric_limits<float>::infinity());
}

// fp16 bit patterns of non-negative values (rt_scene.h WNodeH): the value of a pattern, and the
// largest pattern at or below x / the smallest at or above x (patterns 0 .. 0x7C00 = +inf order like
// their values)
inline double half_value(uint16_t h) {
  const int e = (h >> 10) & 31, m = h & 1023;
  if (e == 31) return std::numeric_limits<double>::infinity();
  return e == 0 ? std::ldexp((double)m, -24) : std::ldexp((double)(1024 + m), e - 25);
}
inline uint16_t half_down(double x) {
  if (!(x >= 0)) return 0;
  uint32_t lo = 0, hi = 0x7C00;  // half_value(lo) <= x
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    (half_value((uint16_t)mid) <= x ? lo : hi) = mid;
  }
  return (uint16_t)(half_value((uint16_t)hi) <= x ? hi : lo);
}
inline uint16_t half_up(double x) {
  if (!(x > 0)) return 0;
  uint32_t lo = 0, hi = 0x7C00;  // half_value(hi) >= x
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    (half_value((uint16_t)mid) >= x ? hi : lo) = mid;
  }
  return (uint16_t)hi;
}
// A wide tree in WNodeH form (rt_scene.h). The float node's planes are already rounded outward; the
// offsets from the origin (float minus float: exact in double) are rounded outward again to fp16.
std::vector<WNodeH> half_nodes(const std::vector<WNode>& wn) {
  std::vector<WNodeH> out(wn.size());
  for (size_t i = 0; i < wn.size(); i++) {
    const WNode& w = wn[i];
    const float* lo[3] = {w.lox, w.loy, w.loz};
    const float* hi[3] = {w.hix, w.hiy, w.hiz};
    WNodeH& h = out[i];
    float* org[3] = {&h.ox, &h.oy, &h.oz};
    for (int a = 0; a < 3; a++) {
      float m = std::numeric_limits<float>::infinity();
      for (int c = 0; c < 4; c++)
        if (std::isfinite(lo[a][c])) m = std::min(m, lo[a][c]);
      *org[a] = std::isfinite(m) ? m : 0.f;
      uint16_t ql[4], qh[4];
      for (int c = 0; c < 4; c++) {
        // unused slots are exactly the builder's sentinel lo = +inf; a used child whose float plane saturated
        // (a box beyond float range: down() / up() give -inf / +inf) keeps an infinite offset on that side
        // (fp16 -inf = 0xFC00 below the origin, half_up(+inf) = +inf above it), so fp64 rays cull it no more
        // than the float node does
        const bool used = !(lo[a][c] == std::numeric_limits<float>::infinity());
        const bool lo_inf = lo[a][c] == -std::numeric_limits<float>::infinity();
        ql[c] = !used ? (uint16_t)0x7C00 : lo_inf ? (uint16_t)0xFC00 : half_down((double)lo[a][c] - (double)*org[a]);
        qh[c] = used ? half_up((double)hi[a][c] - (double)*org[a]) : (uint16_t)0x7C00;
      }
      for (int k = 0; k < 2; k++) {
        h.lo[2 * a + k] = (uint32_t)ql[2 * k] | (uint32_t)ql[2 * k + 1] << 16;
        h.hi[2 * a + k] = (uint32_t)qh[2 * k] | (uint32_t)qh[2 * k + 1] << 16;
      }
    }
    h.pad = 0;
    for (int c = 0; c < 4; c++) h.child[c] = w.child[c];
  }
  return out;
}

template <class D, class S>
void cvt3(D* d, const S* s) {
  for (int k = 0; k < 3; k++) d[k] = (D)s[k];
}

Quad<float> to32(const Quad<double>& q) {
  Quad<float> r{};
  cvt3(r.n, q.n);
  r.D = (float)q.D;
  cvt3(r.q, q.q);
  r.mat = q.mat;
  cvt3(r.a, q.a);
  r.area = (float)q.area;
  cvt3(r.b, q.b);
  return r;
}
Sphere<float> to32(const Sphere<double>& s) {
  Sphere<float> r{};
  cvt3(r.c1, s.c1);
  r.r = (float)s.r;
  cvt3(r.dc, s.dc);
  r.mat = s.mat;
  cvt3(r.cn, s.cn);
  r.moving = s.moving;
  return r;
}
Tri<float> to32(const Tri<double>& t) {
  Tri<float> r{};
  cvt3(r.p0, t.p0);
  r.mat = t.mat;
  cvt3(r.e1, t.e1);
  cvt3(r.e2, t.e2);
  cvt3(r.n, t.n);
  return r;
}
Instance<float> to32(const Instance<double>& in) {
  Instance<float> r{};
  for (int k = 0; k < kMaxChain; k++) r.op[k] = {(float)in.op[k].x, (float)in.op[k].y, (float)in.op[k].z, in.op[k].kind};
  r.nops = in.nops;
  r.blas = in.blas;
  return r;
}
Volume<float> to32(const Volume<double>& v) {
  return {(float)v.neg_inv_density, v.inst, v.boundary, v.phase_mat, {(float)v.lo[0], (float)v.lo[1], (float)v.lo[2]},
          v.is_box, {(float)v.hi[0], (float)v.hi[1], (float)v.hi[2]}, 0};
}
Node<float> to32(const Node<double>& n) {
  Node<float> r{};
  for (int c = 0; c < 2; c++)
    for (int k = 0; k < 3; k++) {
      r.lo[c][k] = down(n.lo[c][k]);
      r.hi[c][k] = up(n.hi[c][k]);
    }
  r.child[0] = n.child[0];
  r.child[1] = n.child[1];
  return r;
}
Texture<float> to32(const Texture<double>& t);
Material<float> to32(const Material<double>& m) {
  return {m.kind, m.tex, (float)m.fuzz, (float)m.refr, (float)m.smooth, (float)m.spec, {0, 0}, to32(m.tx)};
}
LinRec<float> to32(const LinRec<double>& l) {
  LinRec<float> r{};
  r.op = l.op;
  r.aux = l.aux;
  for (int k = 0; k < 14; k++) r.f[k] = (float)l.f[k];
  return r;
}
Texture<float> to32(const Texture<double>& t) {
  Texture<float> r{};
  cvt3(r.c0, t.c0);
  r.kind = t.kind;
  cvt3(r.c1, t.c1);
  r.scale = (float)t.scale;
  r.data = t.data;
  r.n = t.n;
  r.h = t.h;
  return r;
}
Light<float> to32(const Light<double>& l) {
  Light<float> r{};
  r.kind = l.kind;
  r.quad = to32(l.quad);
  cvt3(r.u, l.u);
  cvt3(r.v, l.v);
  cvt3(r.center, l.center);
  r.radius = (float)l.radius;
  r.aligned = l.aligned;
  for (int k = 0; k < 8; k++) r.af[k] = (float)l.af[k];
  return r;
}
template <class T>
auto map32(const std::vector<T>& v) {
  std::vector<decltype(to32(v[0]))> r;
  r.reserve(v.size());
  for (auto& x : v) r.push_back(to32(x));
  return r;
}

template <class Q, class S, class T, class I, class V, class N, class M, class X, class L, class LR>
SceneHeader pack(std::vector<unsigned char>& blob, const std::vector<Q>& q, const std::vector<S>& s,
                 const std::vector<T>& t, const std::vector<I>& in, const std::vector<V>& vo, const std::vector<N>& nd,
                 const std::vector<uint32_t>& refs, const std::vector<M>& m, const std::vector<X>& x, const L& light,
                 const std::vector<LR>& linear, const std::vector<double>& texdata,
                 const std::vector<uint8_t>& images) {
  SceneHeader h{};
  blob.clear();
  h.off_quads = append(blob, q);
  h.off_spheres = append(blob, s);
  h.off_tris = append(blob, t);
  h.off_instances = append(blob, in);
  h.off_volumes = append(blob, vo);
  h.off_nodes = append(blob, nd);
  h.off_refs = append(blob, refs);
  h.off_mats = append(blob, m);
  h.off_texs = append(blob, x);
  h.off_light = append(blob, std::vector<L>{light});
  h.off_linear = append(blob, linear);
  h.n_linear = (uint32_t)linear.size();
  h.off_texdata = append(blob, texdata);
  h.n_texdata = texdata.size();
  h.off_images = append(blob, images);
  h.n_images = images.size();
  blob.resize((blob.size() + 255) & ~size_t(255));
  h.bytes = blob.size();
  h.n_quads = (uint32_t)q.size();
  h.n_spheres = (uint32_t)s.size();
  h.n_tris = (uint32_t)t.size();
  h.n_volumes = (uint32_t)vo.size();
  h.n_nodes = (uint32_t)nd.size();
  h.n_refs = (uint32_t)refs.size();
  h.n_mats = (uint32_t)m.size();
  h.n_texs = (uint32_t)x.size();
  h.num_instances = (int32_t)in.size();
  for (const auto& mm : m) {
    h.mat_kinds |= 1u << (mm.kind & 31);
    h.tex_kinds |= 1u << (mm.tx.kind & 31);
  }
  for (const auto& tx : x) h.tex_kinds |= 1u << (tx.kind & 31);  // the background's texture (and the rest)
  h.light_kind = light.kind;
  h.light_aligned = light.aligned;
  return h;
}

// perm -> (A, U, V): the plane axis and the axes of u and v (rt_scene.h LinRec)

LinRec<double> Compiler::lin_record(uint32_t op) const {
  LinRec<double> r{};
  r.op = op;
  const uint32_t ty = etype(op), i = epay(op);
  if (op == kInstEnd || ty == E_VOLUME) return r;
  if (ty == E_INSTANCE) {
    const Instance<double>& in = insts_[i];
    r.aux = (uint32_t)in.nops;
    for (int k = 0; k < in.nops; k++) {
      r.aux |= (uint32_t)in.op[k].kind << (4 + 2 * k);
      r.f[3 * k] = in.op[k].x;
      r.f[3 * k + 1] = in.op[k].y;
      r.f[3 * k + 2] = in.op[k].z;
    }
    return r;
  }
  if (ty == E_QUAD) {
    const Quad<double>& q = quads_[i];
    if (aligned_[i]) {
      const int* ax = kPermAxes[aligned_[i] - 1];
      r.aux = (uint32_t)aligned_[i];
      r.f[0] = q.q[ax[0]];
      r.f[1] = q.q[ax[1]];
      r.f[2] = q.q[ax[2]];
      r.f[3] = 1.0 / qu_[i];
      r.f[4] = 1.0 / qv_[i];
      r.f[5] = qu_[i];
      r.f[6] = qv_[i];
    } else {
      for (int k = 0; k < 3; k++) {
        r.f[k] = q.n[k];
        r.f[4 + k] = q.q[k];
        r.f[7 + k] = q.a[k];
        r.f[10 + k] = q.b[k];
      }
      r.f[3] = q.D;
    }
  } else if (ty == E_SPHERE) {
    const Sphere<double>& sp = spheres_[i];
    for (int k = 0; k < 3; k++) {
      r.f[k] = sp.c1[k];
      r.f[4 + k] = sp.dc[k];
    }
    r.f[3] = sp.r;
    r.aux = (uint32_t)sp.moving;
  } else if (ty == E_TRI) {
    const Tri<double>& t = tris_[i];
    for (int k = 0; k < 3; k++) {
      r.f[k] = t.p0[k];
      r.f[3 + k] = t.e1[k];
      r.f[6 + k] = t.e2[k];
    }
  }
  return r;
}

// The flat program of rt_scene.h: the linear program's ops are all axis-aligned quads, at world
// level or in translate-only instances. Returns false (no flat program) for anything else. The
// records come out in double (the fp64 blob) and are rounded once for the fp32 blob (flat32).
bool Compiler::flat_program(const std::vector<uint32_t>& lin, std::vector<FlatQuadT<double>>& quads, uint32_t nq[3],
                            std::vector<FlatBoxT<double>>& boxes) {
  struct Q {
    uint32_t e;
    int32_t inst;
    int A, U, W;        // plane axis; U < W the other two
    double plane, lo_u, lo_w, len_u, len_w;  // object space
  };
  auto quad_of = [&](uint32_t op, int32_t inst, Q& q) {
    const uint32_t i = epay(op);
    if (etype(op) != E_QUAD || !aligned_[i]) return false;
    const int* ax = kPermAxes[aligned_[i] - 1];  // A, axis of u, axis of v
    q.e = op;
    q.inst = inst;
    q.A = ax[0];
    q.plane = quads_[i].q[ax[0]];
    double lu = quads_[i].q[ax[1]], lv = quads_[i].q[ax[2]], su = qu_[i], sv = qv_[i];
    if (ax[1] < ax[2]) {
      q.U = ax[1], q.W = ax[2], q.lo_u = lu, q.lo_w = lv, q.len_u = su, q.len_w = sv;
    } else {
      q.U = ax[2], q.W = ax[1], q.lo_u = lv, q.lo_w = lu, q.len_u = sv, q.len_w = su;
    }
    return true;
  };
  std::vector<FlatQuadT<double>> grp[3];
  auto add_quad = [&](const Q& q, const double* off) {
    FlatQuadT<double> r{};
    r.plane = q.plane + off[q.A];
    r.lo_u = q.lo_u + off[q.U];
    r.lo_w = q.lo_w + off[q.W];
    r.inv_u = 1.0 / q.len_u;
    r.inv_w = 1.0 / q.len_w;
    r.e = q.e;
    r.inst = q.inst;
    const Quad<double>& qq = quads_[epay(q.e)];
    r.nm = (uint32_t)qq.mat | (uint32_t)q.A << 28 | (qq.n[q.A] < 0 ? 1u << 31 : 0u);
    grp[q.A].push_back(r);
  };
  // six quads of box() (quad.h:91-112) with one lambertian material -> one slab record
  auto as_box = [&](const std::vector<Q>& qs, const double* off, FlatBoxT<double>& b) {  // b.face: original entries
    if (qs.size() != 6) return false;
    const int32_t mat = quads_[epay(qs[0].e)].mat;
    if (mats_[(size_t)mat].kind != M_LAMBERTIAN) return false;
    double lo[3], hi[3];
    int cnt[3] = {0, 0, 0};
    for (const Q& q : qs) {
      if (quads_[epay(q.e)].mat != mat) return false;
      if (cnt[q.A] == 0) lo[q.A] = hi[q.A] = q.plane;
      lo[q.A] = std::min(lo[q.A], q.plane);
      hi[q.A] = std::max(hi[q.A], q.plane);
      cnt[q.A]++;
    }
    for (int k = 0; k < 3; k++)
      if (cnt[k] != 2 || !(lo[k] < hi[k])) return false;
    int seen[6] = {0, 0, 0, 0, 0, 0};
    for (const Q& q : qs) {  // each face spans the box exactly in its two in-plane axes
      const double u0 = std::min(q.lo_u, q.lo_u + q.len_u), u1 = std::max(q.lo_u, q.lo_u + q.len_u);
      const double w0 = std::min(q.lo_w, q.lo_w + q.len_w), w1 = std::max(q.lo_w, q.lo_w + q.len_w);
      if (u0 != lo[q.U] || u1 != hi[q.U] || w0 != lo[q.W] || w1 != hi[q.W]) return false;
      const int f = 2 * q.A + (q.plane == hi[q.A] ? 1 : 0);
      if (seen[f]++) return false;
      b.face[f] = q.e;
      if (quads_[epay(q.e)].n[q.A] < 0) b.neg |= 1u << f;
    }
    for (int k = 0; k < 3; k++) {
      b.lo[k] = lo[k] + off[k];
      b.hi[k] = hi[k] + off[k];
    }
    b.inst = qs[0].inst;
    b.mat = (uint32_t)mat;
    return true;
  };
  const double zero[3] = {0, 0, 0};
  const size_t quads_before = quads_.size();
  auto undo = [&]() {
    quads_.resize(quads_before);
    aligned_.resize(quads_before);
    qu_.resize(quads_before);
    qv_.resize(quads_before);
    return false;
  };
  for (size_t k = 0; k < lin.size(); k++) {
    const uint32_t op = lin[k];
    if (etype(op) == E_QUAD) {
      Q q;
      if (!quad_of(op, -1, q)) return undo();
      add_quad(q, zero);
      continue;
    }
    if (etype(op) != E_INSTANCE) return undo();
    const int32_t ii = (int32_t)epay(op);
    const Instance<double>& in = insts_[(size_t)ii];
    double off[3] = {0, 0, 0};
    for (int j = 0; j < in.nops; j++) {
      if (in.op[j].kind != 0) return undo();  // rotations: the linear program
      off[0] += in.op[j].x;
      off[1] += in.op[j].y;
      off[2] += in.op[j].z;
    }
    std::vector<Q> qs;
    for (k++; k < lin.size() && lin[k] != kInstEnd; k++) {
      Q q;
      if (!quad_of(lin[k], ii, q)) return undo();
      qs.push_back(q);
    }
    if (k == lin.size()) return undo();
    FlatBoxT<double> b{};
    if (as_box(qs, off, b)) {
      // the faces get copies of their quad records at an 8-aligned index, face j at base + j:
      // a ray leaving the box knows from its entry which slab plane it starts on (trace_flat)
      while (quads_.size() % 8) {
        quads_.push_back(quads_[0]);
        aligned_.push_back(aligned_[0]);
        qu_.push_back(qu_[0]);
        qv_.push_back(qv_[0]);
      }
      for (int f = 0; f < 6; f++) {
        const uint32_t i = epay(b.face[f]);
        quads_.push_back(quads_[i]);
        aligned_.push_back(aligned_[i]);
        qu_.push_back(qu_[i]);
        qv_.push_back(qv_[i]);
        b.face[f] = mk(E_QUAD, (uint32_t)quads_.size() - 1);
      }
      boxes.push_back(b);
    } else
      for (const Q& q : qs) add_quad(q, off);
  }
  quads.clear();
  for (int a = 0; a < 3; a++) {
    nq[a] = (uint32_t)grp[a].size();
    quads.insert(quads.end(), grp[a].begin(), grp[a].end());
  }
  return true;
}

// Six axis-aligned quads that are exactly the faces of one box (as box(), quad.h:91-112, makes them):
// each axis has two face planes, and every face spans the box in its two in-plane axes.
bool Compiler::box_of_quads(const std::vector<Item>& prims, double lo[3], double hi[3]) const {
  if (prims.size() != 6) return false;
  int cnt[3] = {0, 0, 0};
  for (const Item& it : prims) {
    if (etype(it.entry) != E_QUAD || !aligned_[epay(it.entry)]) return false;
    const int A = kPermAxes[aligned_[epay(it.entry)] - 1][0];
    const double plane = quads_[epay(it.entry)].q[A];
    if (cnt[A] == 0) lo[A] = hi[A] = plane;
    lo[A] = std::min(lo[A], plane);
    hi[A] = std::max(hi[A], plane);
    cnt[A]++;
  }
  for (int k = 0; k < 3; k++)
    if (cnt[k] != 2 || !(lo[k] < hi[k])) return false;
  int faces = 0;
  for (const Item& it : prims) {
    const uint32_t i = epay(it.entry);
    const int* ax = kPermAxes[aligned_[i] - 1];  // A, axis of u, axis of v
    const double q[3] = {quads_[i].q[0], quads_[i].q[1], quads_[i].q[2]};
    const double u0 = std::min(q[ax[1]], q[ax[1]] + qu_[i]), u1 = std::max(q[ax[1]], q[ax[1]] + qu_[i]);
    const double v0 = std::min(q[ax[2]], q[ax[2]] + qv_[i]), v1 = std::max(q[ax[2]], q[ax[2]] + qv_[i]);
    if (u0 != lo[ax[1]] || u1 != hi[ax[1]] || v0 != lo[ax[2]] || v1 != hi[ax[2]]) return false;
    faces |= 1 << (2 * ax[0] + (q[ax[0]] == hi[ax[0]] ? 1 : 0));
  }
  return faces == 63;
}

// The wide BVH of rt_scene.h (fp32 kernels) over world-level primitives: a binned SAH binary
// tree, collapsed into 4-wide nodes by repeatedly opening the child of largest surface area.
// Leaves hold their primitives' records in leaf order (no reference list). Closest hits do not
// depend on the tree except on exact-t ties, as for the binary BVH.
bool Compiler::wide_bvh(const std::vector<Item>& all, CompiledScene* out) {
  // Primitives whose box covers a large part of the scene (the RTOW ground sphere, r = 1000) would
  // sit in a leaf that almost every ray reaches, beside leaves of small primitives whose tests
  // diverge from it. They are tested first, by every lane alike, before the tree (whose traversal
  // then starts with their hit distance as its bound).
  std::vector<Item> prims, big;
  {
    Box scene;
    for (const Item& it : all) scene.grow(it.box);
    const double sa = scene.area();
    for (const Item& it : all)
      (sa > 0 && it.box.area() > 0.25 * sa && big.size() < 4 ? big : prims).push_back(it);
    if (prims.size() < 2) {
      prims = all;
      big.clear();
    }
  }
  struct BN {
    Box box;
    int left = -1, right = -1;  // children (inner), or -1
    size_t first = 0, count = 0;  // primitive range (leaf)
  };
  std::vector<BN> bn;
  std::vector<size_t> order(prims.size());
  for (size_t i = 0; i < order.size(); i++) order[i] = i;
  std::vector<double> cen(prims.size() * 3);
  for (size_t i = 0; i < prims.size(); i++)
    for (int k = 0; k < 3; k++) cen[3 * i + k] = prims[i].box.center(k);
  // binary build, iterative (meshes are deep); SAH with a node traversal cost of 1 primitive test
  constexpr int kBins = 32;
  // leaves of up to kWLeafMax primitives, kWLeafMaxSpheres when all are spheres (a sphere test is
  // cheap next to a node visit; C3: leaves of 1/2/3/4/5/6/7/8 spheres 82.8/69.2/71.9/66.3/64.9/
  // 64.0/66.2/67.8 ms/frame; C4's triangles in HBM: 4 -> 742, 6 -> 817). A SAH leaf test on top
  // (node cost 1-8 primitive tests) was no better than the fixed sizes.
  bool all_spheres = true;
  for (const Item& it : prims) all_spheres = all_spheres && etype(it.entry) == E_SPHERE;
  size_t leaf_max = (size_t)(all_spheres ? kWLeafMaxSpheres : kWLeafMax);  // triangles: 3 (r03j C4 357.9 vs 362.7)
  if (const char* v = std::getenv("RT_DEV_WIDE_LEAF")) leaf_max = (size_t)std::max(1, std::min(8, std::atoi(v)));
  // split planes: binned SAH over all three axes (C4's triangles: 743 -> 458 ms/frame against the
  // largest centroid extent only), but the largest axis only for sphere trees (C3: 64.2 vs 65.1)
  int sah_axes = all_spheres ? 1 : 3;
  if (const char* v = std::getenv("RT_DEV_WIDE_AXES")) sah_axes = std::atoi(v);
  bn.push_back(BN{});
  bn[0].first = 0;
  bn[0].count = prims.size();
  std::vector<int> todo{0};
  while (!todo.empty()) {
    const int ni = todo.back();
    todo.pop_back();
    const size_t b = bn[(size_t)ni].first, n = bn[(size_t)ni].count, e = b + n;
    Box bounds, cb;
    for (size_t i = b; i < e; i++) {
      bounds.grow(prims[order[i]].box);
      cb.grow(&cen[3 * order[i]]);
    }
    bn[(size_t)ni].box = bounds;
    if (n <= leaf_max) continue;  // a leaf: one 4-wide node's worth of tests
    int axis = 0;
    for (int k = 1; k < 3; k++)
      if (cb.hi[k] - cb.lo[k] > cb.hi[axis] - cb.lo[axis]) axis = k;
    size_t mid = b + n / 2;
    bool split = false;
    // binned SAH over every axis with a centroid extent (or the largest one only: sah_axes = 1)
    double best = kInf;
    int best_k = -1, best_axis = axis;
    for (int ax = 0; ax < 3; ax++) {
      if (sah_axes == 1 && ax != axis) continue;
      const double extent = cb.hi[ax] - cb.lo[ax];
      if (!(extent > 0)) continue;
      Box bin_box[kBins];
      size_t bin_cnt[kBins] = {};
      for (size_t i = b; i < e; i++) {
        const size_t p = order[i];
        const int k = std::min(kBins - 1, std::max(0, (int)((cen[3 * p + ax] - cb.lo[ax]) / extent * kBins)));
        bin_cnt[k]++;
        bin_box[k].grow(prims[p].box);
      }
      Box rb[kBins];
      size_t rc[kBins] = {};
      Box acc;
      size_t cnt = 0;
      for (int k = kBins - 1; k > 0; k--) {
        acc.grow(bin_box[k]);
        cnt += bin_cnt[k];
        rb[k] = acc;
        rc[k] = cnt;
      }
      Box lb;
      size_t lc = 0;
      for (int k = 1; k < kBins; k++) {
        lb.grow(bin_box[k - 1]);
        lc += bin_cnt[k - 1];
        if (!lc || !rc[k]) continue;
        const double cost = lb.area() * (double)lc + rb[k].area() * (double)rc[k];
        if (cost < best) {
          best = cost;
          best_k = k;
          best_axis = ax;
        }
      }
    }
    if (best_k > 0) {
      axis = best_axis;
      const double extent = cb.hi[axis] - cb.lo[axis];
      auto it = std::partition(order.begin() + (long)b, order.begin() + (long)e, [&](size_t p) {
        return std::min(kBins - 1, std::max(0, (int)((cen[3 * p + axis] - cb.lo[axis]) / extent * kBins))) < best_k;
      });
      mid = (size_t)(it - order.begin());
      split = mid > b && mid < e;
    }
    if (!split) {
      mid = b + n / 2;
      std::nth_element(order.begin() + (long)b, order.begin() + (long)mid, order.begin() + (long)e,
                       [&](size_t x, size_t y) { return cen[3 * x + axis] < cen[3 * y + axis]; });
    }
    const int l = (int)bn.size(), r = l + 1;
    bn.push_back(BN{});
    bn.push_back(BN{});
    bn[(size_t)l].first = b;
    bn[(size_t)l].count = mid - b;
    bn[(size_t)r].first = mid;
    bn[(size_t)r].count = e - mid;
    bn[(size_t)ni].left = l;
    bn[(size_t)ni].right = r;
    todo.push_back(r);
    todo.push_back(l);
  }

  // primitive records in leaf order
  struct W4 {
    float x, y, z, w;
  };
  std::vector<W4> words;
  // the same stream in double for the fp64 blob (fp64 rays over the same float boxes, rt_device.h
  // trace_wide): word for word, so the leaf codes serve both; the entry in the low bits of w
  struct W8 {
    double x, y, z, w;
  };
  std::vector<W8> words64;
  uint32_t kinds = 0;
  auto bits = [](uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
  };
  auto bits64 = [](uint32_t u) {
    const uint64_t v = u;
    double f;
    std::memcpy(&f, &v, 8);
    return f;
  };
  auto put_prim = [&](uint32_t e) {  // the record of one primitive (rt_scene.h WNode)
    const uint32_t ix = epay(e);
    auto put = [&](const double* v, double w, bool entry) {
      words.push_back({(float)v[0], (float)v[1], (float)v[2], entry ? bits(e) : (float)w});
      words64.push_back({v[0], v[1], v[2], entry ? bits64(e) : w});
    };
    if (etype(e) == E_SPHERE) {
      const Sphere<double>& s = spheres_[ix];
      kinds |= WK_SPHERE | (s.moving ? WK_MOVING : 0u);
      put(s.c1, 0, true);
      put(s.dc, s.r, false);
    } else if (etype(e) == E_TRI) {
      const Tri<double>& t = tris_[ix];
      kinds |= WK_TRI;
      put(t.p0, 0, true);
      put(t.e1, 0, false);
      put(t.e2, 0, false);
    } else if (etype(e) == E_QUAD) {
      const Quad<double>& q = quads_[ix];
      kinds |= WK_QUAD;
      put(q.q, 0, true);
      put(q.n, q.D, false);
      put(q.a, 0, false);
      put(q.b, 0, false);
    } else {
      return false;
    }
    return true;
  };
  for (const Item& it : big)
    if (!put_prim(it.entry)) return false;
  // a leaf's words are emitted once; the 8-wide tree below refers to the same words
  std::vector<int64_t> leaf_memo(bn.size(), -1);
  auto leaf_code = [&](int b, uint32_t& code) {
    if (leaf_memo[(size_t)b] >= 0) {
      code = (uint32_t)leaf_memo[(size_t)b];
      return true;
    }
    const BN& nd = bn[(size_t)b];
    const size_t first = words.size();
    if (nd.count == 0 || nd.count > 64 || first > kWFirstMask) return false;
    for (size_t i = nd.first; i < nd.first + nd.count; i++)
      if (!put_prim(prims[order[i]].entry)) return false;
    code = kWLeaf | (uint32_t)(nd.count - 1) << kWCountShift | (uint32_t)first;
    leaf_memo[(size_t)b] = code;
    return true;
  };
  // the children of binary node b in a `width`-wide node: open the child of largest area until full
  auto collapse = [&](int b, size_t width) {
    const BN& nd = bn[(size_t)b];
    std::vector<int> ch{nd.left, nd.right};
    while (ch.size() < width) {
      int pick = -1;
      double best = -1;
      for (size_t k = 0; k < ch.size(); k++) {
        const BN& c = bn[(size_t)ch[k]];
        if (c.left >= 0 && c.box.area() > best) {
          best = c.box.area();
          pick = (int)k;
        }
      }
      if (pick < 0) break;
      const BN& c = bn[(size_t)ch[(size_t)pick]];
      const int l = c.left, r = c.right;
      ch[(size_t)pick] = l;
      ch.insert(ch.begin() + pick + 1, r);
    }
    return ch;
  };
  std::vector<WNode> wn;
  // collapse: node of binary node `b` -> its index; stack need returned through `need`
  std::function<bool(int, uint32_t&, int&)> emit = [&](int b, uint32_t& code, int& need) -> bool {
    const BN& nd = bn[(size_t)b];
    if (nd.left < 0) {
      need = 0;
      return leaf_code(b, code);
    }
    const std::vector<int> ch = collapse(b, 4);
    const size_t idx = wn.size();
    if (idx >= kWLeaf) return false;
    wn.emplace_back();
    const float inf = std::numeric_limits<float>::infinity();
    for (int c = 0; c < 4; c++) {
      wn[idx].lox[c] = wn[idx].loy[c] = wn[idx].loz[c] = inf;
      wn[idx].hix[c] = wn[idx].hiy[c] = wn[idx].hiz[c] = inf;
      wn[idx].child[c] = kWLeaf;
    }
    int sub = 0;
    for (size_t c = 0; c < ch.size(); c++) {
      uint32_t cc;
      int cn;
      if (!emit(ch[c], cc, cn)) return false;
      sub = std::max(sub, cn);
      const Box& bx = bn[(size_t)ch[c]].box;
      WNode& w = wn[idx];
      w.lox[c] = down(bx.lo[0]);
      w.loy[c] = down(bx.lo[1]);
      w.loz[c] = down(bx.lo[2]);
      w.hix[c] = up(bx.hi[0]);
      w.hiy[c] = up(bx.hi[1]);
      w.hiz[c] = up(bx.hi[2]);
      w.child[c] = cc;
    }
    need = (int)ch.size() - 1 + sub;
    code = (uint32_t)idx;
    return true;
  };
  uint32_t root;
  int need;
  const bool ok = emit(0, root, need);
  // The top of the tree first (round 5): the nodes of the first levels, in breadth-first order, take
  // indices [0, top) -- kernels over a tree in HBM keep them in LDS (every ray visits them) -- and the rest
  // keep their depth-first order (subtrees contiguous). The deepest level that fits kWideTopMax nodes.
  uint32_t top = 0;
  if (ok && !(root & kWLeaf) && wn.size() > 1) {
    std::vector<uint32_t> bfs{root}, level{root};
    std::vector<uint32_t> chosen;
    for (int depth = 0; depth < 8 && !level.empty(); depth++) {
      if (bfs.size() > kWideTopMax) break;
      chosen = bfs;
      std::vector<uint32_t> next;
      for (uint32_t n : level)
        for (int c = 0; c < 4; c++)
          if (!(wn[n].child[c] & kWLeaf)) next.push_back(wn[n].child[c]);
      bfs.insert(bfs.end(), next.begin(), next.end());
      level.swap(next);
    }
    top = (uint32_t)chosen.size();
    std::vector<uint32_t> perm(wn.size(), 0xFFFFFFFFu);
    uint32_t k = 0;
    for (uint32_t n : chosen) perm[n] = k++;
    for (uint32_t n = 0; n < wn.size(); n++)
      if (perm[n] == 0xFFFFFFFFu) perm[n] = k++;
    std::vector<WNode> re(wn.size());
    for (uint32_t n = 0; n < wn.size(); n++) {
      WNode w = wn[n];
      for (int c = 0; c < 4; c++)
        if (!(w.child[c] & kWLeaf)) w.child[c] = perm[w.child[c]];
      re[perm[n]] = w;
    }
    wn.swap(re);
    root = perm[root];
  }
  if (std::getenv("RT_DEBUG_WIDE"))
    std::fprintf(stderr, "[wide] ok %d need %d nodes %zu words %zu binary nodes %zu\n", (int)ok, need, wn.size(),
                 words.size(), bn.size());
  if (!ok || need > kWideStackMax) return false;
  // the HBM kernels address nodes and primitive words by 32-bit byte offsets from the tree's base (fp32
  // rays: node * sizeof(WNode), word * 16; fp64 rays: node * sizeof(WNodeH), word * 32): a tree past 4 GiB
  // (~40 M nodes) takes the binary BVH instead
  if ((uint64_t)wn.size() * std::max(sizeof(WNode), sizeof(WNodeH)) >= (1ull << 32) ||
      ((uint64_t)words.size() + 2) * 32u >= (1ull << 32))
    return false;

  // two zero words past the last record: kernels with triangles read a record's next two words with
  // its first (trace_wide test_prims), past the end for a trailing sphere
  words.push_back({0.f, 0.f, 0.f, 0.f});
  words.push_back({0.f, 0.f, 0.f, 0.f});
  words64.push_back({0, 0, 0, 0});
  words64.push_back({0, 0, 0, 0});
  const std::vector<WNodeH> wh = half_nodes(wn);
  {  // the fp64 blob: the same float nodes, the double words
    SceneHeader& h = out->hdr64;
    h.off_wnodes = append(out->blob64, wn);
    h.off_wnodesh = append(out->blob64, wh);
    h.has_wnodesh = 1;
    h.off_wprims = append(out->blob64, words64);
    out->blob64.resize((out->blob64.size() + 255) & ~size_t(255));
    h.bytes = out->blob64.size();
    h.n_wnodes = (uint32_t)wn.size();
    h.n_wprim_words = (uint32_t)words64.size();
    h.wroot = root;
    h.wide_stack = (uint32_t)std::max(1, need);
    h.wide_kinds = kinds;
    h.wide_big = (uint32_t)big.size();
    h.wide_top = top;
    h.has_wide = 1;
  }
  SceneHeader& h = out->hdr;
  h.off_wnodes = append(out->blob32, wn);
  h.has_wnodesh = 0;  // only fp64 rays read the fp16 form (RT_WIDE_HALF_F64): it stays out of the fp32 blob
  h.off_wprims = append(out->blob32, words);
  out->blob32.resize((out->blob32.size() + 255) & ~size_t(255));
  h.bytes = out->blob32.size();
  h.n_wnodes = (uint32_t)wn.size();
  h.n_wprim_words = (uint32_t)words.size();
  h.wroot = root;
  h.wide_stack = (uint32_t)std::max(1, need);
  h.wide_kinds = kinds;
  h.wide_big = (uint32_t)big.size();
  h.wide_top = top;
  h.has_wide = 1;
  return true;
}

bool Compiler::run(CompiledScene* out, std::string* err) {
  if (!d_) {
    *err = "null scene descriptor";
    return false;
  }
  // textures (texture.h:12-63) and materials (material.h:57-219)
  for (int i = 0; i < d_->num_textures; i++) {
    const rt_texture& t = d_->textures[i];
    Texture<double> r{};
    if (t.kind == RT_TEX_SOLID) {
      r.kind = T_SOLID;
      for (int k = 0; k < 3; k++) r.c0[k] = t.color[k];
    } else if (t.kind == RT_TEX_CHECKER) {
      r.kind = T_CHECKER;
      for (int k = 0; k < 3; k++) {
        r.c0[k] = t.odd[k];
        r.c1[k] = t.even[k];
      }
      r.scale = t.scale;
    } else if (t.kind == RT_TEX_PERLIN) {  // texture.h:80-92: the tables perlin's constructor drew
      const int64_t need = 3 * kPerlinPoints + 3 * kPerlinPoints;  // rand_offset, perm_x, perm_y, perm_z
      if (!d_->tex_data || t.data < 0 || (int64_t)t.data + need > d_->num_tex_data) {
        *err = "perlin texture " + std::to_string(i) + ": tex_data too short";
        return false;
      }
      const double* src = d_->tex_data + t.data;
      r.kind = T_PERLIN;
      r.scale = t.scale;
      r.data = (uint32_t)texdata_.size();
      texdata_.insert(texdata_.end(), src, src + 3 * kPerlinPoints);  // rand_offset
      for (uint32_t k = 0; k < kPerlinPoints; k++) {  // perm_x: the only one noise.h:36 reads
        const double v = src[3 * kPerlinPoints + k];
        if (!(v >= 0 && v < kPerlinPoints)) {
          *err = "perlin texture " + std::to_string(i) + ": permutation entry out of range";
          return false;
        }
        texdata_.push_back(v);
      }
    } else if (t.kind == RT_TEX_VALUE) {  // texture.h:95-103: n^3 values
      const double n = t.scale;
      if (!(n >= 1 && n <= 1024 && n == (double)(int64_t)n) || !d_->tex_data || t.data < 0 ||
          (int64_t)t.data + (int64_t)(n * n * n) > d_->num_tex_data) {
        *err = "value texture " + std::to_string(i) + ": bad resolution or tex_data too short";
        return false;
      }
      r.kind = T_VALUE;
      r.n = (uint32_t)n;
      r.data = (uint32_t)texdata_.size();
      texdata_.insert(texdata_.end(), d_->tex_data + t.data, d_->tex_data + t.data + (int64_t)(n * n * n));
    } else if (t.kind == RT_TEX_IMAGE) {  // texture.h:65-78: width x height RGB bytes
      const double w = t.color[0], hh = t.color[1];
      if (!(w >= 0 && hh >= 0 && w == (double)(int64_t)w && hh == (double)(int64_t)hh && w * hh <= 1e9) ||
          (w * hh > 0 && (!d_->image_data || t.data < 0 || (int64_t)t.data + (int64_t)(w * hh * 3) > d_->num_image_data))) {
        *err = "image texture " + std::to_string(i) + ": bad size or image_data too short";
        return false;
      }
      r.kind = T_IMAGE;
      r.n = (uint32_t)w;
      r.h = (uint32_t)hh;
      r.data = (uint32_t)images_.size();
      if (w * hh > 0) images_.insert(images_.end(), d_->image_data + t.data, d_->image_data + t.data + (int64_t)(w * hh * 3));
      cell_noise_ = true;  // EXT kernels
    } else if (t.kind == RT_TEX_WORLEY || t.kind == RT_TEX_VORONOI) {  // stateless (noise.h:139-201)
      r.kind = t.kind == RT_TEX_WORLEY ? T_WORLEY : T_VORONOI;
      cell_noise_ = true;
    } else {
      *err = "texture kind " + std::to_string(t.kind) + " is not implemented on the device";
      return false;
    }
    texs_.push_back(r);
  }
  for (int i = 0; i < d_->num_materials; i++) {
    const rt_material& m = d_->materials[i];
    if (m.texture < 0 || m.texture >= d_->num_textures) {
      *err = "material " + std::to_string(i) + " has no valid texture";
      return false;
    }
    if (m.kind < RT_MAT_LAMBERTIAN || m.kind > RT_MAT_GLOSS) {
      *err = "material kind " + std::to_string(m.kind) + " is not implemented on the device";
      return false;
    }
    // gloss: interval(0, 1).clamp(smoothness) (material.h:149, interval.h) -- NaN passes through
    const float sm = m.smoothness < 0.f ? 0.f : (m.smoothness > 1.f ? 1.f : m.smoothness);
    Material<double> r{m.kind, m.texture, (double)m.fuzz, (double)m.refraction, (double)sm,
                       (double)m.specular_prob, {0, 0}, texs_[m.texture]};
    // value-identical materials share one record (main.cc:476-484 gives each of Sponza's
    // 262k triangles its own lambertian(solid_color(1))): the key is everything shading reads
    std::string key;
    auto put = [&key](const void* p, size_t n) { key.append((const char*)p, n); };
    put(&r.kind, 4);
    put(&r.fuzz, 8);
    put(&r.refr, 8);
    put(&r.smooth, 8);
    put(&r.spec, 8);
    put(&r.tx.kind, 4);
    put(r.tx.c0, 24);
    put(r.tx.c1, 24);
    put(&r.tx.scale, 8);
    put(&r.tx.data, 4);
    put(&r.tx.n, 4);
    put(&r.tx.h, 4);
    auto it = mat_index_.find(key);
    if (it == mat_index_.end()) {
      it = mat_index_.emplace(key, (int32_t)mats_.size()).first;
      mats_.push_back(r);
    }
    mat_remap_.push_back(it->second);
  }
  if (d_->background >= d_->num_textures) {
    *err = "background texture out of range";
    return false;
  }
  std::vector<Item> top;
  gather(d_->world, {}, top, false);
  if (ok_) light_from(d_->light);
  if (!ok_) {
    *err = err_;
    return false;
  }
  // the world object itself decides ordering: a list stays a list when it holds a volume or is small
  const rt_object* w = &d_->objects[d_->world];
  bool ordered = (w->kind == RT_OBJ_LIST);
  Item root;
  if (top.empty()) {
    root = list_of(top);
  } else if (ordered) {
    root = container(top, false);
  } else {
    root = top.size() == 1 ? top[0] : bvh(top, 0, top.size(), 0);
  }
  if (root.need + 1 > kStackDepth) {
    *err = "scene needs a deeper traversal stack than the device provides";
    return false;
  }
  Item lin_top;
  join_lin(lin_top, top);
  std::vector<LinRec<double>> linear;
  if (lin_top.lin_ok)
    for (uint32_t op : lin_top.lin) linear.push_back(lin_record(op));
  // the flat program of both blobs, when the linear program has that form (may add quad records)
  std::vector<FlatQuadT<double>> fq;
  std::vector<FlatBoxT<double>> fb;
  uint32_t nq[3] = {0, 0, 0};
  out->desc_quads = (int)quads_.size();
  const bool has_flat = lin_top.lin_ok && !lin_top.lin.empty() && flat_program(lin_top.lin, fq, nq, fb);
  if (has_flat) {
    for (const FlatQuadT<double>& q : fq) out->flat_quads += q.inst != -2;
    out->flat_boxes = (int)fb.size();
  }
  out->stack_need = std::max(1, root.need);
  out->bvh_depth = root.depth;
  out->num_items = (int)top.size();
  out->hdr64 =
      pack(out->blob64, quads_, spheres_, tris_, insts_, vols_, nodes_, refs_, mats_, texs_, light_, linear, texdata_, images_);
  out->hdr = pack(out->blob32, map32(quads_), map32(spheres_), map32(tris_), map32(insts_), map32(vols_),
                  map32(nodes_), refs_, map32(mats_), map32(texs_), to32(light_), map32(linear), texdata_, images_);
  if (!quads_.empty()) {  // the fp32 quad test re-decides hits near an edge in fp64 (rt_device.h quad_t)
    out->hdr.off_quads64 = append(out->blob32, quads_);
    out->hdr.has_quads64 = 1;
    out->blob32.resize((out->blob32.size() + 255) & ~size_t(255));
    out->hdr.bytes = out->blob32.size();
  }
  if (has_flat) {
    std::vector<FlatQuadT<float>> fq32;
    std::vector<FlatBoxT<float>> fb32;
    for (const FlatQuadT<double>& q : fq)
      fq32.push_back({(float)q.plane, (float)q.lo_u, (float)q.lo_w, (float)q.inv_u, (float)q.inv_w, q.e, q.inst, q.nm});
    for (const FlatBoxT<double>& b : fb) {
      FlatBoxT<float> r{};
      for (int k = 0; k < 3; k++) {
        r.lo[k] = (float)b.lo[k];
        r.hi[k] = (float)b.hi[k];
      }
      r.inst = b.inst;
      r.mat = b.mat;
      for (int f = 0; f < 6; f++) r.face[f] = b.face[f];
      r.neg = b.neg;
      fb32.push_back(r);
    }
    auto put = [&](std::vector<unsigned char>& blob, SceneHeader& h, const auto& q, const auto& b) {
      h.off_flat_quad = append(blob, q);
      h.off_flat_box = append(blob, b);
      blob.resize((blob.size() + 255) & ~size_t(255));
      h.bytes = blob.size();
      for (int a = 0; a < 3; a++) h.n_flat_quad[a] = nq[a];
      h.n_flat_box = (uint32_t)b.size();
      h.has_flat = 1;
    };
    put(out->blob32, out->hdr, fq32, fb32);
    put(out->blob64, out->hdr64, fq, fb);
  }
  // the wide BVH (fp32) when the world is a BVH over world-level primitives only
  bool prims_only = etype(root.entry) == E_NODE;
  for (const Item& it : top) prims_only = prims_only && etype(it.entry) <= E_TRI;
  if (prims_only && !wide_bvh(top, out)) out->hdr.has_wide = out->hdr64.has_wide = 0;
  for (SceneHeader* h : {&out->hdr, &out->hdr64}) {
    h->has_cell_noise = cell_noise_ ? 1 : 0;
    h->root = root.entry;
    h->background = d_->background;
    h->has_volumes = vols_.empty() ? 0 : 1;
  }
  return true;
}

}  // namespace

rt_status compile_scene(const rt_scene_desc* desc, CompiledScene* out, std::string* err) {
  if (!desc || !out || !err) return RT_ERR_INVALID_ARGUMENT;
  if (desc->world < 0 || desc->world >= desc->num_objects) {
    *err = "world object index out of range";
    return RT_ERR_INVALID_ARGUMENT;
  }
  try {
    Compiler c(desc);
    if (!c.run(out, err)) return RT_ERR_UNSUPPORTED;
  } catch (const std::bad_alloc&) {
    *err = "out of host memory while compiling the scene";
    return RT_ERR_OUT_OF_MEMORY;
  } catch (const std::exception& e) {
    *err = std::string("scene compilation failed: ") + e.what();
    return RT_ERR_INVALID_ARGUMENT;
  }
  return RT_OK;
}

}  // namespace rtd
