// bvh_node.h (reference: src/bvh_node.h:11-65). Constructed from a list like the reference;
// rendering flattens the list's objects and the device builds its own SAH BVH over them (the
// closest hit does not depend on the tree). Host queries (hit) walk the
// reference's own tree: objects sorted by their box's x minimum, split at the median, a single
// object duplicated into both children, left then right with the interval shrunk by a left hit.
#pragma once
#include <algorithm>
#include <vector>

#include "hittable_list.h"

class bvh_node : public hittable_list {
 public:
  bvh_node(hittable_list list) {
    objects = list.objects;  // flattened in the caller's order
    if (!objects.empty()) build(list.objects, 0, list.objects.size());
  }
  int flatten(scene_builder& sb) const override { return flatten_as(sb, RT_OBJ_BVH); }
  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {  // bvh_node.h:49-59
    if (!left_ || !box_.hit(r, ray_t)) return false;
    const bool hl = left_->hit(r, ray_t, rec);
    const bool hr = right_->hit(r, interval(ray_t.min, hl ? rec.t : ray_t.max), rec);
    return hl || hr;
  }
  aabb get_bounding_box() const override { return box_; }

 private:
  std::shared_ptr<hittable> left_, right_;
  aabb box_;
  bvh_node() = default;
  void build(std::vector<std::shared_ptr<hittable>>& v, size_t b, size_t e) {  // bvh_node.h:13-47
    std::sort(v.begin() + (long)b, v.begin() + (long)e, [](const auto& x, const auto& y) {
      return x->get_bounding_box().axis_interval(0).min < y->get_bounding_box().axis_interval(0).min;
    });
    const size_t n = e - b;
    if (n <= 2) {
      left_ = v[b];
      right_ = v[n == 1 ? b : b + 1];
    } else {
      const size_t mid = (b + e) / 2;
      auto l = std::shared_ptr<bvh_node>(new bvh_node());
      auto r = std::shared_ptr<bvh_node>(new bvh_node());
      l->build(v, b, mid);
      r->build(v, mid, e);
      left_ = l;
      right_ = r;
    }
    box_ = aabb::enclose(left_->get_bounding_box(), right_->get_bounding_box());
  }
};
