// hittable_list.h (reference: src/hittable_list.h:7-37): an ordered list; the
// closest hit wins and, on equal t, the later object (kept on the device).
#pragma once
#include <memory>
#include <vector>

#include "hittable.h"

class hittable_list : public hittable {
 public:
  std::vector<std::shared_ptr<hittable>> objects;
  hittable_list() = default;
  hittable_list(std::shared_ptr<hittable> object) { push_back(std::move(object)); }
  void clear() { objects.clear(); }
  void push_back(std::shared_ptr<hittable> object) { objects.push_back(std::move(object)); }
  int flatten(scene_builder& sb) const override { return flatten_as(sb, RT_OBJ_LIST); }
  // hittable_list.h:20-31: every object in order against the shrinking interval, so the closest
  // hit wins and, on equal t, the later object
  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
    bool any = false;
    for (const auto& o : objects) {
      hit_record h;
      if (!o->hit(r, ray_t, h)) continue;
      any = true;
      ray_t.max = h.t;
      rec = h;
    }
    return any;
  }
  aabb get_bounding_box() const override {  // hittable_list.h:14-17: enclose of the members, in order
    aabb b;
    for (const auto& o : objects) b = aabb::enclose(b, o->get_bounding_box());
    return b;
  }

 protected:
  int flatten_as(scene_builder& sb, int32_t kind) const {
    std::vector<int> kids;
    kids.reserve(objects.size());
    for (const auto& o : objects) kids.push_back(sb.add(*o));
    rt_object o = scene_builder::blank(kind);
    o.first_child = sb.emit_children(kids);
    o.child_count = (int32_t)kids.size();
    return sb.emit_object(o);
  }
};
