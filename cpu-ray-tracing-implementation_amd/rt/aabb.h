// aabb.h -- axis-aligned box (reference: src/aabb.h:4-90). Kept for API
// compatibility (get_bounding_box); the device builds its own BVH boxes.
#pragma once
#include "host_geometry.h"
#include "interval.h"

class aabb {
 public:
  aabb() = default;
  aabb(interval x, interval y, interval z) : x_(x), y_(y), z_(z) { pad(); }
  aabb(const point3& a, const point3& b)
      : x_(a[0] <= b[0] ? interval(a[0], b[0]) : interval(b[0], a[0])),
        y_(a[1] <= b[1] ? interval(a[1], b[1]) : interval(b[1], a[1])),
        z_(a[2] <= b[2] ? interval(a[2], b[2]) : interval(b[2], a[2])) {}
  const interval& axis_interval(int n) const { return n == 1 ? y_ : (n == 2 ? z_ : x_); }
  static aabb enclose(const aabb& a, const aabb& b) {
    return aabb(interval::enclose(a.x_, b.x_), interval::enclose(a.y_, b.y_), interval::enclose(a.z_, b.z_));
  }
  aabb offset(const vec3& o) const { return aabb(x_.offset(o.x()), y_.offset(o.y()), z_.offset(o.z())); }
  bool hit(const ray& r, interval ray_t) const { return rt_host::slab_overlap(x_, y_, z_, r, ray_t); }  // aabb.h:28-33

 private:
  interval x_, y_, z_;
  void pad() {  // aabb.h:81-86
    for (interval* i : {&x_, &y_, &z_})
      if (i->size() < 0.0001) *i = i->expand(0.0001);
  }
};
