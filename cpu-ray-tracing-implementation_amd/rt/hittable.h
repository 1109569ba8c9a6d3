// hittable.h -- the hittable interface and the translate / rotate_x/y/z
// wrappers (reference: src/hittable.h:7-293). Ray queries run on the device;
// on the host every hittable only knows how to flatten itself into the
// scene descriptor (scene_builder) that camera::render hands to librt_hip.
#pragma once
#include <memory>

#include "aabb.h"
#include "host_geometry.h"
#include "interval.h"
#include "ray.h"
#include "scene_builder.h"

class material;

class hit_record {  // hittable.h:7-30 (kept for source compatibility)
 public:
  point3 p;
  vec3 normal;
  double t = 0, u = 0, v = 0;
  bool front_face = false;
  std::shared_ptr<material> mat;
  void set_face_normal(const ray& r, const vec3& outward) {
    front_face = dot(r.direction(), outward) < 0.0;
    normal = front_face ? outward : -outward;
  }
};

class hittable {
 public:
  virtual ~hittable() = default;
  // Serialise this object (and what it wraps) into the descriptor; returns its object index.
  // A user subclass that does not implement it makes camera::render fail with unsupported_object.
  virtual int flatten(scene_builder&) const {
    throw unsupported_object("hittable type has no device representation (flatten not implemented)");
  }
  // Host-side queries (host_geometry.h; renders trace every ray on the device). As in the
  // reference, a subclass must answer hit and get_bounding_box; pdf_value / random default to
  // the base class's 0 and (1, 0, 0) (hittable.h:39-41).
  virtual bool hit(const ray& r, interval ray_t, hit_record& rec) const = 0;
  virtual aabb get_bounding_box() const = 0;
  virtual double pdf_value(const point3&, const vec3&) const { return 0.0; }
  virtual vec3 random(const point3&) const { return vec3(1, 0, 0); }
};

inline int scene_builder::add(const hittable& h) {
  auto it = seen_obj_.find(&h);
  if (it != seen_obj_.end()) return it->second;
  int idx = h.flatten(*this);
  seen_obj_[&h] = idx;
  return idx;
}

class translate : public hittable {  // hittable.h:67-89
 public:
  translate(vec3 offset, std::shared_ptr<hittable> object) : object_(std::move(object)), offset_(offset) {}
  int flatten(scene_builder& sb) const override {
    int child = sb.add(*object_);
    rt_object o = scene_builder::blank(RT_OBJ_TRANSLATE);
    o.child = child;
    scene_builder::put3(o.a, offset_);
    return sb.emit_object(o);
  }
  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {  // hittable.h:75-82
    if (!object_->hit(ray(r.origin() - offset_, r.direction(), r.time()), ray_t, rec)) return false;
    rec.p += offset_;
    return true;
  }
  aabb get_bounding_box() const override { return object_->get_bounding_box().offset(offset_); }

 private:
  std::shared_ptr<hittable> object_;
  vec3 offset_;
};

// rotate_x / rotate_y / rotate_z (hittable.h:93-293): sin and cos of the angle, as the reference computes them
template <int32_t Kind>
class rotate_axis : public hittable {
 public:
  rotate_axis(std::shared_ptr<hittable> object, double angle) : object_(std::move(object)) {
    double r = degrees_to_radians(angle);
    sin_theta_ = std::sin(r);
    cos_theta_ = std::cos(r);
    // the object's box turned into world space, corner by corner
    const aabb in = object_->get_bounding_box();
    point3 lo(infinity), hi(-infinity);
    for (int i = 0; i < 8; i++) {
      const point3 c((i & 1) ? in.axis_interval(0).max : in.axis_interval(0).min,
                     (i & 2) ? in.axis_interval(1).max : in.axis_interval(1).min,
                     (i & 4) ? in.axis_interval(2).max : in.axis_interval(2).min);
      const vec3 w = rt_host::rotate<Kind - RT_OBJ_ROTATE_X>(c, sin_theta_, cos_theta_, false);
      for (int k = 0; k < 3; k++) {
        lo[k] = std::fmin(lo[k], w[k]);
        hi[k] = std::fmax(hi[k], w[k]);
      }
    }
    box_ = aabb(lo, hi);
  }
  // hittable.h:125-149 (x), 192-216 (y), 259-284 (z): the ray turned by -theta, the hit point and
  // normal turned back
  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
    constexpr int K = Kind - RT_OBJ_ROTATE_X;
    const ray local(rt_host::rotate<K>(r.origin(), sin_theta_, cos_theta_, true),
                    rt_host::rotate<K>(r.direction(), sin_theta_, cos_theta_, true), r.time());
    if (!object_->hit(local, ray_t, rec)) return false;
    rec.p = rt_host::rotate<K>(rec.p, sin_theta_, cos_theta_, false);
    rec.normal = rt_host::rotate<K>(rec.normal, sin_theta_, cos_theta_, false);
    return true;
  }
  aabb get_bounding_box() const override { return box_; }
  int flatten(scene_builder& sb) const override {
    int child = sb.add(*object_);
    rt_object o = scene_builder::blank(Kind);
    o.child = child;
    o.s0 = sin_theta_;
    o.s1 = cos_theta_;
    return sb.emit_object(o);
  }

 private:
  std::shared_ptr<hittable> object_;
  double sin_theta_, cos_theta_;
  aabb box_;
};
using rotate_x = rotate_axis<RT_OBJ_ROTATE_X>;
using rotate_y = rotate_axis<RT_OBJ_ROTATE_Y>;
using rotate_z = rotate_axis<RT_OBJ_ROTATE_Z>;
