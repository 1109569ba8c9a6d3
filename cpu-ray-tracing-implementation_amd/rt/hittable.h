// hittable.h -- the hittable interface and the translate / rotate_x/y/z
// wrappers (reference: src/hittable.h:7-293). Ray queries run on the device;
// on the host every hittable only knows how to flatten itself into the
// scene descriptor (scene_builder) that camera::render hands to librt_hip.
#pragma once
#include <memory>

#include "aabb.h"
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
  // The host does not answer ray queries (they run on the device); kept so subclasses still compile.
  virtual bool hit(const ray&, interval, hit_record&) const { return false; }
  virtual aabb get_bounding_box() const { return aabb(); }
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
  }
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
};
using rotate_x = rotate_axis<RT_OBJ_ROTATE_X>;
using rotate_y = rotate_axis<RT_OBJ_ROTATE_Y>;
using rotate_z = rotate_axis<RT_OBJ_ROTATE_Z>;
