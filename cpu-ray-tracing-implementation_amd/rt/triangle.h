// triangle.h (reference: src/triangle.h:17-56)
#pragma once
#include <memory>

#include "hittable.h"
#include "material.h"

class triangle : public hittable {
 public:
  triangle(vec3 p0, vec3 p1, vec3 p2, std::shared_ptr<material> mat) : p0_(p0), p1_(p1), p2_(p2), mat_(std::move(mat)) {}
  int flatten(scene_builder& sb) const override {
    if (!mat_) throw unsupported_object("triangle without a material");
    rt_object o = scene_builder::blank(RT_OBJ_TRIANGLE);
    o.material = sb.add_material(*mat_);
    scene_builder::put3(o.a, p0_);
    scene_builder::put3(o.b, p1_);
    scene_builder::put3(o.c, p2_);
    return sb.emit_object(o);
  }
  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {  // triangle.h:30-40 (u, v untouched)
    const double t = rt_host::triangle_root(p0_, p1_, p2_, r, ray_t);
    if (std::isnan(t)) return false;
    rec.t = t;
    rec.p = r.at(t);
    rec.set_face_normal(r, unit_vector(cross(p1_ - p0_, p2_ - p0_)));
    rec.mat = mat_;
    return true;
  }
  aabb get_bounding_box() const override {  // triangle.h:42-48
    point3 lo, hi;
    for (int k = 0; k < 3; k++) {
      lo[k] = std::fmin(p0_[k], std::fmin(p1_[k], p2_[k]));
      hi[k] = std::fmax(p0_[k], std::fmax(p1_[k], p2_[k]));
    }
    return aabb(lo, hi);
  }

 private:
  vec3 p0_, p1_, p2_;
  std::shared_ptr<material> mat_;
};
