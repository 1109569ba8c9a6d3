// sphere.h (reference: src/sphere.h:4-107). Three constructors as in the
// reference; the moving one keeps the reference's normal from center_ = (0,0,0)
// (sphere.h:69), see DESIGN.md §Quirks.
#pragma once
#include <algorithm>
#include <memory>

#include "hittable.h"
#include "material.h"

class sphere : public hittable {
 public:
  sphere(point3 center, double radius, std::shared_ptr<material> mat)
      : c1_(center), c2_(center), radius_(std::max(0.0, radius)), mat_(std::move(mat)) {}
  sphere(double radius, std::shared_ptr<material> mat) : sphere(point3(0), radius, std::move(mat)) {}
  sphere(point3 center1, point3 center2, double radius, std::shared_ptr<material> mat)
      : c1_(center1), c2_(center2), radius_(std::max(0.0, radius)), mat_(std::move(mat)), moving_(true) {}
  int flatten(scene_builder& sb) const override {
    if (!mat_) throw unsupported_object("sphere without a material");
    rt_object o = scene_builder::blank(RT_OBJ_SPHERE);
    o.material = sb.add_material(*mat_);
    scene_builder::put3(o.a, c1_);
    scene_builder::put3(o.b, c2_);
    o.s0 = radius_;
    o.moving = moving_ ? 1 : 0;
    return sb.emit_object(o);
  }
  // sphere.h:40-74: the moving sphere intersects at its centre for the ray's time but, as in the
  // reference, takes the normal from center_ (never set by that constructor: the origin)
  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
    const point3 c = moving_ ? c1_ + r.time() * (c2_ - c1_) : c1_;
    const double t = rt_host::sphere_root(c, radius_, r, ray_t);
    if (std::isnan(t)) return false;
    rec.t = t;
    rec.p = r.at(t);
    const vec3 outward = (rec.p - normal_center()) / radius_;
    rt_host::sphere_uv(outward, rec.u, rec.v);
    rec.set_face_normal(r, outward);
    rec.mat = mat_;
    return true;
  }
  aabb get_bounding_box() const override {
    const vec3 rv(radius_);
    const aabb b1(c1_ - rv, c1_ + rv);
    return moving_ ? aabb::enclose(b1, aabb(c2_ - rv, c2_ + rv)) : b1;
  }
  double pdf_value(const point3& origin, const vec3&) const override {  // sphere.h:76-78
    return radius_ * radius_ * pi / (origin - normal_center()).length_squared();
  }
  vec3 random(const point3&) const override { return random_in_unit_sphere() * radius_; }  // sphere.h:80-81

 private:
  point3 c1_, c2_;
  double radius_;
  std::shared_ptr<material> mat_;
  bool moving_ = false;
  point3 normal_center() const { return moving_ ? point3(0) : c1_; }
};
