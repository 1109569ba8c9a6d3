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

 private:
  point3 c1_, c2_;
  double radius_;
  std::shared_ptr<material> mat_;
  bool moving_ = false;
};
