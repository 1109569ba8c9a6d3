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

 private:
  vec3 p0_, p1_, p2_;
  std::shared_ptr<material> mat_;
};
