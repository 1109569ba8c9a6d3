// volumne.h (reference: src/volumne.h:9-59, spelling kept): a constant-density
// medium inside a closed boundary, with an isotropic phase function.
#pragma once
#include <memory>

#include "hittable.h"
#include "material.h"

class volumne : public hittable {
 public:
  volumne(std::shared_ptr<hittable> boundary, double density, std::shared_ptr<texture> tex)
      : boundary_(std::move(boundary)), density_(density), phase_(std::make_shared<isotropic>(std::move(tex))) {}
  int flatten(scene_builder& sb) const override {
    int child = sb.add(*boundary_);
    rt_object o = scene_builder::blank(RT_OBJ_VOLUME);
    o.child = child;
    o.s0 = density_;
    o.material = sb.add_material(*phase_);
    return sb.emit_object(o);
  }

 private:
  std::shared_ptr<hittable> boundary_;
  double density_;
  std::shared_ptr<material> phase_;
};
