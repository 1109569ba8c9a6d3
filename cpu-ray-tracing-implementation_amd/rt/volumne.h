// volumne.h (reference: src/volumne.h:9-59, spelling kept): a constant-density
// medium inside a closed boundary, with an isotropic phase function.
#pragma once
#include <cmath>
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
  // volumne.h:18-46: entry and exit of the boundary, clamped to the interval, then an exponential
  // free-flight distance drawn from rand() inside the hit, as the reference does
  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
    hit_record in, out;
    if (!boundary_->hit(r, interval::universe, in)) return false;
    if (!boundary_->hit(r, interval(in.t + 0.0001, infinity), out)) return false;
    double t1 = in.t, t2 = out.t;
    if (t1 < ray_t.min) t1 = ray_t.min;
    if (t2 > ray_t.max) t2 = ray_t.max;
    if (t1 >= t2) return false;
    if (t1 < 0) t1 = 0;
    const double speed = r.direction().length();
    const double travel = -1.0 / density_ * std::log(random_double());
    if (travel > (t2 - t1) * speed) return false;
    rec.t = t1 + travel / speed;
    rec.p = r.at(rec.t);
    rec.normal = vec3(1, 0, 0);  // arbitrary, as the reference
    rec.front_face = true;
    rec.mat = phase_;
    return true;
  }
  aabb get_bounding_box() const override { return boundary_->get_bounding_box(); }

 private:
  std::shared_ptr<hittable> boundary_;
  double density_;
  std::shared_ptr<material> phase_;
};
