// ray.h (reference: src/ray.h:3-17)
#pragma once
#include "vec3.h"

class ray {
 public:
  ray() = default;
  ray(const point3& o, const vec3& d, double time = 0) : orig_(o), dir_(d), tm_(time) {}
  const point3& origin() const { return orig_; }
  const vec3& direction() const { return dir_; }
  double time() const { return tm_; }
  point3 at(double t) const { return orig_ + t * dir_; }

 private:
  point3 orig_;
  vec3 dir_;
  double tm_ = 0;
};
