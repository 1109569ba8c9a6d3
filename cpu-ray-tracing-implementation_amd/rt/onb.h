// onb.h (reference: src/onb.h:4-29): orthonormal basis with y along the normal.
#pragma once
#include <cmath>

#include "vec3.h"

class frame {
 public:
  vec3 transform(vec3 v) const { return v.x() * x + v.y() * y + v.z() * z; }
  vec3 x, y, z, o;
};

class onb : public frame {
 public:
  onb(const vec3& n) {
    y = unit_vector(n);
    vec3 a = std::fabs(y.x()) > 0.9 ? vec3(0, 0, 1) : vec3(1, 0, 0);
    z = unit_vector(cross(y, a));
    x = cross(y, z);
  }
};
