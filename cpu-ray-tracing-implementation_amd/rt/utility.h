// utility.h -- constants and the host random numbers scene construction uses
// (reference: src/utility.h:13-88). Rendering draws its random numbers on the
// device from a counter RNG; these are for building scenes
// (e.g. the random-spheres scene, main.cc:105-153).
#pragma once
#include <cmath>
#include <cstdlib>
#include <limits>
#include <memory>

#include "color.h"
#include "ray.h"
#include "vec3.h"

const double infinity = std::numeric_limits<double>::infinity();
const double pi = 3.1415926535897932385;

inline double degrees_to_radians(double degrees) { return degrees * pi / 180.0; }
inline double random_double() { return std::rand() / (RAND_MAX + 1.0); }
inline double random_double(double lo, double hi) { return lo + (hi - lo) * random_double(); }
inline int random_int(int lo, int hi) { return int(lo + (hi - lo) * random_double()); }
inline vec3 random_vec() {
  double z = random_double(), y = random_double(), x = random_double();  // GCC's right-to-left order
  return vec3(x, y, z);
}
inline vec3 random_vec(double lo, double hi) {
  double z = random_double(lo, hi), y = random_double(lo, hi), x = random_double(lo, hi);
  return vec3(x, y, z);
}
inline double clamp(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
// utility.h:30-42: uniform on (not in) the unit sphere, cos(theta) from the first draw, phi from the second
inline vec3 random_in_unit_sphere() {
  const double u_cos = random_double();
  const double u_phi = random_double();
  const double ct = 1 - 2 * u_cos, st = std::sqrt(1 - ct * ct), phi = 2 * pi * u_phi;
  return vec3(st * std::cos(phi), ct, st * std::sin(phi));
}
inline vec3 random_unit_vec() { return unit_vector(random_in_unit_sphere()); }  // utility.h:44
