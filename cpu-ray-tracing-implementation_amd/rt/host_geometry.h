// host_geometry.h -- fp64 host-side answers to the hittable queries of the plugin surface
// (hittable::hit / get_bounding_box / pdf_value / random, reference src/hittable.h:32-41).
//
// camera::render never calls these: every ray of a render is traced on the device. They exist
// so that code written against the reference's classes can still ask a scene object a question
// on the host (pick a point, test visibility, evaluate a light pdf) and get the answer the
// reference's object would give: same arithmetic order, closed intervals, later-wins ties in
// lists, the x-median bvh_node tree, and the reference's quirks (the moving sphere's normal
// from center_ = 0, triangles that leave u, v untouched, a volume that draws rand()).
#pragma once
#include <algorithm>
#include <cmath>
#include <memory>

#include "interval.h"
#include "ray.h"
#include "utility.h"
#include "vec3.h"

namespace rt_host {

// sphere::get_sphere_uv (sphere.h:90-95) of an outward normal
inline void sphere_uv(const vec3& n, double& u, double& v) {
  const double theta = std::acos(-n.y());
  const double phi = std::atan2(-n.z(), n.x()) + pi;
  u = phi / (2 * pi);
  v = theta / pi;
}

// The quadratic of sphere.h:40-74 as the reference writes it (b = 2 d.(o - c), roots (-b -+ sqrt)/2a,
// the smaller first, both against the closed interval). Returns the root or NaN.
inline double sphere_root(const point3& center, double radius, const ray& r, const interval& t_range) {
  const vec3 oc = r.origin() - center;
  const double a = dot(r.direction(), r.direction());
  const double b = 2.0 * dot(r.direction(), oc);
  const double c = dot(oc, oc) - radius * radius;
  const double disc = b * b - 4 * a * c;
  if (disc < 0) return std::nan("");
  const double sq = std::sqrt(disc);
  for (double root : {(-b - sq) / (2.0 * a), (-b + sq) / (2.0 * a)})
    if (t_range.is_contains(root)) return root;
  return std::nan("");
}

// quad::hit's plane and interior test (quad.h:30-64); alpha, beta out
inline double quad_root(const point3& corner, const vec3& u, const vec3& v, const vec3& unit_n, const ray& r,
                        const interval& t_range, double& alpha, double& beta) {
  const double t = (dot(unit_n, corner) - dot(unit_n, r.origin())) / dot(unit_n, r.direction());
  if (!t_range.is_contains(t)) return std::nan("");
  const vec3 rel = r.at(t) - corner;
  const vec3 n = cross(u, v);
  const vec3 w = n / dot(n, n);
  alpha = dot(w, cross(rel, v));
  beta = dot(w, cross(u, rel));
  const interval unit(0, 1);
  if (!unit.is_contains(alpha) || !unit.is_contains(beta)) return std::nan("");
  return t;
}

// moller_trumbore + triangle::hit (triangle.h:8-40): (t, b0, b1) divided by s1.e1 as one vec3
inline double triangle_root(const point3& p0, const point3& p1, const point3& p2, const ray& r,
                            const interval& t_range) {
  const vec3 e1 = p1 - p0, e2 = p2 - p0, s = r.origin() - p0;
  const vec3 s1 = cross(r.direction(), e2), s2 = cross(s, e1);
  const vec3 tb = vec3(dot(s2, e2), dot(s1, s), dot(s2, r.direction())) / dot(s1, e1);
  if (tb.x() < t_range.min || tb.x() > t_range.max) return std::nan("");
  if (tb.y() < 0 || tb.z() < 0 || tb.y() + tb.z() > 1) return std::nan("");
  return tb.x();
}

// rotate_x/y/z (hittable.h:125-149, 192-216, 259-284): the two coordinates a rotation mixes,
// world -> object (`inverse`: by -theta) and object -> world (by +theta)
template <int Axis>
inline vec3 rotate(const vec3& p, double s, double c, bool to_object) {
  constexpr int A = Axis == 0 ? 1 : 0, B = Axis == 2 ? 1 : 2;
  vec3 q = p;
  if (to_object) {
    q[A] = c * p[A] - s * p[B];
    q[B] = s * p[A] + c * p[B];
  } else {
    q[A] = c * p[A] + s * p[B];
    q[B] = -s * p[A] + c * p[B];
  }
  return q;
}

// aabb::hit (aabb.h:28-69): per-axis division, std::min / std::max, strict overlap
inline bool slab_overlap(const interval& x, const interval& y, const interval& z, const ray& r, interval t_range) {
  const interval* ax[3] = {&x, &y, &z};
  double lo = -infinity, hi = infinity;
  for (int k = 0; k < 3; k++) {
    const double t1 = (ax[k]->min - r.origin()[k]) / r.direction()[k];
    const double t2 = (ax[k]->max - r.origin()[k]) / r.direction()[k];
    lo = k == 0 ? std::min(t1, t2) : std::max(lo, std::min(t1, t2));
    hi = k == 0 ? std::max(t1, t2) : std::min(hi, std::max(t1, t2));
  }
  if (lo > t_range.min) t_range.min = lo;
  if (hi < t_range.max) t_range.max = hi;
  return t_range.min < t_range.max;
}

}  // namespace rt_host
