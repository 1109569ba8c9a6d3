// vec3.h -- double-precision 3-vector of the plugin surface (reference: src/vec3.h:5-87).
// Same names and operators, so scene code written against the reference compiles unchanged.
#pragma once
#include <cmath>
#include <iostream>

class vec3 {
 public:
  double e[3];
  vec3() : e{0, 0, 0} {}
  vec3(double v) : e{v, v, v} {}
  vec3(double x, double y, double z) : e{x, y, z} {}
  double x() const { return e[0]; }
  double y() const { return e[1]; }
  double z() const { return e[2]; }
  vec3 operator-() const { return vec3(-e[0], -e[1], -e[2]); }
  double operator[](int i) const { return e[i]; }
  double& operator[](int i) { return e[i]; }
  vec3& operator+=(const vec3& o) {
    for (int k = 0; k < 3; k++) e[k] += o.e[k];
    return *this;
  }
  vec3& operator-=(const vec3& o) {
    for (int k = 0; k < 3; k++) e[k] -= o.e[k];
    return *this;
  }
  vec3& operator*=(double c) {
    for (double& v : e) v *= c;
    return *this;
  }
  vec3& operator/=(double c) {
    for (double& v : e) v /= c;
    return *this;
  }
  double length_squared() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }
  double length() const { return std::sqrt(length_squared()); }
  bool near_zero() const { return std::fabs(e[0]) < 1e-8 && std::fabs(e[1]) < 1e-8 && std::fabs(e[2]) < 1e-8; }
};
using point3 = vec3;

inline std::ostream& operator<<(std::ostream& os, const vec3& v) { return os << v.x() << ' ' << v.y() << ' ' << v.z(); }
inline vec3 operator+(const vec3& a, const vec3& b) { return vec3(a.x() + b.x(), a.y() + b.y(), a.z() + b.z()); }
inline vec3 operator-(const vec3& a, const vec3& b) { return vec3(a.x() - b.x(), a.y() - b.y(), a.z() - b.z()); }
inline vec3 operator*(const vec3& a, const vec3& b) { return vec3(a.x() * b.x(), a.y() * b.y(), a.z() * b.z()); }
inline vec3 operator*(const vec3& a, double c) { return vec3(a.x() * c, a.y() * c, a.z() * c); }
inline vec3 operator*(double c, const vec3& a) { return a * c; }
inline vec3 operator/(const vec3& a, const vec3& b) { return vec3(a.x() / b.x(), a.y() / b.y(), a.z() / b.z()); }
inline vec3 operator/(const vec3& a, double c) { return vec3(a.x() / c, a.y() / c, a.z() / c); }
inline double dot(const vec3& a, const vec3& b) { return a.x() * b.x() + a.y() * b.y() + a.z() * b.z(); }
inline vec3 cross(const vec3& a, const vec3& b) {
  return vec3(a.y() * b.z() - a.z() * b.y(), a.z() * b.x() - a.x() * b.z(), a.x() * b.y() - a.y() * b.x());
}
inline vec3 unit_vector(const vec3& v) { return v / v.length(); }
inline vec3 floor(const vec3& v) { return vec3(std::floor(v.x()), std::floor(v.y()), std::floor(v.z())); }
inline vec3 ceil(const vec3& v) { return vec3(std::ceil(v.x()), std::ceil(v.y()), std::ceil(v.z())); }
inline vec3 fmod(const vec3& v, const vec3& m) {  // vec3.h:86, per component
  vec3 r;
  for (int k = 0; k < 3; k++) r[k] = std::fmod(v[k], m[k]);
  return r;
}
inline vec3 fract(const vec3& v) { return v - floor(v); }
