// color.h -- colors and the P3 pixel writer (reference: src/color.h:5-36).
#pragma once
#include <cmath>
#include <iostream>

#include "vec3.h"
using color = vec3;

inline color red = color(1, 0, 0);
inline color green = color(0, 1, 0);
inline color blue = color(0, 0, 1);
inline color yellow = color(1, 1, 0);
inline color cyan = color(0, 1, 1);
inline color magenta = color(1, 0, 1);
inline color white = color(1, 1, 1);
inline color black = color(0, 0, 0);

// gamma 2.2 (color.h:16-20)
inline double linear_to_gamma(double c) { return c > 0 ? std::pow(c, 1 / 2.2) : 0; }

// One "r g b" line; like the reference, values are not clamped (color.h:31-35).
inline void write_color(std::ostream& out, const color& c) {
  out << int(255.999 * linear_to_gamma(c.x())) << ' ' << int(255.999 * linear_to_gamma(c.y())) << ' '
      << int(255.999 * linear_to_gamma(c.z())) << '\n';
}
