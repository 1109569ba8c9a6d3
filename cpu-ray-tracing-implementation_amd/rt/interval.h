// interval.h (reference: src/interval.h:4-41)
#pragma once
#include "utility.h"

class interval {
 public:
  double min, max;
  interval() : min(infinity), max(-infinity) {}
  interval(double lo, double hi) : min(lo), max(hi) {}
  double size() const { return max - min; }
  bool is_contains(double x) const { return min <= x && x <= max; }
  bool is_surrounds(double x) const { return min < x && x < max; }
  double clamp(double x) const { return x < min ? min : (x > max ? max : x); }
  interval expand(double delta) const { return interval(min - delta / 2, max + delta / 2); }
  interval offset(double d) const { return interval(min + d, max + d); }
  static interval enclose(interval a, interval b) {
    return interval(a.min < b.min ? a.min : b.min, a.max > b.max ? a.max : b.max);
  }
  static const interval empty, universe;  // interval.h:32,40-41
};
// C++17 inline variables: one definition however many translation units include this header
inline const interval interval::empty = interval(+infinity, -infinity);
inline const interval interval::universe = interval(-infinity, +infinity);
