// Host build of rtd::sin_cr (csrc/rt_sin.h) for tests/test_sin_cr.py: reads hex doubles from
// stdin, prints sin_cr(x) and the host libm's sin(x) in hex.
#include <cmath>
#include <cstdio>

#include "rt_sin.h"

int main() {
  double x;
  while (scanf("%la", &x) == 1) printf("%a %a\n", rtd::sin_cr(x), sin(x));
  return 0;
}
