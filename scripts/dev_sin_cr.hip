// Dev check: rtd::sin_cr on the device vs the same function on the host, and vs libm.
#include <cmath>
#include <cstdio>
#include <vector>

#include "rt_sin.h"

__global__ void k(const double* x, double* y, double* z, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    y[i] = rtd::sin_cr(x[i]);
    z[i] = sin(x[i]);
  }
}

int main() {
  const int n = 1 << 16;
  std::vector<double> x(n), y(n), z(n);
  unsigned s = 12345;
  for (int i = 0; i < n; i++) {
    s = s * 1664525u + 1013904223u;
    x[i] = (s / 4294967296.0 - 0.5) * 4e4;
  }
  double *dx, *dy, *dz;
  (void)hipMalloc(&dx, n * 8);
  (void)hipMalloc(&dy, n * 8);
  (void)hipMalloc(&dz, n * 8);
  (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, dy, dz, n);
  (void)hipMemcpy(y.data(), dy, n * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(z.data(), dz, n * 8, hipMemcpyDeviceToHost);
  int dev_host = 0, dev_libm = 0, ocml_libm = 0, shown = 0;
  for (int i = 0; i < n; i++) {
    const double h = rtd::sin_cr(x[i]), l = sin(x[i]);
    dev_host += y[i] != h;
    dev_libm += y[i] != l;
    ocml_libm += z[i] != l;
    if (y[i] != h && shown++ < 5) printf("x=%a dev=%a host=%a libm=%a\n", x[i], y[i], h, l);
  }
  printf("n=%d device!=host %d device!=glibc %d ocml!=glibc %d\n", n, dev_host, dev_libm, ocml_libm);
  return 0;
}
