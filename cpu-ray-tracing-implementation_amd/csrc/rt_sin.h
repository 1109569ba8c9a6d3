// rt_sin.h -- a correctly rounded double sin for the worley/voronoi hash (noise.h:141-145).
//
// The hash computes fract(43758.5453 * sin(dot(p, k))) and voronoi hashes the feature point
// that first hash produced, so one last-bit difference in sin moves the second argument by
// ~1e-12 and the returned colour by ~1e-4: the texture is chaotic in the libm's last ulp.
// The device libm and glibc disagree in about 4 % of arguments; glibc is correctly rounded in
// all but ~0.2 % (measured over [0, 2e4]). So the device evaluates sin in double-double and
// rounds once, which matches glibc wherever glibc is correctly rounded.
//
// Method: k = rint(x * 2/pi); r = x - k*pi/2 with pi/2 split in four doubles (k*P0 as an
// exact two-product, x - k*P0 exact by Sterbenz), giving r to ~2^-104; then the Taylor series
// of sin or cos at r (|r| <= pi/4) in double-double Horner form up to r^29 / r^28, whose
// truncation error is below 2^-110. Arguments beyond 2^30 use the libm sin. Every helper turns
// FP contraction off: the device compiler otherwise fuses a product into a following add
// across statements (p = a*b; s = p + e -> fma), which breaks the error-free transformations.
#pragma once
#include <hip/hip_runtime.h>

namespace rtd {

struct dd {
  double h, l;
};
__host__ __device__ __forceinline__ dd dd_two_sum(double a, double b) {
#pragma clang fp contract(off)
  const double s = a + b, bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
__host__ __device__ __forceinline__ dd dd_fast(double a, double b) {  // |a| >= |b|
#pragma clang fp contract(off)
  const double s = a + b;
  return {s, b - (s - a)};
}
__host__ __device__ __forceinline__ dd dd_add(dd a, dd b) {
#pragma clang fp contract(off)
  dd s = dd_two_sum(a.h, b.h);
  const dd t = dd_two_sum(a.l, b.l);
  s.l += t.h;
  s = dd_fast(s.h, s.l);
  s.l += t.l;
  return dd_fast(s.h, s.l);
}
__host__ __device__ __forceinline__ dd dd_mul(dd a, dd b) {
#pragma clang fp contract(off)
  const double p = a.h * b.h;
  const double e = fma(a.h, b.h, -p) + (a.h * b.l + a.l * b.h);
  return dd_fast(p, e);
}

// 1/n! as double-double, n = 0..29 (hi, lo)
__host__ __device__ __forceinline__ dd inv_fact(int n) {
  switch (n) {
    case 0: case 1: return {1.0, 0.0};
    case 2: return {0x1.0p-1, 0.0};
    case 3: return {0x1.5555555555555p-3, 0x1.5555555555555p-57};
    case 4: return {0x1.5555555555555p-5, 0x1.5555555555555p-59};
    case 5: return {0x1.1111111111111p-7, 0x1.1111111111111p-63};
    case 6: return {0x1.6c16c16c16c17p-10, -0x1.f49f49f49f49fp-65};
    case 7: return {0x1.a01a01a01a01ap-13, 0x1.a01a01a01a01ap-73};
    case 8: return {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76};
    case 9: return {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73};
    case 10: return {0x1.27e4fb7789f5cp-22, 0x1.cbbc05b4fa99ap-76};
    case 11: return {0x1.ae64567f544e4p-26, -0x1.c062e06d1f209p-80};
    case 12: return {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83};
    case 13: return {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87};
    case 14: return {0x1.93974a8c07c9dp-37, 0x1.05d6f8a2efd1fp-92};
    case 15: return {0x1.ae7f3e733b81fp-41, 0x1.1d8656b0ee8cbp-97};
    case 16: return {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101};
    case 17: return {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103};
    case 18: return {0x1.6827863b97d97p-53, 0x1.eec01221a8b0bp-107};
    case 19: return {0x1.2f49b46814157p-57, 0x1.2650f61dbdcb4p-112};
    case 20: return {0x1.e542ba4020225p-62, 0.0};
    case 21: return {0x1.71b8ef6dcf572p-66, 0.0};
    case 22: return {0x1.0ce396db7f853p-70, 0.0};
    case 23: return {0x1.761b41316381ap-75, 0.0};
    case 24: return {0x1.f2cf01972f578p-80, 0.0};
    case 25: return {0x1.3f3ccdd165fa9p-84, 0.0};
    case 26: return {0x1.88e85fc6a4e5ap-89, 0.0};
    case 27: return {0x1.d1ab1c2dccea3p-94, 0.0};
    case 28: return {0x1.0a18a2635085dp-98, 0.0};
    default: return {0x1.259f98b4358adp-103, 0.0};
  }
}

__host__ __device__ inline double sin_cr(double x) {
#pragma clang fp contract(off)  // x - k*P0 must round k*P0 first: e0 carries that rounding
  if (!(fabs(x) < 0x1.0p30) || x == 0) return sin(x);  // huge, inf/nan, and the signed zeros
  const double k = rint(x * 0x1.45f306dc9c883p-1);
  const double P0 = 0x1.921fb54442d18p+0, P1 = 0x1.1a62633145c07p-54, P2 = -0x1.f1976b7ed8fbcp-110,
               P3 = 0x1.4cf98e804177dp-164;
  // r = x - k*(P0 + P1 + P2 + P3)
  const double a0 = k * P0, e0 = fma(k, P0, -a0);
  const double a1 = k * P1, e1 = fma(k, P1, -a1);
  dd r = dd_two_sum(x - a0, -e0);
  r = dd_add(r, dd{-a1, -e1});
  r = dd_add(r, dd{-k * P2, -fma(k, P2, -k * P2) - k * P3});
  const int q = (int)((long long)k & 3);
  const dd r2 = dd_mul(r, r);
  // sin(r) = r * sum (-1)^i r^2i / (2i+1)!, cos(r) = sum (-1)^i r^2i / (2i)!
  const bool use_cos = q & 1;
  const int top = use_cos ? 28 : 29;
  dd p = inv_fact(top);
  if ((top >> 1) & 1) p = dd{-p.h, -p.l};
  for (int n = top - 2; n >= 0; n -= 2) {
    dd c = inv_fact(n);
    if ((n >> 1) & 1) c = dd{-c.h, -c.l};
    p = dd_add(dd_mul(p, r2), c);
  }
  if (!use_cos) p = dd_mul(p, r);
  const double y = p.h + p.l;
  return (q & 2) ? -y : y;
}

}  // namespace rtd
