// rt_device.h -- device-side math, RNG, intersection, traversal and shading of
// the wavefront path tracer. Templated on the arithmetic type R (float: the
// production path; double: the parity path that tracks the fp64 reference).
// Each routine cites the reference code it implements.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "rt_scene.h"
#include "rt_sin.h"

namespace rtd {

// fp32: spheres larger than this are intersected (and their hit points rebuilt) in fp64
#ifndef RT_BIG_SPHERE_R
#define RT_BIG_SPHERE_R 16
#endif
#ifndef RT_WIDE_SPEC  // wide BVH in HBM: speculative while-while traversal (trace_wide)
#define RT_WIDE_SPEC 1
#endif
// RT_WIDE_FMA (retired in round 6, always on): fp64 rays over the wide BVH: octant-ordered planes, one fma per plane
// distance
// RT_WIDE_OCT32 (retired in round 6, always on): fp32 rays over the wide BVH: octant-ordered planes, (p - o) * inv (C3
// fp32 60.87 -> 57.22 ms/frame, C4 351.9 -> 341.6)
// RT_WIDE_HALF_F64 (retired in round 6, always on): fp64 rays over trees in HBM read the fp16 node form (rt_scene.h
// WNodeH): 5 loads per node visit instead of 7 (C4 fp64 504.0 -> 480.8 ms/frame; fp32 rays lose, see WNodeH)
#ifndef RT_WIDE_FMA32  // fp32 rays over an LDS tree: one fma per plane distance, three per-ray constants and one
#define RT_WIDE_FMA32 1  // bound (trace_wide; C3 fp32 49.63 -> 48.54 ms/frame; 2, per-axis constants: 49.01)
#endif
// RT_WIDE_OFS64 (retired in round 6, always on): fp64 rays keep 64-bit addresses into trees in HBM (C4 fp64: 32-bit
// offsets 573.5 ms/frame, 64-bit 545.1; fp32 the other way round, 340.7 -> 329.1)
// RT_WIDE_PREFETCH (retired in round 6, always on): a triangle's words loaded with the record's first word (C4 358.9 ->
// 357.2 ms)
// The extended (CAMX) kernels' heavy, rarely taken code -- fp64 OCML trigonometry (sphere_uv, the fisheye
// camera), the noise textures -- as real calls (round 5): inlined, their temporaries sized the whole kernel
// (~290 registers, 1 wave per SIMD); called, the loop keeps its own budget and the live state is saved
// around the call only when it is taken.
#define RT_EXT_FN __device__ __attribute__((noinline))
#ifndef RT_MIX_SELECT  // the light / material halves of the mixture pdf (pdf.h:52-56) as one select path: 1 in
#define RT_MIX_SELECT 1  // the flat program (C2 fp64 28.33 -> 28.15 ms/frame, fp32 18.83 -> 18.49, r05e), 2 in every kernel
#endif
// RT_LIGHT_PDF_F64 (retired in round 6, always on): fp64 axis-aligned light pdf by one reciprocal (light_pdf_aligned,
// round 4)

// Math policy. fp64 (the parity path): libm where the reference calls it (log), and division,
// reciprocal and square root refined from the hardware estimates to about an ulp (below).
// fp32 (the production path): the hardware ops -- v_rcp_f32, v_sqrt_f32, v_rsq_f32,
// v_log_f32, and v_sin_f32 / v_cos_f32, which take their argument in revolutions, so
// sin(2*pi*u) for u in [0,1) needs no range reduction.
// RT_PRECISE_F32 (a development build, see scripts/dev_divergence.py) swaps the fp32 ops
// for the correctly rounded ones to measure what the hardware ops cost in path divergence.
#ifndef RT_PRECISE_F32
__device__ __forceinline__ float fdiv(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float flog(float x) { return __builtin_amdgcn_logf(x) * 0.693147180559945309f; }
__device__ __forceinline__ float frsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ void sincos2pi(float u, float& s, float& c) {
  s = __builtin_amdgcn_sinf(u);
  c = __builtin_amdgcn_cosf(u);
}
#else
__device__ __forceinline__ float fdiv(float a, float b) { return a / b; }
__device__ __forceinline__ float fsqrt(float x) { return sqrtf(x); }
__device__ __forceinline__ float flog(float x) { return logf(x); }
__device__ __forceinline__ float frsq(float x) { return 1.0f / sqrtf(x); }
__device__ __forceinline__ void sincos2pi(float u, float& s, float& c) {
  float phi = 2 * 3.14159265358979f * u;
  s = sinf(phi);
  c = cosf(phi);
}
#endif
// fp64 division, reciprocal and square root (round 3). IEEE fp64 division on gfx950 is a
// v_div_scale / v_rcp / 5 x v_fma / v_div_fmas / v_div_fixup sequence, and sqrt a similar one: the
// fp64 Cornell kernel spent ~60 % of its fp64 instructions in ~32 of them per segment (r03c counters:
// 35 v_rcp/v_rsq per lane-segment). Here: the hardware estimate (v_rcp_f64 / v_rsq_f64, ~2^-23
// relative) refined by Newton-Raphson to within an ulp or two of the IEEE result -- far inside the
// fp64 parity tolerance against the oracle (1e-9 relative; measured ~1e-15). Zero, infinite and NaN
// operands, where the refinement would turn an exact infinity into NaN, fall back to the raw
// estimate, which v_rcp / v_rsq compute exactly for them (1/0 = inf, 1/inf = 0, rsq(0) = inf).
__device__ __forceinline__ double frcp(double b) {
  const double r0 = __builtin_amdgcn_rcp(b);
  double r = r0;
  double e = fma(-b, r, 1.0);
  r = fma(r, e, r);
  e = fma(-b, r, 1.0);
  r = fma(r, e, r);
  return __builtin_isfinite(r) ? r : r0;
}
__device__ __forceinline__ double fdiv(double a, double b) {
  const double r = frcp(b);
  const double q = a * r;
  const double res = fma(fma(-b, q, a), r, q);  // one residual step: ~correctly rounded
  return __builtin_isfinite(res) ? res : q;     // a/0, inf/b, 0/0 as IEEE
}
// a / b where the quotient is finite for every ray that can hit (the fp64 sphere roots' (-b -+ sq) / 2a,
// 2a = 2|d|^2 > 0): fdiv without its non-finite fallback, a class test and two selects per division
// (round 4: ~13 of the ~60 SIMD cycles; the same bits whenever the result is finite)
__device__ __forceinline__ double fdiv_fin(double a, double b) {
  const double r = frcp(b);
  const double q = a * r;
  return fma(fma(-b, q, a), r, q);
}
__device__ __forceinline__ double frsq(double x) {  // 1/sqrt(x)
  const double r0 = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  double r = r0;
  r = r * fma(-h * r, r, 1.5);
  r = r * fma(-h * r, r, 1.5);
  return __builtin_isfinite(r) ? r : r0;
}
// 1/sqrt(x) without the fallback (round 4): for unit(v), where it cannot matter -- a zero vector gives NaN
// with or without it (0 * inf), as the reference's v / 0 does -- and the class test and two selects it
// costs are 13 of the ~30 SIMD cycles of the refined rsqrt (measured issue costs)
__device__ __forceinline__ double frsq_nz(double x) {
  const double r0 = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  double r = r0;
  r = r * fma(-h * r, r, 1.5);
  r = r * fma(-h * r, r, 1.5);
  return r;
}
// sqrt of x in [0, 1] (the sampling formulas' sqrt(r2), sqrt(1 - r2), sqrt(1 - cos^2)): x = 0 is the only
// operand the refinement cannot take (rsq(0) = inf), so one compare replaces fsqrt's three
__device__ __forceinline__ double fsqrt01(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  double g = x * r, h = 0.5 * r;
  const double e = fma(-g, h, 0.5);
  g = fma(g, e, g);
  h = fma(h, e, h);
  g = fma(fma(-g, g, x), h, g);
  return x > 0.0 ? g : 0.0;
}
__device__ __forceinline__ float fsqrt01(float x) { return fsqrt(x); }
__device__ __forceinline__ double fsqrt(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  double g = x * r, h = 0.5 * r;
  const double e = fma(-g, h, 0.5);  // Goldschmidt step
  g = fma(g, e, g);
  h = fma(h, e, h);
  g = fma(fma(-g, g, x), h, g);  // residual correction
  return (x > 0.0 && x < __builtin_huge_val()) ? g : (x >= 0.0 ? x : __builtin_nan(""));
}
// a / b given inv_b = rcp3(..) of b computed once per ray: bit-identical to fdiv(a, b) in fp32
// (the precise build divides; rcp3 then returns nothing the compiler keeps)
__device__ __forceinline__ float fdiv_inv(float a, float b, float inv_b) {
#ifndef RT_PRECISE_F32
  return a * inv_b;
#else
  return a / b;
#endif
}
__device__ __forceinline__ double fdiv_inv(double a, double b, double) { return fdiv(a, b); }
__device__ __forceinline__ double flog(double x) { return log(x); }
// sin(2*pi*u), cos(2*pi*u) for u in [0, 1) (utility.h:36,64 evaluate sin(phi) of phi = 2*pi*u).
// fp64: sincospi(2u) -- 2u is exact, and the reduction is an exact subtraction, so there is no
// Payne-Hanek path: OCML's general sin/cos carry one, whose registers (the kernel's budget is its
// heaviest path) held the fp64 kernels at 2-3 waves per SIMD. Within an ulp or two of
// sin(fl(2 pi u)): far inside the fp64 parity tolerance (1e-9 relative against the oracle).
// Round 4: a 1024-entry table of (sin, cos)(2 pi j / 1024), correctly rounded on the host (rt_kernels.hip
// sincos_table_init), and the angle addition formulas for the rest, delta = 2 pi (u - j / 1024) < 2 pi / 1024:
// sin delta = delta (1 - delta^2 / 6 + delta^4 / 120) and cos delta - 1 = delta^2 (-1/2 + delta^2 / 24 -
// delta^4 / 720) leave truncation errors below 1e-19, so the result is within about an ulp, like
// OCML's sincospi, at one table read and 13 fp64 operations instead of ~22 fp64 and ~20 other VALU
// operations (and the polynomial constants OCML's version kept in 18 VGPRs across the path loop).
// u * 1024 and its fractional part are exact for every double u in [0, 1).
constexpr int kSinCosTab = 1024;
__device__ double2 g_sincos_tab[kSinCosTab];
__device__ __forceinline__ void sincos2pi(double u, double& s, double& c) {
#ifdef RT_OCML_SINCOS
  sincospi(2.0 * u, &s, &c);
#else
  const double t = u * double(kSinCosTab);
  const double h = floor(t);
  const double2 sc = g_sincos_tab[(uint32_t)(int32_t)h & (kSinCosTab - 1)];
  const double d = (t - h) * (2.0 * 3.14159265358979323846 / kSinCosTab);
  const double d2 = d * d;
  const double sd = d * fma(d2, fma(d2, 1.0 / 120.0, -1.0 / 6.0), 1.0);
  const double cm1 = d2 * fma(d2, fma(d2, -1.0 / 720.0, 1.0 / 24.0), -0.5);
  s = fma(sc.y, sd, fma(sc.x, cm1, sc.x));
  c = fma(-sc.x, sd, fma(sc.y, cm1, sc.y));
#endif
}
// x / pi (pdf.h:27-29 cosine_pdf::value): fp32 as before, fp64 as a product with 1/pi
__device__ __forceinline__ float div_pi(float x) { return fdiv(x, 3.14159265358979323846f); }
__device__ __forceinline__ double div_pi(double x) { return x * 0.318309886183790671537767526745; }
__device__ __forceinline__ float pow5(float x) { return (x * x) * (x * x) * x; }
// material.h:131 std::pow(1 - cosine, 5), as products (a few ulp; OCML's pow is a log/exp pair)
__device__ __forceinline__ double pow5(double x) { return (x * x) * (x * x) * x; }

// ------------------------------------------------------------------ vectors
template <class R>
struct V {
  R x, y, z;
};
template <class R>
__device__ __forceinline__ V<R> mkv(R x, R y, R z) {
  return {x, y, z};
}
template <class R>
__device__ __forceinline__ V<R> ld3(const R* p) {
  return {p[0], p[1], p[2]};
}
template <class R>
__device__ __forceinline__ V<R> operator+(V<R> a, V<R> b) {
  return {a.x + b.x, a.y + b.y, a.z + b.z};
}
template <class R>
__device__ __forceinline__ V<R> operator-(V<R> a, V<R> b) {
  return {a.x - b.x, a.y - b.y, a.z - b.z};
}
template <class R>
__device__ __forceinline__ V<R> operator-(V<R> a) {
  return {-a.x, -a.y, -a.z};
}
template <class R>
__device__ __forceinline__ V<R> operator*(V<R> a, V<R> b) {
  return {a.x * b.x, a.y * b.y, a.z * b.z};
}
template <class R>
__device__ __forceinline__ V<R> operator*(R c, V<R> a) {
  return {a.x * c, a.y * c, a.z * c};
}
template <class R>
__device__ __forceinline__ V<R> operator*(V<R> a, R c) {
  return {a.x * c, a.y * c, a.z * c};
}
__device__ __forceinline__ double frcp(double b);
template <class R>
__device__ __forceinline__ V<R> operator/(V<R> a, R c) {
  if constexpr (sizeof(R) == 8) {  // one reciprocal for the three (within ~1.5 ulp of each quotient)
    const R r = frcp(c);
    return {a.x * r, a.y * r, a.z * r};
  } else {
    return {a.x / c, a.y / c, a.z / c};
  }
}
template <class R>
__device__ __forceinline__ R dot(V<R> a, V<R> b) {  // vec3.h:61
  return a.x * b.x + a.y * b.y + a.z * b.z;
}
template <class R>
__device__ __forceinline__ V<R> cross(V<R> a, V<R> b) {  // vec3.h:79-82
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
template <class R>
__device__ __forceinline__ R len(V<R> a);
template <class R>
__device__ __forceinline__ V<R> unit(V<R> a);
template <class R>
__device__ __forceinline__ V<R> reflect(V<R> v, V<R> n) {  // utility.h:70
  return v - (R(2) * dot(v, n)) * n;
}
template <class R>
__device__ __forceinline__ V<R> refract(V<R> v, V<R> n, R eta) {  // utility.h:71-76
  R cos_theta = fmin(dot(-v, n), R(1));
  V<R> perp = eta * (v + cos_theta * n);
  V<R> par = (-fsqrt(fabs(R(1) - dot(perp, perp)))) * n;
  return perp + par;
}


template <class R>
__device__ __forceinline__ R len(V<R> a) {
  return fsqrt(a.x * a.x + a.y * a.y + a.z * a.z);
}
template <>
__device__ __forceinline__ V<float> unit(V<float> a) {  // vec3.h:77 (v / |v|), as v * rsqrt(v.v)
  return a * frsq(a.x * a.x + a.y * a.y + a.z * a.z);
}
template <>
__device__ __forceinline__ V<double> unit(V<double> a) {  // vec3.h:77 (v / |v|), as v * rsqrt(v.v) refined
  return a * frsq_nz(a.x * a.x + a.y * a.y + a.z * a.z);
}

template <class R>
struct Num;
template <>
struct Num<float> {
  static constexpr float inf() { return __builtin_huge_valf(); }
  static constexpr float pi() { return 3.14159265358979323846f; }
  // 1 + 2*gamma(5): the robust bound 1 + 2*gamma(3) for correctly rounded 1/d, widened for
  // v_rcp_f32's 1-ulp reciprocal (box_inv)
  static constexpr float box_slack() { return 1.0f + 2.0f * 5.0f * 5.9604645e-08f; }
};
template <>
struct Num<double> {
  static constexpr double inf() { return __builtin_huge_val(); }
  static constexpr double pi() { return 3.1415926535897932385; }  // utility.h:15
  static constexpr double box_slack() { return 1.0 + 2.0 * 3.0 * 1.1102230246251565e-16; }
};

// ------------------------------------------------------------------ counter RNG
// 32-bit draw for (seed, pixel, sample, dim); identical to the oracle's
// (oracle/oracle.cpp) and to rt_rng_u32 on the host.
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x21f0aaadu;
  x ^= x >> 15;
#ifndef RT_EXP_CHEAPMIX  // timing experiment only (wrong images)
  x *= 0xd35a2d97u;
  x ^= x >> 15;
#endif
  return x;
}
__host__ __device__ __forceinline__ uint32_t key_pixel(uint64_t seed, uint32_t pixel) {
  return mix32(pixel ^ mix32((uint32_t)seed ^ 0x9E3779B9u));
}
__host__ __device__ __forceinline__ uint32_t key_sample(uint64_t seed, uint32_t sample) {
  return mix32(sample + mix32((uint32_t)(seed >> 32) + 0x7F4A7C15u));
}
// the key of one camera sample; each draw is then a single mix (two 32-bit multiplies)
__host__ __device__ __forceinline__ uint32_t key_path(uint32_t ka, uint32_t kb) { return mix32(ka ^ kb); }
__host__ __device__ __forceinline__ uint32_t draw_u32(uint32_t ks, uint32_t dim) {
  return mix32(ks + dim * 0x9E3779B9u);
}
template <class R>
__device__ __forceinline__ R to_unit(uint32_t x) {  // exact 24-bit value in [0,1)
  return R(x >> 8) * R(1.0 / 16777216.0);
}
// draw dimensions: camera 0..2; bounce b: 3 + 16 b + j,
// j in [0,12) volume draws (volumne.h:36), j in [12,16) scatter/pdf draws.
constexpr uint32_t kDimsCamera = 3, kDimsPerBounce = 16, kVolumeSlots = 12;
__device__ __forceinline__ uint32_t dim_volume(uint32_t bounce, uint32_t j) {
  return kDimsCamera + kDimsPerBounce * bounce + (j < kVolumeSlots ? j : kVolumeSlots - 1);
}
__device__ __forceinline__ uint32_t dim_scatter(uint32_t bounce, uint32_t j) {
  return kDimsCamera + kDimsPerBounce * bounce + kVolumeSlots + (j < 4u ? j : 3u);
}

struct Keys {
  uint32_t ks;  // key_path of the camera sample
};

// ------------------------------------------------------------------ scene view
// A word of the wide BVH's primitive stream (rt_scene.h WNode): 16 bytes of floats in the fp32
// blob, 32 bytes of doubles in the fp64 one (same word indices, so the leaf codes are shared); the
// primitive's entry is in the bits of w (the low 32 bits of the double).
template <class R>
struct WWord;
template <>
struct WWord<float> {
  using T = float4;
};
struct alignas(32) double4w {
  double x, y, z, w;
};
template <>
struct WWord<double> {
  using T = double4w;
};
__device__ __forceinline__ uint32_t wentry(const float4& h) { return __float_as_uint(h.w); }
__device__ __forceinline__ uint32_t wentry(const double4w& h) { return (uint32_t)__double_as_longlong(h.w); }

// The camera as camera::render/generate_ray use it (camera.h:137-141, 244-290), in double.
struct CamDev {
  int32_t mode;  // rt_camera_mode
  int32_t pad;
  V<double> pos, du, dv;
  V<double> dir00;   // perspective / fisheye: f dir - vw/2 right + vh/2 up + (du + dv)/2 (camera.h:246, 260)
  V<double> pos00;   // orthonormal / lens: pos - vw/2 right + vh/2 up + (du + dv)/2 (camera.h:253, 278)
  V<double> dir;     // dir_, unit
  V<double> fdir;    // focus_dist_ * dir_ (camera.h:279)
  V<double> disk_u, disk_v;  // defocus_disk_u/v (camera.h:129-131)
  double focal;      // focal_length_ (camera.h:266)
};

template <class R>
struct DevScene {
  const Quad<R>* quads;
  const Sphere<R>* spheres;
  const Tri<R>* tris;
  const Instance<R>* insts;
  const Volume<R>* vols;
  const Node<R>* nodes;
  const uint32_t* refs;
  const Material<R>* mats;
  const Texture<R>* texs;
  const Light<R>* light;
  const LinRec<R>* lin;  // linear program (n_linear > 0)
  uint32_t n_linear;
  const FlatQuadT<R>* flatq;  // flat program (has_flat): quads grouped by plane axis, then boxes
  const FlatBoxT<R>* flatb;
  uint32_t n_flatq[3], n_flatb;
  uint32_t n_mats;
  int32_t has_flat;
  uint32_t root;
  int32_t background;
  int32_t has_volumes;
  uint32_t n_nodes;
  const double* texdata;  // procedural-texture tables (Texture::data)
  const uint8_t* images;  // picture-texture pixels (Texture::data)
  int32_t has_procedural; // any perlin / value / worley / voronoi texture: the EXT kernels
  // wide BVH (rt_scene.h WNode; float boxes in both blobs): nodes, primitive words, root code,
  // stack need, WK_* kinds
  const WNode* wnodes;
  const typename WWord<R>::T* wprims;
  uint32_t n_wnodes, n_wprim_words, wroot, wide_stack, wide_kinds;
  int32_t has_wide;
  uint32_t wide_big;  // primitives at the head of the word stream, tested before the tree
  uint32_t wide_top;  // nodes [0, wide_top): the tree's first levels (HBM trees: read from an LDS copy)
  const WNodeH* wnodesh;  // the fp16 form of the tree (rt_scene.h WNodeH; 0: none)
  const Quad<double>* quads64;  // fp32 scenes: the fp64 quads (RT_QUAD_REFINE; 0: none)
  // the render's camera when it is perspective (0: another model): near-edge quad hits of camera rays are re-decided
  // on the fp64 camera ray (quad_edge64)
  const CamDev* cam64;
  // a tree in HBM keeps at most wide_lds_stack<R>() stack entries per lane in LDS; deeper entries go to
  // wide_spill[(depth - wide_lds_stack<R>()) * spill_lanes + lane]
  uint32_t* wide_spill;
  uint32_t spill_lanes;
};
// RT_WIDE_TOP (retired in round 6, always on): fp32 rays over trees in HBM: the tree's first levels read from LDS
// (trace_wide)
#ifndef RT_WIDE_TOP_N  // at most this many of them (the builder orders up to kWideTopMax breadth-first)
#define RT_WIDE_TOP_N 55
#endif
// RT_WIDE_TOP_F64 (retired in round 6, always on): the same for fp64 rays, whose HBM trees are read in the fp16 form
// (WNodeH)
#ifndef RT_WIDE_TOP_N_F64
#define RT_WIDE_TOP_N_F64 85
#endif
#ifndef RT_WIDE_LDS_STACK
#define RT_WIDE_LDS_STACK 12
#endif
#ifndef RT_WIDE_LDS_STACK_F64  // 18 since round 6: the fp64 LL kernel's LDS also holds the throughput (Path LT)
#define RT_WIDE_LDS_STACK_F64 18
#endif
// stack entries per lane kept in LDS for a tree in HBM, by ray precision (fp32: fewer, so the LDS also holds
// the top of the tree and 8 blocks fit a CU; C4 fp32, stack / top nodes / waves: 24 / 0 / 6 309.4 ms/frame,
// 22 / 21 / 6 290.1, 16 / 47 / 7 268.8, 14 / 63 / 7 268.1, 12 / 55 / 8 265.2; r05r-r05u)
template <class R>
constexpr uint32_t wide_lds_stack() {
  return sizeof(R) == 4 ? RT_WIDE_LDS_STACK : RT_WIDE_LDS_STACK_F64;
}

// World -> object through an instance chain (hittable.h:75-82, 125-135, 192-202, 259-270).
template <class R>
__device__ __forceinline__ V<R> op_in(const XOp<R>& op, V<R> p, bool point) {
  if (op.kind == 0) {
    if (point) p = mkv(p.x - op.x, p.y - op.y, p.z - op.z);
    return p;
  }
  const R s = op.x, c = op.y;
  if (op.kind == 1) return mkv(p.x, c * p.y - s * p.z, s * p.y + c * p.z);  // rotate_x
  if (op.kind == 2) return mkv(c * p.x - s * p.z, p.y, s * p.x + c * p.z);  // rotate_y
  return mkv(c * p.x - s * p.y, s * p.x + c * p.y, p.z);                    // rotate_z
}
// Object -> world for a hit point or normal (hittable.h:80, 138-147, 205-214, 273-282).
template <class R>
__device__ __forceinline__ V<R> op_out(const XOp<R>& op, V<R> p, bool point) {
  if (op.kind == 0) {
    if (point) p = mkv(p.x + op.x, p.y + op.y, p.z + op.z);
    return p;
  }
  const R s = op.x, c = op.y;
  if (op.kind == 1) return mkv(p.x, c * p.y + s * p.z, -s * p.y + c * p.z);
  if (op.kind == 2) return mkv(c * p.x + s * p.z, p.y, -s * p.x + c * p.z);
  return mkv(c * p.x + s * p.y, -s * p.x + c * p.y, p.z);
}
template <class R>
__device__ __forceinline__ void chain_in(const Instance<R>& in, V<R>& o, V<R>& d) {
  for (int k = 0; k < in.nops; k++) {
    o = op_in(in.op[k], o, true);
    d = op_in(in.op[k], d, false);
  }
}
// the same for an instance held in registers (a scalar-loaded record): unrolled, so the ops
// are indexed statically and the record is not copied to the stack
template <class R>
__device__ __forceinline__ void chain_in_regs(const Instance<R>& in, V<R>& o, V<R>& d) {
#pragma unroll
  for (int k = 0; k < kMaxChain; k++) {
    if (k >= in.nops) break;
    o = op_in(in.op[k], o, true);
    d = op_in(in.op[k], d, false);
  }
}

// ------------------------------------------------------------------ primitive tests
// 1/d for the slab test: v_rcp_f32 in fp32 (its error is covered by box_slack), IEEE in fp64.
template <class R>
__device__ __forceinline__ V<R> box_inv(V<R> d) {
  if constexpr (sizeof(R) == 4)
    return mkv(__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z));
  else
    return mkv(frcp(d.x), frcp(d.y), frcp(d.z));
}

// Ray/box slab test with IEEE min/max (a NaN slab is ignored: conservative) and
// the robust 1 + 2*gamma(3) widening of the exit distance.
template <class R>
__device__ __forceinline__ bool box_hit(const R* lo, const R* hi, V<R> o, V<R> inv, R tmin, R tmax, R& tnear) {
  R tx0 = (lo[0] - o.x) * inv.x, tx1 = (hi[0] - o.x) * inv.x;
  R ty0 = (lo[1] - o.y) * inv.y, ty1 = (hi[1] - o.y) * inv.y;
  R tz0 = (lo[2] - o.z) * inv.z, tz1 = (hi[2] - o.z) * inv.z;
  R tn = fmax(fmax(fmin(tx0, tx1), fmin(ty0, ty1)), fmax(fmin(tz0, tz1), tmin));
  R tf = fmin(fmin(fmax(tx0, tx1), fmax(ty0, ty1)), fmin(fmax(tz0, tz1), tmax)) * Num<R>::box_slack();
  tnear = tn;
  return tn <= tf;
}

// quad::hit (quad.h:30-52) with the alpha/beta triple products precomputed (fields of Quad).
template <class R>
__device__ __forceinline__ bool quad_test(V<R> n, R D, V<R> q, V<R> qa, V<R> qb, V<R> o, V<R> d, R tmin, R tmax,
                                          R& t) {
  R th = fdiv(D - dot(n, o), dot(n, d));
  if (!(tmin <= th && th <= tmax)) return false;  // interval::is_contains, NaN fails
  V<R> p = (o + th * d) - q;
  R a = dot(p, qa), b = dot(p, qb);
  if (!(R(0) <= a && a <= R(1) && R(0) <= b && b <= R(1))) return false;  // quad.h:58-64
  t = th;
  return true;
}
// Near-edge quad hits in fp32 (round 5, extended in round 6). fp32 decides a quad's edges to ~1e-7 of the quad's
// size plus the rounding of the hit point to its world-space magnitude (1.5e-5 at 400: a camera ray over the f3
// scene's light edge at x = 423 lands on 423.0f and hits, where fp64 misses -- 21 such samples of emission 7 were f3's
// whole fp32 RMSE of 1.1e-4, round 5). A test whose alpha or beta lies within 2^-12 of 0 or 1 is re-decided in fp64
// with the quad's fp64 record (DevScene::quads64) by quad_edge64, a call (RT_EXT_FN): rare (a few 1e-4 of the tests
// that pass the distance test), so the kernels keep their register budget and pay for the call only when it is taken.
// The fp64 ray is the path's own camera ray when the ray is one (bounce 0, world space, a perspective camera):
// camera rays are built in fp64 (begin_sample) and rounded, so the oracle's edge decision is then reproduced up to
// the fp64 arithmetic; for later bounces the fp32 ray itself, whose origin is the fp32 path's own hit point.
#ifndef RT_QUAD_REFINE
#define RT_QUAD_REFINE 1
#endif
// what quad_edge64 rebuilds the camera ray from: the path key and pixel (begin_sample), the bounce
struct EdgeRay {
  uint32_t ks, xy, bounce;
};
RT_EXT_FN bool quad_edge64(const Quad<double>* q64, const CamDev* cam, V<float> o, V<float> d, float tmin, float tmax,
                           EdgeRay er) {
  V<double> od = mkv((double)o.x, (double)o.y, (double)o.z), dd = mkv((double)d.x, (double)d.y, (double)d.z);
  if (cam != nullptr && er.bounce == 0) {  // begin_sample's ray (camera.h:245-251, 293), same operations
    const double ox = to_unit<double>(draw_u32(er.ks, 0)) - 0.5, oy = to_unit<double>(draw_u32(er.ks, 1)) - 0.5;
    const double x = double(er.xy & 0xFFFFu), y = double(er.xy >> 16);
    od = cam->pos;
    dd = ((cam->dir00 + x * cam->du) + y * cam->dv + ox * cam->du) + oy * cam->dv;
  }
  const Quad<double>& q = *q64;
  double t64;
  return quad_test(ld3(q.n), q.D, ld3(q.q), ld3(q.a), ld3(q.b), od, dd, (double)tmin, (double)tmax, t64);
}
// the fp32 test with the near-edge re-decision: ref64(tmin, tmax) decides a near-edge hit (have64 false: none)
template <class REF>
__device__ __forceinline__ bool quad_test_near(V<float> n, float D, V<float> q, V<float> qa, V<float> qb, V<float> o,
                                               V<float> d, float tmin, float tmax, float& t, bool have64, REF ref64) {
  const float th = fdiv(D - dot(n, o), dot(n, d));
  if (!(tmin <= th && th <= tmax)) return false;  // interval::is_contains, NaN fails
  const V<float> p = (o + th * d) - q;
  const float a = dot(p, qa), b = dot(p, qb);
  const float m = fminf(fminf(fabsf(a), fabsf(a - 1.0f)), fminf(fabsf(b), fabsf(b - 1.0f)));
  if (have64 && m < 0x1p-12f) {
    if (!ref64(tmin, tmax)) return false;
    t = th;
    return true;
  }
  if (!(0.0f <= a && a <= 1.0f && 0.0f <= b && b <= 1.0f)) return false;  // quad.h:58-64
  t = th;
  return true;
}
template <class R>
__device__ __forceinline__ bool quad_t(const Quad<R>& q, V<R> o, V<R> d, R tmin, R tmax, R& t) {
  return quad_test(ld3(q.n), q.D, ld3(q.q), ld3(q.a), ld3(q.b), o, d, tmin, tmax, t);
}
// quad i of the scene (binary BVH traversal); fp32 with the fp64 re-decision near an edge (`world`: the ray is in
// world space, not an instance's object space, so a camera ray can be rebuilt in fp64)
template <class R>
__device__ __forceinline__ bool quad_t_near(const DevScene<R>& sc, uint32_t i, V<R> o, V<R> d, R tmin, R tmax, R& t,
                                            EdgeRay er, bool world) {
  const Quad<R>& q = sc.quads[i];
  if constexpr (sizeof(R) == 4 && RT_QUAD_REFINE) {
    const Quad<double>* q64 = sc.quads64;
    return quad_test_near(ld3(q.n), q.D, ld3(q.q), ld3(q.a), ld3(q.b), o, d, tmin, tmax, t, q64 != nullptr,
                          [&](float t0, float t1) {
                            return quad_edge64(q64 + i, world ? sc.cam64 : nullptr, o, d, t0, t1, er);
                          });
  }
  return quad_t(q, o, d, tmin, tmax, t);
}

// triangle::hit / moller_trumbore (triangle.h:8-40).
template <class R>
__device__ __forceinline__ bool tri_test(V<R> p0, V<R> e1, V<R> e2, V<R> o, V<R> d, R tmin, R tmax, R& t) {
  V<R> s = o - p0;
  V<R> s1 = cross(d, e2), s2 = cross(s, e1);
  R inv = fdiv(R(1), dot(s1, e1));
  R th = dot(s2, e2) * inv, b0 = dot(s1, s) * inv, b1 = dot(s2, d) * inv;
  if constexpr (sizeof(R) == 8) {  // the parity path divides like triangle.h:14
    R den = dot(s1, e1);
    th = fdiv(dot(s2, e2), den);
    b0 = fdiv(dot(s1, s), den);
    b1 = fdiv(dot(s2, d), den);
  }
  if (th < tmin || th > tmax) return false;
  // (round 6 measured an fp32 edge tolerance of 8 u |s| |e| |d| / |det| -- the tests' rounding bound -- against the
  // fp32 misses of triangles the fp64 test hits, e.g. a grazing ray through one of the C4 stand-in's grids (r06d
  // traces): C4 lit fp32 against fp64 over 400 tiles went from 1.71e-4 to 1.3e-3, every triangle growing by it)
  if (b0 < R(0) || b1 < R(0) || b0 + b1 > R(1)) return false;
  if (th != th) return false;  // 0/0 determinant: the reference's comparisons reject NaN too
  t = th;
  return true;
}
template <class R>
__device__ __forceinline__ bool tri_t(const Tri<R>& tr, V<R> o, V<R> d, R tmin, R tmax, R& t) {
  return tri_test(ld3(tr.p0), ld3(tr.e1), ld3(tr.e2), o, d, tmin, tmax, t);
}

// sphere::hit (sphere.h:40-74). `far_only` is used for the sphere the ray
// starts on: in exact arithmetic its near root is 0 (rejected by the 0.001
// interval) and the ray re-enters only if it points inside.
//
// fp64 evaluates the reference's formula as written. In fp32 that formula loses
// the hit: b^2 - 4ac cancels for a small sphere seen from afar (|o-c|^2 ~ 85 for
// a unit sphere 9 away leaves t ~1e-5 off, which two mirror bounces turn into a
// different path). fp32 therefore takes the discriminant from the ray's
// perpendicular distance to the center, a (r^2 - |l|^2) with l = f - (f.d/a) d,
// and the roots in the cancellation-free form q/a, c/q (Ray Tracing Gems I, ch. 7):
// the same roots, accurate to fp32 rounding.
template <class T>
__device__ __forceinline__ bool sphere_roots(T ox, T oy, T oz, T dx, T dy, T dz, T cx, T cy, T cz, T r, T tmin,
                                             T tmax, bool far_only, T& t) {
  T fx = ox - cx, fy = oy - cy, fz = oz - cz;
  T a = dx * dx + dy * dy + dz * dz;
  T lo, hi;
  if constexpr (sizeof(T) == 8) {
    // sphere.h:48-57 with b = 2 h: b^2 - 4ac = 4 (h^2 - ac), sqrt of it 2 sqrt(h^2 - ac), and (-b -+ sqrt) / 2a =
    // (-h -+ sqrt(h^2 - ac)) / a -- every scaling a power of two, so the same roots up to where the compiler contracts
    // (round 6: one multiply fewer;
    // C3 fp64 62.45 -> 61.47 ms/frame, r06j)
    T h = dx * fx + dy * fy + dz * fz;
    T c = (fx * fx + fy * fy + fz * fz) - r * r;
    T disc = h * h - a * c;
    if (disc < T(0)) return false;
    // disc >= 0 here: the refined sqrt needs only the zero check (fsqrt01), and the roots are finite
    const T sq = fsqrt01(disc);
    lo = fdiv_fin(-h - sq, a);
    hi = fdiv_fin(-h + sq, a);
  } else {
    T ia = fdiv(T(1), a);
    T bh = -(dx * fx + dy * fy + dz * fz);  // -b/2
    T s = bh * ia;
    T lx = fx + s * dx, ly = fy + s * dy, lz = fz + s * dz;
    T disc = a * (r * r - (lx * lx + ly * ly + lz * lz));
    if (disc < T(0)) return false;
    T q = bh + copysignf(fsqrt(disc), bh);
    T c = (fx * fx + fy * fy + fz * fz) - r * r;
    T t0 = fdiv(c, q), t1 = q * ia;
    lo = fminf(t0, t1);
    hi = fmaxf(t0, t1);
  }
  T root = lo;
  if (far_only || !(tmin <= root && root <= tmax)) {
    root = hi;
    if (!(tmin <= root && root <= tmax)) return false;
  }
  t = root;
  return true;
}

template <class R>
__device__ __forceinline__ V<R> sphere_center(const Sphere<R>& s, R time) {  // sphere.h:83
  V<R> c = ld3(s.c1);
  if (s.moving) c = c + time * ld3(s.dc);
  return c;
}

template <class R>
__device__ __forceinline__ bool sphere_test(V<R> c1, V<R> dc, R r, bool moving, V<R> o, V<R> d, R time, R tmin,
                                            R tmax, bool self, R& t) {
  V<R> c = moving ? c1 + time * dc : c1;  // sphere.h:83
  bool far_only = false;
  if (self) {
    if (dot(d, o - c) >= R(0)) return false;  // leaving the sphere it starts on
    far_only = true;
  }
  if constexpr (sizeof(R) == 4) {
    if (r > R(RT_BIG_SPHERE_R)) {
      // big spheres (the RTOW ground, r = 1000): |o-c|^2 - r^2 cancels catastrophically in fp32 (and
      // so does the perpendicular-distance discriminant of sphere_roots). Only that quantity is formed
      // in fp64; then disc = b^2 - a c and the roots q/a, c/q (q = b + sign(b) sqrt(disc)) have no
      // cancellation left except at a grazing double root.
      const double gx = (double)o.x - (double)c.x, gy = (double)o.y - (double)c.y, gz = (double)o.z - (double)c.z;
      const float cc = (float)((gx * gx + gy * gy + gz * gz) - (double)r * (double)r);
      const float a = d.x * d.x + d.y * d.y + d.z * d.z;
      const float bh = -(d.x * (float)gx + d.y * (float)gy + d.z * (float)gz);  // -b/2
      const float disc = bh * bh - a * cc;
      if (disc < 0.f) return false;
      const float q = bh + copysignf(fsqrt(disc), bh);
      const float r0 = fdiv(cc, q), r1 = fdiv(q, a);
      float root = fminf(r0, r1);
      if (far_only || !(tmin <= root && root <= tmax)) {
        root = fmaxf(r0, r1);
        if (!(tmin <= root && root <= tmax)) return false;
      }
      t = root;
      return true;
    }
  }
  return sphere_roots<R>(o.x, o.y, o.z, d.x, d.y, d.z, c.x, c.y, c.z, r, tmin, tmax, far_only, t);
}
template <class R>
__device__ __forceinline__ bool sphere_t(const Sphere<R>& s, V<R> o, V<R> d, R time, R tmin, R tmax, bool self, R& t) {
  return sphere_test(ld3(s.c1), ld3(s.dc), s.r, s.moving != 0, o, d, time, tmin, tmax, self, t);
}

// Wave-uniform read through the constant address space: always a scalar load (s_load),
// which the compiler cannot prove for a loop-carried prefetch from a generic pointer.
template <class T>
__device__ __forceinline__ T ld_uniform(const T* p, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
  i = __builtin_amdgcn_readfirstlane(i);
  return ((const __attribute__((address_space(4))) T*)p)[i];
#else
  return p[i];  // host pass of a device function: never executed
#endif
}
// A wave-uniform record into SGPRs by explicit scalar loads (s_load_dwordx16 / x8 / x4, one s_waitcnt for
// all of them). ld_uniform's constant-address-space load is turned back into per-lane vector loads
// (global_load with a zero VGPR offset) in the large persistent kernels (round 3: the flat program's
// record pairs, boxes and the linear program's records), each a VMEM issue and an L1 round trip.
typedef uint32_t SRegs16 __attribute__((ext_vector_type(16)));
typedef uint32_t SRegs8 __attribute__((ext_vector_type(8)));
typedef uint32_t SRegs4 __attribute__((ext_vector_type(4)));
template <class T>
__device__ __forceinline__ T ld_scalar(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr uint32_t n = sizeof(T) / 4;
  static_assert(sizeof(T) % 16 == 0 && n <= 32, "ld_scalar: 16-byte multiples up to 128 bytes");
  T t;
  if constexpr (n == 32) {
    SRegs16 a, b;
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b) : "s"(p));
    __builtin_memcpy((char*)&t, &a, 64);
    __builtin_memcpy((char*)&t + 64, &b, 64);
  } else if constexpr (n == 24) {
    SRegs16 a;
    SRegs8 b;
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx8 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b) : "s"(p));
    __builtin_memcpy((char*)&t, &a, 64);
    __builtin_memcpy((char*)&t + 64, &b, 32);
  } else if constexpr (n == 20) {
    SRegs16 a;
    SRegs4 b;
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx4 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b) : "s"(p));
    __builtin_memcpy((char*)&t, &a, 64);
    __builtin_memcpy((char*)&t + 64, &b, 16);
  } else if constexpr (n == 16) {
    SRegs16 a;
    asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=&s"(a) : "s"(p));
    __builtin_memcpy((char*)&t, &a, 64);
  } else if constexpr (n == 12) {
    SRegs8 a;
    SRegs4 b;
    asm volatile("s_load_dwordx8 %0, %2, 0x0\n\ts_load_dwordx4 %1, %2, 0x20\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b) : "s"(p));
    __builtin_memcpy((char*)&t, &a, 32);
    __builtin_memcpy((char*)&t + 32, &b, 16);
  } else if constexpr (n == 8) {
    SRegs8 a;
    asm volatile("s_load_dwordx8 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=&s"(a) : "s"(p));
    __builtin_memcpy((char*)&t, &a, 32);
  } else {
    static_assert(n == 4, "ld_scalar size");
    SRegs4 a;
    asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=&s"(a) : "s"(p));
    __builtin_memcpy((char*)&t, &a, 16);
  }
  return t;
#else
  return ld_uniform(p, 0);
#endif
}
// ld_uniform at the point of use: the index is an opaque zero, so the scalar load cannot be
// hoisted out of the path loop. Loop-invariant uniforms (the light, the camera) hoisted to the
// kernel entry outlive the SGPR budget and are spilled into VGPR lanes, and every use then costs
// a v_readlane (a VALU issue slot); a scalar reload from the constant cache costs none.
template <class T>
__device__ __forceinline__ T ld_here(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return ((const __attribute__((address_space(4))) T*)p)[z];
#else
  return *p;
#endif
}

// Per-ray reciprocal direction for fdiv_inv (fp32 fast path only).
template <class R>
__device__ __forceinline__ V<R> rcp3(V<R> d) {
#ifndef RT_PRECISE_F32
  if constexpr (sizeof(R) == 4)
    return mkv(__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z));
#endif
  return d;
}
// 1/d for the flat program: v_rcp_f32 in fp32 (as rcp3), the refined reciprocal (frcp) in fp64
template <class R>
__device__ __forceinline__ V<R> flat_inv(V<R> d) {
  if constexpr (sizeof(R) == 4)
    return rcp3(d);
  else
    return mkv(frcp(d.x), frcp(d.y), frcp(d.z));
}

// Axis-aligned quad (rt_scene.h LinRec): n = +-e_A exactly, so quad.h:32-33 reduce to
// t = (q_A - o_A) / d_A bit for bit; alpha = (p_U - q_U) / u_U, beta = (p_V - q_V) / v_V.
template <int K, class R>
__device__ __forceinline__ R comp(V<R> v) {
  return K == 0 ? v.x : (K == 1 ? v.y : v.z);
}
// fp32 evaluates the test without branches: for non-negative floats the IEEE order is the
// order of the bit patterns, so with 0 < tmin <= tmax
//   tmin <= t <= tmax        <=>  bits(t) - bits(tmin) <= bits(tmax) - bits(tmin)  (unsigned)
//   0 <= alpha, beta <= 1     <=>  max(bits(alpha), bits(beta)) <= bits(1.0f)
// and NaN or negative values fail both. One compare each instead of a branch per condition.
// alpha = (p - lo) * inv is -0.0 on the quad's Q edge when inv < 0 (a negative edge vector, as
// box() faces have), which the reference accepts (0 <= -0.0) and the bit order would not: the
// product is formed as fma(p - lo, inv, +0.0), equal to it except that -0.0 becomes +0.0.
template <int A, int U, int W, class R>
__device__ __forceinline__ bool aquad_t(const R* f, V<R> o, V<R> d, V<R> inv, R tmin, R tmax, R& t) {
  const R th = fdiv_inv(f[0] - comp<A>(o), comp<A>(d), comp<A>(inv));
  if constexpr (sizeof(R) == 4) {
    const R a = __builtin_fmaf((comp<U>(o) + th * comp<U>(d)) - f[1], f[3], 0.0f);
    const R b = __builtin_fmaf((comp<W>(o) + th * comp<W>(d)) - f[2], f[4], 0.0f);
    const uint32_t lo = __float_as_uint(tmin);
    const bool in_t = __float_as_uint(th) - lo <= __float_as_uint(tmax) - lo;
    const bool in_ab = max(__float_as_uint(a), __float_as_uint(b)) <= 0x3f800000u;
    t = th;
    return in_t & in_ab;
  }
  // fp64 (round 6): the same without branches, as the flat program's quads: plain compares for t, the bit order for
  // alpha and beta (the products with the stored reciprocals 1/u_U, 1/v_V, within an ulp of pu / u_U) (C5 fp64
  // 2,121 -> 2,092 ms/frame, r06i)
  const R a = fma((comp<U>(o) + th * comp<U>(d)) - f[1], f[3], R(0));
  const R b = fma((comp<W>(o) + th * comp<W>(d)) - f[2], f[4], R(0));
  const bool in_t = (th >= tmin) & (th <= tmax);
  const uint64_t ua = (uint64_t)__double_as_longlong(a), ub = (uint64_t)__double_as_longlong(b);
  t = th;
  return in_t & (ua <= 0x3FF0000000000000ull) & (ub <= 0x3FF0000000000000ull);
}
template <class R>
__device__ __forceinline__ bool lin_quad_t(const LinRec<R>& r, V<R> o, V<R> d, V<R> inv, R tmin, R tmax, R& t) {
  switch (r.aux) {
    case 1: return aquad_t<2, 0, 1>(r.f, o, d, inv, tmin, tmax, t);
    case 2: return aquad_t<1, 0, 2>(r.f, o, d, inv, tmin, tmax, t);
    case 3: return aquad_t<2, 1, 0>(r.f, o, d, inv, tmin, tmax, t);
    case 4: return aquad_t<0, 1, 2>(r.f, o, d, inv, tmin, tmax, t);
    case 5: return aquad_t<1, 2, 0>(r.f, o, d, inv, tmin, tmax, t);
    case 6: return aquad_t<0, 2, 1>(r.f, o, d, inv, tmin, tmax, t);
    default: break;
  }
  // general quad: the fields of Quad<R> (quad.h:30-52)
  V<R> n = ld3(r.f);
  R th = fdiv(r.f[3] - dot(n, o), dot(n, d));
  if (!(tmin <= th && th <= tmax)) return false;
  V<R> p = (o + th * d) - ld3(r.f + 4);
  R a = dot(p, ld3(r.f + 7)), b = dot(p, ld3(r.f + 10));
  if (!(R(0) <= a && a <= R(1) && R(0) <= b && b <= R(1))) return false;
  t = th;
  return true;
}

// Closest hit over a primitive list (refs until END); used for volume boundaries.
template <class R>
__device__ bool list_closest(const DevScene<R>& sc, uint32_t pos, V<R> o, V<R> d, R time, R tmin, R tmax, R& t) {
  bool any = false;
  for (;; pos++) {
    uint32_t e = sc.refs[pos];
    if (e == kEnd) break;
    uint32_t ty = etype(e), i = epay(e);
    R th;
    bool h = false;
    if (ty == E_QUAD)
      h = quad_t(sc.quads[i], o, d, tmin, tmax, th);
    else if (ty == E_SPHERE)
      h = sphere_t(sc.spheres[i], o, d, time, tmin, tmax, false, th);
    else if (ty == E_TRI)
      h = tri_t(sc.tris[i], o, d, tmin, tmax, th);
    if (h) {
      any = true;
      tmax = th;
      t = th;
    }
  }
  return any;
}

// volumne::hit (volumne.h:18-46). o, d: the ray as the volume sees it.
// wo, wd: the world ray (the boundary's wrapper chain is absolute, world -> boundary space);
// d: the ray as the volume itself sees it (its length scales the free-flight distance).
// UNI: the volume is the same for the whole wave (the linear program): v is already in SGPRs and
// its instance is scalar-loaded too (a vector load of a uniform address costs a VMEM round trip).
template <class R, bool UNI = false>
__device__ bool volume_t(const DevScene<R>& sc, const Volume<R>& v, V<R> wo, V<R> wd, V<R> d, R time, R tmin,
                         R tmax, Keys k, uint32_t bounce, uint32_t& jv, R& t) {
  V<R> bo = wo, bd = wd;
  if (v.inst >= 0) {
    if constexpr (UNI) {
      const Instance<R> in = ld_uniform(sc.insts, (uint32_t)v.inst);
      chain_in_regs(in, bo, bd);
    } else {
      chain_in(sc.insts[v.inst], bo, bd);
    }
  }
  R t1 = R(0), t2 = R(0);  // set by the slab test or by list_closest before any use
  bool boxed = false;
  if (v.is_box) {
    // box() boundary: the closest face hit over (-inf, inf) is the slab entry, the next one past it
    // + 1e-4 the exit (volumne.h:21-22); fp32: the same t = (plane - o) * rcp(d) as the quad tests;
    // fp64 (round 3): the planes' distances by the refined division, within an ulp of the twelve quad
    // tests of the boundary list (C5 fp64 7,292 ms/frame before)
    V<R> inv;
    if constexpr (sizeof(R) == 4)
      inv = rcp3(bd);
    else
      inv = mkv(frcp(bd.x), frcp(bd.y), frcp(bd.z));
    R tn = -Num<R>::inf(), tf = Num<R>::inf();
    const R los[3] = {v.lo[0], v.lo[1], v.lo[2]}, his[3] = {v.hi[0], v.hi[1], v.hi[2]};
    const R os[3] = {bo.x, bo.y, bo.z}, ds[3] = {bd.x, bd.y, bd.z}, is[3] = {inv.x, inv.y, inv.z};
#pragma unroll
    for (int a = 0; a < 3; a++) {
      R ta, tb;
      if constexpr (sizeof(R) == 4) {
        ta = fdiv_inv(los[a] - os[a], ds[a], is[a]);
        tb = fdiv_inv(his[a] - os[a], ds[a], is[a]);
      } else {
        ta = (los[a] - os[a]) * is[a];
        tb = (his[a] - os[a]) * is[a];
      }
      tn = fmax(tn, fmin(ta, tb));
      tf = fmin(tf, fmax(ta, tb));
    }
    if (!(tn <= tf) || !(tf >= tn + R(0.0001))) return false;
    t1 = tn;
    t2 = tf;
    boxed = true;
  }
  if (!boxed) {
    if (!list_closest(sc, epay(v.boundary), bo, bd, time, -Num<R>::inf(), Num<R>::inf(), t1)) return false;
    if (!list_closest(sc, epay(v.boundary), bo, bd, time, t1 + R(0.0001), Num<R>::inf(), t2)) return false;
  }
  if (t1 < tmin) t1 = tmin;
  if (t2 > tmax) t2 = tmax;
  if (t1 >= t2) return false;
  if (t1 < R(0)) t1 = R(0);
  R rl = len(d);
  R inside = (t2 - t1) * rl;
  R u = to_unit<R>(draw_u32(k.ks, dim_volume(bounce, jv++)));
  R hd = v.neg_inv_density * flog(u);
  if (hd > inside) return false;
  t = t1 + fdiv(hd, rl);
  return true;
}

// ------------------------------------------------------------------ traversal
// world.hit(r, interval(0.001, inf), rec) (camera.h:198) as a stack machine.
// excl_*: the surface the ray leaves (its previous hit); in fp32 a planar primitive
// cannot be re-hit from its own surface, a sphere only through its far side (fp64: no exclusion).
#ifdef RT_SECTION_CLOCKS
// development build: traversal counts (pops, node pops, primitive tests), summed over rays
__device__ unsigned long long g_trace_totals[3];
#define g_trace_counts tc
#endif
template <class R, int STACK, int BLOCK>
__device__ void trace(const DevScene<R>& sc, const Node<R>* nodes, V<R> wo, V<R> wd, R time, uint32_t excl_e,
                      int32_t excl_i, Keys keys, uint32_t bounce, uint32_t xy, uint32_t* stk, R& t_best, uint32_t& e_best,
                      int32_t& i_best) {
  const R tmin = R(0.001);
  R tmax = Num<R>::inf();
  V<R> o = wo, d = wd;
  V<R> inv = box_inv(d);
  int32_t cur = -1;
  uint32_t jv = 0;
  int sp = 0;
#ifdef RT_SECTION_CLOCKS
  uint32_t tc[3] = {0, 0, 0};
#endif
  e_best = kNoHit;
  i_best = -1;
  stk[0] = sc.root;
  sp = 1;

  auto test_prim = [&](uint32_t e) {
#ifdef RT_SECTION_CLOCKS
    g_trace_counts[2] += 1;
#endif
    uint32_t ty = etype(e), i = epay(e);
    // (fp32 only: in fp64 the surface a ray leaves is re-hit at ~ulp(o) / |d.n|, below tmin unless the ray grazes it,
    // when the reference's own test, which excludes nothing, re-hits it too -- the flat program's argument, round 6)
    const bool self = sizeof(R) == 4 && (e == excl_e) && (cur == excl_i);
    R th;
    bool h;
    if (ty == E_QUAD) {
      if (self) return;
      h = quad_t_near(sc, i, o, d, tmin, tmax, th, EdgeRay{keys.ks, xy, bounce}, cur < 0);
    } else if (ty == E_SPHERE) {
      h = sphere_t(sc.spheres[i], o, d, time, tmin, tmax, self, th);
    } else {
      if (self) return;
      h = tri_t(sc.tris[i], o, d, tmin, tmax, th);
    }
    if (h) {
      tmax = th;
      e_best = e;
      i_best = cur;
    }
  };
  auto test_volume = [&](uint32_t e) {
    R th;
    if (volume_t(sc, sc.vols[epay(e)], wo, wd, d, time, tmin, tmax, keys, bounce, jv, th)) {
      tmax = th;
      e_best = e;
      i_best = cur;
    }
  };

  // "while-while" traversal (Aila & Laine 2009): each lane walks inner nodes until it holds a
  // leaf entry (or its stack is empty), then the wave handles leaves together, so the box-test
  // code and the primitive code are not both executed on every iteration of a divergent loop.
  for (;;) {
    uint32_t e = kEnd;
    while (sp > 0) {
      const uint32_t x = stk[(--sp) * BLOCK];
#ifdef RT_SECTION_CLOCKS
      g_trace_counts[0] += 1;  // pops (per lane; divided by segments on the host)
      if (etype(x) == E_NODE) g_trace_counts[1] += 1;
#endif
      if (etype(x) != E_NODE) {
        e = x;
        break;
      }
      const Node<R>& nd = nodes[epay(x)];  // sc.nodes, or their copy in LDS
      R t0, t1;
      bool h0 = box_hit(nd.lo[0], nd.hi[0], o, inv, tmin, tmax, t0);
      bool h1 = box_hit(nd.lo[1], nd.hi[1], o, inv, tmin, tmax, t1);
      uint32_t c0 = nd.child[0], c1 = nd.child[1];
      if (h0 && h1) {
        if (t1 < t0) {
          uint32_t tmp = c0;
          c0 = c1;
          c1 = tmp;
        }
        stk[(sp++) * BLOCK] = c1;  // far first, near on top
        stk[(sp++) * BLOCK] = c0;
      } else if (h0) {
        stk[(sp++) * BLOCK] = c0;
      } else if (h1) {
        stk[(sp++) * BLOCK] = c1;
      }
    }
    if (e == kEnd) break;
    const uint32_t ty = etype(e);
    if (ty == E_LIST) {
      uint32_t pos = epay(e);
      for (;;) {
        uint32_t r = sc.refs[pos];
        if (r == kEnd) break;
        uint32_t rt = etype(r);
        if (rt <= E_TRI) {
          test_prim(r);
        } else if (rt == E_VOLUME) {
          test_volume(r);
        } else {
          if (sc.refs[pos + 1] != kEnd) stk[(sp++) * BLOCK] = mk(E_LIST, pos + 1);
          stk[(sp++) * BLOCK] = r;
          break;
        }
        pos++;
      }
    } else if (ty <= E_TRI) {
      test_prim(e);
    } else if (ty == E_INSTANCE) {
      const Instance<R>& in = sc.insts[epay(e)];
      stk[(sp++) * BLOCK] = kRestoreBase + (uint32_t)(cur + 1);
      stk[(sp++) * BLOCK] = in.blas;
      cur = (int32_t)epay(e);
      o = wo;
      d = wd;
      chain_in(in, o, d);
      inv = box_inv(d);
    } else if (ty == E_VOLUME) {
      test_volume(e);
    } else {  // RESTORE(k)
      cur = (int32_t)(e - kRestoreBase) - 1;
      o = wo;
      d = wd;
      if (cur >= 0) chain_in(sc.insts[cur], o, d);
      inv = box_inv(d);
    }
  }
  t_best = tmax;
#ifdef RT_SECTION_CLOCKS
  atomicAdd(&g_trace_totals[0], (unsigned long long)tc[0]);
  atomicAdd(&g_trace_totals[1], (unsigned long long)tc[1]);
  atomicAdd(&g_trace_totals[2], (unsigned long long)tc[2]);
#endif
}

// Wide BVH traversal (fp32, rt_scene.h WNode): world-level primitives only, so no instance
// state and no volume draws. Each node tests its four child boxes at once (independent slab
// tests, which hide one another's latency), sorts the hits near-to-far with a 5-comparator
// network on (t bits | slot) keys, continues with the nearest in a register and pushes the
// others to the per-lane LDS stack (far first). Leaves walk their primitive words in place.
// Primitive tests are the same functions as the other traversals (bit-identical hits); the
// closest hit differs from the binary BVH's only on exact-t ties.
// LDS copy of a node: 144-byte stride (36 dwords), so the 16 lanes of a ds_read_b128 group that
// read 16 consecutive nodes hit 16 distinct 4-bank windows (a 128-byte stride gives 2).
constexpr uint32_t kWNodeLdsStride = 144;
// The LDS copy of the top of a tree in HBM (RT_WIDE_TOP, fp32 rays): a node's six plane rows and its child codes,
// 112 bytes (28 banks) apart, so the 4-bank windows of 16 consecutive nodes are 16 distinct ones of the 64 banks.
// The WNode stride of 128 bytes put every node's row r on one of only two windows: lanes reading the top of the
// tree serialised on the banks (C4 fp32: 43 G bank-conflict cycles per launch against 93 G of LDS activity,
// r05fin4_c4_f32_pmc.json).
// (112 against the 128-byte stride measured the same time, 264.6 / 264.9 ms/frame, r06a; the conflicts: §4 of DESIGN.md)
constexpr uint32_t kWTopStride = 112;
#ifdef RT_SECTION_CLOCKS
// development build (scripts/dev_wide_stats.py): wave-level counts of the wide kernels, per block
// in LDS, added to g_wide_stats at the end: [0] node-loop iterations, [1] lanes in them, [2]
// primitive tests (wave iterations), [3] lanes in them, [4] shade calls, [5] lanes in them,
// [6] trace clocks, [7] shade clocks (both per wave, summed), [8] finished samples, [9] lanes in them
__device__ unsigned long long g_wide_stats[10];
__device__ __forceinline__ unsigned long long* wide_stats_lds() {
  __shared__ unsigned long long ws[10];
  return ws;
}
__device__ __forceinline__ void wide_stat(int k) {  // one wave-level event with the calling lanes
  const uint64_t m = __ballot(1);
  if (__lane_id() == (uint32_t)__ffsll((unsigned long long)m) - 1) {
    atomicAdd(wide_stats_lds() + k, 1ull);
    atomicAdd(wide_stats_lds() + k + 1, (unsigned long long)__popcll(m));
  }
}
#define RT_WIDE_STAT(k) wide_stat(k)
#else
#define RT_WIDE_STAT(k)
#endif
// The traversal of one ray is resumable: (cur, sp, tmax, e_best) and the LDS stack are its whole
// state. It returns true once the ray is finished, or false -- the ray paused -- when `pause` of
// the wave's lanes that entered are finished and waiting: the persistent kernel then shades those
// together and the paused lanes carry on beside the new rays (trace_wide callers in rt_kernels.hip).
// Without the pause a wave would traverse until its slowest ray is done, its finished lanes idle.
template <class R>
struct WideRayT {
  uint32_t cur;   // node index or leaf code to visit next
  int32_t sp;     // entries on the LDS stack
  R tmax;         // closest hit so far
  uint32_t e;     // its entry (kNoHit: none)
  uint32_t fresh; // 1: the head primitives (DevScene::wide_big) are still to be tested
};
// An LDS-resident tree (LDSN) is small: its child codes are rewritten to 16 bits when it is copied
// into LDS -- a node as its LDS offset in 16-byte units (index * 9 < 2^15), a leaf as
// 0x8000 | (count - 1) << 12 | first word (< 2^12) -- which halves the per-lane stack (uint16
// entries), and with it the LDS a block needs; the four codes of a node are one 8-byte word.
constexpr uint32_t kWLeaf16 = 0x8000u;
constexpr uint32_t kWNodeLdsUnits = kWNodeLdsStride / 16u;
__host__ __device__ __forceinline__ uint32_t wide_code16(uint32_t c) {
  return (c & kWLeaf) ? (kWLeaf16 | (((c >> kWCountShift) & 7u) << 12) | (c & 0xFFFu)) : c * kWNodeLdsUnits;
}
template <bool LDSN>
using WStackT = typename std::conditional<LDSN, uint16_t, uint32_t>::type;
// fp64 rays (round 3) traverse the same float boxes: the ray is rounded to float for the slab tests
// and every slab is widened by the distance the rounding moved the origin along that axis, |delta_a|
// / |d_a| (delta = o - float(o), exact in double, scaled by 1 + 2^-20), the direction's rounding
// being covered, like the fp32 path's own, by the relative box_slack of the exit distance; the
// lower bound is 0.00099 instead of 0.001. The boxes only cull: the primitive tests are the fp64
// ones of the other fp64 traversals, so the closest hit is theirs (exact-t ties aside).
template <class R, bool SPH, bool TRI, bool QUAD, bool MOV, bool LDSN, int BLOCK, int PAUSE>
__device__ __forceinline__ bool trace_wide(const DevScene<R>& sc, const unsigned char* lds_nodes,
                                           const typename WWord<R>::T* lds_prims, V<R> ro, V<R> rd, R time,
                                           uint32_t excl_e, WStackT<LDSN>* stk, WideRayT<R>& ry) {
  using WW = typename WWord<R>::T;
  constexpr bool F64 = sizeof(R) == 8;
  constexpr uint32_t kLeafBit = LDSN ? kWLeaf16 : kWLeaf;
  const R tmin = R(0.001);
  const float tmin_box = F64 ? 0.00099f : 0.001f;
  const V<float> o = mkv((float)ro.x, (float)ro.y, (float)ro.z);
  V<float> inv = box_inv(mkv((float)rd.x, (float)rd.y, (float)rd.z));
  [[maybe_unused]] float wx = 0.f, wy = 0.f, wz = 0.f;  // fp64: the slab widening per axis
  if constexpr (F64) {
    // A direction component that is 0 in float (an exactly axis-parallel ray: a cosine sample with r2 = 0,
    // random_cosine_direction's (0, 1, 0), about 10 times per C4 frame) gives inv = inf, and an infinite
    // widening made that axis cull nothing: the ray visited most of the tree (C4 fp64: single items of
    // 260-400 ms, the frame's tail, r05n/r05o). Such an axis takes inv = +-2^100 instead, and the widening
    // covers the origin's rounding plus an ulp of it (a plane exactly through the float origin):
    // (|delta| + |o| 2^-22 + 2^-126) 2^100. Any box the exact test accepts still passes.
    auto widen = [](double dlt, float oa, float& iv) {
      if (!(fabsf(iv) < 1.2676506002282294e30f)) {  // 2^100 (inf, or a float direction that underflowed)
        iv = __builtin_copysignf(1.2676506002282294e30f, iv);
        return ((float)fabs(dlt) + fabsf(oa) * 2.384185791015625e-07f + 1.1754943508222875e-38f) *
               1.2676506002282294e30f * (1.0f + 9.5367431640625e-07f);
      }
      return dlt == 0.0 ? 0.f : fabsf((float)dlt * iv) * (1.0f + 9.5367431640625e-07f);
    };
    wx = widen(ro.x - (double)o.x, o.x, inv.x);
    wy = widen(ro.y - (double)o.y, o.y, inv.y);
    wz = widen(ro.z - (double)o.z, o.z, inv.z);
  }
  const WW* prims = LDSN ? lds_prims : sc.wprims;
  uint32_t keep_going = 0;  // pause at or below this many traversing lanes
  if constexpr (PAUSE < 64) {
    const uint32_t entered = (uint32_t)__popcll(__ballot(1));
    keep_going = entered > (uint32_t)PAUSE ? entered - (uint32_t)PAUSE : 0u;
  }
  uint32_t cur = ry.cur;
  int sp = ry.sp;
  R tmax = ry.tmax;
  uint32_t e_best = ry.e;
  // the lane's stack: LDS, and for a tree in HBM its spill area past wide_lds_stack<R>() entries
  constexpr uint32_t kWideLdsStack = wide_lds_stack<R>();
  [[maybe_unused]] const uint32_t lane = blockIdx.x * BLOCK + threadIdx.x;
  auto push = [&](uint32_t v) {
    if (LDSN || sp < (int)kWideLdsStack)
      stk[sp * BLOCK] = (WStackT<LDSN>)v;
    else
      sc.wide_spill[(uint32_t)(sp - (int)kWideLdsStack) * sc.spill_lanes + lane] = v;
    sp++;
  };
  // (Round 3 measured three rewrites of push / pop / child below that the compiler's branchy code
  // beat on C4 / C3: a branch-free push writing the entry either way, 358.9 -> 365.9 / 60.76 -> 61.84
  // ms; the child code chosen by masks instead of ?:, 388.5 ms; a clamped LDS pop, neutral.)
  auto pop = [&]() -> uint32_t {
    --sp;
    if (LDSN || sp < (int)kWideLdsStack) return stk[sp * BLOCK];
    return sc.wide_spill[(uint32_t)(sp - (int)kWideLdsStack) * sc.spill_lanes + lane];
  };
  // Node tests (round 3). Octant-ordered: per axis the near plane (lo for a positive direction, hi
  // for a negative one) is read from its byte offset in the node (lo_a at 16a, hi_a at 48 + 16a), so a
  // child needs no min/max per axis. fp64 rays (RT_WIDE_FMA): each plane distance is one fma,
  // p * inv + c with c = -o * inv per ray; c carries the rounding of o * inv: the near constant is
  // lowered and the far one raised by |o * inv| 2^-22 (> twice the two roundings involved) plus the
  // widening w of the ray's rounding to float, the fma's own rounding being covered, like the
  // subtraction's, by box_slack. A direction component of 0 gives inv = inf: its planes' distances
  // are NaN or -inf, which the IEEE min/max ignore (no culling on that axis, as before). The six
  // constants cost the fp32 kernels, at their tighter register budgets, more spills than the fmas
  // save (C4 fp32 351 -> 460 ms/frame; fp64 C3 89.8 -> 81.7, C4 561 -> 545), so fp32 keeps
  // (p - o) * inv, octant-ordered (RT_WIDE_OCT32: C3 fp32 60.9 -> 57.2, C4 351.9 -> 341.6).
  // RT_WIDE_FMA32 (round 4): fp32 rays form p * inv + c too, with c = -o * inv rounded and ONE per-ray
  // bound instead of six constants: each distance is within |o_a * inv_a| 2^-24 of (p - o) * inv
  // (c's rounding; the fma's own is relative, covered by box_slack), so the test tn <= tf * slack +
  // 2 e with e = max_a |o_a inv_a| 2^-23 accepts every box the exact test accepts. An infinite or NaN
  // o_a * inv_a (a zero direction component) gives planes of the right sign or NaN, and no bound.
  // Over a tree in HBM (C4 stand-in) the one bound culls too little: a ray with a small direction
  // component has a large o_a * inv_a, and the bound then widens every axis (C4 fp32 310.7 -> 378.5
  // ms/frame; C3 49.8 -> 48.8). RT_WIDE_FMA32=2: per-axis constants, as the fp64 rays'.
  constexpr bool kFma = (F64) || (!F64 && LDSN && RT_WIDE_FMA32 == 2);
  constexpr bool kFma32 = !F64 && LDSN && RT_WIDE_FMA32 == 1;
  constexpr bool kOct = kFma || kFma32 || (!F64);
  [[maybe_unused]] const uint32_t onx0 = (__float_as_uint(inv.x) >> 31) * 48u,
                                 ony0 = 16u + (__float_as_uint(inv.y) >> 31) * 48u,
                                 onz0 = 32u + (__float_as_uint(inv.z) >> 31) * 48u;
  // RT_WIDE_OCTPACK: the three near-plane offsets packed in one register and unpacked per node visit
  // (three bit-field extracts instead of two registers held through the traversal)
  [[maybe_unused]] uint32_t oct = onx0 | ony0 << 8 | onz0 << 16;
  [[maybe_unused]] float cnx = 0.f, cny = 0.f, cnz = 0.f, cfx = 0.f, cfy = 0.f, cfz = 0.f;
  if constexpr (kFma) {
    auto cpair = [](float oa, float ia, float wa, float& cn, float& cf) {
      const float oi = oa * ia;
      const float ea = fmaf(fabsf(oi), 2.384185791015625e-07f, wa);
      cn = -oi - ea;
      cf = -oi + ea;
    };
    cpair(o.x, inv.x, wx, cnx, cfx);
    cpair(o.y, inv.y, wy, cny, cfy);
    cpair(o.z, inv.z, wz, cnz, cfz);
  }
  [[maybe_unused]] float e2 = 0.f;  // kFma32: twice the bound e
  if constexpr (kFma32) {
    auto cterm = [](float oa, float ia, float& c) {
      const float oi = oa * ia;
      c = -oi;
      return fabsf(oi) < Num<float>::inf() ? fabsf(oi) : 0.f;
    };
    const float m = fmaxf(fmaxf(cterm(o.x, inv.x, cnx), cterm(o.y, inv.y, cny)), cterm(o.z, inv.z, cnz));
    e2 = m * 2.384185791015625e-07f;  // 2^-22
  }
  // the four children's sort keys (bits(t_near) with the slot in the low 2 bits; 0xFFFFFFFF: missed)
  // of the float node at nb (LDS or HBM)
  // (a tree in HBM is addressed as its base plus a 32-bit byte offset, so each load is one global_load
  // with the base in SGPRs and the offset in one VGPR, not a 64-bit address per plane)
  // (RT_WIDE_OFS64: the fp64 kernels keep 64-bit addresses)
  constexpr bool kOfs = LDSN || !F64;
  const unsigned char* nbase = LDSN ? lds_nodes : (const unsigned char*)sc.wnodes;
  using OfsT = typename std::conditional<kOfs, uint32_t, uint64_t>::type;
  auto node_off = [](uint32_t c) -> OfsT { return LDSN ? (OfsT)(c << 4) : (OfsT)c * (OfsT)sizeof(WNode); };
  // a node's 16-byte rows: from the tree's memory, or (RT_WIDE_TOP) from the LDS copy of its first levels
  auto ld_mem = [&](OfsT off) -> float4 { return *(const float4*)(nbase + off); };
  using LdsF = const __attribute__((address_space(3))) float;
  [[maybe_unused]] auto ld_top = [&](OfsT off) -> float4 {
    LdsF* q = (LdsF*)(lds_nodes + off);
    return make_float4(q[0], q[1], q[2], q[3]);
  };
  auto node_keys_from = [&](auto ld4, OfsT nof, uint32_t& k0, uint32_t& k1, uint32_t& k2, uint32_t& k3) {
    const float tmx = (float)tmax;
    // tn >= tmin > 0: the bit pattern orders like the value; the low 2 bits carry the slot
    auto keyof = [](float tn, float tf, uint32_t c) {
      return tn <= tf ? ((__float_as_uint(tn) & ~3u) | c) : 0xFFFFFFFFu;
    };
    if constexpr (kOct) {
      uint32_t onx = onx0, ony = ony0, onz = onz0;
      {  // (RT_WIDE_OCTPACK, always on)
        asm volatile("" : "+v"(oct));  // not loop-invariant to the compiler: unpacked here, per visit
        onx = oct & 0xFFu;
        ony = (oct >> 8) & 0xFFu;
        onz = oct >> 16;
      }
      const float4 nx = ld4(nof + onx), ny = ld4(nof + ony), nz = ld4(nof + onz);
      const float4 fx = ld4(nof + (48u - onx)), fy = ld4(nof + (80u - ony)), fz = ld4(nof + (112u - onz));
      auto key = [&](float px, float py, float pz, float qx, float qy, float qz, uint32_t c) {
        float tn, tf;
        if constexpr (kFma) {
          tn = fmaxf(fmaxf(fmaf(px, inv.x, cnx), fmaf(py, inv.y, cny)), fmaxf(fmaf(pz, inv.z, cnz), tmin_box));
          tf = fminf(fminf(fmaf(qx, inv.x, cfx), fmaf(qy, inv.y, cfy)), fminf(fmaf(qz, inv.z, cfz), tmx));
        } else if constexpr (kFma32) {
          tn = fmaxf(fmaxf(fmaf(px, inv.x, cnx), fmaf(py, inv.y, cny)), fmaxf(fmaf(pz, inv.z, cnz), tmin_box));
          tf = fminf(fminf(fmaf(qx, inv.x, cnx), fmaf(qy, inv.y, cny)), fminf(fmaf(qz, inv.z, cnz), tmx));
          return keyof(tn, fmaf(tf, Num<float>::box_slack(), e2), c);
        } else {
          tn = fmaxf(fmaxf((px - o.x) * inv.x, (py - o.y) * inv.y), fmaxf((pz - o.z) * inv.z, tmin_box));
          tf = fminf(fminf((qx - o.x) * inv.x, (qy - o.y) * inv.y), fminf((qz - o.z) * inv.z, tmx));
        }
        return keyof(tn, tf * Num<float>::box_slack(), c);
      };
      k0 = key(nx.x, ny.x, nz.x, fx.x, fy.x, fz.x, 0u);
      k1 = key(nx.y, ny.y, nz.y, fx.y, fy.y, fz.y, 1u);
      k2 = key(nx.z, ny.z, nz.z, fx.z, fy.z, fz.z, 2u);
      k3 = key(nx.w, ny.w, nz.w, fx.w, fy.w, fz.w, 3u);
    } else {
      const float4* nd = (const float4*)(nbase + nof);
      const float4 lx = nd[0], ly = nd[1], lz = nd[2], hx = nd[3], hy = nd[4], hz = nd[5];
      auto slab = [&](float lx, float ly, float lz, float hx, float hy, float hz, uint32_t c) {
        const float tx0 = (lx - o.x) * inv.x, tx1 = (hx - o.x) * inv.x;
        const float ty0 = (ly - o.y) * inv.y, ty1 = (hy - o.y) * inv.y;
        const float tz0 = (lz - o.z) * inv.z, tz1 = (hz - o.z) * inv.z;
        float tn, tf;
        if constexpr (F64) {
          tn = fmaxf(fmaxf(fminf(tx0, tx1) - wx, fminf(ty0, ty1) - wy), fmaxf(fminf(tz0, tz1) - wz, tmin_box));
          tf = fminf(fminf(fmaxf(tx0, tx1) + wx, fmaxf(ty0, ty1) + wy), fminf(fmaxf(tz0, tz1) + wz, tmx));
        } else {
          tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), tmin_box));
          tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmx));
        }
        return keyof(tn, tf * Num<float>::box_slack(), c);
      };
      k0 = slab(lx.x, ly.x, lz.x, hx.x, hy.x, hz.x, 0u);
      k1 = slab(lx.y, ly.y, lz.y, hx.y, hy.y, hz.y, 1u);
      k2 = slab(lx.z, ly.z, lz.z, hx.z, hy.z, hz.z, 2u);
      k3 = slab(lx.w, ly.w, lz.w, hx.w, hy.w, hz.w, 3u);
    }
  };
  auto node_keys = [&](OfsT nof, uint32_t& k0, uint32_t& k1, uint32_t& k2, uint32_t& k3) {
    node_keys_from(ld_mem, nof, k0, k1, k2, k3);
  };
  // RT_WIDE_TOP (fp32 rays over a tree in HBM): nodes [0, wide_top) -- the first levels, which every ray
  // visits -- are read from the LDS copy the kernel made at its start (WideTrav::fill), so those visits
  // take no slot of the L1 address path, the C4 kernel's bound
  constexpr bool kTopL = !LDSN && !F64;
  [[maybe_unused]] const uint32_t ntop = kTopL ? min(sc.wide_top, (uint32_t)RT_WIDE_TOP_N) : 0u;
  // RT_WIDE_HALF_F64: the keys of node c from the tree's fp16 form (rt_scene.h WNodeH), and its child codes.
  // A plane's distance is one fma of its fp16 offset (v_fma_mix_f32): h * inv + b, b = (origin - o) *
  // inv per node and axis. b carries two roundings, |b| 2^-23 at most: the near planes take b - e and
  // the far ones b + e, e = |b| 2^-22 + the fp64 ray's widening w, so no box the float node would enter
  // is culled; the fma's own rounding is relative, covered by box_slack like the float path's. The near
  // and far words of each axis are picked by v_perm_b32 with a per-ray selector (0x07060504: the hi
  // word, for a negative direction; 0x03020100: the lo word).
  constexpr bool kHalf = !LDSN && F64;
  [[maybe_unused]] const unsigned char* hbase = kHalf ? (const unsigned char*)sc.wnodesh : nullptr;
  [[maybe_unused]] const uint32_t selx = (__float_as_uint(inv.x) >> 31) ? 0x07060504u : 0x03020100u,
                                  sely = (__float_as_uint(inv.y) >> 31) ? 0x07060504u : 0x03020100u,
                                  selz = (__float_as_uint(inv.z) >> 31) ? 0x07060504u : 0x03020100u;
  // the node's 16-byte words from the tree in HBM, or (RT_WIDE_TOP_F64) from the LDS copy of its first levels
  [[maybe_unused]] auto ldh_mem = [&](uint32_t off) -> uint4 { return *(const uint4*)(hbase + off); };
  using LdsU = const __attribute__((address_space(3))) uint32_t;
  [[maybe_unused]] auto ldh_top = [&](uint32_t off) -> uint4 {
    LdsU* q = (LdsU*)(lds_nodes + off);
    return make_uint4(q[0], q[1], q[2], q[3]);
  };
  [[maybe_unused]] auto half_keys_from = [&](auto ld16, uint32_t c, uint32_t& k0, uint32_t& k1, uint32_t& k2,
                                             uint32_t& k3, uint4& cc) {
    const uint32_t hp = c * (uint32_t)sizeof(WNodeH);
    const uint4 h0 = ld16(hp);
    uint4 h1 = ld16(hp + 16), h2 = ld16(hp + 32), h3 = ld16(hp + 48);
    cc = ld16(hp + 64);
    {  // lo: x h1.xy, y h1.zw, z h2.xy; hi: x h2.zw, y h3.xy, z h3.zw -> near in the lo words, far in the hi
      auto pick = [](uint32_t& lo, uint32_t& hi, uint32_t sel) {
        const uint32_t n = __builtin_amdgcn_perm(hi, lo, sel), f = __builtin_amdgcn_perm(lo, hi, sel);
        lo = n;
        hi = f;
      };
      pick(h1.x, h2.z, selx);
      pick(h1.y, h2.w, selx);
      pick(h1.z, h3.x, sely);
      pick(h1.w, h3.y, sely);
      pick(h2.x, h3.z, selz);
      pick(h2.y, h3.w, selz);
    }
    const float tmx = (float)tmax;
    auto bounds = [](float org, float oa, float iv, float wa, float& bn, float& bf) {
      const float b = (org - oa) * iv;
      const float e = fmaf(fabsf(b), 2.384185791015625e-07f, wa);  // 2^-22
      bn = b - e;
      bf = b + e;
    };
    float bnx, bfx, bny, bfy, bnz, bfz;
    bounds(__uint_as_float(h0.x), o.x, inv.x, wx, bnx, bfx);
    bounds(__uint_as_float(h0.y), o.y, inv.y, wy, bny, bfy);
    bounds(__uint_as_float(h0.z), o.z, inv.z, wz, bnz, bfz);
    auto H = [](uint32_t w, bool hi) {
      return (float)__builtin_bit_cast(_Float16, (uint16_t)(hi ? (w >> 16) : (w & 0xFFFFu)));
    };
    // near: x h1.x h1.y, y h1.z h1.w, z h2.x h2.y; far: x h2.z h2.w, y h3.x h3.y, z h3.z h3.w
    auto key = [&](uint32_t nx, uint32_t ny, uint32_t nz, uint32_t fx, uint32_t fy, uint32_t fz, bool hi,
                   uint32_t slot) {
      const float tn = fmaxf(fmaxf(fmaf(H(nx, hi), inv.x, bnx), fmaf(H(ny, hi), inv.y, bny)),
                             fmaxf(fmaf(H(nz, hi), inv.z, bnz), tmin_box));
      const float tf = fminf(fminf(fmaf(H(fx, hi), inv.x, bfx), fmaf(H(fy, hi), inv.y, bfy)),
                             fminf(fmaf(H(fz, hi), inv.z, bfz), tmx)) *
                       Num<float>::box_slack();
      return tn <= tf ? ((__float_as_uint(tn) & ~3u) | slot) : 0xFFFFFFFFu;
    };
    k0 = key(h1.x, h1.z, h2.x, h2.z, h3.x, h3.z, false, 0u);
    k1 = key(h1.x, h1.z, h2.x, h2.z, h3.x, h3.z, true, 1u);
    k2 = key(h1.y, h1.w, h2.y, h2.w, h3.y, h3.w, false, 2u);
    k3 = key(h1.y, h1.w, h2.y, h2.w, h3.y, h3.w, true, 3u);
  };
  // the primitives of a leaf (or of the head list), their records from word w on
  // a primitive word by 32-bit byte offset from the base (one VGPR of address; see node_keys)
  auto pw = [&](uint32_t k) -> WW {
    if constexpr (kOfs) return *(const WW*)((const unsigned char*)prims + k * (uint32_t)sizeof(WW));
    return prims[k];
  };
  auto test_prims = [&](uint32_t w, uint32_t count) {
    for (uint32_t n = count; n > 0; n--) {
      RT_WIDE_STAT(2);
      const WW h = pw(w);
      // a kernel with triangles loads a record's next two words with its first (the word stream is
      // padded, rt_scene.h), so a triangle costs one memory latency, not two: its kind is in word 0
      [[maybe_unused]] WW a1{}, a2{};
      constexpr bool PF = TRI;
      if constexpr (PF) {
        a1 = pw(w + 1);
        a2 = pw(w + 2);
      }
      const uint32_t e = wentry(h);
      const uint32_t ty = etype(e);
      R th;
      bool hit = false;
      if (SPH && (!(TRI || QUAD) || ty == E_SPHERE)) {
        const WW b = PF ? a1 : pw(w + 1);
        w += 2;
        // (fp64 excludes nothing, as the reference: trace's note)
        hit = sphere_test(mkv(h.x, h.y, h.z), mkv(b.x, b.y, b.z), b.w, MOV, ro, rd, time, tmin, tmax, !F64 && e == excl_e, th);
      } else if (TRI && (!QUAD || ty == E_TRI)) {
        const WW a = PF ? a1 : pw(w + 1), b = PF ? a2 : pw(w + 2);
        w += 3;
        hit = (F64 || e != excl_e) && tri_test(mkv(h.x, h.y, h.z), mkv(a.x, a.y, a.z), mkv(b.x, b.y, b.z), ro, rd, tmin, tmax, th);
      } else if (QUAD) {
        const WW nD = PF ? a1 : pw(w + 1), qa = PF ? a2 : pw(w + 2), qb = pw(w + 3);
        // (no fp64 re-decision near edges here, unlike quad_t_near. Inline, its registers spilled the C4 fp32
        // kernel: 8 -> 104 B per lane, 264 -> 288 ms/frame (r05fin). As a call (quad_edge64, round 6) the state
        // saved around it spilled the kernel's loop instead: 264.6 -> 307.5 ms/frame, for a C4 lit fp32 RMSE
        // (fp32 against fp64 over 400 tiles) of 1.71e-4 -> 1.30e-4 -- the rest are triangle edges and the
        // fp32 paths' own rounding (r06a))
        hit = (F64 || e != excl_e) && quad_test(mkv(nD.x, nD.y, nD.z), nD.w, mkv(h.x, h.y, h.z), mkv(qa.x, qa.y, qa.z),
                                       mkv(qb.x, qb.y, qb.z), ro, rd, tmin, tmax, th);
        w += 4;
      }
      if (hit) {
        tmax = th;
        e_best = e;
      }
    }
  };
  [[maybe_unused]] auto half_keys = [&](uint32_t c, uint32_t& k0, uint32_t& k1, uint32_t& k2, uint32_t& k3, uint4& cc) {
    half_keys_from(ldh_mem, c, k0, k1, k2, k3, cc);
  };
  constexpr bool kTopH = kHalf;
  [[maybe_unused]] const uint32_t ntoph = kTopH ? min(sc.wide_top, (uint32_t)RT_WIDE_TOP_N_F64) : 0u;
  if (ry.fresh) {  // every lane alike: no divergence, and the tree starts bounded by their hit
    test_prims(0u, sc.wide_big);
    ry.fresh = 0;
  }
  bool done = false;
#ifdef RT_WIDE_DEBUG_LONG
  uint32_t dbg_visits = 0;
#endif
  // Speculative while-while (Aila & Laine 2009), for trees in HBM: a lane that reaches a leaf
  // postpones it and keeps traversing until every traversing lane of the wave holds one, so the
  // leaf tests run with the wave's lanes together instead of a few at a time, and node fetches
  // overlap. The postponed leaf is tested with the tmax of its time. C4 stand-in 459.6 -> 426.4
  // ms/frame; the LDS-resident C3 tree, whose node visits are cheap and whose leaves hold up to 6
  // spheres, lost (62.2 -> 63.6: nodes visited past a postponed leaf are not culled by its hits).
  if constexpr (!LDSN && RT_WIDE_SPEC) {
  bool have = true;  // cur holds a node or a leaf still to visit
  for (;;) {
    uint32_t leaf = 0u;  // the postponed leaf (a leaf code is never 0)
    while (have) {
      RT_WIDE_STAT(0);
#ifdef RT_WIDE_DEBUG_LONG  // development: a traversal far longer than the tree warrants
      if (++dbg_visits == 20000u)
        printf("[long] o=(%.17g %.17g %.17g) d=(%.17g %.17g %.17g) inv=(%g %g %g) w=(%g %g %g) tmax=%g sp=%d cur=%u\n",
               (double)ro.x, (double)ro.y, (double)ro.z, (double)rd.x, (double)rd.y, (double)rd.z, inv.x, inv.y, inv.z,
               wx, wy, wz, (double)tmax, sp, cur);
#endif
      if (cur & kLeafBit) {
        if (leaf) break;  // a second leaf: test the first, come back with this one
        leaf = cur;
        if (sp == 0) {
          have = false;
          break;
        }
        cur = pop();
      } else {
        uint4 cc{};
        uint32_t k0, k1, k2, k3;
        [[maybe_unused]] OfsT nof{};
        if constexpr (kTopH) {
          if (cur < ntoph)
            half_keys_from(ldh_top, cur, k0, k1, k2, k3, cc);
          else
            half_keys(cur, k0, k1, k2, k3, cc);
        } else if constexpr (kHalf) {
          half_keys(cur, k0, k1, k2, k3, cc);
        } else if constexpr (kTopL) {
          nof = node_off(cur);
          if (cur < ntop) {
            const OfsT tof = cur * kWTopStride;
            const float4 c4 = ld_top(tof + 96u);
            cc = make_uint4(__float_as_uint(c4.x), __float_as_uint(c4.y), __float_as_uint(c4.z), __float_as_uint(c4.w));
            node_keys_from(ld_top, tof, k0, k1, k2, k3);
          } else {
            cc = *(const uint4*)(nbase + (nof + 96u));
            node_keys(nof, k0, k1, k2, k3);
          }
        } else {
          nof = node_off(cur);
          if constexpr (!LDSN) cc = *(const uint4*)(nbase + (nof + 96u));
          node_keys(nof, k0, k1, k2, k3);
        }
        auto child = [&](uint32_t k) -> uint32_t {
          if constexpr (LDSN) {
            return ((const uint16_t*)(nbase + (nof + 96u)))[k & 3u];
          } else {
            const uint32_t sl = k & 3u;
            return sl == 0 ? cc.x : (sl == 1 ? cc.y : (sl == 2 ? cc.z : cc.w));
          }
        };
#define RT_CS(a, b)                 \
  {                                 \
    const uint32_t lo_ = min(a, b); \
    b = max(a, b);                  \
    a = lo_;                        \
  }
        RT_CS(k0, k1);
        RT_CS(k2, k3);
        RT_CS(k0, k2);
        RT_CS(k1, k3);
        RT_CS(k1, k2);
#undef RT_CS
        if (k0 == 0xFFFFFFFFu) {
          if (sp == 0) {
            have = false;
            break;
          }
          cur = pop();
        } else {
          if (k3 != 0xFFFFFFFFu) push(child(k3));
          if (k2 != 0xFFFFFFFFu) push(child(k2));
          if (k1 != 0xFFFFFFFFu) push(child(k1));
          cur = child(k0);
        }
      }
      const bool all_hold = __ballot(leaf == 0u) == 0ull;  // over the lanes still in this loop
      if (all_hold) break;
    }
    if (leaf)
      test_prims(LDSN ? (leaf & 0xFFFu) : (leaf & kWFirstMask),
                 (LDSN ? ((leaf >> 12) & 7u) : ((leaf >> kWCountShift) & 63u)) + 1u);
    if (!have) {
      done = true;
      break;
    }
    if constexpr (PAUSE < 64) {
      // active-ray control: once PAUSE of the lanes that entered have finished (__ballot count), the
      // others pause with their state in (cur, sp, tmax, e_best) and the LDS stack, the finished ones
      // are shaded and start their next rays, and the wave traverses again at full width
      if ((uint32_t)__popcll(__ballot(1)) <= keep_going) break;
    }
  }
  } else {
  for (;;) {
    while (!(cur & kLeafBit)) {  // inner nodes until this lane holds a leaf (while-while)
      RT_WIDE_STAT(0);
      const OfsT nof = node_off(cur);
      // LDS tree: a child's code is loaded when it is pushed (loading all four with the boxes keeps them
      // live through the slab tests and the sort, which spilled: C3 76.4 -> 81.5 ms/frame). Tree in HBM:
      // all four come with the boxes, one latency instead of one per push (C4 462 -> 421 ms/frame).
      // (Round 6: the LDS tree's four codes in one 8-byte read after the sort spilled 16 B more: C3 fp64 62.4 -> 65.7,
      // fp32 47.0 -> 49.4 ms/frame, r06i.)
      uint4 cc{};
      uint32_t k0, k1, k2, k3;
      if constexpr (kHalf) {
        half_keys(cur, k0, k1, k2, k3, cc);
      } else {
        if constexpr (!LDSN) cc = *(const uint4*)(nbase + (nof + 96u));
        node_keys(nof, k0, k1, k2, k3);
      }
      auto child = [&](uint32_t k) -> uint32_t {
        if constexpr (LDSN) {
          return ((const uint16_t*)(nbase + (nof + 96u)))[k & 3u];
        } else {
          const uint32_t sl = k & 3u;
          return sl == 0 ? cc.x : (sl == 1 ? cc.y : (sl == 2 ? cc.z : cc.w));
        }
      };
#define RT_CS(a, b)                 \
  {                                 \
    const uint32_t lo_ = min(a, b); \
    b = max(a, b);                  \
    a = lo_;                        \
  }
      RT_CS(k0, k1);
      RT_CS(k2, k3);
      RT_CS(k0, k2);
      RT_CS(k1, k3);
      RT_CS(k1, k2);
#undef RT_CS
      if (k0 == 0xFFFFFFFFu) {  // no child hit
        if (sp == 0) {
          done = true;
          break;
        }
        cur = pop();
        continue;
      }
      if (k3 != 0xFFFFFFFFu) push(child(k3));
      if (k2 != 0xFFFFFFFFu) push(child(k2));
      if (k1 != 0xFFFFFFFFu) push(child(k1));
      cur = child(k0);
    }
    if (done) break;
    test_prims(LDSN ? (cur & 0xFFFu) : (cur & kWFirstMask),
               (LDSN ? ((cur >> 12) & 7u) : ((cur >> kWCountShift) & 63u)) + 1u);
    if (sp == 0) {
      done = true;
      break;
    }
    cur = pop();
    if constexpr (PAUSE < 64) {
      if ((uint32_t)__popcll(__ballot(1)) <= keep_going) break;  // enough of the wave waits to be shaded
    }
  }
  }
  ry.cur = cur;
  ry.sp = sp;
  ry.tmax = tmax;
  ry.e = e_best;
  return done;
}

// Linear program (small scenes, rt_scene.h): every lane walks the same ops, so
// the loop, the op and the primitive records are wave-uniform (scalar loads).
template <class R, bool SPH, bool TRI, bool VOL>
__device__ __forceinline__ void trace_linear(const DevScene<R>& sc, V<R> wo, V<R> wd, R time, uint32_t excl_e,
                                             int32_t excl_i, Keys keys, uint32_t bounce, R& t_best,
                                             uint32_t& e_best, int32_t& i_best) {
  const R tmin = R(0.001);
  R tmax = Num<R>::inf();
  V<R> o = wo, d = wd;
  // fp32: v_rcp_f32 once per ray and instance (fp64 divides per quad: per-ray refined reciprocals were
  // neutral at 3 waves and cost 24 VGPRs)
  const V<R> winv = rcp3(wd);
  V<R> inv = winv;
  int32_t cur = -1;
  uint32_t jv = 0;
  e_best = kNoHit;
  i_best = -1;
  const uint32_t n = sc.n_linear;
  for (uint32_t k = 0; k < n; k++) {
    const LinRec<R> rec = ld_scalar(sc.lin + k);  // the whole record into SGPRs at once
    const uint32_t op = rec.op;
    const uint32_t ty = etype(op), idx = epay(op);
    R th;
    bool h = false;
    if (ty == E_QUAD) {
      if constexpr (sizeof(R) == 4)  // evaluated for every lane, excluded lanes masked (no branch)
        h = lin_quad_t(rec, o, d, inv, tmin, tmax, th) & !(op == excl_e && cur == excl_i);
      else  // fp64 excludes nothing, as the reference (trace's note)
        h = lin_quad_t(rec, o, d, inv, tmin, tmax, th);
    } else if (SPH && ty == E_SPHERE) {
      h = sphere_test(ld3(rec.f), ld3(rec.f + 4), rec.f[3], rec.aux != 0, o, d, time, tmin, tmax,
                      sizeof(R) == 4 && op == excl_e && cur == excl_i, th);
    } else if (TRI && ty == E_TRI) {
      if (sizeof(R) == 8 || !(op == excl_e && cur == excl_i)) {
        Tri<R> tr;
        for (int q = 0; q < 3; q++) {
          tr.p0[q] = rec.f[q];
          tr.e1[q] = rec.f[3 + q];
          tr.e2[q] = rec.f[6 + q];
        }
        h = tri_t(tr, o, d, tmin, tmax, th);
      }
    } else if (ty == E_INSTANCE) {  // the chain inline in the record (rt_scene.h LinRec)
      cur = (int32_t)idx;
      o = wo;
      d = wd;
      const uint32_t nops = rec.aux & 7u;
#pragma unroll
      for (uint32_t q = 0; q < (uint32_t)kMaxChain; q++) {
        if (q >= nops) break;
        XOp<R> x;
        x.kind = (int32_t)((rec.aux >> (4 + 2 * q)) & 3u);
        x.x = rec.f[3 * q];
        x.y = rec.f[3 * q + 1];
        x.z = rec.f[3 * q + 2];
        o = op_in(x, o, true);
        d = op_in(x, d, false);
      }
      inv = rcp3(d);
    } else if (VOL && ty == E_VOLUME) {
      const Volume<R> vol = ld_uniform(sc.vols, idx);
      h = volume_t<R, true>(sc, vol, wo, wd, d, time, tmin, tmax, keys, bounce, jv, th);
    } else {  // kInstEnd
      cur = -1;
      o = wo;
      d = wd;
      // fp64: recomputed rather than kept through the loop (6 registers)
      inv = winv;
    }
    if (h) {
      tmax = th;
      e_best = op;
      i_best = cur;
    }
  }
  t_best = tmax;
}

// ------------------------------------------------------------------ flat program
// rt_scene.h FlatQuadT / FlatBoxT: world-space axis-aligned quads in three branch-free loops
// (one per plane axis, records scalar-loaded in pairs), then the slab tests of the boxes.
// A quad is the aquad_t test (quad.h:30-64 for n = +-e_A); the record index of the closest
// hit is kept and turned into (entry, instance) once at the end. fp64 (round 3): the same
// program with the per-ray reciprocal 1/d in IEEE double, so a quad costs multiplies instead
// of the three fp64 divisions of the ordered linear program.
template <class R>
struct FlatQuad2 {
  FlatQuadT<R> a, b;
};
template <int A, class R>
__device__ __forceinline__ void flat_quad_test(const FlatQuadT<R>& r, int32_t idx, V<R> o, V<R> d, V<R> inv,
                                               R tmin, R& tmax, int32_t& best, uint64_t xkey) {
  constexpr int U = A == 0 ? 1 : 0, W = A == 2 ? 1 : 2;
  const R th = (r.plane - comp<A>(o)) * comp<A>(inv);
  // fma(., inv, +0.0): the product, with an exact edge hit's -0.0 as +0.0 (aquad_t)
  const R a = fma((comp<U>(o) + th * comp<U>(d)) - r.lo_u, r.inv_u, R(0));
  const R b = fma((comp<W>(o) + th * comp<W>(d)) - r.lo_w, r.inv_w, R(0));
  bool in_t, in_ab;
  if constexpr (sizeof(R) == 4) {
    const uint32_t lo = __float_as_uint(tmin);
    in_t = __float_as_uint(th) - lo <= __float_as_uint(tmax) - lo;
    in_ab = max(__float_as_uint(a), __float_as_uint(b)) <= 0x3f800000u;
  } else {
    // fp64 (round 4): two compares each, no 64-bit subtractions or max. Every compare costs ~4.7 SIMD
    // cycles whatever its width, a 64-bit add or a v_cndmask with an SGPR mask 4: the
    // order trick on the bit patterns (2 x v_lshl_add_u64 + compare: 12.7; the u64 max: compare + 2
    // selects + compare, 17.4) costs more than the plain tests (9.4 each). th in [tmin, tmax] with NaN
    // and -0.0 outside, as before; a, b in [0, 1] on the bit patterns (non-negative doubles order like
    // their bits; -0.0 and NaN are above 1.0's)
    in_t = (th >= tmin) & (th <= tmax);
    const uint64_t ua = (uint64_t)__double_as_longlong(a), ub = (uint64_t)__double_as_longlong(b);
    in_ab = (ua <= 0x3FF0000000000000ull) & (ub <= 0x3FF0000000000000ull);
  }
  // the quad the ray leaves is excluded in fp32 only: in fp64 its re-hit distance is ~ulp(o) / |d_A|, which
  // tmin rejects unless the ray grazes the quad, when the reference's quad test (quad.h:30-35, no exclusion)
  // re-hits it too -- the same argument as the boxes' faces below (round 6: one 64-bit compare per quad)
  bool keep = true;
  if constexpr (sizeof(R) == 4) keep = (((uint64_t)(uint32_t)r.inst << 32) | r.e) != xkey;
  const bool h = in_t & in_ab & keep;
  tmax = h ? th : tmax;
  best = h ? idx : best;
}
template <int A, class R>
__device__ __forceinline__ void flat_quads(const FlatQuadT<R>* q, uint32_t n, int32_t base, V<R> o, V<R> d,
                                           V<R> inv, R tmin, R& tmax, int32_t& best, uint64_t xkey) {
  // pairs of records in one scalar load each, then the odd one (round 3: groups are no longer padded
  // to pairs with never-hit records -- Cornell's y and z groups had one each, 2 of 8 quad tests)
#pragma unroll 1
  for (uint32_t k = 0; k + 1 < n; k += 2) {
    const FlatQuad2<R> r = ld_scalar(reinterpret_cast<const FlatQuad2<R>*>(q + k));
    flat_quad_test<A>(r.a, base + (int32_t)k, o, d, inv, tmin, tmax, best, xkey);
    flat_quad_test<A>(r.b, base + (int32_t)k + 1, o, d, inv, tmin, tmax, best, xkey);
  }
  if (n & 1u) flat_quad_test<A>(ld_scalar(q + (n - 1)), base + (int32_t)(n - 1), o, d, inv, tmin, tmax, best, xkey);
}
// Slab test of a box (= the closest of its six quads): entry distance tn, or the exit tf for
// a ray that starts inside (what the quads give). A ray leaving one of the box's faces
// (excl_i == inst; the face is excl_e & 7, rt_scene.h) starts on that face's plane: its
// distance to it becomes -inf, i.e. the plane is behind the ray whichever way it goes --
// a ray going out then has tf < 0 (no hit), one going in exits through another face.
template <class R>
struct Slab {
  R t0[3], t1[3], tn, tf, th;
};
// fp64: no face exclusion. The face a ray leaves is at distance |t| ~ ulp(o) / |d_k| from it, below
// tmin = 0.001 unless the ray grazes the face, which is also when the reference's own quad test of that face
// (quad.h:30-35, no exclusion either) re-hits it; the six selects per box cost ~100 SIMD cycles per segment
// (C2 fp64 34.6 -> 32.7 ms/frame, parity unchanged). Distances as fma(p, inv, -o * inv) were
// 1.5 % faster but moved edge decisions (9 of 364,800 C2 pixels beyond 1e-9): not kept.
template <class R>
__device__ __forceinline__ Slab<R> flat_slab(const FlatBoxT<R>& b, V<R> o, V<R> inv, R tmin, int32_t excl_i,
                                             uint32_t xf) {
  Slab<R> s;
  const bool left = sizeof(R) == 4 && excl_i == b.inst;
  const R ninf = -Num<R>::inf();
  auto dist = [&](R p, R oa, R ia) { return (p - oa) * ia; };
  s.t0[0] = (left & (xf == 0)) ? ninf : dist(b.lo[0], o.x, inv.x);
  s.t1[0] = (left & (xf == 1)) ? ninf : dist(b.hi[0], o.x, inv.x);
  s.t0[1] = (left & (xf == 2)) ? ninf : dist(b.lo[1], o.y, inv.y);
  s.t1[1] = (left & (xf == 3)) ? ninf : dist(b.hi[1], o.y, inv.y);
  s.t0[2] = (left & (xf == 4)) ? ninf : dist(b.lo[2], o.z, inv.z);
  s.t1[2] = (left & (xf == 5)) ? ninf : dist(b.hi[2], o.z, inv.z);
  s.tn = fmax(fmax(fmin(s.t0[0], s.t1[0]), fmin(s.t0[1], s.t1[1])), fmin(s.t0[2], s.t1[2]));
  s.tf = fmin(fmin(fmax(s.t0[0], s.t1[0]), fmax(s.t0[1], s.t1[1])), fmax(s.t0[2], s.t1[2]));
  s.th = s.tn >= tmin ? s.tn : s.tf;
  return s;
}
// fq / fb: where the hit's record is read at the end (the scene's, or the kernel's LDS copy)
template <class R>
__device__ __forceinline__ void trace_flat(const DevScene<R>& sc, V<R> o, V<R> d, uint32_t excl_e, int32_t excl_i,
                                           R& t_best, uint32_t& e_best, int32_t& i_best, uint32_t& nm,
                                           const FlatQuadT<R>* fq, const FlatBoxT<R>* fb) {
  const R tmin = R(0.001);
  R tmax = Num<R>::inf();
  const V<R> inv = flat_inv(d);
  const uint64_t xkey = ((uint64_t)(uint32_t)excl_i << 32) | excl_e;
  const uint32_t xf = excl_e & 7u;
  int32_t best = -1;
  const uint32_t n0 = sc.n_flatq[0], n1 = sc.n_flatq[1], n2 = sc.n_flatq[2], nq = n0 + n1 + n2;
  flat_quads<0>(sc.flatq, n0, 0, o, d, inv, tmin, tmax, best, xkey);
  flat_quads<1>(sc.flatq + n0, n1, (int32_t)n0, o, d, inv, tmin, tmax, best, xkey);
  flat_quads<2>(sc.flatq + n0 + n1, n2, (int32_t)(n0 + n1), o, d, inv, tmin, tmax, best, xkey);
#pragma unroll 1
  for (uint32_t k = 0; k < sc.n_flatb; k++) {
    const FlatBoxT<R> b = ld_scalar(sc.flatb + k);
    const Slab<R> s = flat_slab(b, o, inv, tmin, excl_i, xf);
    // (tn <= tf) & (th >= tmin) & (th <= tmax) with one compare fewer: th is tn when tn >= tmin, else tf, so
    // tf >= max(tn, tmin) is the first two (round 6: C2 fp64 25.28 -> 25.27 ms/frame, fp32 18.37 -> 18.34, r06g)
    const bool h = (s.tf >= fmax(s.tn, tmin)) & (s.th <= tmax);
    tmax = h ? s.th : tmax;
    best = h ? (int32_t)(nq + k) : best;
  }
  t_best = tmax;
  e_best = kNoHit;
  i_best = -1;
  nm = 0;
  if (best < 0) return;
  if ((uint32_t)best < nq) {
    const FlatQuadT<R>& r = fq[best];
    e_best = r.e;
    i_best = r.inst;
    nm = r.nm;
    return;
  }
  // the face of the box: the axis whose slab bound is the hit distance (recomputed exactly
  // as in the loop), on the side the ray enters (or leaves, from inside)
  const FlatBoxT<R>& b = fb[(uint32_t)best - nq];
  const Slab<R> s = flat_slab(b, o, inv, tmin, excl_i, xf);
  const bool enter = s.tn >= tmin;
  int k = 2;
  if (enter) {
    if (s.tn == fmin(s.t0[0], s.t1[0])) k = 0;
    else if (s.tn == fmin(s.t0[1], s.t1[1])) k = 1;
  } else {
    if (s.tf == fmax(s.t0[0], s.t1[0])) k = 0;
    else if (s.tf == fmax(s.t0[1], s.t1[1])) k = 1;
  }
  const R dk = k == 0 ? d.x : (k == 1 ? d.y : d.z);
  const int side = enter ? (dk < R(0) ? 1 : 0) : (dk < R(0) ? 0 : 1);
  e_best = b.face[2 * k + side];
  i_best = b.inst;
  nm = b.mat | (uint32_t)k << 28 | ((b.neg >> (2 * k + side)) & 1u) << 31;
}

// ------------------------------------------------------------------ textures, pdfs
// ---- procedural noise (noise.h), in fp64 for both paths: the sin hashes of worley/voronoi
// pick different cells in fp32, and the reference evaluates all of it in double.
// perlin::noise / perlin_interp (noise.h:22-42, 56-68); tb = rand_offset[256][3], perm_x[256]
__device__ __forceinline__ double perlin_noise(const double* tb, double px, double py, double pz) {
#pragma clang fp contract(off)  // the reference's rounding: the sin hash amplifies any FMA
  int iu = (int)floor(px), iv = (int)floor(py), iw = (int)floor(pz);
  const double u = px - iu, v = py - iv, w = pz - iw;
  iu &= 255;
  iv &= 255;
  iw &= 255;
  const double* perm = tb + 3 * kPerlinPoints;
  const double uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
  double accum = 0.0;
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 2; j++)
      for (int k = 0; k < 2; k++) {
        // perm_x for all three axes, as the reference (noise.h:36)
        const int g = (int)perm[(iu + i) % 256] ^ (int)perm[(iv + j) % 256] ^ (int)perm[(iw + k) % 256];
        const double* r = tb + 3 * g;
        const double d = r[0] * (u - i) + r[1] * (v - j) + r[2] * (w - k);
        accum += (i * uu + (1 - i) * (1 - uu)) * (j * vv + (1 - j) * (1 - vv)) * (k * ww + (1 - k) * (1 - ww)) * d;
      }
  return accum;
}
// perlin_texture::sample (texture.h:84-88) with turb(7, p / scale) (noise.h:44-54)
RT_EXT_FN double perlin_texture(const double* tb, double scale, double px, double py, double pz) {
#pragma clang fp contract(off)  // the reference's rounding: the sin hash amplifies any FMA
  double qx = px / scale, qy = py / scale, qz = pz / scale;
  double accum = 0, weight = 1.0;
  for (int i = 0; i < 7; i++) {
    accum += weight * perlin_noise(tb, qx, qy, qz);
    weight *= 0.5;
    qx *= 2.0;
    qy *= 2.0;
    qz *= 2.0;
  }
  return .5 * (1 + sin(px + 70 * fabs(accum)));
}
// value_noise::noise (noise.h:109-131): trilinear over a float table indexed without wrapping;
// an index outside the table (undefined behaviour in the reference) reads 0
RT_EXT_FN double value_noise(const double* tb, uint32_t n, double px, double py, double pz) {
#pragma clang fp contract(off)  // the reference's rounding: the sin hash amplifies any FMA
  const double fx = floor(px), fy = floor(py), fz = floor(pz);
  const double nn = (double)n, n3 = nn * nn * nn;
  auto at = [&](double ix, double iy, double iz) -> double {
    const double k = ix * nn * nn + iy * nn + iz;
    return (k >= 0 && k < n3) ? (double)(float)tb[(size_t)k] : 0.0;
  };
  const double x000 = at(fx, fy, fz), x100 = at(fx + 1, fy, fz), x010 = at(fx, fy + 1, fz),
               x110 = at(fx + 1, fy + 1, fz), x001 = at(fx, fy, fz + 1), x101 = at(fx + 1, fy, fz + 1),
               x011 = at(fx, fy + 1, fz + 1), x111 = at(fx + 1, fy + 1, fz + 1);
  const double x = px - fx, y = py - fy, z = pz - fz;
  auto lerp = [](double t, double a, double b) { return (1 - t) * a + t * b; };  // utility.h:84
  const double y0z0 = lerp(x, x000, x100), y1z0 = lerp(x, x010, x110), y0z1 = lerp(x, x001, x101),
               y1z1 = lerp(x, x011, x111);
  return lerp(z, lerp(y, y0z0, y1z0), lerp(y, y0z1, y1z1));
}
// worley_noise / voronoi_noise get_rand_offset (noise.h:141-145, 172-176)
__device__ __forceinline__ void cell_hash(double ux, double uy, double uz, double& hx, double& hy, double& hz) {
#pragma clang fp contract(off)  // the reference's rounding: the sin hash amplifies any FMA
  const double ax = ux * 127.1 + uy * 311.7 + uz * 74.7;
  const double ay = ux * 269.5 + uy * 183.3 + uz * 246.1;
  const double az = ux * 113.5 + uy * 271.9 + uz * 307.7;
  // correctly rounded sin (rt_sin.h): the hash is chaotic in sin's last bit
  const double sx = sin_cr(ax) * 43758.5453, sy = sin_cr(ay) * 43758.5453, sz = sin_cr(az) * 43758.5453;
  hx = sx - floor(sx);
  hy = sy - floor(sy);
  hz = sz - floor(sz);
}
// noise.h:147-167 (worley: squared distance to the nearest feature point) and 178-200 (voronoi:
// a hash of the nearest feature point), float distances as in the reference
RT_EXT_FN double cell_noise(bool voronoi, double px, double py, double pz) {
#pragma clang fp contract(off)  // the reference's rounding: the sin hash amplifies any FMA
  const double fx = floor(px), fy = floor(py), fz = floor(pz);
  float min_dist = 3.40282347e+38f, color = 0.0f;
  for (int i = -1; i <= 1; i++)
    for (int j = -1; j <= 1; j++)
      for (int k = -1; k <= 1; k++) {
        const double cx = fx + i, cy = fy + j, cz = fz + k;
        double hx, hy, hz;
        cell_hash(cx, cy, cz, hx, hy, hz);
        const double qx = cx + hx, qy = cy + hy, qz = cz + hz;
        const double dx = qx - px, dy = qy - py, dz = qz - pz;
        const float dist = (float)sqrt(dx * dx + dy * dy + dz * dz);
        if (dist < min_dist) {
          min_dist = dist;
          if (voronoi) {
            double gx, gy, gz;
            cell_hash(qx, qy, qz, gx, gy, gz);
            color = (float)gx;
          }
        }
      }
  return voronoi ? (double)color : (double)(min_dist * min_dist);
}

// EXT: the kernel instantiation for scenes with procedural textures (or non-perspective
// cameras); the base kernels only contain the solid and checker textures.
// sphere::get_sphere_uv (sphere.h:90-95) of a unit vector
template <class R>
RT_EXT_FN void sphere_uv(V<R> n, double& u, double& v) {
  const double theta = acos(-(double)n.y);
  const double phi = atan2(-(double)n.z, (double)n.x) + 3.1415926535897932385;
  u = phi / (2 * 3.1415926535897932385);
  v = theta / 3.1415926535897932385;
}

template <class R, bool EXT>
__device__ __forceinline__ V<R> tex_sample(const DevScene<R>& sc, const Texture<R>& tx, V<R> p, double u = 0,
                                           double v = 0) {  // texture.h
  if (!EXT || tx.kind == T_SOLID || tx.kind == T_CHECKER) {
    if (tx.kind == T_SOLID) return ld3(tx.c0);  // texture.h:15
    V<R> uv = p / tx.scale;                     // texture.h:47-56
    int total = (int)floor(uv.x) + (int)floor(uv.y) + (int)floor(uv.z);
    return (total % 2 == 0) ? ld3(tx.c1) : ld3(tx.c0);
  }
  if (tx.kind == T_IMAGE) {  // picture_texture::sample (texture.h:68-74), image::pixel_data (image.h:71-82)
    const double cs = 1 / 256.0;
    if (tx.n == 0 || tx.h == 0) return mkv(R(255 * cs), R(0), R(255 * cs));  // no image: magenta
    int i = (int)(tx.n * u), j = (int)(tx.h * (1 - v));
    i = i < 0 ? 0 : (i < (int)tx.n ? i : (int)tx.n - 1);  // clamp to [0, width)
    j = j < 0 ? 0 : (j < (int)tx.h ? j : (int)tx.h - 1);
    const uint8_t* px = sc.images + tx.data + 3 * ((size_t)j * tx.n + (size_t)i);
    return mkv(R(px[0] * cs), R(px[1] * cs), R(px[2] * cs));
  }
  double g;
  if (tx.kind == T_PERLIN)
    g = perlin_texture(sc.texdata + tx.data, (double)tx.scale, p.x, p.y, p.z);
  else if (tx.kind == T_VALUE)
    g = value_noise(sc.texdata + tx.data, tx.n, p.x, p.y, p.z);
  else
    g = cell_noise(tx.kind == T_VORONOI, p.x, p.y, p.z);
  return mkv(R(g), R(g), R(g));  // color(noise) (texture.h:99, 107, 115)
}

template <class R>
struct Onb {  // onb.h:18-29
  V<R> x, y, z;
};
template <class R>
__device__ __forceinline__ Onb<R> make_onb(V<R> n) {
  Onb<R> b;
  b.y = unit(n);
  if constexpr (sizeof(R) == 4) {
    // cross(y, a) for a = e_z or e_x has an exact zero component: (y.y, -y.x, 0) or (0, y.z, -y.y)
    const bool ez = fabsf(b.y.x) > 0.9f;
    const float c0 = ez ? b.y.y : 0.f, c1 = ez ? -b.y.x : b.y.z, c2 = ez ? 0.f : -b.y.y;
    const float r = frsq(ez ? c0 * c0 + c1 * c1 : c1 * c1 + c2 * c2);
    b.z = mkv(c0 * r, c1 * r, c2 * r);
  } else {
    V<R> a = (fabs(b.y.x) > R(0.9)) ? mkv(R(0), R(0), R(1)) : mkv(R(1), R(0), R(0));
    b.z = unit(cross(b.y, a));
  }
  b.x = cross(b.y, b.z);
  return b;
}
// The onb of an axis-aligned normal n = +-e_A (every hit of the flat program): unit(n) = n and the
// cross product before the second normalisation has length exactly 1, so this is make_onb without
// its two normalisations -- bit-identical (the refined rsqrt of 1 is 1, and v * 1 = v), cheaper.
template <class R>
__device__ __forceinline__ Onb<R> make_onb_axis(V<R> n) {
  Onb<R> b;
  b.y = n;
  if constexpr (sizeof(R) == 4) {
    const bool ez = fabsf(b.y.x) > 0.9f;
    b.z = mkv(ez ? b.y.y : 0.f, ez ? -b.y.x : b.y.z, ez ? 0.f : -b.y.y);
  } else {
    const V<R> a = (fabs(b.y.x) > R(0.9)) ? mkv(R(0), R(0), R(1)) : mkv(R(1), R(0), R(0));
    b.z = cross(b.y, a);
  }
  b.x = cross(b.y, b.z);
  return b;
}
template <class R>
__device__ __forceinline__ V<R> onb_transform(const Onb<R>& b, V<R> v) {  // onb.h:6
  V<R> r = mkv(R(0), R(0), R(0));
  r = r + v.x * b.x;
  r = r + v.y * b.y;
  r = r + v.z * b.z;
  return r;
}
// random_in_unit_sphere (utility.h:30-42): a point ON the unit sphere
// (the _sc forms take sin/cos(2 pi u) computed by the caller: shade's NL form computes one for every lane)
template <class R>
__device__ __forceinline__ V<R> on_sphere_sc(R u1, R sp, R cp) {
  R cos_theta = R(1) - R(2) * u1;
  R sin_theta = fsqrt01(R(1) - cos_theta * cos_theta);
  return mkv(sin_theta * cp, cos_theta, sin_theta * sp);
}
template <class R>
__device__ __forceinline__ V<R> on_sphere(R u1, R u2) {
  R sp, cp;
  sincos2pi(u2, sp, cp);
  return on_sphere_sc(u1, sp, cp);
}
// random_cosine_direction (utility.h:61-69)
template <class R>
__device__ __forceinline__ V<R> cosine_dir_sc(R r2, R sp, R cp) {
  R sr2 = fsqrt01(r2);
  return mkv(cp * sr2, fsqrt01(R(1) - r2), sp * sr2);
}
template <class R>
__device__ __forceinline__ V<R> cosine_dir(R r1, R r2) {
  R sp, cp;
  sincos2pi(r1, sp, cp);
  return cosine_dir_sc(r2, sp, cp);
}

// hittable_pdf over the light (hittable_list.h:39-50 -> quad.h:66-78 / sphere.h:76-81 / hittable.h:39-41)
// `sampled`: dir came from light_random, i.e. dir = (a point on the light) - o. Then it hits the
// light at t = 1 by construction, and fp32 uses that instead of re-testing: a point sampled on
// the light's edge (u1 or u2 ~ 0) can round to just outside it, giving pdf 0 for a direction
// the light itself produced (and 0/0 = NaN when the material pdf is 0 too).
// The light is read where it is used, field group by field group (ld_here), so no light data
// stays live across the path loop (it would be spilled to VGPR lanes).
template <class R>
struct R4s {
  R v[4];
};
template <class R>
struct LightUV {  // Light::u, pad1, v, pad2
  R u[3], pad1, v[3], pad2;
};
template <class R>
struct LightAF {  // Light::af
  R f[8];
};
// quad::pdf_value of an axis-aligned light in fp64 (round 4): one refined reciprocal of d_A serves the hit
// distance t = (q_A - o_A) / d_A and the cosine |d_A| / |d|, so distance_squared / (cosine * area) =
// t^2 (d.d) |d| |1/d_A| / area, |d| = (d.d) rsqrt(d.d) (the rsqrt unit(dir) computes too), 1/area stored
// (af[7]): one reciprocal instead of two refined divisions and no dot product with the normal (+-e_A).
// Within a few ulp of the reference's expression; the hit test is aquad_t's.
template <int A, int U, int W>
__device__ __forceinline__ double light_pdf_aligned(const double* f, V<double> o, V<double> d) {
  const double rA = frcp(comp<A>(d));
  const double th = (f[0] - comp<A>(o)) * rA;
  // (round 6: the same test without branches -- a and b by the bit order, as the flat program's quads -- measured
  // neutral: C2 fp64 25.36 / 25.36 ms/frame, C5 fp64 2,077 / 2,071, r06k)
  if (!(0.001 <= th)) return 0.0;  // interval(0.001, inf) (quad.h:70); th = +inf fails the alpha test
  const double a = ((comp<U>(o) + th * comp<U>(d)) - f[1]) * f[3];
  const double b = ((comp<W>(o) + th * comp<W>(d)) - f[2]) * f[4];
  if (!(0.0 <= a && a <= 1.0 && 0.0 <= b && b <= 1.0)) return 0.0;
  const double dd = d.x * d.x + d.y * d.y + d.z * d.z;
  return ((th * th) * dd) * (dd * frsq_nz(dd)) * fabs(rA) * f[7];
}
// SEL: the fp32 sampled directions (dir from light_random) by select, not a branch (RT_MIX_SELECT)
template <class R, bool SEL = false>
__device__ __forceinline__ R light_pdf(const Light<R>* Lp, V<R> o, V<R> dir, bool sampled = false) {
  const int32_t kind = ld_here(&Lp->kind);
  if (kind == L_QUAD) {
    R t;
    bool hit;
    const int32_t aligned = ld_here(&Lp->aligned);
    if constexpr (sizeof(R) == 8) {
      if (aligned) {  // uniform branch
        const LightAF<R> af = ld_here(reinterpret_cast<const LightAF<R>*>(Lp->af));
        switch (aligned) {
          case 1: return light_pdf_aligned<2, 0, 1>(af.f, o, dir);
          case 2: return light_pdf_aligned<1, 0, 2>(af.f, o, dir);
          case 3: return light_pdf_aligned<2, 1, 0>(af.f, o, dir);
          case 4: return light_pdf_aligned<0, 1, 2>(af.f, o, dir);
          case 5: return light_pdf_aligned<1, 2, 0>(af.f, o, dir);
          default: return light_pdf_aligned<0, 2, 1>(af.f, o, dir);
        }
      }
    }
    if (sizeof(R) == 4 && sampled && !(SEL && aligned)) {
      t = R(1);
      hit = true;
    } else if (aligned) {  // uniform branch
      const LightAF<R> af = ld_here(reinterpret_cast<const LightAF<R>*>(Lp->af));
      const V<R> inv = rcp3(dir);
      switch (aligned) {
        case 1: hit = aquad_t<2, 0, 1>(af.f, o, dir, inv, R(0.001), Num<R>::inf(), t); break;
        case 2: hit = aquad_t<1, 0, 2>(af.f, o, dir, inv, R(0.001), Num<R>::inf(), t); break;
        case 3: hit = aquad_t<2, 1, 0>(af.f, o, dir, inv, R(0.001), Num<R>::inf(), t); break;
        case 4: hit = aquad_t<0, 1, 2>(af.f, o, dir, inv, R(0.001), Num<R>::inf(), t); break;
        case 5: hit = aquad_t<1, 2, 0>(af.f, o, dir, inv, R(0.001), Num<R>::inf(), t); break;
        default: hit = aquad_t<0, 2, 1>(af.f, o, dir, inv, R(0.001), Num<R>::inf(), t); break;
      }
      if constexpr (sizeof(R) == 4 && SEL) {  // the sampled directions by select, not a branch
        t = sampled ? R(1) : t;
        hit = hit | sampled;
        const Quad<R> q = ld_here(&Lp->quad);
        const R pdf = fdiv(t * t * dot(dir, dir), fabs(dot(unit(dir), ld3(q.n))) * q.area);
        return hit ? pdf : R(0);
      }
    } else {
      hit = quad_t(ld_here(&Lp->quad), o, dir, R(0.001), Num<R>::inf(), t);
    }
    if (!hit) return R(0);
    const Quad<R> q = ld_here(&Lp->quad);
    R dist2 = t * t * dot(dir, dir);
    R cosine = fabs(dot(unit(dir), ld3(q.n)));
    return fdiv(dist2, cosine * q.area);
  }
  if (kind == L_SPHERE) {
    const R4s<R> c = ld_here(reinterpret_cast<const R4s<R>*>(Lp->center));  // center[3], radius
    V<R> f = o - mkv(c.v[0], c.v[1], c.v[2]);
    return fdiv(c.v[3] * c.v[3] * Num<R>::pi(), dot(f, f));
  }
  return R(0);
}
template <class R>
__device__ __forceinline__ V<R> light_random(const Light<R>* Lp, V<R> o, R u1, R u2) {
  const int32_t kind = ld_here(&Lp->kind);
  if (kind == L_QUAD) {
    const Quad<R> q = ld_here(&Lp->quad);
    const LightUV<R> uv = ld_here(reinterpret_cast<const LightUV<R>*>(Lp->u));
    V<R> p = (ld3(q.q) + u1 * ld3(uv.u)) + u2 * ld3(uv.v);
    return p - o;
  }
  if (kind == L_SPHERE) return on_sphere(u1, u2) * ld_here(&Lp->radius);
  return mkv(R(1), R(0), R(0));
}

}  // namespace rtd
