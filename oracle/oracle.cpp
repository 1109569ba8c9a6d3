// oracle.cpp -- fp64 CPU restatement of the reference render path.
// TEST INFRASTRUCTURE ONLY (see oracle.h). Built with g++ -O2 -ffp-contract=off,
// no -ffast-math, no FMA: every double operation is evaluated in the order the
// reference source writes it, so the glibc-compat mode reproduces the
// reference bit for bit (pinned by tests/test_oracle_pins.py).
//
// Each routine cites the reference file:line it restates.

#include "oracle.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace orc {

const double kInf = std::numeric_limits<double>::infinity();
const double kPi = 3.1415926535897932385;  // utility.h:15

// ---------------------------------------------------------------- vectors (vec3.h)
struct v3 {
  double x = 0, y = 0, z = 0;
  v3() = default;
  v3(double a, double b, double c) : x(a), y(b), z(c) {}
  double operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
  double& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
inline v3 operator+(const v3& a, const v3& b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline v3 operator-(const v3& a, const v3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline v3 operator-(const v3& a) { return {-a.x, -a.y, -a.z}; }
inline v3 operator*(const v3& a, const v3& b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline v3 operator*(double c, const v3& a) { return {a.x * c, a.y * c, a.z * c}; }
inline v3 operator*(const v3& a, double c) { return {a.x * c, a.y * c, a.z * c}; }
inline v3 operator/(const v3& a, double c) { return {a.x / c, a.y / c, a.z / c}; }
inline double dot(const v3& a, const v3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // vec3.h:61
inline v3 cross(const v3& a, const v3& b) {                                              // vec3.h:79-82
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline double len2(const v3& a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
inline double len(const v3& a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
inline v3 unit(const v3& a) { return a / len(a); }  // vec3.h:77
inline v3 v3_from(const double* p) { return {p[0], p[1], p[2]}; }

// reflect / refract (utility.h:70-76)
inline v3 reflect(const v3& v, const v3& n) { return v - 2 * dot(v, n) * n; }
inline v3 refract(const v3& v, const v3& n, double eta) {
  double cos_theta = std::fmin(dot(-v, n), 1.0);
  v3 perp = eta * (v + cos_theta * n);
  v3 par = -std::sqrt(std::fabs(1.0 - len2(perp))) * n;
  return perp + par;
}

// ---------------------------------------------------------------- RNG
inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x21f0aaadu;
  x ^= x >> 15;
  x *= 0xd35a2d97u;
  x ^= x >> 15;
  return x;
}
inline uint32_t key_pixel(uint64_t seed, uint32_t pixel) {
  return mix32(pixel ^ mix32((uint32_t)seed ^ 0x9E3779B9u));
}
inline uint32_t key_sample(uint64_t seed, uint32_t sample) {
  return mix32(sample + mix32((uint32_t)(seed >> 32) + 0x7F4A7C15u));
}
// the key of one camera sample (pixel, sample); a draw is one more mix of key + dim * phi
inline uint32_t key_path(uint32_t ka, uint32_t kb) { return mix32(ka ^ kb); }
inline uint32_t draw_u32(uint32_t ks, uint32_t dim) { return mix32(ks + dim * 0x9E3779B9u); }
inline double to_unit(uint32_t x) { return (double)(x >> 8) * (1.0 / 16777216.0); }

// Draw-dimension layout per camera sample (counter mode):
//   0, 1, 2      camera offset x, offset y, ray time           (camera.h:248-250)
//   3 + 16*b + j bounce b: j in [0,12) volume distance draws    (volumne.h:36)
//                          j in [12,16) scatter / pdf draws      (material.h, pdf.h)
enum { kDimsCamera = 3, kDimsPerBounce = 16, kVolumeSlots = 12 };

struct rngctx {
  int mode = ORC_RNG_COUNTER;
  uint32_t ks = 0;  // key_path(key_pixel, key_sample)
  uint32_t bounce = 0, jv = 0, js = 0;
  double glibc() const { return std::rand() / (RAND_MAX + 1.0); }  // utility.h:20
  double at(uint32_t dim) const { return to_unit(draw_u32(ks, dim)); }
  double camera(int k) const { return mode == ORC_RNG_COMPAT ? glibc() : at((uint32_t)k); }
  double volume() {
    if (mode == ORC_RNG_COMPAT) return glibc();
    uint32_t j = jv++;
    if (j >= (uint32_t)kVolumeSlots) j = kVolumeSlots - 1;  // device clamps the same way
    return at(kDimsCamera + kDimsPerBounce * bounce + j);
  }
  double scatter() {
    if (mode == ORC_RNG_COMPAT) return glibc();
    uint32_t j = js++;
    if (j >= (uint32_t)(kDimsPerBounce - kVolumeSlots)) j = kDimsPerBounce - kVolumeSlots - 1;
    return at(kDimsCamera + kDimsPerBounce * bounce + kVolumeSlots + j);
  }
  void next_bounce(uint32_t b) {
    bounce = b;
    jv = js = 0;
  }
};

// random_in_unit_sphere / random_unit_vec / random_cosine_direction (utility.h:30-69)
inline v3 random_on_sphere(rngctx& g) {
  double u1 = g.scatter();
  double u2 = g.scatter();
  double cos_theta = 1 - 2 * u1;
  double sin_theta = std::sqrt(1 - cos_theta * cos_theta);
  double phi = 2 * kPi * u2;
  return {sin_theta * std::cos(phi), cos_theta, sin_theta * std::sin(phi)};
}
inline v3 random_unit_vec(rngctx& g) { return unit(random_on_sphere(g)); }
inline v3 random_cosine_direction(rngctx& g) {
  double r1 = g.scatter();
  double r2 = g.scatter();
  double phi = 2 * kPi * r1;
  double x = std::cos(phi) * std::sqrt(r2);
  double y = std::sqrt(1 - r2);
  double z = std::sin(phi) * std::sqrt(r2);
  return {x, y, z};
}

// ---------------------------------------------------------------- ray, interval, aabb
struct ray3 {
  v3 o, d;
  double tm = 0;
  v3 at(double t) const { return o + t * d; }  // ray.h:11
};

struct ivl {  // interval.h
  double lo = kInf, hi = -kInf;
  ivl() = default;
  ivl(double a, double b) : lo(a), hi(b) {}
  bool contains(double x) const { return lo <= x && x <= hi; }
  ivl expand(double delta) const {
    double pad = delta / 2;
    return {lo - pad, hi + pad};
  }
  static ivl enclose(const ivl& a, const ivl& b) {
    return {a.lo < b.lo ? a.lo : b.lo, a.hi > b.hi ? a.hi : b.hi};
  }
};

template <class T>
inline const T& smin(const T& a, const T& b) { return (b < a) ? b : a; }  // std::min
template <class T>
inline const T& smax(const T& a, const T& b) { return (a < b) ? b : a; }  // std::max

struct box3 {  // aabb.h
  ivl ax[3];
  box3() = default;
  static box3 padded(const ivl& x, const ivl& y, const ivl& z) {  // aabb.h:7-12,81-86
    box3 b;
    b.ax[0] = x;
    b.ax[1] = y;
    b.ax[2] = z;
    for (auto& i : b.ax)
      if (i.hi - i.lo < 0.0001) i = i.expand(0.0001);
    return b;
  }
  static box3 points(const v3& a, const v3& c) {  // aabb.h:15-19
    box3 b;
    for (int k = 0; k < 3; k++) b.ax[k] = (a[k] <= c[k]) ? ivl(a[k], c[k]) : ivl(c[k], a[k]);
    return b;
  }
  static box3 enclose(const box3& a, const box3& b) {
    return padded(ivl::enclose(a.ax[0], b.ax[0]), ivl::enclose(a.ax[1], b.ax[1]), ivl::enclose(a.ax[2], b.ax[2]));
  }
  box3 offset(const v3& o) const {
    return padded({ax[0].lo + o.x, ax[0].hi + o.x}, {ax[1].lo + o.y, ax[1].hi + o.y}, {ax[2].lo + o.z, ax[2].hi + o.z});
  }
  bool hit(const ray3& r, ivl t) const {  // aabb.h:28-33,45-69
    ivl s[3];
    for (int k = 0; k < 3; k++) {
      double t1 = (ax[k].lo - r.o[k]) / r.d[k];
      double t2 = (ax[k].hi - r.o[k]) / r.d[k];
      s[k] = ivl(smin(t1, t2), smax(t1, t2));
    }
    double tmin = smax(smax(s[0].lo, s[1].lo), s[2].lo);
    double tmax = smin(smin(s[0].hi, s[1].hi), s[2].hi);
    if (tmin > t.lo) t.lo = tmin;
    if (tmax < t.hi) t.hi = tmax;
    return t.lo < t.hi;
  }
};

// ---------------------------------------------------------------- textures (texture.h)
// noise.h:10-201 restated. perlin keeps the tables its constructor drew (rand_offset, perm_x;
// perm_y/perm_z are drawn but never read: noise.h:36 indexes perm_x for all three axes).
struct onoise {
  std::vector<v3> rand_offset;   // perlin (256) -- noise.h:76-80
  std::vector<int> perm_x;       // perlin
  std::vector<float> values;     // value noise, resolution^3 (noise.h:134-136)
  int resolution = 0;
  double perlin(const v3& p) const {  // noise.h:56-68, 22-42
    int iu = int(std::floor(p.x)), iv = int(std::floor(p.y)), iw = int(std::floor(p.z));
    double u = p.x - iu, v = p.y - iv, w = p.z - iw;
    iu = iu & 255;
    iv = iv & 255;
    iw = iw & 255;
    double uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
    double accum = 0.0;
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 2; j++)
        for (int k = 0; k < 2; k++) {
          v3 weight(u - i, v - j, w - k);
          const v3& g = rand_offset[perm_x[(iu + i) % 256] ^ perm_x[(iv + j) % 256] ^ perm_x[(iw + k) % 256]];
          accum += (i * uu + (1 - i) * (1 - uu)) * (j * vv + (1 - j) * (1 - vv)) * (k * ww + (1 - k) * (1 - ww)) *
                   dot(g, weight);
        }
    return accum;
  }
  double turb(int depth, const v3& p) const {  // noise.h:44-54
    double accum = 0;
    v3 q = p;
    double weight = 1.0;
    for (int i = 0; i < depth; i++) {
      accum += weight * perlin(q);
      weight *= 0.5;
      q = q * 2.0;
    }
    return std::fabs(accum);
  }
  double value(const v3& p) const {  // noise.h:109-131; an index outside the table reads 0
    double fx = std::floor(p.x), fy = std::floor(p.y), fz = std::floor(p.z);
    double n = resolution, n3 = n * n * n;
    auto at = [&](double x, double y, double z) -> float {
      double k = x * n * n + y * n + z;
      return (k >= 0 && k < n3) ? values[(size_t)k] : 0.0f;
    };
    float x000 = at(fx, fy, fz), x100 = at(fx + 1, fy, fz), x010 = at(fx, fy + 1, fz), x110 = at(fx + 1, fy + 1, fz);
    float x001 = at(fx, fy, fz + 1), x101 = at(fx + 1, fy, fz + 1), x011 = at(fx, fy + 1, fz + 1),
          x111 = at(fx + 1, fy + 1, fz + 1);
    double x = p.x - fx, y = p.y - fy, z = p.z - fz;
    auto lerp = [](double t, double a, double b) { return (1 - t) * a + t * b; };  // utility.h:84
    double y0z0 = lerp(x, x000, x100), y1z0 = lerp(x, x010, x110), y0z1 = lerp(x, x001, x101),
           y1z1 = lerp(x, x011, x111);
    return lerp(z, lerp(y, y0z0, y1z0), lerp(y, y0z1, y1z1));
  }
  static v3 hash(const v3& u) {  // noise.h:141-145
    v3 r(dot(u, v3(127.1, 311.7, 74.7)), dot(u, v3(269.5, 183.3, 246.1)), dot(u, v3(113.5, 271.9, 307.7)));
    v3 q = v3(std::sin(r.x), std::sin(r.y), std::sin(r.z)) * 43758.5453;
    return q - v3(std::floor(q.x), std::floor(q.y), std::floor(q.z));  // fract (vec3.h:87)
  }
  static double cells(const v3& p, bool voronoi) {  // noise.h:147-167, 178-200
    v3 f(std::floor(p.x), std::floor(p.y), std::floor(p.z));
    float min_dist = std::numeric_limits<float>::max(), color = 0.0f;
    for (int i = -1; i <= 1; i++)
      for (int j = -1; j <= 1; j++)
        for (int k = -1; k <= 1; k++) {
          v3 cell = f + v3(i, j, k);
          v3 pos = cell + hash(cell);
          float dist = (float)len(pos - p);
          if (dist < min_dist) {
            min_dist = dist;
            if (voronoi) color = (float)hash(pos).x;
          }
        }
    return voronoi ? color : min_dist * min_dist;
  }
};

struct otex {
  int kind = RT_TEX_SOLID;
  v3 color, odd, even;
  double scale = 1;
  onoise noise;
  int width = 0, height = 0;   // image
  std::vector<uint8_t> pixels;  // image, RGB rows from the top (image.h bdata)
  v3 sample(double u, double v, const v3& p) const {
    switch (kind) {
      case RT_TEX_IMAGE: {  // picture_texture::sample (texture.h:68-74), image::pixel_data (image.h:71-82)
        double cs = 1 / 256.0;
        if (width == 0 || height == 0) return v3(255 * cs, 0, 255 * cs);  // magenta: no image data
        int i = width * u;
        int j = height * (1 - v);
        i = i < 0 ? 0 : (i < width ? i : width - 1);
        j = j < 0 ? 0 : (j < height ? j : height - 1);
        const uint8_t* px = pixels.data() + 3 * ((size_t)j * width + i);
        return v3(px[0] * cs, px[1] * cs, px[2] * cs);
      }
      case RT_TEX_SOLID: return color;
      case RT_TEX_CHECKER: {
        v3 uv = p / scale;  // texture.h:48-55
        int ix = (int)std::floor(uv.x);
        int iy = (int)std::floor(uv.y);
        int iz = (int)std::floor(uv.z);
        int total = ix + iy + iz;
        return (total % 2 == 0) ? even : odd;
      }
      case RT_TEX_PERLIN: {  // texture.h:84-88
        double g = .5 * (1 + std::sin((p.x + 70 * noise.turb(7, p / scale))));
        return {g, g, g};
      }
      case RT_TEX_VALUE: {
        double g = noise.value(p);
        return {g, g, g};
      }
      default: {
        double g = onoise::cells(p, kind == RT_TEX_VORONOI);
        return {g, g, g};
      }
    }
  }
};

// ---------------------------------------------------------------- hit record (hittable.h:7-30)
// development aid: orc_set_trace(1) prints every segment of single-threaded renders to stderr
static int g_trace = 0;

struct omat;
struct hrec {
  v3 p, n;
  double t = 0, u = 0, v = 0;
  bool front = false;
  const omat* mat = nullptr;
  void set_face_normal(const ray3& r, const v3& outward) {
    front = dot(r.d, outward) < 0.0;
    n = front ? outward : -outward;
  }
};

// ---------------------------------------------------------------- materials (material.h)
enum class smode { random, determined };
struct pdfsel {  // which pdf a kRandom scatter returned
  enum { cosine, sphere } kind = cosine;
  v3 onb_x, onb_y, onb_z;  // onb.h:18-29 (cosine only)
};
struct srec {
  smode mode = smode::random;
  v3 att;
  ray3 scattered;
  pdfsel pdf;
};

inline void make_onb(const v3& n, v3& x, v3& y, v3& z) {  // onb.h:20-28
  y = unit(n);
  v3 a = (std::fabs(y.x) > 0.9) ? v3(0, 0, 1) : v3(1, 0, 0);
  z = unit(cross(y, a));
  x = cross(y, z);
}
inline v3 onb_transform(const v3& x, const v3& y, const v3& z, const v3& v) {  // onb.h:6
  v3 r(0, 0, 0);
  r = r + v.x * x;
  r = r + v.y * y;
  r = r + v.z * z;
  return r;
}

struct omat {
  int kind = RT_MAT_LAMBERTIAN;
  const otex* tex = nullptr;
  float fuzz = 0, refr = 1, smooth = 0, spec = 0;

  static double reflectance(double cosine, double ri) {  // material.h:135-139
    double r0 = (1 - ri) / (1 + ri);
    r0 = r0 * r0;
    return r0 + (1 - r0) * std::pow((1 - cosine), 5);
  }

  bool scatter(const ray3& rin, const hrec& h, srec& s, rngctx& g) const {
    switch (kind) {
      case RT_MAT_LAMBERTIAN:  // material.h:62-67
        s.mode = smode::random;
        s.att = tex->sample(h.u, h.v, h.p);
        s.pdf.kind = pdfsel::cosine;
        make_onb(h.n, s.pdf.onb_x, s.pdf.onb_y, s.pdf.onb_z);
        return true;
      case RT_MAT_METAL: {  // material.h:85-92
        v3 dir = unit(reflect(rin.d, h.n));
        dir = dir + (double)fuzz * random_unit_vec(g);
        s.mode = smode::determined;
        s.scattered = {h.p, dir, rin.tm};
        s.att = tex->sample(h.u, h.v, h.p);
        return true;
      }
      case RT_MAT_DIELECTRIC: {  // material.h:113-131
        s.mode = smode::determined;
        s.att = tex->sample(h.u, h.v, h.p);
        double ri = h.front ? (1.0 / refr) : (double)refr;
        v3 ud = unit(rin.d);
        double cos_theta = std::fmin(dot(-ud, h.n), 1.0);
        double sin_theta = std::sqrt(1.0 - cos_theta * cos_theta);
        bool cant = ri * sin_theta > 1.0;
        if (cant || reflectance(cos_theta, ri) > g.scatter())
          s.scattered = {h.p, reflect(ud, h.n), rin.tm};
        else
          s.scattered = {h.p, refract(ud, h.n, ri), rin.tm};
        return true;
      }
      case RT_MAT_GLOSS: {  // material.h:158-174
        v3 spec_dir = reflect(rin.d, h.n);
        bool specular = g.scatter() <= (double)spec;
        if (specular) {
          v3 x, y, z;
          make_onb(h.n, x, y, z);
          v3 diffuse = onb_transform(x, y, z, random_cosine_direction(g));
          double t = smooth;
          v3 dir = unit((1 - t) * diffuse + t * spec_dir);
          s.mode = smode::determined;
          s.att = v3(1.0, 1.0, 1.0);
          s.scattered = {h.p, dir, rin.tm};
        } else {
          s.mode = smode::random;
          s.att = tex->sample(h.u, h.v, h.p);
          s.pdf.kind = pdfsel::cosine;
          make_onb(h.n, s.pdf.onb_x, s.pdf.onb_y, s.pdf.onb_z);
        }
        return true;
      }
      case RT_MAT_ISOTROPIC:  // material.h:193-198
        s.mode = smode::random;
        s.att = tex->sample(h.u, h.v, h.p);
        s.pdf.kind = pdfsel::sphere;
        return true;
      default:
        return false;  // diffuse_light and the base class do not scatter
    }
  }
  double p_scattered(const hrec& h, const ray3& sc) const {
    if (kind == RT_MAT_LAMBERTIAN || kind == RT_MAT_GLOSS) {  // material.h:69-72, 176-179
      double c = dot(h.n, unit(sc.d));
      return c < 0 ? 0 : c / kPi;
    }
    if (kind == RT_MAT_ISOTROPIC) return 1 / (4 * kPi);  // material.h:200
    return 0;
  }
  v3 emitted(const hrec& h) const {  // material.h:211-215
    if (kind != RT_MAT_DIFFUSE_LIGHT) return {};
    if (!h.front) return {0, 0, 0};
    return tex->sample(h.u, h.v, h.p);
  }
};

// pdf value / generate for the material's own pdf (pdf.h:15-45)
inline double pdf_value(const pdfsel& p, const v3& dir) {
  if (p.kind == pdfsel::sphere) return 1 / (4 * kPi);
  double c = dot(unit(dir), p.onb_y);
  return std::fmax(0, c / kPi);
}
inline v3 pdf_generate(const pdfsel& p, rngctx& g) {
  if (p.kind == pdfsel::sphere) return random_unit_vec(g);
  return onb_transform(p.onb_x, p.onb_y, p.onb_z, random_cosine_direction(g));
}

// ---------------------------------------------------------------- hittables
struct ohit {
  virtual ~ohit() = default;
  virtual bool hit(const ray3& r, ivl t, hrec& rec, rngctx& g) const = 0;
  virtual box3 bbox() const = 0;
  virtual double pdf_value(const v3&, const v3&, rngctx&) const { return 0.0; }  // hittable.h:39
  virtual v3 random(const v3&, rngctx&) const { return {1, 0, 0}; }             // hittable.h:41
  virtual bool is_quad() const { return false; }
};

struct osphere : ohit {  // sphere.h
  v3 center, c1, c2;  // `center` stays (0,0,0) for the moving constructor (sphere.h:25-35)
  double radius = 0;
  bool moving = false;
  const omat* mat = nullptr;
  box3 box;
  static osphere* make_static(const v3& c, double r, const omat* m) {
    auto* s = new osphere;
    s->center = c;
    s->radius = std::fmax(0, r);
    s->mat = m;
    v3 rv(r, r, r);
    s->box = box3::points(c - rv, c + rv);
    return s;
  }
  static osphere* make_moving(const v3& a, const v3& b, double r, const omat* m) {
    auto* s = new osphere;
    s->c1 = a;
    s->c2 = b;
    s->radius = std::fmax(0, r);
    s->moving = true;
    s->mat = m;
    v3 rv(s->radius, s->radius, s->radius);
    s->box = box3::enclose(box3::points(a - rv, a + rv), box3::points(b - rv, b + rv));
    return s;
  }
  static void sphere_uv(const v3& p, double& u, double& v) {  // sphere.h:90-95
    double theta = std::acos(-p.y);
    double phi = std::atan2(-p.z, p.x) + kPi;
    u = phi / (2 * kPi);
    v = theta / kPi;
  }
  bool hit(const ray3& r, ivl t, hrec& rec, rngctx&) const override {  // sphere.h:40-74
    v3 c = moving ? c1 + r.tm * (c2 - c1) : center;
    double a = dot(r.d, r.d);
    double b = 2.0 * dot(r.d, (r.o - c));
    double cc = dot(r.o - c, r.o - c) - radius * radius;
    double disc = b * b - 4 * a * cc;
    if (disc < 0) return false;
    double sq = std::sqrt(disc);
    double root = (-b - sq) / (2.0 * a);
    if (!t.contains(root)) {
      root = (-b + sq) / (2.0 * a);
      if (!t.contains(root)) return false;
    }
    rec.t = root;
    rec.p = r.at(root);
    v3 outward = (rec.p - center) / radius;
    sphere_uv(outward, rec.u, rec.v);
    rec.set_face_normal(r, outward);
    rec.mat = mat;
    return true;
  }
  box3 bbox() const override { return box; }
  double pdf_value(const v3& o, const v3&, rngctx&) const override {  // sphere.h:76-78
    return radius * radius * kPi / len2(o - center);
  }
  v3 random(const v3&, rngctx& g) const override { return random_on_sphere(g) * radius; }  // sphere.h:81
};

struct oquad : ohit {  // quad.h
  v3 q, u, v, unorm;
  double area = 0;
  const omat* mat = nullptr;
  box3 box;
  oquad(const v3& q_, const v3& u_, const v3& v_, const omat* m) : q(q_), u(u_), v(v_), mat(m) {
    v3 n = cross(u, v);
    unorm = unit(n);
    area = len(n);
    box = box3::enclose(box3::points(q, q + u + v), box3::points(q + u, q + v));
  }
  bool is_quad() const override { return true; }
  bool hit(const ray3& r, ivl t, hrec& rec, rngctx&) const override {  // quad.h:30-52
    double d = dot(unorm, q);
    double th = (d - dot(unorm, r.o)) / dot(unorm, r.d);
    if (!t.contains(th)) return false;
    v3 hp = r.at(th);
    v3 p = hp - q;
    v3 n = cross(u, v);
    v3 w = n / dot(n, n);
    double a = dot(w, cross(p, v));
    double b = dot(w, cross(u, p));
    ivl unit_ivl(0, 1);  // quad.h:58-64
    if (!unit_ivl.contains(a) || !unit_ivl.contains(b)) return false;
    rec.u = a;
    rec.v = b;
    rec.t = th;
    rec.p = hp;
    rec.mat = mat;
    rec.set_face_normal(r, unorm);
    return true;
  }
  box3 bbox() const override { return box; }
  double pdf_value(const v3& o, const v3& dir, rngctx& g) const override {  // quad.h:66-73
    hrec rec;
    ray3 r{o, dir, 0};
    if (!hit(r, ivl(0.001, kInf), rec, g)) return 0;
    double dist2 = rec.t * rec.t * len2(dir);
    double cosine = std::fabs(dot(unit(dir), rec.n));
    return dist2 / (cosine * area);
  }
  v3 random(const v3& o, rngctx& g) const override {  // quad.h:75-78
    double ru, rv;
    if (g.mode == ORC_RNG_COMPAT) {
      rv = g.scatter();  // GCC evaluates the right operand of the outer + first
      ru = g.scatter();
    } else {
      ru = g.scatter();
      rv = g.scatter();
    }
    v3 p = q + (ru * u) + (rv * v);
    return p - o;
  }
};

struct otri : ohit {  // triangle.h
  v3 p0, p1, p2, normal;
  const omat* mat = nullptr;
  otri(const v3& a, const v3& b, const v3& c, const omat* m) : p0(a), p1(b), p2(c), mat(m) {
    normal = unit(cross(p1 - p0, p2 - p0));
  }
  bool hit(const ray3& r, ivl t, hrec& rec, rngctx&) const override {  // triangle.h:8-15,27-40
    v3 e1 = p1 - p0, e2 = p2 - p0, s = r.o - p0;
    v3 s1 = cross(r.d, e2), s2 = cross(s, e1);
    double den = dot(s1, e1);
    double th = dot(s2, e2) / den, b0 = dot(s1, s) / den, b1 = dot(s2, r.d) / den;
    if (th < t.lo || th > t.hi) return false;
    if (b0 < 0 || b1 < 0 || b0 + b1 > 1) return false;
    rec.t = th;
    rec.p = r.at(th);
    rec.u = rec.v = 0;  // the reference leaves u, v stale (triangle.h:27-40); the device uses 0 too
    rec.set_face_normal(r, normal);
    rec.mat = mat;
    return true;
  }
  box3 bbox() const override {  // triangle.h:42-48
    v3 mn(std::fmin(p0.x, std::fmin(p1.x, p2.x)), std::fmin(p0.y, std::fmin(p1.y, p2.y)),
          std::fmin(p0.z, std::fmin(p1.z, p2.z)));
    v3 mx(std::fmax(p0.x, std::fmax(p1.x, p2.x)), std::fmax(p0.y, std::fmax(p1.y, p2.y)),
          std::fmax(p0.z, std::fmax(p1.z, p2.z)));
    return box3::points(mn, mx);
  }
};

struct olist : ohit {  // hittable_list.h:7-37
  std::vector<const ohit*> objs;
  box3 box;
  void add(const ohit* o) {
    objs.push_back(o);
    box = box3::enclose(box, o->bbox());
  }
  bool hit(const ray3& r, ivl t, hrec& rec, rngctx& g) const override {
    hrec tmp;
    bool any = false;
    for (const ohit* o : objs) {
      if (o->hit(r, t, tmp, g)) {
        any = true;
        t.hi = tmp.t;
        rec = tmp;
      }
    }
    return any;
  }
  box3 bbox() const override { return box; }
};

struct obvh : ohit {  // bvh_node.h
  const ohit* left = nullptr;
  const ohit* right = nullptr;
  box3 box;
  std::vector<std::unique_ptr<obvh>>* pool = nullptr;
  static const ohit* build(std::vector<const ohit*>& objs, size_t b, size_t e,
                           std::vector<std::unique_ptr<obvh>>& pool) {  // bvh_node.h:18-47
    auto node = std::make_unique<obvh>();
    std::sort(objs.begin() + b, objs.begin() + e,
              [](const ohit* a, const ohit* c) { return a->bbox().ax[0].lo < c->bbox().ax[0].lo; });
    size_t n = e - b;
    if (n == 1) {
      node->left = node->right = objs[b];
    } else if (n == 2) {
      node->left = objs[b];
      node->right = objs[b + 1];
    } else {
      size_t mid = (b + e) / 2;
      node->left = build(objs, b, mid, pool);
      node->right = build(objs, mid, e, pool);
    }
    node->box = box3::enclose(node->left->bbox(), node->right->bbox());
    pool.push_back(std::move(node));
    return pool.back().get();
  }
  bool hit(const ray3& r, ivl t, hrec& rec, rngctx& g) const override {  // bvh_node.h:49-59
    if (!box.hit(r, t)) return false;
    bool hl = left->hit(r, t, rec, g);
    ivl t2(t.lo, hl ? rec.t : t.hi);
    bool hr = right->hit(r, t2, rec, g);
    return hl || hr;
  }
  box3 bbox() const override { return box; }
};

struct otranslate : ohit {  // hittable.h:67-89
  const ohit* obj;
  v3 off;
  otranslate(const ohit* o, const v3& d) : obj(o), off(d) {}
  bool hit(const ray3& r, ivl t, hrec& rec, rngctx& g) const override {
    ray3 rr{r.o - off, r.d, r.tm};
    if (!obj->hit(rr, t, rec, g)) return false;
    rec.p = rec.p + off;
    return true;
  }
  box3 bbox() const override { return obj->bbox().offset(off); }
};

struct orotate : ohit {  // hittable.h:93-293; axis 0 = x, 1 = y, 2 = z
  const ohit* obj;
  int axis;
  double s, c;
  box3 box;
  // the two coordinates a rotation about `axis` mixes, in the reference's order
  int ia() const { return axis == 0 ? 1 : 0; }
  int ib() const { return axis == 2 ? 1 : 2; }
  orotate(const ohit* o, int ax, double sin_t, double cos_t) : obj(o), axis(ax), s(sin_t), c(cos_t) {
    box3 bb = o->bbox();
    v3 mn(kInf, kInf, kInf), mx(-kInf, -kInf, -kInf);
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 2; j++)
        for (int k = 0; k < 2; k++) {
          double x = i * bb.ax[0].hi + (1 - i) * bb.ax[0].lo;
          double y = j * bb.ax[1].hi + (1 - j) * bb.ax[1].lo;
          double z = k * bb.ax[2].hi + (1 - k) * bb.ax[2].lo;
          v3 p(x, y, z);
          double pa = p[ia()], pb = p[ib()];
          p[ia()] = c * pa + s * pb;
          p[ib()] = -s * pa + c * pb;
          for (int q = 0; q < 3; q++) {
            mn[q] = std::fmin(mn[q], p[q]);
            mx[q] = std::fmax(mx[q], p[q]);
          }
        }
    box = box3::points(mn, mx);
  }
  bool hit(const ray3& r, ivl t, hrec& rec, rngctx& g) const override {
    int a = ia(), b = ib();
    v3 o = r.o, d = r.d;
    o[a] = c * r.o[a] - s * r.o[b];
    o[b] = s * r.o[a] + c * r.o[b];
    d[a] = c * r.d[a] - s * r.d[b];
    d[b] = s * r.d[a] + c * r.d[b];
    ray3 rr{o, d, r.tm};
    if (!obj->hit(rr, t, rec, g)) return false;
    v3 p = rec.p, n = rec.n;
    p[a] = c * rec.p[a] + s * rec.p[b];
    p[b] = -s * rec.p[a] + c * rec.p[b];
    n[a] = c * rec.n[a] + s * rec.n[b];
    n[b] = -s * rec.n[a] + c * rec.n[b];
    rec.p = p;
    rec.n = n;
    return true;
  }
  box3 bbox() const override { return box; }
};

struct ovolume : ohit {  // volumne.h
  const ohit* boundary;
  double density;
  const omat* phase;
  ovolume(const ohit* b, double dens, const omat* ph) : boundary(b), density(dens), phase(ph) {}
  bool hit(const ray3& r, ivl t, hrec& rec, rngctx& g) const override {  // volumne.h:18-46
    hrec r1, r2;
    if (!boundary->hit(r, ivl(-kInf, kInf), r1, g)) return false;
    if (!boundary->hit(r, ivl(r1.t + 0.0001, kInf), r2, g)) return false;
    if (r1.t < t.lo) r1.t = t.lo;
    if (r2.t > t.hi) r2.t = t.hi;
    if (r1.t >= r2.t) return false;
    if (r1.t < 0) r1.t = 0;
    double rl = len(r.d);
    double inside = (r2.t - r1.t) * rl;
    double hd = -1.0 / density * std::log(g.volume());
    if (hd > inside) return false;
    rec.t = r1.t + hd / rl;
    rec.p = r.at(rec.t);
    rec.n = v3(1, 0, 0);
    rec.u = rec.v = 0;  // stale in the reference (volumne.h:40-44); 0 here and on the device
    rec.front = true;
    rec.mat = phase;
    return true;
  }
  box3 bbox() const override { return boundary->bbox(); }
};

// ---------------------------------------------------------------- scene + camera
struct scene {
  std::vector<std::unique_ptr<ohit>> owned;
  std::vector<std::unique_ptr<obvh>> bvh_pool;
  std::vector<std::unique_ptr<omat>> mats;
  std::vector<std::unique_ptr<otex>> texs;
  const ohit* world = nullptr;
  const ohit* light = nullptr;
  const otex* background = nullptr;

  template <class T>
  T* own(T* p) {
    owned.emplace_back(p);
    return p;
  }
  const otex* solid(const v3& c) {
    auto t = std::make_unique<otex>();
    t->kind = RT_TEX_SOLID;
    t->color = c;
    texs.push_back(std::move(t));
    return texs.back().get();
  }
  const otex* checker(const v3& odd, const v3& even, double scale) {
    auto t = std::make_unique<otex>();
    t->kind = RT_TEX_CHECKER;
    t->odd = odd;
    t->even = even;
    t->scale = scale;
    texs.push_back(std::move(t));
    return texs.back().get();
  }
  const omat* mat(int kind, const otex* tex, float fuzz = 0, float refr = 1) {
    auto m = std::make_unique<omat>();
    m->kind = kind;
    m->tex = tex;
    m->fuzz = fuzz;
    m->refr = refr;
    mats.push_back(std::move(m));
    return mats.back().get();
  }
  const ohit* bvh_from(const std::vector<const ohit*>& list) {  // bvh_node(hittable_list) copies the list
    std::vector<const ohit*> copy = list;
    return obvh::build(copy, 0, copy.size(), bvh_pool);
  }
};

struct camera {  // camera.h fields used by perspective rendering
  int W = 1, H = 1;
  v3 pos, dir, right, up;
  double vw = 0, vh = 0, focal = 1;
};

inline void perspective(camera& c, rt_camera_desc* out, int image_width, double aspect, const v3& pos,
                        const v3& lookat, float focal_length, float fovy_degree) {  // camera.h:21-50
  c.pos = pos;
  v3 world_up(0, 1, 0);
  c.dir = unit(lookat - pos);
  c.right = unit(cross(c.dir, world_up));
  c.up = cross(c.right, c.dir);
  c.focal = focal_length;
  c.W = image_width;
  c.H = int(image_width / aspect);
  c.H = (c.H < 1) ? 1 : c.H;
  float theta = (float)((double)fovy_degree * kPi / 180.0);
  c.vh = 2.0 * std::tan(theta / 2.0) * c.focal;
  c.vw = c.vh * (double(c.W) / c.H);
  if (out) {
    std::memset(out, 0, sizeof(*out));
    out->mode = RT_CAM_PERSPECTIVE;
    out->image_width = c.W;
    out->image_height = c.H;
    for (int k = 0; k < 3; k++) {
      out->pos[k] = c.pos[k];
      out->dir[k] = c.dir[k];
      out->right[k] = c.right[k];
      out->up[k] = c.up[k];
    }
    out->viewport_width = c.vw;
    out->viewport_height = c.vh;
    out->focal_length = c.focal;
    out->focus_dist = 3.4;
  }
}

// ---------------------------------------------------------------- integrator (camera.h:180-241)
struct integrator {
  const scene* sc;
  int max_depth;
  mutable uint64_t segments = 0;

  v3 miss(const ray3& r, rngctx& g) const {  // camera.h:180-190
    if (!sc->background) return {0, 0, 0};
    osphere s;
    s.center = r.o;
    s.radius = 1.0f;
    hrec rec;
    if (s.hit(r, ivl(0.001, kInf), rec, g)) return sc->background->sample(rec.u, rec.v, rec.p);
    return {0, 0, 0};
  }

  v3 ray_color(const ray3& r, int iteration, rngctx& g) const {  // camera.h:193-241
    if (iteration <= 0) return {0, 0, 0};
    g.next_bounce((uint32_t)(max_depth - iteration));
    segments++;
    hrec rec;
    if (!sc->world->hit(r, ivl(0.001, kInf), rec, g)) {
      if (g_trace) std::fprintf(stderr, "[trace] bounce %d o=(%.17g %.17g %.17g) d=(%.17g %.17g %.17g) miss\n",
                                max_depth - iteration, r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z);
      return miss(r, g);
    }
    if (g_trace)
      std::fprintf(stderr, "[trace] bounce %d o=(%.17g %.17g %.17g) d=(%.17g %.17g %.17g) t=%.17g p=(%.17g %.17g %.17g) "
                   "n=(%.9g %.9g %.9g) front=%d mat=%d\n", max_depth - iteration, r.o.x, r.o.y, r.o.z, r.d.x, r.d.y,
                   r.d.z, rec.t, rec.p.x, rec.p.y, rec.p.z, rec.n.x, rec.n.y, rec.n.z, (int)rec.front, rec.mat->kind);
    v3 emission = rec.mat->emitted(rec);
    srec s;
    if (!rec.mat->scatter(r, rec, s, g)) return emission;
    if (s.mode == smode::determined) {
      v3 in = ray_color(s.scattered, iteration - 1, g);
      return s.att * in + emission;
    }
    if (!sc->light) {
      ray3 sr{rec.p, pdf_generate(s.pdf, g), r.tm};
      double pv = pdf_value(s.pdf, sr.d);
      double ps = rec.mat->p_scattered(rec, sr);
      v3 in = ray_color(sr, iteration - 1, g);
      v3 from_scatter = (s.att * ps * in) / pv;
      return from_scatter + emission;
    }
    // dual_pdf(hittable_pdf(light, p), material pdf) (camera.h:228-233, pdf.h:48-61)
    v3 dir;
    if (g.scatter() < 0.5)
      dir = sc->light->random(rec.p, g);
    else
      dir = pdf_generate(s.pdf, g);
    ray3 sr{rec.p, dir, r.tm};
    double pv = 0.5 * sc->light->pdf_value(rec.p, sr.d, g) + 0.5 * pdf_value(s.pdf, sr.d);
    double ps = rec.mat->p_scattered(rec, sr);
    v3 in = ray_color(sr, iteration - 1, g);
    v3 from_scatter = (s.att * ps * in) / pv;
    return from_scatter + emission;
  }
};

struct view {  // precomputed per render (camera.h:137-141, 246, 253, 260, 278)
  int mode = RT_CAM_PERSPECTIVE;
  v3 du, dv, dir00, pos;
  v3 pos00;          // orthonormal / lens: pos - vw/2 right + vh/2 up + (du + dv)/2 (camera.h:253, 278)
  v3 dir, fdir;      // dir_ (unit) and focus_dist_ * dir_ (camera.h:279)
  double focal = 1;  // focal_length_ (camera.h:266)
  v3 disk_u, disk_v; // defocus_disk_u/v (camera.h:129-131)
};

inline view make_view(const rt_camera_desc& c) {
  view v;
  v3 right = v3_from(c.right), up = v3_from(c.up), dir = v3_from(c.dir);
  v.mode = c.mode;
  v.du = c.viewport_width * right / c.image_width;
  v.dv = -c.viewport_height * up / c.image_height;
  v.dir00 = c.focal_length * dir - c.viewport_width / 2.0 * right + c.viewport_height / 2.0 * up + 0.5 * (v.du + v.dv);
  v.pos = v3_from(c.pos);
  v.pos00 = v.pos - c.viewport_width / 2.0 * right + c.viewport_height / 2.0 * up + 0.5 * (v.du + v.dv);
  v.dir = dir;
  v.fdir = c.focus_dist * dir;
  v.focal = c.focal_length;
  v.disk_u = v3_from(c.defocus_u);
  v.disk_v = v3_from(c.defocus_v);
  return v;
}

// camera.h:293 sample_square: (U - 1/2, U - 1/2); GCC evaluates vec3(...) arguments right to left
inline void sample_square(rngctx& g, double& ox, double& oy) {
  if (g.mode == ORC_RNG_COMPAT) {
    oy = g.camera(1) - 0.5;
    ox = g.camera(0) - 0.5;
  } else {
    ox = g.camera(0) - 0.5;
    oy = g.camera(1) - 0.5;
  }
}

// utility.h:46-52 random_in_unit_disk by rejection. Counter mode: attempt k draws dimensions
// kDimDisk + 2k (x) and + 2k + 1 (y); both modes give up after kDiskTries (never reached in
// practice: (1 - pi/4)^64 ~ 1e-43) and return the origin.
enum : uint32_t { kDimDisk = 0x7FFF0000u, kDiskTries = 64 };
inline void random_in_unit_disk(rngctx& g, double& px, double& py) {
  for (uint32_t k = 0; k < kDiskTries; k++) {
    if (g.mode == ORC_RNG_COMPAT) {
      py = -1 + 2 * g.glibc();  // random_double(-1, 1) (utility.h:22), right-to-left
      px = -1 + 2 * g.glibc();
    } else {
      px = -1 + 2 * g.at(kDimDisk + 2 * k);
      py = -1 + 2 * g.at(kDimDisk + 2 * k + 1);
    }
    if (px * px + py * py + 0.0 * 0.0 < 1) return;  // length_squared of (x, y, 0)
  }
  px = py = 0;
}

inline ray3 generate_ray(const view& vw, int y, int x, rngctx& g) {  // camera.h:244-284
  double ox, oy;
  if (vw.mode == RT_CAM_ORTHONORMAL) {  // camera.h:252-258
    v3 p = vw.pos00 + x * vw.du + y * vw.dv;
    sample_square(g, ox, oy);
    v3 rp = p + ox * vw.du + oy * vw.dv;
    double tm = g.camera(2);
    return {rp, vw.dir, tm};
  }
  if (vw.mode == RT_CAM_LENS) {  // camera.h:276-283, 287-290
    sample_square(g, ox, oy);
    v3 rd = vw.pos00 + x * vw.du + y * vw.dv + ox * vw.du + oy * vw.dv + vw.fdir;
    double px, py;
    random_in_unit_disk(g, px, py);
    v3 org = vw.pos + (px * vw.disk_u + py * vw.disk_v);
    rd = rd - org;
    return {org, rd, 0.0};  // ray(origin, direction): time 0, no draw
  }
  v3 ray_dir = vw.dir00 + x * vw.du + y * vw.dv;
  sample_square(g, ox, oy);
  v3 d = ray_dir + ox * vw.du + oy * vw.dv;
  if (vw.mode == RT_CAM_FISHEYE) {  // camera.h:259-275
    double r = len(d - vw.dir);  // vec3::length (vec3.h:31-32)
    double theta = std::asin(r / vw.focal);
    v3 v1 = unit(vw.dir);
    v3 v2 = unit(d);
    double b = std::sqrt(std::sin(theta) * std::sin(theta) / (1 - dot(v1, v2) * dot(v1, v2)));
    double a = std::cos(theta) - b * dot(v1, v2);
    d = a * v1 + b * v2;
  }
  double tm = g.camera(2);
  return {vw.pos, d, tm};
}

// ---------------------------------------------------------------- builtin scenes (main.cc)
scene* build_cornell(bool triangles) {  // main.cc:198-225
  auto* s = new scene;
  auto red = s->mat(RT_MAT_LAMBERTIAN, s->solid({.65, .05, .05}));
  auto white = s->mat(RT_MAT_LAMBERTIAN, s->solid({0.73, 0.73, 0.73}));
  auto green = s->mat(RT_MAT_LAMBERTIAN, s->solid({.12, .45, .15}));
  auto light = s->mat(RT_MAT_DIFFUSE_LIGHT, s->solid({15, 15, 15}));
  auto quad = [&](const v3& q, const v3& u, const v3& v, const omat* m) -> const ohit* {
    return s->own(new oquad(q, u, v, m));
  };
  // A quad as two triangles (q, q+u, q+v) and (q+u+v, q+v, q+u): same facing.
  auto add_q = [&](std::vector<const ohit*>& to, const v3& q, const v3& u, const v3& v, const omat* m) {
    if (!triangles) {
      to.push_back(quad(q, u, v, m));
      return;
    }
    to.push_back(s->own(new otri(q, q + u, q + v, m)));
    to.push_back(s->own(new otri(q + u + v, q + v, q + u, m)));
  };
  auto make_box = [&](const v3& a, const v3& b, const omat* m) {  // quad.h:91-112
    auto* sides = s->own(new olist);
    v3 mn(std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z));
    v3 mx(std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z));
    v3 dx(mx.x - mn.x, 0, 0), dy(0, mx.y - mn.y, 0), dz(0, 0, mx.z - mn.z);
    std::vector<const ohit*> v;
    add_q(v, {mn.x, mn.y, mx.z}, dy, dx, m);
    add_q(v, {mx.x, mn.y, mx.z}, dy, -dz, m);
    add_q(v, {mx.x, mn.y, mn.z}, dy, -dx, m);
    add_q(v, {mn.x, mn.y, mn.z}, dy, dz, m);
    add_q(v, {mn.x, mx.y, mx.z}, -dz, dx, m);
    add_q(v, {mn.x, mn.y, mn.z}, dz, dx, m);
    for (auto* o : v) sides->add(o);
    return sides;
  };
  std::vector<const ohit*> world;
  add_q(world, {555, 0, 0}, {0, 555, 0}, {0, 0, 555}, green);
  add_q(world, {0, 0, 0}, {0, 555, 0}, {0, 0, 555}, red);
  add_q(world, {0, 0, 0}, {555, 0, 0}, {0, 0, 555}, white);
  add_q(world, {555, 555, 555}, {-555, 0, 0}, {0, 0, -555}, white);
  add_q(world, {0, 0, 555}, {555, 0, 0}, {0, 555, 0}, white);
  world.push_back(s->own(new otranslate(make_box({0, 0, 0}, {165, 330, 165}, white), {100, 0, 200})));
  world.push_back(s->own(new otranslate(make_box({0, 0, 0}, {165, 165, 165}, white), {50, 0, 100})));
  const ohit* lq = quad({343, 554, 332}, {-130, 0, 0}, {0, 0, -105}, light);
  world.push_back(lq);
  s->world = s->bvh_from(world);
  s->light = lq;
  s->background = s->solid({0, 0, 0});  // solid_color::black (main.cc:223)
  return s;
}

scene* build_cornell_volume() {  // main.cc:227-253
  auto* s = new scene;
  auto red = s->mat(RT_MAT_LAMBERTIAN, s->solid({.65, .05, .05}));
  auto white = s->mat(RT_MAT_LAMBERTIAN, s->solid({.73, .73, .73}));
  auto green = s->mat(RT_MAT_LAMBERTIAN, s->solid({.12, .45, .15}));
  auto light = s->mat(RT_MAT_DIFFUSE_LIGHT, s->solid({7, 7, 7}));
  auto* world = s->own(new olist);
  world->add(s->own(new oquad({555, 0, 0}, {0, 555, 0}, {0, 0, 555}, green)));
  world->add(s->own(new oquad({0, 0, 0}, {0, 555, 0}, {0, 0, 555}, red)));
  world->add(s->own(new oquad({0, 555, 0}, {555, 0, 0}, {0, 0, 555}, white)));
  world->add(s->own(new oquad({0, 0, 0}, {555, 0, 0}, {0, 0, 555}, white)));
  world->add(s->own(new oquad({0, 0, 555}, {555, 0, 0}, {0, 555, 0}, white)));
  auto make_box = [&](const v3& b, const omat* m) {
    auto* sides = s->own(new olist);
    v3 dx(b.x, 0, 0), dy(0, b.y, 0), dz(0, 0, b.z);
    sides->add(s->own(new oquad({0, 0, b.z}, dy, dx, m)));
    sides->add(s->own(new oquad({b.x, 0, b.z}, dy, -dz, m)));
    sides->add(s->own(new oquad({b.x, 0, 0}, dy, -dx, m)));
    sides->add(s->own(new oquad({0, 0, 0}, dy, dz, m)));
    sides->add(s->own(new oquad({0, b.y, b.z}, -dz, dx, m)));
    sides->add(s->own(new oquad({0, 0, 0}, dz, dx, m)));
    return sides;
  };
  auto rot_y = [&](const ohit* o, double deg) {
    double rad = deg * kPi / 180.0;
    return s->own(new orotate(o, 1, std::sin(rad), std::cos(rad)));
  };
  auto box1 = s->own(new otranslate(rot_y(make_box({150, 280, 150}, white), 45), {265, 0, 285}));
  auto box2 = s->own(new otranslate(rot_y(make_box({140, 140, 140}, white), -15), {130, 0, 65}));
  world->add(s->own(new ovolume(box1, 0.02, s->mat(RT_MAT_ISOTROPIC, s->solid({0, 0, 0})))));
  world->add(s->own(new ovolume(box2, 0.02, s->mat(RT_MAT_ISOTROPIC, s->solid({1, 1, 1})))));
  const ohit* lq = s->own(new oquad({113, 554, 127}, {330, 0, 0}, {0, 0, 305}, light));
  world->add(lq);
  s->world = world;
  s->light = lq;
  s->background = s->solid({0, 0, 0});
  return s;
}

inline double rnd() { return std::rand() / (RAND_MAX + 1.0); }

scene* build_rtow(bool moving) {  // main.cc:105-153, draws sequenced as GCC evaluates them
  std::srand(1);
  auto* s = new scene;
  auto ground = s->mat(RT_MAT_LAMBERTIAN, s->checker({1.0, 1.0, 1.0}, {0.6, 0.6, 0.2}, 1.0));
  std::vector<const ohit*> world;
  world.push_back(s->own(osphere::make_static({0, -1000, 0}, 1000, ground)));
  for (int a = -11; a < 11; a++) {
    for (int b = -11; b < 11; b++) {
      double choose = rnd();
      double rz = rnd();  // point3 center1(a + 0.7*rd(), 0.2, b + 0.7*rd()): z first
      double rx = rnd();
      v3 c1(a + 0.7 * rx, 0.2, b + 0.7 * rz);
      v3 c2 = c1 + v3(0, 0 + (.15 - 0) * rnd(), 0);
      if (len(c1 - v3(4, 0.2, 0)) <= 0.9) continue;
      const omat* m = nullptr;
      if (choose < 0.3) {
        continue;
      } else if (choose < 0.8) {
        // random_vec() * random_vec(): right operand first, components z, y, x
        double bz = rnd(), by = rnd(), bx = rnd();
        double az = rnd(), ay = rnd(), ax = rnd();
        v3 albedo = v3(ax, ay, az) * v3(bx, by, bz);
        m = s->mat(RT_MAT_LAMBERTIAN, s->solid(albedo));
      } else if (choose < 0.95) {
        double z = 0.5 + (1 - 0.5) * rnd();
        double y = 0.5 + (1 - 0.5) * rnd();
        double x = 0.5 + (1 - 0.5) * rnd();
        m = s->mat(RT_MAT_METAL, s->solid({x, y, z}), 0.0f);
      } else {
        m = s->mat(RT_MAT_DIELECTRIC, s->solid({1, 1, 1}), 0.0f, 1.5f);
      }
      if (moving)
        world.push_back(s->own(osphere::make_moving(c1, c2, 0.2, m)));
      else
        world.push_back(s->own(osphere::make_static(c1, 0.2, m)));
    }
  }
  auto glass = s->mat(RT_MAT_DIELECTRIC, s->solid({1, 1, 1}), 0.0f, 1.5f);
  auto matte = s->mat(RT_MAT_LAMBERTIAN, s->solid({0.4, 0.2, 0.1}));
  (void)s->mat(RT_MAT_METAL, s->solid({0.7, 0.6, 0.5}), 0.0f);  // metal_mat: built, unused (main.cc:144)
  world.push_back(s->own(osphere::make_static({0, 1, 0}, 1.0, glass)));
  world.push_back(s->own(osphere::make_static({-4, 1, 0}, 1.0, matte)));
  world.push_back(s->own(osphere::make_static({4, 1, 0}, 1.0, glass)));
  s->world = s->bvh_from(world);
  s->background = s->solid({0.7, 0.8, 1.0});
  return s;
}

scene* build_three_material_ball() {  // main.cc:67-84
  auto* s = new scene;
  auto ground = s->mat(RT_MAT_LAMBERTIAN, s->checker({1.0, 1.0, 1.0}, {0.6, 0.6, 0.2}, 1.0));
  auto glass = s->mat(RT_MAT_DIELECTRIC, s->solid({1.0, 1.0, 1.0}), 0.0f, 1.5f);
  auto matte = s->mat(RT_MAT_LAMBERTIAN, s->solid({0.4, 0.2, 0.1}));
  auto metal = s->mat(RT_MAT_METAL, s->solid({0.7, 0.6, 0.5}), 0.0f);
  auto* world = s->own(new olist);
  world->add(s->own(osphere::make_static({0, -1000, 0}, 1000, ground)));
  world->add(s->own(osphere::make_static({0, 1, 0}, 1.0, glass)));
  world->add(s->own(osphere::make_static({-4, 1, 0}, 1.0, matte)));
  world->add(s->own(osphere::make_static({4, 1, 0}, 1.0, metal)));
  s->world = world;
  s->background = s->solid({0.7, 0.8, 1.0});
  return s;
}

// ---------------------------------------------------------------- scene from a descriptor
struct desc_builder {
  const rt_scene_desc* d;
  scene* s;
  std::vector<const ohit*> built;
  std::vector<int> state;  // 0 = not built, 1 = building, 2 = built
  std::vector<const otex*> tex;
  std::vector<const omat*> mat;
  std::string err;

  const ohit* build(int idx) {
    if (idx < 0 || idx >= d->num_objects) {
      err = "object index out of range";
      return nullptr;
    }
    if (state[idx] == 2) return built[idx];
    if (state[idx] == 1) {
      err = "cycle in the object graph";
      return nullptr;
    }
    state[idx] = 1;
    const rt_object& o = d->objects[idx];
    const omat* m = (o.material >= 0 && o.material < (int)mat.size()) ? mat[o.material] : nullptr;
    const ohit* r = nullptr;
    switch (o.kind) {
      case RT_OBJ_SPHERE:
        r = o.moving ? s->own(osphere::make_moving(v3_from(o.a), v3_from(o.b), o.s0, m))
                     : s->own(osphere::make_static(v3_from(o.a), o.s0, m));
        break;
      case RT_OBJ_QUAD:
        r = s->own(new oquad(v3_from(o.a), v3_from(o.b), v3_from(o.c), m));
        break;
      case RT_OBJ_TRIANGLE:
        r = s->own(new otri(v3_from(o.a), v3_from(o.b), v3_from(o.c), m));
        break;
      case RT_OBJ_LIST:
      case RT_OBJ_BVH: {
        if (o.first_child < 0 || o.child_count < 0 || o.first_child + o.child_count > d->num_children) {
          err = "child range out of bounds";
          return nullptr;
        }
        std::vector<const ohit*> kids;
        for (int k = 0; k < o.child_count; k++) {
          const ohit* c = build(d->children[o.first_child + k]);
          if (!c) return nullptr;
          kids.push_back(c);
        }
        if (o.kind == RT_OBJ_LIST || kids.empty()) {
          auto* l = s->own(new olist);
          for (auto* c : kids) l->add(c);
          r = l;
        } else {
          r = s->bvh_from(kids);
        }
        break;
      }
      case RT_OBJ_TRANSLATE: {
        const ohit* c = build(o.child);
        if (!c) return nullptr;
        r = s->own(new otranslate(c, v3_from(o.a)));
        break;
      }
      case RT_OBJ_ROTATE_X:
      case RT_OBJ_ROTATE_Y:
      case RT_OBJ_ROTATE_Z: {
        const ohit* c = build(o.child);
        if (!c) return nullptr;
        r = s->own(new orotate(c, o.kind - RT_OBJ_ROTATE_X, o.s0, o.s1));
        break;
      }
      case RT_OBJ_VOLUME: {
        const ohit* c = build(o.child);
        if (!c) return nullptr;
        if (!m) {
          err = "volume without phase material";
          return nullptr;
        }
        r = s->own(new ovolume(c, o.s0, m));
        break;
      }
      default:
        err = "unknown object kind";
        return nullptr;
    }
    state[idx] = 2;
    built[idx] = r;
    return r;
  }
};

// ---------------------------------------------------------------- rendering
struct job {
  const scene* sc;
  view vw;
  int W, H;
  int spp, first, depth;
  uint64_t seed;
  int mode;
};

inline v3 render_pixel(const job& jb, int x, int y, uint64_t& segs) {  // camera.h:164-170
  integrator it{jb.sc, jb.depth};
  v3 sum(0, 0, 0);
  rngctx g;
  g.mode = jb.mode;
  uint32_t ka = key_pixel(jb.seed, (uint32_t)(y * jb.W + x));
  for (int k = 0; k < jb.spp; k++) {
    g.ks = key_path(ka, key_sample(jb.seed, (uint32_t)(jb.first + k)));
    g.bounce = 0;
    ray3 r = generate_ray(jb.vw, y, x, g);
    sum = sum + it.ray_color(r, jb.depth, g);
  }
  segs += it.segments;
  return sum / jb.spp;
}

}  // namespace orc

using namespace orc;

extern "C" {

void orc_set_trace(int on) { g_trace = on; }

void* orc_scene_from_desc(const rt_scene_desc* d, char* err, int errlen) {
  auto fail = [&](const std::string& m) -> void* {
    if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", m.c_str());
    return nullptr;
  };
  if (!d) return fail("null descriptor");
  auto s = std::make_unique<scene>();
  desc_builder b{d, s.get(), {}, {}, {}, {}, {}};
  b.built.assign((size_t)std::max(0, d->num_objects), nullptr);
  b.state.assign((size_t)std::max(0, d->num_objects), 0);
  for (int i = 0; i < d->num_textures; i++) {
    const rt_texture& t = d->textures[i];
    if (t.kind == RT_TEX_SOLID)
      b.tex.push_back(s->solid(v3_from(t.color)));
    else if (t.kind == RT_TEX_CHECKER)
      b.tex.push_back(s->checker(v3_from(t.odd), v3_from(t.even), t.scale));
    else if (t.kind == RT_TEX_IMAGE) {
      auto tx = std::make_unique<otex>();
      tx->kind = RT_TEX_IMAGE;
      tx->width = (int)t.color[0];
      tx->height = (int)t.color[1];
      const int64_t n = 3LL * tx->width * tx->height;
      if (n > 0 && (!d->image_data || t.data < 0 || t.data + n > d->num_image_data)) return fail("image: data too short");
      if (n > 0) tx->pixels.assign(d->image_data + t.data, d->image_data + t.data + n);
      s->texs.push_back(std::move(tx));
      b.tex.push_back(s->texs.back().get());
    } else if (t.kind >= RT_TEX_PERLIN && t.kind <= RT_TEX_VORONOI) {
      auto tx = std::make_unique<otex>();
      tx->kind = t.kind;
      tx->scale = t.scale;
      if (t.kind == RT_TEX_PERLIN) {
        if (!d->tex_data || t.data < 0 || t.data + 6 * 256 > d->num_tex_data) return fail("perlin: tex_data too short");
        const double* src = d->tex_data + t.data;
        for (int k = 0; k < 256; k++) tx->noise.rand_offset.push_back(v3(src[3 * k], src[3 * k + 1], src[3 * k + 2]));
        for (int k = 0; k < 256; k++) tx->noise.perm_x.push_back((int)src[768 + k]);
      } else if (t.kind == RT_TEX_VALUE) {
        int n = (int)t.scale;
        if (n < 1 || !d->tex_data || t.data < 0 || t.data + (int64_t)n * n * n > d->num_tex_data)
          return fail("value: bad resolution or tex_data too short");
        tx->noise.resolution = n;
        for (int64_t k = 0; k < (int64_t)n * n * n; k++) tx->noise.values.push_back((float)d->tex_data[t.data + k]);
      }
      s->texs.push_back(std::move(tx));
      b.tex.push_back(s->texs.back().get());
    } else
      return fail("unsupported texture kind");
  }
  for (int i = 0; i < d->num_materials; i++) {
    const rt_material& m = d->materials[i];
    if (m.texture < 0 || m.texture >= (int)b.tex.size()) return fail("material texture out of range");
    auto mm = std::make_unique<omat>();
    mm->kind = m.kind;
    mm->tex = b.tex[m.texture];
    mm->fuzz = m.fuzz;
    mm->refr = m.refraction;
    mm->smooth = m.smoothness < 0.f ? 0.f : (m.smoothness > 1.f ? 1.f : m.smoothness);  // material.h:149
    mm->spec = m.specular_prob;
    s->mats.push_back(std::move(mm));
    b.mat.push_back(s->mats.back().get());
  }
  s->world = b.build(d->world);
  if (!s->world) return fail("world: " + b.err);
  if (d->light >= 0) {
    s->light = b.build(d->light);
    if (!s->light) return fail("light: " + b.err);
  }
  if (d->background >= 0) {
    if (d->background >= (int)b.tex.size()) return fail("background texture out of range");
    s->background = b.tex[d->background];
  }
  return s.release();
}

void* orc_builtin(const char* name, int image_width, double aspect, rt_camera_desc* cam, int* spp,
                  int* max_depth) {
  std::string n = name ? name : "";
  scene* s = nullptr;
  camera c;
  int dspp = 0, ddepth = 0;
  if (n == "cornell_box" || n == "cornell_triangles") {  // main.cc:222
    s = build_cornell(n == "cornell_triangles");
    perspective(c, cam, image_width > 0 ? image_width : 600, aspect > 0 ? aspect : 1.0, {278, 278, -800},
                {278, 278, 0}, 1, 40.0f);
    dspp = 40;
    ddepth = 4;
  } else if (n == "cornell_box_with_volume") {  // main.cc:249
    s = build_cornell_volume();
    perspective(c, cam, image_width > 0 ? image_width : 600, aspect > 0 ? aspect : 1.0, {278, 278, -800},
                {278, 278, 0}, 1, 40);
    dspp = 100;
    ddepth = 5;
  } else if (n == "rtow" || n == "rtow_motion") {  // main.cc:149
    s = build_rtow(n == "rtow_motion");
    perspective(c, cam, image_width > 0 ? image_width : 1280, aspect > 0 ? aspect : 16.0 / 9.0, {13, 2, 3},
                {0, 0, 0}, 1, 20);
    dspp = 20;
    ddepth = 50;
  } else if (n == "three_material_ball") {  // main.cc:81
    s = build_three_material_ball();
    perspective(c, cam, image_width > 0 ? image_width : 1280, aspect > 0 ? aspect : 16.0 / 9.0, {13, 2, 3},
                {0, 0, 0}, 1, 20.0f);
    dspp = 100;
    ddepth = 5;
  } else {
    return nullptr;
  }
  if (spp) *spp = dspp;
  if (max_depth) *max_depth = ddepth;
  return s;
}

void orc_scene_free(void* p) { delete static_cast<scene*>(p); }

int orc_render(const void* scp, const rt_camera_desc* cam, int spp, int first_sample, int max_depth,
               uint64_t seed, int rng_mode, int threads, const rt_tile* tiles, int ntiles, double* out,
               uint64_t* segments) {
  if (!scp || !cam || !tiles || ntiles <= 0 || !out || spp <= 0 || cam->mode < RT_CAM_PERSPECTIVE ||
      cam->mode > RT_CAM_LENS)
    return 1;
  job jb;
  jb.sc = static_cast<const scene*>(scp);
  jb.vw = make_view(*cam);
  jb.W = cam->image_width;
  jb.H = cam->image_height;
  jb.spp = spp;
  jb.first = first_sample;
  jb.depth = max_depth;
  jb.seed = seed;
  jb.mode = rng_mode;
  // flatten tiles into a pixel list in output order
  std::vector<std::pair<int, int>> px;
  for (int t = 0; t < ntiles; t++)
    for (int y = 0; y < tiles[t].height; y++)
      for (int x = 0; x < tiles[t].width; x++) px.emplace_back(tiles[t].x0 + x, tiles[t].y0 + y);
  uint64_t total_segs = 0;
  if (rng_mode == ORC_RNG_COMPAT) {
    if (seed != 0) std::srand((unsigned)seed);
    for (size_t i = 0; i < px.size(); i++) {
      v3 c = render_pixel(jb, px[i].first, px[i].second, total_segs);
      out[3 * i] = c.x;
      out[3 * i + 1] = c.y;
      out[3 * i + 2] = c.z;
    }
  } else {
    int nt = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    std::atomic<size_t> next{0};
    std::vector<uint64_t> segs((size_t)nt, 0);
    const size_t chunk = 64;
    auto worker = [&](int id) {
      for (;;) {
        size_t b = next.fetch_add(chunk);
        if (b >= px.size()) break;
        size_t e = std::min(px.size(), b + chunk);
        for (size_t i = b; i < e; i++) {
          v3 c = render_pixel(jb, px[i].first, px[i].second, segs[(size_t)id]);
          out[3 * i] = c.x;
          out[3 * i + 1] = c.y;
          out[3 * i + 2] = c.z;
        }
      }
    };
    std::vector<std::thread> pool;
    for (int i = 1; i < nt; i++) pool.emplace_back(worker, i);
    worker(0);
    for (auto& t : pool) t.join();
    for (uint64_t s : segs) total_segs += s;
  }
  if (segments) *segments = total_segs;
  return 0;
}

size_t orc_write_ppm(const double* img, int w, int h, char* buf, size_t cap) {  // camera.h:149-151,174
  std::string s = "P3\n" + std::to_string(w) + ' ' + std::to_string(h) + '\n' + "255\n";
  auto gamma = [](double x) { return x > 0 ? std::pow(x, 1 / 2.2) : 0.0; };  // color.h:16-20
  char line[96];
  for (long i = 0; i < (long)w * h; i++) {
    double r = gamma(img[3 * i]), g = gamma(img[3 * i + 1]), b = gamma(img[3 * i + 2]);
    int n = std::snprintf(line, sizeof line, "%d %d %d\n", int(255.999 * r), int(255.999 * g), int(255.999 * b));
    s.append(line, (size_t)n);
  }
  if (buf && cap >= s.size()) std::memcpy(buf, s.data(), s.size());
  return s.size();
}

uint32_t orc_rng_u32(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t dim) {
  return draw_u32(key_path(key_pixel(seed, pixel), key_sample(seed, sample)), dim);
}

int orc_kat_sphere_hit(const double c[3], double r, const double o[3], const double d[3], double tmin, double tmax,
                       double out[9]) {
  std::unique_ptr<osphere> s(osphere::make_static(v3_from(c), r, nullptr));
  hrec rec;
  rngctx g;
  if (!s->hit({v3_from(o), v3_from(d), 0}, ivl(tmin, tmax), rec, g)) return 0;
  double v[9] = {rec.t, rec.p.x, rec.p.y, rec.p.z, rec.n.x, rec.n.y, rec.n.z, rec.u, rec.v};
  std::memcpy(out, v, sizeof v);
  return 1;
}

int orc_kat_quad_hit(const double q[3], const double u[3], const double v[3], const double o[3], const double d[3],
                     double tmin, double tmax, double out[9]) {
  oquad s(v3_from(q), v3_from(u), v3_from(v), nullptr);
  hrec rec;
  rngctx g;
  if (!s.hit({v3_from(o), v3_from(d), 0}, ivl(tmin, tmax), rec, g)) return 0;
  double r[9] = {rec.t, rec.p.x, rec.p.y, rec.p.z, rec.n.x, rec.n.y, rec.n.z, rec.u, rec.v};
  std::memcpy(out, r, sizeof r);
  return 1;
}

int orc_kat_triangle_hit(const double p0[3], const double p1[3], const double p2[3], const double o[3],
                         const double d[3], double tmin, double tmax, double out[7]) {
  otri s(v3_from(p0), v3_from(p1), v3_from(p2), nullptr);
  hrec rec;
  rngctx g;
  if (!s.hit({v3_from(o), v3_from(d), 0}, ivl(tmin, tmax), rec, g)) return 0;
  double r[7] = {rec.t, rec.p.x, rec.p.y, rec.p.z, rec.n.x, rec.n.y, rec.n.z};
  std::memcpy(out, r, sizeof r);
  return 1;
}

void orc_kat_onb(const double n[3], double out[9]) {
  v3 x, y, z;
  make_onb(v3_from(n), x, y, z);
  double r[9] = {x.x, x.y, x.z, y.x, y.y, y.z, z.x, z.y, z.z};
  std::memcpy(out, r, sizeof r);
}

void orc_kat_refract(const double v[3], const double n[3], double eta, double out[3]) {
  v3 r = refract(v3_from(v), v3_from(n), eta);
  out[0] = r.x;
  out[1] = r.y;
  out[2] = r.z;
}

double orc_kat_reflectance(double cosine, double ri) { return omat::reflectance(cosine, ri); }

int orc_kat_aabb_hit(const double a[3], const double b[3], const double o[3], const double d[3], double tmin,
                     double tmax) {
  return box3::points(v3_from(a), v3_from(b)).hit({v3_from(o), v3_from(d), 0}, ivl(tmin, tmax)) ? 1 : 0;
}

// closest hit over n spheres (xyzr[4k..4k+3]) through hittable_list (bvh = 0) or bvh_node (bvh = 1)
int orc_kat_world_hit(const double* xyzr, int n, int bvh, const double o[3], const double d[3], double tmin,
                      double tmax, double out[7]) {
  std::vector<std::unique_ptr<osphere>> sp;
  olist list;
  for (int k = 0; k < n; k++) {
    sp.emplace_back(osphere::make_static({xyzr[4 * k], xyzr[4 * k + 1], xyzr[4 * k + 2]}, xyzr[4 * k + 3], nullptr));
    list.add(sp.back().get());
  }
  std::vector<std::unique_ptr<obvh>> pool;
  std::vector<const ohit*> objs = list.objs;
  const ohit* world = bvh ? obvh::build(objs, 0, objs.size(), pool) : static_cast<const ohit*>(&list);
  hrec rec;
  rngctx g;
  if (!world->hit({v3_from(o), v3_from(d), 0}, ivl(tmin, tmax), rec, g)) return 0;
  double r[7] = {rec.t, rec.p.x, rec.p.y, rec.p.z, rec.n.x, rec.n.y, rec.n.z};
  std::memcpy(out, r, sizeof r);
  return 1;
}

double orc_kat_sphere_pdf(const double c[3], double r, const double o[3], const double dir[3]) {
  std::unique_ptr<osphere> s(osphere::make_static(v3_from(c), r, nullptr));
  rngctx g;
  return s->pdf_value(v3_from(o), v3_from(dir), g);
}

double orc_kat_cosine_pdf(const double n[3], const double dir[3]) {
  pdfsel p;
  make_onb(v3_from(n), p.onb_x, p.onb_y, p.onb_z);
  return pdf_value(p, v3_from(dir));
}

// noise.h evaluated on given tables: kind 0 perlin (table = 256 offsets xyz, then perm_x, perm_y,
// perm_z as the host draws them; turb(7) into out_turb), 1 value noise (resolution^3 values),
// 2 worley, 3 voronoi (no table)
void orc_kat_noise(int kind, const double* table, int resolution, const double* pts, int n, double* out,
                   double* out_turb) {
  onoise nz;
  if (kind == 0) {
    for (int i = 0; i < 256; i++) nz.rand_offset.emplace_back(table[3 * i], table[3 * i + 1], table[3 * i + 2]);
    for (int i = 0; i < 256; i++) nz.perm_x.push_back((int)table[768 + i]);
  } else if (kind == 1) {
    nz.resolution = resolution;
    for (int i = 0; i < resolution * resolution * resolution; i++) nz.values.push_back((float)table[i]);
  }
  for (int i = 0; i < n; i++) {
    const v3 p(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
    out[i] = kind == 0 ? nz.perlin(p) : kind == 1 ? nz.value(p) : onoise::cells(p, kind == 3);
    if (kind == 0 && out_turb) out_turb[i] = nz.turb(7, p);
  }
}

// kind 0: random_in_unit_sphere, 1: random_unit_vec, 2: random_cosine_direction, n vectors after
// srand(seed), in the glibc-compat mode (the reference's rand() draws)
void orc_kat_compat_draws(unsigned seed, int kind, int n, double* out) {
  std::srand(seed);
  rngctx g;
  g.mode = ORC_RNG_COMPAT;
  for (int i = 0; i < n; i++) {
    const v3 v = kind == 0 ? random_on_sphere(g) : kind == 1 ? random_unit_vec(g) : random_cosine_direction(g);
    out[3 * i] = v.x;
    out[3 * i + 1] = v.y;
    out[3 * i + 2] = v.z;
  }
}

}  // extern "C"
