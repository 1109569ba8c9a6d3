// noise.h -- procedural noise of the plugin surface (reference: src/noise.h:5-201).
// The constructors draw from the global std::rand exactly as the reference's do (perlin: 256
// random unit vectors, then the x, y and z permutations; value_noise: n^3 values), so a scene
// built in the reference's order gets the reference's tables. noise() is evaluated on the host
// here and on the device after flattening (csrc/rt_device.h); like the reference, perlin reads
// perm_x for all three axes (noise.h:36), and value_noise indexes its table without wrapping
// (an index outside it reads 0 here, undefined behaviour in the reference).
#pragma once
#include <cmath>
#include <limits>
#include <vector>

#include "utility.h"
#include "vec3.h"

class noise_base {
 public:
  virtual ~noise_base() = default;
  virtual double noise(const point3& p) const = 0;
};

class perlin : public noise_base {
 public:
  static const int point_count = 256;
  perlin() {
    for (int i = 0; i < point_count; i++) rand_offset_[i] = unit_vector(random_vec(-1, 1));
    generate_perm(perm_x_);
    generate_perm(perm_y_);
    generate_perm(perm_z_);
  }
  double noise(const point3& p) const override {
    int iu = int(std::floor(p.x())), iv = int(std::floor(p.y())), iw = int(std::floor(p.z()));
    double u = p.x() - iu, v = p.y() - iv, w = p.z() - iw;
    iu &= point_count - 1;
    iv &= point_count - 1;
    iw &= point_count - 1;
    double uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
    double accum = 0.0;
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 2; j++)
        for (int k = 0; k < 2; k++) {
          const vec3& g = rand_offset_[perm_x_[(iu + i) % point_count] ^ perm_x_[(iv + j) % point_count] ^
                                       perm_x_[(iw + k) % point_count]];
          accum += (i * uu + (1 - i) * (1 - uu)) * (j * vv + (1 - j) * (1 - vv)) * (k * ww + (1 - k) * (1 - ww)) *
                   dot(g, vec3(u - i, v - j, w - k));
        }
    return accum;
  }
  double turb(int depth, const point3& p) const {
    double accum = 0, weight = 1.0;
    point3 q = p;
    for (int i = 0; i < depth; i++) {
      accum += weight * noise(q);
      weight *= 0.5;
      q *= 2.0;
    }
    return std::fabs(accum);
  }
  // rt_texture tables (RT_TEX_PERLIN): rand_offset xyz, perm_x, perm_y, perm_z
  std::vector<double> tables() const {
    std::vector<double> t;
    for (const vec3& v : rand_offset_) t.insert(t.end(), {v.x(), v.y(), v.z()});
    for (const int* pm : {perm_x_, perm_y_, perm_z_}) t.insert(t.end(), pm, pm + point_count);
    return t;
  }

 private:
  vec3 rand_offset_[point_count];
  int perm_x_[point_count], perm_y_[point_count], perm_z_[point_count];
  static void generate_perm(int* p) {  // identity, then a Fisher-Yates shuffle (noise.h:82-97)
    for (int i = 0; i < point_count; i++) p[i] = i;
    for (int i = point_count - 1; i > 0; i--) {
      int target = random_int(0, i);
      int tmp = p[i];
      p[i] = p[target];
      p[target] = tmp;
    }
  }
};

class value_noise : public noise_base {
 public:
  explicit value_noise(int resolution) : n_(resolution), values_((size_t)resolution * resolution * resolution) {
    for (int i = 0; i < n_; i++)
      for (int j = 0; j < n_; j++)
        for (int k = 0; k < n_; k++) values_[(size_t)i * n_ * n_ + (size_t)j * n_ + k] = (float)random_double();
  }
  double noise(const point3& p) const override {
    const double fx = std::floor(p.x()), fy = std::floor(p.y()), fz = std::floor(p.z());
    auto at = [&](double x, double y, double z) -> float {
      const double k = x * n_ * n_ + y * n_ + z;
      return (k >= 0 && k < (double)values_.size()) ? values_[(size_t)k] : 0.0f;
    };
    const double x = p.x() - fx, y = p.y() - fy, z = p.z() - fz;
    auto lerp = [](double t, double a, double b) { return (1 - t) * a + t * b; };
    const double y0z0 = lerp(x, at(fx, fy, fz), at(fx + 1, fy, fz)), y1z0 = lerp(x, at(fx, fy + 1, fz), at(fx + 1, fy + 1, fz)),
                 y0z1 = lerp(x, at(fx, fy, fz + 1), at(fx + 1, fy, fz + 1)),
                 y1z1 = lerp(x, at(fx, fy + 1, fz + 1), at(fx + 1, fy + 1, fz + 1));
    return lerp(z, lerp(y, y0z0, y1z0), lerp(y, y0z1, y1z1));
  }
  int resolution() const { return n_; }
  std::vector<double> tables() const { return std::vector<double>(values_.begin(), values_.end()); }

 private:
  int n_;
  std::vector<float> values_;
};

// worley (squared distance to the nearest feature point) and voronoi (a hash of it), noise.h:139-201
class cell_noise_base : public noise_base {
 protected:
  static vec3 cell_offset(const vec3& u) {
    vec3 r(dot(u, vec3(127.1, 311.7, 74.7)), dot(u, vec3(269.5, 183.3, 246.1)), dot(u, vec3(113.5, 271.9, 307.7)));
    vec3 q = vec3(std::sin(r.x()), std::sin(r.y()), std::sin(r.z())) * 43758.5453;
    return q - vec3(std::floor(q.x()), std::floor(q.y()), std::floor(q.z()));
  }
  static double nearest(const point3& p, bool voronoi) {
    const vec3 f(std::floor(p.x()), std::floor(p.y()), std::floor(p.z()));
    float min_dist = std::numeric_limits<float>::max(), color = 0.0f;
    for (int i = -1; i <= 1; i++)
      for (int j = -1; j <= 1; j++)
        for (int k = -1; k <= 1; k++) {
          const vec3 cell = f + vec3(i, j, k);
          const vec3 pos = cell + cell_offset(cell);
          const float dist = (float)(pos - p).length();
          if (dist < min_dist) {
            min_dist = dist;
            if (voronoi) color = (float)cell_offset(pos).x();
          }
        }
    return voronoi ? color : min_dist * min_dist;
  }
};
class worley_noise : public cell_noise_base {
 public:
  double noise(const point3& p) const override { return nearest(p, false); }
};
class voronoi_noise : public cell_noise_base {
 public:
  double noise(const point3& p) const override { return nearest(p, true); }
};
