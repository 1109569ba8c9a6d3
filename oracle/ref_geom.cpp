// oracle/_ref/ref_geom -- test infrastructure only: runs the reference's own geometry and sampling
// code, compiled where it lies (/root/reference/src, oracle/Makefile's `ref` target), on
// deterministic cases and prints them with the reference's results as one JSON document:
//   sphere    sphere::hit (sphere.h:40-74): t, p, normal, front_face, u, v
//   triangle  triangle::hit (triangle.h:8-40): t, p, normal, front_face
//   aabb      aabb::hit (aabb.h:28-33, 45-69)
//   world     hittable_list::hit (hittable_list.h:20-31) and bvh_node::hit over the same spheres
//             (bvh_node.h:12-59, x-median tree): t, p, normal
//   onb       onb(n) (onb.h:18-29); refract (utility.h:71-76)
//   pdf       sphere::pdf_value (sphere.h:76-78), hemisphere_cosine_pdf::value (pdf.h:34-41)
//   draws     random_in_unit_sphere / random_unit_vec / random_cosine_direction after srand(seed)
//             (utility.h:30-69: glibc rand(), the oracle's compat mode)
//   noise     perlin noise / turb(7) and value noise with the tables their constructors draw after
//             srand(seed) (noise.h:10-136), worley and voronoi (noise.h:139-201)
// Only headers that do not reach image.h (which needs the absent tinyexr) are included; quad.h,
// material.h and camera.h do (quad.h includes material.h), so they are pinned elsewhere
// (DESIGN.md §6). Doubles are printed with 17 significant digits (round-trip exact).
// Built only in the container that has /root/reference; tests/golden/make_ref_geom_golden.py
// turns its output into tests/golden/ref_geom.json, which tests/test_oracle_refpins.py checks the
// oracle against. Never linked into the product.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "utility.h"
#include "aabb.h"
#include "hittable.h"
#include "sphere.h"
#include "triangle.h"
#include "hittable_list.h"
#include "bvh_node.h"
#include "onb.h"
#include "pdf.h"
#include "noise.h"

namespace {

struct Gen {  // splitmix64: the case generator (not the reference's RNG)
  uint64_t s;
  double u() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
  }
  double in(double a, double b) { return a + (b - a) * u(); }
  vec3 v(double a, double b) { return vec3(in(a, b), in(a, b), in(a, b)); }
};

std::string num(double x) {
  if (x != x) return "\"nan\"";
  if (x == infinity) return "\"inf\"";
  if (x == -infinity) return "\"-inf\"";
  char b[40];
  std::snprintf(b, sizeof b, "%.17g", x);
  return b;
}
std::string vec(const vec3& a) { return "[" + num(a.x()) + "," + num(a.y()) + "," + num(a.z()) + "]"; }

std::string hit_json(bool h, const hit_record& r, bool uv) {
  if (!h) return "\"hit\":false";
  std::string s = "\"hit\":true,\"t\":" + num(r.t) + ",\"p\":" + vec(r.p) + ",\"n\":" + vec(r.normal) +
                  ",\"front\":" + (r.front_face ? "true" : "false");
  if (uv) s += ",\"u\":" + num(r.u) + ",\"v\":" + num(r.v);
  return s;
}

}  // namespace

int main() {
  Gen g{20261016};
  std::printf("{\n\"sphere\":[\n");
  for (int i = 0; i < 300; i++) {
    const vec3 c = g.v(-3, 3), o = g.v(-8, 8);
    const double r = g.in(0.05, 2.5);
    // aim near the sphere (most cases hit, some graze or miss); a few rays start inside
    vec3 d = (c + g.v(-1.5 * r, 1.5 * r)) - o;
    vec3 o2 = i % 10 == 9 ? c + g.v(-0.3 * r, 0.3 * r) : o;
    if (i % 7 == 3) d = d * g.in(0.1, 5.0);  // unnormalised directions scale t
    const double tmin = i % 5 == 0 ? 0.001 : g.in(0.0, 1.0), tmax = i % 11 == 4 ? g.in(2, 10) : infinity;
    sphere s(c, r, nullptr);
    hit_record rec;
    const bool h = s.hit(ray(o2, d), interval(tmin, tmax), rec);
    std::printf("%s{\"c\":%s,\"r\":%s,\"o\":%s,\"d\":%s,\"tmin\":%s,\"tmax\":%s,%s}\n", i ? "," : "", vec(c).c_str(),
                num(r).c_str(), vec(o2).c_str(), vec(d).c_str(), num(tmin).c_str(), num(tmax).c_str(),
                hit_json(h, rec, true).c_str());
  }
  std::printf("],\n\"triangle\":[\n");
  for (int i = 0; i < 300; i++) {
    const vec3 p0 = g.v(-3, 3), p1 = g.v(-3, 3), p2 = g.v(-3, 3), o = g.v(-8, 8);
    const double b0 = g.in(-0.2, 1.0), b1 = g.in(-0.2, 1.0);
    const vec3 target = p0 + b0 * (p1 - p0) + b1 * (p2 - p0);  // about half of them inside
    const vec3 d = (target - o) * g.in(0.2, 3.0);
    const double tmin = 0.001, tmax = i % 9 == 2 ? g.in(0.1, 1.0) : infinity;
    triangle t(p0, p1, p2, nullptr);
    hit_record rec;
    const bool h = t.hit(ray(o, d), interval(tmin, tmax), rec);
    std::printf("%s{\"p0\":%s,\"p1\":%s,\"p2\":%s,\"o\":%s,\"d\":%s,\"tmin\":%s,\"tmax\":%s,%s}\n", i ? "," : "",
                vec(p0).c_str(), vec(p1).c_str(), vec(p2).c_str(), vec(o).c_str(), vec(d).c_str(), num(tmin).c_str(),
                num(tmax).c_str(), hit_json(h, rec, false).c_str());
  }
  std::printf("],\n\"aabb\":[\n");
  for (int i = 0; i < 300; i++) {
    const vec3 a = g.v(-3, 3), b = g.v(-3, 3), o = g.v(-6, 6);
    vec3 d = (0.5 * (a + b) + g.v(-2, 2)) - o;
    if (i % 13 == 5) d = vec3(0, d.y(), d.z());  // axis-parallel rays: 0 / 0 and +-inf slabs
    const double tmin = 0.001, tmax = i % 4 == 1 ? g.in(0.2, 2.0) : infinity;
    const aabb box(a, b);
    const bool h = box.hit(ray(o, d), interval(tmin, tmax));
    std::printf("%s{\"a\":%s,\"b\":%s,\"o\":%s,\"d\":%s,\"tmin\":%s,\"tmax\":%s,\"hit\":%s}\n", i ? "," : "",
                vec(a).c_str(), vec(b).c_str(), vec(o).c_str(), vec(d).c_str(), num(tmin).c_str(), num(tmax).c_str(),
                h ? "true" : "false");
  }
  std::printf("],\n\"world\":[\n");
  for (int w = 0; w < 6; w++) {
    const int n = 5 + 9 * w;
    hittable_list list;
    std::string sp;
    for (int k = 0; k < n; k++) {
      const vec3 c = g.v(-5, 5);
      const double r = g.in(0.2, 1.2);
      list.push_back(std::make_shared<sphere>(c, r, nullptr));
      sp += std::string(k ? "," : "") + "[" + num(c.x()) + "," + num(c.y()) + "," + num(c.z()) + "," + num(r) + "]";
    }
    hittable_list for_bvh = list;
    bvh_node bvh(for_bvh);
    std::printf("%s{\"spheres\":[%s],\"rays\":[\n", w ? "," : "", sp.c_str());
    for (int i = 0; i < 60; i++) {
      const vec3 o = g.v(-9, 9), d = g.v(-5, 5) - o;
      hit_record rl, rb;
      const bool hl = list.hit(ray(o, d), interval(0.001, infinity), rl);
      const bool hb = bvh.hit(ray(o, d), interval(0.001, infinity), rb);
      std::printf("%s{\"o\":%s,\"d\":%s,\"list\":{%s},\"bvh\":{%s}}\n", i ? "," : "", vec(o).c_str(), vec(d).c_str(),
                  hit_json(hl, rl, false).c_str(), hit_json(hb, rb, false).c_str());
    }
    std::printf("]}\n");
  }
  std::printf("],\n\"onb\":[\n");
  for (int i = 0; i < 100; i++) {
    vec3 n = g.v(-2, 2);
    if (i % 10 == 0) n = vec3(g.in(0.95, 1.0) * (i % 20 ? 1 : -1), g.in(-0.1, 0.1), g.in(-0.1, 0.1));  // |y.x| > 0.9
    onb b(n);
    std::printf("%s{\"n\":%s,\"x\":%s,\"y\":%s,\"z\":%s}\n", i ? "," : "", vec(n).c_str(), vec(b.x).c_str(),
                vec(b.y).c_str(), vec(b.z).c_str());
  }
  std::printf("],\n\"refract\":[\n");
  for (int i = 0; i < 100; i++) {
    const vec3 v = unit_vector(g.v(-1, 1)), nn = unit_vector(g.v(-1, 1));
    const vec3 n = dot(v, nn) > 0 ? -nn : nn;
    const double eta = i % 2 ? 1 / 1.5 : g.in(0.3, 2.5);
    std::printf("%s{\"v\":%s,\"n\":%s,\"eta\":%s,\"out\":%s}\n", i ? "," : "", vec(v).c_str(), vec(n).c_str(),
                num(eta).c_str(), vec(refract(v, n, eta)).c_str());
  }
  std::printf("],\n\"pdf\":[\n");
  for (int i = 0; i < 100; i++) {
    const vec3 c = g.v(-3, 3), o = g.v(-8, 8), n = g.v(-1, 1), dir = g.v(-1, 1);
    const double r = g.in(0.1, 2);
    sphere s(c, r, nullptr);
    hemisphere_cosine_pdf cp(n);
    std::printf("%s{\"c\":%s,\"r\":%s,\"o\":%s,\"n\":%s,\"dir\":%s,\"sphere\":%s,\"cosine\":%s}\n", i ? "," : "",
                vec(c).c_str(), num(r).c_str(), vec(o).c_str(), vec(n).c_str(), vec(dir).c_str(),
                num(s.pdf_value(o, dir)).c_str(), num(cp.value(dir)).c_str());
  }
  std::printf("],\n\"draws\":[\n");
  const char* kinds[3] = {"in_unit_sphere", "unit_vec", "cosine_direction"};
  for (int k = 0; k < 3; k++) {
    const unsigned seed = 7u + 1000u * (unsigned)k;
    std::srand(seed);
    std::string vs;
    for (int i = 0; i < 40; i++) {
      const vec3 v = k == 0 ? random_in_unit_sphere() : k == 1 ? random_unit_vec() : random_cosine_direction();
      vs += (i ? "," : "") + vec(v);
    }
    std::printf("%s{\"kind\":\"%s\",\"seed\":%u,\"v\":[%s]}\n", k ? "," : "", kinds[k], seed, vs.c_str());
  }
  std::printf("],\n\"noise\":[\n");
  for (int k = 0; k < 4; k++) {
    const unsigned seed = 11u + 100u * (unsigned)k;
    std::srand(seed);
    const int res = 8;
    perlin pn;  // draws its tables now, as the reference's texture constructors do
    value_noise vn(res);
    worley_noise wn;
    voronoi_noise on;
    const char* kind = k == 0 ? "perlin" : k == 1 ? "value" : k == 2 ? "worley" : "voronoi";
    std::string ps, ns, ts;
    for (int i = 0; i < 60; i++) {
      // value noise indexes its table without wrapping: keep floor(p) + 1 inside [0, res)
      const vec3 p = k == 1 ? g.v(0.0, res - 1.0 - 1e-9) : g.v(-20, 20);
      const double n = k == 0 ? pn.noise(p) : k == 1 ? vn.noise(p) : k == 2 ? wn.noise(p) : on.noise(p);
      ps += (i ? "," : "") + vec(p);
      ns += (i ? "," : "") + num(n);
      if (k == 0) ts += (i ? "," : "") + num(pn.turb(7, p));
    }
    std::printf("%s{\"kind\":\"%s\",\"seed\":%u,\"resolution\":%d,\"p\":[%s],\"noise\":[%s],\"turb\":[%s]}\n",
                k ? "," : "", kind, seed, res, ps.c_str(), ns.c_str(), ts.c_str());
  }
  std::printf("]\n}\n");
  return 0;
}
