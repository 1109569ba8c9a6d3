// Host-side hittable queries of the plugin surface (rt/host_geometry.h and the classes' hit /
// get_bounding_box / pdf_value / random): known answers and cross-checks, one "name value..."
// line each, checked by tests/test_host_queries.py. Reference semantics: hittable.h:32-41.
#include <cstdio>
#include <cstdlib>

#include "bvh_node.h"
#include "hittable.h"
#include "hittable_list.h"
#include "material.h"
#include "quad.h"
#include "sphere.h"
#include "texture.h"
#include "triangle.h"
#include "volumne.h"

static void print_rec(const char* name, bool h, const hit_record& r) {
  std::printf("%s %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %d %.17g %.17g\n", name, (int)h, r.t, r.p.x(), r.p.y(),
              r.p.z(), r.normal.x(), r.normal.y(), r.normal.z(), (int)r.front_face, r.u, r.v);
}

int main() {
  auto grey = std::make_shared<lambertian>(color(0.5, 0.5, 0.5));
  const interval fwd(0.001, infinity);
  hit_record rec;

  // sphere: (0,0,-2) r 0.5 from the origin straight ahead: t 1.5, normal +z, front face
  sphere s(point3(0, 0, -2), 0.5, grey);
  print_rec("sphere", s.hit(ray(point3(0), vec3(0, 0, -1)), fwd, rec), rec);
  // from inside: the far root, back face
  print_rec("sphere_inside", s.hit(ray(point3(0, 0, -2), vec3(0, 0, -1)), fwd, rec), rec);
  print_rec("sphere_miss", s.hit(ray(point3(0), vec3(0, 1, 0)), fwd, rec), hit_record());
  // moving sphere at time 0.5: centre (0,0,-2) -> (0,1,-2) is at y 0.5; normal from center_ = 0
  sphere mv(point3(0, 0, -2), point3(0, 1, -2), 0.5, grey);
  print_rec("moving", mv.hit(ray(point3(0, 0.5, 0), vec3(0, 0, -1), 0.5), fwd, rec), rec);

  // quad: unit square at z = -3, hit at its centre; alpha, beta = 0.5
  quad q(point3(-0.5, -0.5, -3), vec3(1, 0, 0), vec3(0, 1, 0), grey);
  print_rec("quad", q.hit(ray(point3(0), vec3(0, 0, -1)), fwd, rec), rec);
  print_rec("quad_edge", q.hit(ray(point3(0.5, 0.5, 0), vec3(0, 0, -1)), fwd, rec), rec);  // closed interior
  // pdf of the direction straight at it from the origin: t^2 |d|^2 / (cos * area) = 9 / 1
  std::printf("quad_pdf %.17g %.17g\n", q.pdf_value(point3(0), vec3(0, 0, -1)), q.pdf_value(point3(0), vec3(0, 1, 0)));
  std::srand(3);
  const vec3 dq = q.random(point3(0));
  std::printf("quad_random %.17g %.17g %.17g\n", dq.x(), dq.y(), dq.z());

  // triangle: hit inside, miss outside, u/v left as they were
  triangle tr(point3(-1, -1, -4), point3(1, -1, -4), point3(0, 1, -4), grey);
  hit_record tr_rec;
  tr_rec.u = 7;
  tr_rec.v = 9;
  print_rec("triangle", tr.hit(ray(point3(0), vec3(0, 0, -1)), fwd, tr_rec), tr_rec);
  print_rec("triangle_miss", tr.hit(ray(point3(0), vec3(0.9, 0.9, -1)), fwd, rec), hit_record());

  // rotate_y(90) of a quad facing +z: it faces +x afterwards; translate moves the hit point
  auto facing = std::make_shared<quad>(point3(-0.5, -0.5, 0), vec3(1, 0, 0), vec3(0, 1, 0), grey);
  rotate_y ry(facing, 90);
  print_rec("rotate_y", ry.hit(ray(point3(3, 0, 0), vec3(-1, 0, 0)), fwd, rec), rec);
  translate tl(vec3(0, 0, -5), facing);
  print_rec("translate", tl.hit(ray(point3(0.25, 0.25, 0), vec3(0, 0, -1)), fwd, rec), rec);
  const aabb rb = ry.get_bounding_box();
  std::printf("rotate_box %.17g %.17g %.17g %.17g\n", rb.axis_interval(0).min, rb.axis_interval(0).max,
              rb.axis_interval(2).min, rb.axis_interval(2).max);

  // list vs bvh_node on random primitives and rays: the same closest hit (the reference's tree)
  std::srand(11);
  hittable_list world;
  for (int i = 0; i < 60; i++) {
    const point3 c(random_double(-5, 5), random_double(-5, 5), random_double(-15, -5));
    const int kind = i % 3;
    if (kind == 0)
      world.push_back(std::make_shared<sphere>(c, random_double(0.2, 1.0), grey));
    else if (kind == 1)
      world.push_back(std::make_shared<quad>(c, vec3(random_double(0.5, 2), 0, 0.3), vec3(0.2, random_double(0.5, 2), 0), grey));
    else
      world.push_back(std::make_shared<triangle>(c, c + vec3(1.5, 0.2, 0), c + vec3(0.3, 1.4, 0.5), grey));
  }
  bvh_node tree(world);
  int agree = 0, hits = 0, n = 2000;
  for (int k = 0; k < n; k++) {
    const vec3 d(random_double(-0.5, 0.5), random_double(-0.5, 0.5), -1);
    hit_record a, b;
    const bool ha = world.hit(ray(point3(0), d), fwd, a), hb = tree.hit(ray(point3(0), d), fwd, b);
    hits += ha;
    agree += (ha == hb) && (!ha || (a.t == b.t && a.p.x() == b.p.x() && a.normal.z() == b.normal.z()));
  }
  std::printf("bvh_vs_list %d %d %d\n", agree, hits, n);
  const aabb wb = world.get_bounding_box(), tb = tree.get_bounding_box();
  std::printf("boxes_equal %d\n", (int)(wb.axis_interval(0).min == tb.axis_interval(0).min &&
                                         wb.axis_interval(2).max == tb.axis_interval(2).max));

  // volume: a unit box of density 1e9 is hit right at its entry; density 1e-9 never
  auto box1 = box(point3(-1, -1, -6), point3(1, 1, -4), grey);
  volumne thick(box1, 1e9, std::make_shared<solid_color>(color(1, 1, 1)));
  volumne thin(box1, 1e-9, std::make_shared<solid_color>(color(1, 1, 1)));
  std::srand(5);
  print_rec("volume_thick", thick.hit(ray(point3(0), vec3(0, 0, -1)), fwd, rec), rec);
  print_rec("volume_thin", thin.hit(ray(point3(0), vec3(0, 0, -1)), fwd, rec), hit_record());
  return 0;
}
