// quad.h (reference: src/quad.h:7-112): parallelogram corner + u + v, and box().
#pragma once
#include <cmath>
#include <memory>

#include "hittable_list.h"
#include "material.h"

class quad : public hittable {
 public:
  quad(point3 corner, vec3 u, vec3 v, std::shared_ptr<material> mat)
      : corner_(corner), u_(u), v_(v), mat_(std::move(mat)) {}
  int flatten(scene_builder& sb) const override {
    if (!mat_) throw unsupported_object("quad without a material");
    rt_object o = scene_builder::blank(RT_OBJ_QUAD);
    o.material = sb.add_material(*mat_);
    scene_builder::put3(o.a, corner_);
    scene_builder::put3(o.b, u_);
    scene_builder::put3(o.c, v_);
    return sb.emit_object(o);
  }
  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {  // quad.h:30-64
    double a, b;
    const double t = rt_host::quad_root(corner_, u_, v_, unit_normal(), r, ray_t, a, b);
    if (std::isnan(t)) return false;
    rec.u = a;
    rec.v = b;
    rec.t = t;
    rec.p = r.at(t);
    rec.mat = mat_;
    rec.set_face_normal(r, unit_normal());
    return true;
  }
  aabb get_bounding_box() const override {  // quad.h:19-21: both diagonals
    return aabb::enclose(aabb(corner_, corner_ + u_ + v_), aabb(corner_ + u_, corner_ + v_));
  }
  // quad.h:66-73: solid-angle pdf of a direction that hits the quad from origin, else 0
  double pdf_value(const point3& origin, const vec3& direction) const override {
    hit_record rec;
    if (!hit(ray(origin, direction), interval(0.001, infinity), rec)) return 0;
    const double dist2 = rec.t * rec.t * direction.length_squared();
    return dist2 / (std::fabs(dot(unit_vector(direction), rec.normal)) * cross(u_, v_).length());
  }
  vec3 random(const point3& origin) const override {  // quad.h:75-78, GCC draws v's coefficient first
    const double bv = random_double(), bu = random_double();
    return corner_ + bu * u_ + bv * v_ - origin;
  }

 private:
  point3 corner_;
  vec3 u_, v_;
  std::shared_ptr<material> mat_;
  vec3 unit_normal() const { return unit_vector(cross(u_, v_)); }
};

// The six sides of the box spanned by two opposite corners (quad.h:91-112), same order and orientation.
inline std::shared_ptr<hittable_list> box(const point3& a, const point3& b, std::shared_ptr<material> mat) {
  auto sides = std::make_shared<hittable_list>();
  point3 lo(std::fmin(a.x(), b.x()), std::fmin(a.y(), b.y()), std::fmin(a.z(), b.z()));
  point3 hi(std::fmax(a.x(), b.x()), std::fmax(a.y(), b.y()), std::fmax(a.z(), b.z()));
  vec3 dx(hi.x() - lo.x(), 0, 0), dy(0, hi.y() - lo.y(), 0), dz(0, 0, hi.z() - lo.z());
  sides->push_back(std::make_shared<quad>(point3(lo.x(), lo.y(), hi.z()), dy, dx, mat));   // front
  sides->push_back(std::make_shared<quad>(point3(hi.x(), lo.y(), hi.z()), dy, -dz, mat));  // right
  sides->push_back(std::make_shared<quad>(point3(hi.x(), lo.y(), lo.z()), dy, -dx, mat));  // back
  sides->push_back(std::make_shared<quad>(point3(lo.x(), lo.y(), lo.z()), dy, dz, mat));   // left
  sides->push_back(std::make_shared<quad>(point3(lo.x(), hi.y(), hi.z()), -dz, dx, mat));  // top
  sides->push_back(std::make_shared<quad>(point3(lo.x(), lo.y(), lo.z()), dz, dx, mat));   // bottom
  return sides;
}
