// scene_builder.h -- serialises the plugin-surface objects (hittables,
// materials, textures) into the POD rt_scene_desc of include/rt_hip.h.
// Shared objects (the same shared_ptr used twice, e.g. the light quad that is
// also in the world) map to one descriptor entry.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/rt_hip.h"
#include "vec3.h"

class hittable;
class material;
class texture;

class unsupported_object : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class scene_builder {
 public:
  int add(const hittable& h);  // defined in hittable.h
  int add_material(const material& m);
  int add_texture(const texture& t);

  // low-level emitters used by the classes' flatten()
  int emit_object(const rt_object& o) {
    objects_.push_back(o);
    return (int)objects_.size() - 1;
  }
  rt_object& object(int i) { return objects_[(size_t)i]; }
  int emit_children(const std::vector<int>& kids) {
    int first = (int)children_.size();
    children_.insert(children_.end(), kids.begin(), kids.end());
    return first;
  }
  int emit_material(const rt_material& m) {
    materials_.push_back(m);
    return (int)materials_.size() - 1;
  }
  int emit_texture(const rt_texture& t) {
    textures_.push_back(t);
    return (int)textures_.size() - 1;
  }
  // picture-texture pixels; returns their byte offset for rt_texture.data
  int32_t emit_image_data(const std::vector<uint8_t>& v) {
    const int32_t off = (int32_t)image_data_.size();
    image_data_.insert(image_data_.end(), v.begin(), v.end());
    return off;
  }
  // procedural-texture tables; returns their offset for rt_texture.data
  int32_t emit_tex_data(const std::vector<double>& v) {
    const int32_t off = (int32_t)tex_data_.size();
    tex_data_.insert(tex_data_.end(), v.begin(), v.end());
    return off;
  }

  rt_scene_desc desc(int world, int light, int background) const {
    rt_scene_desc d{};
    d.objects = objects_.data();
    d.num_objects = (int32_t)objects_.size();
    d.children = children_.data();
    d.num_children = (int32_t)children_.size();
    d.materials = materials_.data();
    d.num_materials = (int32_t)materials_.size();
    d.textures = textures_.data();
    d.num_textures = (int32_t)textures_.size();
    d.world = world;
    d.light = light;
    d.background = background;
    d.tex_data = tex_data_.empty() ? nullptr : tex_data_.data();
    d.num_tex_data = (int64_t)tex_data_.size();
    d.image_data = image_data_.empty() ? nullptr : image_data_.data();
    d.num_image_data = (int64_t)image_data_.size();
    return d;
  }

  static void put3(double* dst, const vec3& v) {
    dst[0] = v.x();
    dst[1] = v.y();
    dst[2] = v.z();
  }
  static rt_object blank(int32_t kind) {
    rt_object o{};
    o.kind = kind;
    o.material = -1;
    o.child = -1;
    return o;
  }

 private:
  std::vector<rt_object> objects_;
  std::vector<int32_t> children_;
  std::vector<rt_material> materials_;
  std::vector<rt_texture> textures_;
  std::vector<double> tex_data_;
  std::vector<uint8_t> image_data_;
  std::unordered_map<const void*, int> seen_obj_, seen_mat_, seen_tex_;
};
