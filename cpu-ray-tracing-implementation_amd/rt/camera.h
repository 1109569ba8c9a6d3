// camera.h -- the drop-in camera (reference: src/camera.h:18-330).
//
// Same initializers, public fields and render() signature as the reference.
// render() serialises the world (and the importance-sampling light) through the
// hittables' flatten(), renders it on an MI355X through the C ABI of
// include/rt_hip.h (librt_hip.so: the wavefront HIP path tracer), fills image_
// with the per-pixel mean (camera.h:169-170) and writes the same P3 text
// (camera.h:149-151,174). Random numbers come from the device's counter RNG
// keyed by (seed_, pixel, sample) instead of the global std::rand stream, so
// the image is independent of scheduling and of how many GPUs render it.
#pragma once
#include <cmath>
#include <cstdint>
#include <fstream>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"
#include "color.h"
#include "hittable.h"
#include "material.h"
#include "texture.h"
#include "utility.h"

enum camera_mode { kPerspective, kOrthnormal, kFisheye, kLens };

class camera {
 public:
  void initialize_perspective(int image_width, double aspect_ratio, point3 pos, vec3 lookat, float focal_length = 1,
                              float fovy_degree = 90, int sample_per_pixel = 100, int max_recur_depth = 5) {
    mode_ = kPerspective;
    frame(image_width, aspect_ratio, pos, lookat, sample_per_pixel, max_recur_depth);
    fovy_degree_ = fovy_degree;
    focal_length_ = focal_length;
    float theta = (float)degrees_to_radians(fovy_degree_);  // float, as camera.h:45
    viewport_height_ = 2.0 * std::tan(theta / 2.0) * focal_length_;
    viewport_width_ = viewport_height_ * (double(image_width_) / image_height_);
  }
  void initialize_orthnormal(int image_width, double aspect_ratio, double viewport_height, point3 pos, vec3 lookat,
                             int sample_per_pixel = 100, int max_recur_depth = 5) {
    mode_ = kOrthnormal;
    frame(image_width, aspect_ratio, pos, lookat, sample_per_pixel, max_recur_depth);
    viewport_height_ = viewport_height;
    viewport_width_ = viewport_height * (double(image_width_) / image_height_);
  }
  void initialize_fisheye(int image_width, double aspect_ratio, point3 pos, vec3 lookat, float focal_length = 1,
                          float fovy_degree = 90, int sample_per_pixel = 100, int max_recur_depth = 5) {
    initialize_perspective(image_width, aspect_ratio, pos, lookat, focal_length, fovy_degree, sample_per_pixel,
                           max_recur_depth);
    mode_ = kFisheye;
  }
  void initialize_lens(int image_width, float aspect_ratio, point3 pos, vec3 lookat, float defocus_angle,
                       float focus_dist = 1, float fovy_degree = 90, int sample_per_pixel = 100,
                       int max_recur_depth = 5) {
    mode_ = kLens;
    frame(image_width, aspect_ratio, pos, lookat, sample_per_pixel, max_recur_depth);
    // camera.h:114: aspect_ratio is a float parameter here, so int / float divides in float
    image_height_ = int(image_width / aspect_ratio);
    image_height_ = image_height_ < 1 ? 1 : image_height_;
    image_.assign((size_t)image_width_ * image_height_, color(0));
    fovy_degree_ = fovy_degree;
    focus_dist_ = focus_dist;
    float theta = (float)degrees_to_radians(fovy_degree_);
    viewport_height_ = 2.0 * std::tan(theta / 2.0) * focus_dist_;
    viewport_width_ = viewport_height_ * (double(image_width_) / image_height_);
    double r = focus_dist * std::tan(degrees_to_radians(defocus_angle / 2));
    defocus_disk_u = right_ * r;
    defocus_disk_v = up_ * r;
  }

  // camera.h:135 -- if light is not null it is importance-sampled (a 50/50 mixture with the material pdf).
  void render(std::ofstream& out, const hittable& world, const std::shared_ptr<const hittable> light = nullptr) {
    std::cout << "Start to render...\n";
    if (!out) {
      std::cerr << "Fail to open file.\n";
      return;
    }
    out << "P3\n" << image_width_ << ' ' << image_height_ << '\n' << 255 << '\n';
    if (!render_image(world, light)) {
      std::cerr << "render failed: " << last_error_ << '\n';
      return;
    }
    for (const color& c : image_) write_color(out, c);
    std::cout << "Done.\n";
  }

  // Renders into image_ without writing a file. Returns false (reason in last_error_) on failure.
  bool render_image(const hittable& world, const std::shared_ptr<const hittable>& light = nullptr) {
    last_error_.clear();
    scene_builder sb;
    int w, l = -1, bg = -1;
    try {
      w = sb.add(world);
      if (light) l = sb.add(*light);
      if (background_) bg = sb.add_texture(*background_);
    } catch (const unsupported_object& e) {
      return fail(e.what());
    }
    rt_scene_desc desc = sb.desc(w, l, bg);
    rt_camera_desc cam = describe();
    rt_render_params p{};
    p.spp = samples_per_pixel_;
    p.max_depth = max_recur_depth_;
    p.seed = seed_;
    p.precision = precision_;
    const size_t n = (size_t)image_width_ * image_height_;
    std::vector<double> px64;
    std::vector<float> px32;
    void* out = nullptr;
    if (precision_ == RT_PREC_F64) {
      px64.resize(3 * n);
      out = px64.data();
    } else {
      px32.resize(3 * n);
      out = px32.data();
    }
    if (!devices_.empty()) {  // the image tiled over several GPUs, one RCCL gather (rt_multi_*)
      if (!h_.multi || h_.multi_devs != devices_) {  // kept across renders on the same devices
        h_.multi.reset();
        rt_multi* mg = nullptr;
        if (rt_multi_create(devices_.data(), (int32_t)devices_.size(), &mg) != RT_OK)
          return fail(rt_multi_last_error(nullptr));
        h_.multi.reset(mg, rt_multi_destroy);
        h_.multi_devs = devices_;
      }
      rt_status s = rt_multi_scene_upload(h_.multi.get(), &desc);
      if (s == RT_OK) s = rt_multi_render(h_.multi.get(), &cam, &p, tile_size_, out);
      if (s != RT_OK) {
        std::string m = rt_multi_last_error(h_.multi.get());
        h_.multi.reset();
        return fail(m);
      }
    } else {
      if (!h_.ctx || h_.ctx_dev != device_) {  // kept across renders on the same device
        h_.ctx.reset();
        rt_context* c = nullptr;
        if (rt_context_create(device_, &c) != RT_OK) return fail(rt_last_error(nullptr));
        h_.ctx.reset(c, rt_context_destroy);
        h_.ctx_dev = device_;
      }
      rt_tile tile{0, 0, image_width_, image_height_};
      rt_status s = rt_scene_upload(h_.ctx.get(), &desc);
      if (s == RT_OK) s = rt_render_tiles(h_.ctx.get(), &cam, &p, &tile, 1, out, 0, nullptr);
      if (s != RT_OK) {
        std::string m = rt_last_error(h_.ctx.get());
        h_.ctx.reset();
        return fail(m);
      }
    }
    image_.resize(n);
    for (size_t i = 0; i < n; i++)
      image_[i] = precision_ == RT_PREC_F64 ? color(px64[3 * i], px64[3 * i + 1], px64[3 * i + 2])
                                            : color(px32[3 * i], px32[3 * i + 1], px32[3 * i + 2]);
    return true;
  }

  // image_ as a Portable Float Map (linear, lossless; little-endian, bottom row first).
  bool write_pfm(const std::string& path) const {
    std::ofstream f(path, std::ios::binary);
    if (!f) return false;
    f << "PF\n" << image_width_ << ' ' << image_height_ << "\n-1.0\n";
    for (int y = image_height_ - 1; y >= 0; y--)
      for (int x = 0; x < image_width_; x++) {
        const color& c = image_[(size_t)y * image_width_ + x];
        const float v[3] = {(float)c.x(), (float)c.y(), (float)c.z()};
        f.write(reinterpret_cast<const char*>(v), sizeof v);
      }
    return bool(f);
  }

  // The camera as the C ABI sees it (the values initialize_* computed).
  rt_camera_desc describe() const {
    rt_camera_desc c{};
    c.mode = mode_;
    c.image_width = image_width_;
    c.image_height = image_height_;
    scene_builder::put3(c.pos, pos_);
    scene_builder::put3(c.dir, dir_);
    scene_builder::put3(c.right, right_);
    scene_builder::put3(c.up, up_);
    c.viewport_width = viewport_width_;
    c.viewport_height = viewport_height_;
    c.focal_length = focal_length_;
    c.focus_dist = focus_dist_;
    scene_builder::put3(c.defocus_u, defocus_disk_u);
    scene_builder::put3(c.defocus_v, defocus_disk_v);
    return c;
  }

 public:
  camera_mode mode_ = kPerspective;
  double aspect_ratio_ = 1;
  int image_width_ = 1;
  int image_height_ = 1;
  float fovy_degree_ = 90;
  int max_recur_depth_ = 10;
  int samples_per_pixel_ = 1;
  double viewport_height_ = 0;
  double viewport_width_ = 0;
  double focal_length_ = 1;
  double focus_dist_ = 3.4;
  double defocus_angle_ = 10.0;
  vec3 defocus_disk_u, defocus_disk_v;
  point3 pos_;
  vec3 dir_, world_up_, up_, right_;
  std::vector<color> image_;
  std::shared_ptr<texture> background_;
  // device-path settings (not in the reference)
  int device_ = 0;                      // HIP device
  // non-empty: render on these devices, tiles of tile_size_ dealt round-robin and gathered over RCCL
  // to devices_[0] (rt_multi_*; replaces camera.h:154-172's per-row par_unseq)
  std::vector<int32_t> devices_;
  int tile_size_ = 16;
  rt_precision precision_ = RT_PREC_F32;  // RT_PREC_F64: the fp64 parity path
  uint64_t seed_ = 1;                   // counter-RNG key
  std::string last_error_;

 private:
  void frame(int image_width, double aspect, point3 pos, vec3 lookat, int spp, int depth) {  // camera.h:23-39
    pos_ = pos;
    world_up_ = vec3(0, 1, 0);
    dir_ = unit_vector(lookat - pos);
    right_ = unit_vector(cross(dir_, world_up_));
    up_ = cross(right_, dir_);
    aspect_ratio_ = aspect;
    image_width_ = image_width;
    image_height_ = int(image_width / aspect);
    image_height_ = image_height_ < 1 ? 1 : image_height_;
    samples_per_pixel_ = spp;
    max_recur_depth_ = depth;
    image_.assign((size_t)image_width_ * image_height_, color(0));
  }
  bool fail(const std::string& m) {
    last_error_ = m;
    return false;
  }
  // The device handles of the last render, reused while devices_ / device_ stay the same: a context
  // per device and, for devices_, one RCCL communicator -- created once, not once per render().
  // They belong to this camera: a copy starts without them (and copy assignment keeps the target's
  // own), so two cameras never share a context's buffers and stream, and copies may render from
  // different threads as before. One camera must still not render from two threads at once.
  struct handles {
    std::shared_ptr<rt_multi> multi;
    std::vector<int32_t> multi_devs;
    std::shared_ptr<rt_context> ctx;
    int ctx_dev = -1;
    handles() = default;
    handles(const handles&) {}
    handles& operator=(const handles&) { return *this; }
    handles(handles&&) = default;
    handles& operator=(handles&&) = default;
  } h_;
};
