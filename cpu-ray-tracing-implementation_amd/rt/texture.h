// texture.h -- textures of the plugin surface (reference: src/texture.h:6-119).
// solid_color, checker_texture and the procedural noise textures run on the device; a texture
// subclass the device does not know makes camera::render fail with unsupported_object.
#pragma once
#include <memory>

#include "color.h"
#include "image.h"
#include "noise.h"
#include "ray.h"
#include "scene_builder.h"

class texture {
 public:
  virtual ~texture() = default;
  virtual color sample(double u, double v, point3 p) = 0;
  // serialise into the descriptor; returns the texture index
  virtual int flatten(scene_builder&) const { throw unsupported_object("texture type not supported on the device"); }
};

inline int scene_builder::add_texture(const texture& t) {
  auto it = seen_tex_.find(&t);
  if (it != seen_tex_.end()) return it->second;
  int idx = t.flatten(*this);
  seen_tex_[&t] = idx;
  return idx;
}

class solid_color : public texture {
 public:
  solid_color(color c) : color_(c) {}
  color sample(double, double, point3) override { return color_; }
  int flatten(scene_builder& sb) const override {
    rt_texture t{};
    t.kind = RT_TEX_SOLID;
    scene_builder::put3(t.color, color_);
    return sb.emit_texture(t);
  }
  static std::shared_ptr<solid_color> black, white, red, green, blue, yellow, cyan, magenta;

 private:
  color color_;
};
inline std::shared_ptr<solid_color> solid_color::black = std::make_shared<solid_color>(color(0, 0, 0));
inline std::shared_ptr<solid_color> solid_color::white = std::make_shared<solid_color>(color(1, 1, 1));
inline std::shared_ptr<solid_color> solid_color::red = std::make_shared<solid_color>(color(1, 0, 0));
inline std::shared_ptr<solid_color> solid_color::green = std::make_shared<solid_color>(color(0, 1, 0));
inline std::shared_ptr<solid_color> solid_color::blue = std::make_shared<solid_color>(color(0, 0, 1));
inline std::shared_ptr<solid_color> solid_color::yellow = std::make_shared<solid_color>(color(1, 1, 0));
inline std::shared_ptr<solid_color> solid_color::cyan = std::make_shared<solid_color>(color(0, 1, 1));
inline std::shared_ptr<solid_color> solid_color::magenta = std::make_shared<solid_color>(color(1, 0, 1));

// 3D checker over floor(p / scale) (texture.h:39-63)
class checker_texture : public texture {
 public:
  checker_texture(color odd, color even, double scale) : odd_(odd), even_(even), scale_(scale) {}
  color sample(double, double, point3 p) override {
    point3 q = p / scale_;
    int total = int(std::floor(q.x())) + int(std::floor(q.y())) + int(std::floor(q.z()));
    return total % 2 == 0 ? even_ : odd_;
  }
  int flatten(scene_builder& sb) const override {
    rt_texture t{};
    t.kind = RT_TEX_CHECKER;
    scene_builder::put3(t.odd, odd_);
    scene_builder::put3(t.even, even_);
    t.scale = scale_;
    return sb.emit_texture(t);
  }

 private:
  color odd_, even_;
  double scale_;
};

// 0.5 (1 + sin(p.x + 70 turb(7, p / scale))) in every channel (texture.h:80-92)
class perlin_texture : public texture {
 public:
  explicit perlin_texture(double scale) : scale_(scale) {}
  color sample(double, double, point3 p) override {
    return color(.5, .5, .5) * (1 + std::sin((p.x() + 70 * noise_.turb(7, p / scale_))));
  }
  int flatten(scene_builder& sb) const override {
    rt_texture t{};
    t.kind = RT_TEX_PERLIN;
    t.scale = scale_;
    t.data = sb.emit_tex_data(noise_.tables());
    return sb.emit_texture(t);
  }

 private:
  perlin noise_;
  double scale_;
};

class value_texture : public texture {  // texture.h:95-103
 public:
  explicit value_texture(int resolution) : noise_(resolution) {}
  color sample(double, double, point3 p) override { return color(noise_.noise(p)); }
  int flatten(scene_builder& sb) const override {
    rt_texture t{};
    t.kind = RT_TEX_VALUE;
    t.scale = noise_.resolution();
    t.data = sb.emit_tex_data(noise_.tables());
    return sb.emit_texture(t);
  }

 private:
  value_noise noise_;
};

class worley_texture : public texture {  // texture.h:105-111
 public:
  color sample(double, double, point3 p) override { return color(noise_.noise(p)); }
  int flatten(scene_builder& sb) const override {
    rt_texture t{};
    t.kind = RT_TEX_WORLEY;
    return sb.emit_texture(t);
  }

 private:
  worley_noise noise_;
};

class voronoi_texture : public texture {  // texture.h:113-119
 public:
  color sample(double, double, point3 p) override { return color(noise_.noise(p)); }
  int flatten(scene_builder& sb) const override {
    rt_texture t{};
    t.kind = RT_TEX_VORONOI;
    return sb.emit_texture(t);
  }

 private:
  voronoi_noise noise_;
};

// image colours at (u, v) (texture.h:65-78); u, v from the hit (sphere.h:90-95, quad.h:58-64)
class picture_texture : public texture {
 public:
  explicit picture_texture(std::shared_ptr<image> img) : image_(std::move(img)) {}
  color sample(double u, double v, point3) override {
    int i = image_->width() * u;
    int j = image_->height() * (1 - v);
    const unsigned char* px = image_->pixel_data(i, j);
    const double color_scale = 1 / 256.0;
    return color(px[0] * color_scale, px[1] * color_scale, px[2] * color_scale);
  }
  int flatten(scene_builder& sb) const override {
    rt_texture t{};
    t.kind = RT_TEX_IMAGE;
    t.color[0] = image_->width();
    t.color[1] = image_->height();
    if (image_->width() > 0) t.data = sb.emit_image_data(image_->bytes());
    return sb.emit_texture(t);
  }

 private:
  std::shared_ptr<image> image_;
};
