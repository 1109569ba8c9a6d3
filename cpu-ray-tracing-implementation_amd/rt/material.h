// material.h -- materials of the plugin surface (reference: src/material.h:36-219).
// Constructors and stored precisions match the reference (fuzz and refraction
// index are float there). Scattering itself runs on the device.
#pragma once
#include <memory>

#include "interval.h"
#include "scene_builder.h"
#include "texture.h"

class material {
 public:
  virtual ~material() = default;
  virtual int flatten(scene_builder&) const { throw unsupported_object("material type not supported on the device"); }

 protected:
  static int emit(scene_builder& sb, int32_t kind, const std::shared_ptr<texture>& tex, float fuzz = 0,
                  float refraction = 1, float smoothness = 0, float specular_prob = 0) {
    rt_material m{};
    m.kind = kind;
    m.texture = sb.add_texture(*tex);
    m.fuzz = fuzz;
    m.refraction = refraction;
    m.smoothness = smoothness;
    m.specular_prob = specular_prob;
    return sb.emit_material(m);
  }
};

inline int scene_builder::add_material(const material& m) {
  auto it = seen_mat_.find(&m);
  if (it != seen_mat_.end()) return it->second;
  int idx = m.flatten(*this);
  seen_mat_[&m] = idx;
  return idx;
}

class lambertian : public material {  // material.h:57-76
 public:
  lambertian(std::shared_ptr<texture> albedo) : tex_(std::move(albedo)) {}
  lambertian(color albedo) : tex_(std::make_shared<solid_color>(albedo)) {}
  int flatten(scene_builder& sb) const override { return emit(sb, RT_MAT_LAMBERTIAN, tex_); }

 private:
  std::shared_ptr<texture> tex_;
};

class metal : public material {  // material.h:78-97
 public:
  metal(std::shared_ptr<texture> albedo, float fuzz = 0.0) : tex_(std::move(albedo)) {
    fuzz_ = (float)interval(0, 1).clamp(fuzz);
  }
  metal(color albedo, float fuzz = 0.0) : tex_(std::make_shared<solid_color>(albedo)) {
    fuzz_ = (float)interval(0, 1).clamp(fuzz);
  }
  int flatten(scene_builder& sb) const override { return emit(sb, RT_MAT_METAL, tex_, fuzz_); }

 private:
  std::shared_ptr<texture> tex_;
  float fuzz_;
};

class dielectric : public material {  // material.h:100-143
 public:
  dielectric(std::shared_ptr<texture> albedo, float refract) : tex_(std::move(albedo)), refract_(refract) {}
  dielectric(float refract) : tex_(std::make_shared<solid_color>(color(1))), refract_(refract) {}
  int flatten(scene_builder& sb) const override { return emit(sb, RT_MAT_DIELECTRIC, tex_, 0, refract_); }

 private:
  std::shared_ptr<texture> tex_;
  float refract_;
};

class gloss : public material {  // material.h:145-185
 public:
  gloss(std::shared_ptr<texture> albedo, float smoothness, float specular_prob) : tex_(std::move(albedo)) {
    smoothness_ = (float)interval(0, 1).clamp(smoothness);
    specular_prob_ = specular_prob;
  }
  gloss(color albedo, float smoothness, float specular_prob)
      : gloss(std::make_shared<solid_color>(albedo), smoothness, specular_prob) {}
  int flatten(scene_builder& sb) const override {
    return emit(sb, RT_MAT_GLOSS, tex_, 0, 1, smoothness_, specular_prob_);
  }

 private:
  std::shared_ptr<texture> tex_;
  float smoothness_, specular_prob_;
};

class isotropic : public material {  // material.h:187-204
 public:
  isotropic(const color& albedo) : tex_(std::make_shared<solid_color>(albedo)) {}
  isotropic(std::shared_ptr<texture> tex) : tex_(std::move(tex)) {}
  int flatten(scene_builder& sb) const override { return emit(sb, RT_MAT_ISOTROPIC, tex_); }

 private:
  std::shared_ptr<texture> tex_;
};

class diffuse_light : public material {  // material.h:206-219
 public:
  diffuse_light(std::shared_ptr<texture> tex) : tex_(std::move(tex)) {}
  diffuse_light(color c) : tex_(std::make_shared<solid_color>(c)) {}
  int flatten(scene_builder& sb) const override { return emit(sb, RT_MAT_DIFFUSE_LIGHT, tex_); }

 private:
  std::shared_ptr<texture> tex_;
};
