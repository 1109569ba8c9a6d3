// image.h -- image loading for picture_texture (reference: src/image.h:9-117).
//
// The reference decodes files with stb_image (stbi_loadf: 8-bit formats come back linear, as
// powf(byte / 255, 2.2)) or tinyexr, then stores bytes with float_to_byte (<= 0 -> 0, >= 1 -> 255,
// else int(256 v)). Here: our own decoders, each pinned byte for byte against the reference's stb_image
// -- baseline JPEG (rt/jpeg.h, incl. the reference's earthmap.jpg), PNG (rt/png.h: all colour types,
// bit depths and Adam7) and Radiance HDR (rt/hdr.h, linear floats as stbi_loadf returns them) -- plus
// binary/ASCII PPM (P6/P3, 8-bit) and PFM (linear floats). EXR (tinyexr, not vendored in the reference)
// and progressive JPEG are not decoded; other hosts decode elsewhere and pass linear floats to
// image(width, height, pixels). As in the reference, a file that cannot be loaded prints an error and
// leaves a 0 x 0 image, which picture_texture samples as magenta.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <iostream>
#include <iterator>
#include <string>
#include <vector>

#include "hdr.h"
#include "jpeg.h"
#include "png.h"

class image {
 public:
  image() = default;
  explicit image(const char* filename) {
    if (!load(filename)) std::cerr << "ERROR: Could not load image file '" << filename << "'.\n";
  }
  // linear RGB floats, row 0 at the top
  image(int width, int height, const std::vector<float>& linear_rgb) { set(width, height, linear_rgb); }

  int width() const { return bytes_.empty() ? 0 : w_; }
  int height() const { return bytes_.empty() ? 0 : h_; }
  const std::vector<uint8_t>& bytes() const { return bytes_; }

  // image.h:71-82: the RGB bytes at (x, y), clamped into the image; magenta without data
  const unsigned char* pixel_data(int x, int y) const {
    static unsigned char magenta[] = {255, 0, 255};
    if (bytes_.empty()) return magenta;
    x = x < 0 ? 0 : (x < w_ ? x : w_ - 1);
    y = y < 0 ? 0 : (y < h_ ? y : h_ - 1);
    return bytes_.data() + 3 * ((size_t)y * w_ + x);
  }

  static unsigned char float_to_byte(float v) {  // image.h:97-101
    if (v <= 0.0) return 0;
    if (1.0 <= v) return 255;
    return static_cast<unsigned char>(256.0 * v);
  }

 private:
  int w_ = 0, h_ = 0;
  std::vector<uint8_t> bytes_;

  void set(int w, int h, const std::vector<float>& f) {
    if (w <= 0 || h <= 0 || f.size() < (size_t)w * h * 3) return;
    w_ = w;
    h_ = h;
    bytes_.resize((size_t)w * h * 3);
    for (size_t i = 0; i < bytes_.size(); i++) bytes_[i] = float_to_byte(f[i]);
  }
  static bool token(std::istream& in, std::string& t) {  // PNM header token, skipping # comments
    t.clear();
    int c;
    while ((c = in.get()) != EOF) {
      if (c == '#') {
        while ((c = in.get()) != EOF && c != '\n') {
        }
        continue;
      }
      if (std::isspace(c)) {
        if (!t.empty()) return true;
        continue;
      }
      t += (char)c;
    }
    return !t.empty();
  }
  // stbi__ldr_to_hdr: powf(byte / 255.0f, 2.2f), float all the way
  static float ldr_to_linear(int v) { return (float)std::pow((float)v / 255.0f, 2.2f); }
  bool load(const std::string& path) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return false;
    if (in.peek() == 0x89 || in.peek() == '#') {  // PNG signature / Radiance "#?RADIANCE"
      std::vector<uint8_t> file((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
      std::string err;
      if (rt_png::is_png(file)) {
        rt_png::Image im;
        if (!rt_png::decode(file, im, &err)) {
          std::cerr << err << "\n";
          return false;
        }
        std::vector<float> f(im.rgb.size());
        for (size_t i = 0; i < f.size(); i++) f[i] = ldr_to_linear(im.rgb[i]);
        set(im.width, im.height, f);
        return !bytes_.empty();
      }
      if (rt_hdr::is_hdr(file)) {
        rt_hdr::Image im;
        if (!rt_hdr::decode(file, im, &err)) {
          std::cerr << err << "\n";
          return false;
        }
        set(im.width, im.height, im.rgb);
        return !bytes_.empty();
      }
      return false;
    }
    if (in.peek() == 0xFF) {  // JPEG (SOI = FF D8)
      std::vector<uint8_t> file((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
      rt_jpeg::Image im;
      std::string err;
      if (!rt_jpeg::decode(file, im, &err)) {
        std::cerr << "JPEG: " << err << "\n";
        return false;
      }
      std::vector<float> f(im.rgb.size());
      for (size_t i = 0; i < f.size(); i++) f[i] = ldr_to_linear(im.rgb[i]);
      set(im.width, im.height, f);
      return !bytes_.empty();
    }
    std::string magic, sw, sh, smax;
    if (!token(in, magic)) return false;
    if (magic == "PF") {  // PFM: linear floats, rows bottom to top, the scale's sign is the byte order
      if (!token(in, sw) || !token(in, sh) || !token(in, smax)) return false;
      const int w = std::stoi(sw), h = std::stoi(sh);
      const bool little = std::stod(smax) < 0;
      std::vector<float> raw((size_t)w * h * 3), f(raw.size());
      if (!in.read(reinterpret_cast<char*>(raw.data()), (std::streamsize)(raw.size() * 4))) return false;
      for (float& x : raw) {
        uint32_t b;
        std::memcpy(&b, &x, 4);
        if (!little) b = __builtin_bswap32(b);
        std::memcpy(&x, &b, 4);
      }
      for (int y = 0; y < h; y++) std::memcpy(&f[(size_t)y * w * 3], &raw[(size_t)(h - 1 - y) * w * 3], (size_t)w * 12);
      set(w, h, f);
      return !bytes_.empty();
    }
    if (magic != "P6" && magic != "P3") return false;
    if (!token(in, sw) || !token(in, sh) || !token(in, smax)) return false;
    const int w = std::stoi(sw), h = std::stoi(sh), maxv = std::stoi(smax);
    if (w <= 0 || h <= 0 || maxv <= 0 || maxv > 255) return false;
    std::vector<float> f((size_t)w * h * 3);
    for (size_t i = 0; i < f.size(); i++) {
      int v;
      if (magic == "P6") {
        v = in.get();
        if (v == EOF) return false;
      } else {
        std::string t;
        if (!token(in, t)) return false;
        v = std::stoi(t);
      }
      f[i] = maxv == 255 ? ldr_to_linear(v) : (float)std::pow((float)v / (float)maxv, 2.2f);
    }
    set(w, h, f);
    return !bytes_.empty();
  }
};
