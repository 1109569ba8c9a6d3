// hdr.h -- Radiance RGBE (.hdr) decoding for picture textures (reference: src/image.h:33-50, stbi_loadf).
//
// Our own reader of the format the reference's stb_image accepts: a "#?RADIANCE" / "#?RGBE" header whose
// lines include FORMAT=32-bit_rle_rgbe, ended by an empty line, then "-Y <h> +X <w>" and the scanlines,
// run-length encoded per component (new-style RLE, widths 8..32767) or flat RGBE quadruples. A pixel is
// (r, g, b) * 2^(e - 136) in float, 0 when e = 0 (stbi__hdr_convert) -- linear, no gamma, as stbi_loadf
// returns it. stb's quirks are kept: a scanline that does not start with the RLE marker switches the rest
// of the file to flat pixels, restarting at pixel 1 of row 0 (its `goto main_decode_loop`), and reads past
// the end return zeros. Pinned against the reference's stb_image (tests/test_png_hdr.py).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace rt_hdr {

struct Image {
  int width = 0, height = 0;
  std::vector<float> rgb;  // linear floats, row 0 at the top
};

inline bool is_hdr(const std::vector<uint8_t>& d) {
  auto starts = [&](const char* s) {
    const size_t n = std::strlen(s);
    return d.size() >= n && std::memcmp(d.data(), s, n) == 0;
  };
  return starts("#?RADIANCE\n") || starts("#?RGBE\n");
}

inline bool decode(const std::vector<uint8_t>& d, Image& im, std::string* err) {
  auto fail = [&](const char* m) {
    if (err) *err = m;
    return false;
  };
  size_t p = 0;
  auto get8 = [&]() -> int { return p < d.size() ? d[p++] : 0; };
  auto line = [&]() {  // stbi__hdr_gettoken: up to the newline (at most 1023 characters kept)
    std::string t;
    while (p < d.size()) {
      const char c = (char)d[p++];
      if (c == '\n') break;
      if (t.size() < 1023) t += c;
    }
    return t;
  };
  const std::string id = line();
  if (id != "#?RADIANCE" && id != "#?RGBE") return fail("HDR: not a Radiance file");
  bool valid = false;
  for (;;) {
    const std::string t = line();
    if (t.empty()) break;
    if (t == "FORMAT=32-bit_rle_rgbe") valid = true;
  }
  if (!valid) return fail("HDR: unsupported format");
  const std::string res = line();
  if (res.compare(0, 3, "-Y ") != 0) return fail("HDR: unsupported data layout");
  const char* s = res.c_str() + 3;
  char* e = nullptr;
  const long h = std::strtol(s, &e, 10);
  s = e;
  while (*s == ' ') ++s;
  if (std::strncmp(s, "+X ", 3) != 0) return fail("HDR: unsupported data layout");
  const long w = std::strtol(s + 3, nullptr, 10);
  if (w <= 0 || h <= 0 || w > (1 << 24) || h > (1 << 24)) return fail("HDR: bad size");
  // stbi__mad4sizes_valid(w, h, 3, sizeof(float)): refused before anything is allocated
  if ((uint64_t)w * (uint64_t)h * 3u * sizeof(float) > 0x7FFFFFFFull) return fail("HDR: image too large");
  im.width = (int)w;
  im.height = (int)h;
  im.rgb.assign((size_t)w * h * 3, 0.0f);
  auto convert = [&](size_t px, const uint8_t* q) {  // stbi__hdr_convert, req_comp = 3
    float* o = &im.rgb[3 * px];
    if (q[3] != 0) {
      const float f1 = (float)std::ldexp(1.0f, q[3] - (int)(128 + 8));
      o[0] = q[0] * f1;
      o[1] = q[1] * f1;
      o[2] = q[2] * f1;
    } else {
      o[0] = o[1] = o[2] = 0.0f;
    }
  };
  auto flat_from = [&](size_t px) {
    for (; px < (size_t)w * h; px++) {
      uint8_t q[4];
      for (int k = 0; k < 4; k++) q[k] = (uint8_t)get8();
      convert(px, q);
    }
    return true;
  };
  if (w < 8 || w >= 32768) return flat_from(0);
  std::vector<uint8_t> sl((size_t)w * 4);
  for (long j = 0; j < h; j++) {
    const int c1 = get8(), c2 = get8();
    int len = get8();
    if (c1 != 2 || c2 != 2 || (len & 0x80)) {  // not run-length encoded: flat from here, at pixel 1 of row 0
      const uint8_t q[4] = {(uint8_t)c1, (uint8_t)c2, (uint8_t)len, (uint8_t)get8()};
      convert(0, q);
      return flat_from(1);
    }
    len = len << 8 | get8();
    if (len != w) return fail("HDR: invalid decoded scanline length");
    for (int k = 0; k < 4; k++) {
      long i = 0;
      while (w - i > 0) {
        const long left = w - i;
        int count = get8();
        if (count > 128) {
          const int v = get8();
          count -= 128;
          if (count == 0 || count > left) return fail("HDR: bad RLE data");
          for (int z = 0; z < count; z++) sl[(size_t)(i++) * 4 + k] = (uint8_t)v;
        } else {
          if (count == 0 || count > left) return fail("HDR: bad RLE data");
          for (int z = 0; z < count; z++) sl[(size_t)(i++) * 4 + k] = (uint8_t)get8();
        }
      }
    }
    for (long i = 0; i < w; i++) convert((size_t)j * w + i, &sl[(size_t)i * 4]);
  }
  return true;
}

}  // namespace rt_hdr
