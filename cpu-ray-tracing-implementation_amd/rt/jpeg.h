// jpeg.h -- baseline JPEG decoding for picture textures (host side).
//
// The reference loads images with its vendored stb_image (v2.30; image.h:33-50: stbi_loadf with
// 3 components). This is our own decoder of the same file format, restating the published
// algorithm stb implements so the bytes come out identical (tests/test_jpeg.py pins that against
// the reference's decoder built from its own header, oracle/ref_stb_decode.cpp):
//   - baseline sequential Huffman JPEG (SOF0 / SOF1, 8-bit samples), 1 or 3 components, any
//     restart interval; each component sampled 1x1, or luma 2x2 / 2x1 / 1x2 over 1x1 chroma;
//   - dequantised coefficients kept as 16-bit integers (coefficient x table entry, truncated);
//   - the integer 8x8 inverse DCT with 12-bit fixed-point constants (the IJG "islow" transform as
//     stb scales it: columns to 1/1024 with 2 extra bits, rows to 1/131072, +128, clamped);
//   - YCbCr -> RGB in 20-bit fixed point (Cr 1.40200, Cb 1.77200, G -0.71414 Cr - 0.34414 Cb with
//     the Cb term's low 16 bits cleared), rounded by +2^19; an Adobe APP14 marker with transform
//     0 means the 3 components are already RGB;
//   - subsampled chroma upsampled with stb's filters: horizontal / vertical 3:1 triangle taps,
//     and for 2x2 the separable triangle filter over rows (3 near + 1 far, then 3:1 columns).
// Progressive, arithmetic-coded, 12-bit and CMYK files are reported as unsupported (the image then
// samples magenta, as the reference does for a file it cannot load).
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace rt_jpeg {

struct Image {
  int width = 0, height = 0;
  std::vector<uint8_t> rgb;  // 3 bytes per pixel, row 0 at the top
};

namespace detail {

// natural (row-major) index of the k-th coefficient in zig-zag order
constexpr uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huffman {  // canonical code tables of one DHT entry
  int mincode[17] = {}, maxcode[18] = {}, valptr[17] = {};
  uint8_t vals[256] = {};
  bool present = false;
};

struct Component {
  int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
  int dc_pred = 0;
  int bw = 0, bh = 0;           // blocks across / down (padded to whole MCUs)
  std::vector<uint8_t> plane;   // bw*8 x bh*8 samples
};

class Decoder {
 public:
  explicit Decoder(const std::vector<uint8_t>& f) : d_(f) {}
  bool run(Image& out, std::string& err);

 private:
  const std::vector<uint8_t>& d_;
  size_t pos_ = 0;
  uint16_t q_[4][64] = {};  // quantisation tables in zig-zag order
  Huffman dc_[4], ac_[4];
  std::vector<Component> comp_;
  int width_ = 0, height_ = 0, hmax_ = 1, vmax_ = 1, restart_ = 0;
  int adobe_transform_ = -1;
  // entropy-coded segment bit reader
  uint32_t bits_ = 0;
  int nbits_ = 0;
  bool marker_hit_ = false;

  int byte() { return pos_ < d_.size() ? d_[pos_++] : -1; }
  int word() {
    const int a = byte(), b = byte();
    return (a < 0 || b < 0) ? -1 : (a << 8 | b);
  }
  void fill() {
    while (nbits_ <= 24) {
      int c = 0;
      if (!marker_hit_) {
        c = byte();
        if (c == 0xFF) {
          const int n = pos_ < d_.size() ? d_[pos_] : -1;
          if (n == 0) {
            pos_++;  // stuffed 0xFF
          } else {  // a marker: the segment ends, zero bits from here
            pos_--;
            marker_hit_ = true;
            c = 0;
          }
        } else if (c < 0) {
          marker_hit_ = true;
          c = 0;
        }
      }
      bits_ |= (uint32_t)c << (24 - nbits_);
      nbits_ += 8;
    }
  }
  int bit() {
    if (nbits_ < 1) fill();
    const int b = (int)(bits_ >> 31);
    bits_ <<= 1;
    nbits_--;
    return b;
  }
  int receive(int s) {  // s raw bits, most significant first
    int v = 0;
    for (int i = 0; i < s; i++) v = (v << 1) | bit();
    return v;
  }
  static int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }
  int decode(const Huffman& h) {
    int code = 0;
    for (int l = 1; l <= 16; l++) {
      code = (code << 1) | bit();
      if (code <= h.maxcode[l]) return h.vals[h.valptr[l] + code - h.mincode[l]];
    }
    return -1;  // corrupt
  }
  bool dqt(int len);
  bool dht(int len);
  bool sof(int len, std::string& err);
  bool sos(int len, std::string& err);
  bool decode_block(Component& c, int16_t* coef);
  bool entropy(std::string& err);
  void to_rgb(Image& out) const;
};

// Integer inverse DCT of one 8x8 block of dequantised coefficients into 8-bit samples.
// One 1-D pass: even part from inputs 0, 2, 4, 6, odd part from 1, 3, 5, 7 (rotations with
// 12-bit constants), outputs i and 7 - i as even +- odd.
struct Idct1 {
  static constexpr int F(float x) { return (int)(x * 4096 + 0.5); }  // float constant x 4096, rounded
  int even[4], odd[4];
  void run(int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7) {
    const int z = (s2 + s6) * F(0.5411961f);
    const int e2 = z + s6 * F(-1.847759065f), e3 = z + s2 * F(0.765366865f);
    const int e0 = (s0 + s4) * 4096, e1 = (s0 - s4) * 4096;
    even[0] = e0 + e3;
    even[3] = e0 - e3;
    even[1] = e1 + e2;
    even[2] = e1 - e2;
    // odd part: inputs 7, 5, 3, 1
    int a = s7, b = s5, c = s3, d = s1;
    const int p3 = a + c, p4 = b + d, p1 = a + d, p2 = b + c;
    const int p5 = (p3 + p4) * F(1.175875602f);
    a *= F(0.298631336f);
    b *= F(2.053119869f);
    c *= F(3.072711026f);
    d *= F(1.501321110f);
    const int q1 = p5 + p1 * F(-0.899976223f), q2 = p5 + p2 * F(-2.562915447f);
    const int q3 = p3 * F(-1.961570560f), q4 = p4 * F(-0.390180644f);
    odd[0] = d + q1 + q4;  // pairs with even[0]
    odd[1] = c + q2 + q3;
    odd[2] = b + q2 + q4;
    odd[3] = a + q1 + q3;
  }
};

inline uint8_t clamp8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

inline void idct8x8(const int16_t* in, uint8_t* out, int stride) {
  int tmp[64];
  for (int col = 0; col < 8; col++) {
    const int16_t* s = in + col;
    bool ac_zero = true;
    for (int r = 1; r < 8; r++) ac_zero = ac_zero && s[8 * r] == 0;
    if (ac_zero) {  // a flat column: every output is the DC term, kept at 4x
      for (int r = 0; r < 8; r++) tmp[8 * r + col] = s[0] * 4;
      continue;
    }
    Idct1 t;
    t.run(s[0], s[8], s[16], s[24], s[32], s[40], s[48], s[56]);
    for (int i = 0; i < 4; i++) {  // scale 2^12 down to 2^2 with rounding
      const int e = t.even[i] + 512;
      tmp[8 * i + col] = (e + t.odd[i]) >> 10;
      tmp[8 * (7 - i) + col] = (e - t.odd[i]) >> 10;
    }
  }
  for (int row = 0; row < 8; row++) {
    const int* s = tmp + 8 * row;
    Idct1 t;
    t.run(s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]);
    uint8_t* o = out + row * stride;
    for (int i = 0; i < 4; i++) {  // 2^17 total scale, rounded, level-shifted by 128
      const int e = t.even[i] + 65536 + (128 << 17);
      o[i] = clamp8((e + t.odd[i]) >> 17);
      o[7 - i] = clamp8((e - t.odd[i]) >> 17);
    }
  }
}

inline bool Decoder::dqt(int len) {
  while (len > 0) {
    const int pq_tq = byte();
    if (pq_tq < 0) return false;
    const int pq = pq_tq >> 4, tq = pq_tq & 15;
    if (tq > 3 || pq > 1) return false;
    for (int k = 0; k < 64; k++) q_[tq][k] = (uint16_t)(pq ? word() : byte());
    len -= 1 + 64 * (pq ? 2 : 1);
  }
  return len == 0;
}

inline bool Decoder::dht(int len) {
  while (len > 0) {
    const int tc_th = byte();
    if (tc_th < 0) return false;
    const int tc = tc_th >> 4, th = tc_th & 15;
    if (tc > 1 || th > 3) return false;
    Huffman& h = tc ? ac_[th] : dc_[th];
    int counts[17] = {}, total = 0;
    for (int l = 1; l <= 16; l++) total += counts[l] = byte();
    if (total > 256) return false;
    for (int i = 0; i < total; i++) h.vals[i] = (uint8_t)byte();
    int code = 0, k = 0;
    for (int l = 1; l <= 16; l++) {  // canonical codes: consecutive within a length, doubled per length
      h.valptr[l] = k;
      h.mincode[l] = code;
      code += counts[l];
      k += counts[l];
      h.maxcode[l] = counts[l] ? code - 1 : -1;
      code <<= 1;
    }
    h.present = true;
    len -= 17 + total;
  }
  return len == 0;
}

inline bool Decoder::sof(int len, std::string& err) {
  if (byte() != 8) return err = "only 8-bit JPEG samples are supported", false;
  height_ = word();
  width_ = word();
  const int n = byte();
  if (width_ <= 0 || height_ <= 0) return err = "JPEG without a size", false;
  if (n != 1 && n != 3) return err = "only 1- and 3-component JPEGs are supported", false;
  if (len != 6 + 3 * n) return false;
  comp_.assign(n, Component{});
  for (auto& c : comp_) {
    c.id = byte();
    const int hv = byte();
    c.h = hv >> 4;
    c.v = hv & 15;
    c.tq = byte();
    if (c.h < 1 || c.h > 2 || c.v < 1 || c.v > 2 || c.tq > 3) return err = "unsupported JPEG sampling", false;
    hmax_ = std::max(hmax_, c.h);
    vmax_ = std::max(vmax_, c.v);
  }
  for (size_t i = 1; i < comp_.size(); i++)
    if (comp_[i].h != 1 || comp_[i].v != 1) return err = "unsupported JPEG chroma sampling", false;
  const int mcux = (width_ + 8 * hmax_ - 1) / (8 * hmax_), mcuy = (height_ + 8 * vmax_ - 1) / (8 * vmax_);
  for (auto& c : comp_) {
    c.bw = mcux * c.h;
    c.bh = mcuy * c.v;
    c.plane.assign((size_t)c.bw * 8 * c.bh * 8, 0);
  }
  return true;
}

inline bool Decoder::decode_block(Component& c, int16_t* coef) {
  std::memset(coef, 0, 64 * sizeof(int16_t));
  const uint16_t* q = q_[c.tq];
  const int t = decode(dc_[c.td]);
  if (t < 0 || t > 16) return false;
  const int diff = t ? extend(receive(t), t) : 0;
  c.dc_pred += diff;
  coef[0] = (int16_t)(c.dc_pred * q[0]);
  for (int k = 1; k < 64;) {
    const int rs = decode(ac_[c.ta]);
    if (rs < 0) return false;
    const int r = rs >> 4, s = rs & 15;
    if (s == 0) {
      if (r != 15) break;  // end of block
      k += 16;
      continue;
    }
    k += r;
    if (k > 63) return false;
    coef[kZigzag[k]] = (int16_t)(extend(receive(s), s) * q[k]);
    k++;
  }
  return true;
}

inline bool Decoder::sos(int len, std::string& err) {
  const int n = byte();
  if (n != (int)comp_.size() || len != 4 + 2 * n) return err = "only interleaved JPEG scans are supported", false;
  for (int i = 0; i < n; i++) {
    const int id = byte(), tdta = byte();
    Component* c = nullptr;
    for (auto& x : comp_)
      if (x.id == id) c = &x;
    if (!c) return false;
    c->td = tdta >> 4;
    c->ta = tdta & 15;
    if (c->td > 3 || c->ta > 3 || !dc_[c->td].present || !ac_[c->ta].present) return false;
  }
  const int ss = byte(), se = byte(), ahal = byte();
  if (ss != 0 || se != 63 || ahal != 0) return err = "progressive JPEGs are not supported", false;
  return entropy(err);
}

inline bool Decoder::entropy(std::string& err) {
  const int mcux = (width_ + 8 * hmax_ - 1) / (8 * hmax_), mcuy = (height_ + 8 * vmax_ - 1) / (8 * vmax_);
  int16_t coef[64];
  bits_ = 0;
  nbits_ = 0;
  marker_hit_ = false;
  int todo = restart_ ? restart_ : 0x7FFFFFFF;
  for (int my = 0; my < mcuy; my++)
    for (int mx = 0; mx < mcux; mx++) {
      for (auto& c : comp_)
        for (int by = 0; by < c.v; by++)
          for (int bx = 0; bx < c.h; bx++) {
            if (!decode_block(c, coef)) return err = "corrupt JPEG data", false;
            const int x0 = (mx * c.h + bx) * 8, y0 = (my * c.v + by) * 8;
            idct8x8(coef, c.plane.data() + (size_t)y0 * c.bw * 8 + x0, c.bw * 8);
          }
      if (--todo == 0 && !(my == mcuy - 1 && mx == mcux - 1)) {  // RSTn: realign, reset the predictors
        todo = restart_;
        nbits_ = 0;
        bits_ = 0;
        marker_hit_ = false;
        if (pos_ + 1 < d_.size() && d_[pos_] == 0xFF && d_[pos_ + 1] >= 0xD0 && d_[pos_ + 1] <= 0xD7) pos_ += 2;
        for (auto& c : comp_) c.dc_pred = 0;
      }
    }
  return true;
}

inline void Decoder::to_rgb(Image& out) const {
  out.width = width_;
  out.height = height_;
  out.rgb.assign((size_t)width_ * height_ * 3, 0);
  const Component& Y = comp_[0];
  const int ys = Y.bw * 8;
  // luma at full resolution; chroma upsampled to it (stb's triangle filters)
  std::vector<uint8_t> cb, cr;
  auto upsample = [&](const Component& c, std::vector<uint8_t>& dst) {
    const int cs = c.bw * 8, ch = c.bh * 8;  // chroma plane stride / rows
    dst.assign((size_t)width_ * height_, 0);
    const int hs = hmax_ / c.h, vs = vmax_ / c.v;
    auto src = [&](int x, int y) -> int { return c.plane[(size_t)y * cs + x]; };
    const int cw = (width_ + hs - 1) / hs, chh = (height_ + vs - 1) / vs;  // chroma samples in use
    (void)ch;
    std::vector<int> col(cw);
    std::vector<uint8_t> row(cw);
    for (int y = 0; y < height_; y++) {
      const int sy = y / vs;
      // vertical: 1x (copy) or 2x: 3 * near + far (stb keeps these as 4x sums for the 2x2 filter)
      if (vs == 2) {
        const int far = (y & 1) ? std::min(sy + 1, chh - 1) : std::max(sy - 1, 0);
        for (int x = 0; x < cw; x++) col[x] = 3 * src(x, sy) + src(x, far);
      }
      uint8_t* o = dst.data() + (size_t)y * width_;
      if (hs == 1 && vs == 1) {
        for (int x = 0; x < width_; x++) o[x] = (uint8_t)src(x, sy);
      } else if (hs == 2 && vs == 1) {  // horizontal 2x: (3 near + far + 2) >> 2, edges copied
        for (int x = 0; x < cw; x++) row[x] = (uint8_t)src(x, sy);
        if (cw == 1) {
          o[0] = row[0];
          if (width_ > 1) o[1] = row[0];
        } else {
          o[0] = row[0];
          o[1] = (uint8_t)((row[0] * 3 + row[1] + 2) >> 2);
          for (int x = 1; x < cw - 1; x++) {
            const int n = 3 * row[x] + 2;
            o[2 * x] = (uint8_t)((n + row[x - 1]) >> 2);
            o[2 * x + 1] = (uint8_t)((n + row[x + 1]) >> 2);
          }
          const int l = cw - 1;  // stb's last pair weights the second-to-last sample 3:1 (as it does)
          if (2 * l < width_) o[2 * l] = (uint8_t)((row[l - 1] * 3 + row[l] + 2) >> 2);
          if (2 * l + 1 < width_) o[2 * l + 1] = row[l];
        }
      } else if (hs == 1 && vs == 2) {  // vertical 2x: (3 near + far + 2) >> 2
        for (int x = 0; x < width_; x++) o[x] = (uint8_t)((col[x] + 2) >> 2);
      } else {  // 2x2: the column sums (x4) filtered horizontally 3:1, /16 with +8 rounding
        if (cw == 1) {
          o[0] = (uint8_t)((col[0] + 2) >> 2);
          if (width_ > 1) o[1] = o[0];
        } else {
          o[0] = (uint8_t)((col[0] + 2) >> 2);
          for (int x = 1; x < cw; x++) {
            const int t0 = col[x - 1], t1 = col[x];
            if (2 * x - 1 < width_) o[2 * x - 1] = (uint8_t)((3 * t0 + t1 + 8) >> 4);
            if (2 * x < width_) o[2 * x] = (uint8_t)((3 * t1 + t0 + 8) >> 4);
          }
          if (2 * cw - 1 < width_) o[2 * cw - 1] = (uint8_t)((col[cw - 1] + 2) >> 2);
        }
      }
    }
  };
  if (comp_.size() == 3) {
    upsample(comp_[1], cb);
    upsample(comp_[2], cr);
  }
  const bool rgb = comp_.size() == 3 && adobe_transform_ == 0;
  for (int y = 0; y < height_; y++)
    for (int x = 0; x < width_; x++) {
      uint8_t* o = out.rgb.data() + 3 * ((size_t)y * width_ + x);
      const int yy = Y.plane[(size_t)y * ys + x];
      if (comp_.size() == 1) {
        o[0] = o[1] = o[2] = (uint8_t)yy;
        continue;
      }
      const int b_ = cb[(size_t)y * width_ + x], r_ = cr[(size_t)y * width_ + x];
      if (rgb) {
        o[0] = (uint8_t)yy;
        o[1] = (uint8_t)b_;
        o[2] = (uint8_t)r_;
        continue;
      }
      auto fix = [](float v) { return ((int)(v * 4096.0f + 0.5f)) << 8; };
      const int base = (yy << 20) + (1 << 19), vcr = r_ - 128, vcb = b_ - 128;
      const int R = (base + vcr * fix(1.40200f)) >> 20;
      const int G = (base + vcr * -fix(0.71414f) + ((vcb * -fix(0.34414f)) & (int)0xffff0000)) >> 20;
      const int B = (base + vcb * fix(1.77200f)) >> 20;
      o[0] = clamp8(R);
      o[1] = clamp8(G);
      o[2] = clamp8(B);
    }
}

inline bool Decoder::run(Image& out, std::string& err) {
  if (byte() != 0xFF || byte() != 0xD8) return err = "not a JPEG file", false;
  bool frame = false;
  for (;;) {
    int c = byte();
    while (c == 0xFF) c = byte();  // fill bytes before a marker
    if (c < 0) return err = "truncated JPEG", false;
    const int m = c;
    if (m == 0xD9) break;  // EOI
    if (m >= 0xD0 && m <= 0xD7) continue;
    const int len = word();
    if (len < 2 || pos_ + (size_t)(len - 2) > d_.size()) return err = "truncated JPEG segment", false;
    const size_t next = pos_ + (size_t)(len - 2);
    bool ok = true;
    if (m == 0xDB) {
      ok = dqt(len - 2);
    } else if (m == 0xC4) {
      ok = dht(len - 2);
    } else if (m == 0xC0 || m == 0xC1) {
      ok = sof(len - 2, err);
      frame = ok;
    } else if (m == 0xC2 || m == 0xC3 || (m >= 0xC5 && m <= 0xCF && m != 0xC8 && m != 0xCC)) {
      return err = "progressive / lossless / arithmetic JPEGs are not supported", false;
    } else if (m == 0xDD) {
      restart_ = word();
    } else if (m == 0xEE && len >= 14) {  // Adobe APP14: the colour transform flag is its last byte
      if (d_[pos_] == 'A' && d_[pos_ + 1] == 'd' && d_[pos_ + 2] == 'o' && d_[pos_ + 3] == 'b' && d_[pos_ + 4] == 'e')
        adobe_transform_ = d_[pos_ + 11];
    } else if (m == 0xDA) {
      if (!frame) return err = "scan before frame", false;
      if (!sos(len - 2, err)) return err.empty() ? (err = "corrupt JPEG scan", false) : false;
      // skip to the next marker after the entropy-coded data
      while (pos_ + 1 < d_.size() && !(d_[pos_] == 0xFF && d_[pos_ + 1] != 0 && !(d_[pos_ + 1] >= 0xD0 && d_[pos_ + 1] <= 0xD7)))
        pos_++;
      continue;
    }
    if (!ok) return err.empty() ? (err = "corrupt JPEG segment", false) : false;
    pos_ = next;
  }
  if (!frame) return err = "JPEG without a frame", false;
  to_rgb(out);
  return true;
}

}  // namespace detail

// Decodes a JPEG file held in memory; false with a message for what is not supported.
inline bool decode(const std::vector<uint8_t>& file, Image& out, std::string* err = nullptr) {
  std::string e;
  detail::Decoder d(file);
  const bool ok = d.run(out, e);
  if (!ok && err) *err = e;
  return ok;
}

}  // namespace rt_jpeg
