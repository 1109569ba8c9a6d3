// png.h -- PNG decoding for picture textures (reference: src/image.h:33-50, which loads every non-EXR
// file through its vendored stb_image's stbi_loadf).
//
// Our own decoder: zlib / DEFLATE (RFC 1950 / 1951: stored, fixed and dynamic Huffman blocks), the five
// scanline filters, Adam7 interlacing, bit depths 1/2/4/8/16 and colour types gray, RGB, palette,
// gray+alpha and RGBA, returned as 8-bit RGB the way stbi_load(..., 3) returns it: 16-bit samples keep
// their high byte, 1/2/4-bit gray is scaled to 0..255 (x 0xFF / 0x55 / 0x11), palette indices are not,
// alpha and tRNS are dropped with the fourth component. Pinned byte for byte against the reference's
// stb_image on generated files (tests/golden/make_image_golden.py, tests/test_png_hdr.py).
#pragma once
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace rt_png {

struct Image {
  int width = 0, height = 0;
  std::vector<uint8_t> rgb;  // 8-bit RGB, row 0 at the top
};

namespace detail {

struct Bits {  // DEFLATE reads bits LSB first
  const uint8_t* p;
  size_t n, pos = 0;
  uint32_t buf = 0;
  int cnt = 0;
  bool bad = false;
  uint32_t get(int k) {
    while (cnt < k) {
      uint32_t b = 0;
      if (pos < n)
        b = p[pos++];
      else
        bad = true;
      buf |= b << cnt;
      cnt += 8;
    }
    const uint32_t v = buf & ((1u << k) - 1u);
    buf >>= k;
    cnt -= k;
    return v;
  }
  void align() {
    buf >>= cnt & 7;
    cnt -= cnt & 7;
  }
};

// canonical Huffman decoding table: counts per length, symbols in code order
struct Huff {
  uint16_t count[16] = {0};
  std::vector<uint16_t> sym;
  bool build(const uint8_t* lens, int n) {
    std::memset(count, 0, sizeof(count));
    for (int i = 0; i < n; i++) count[lens[i]]++;
    count[0] = 0;
    int left = 1;
    for (int l = 1; l < 16; l++) {  // over-subscribed sets are invalid (incomplete ones are allowed)
      left = (left << 1) - count[l];
      if (left < 0) return false;
    }
    uint16_t offs[16];
    offs[1] = 0;
    for (int l = 1; l < 15; l++) offs[l + 1] = (uint16_t)(offs[l] + count[l]);
    sym.assign((size_t)n, 0);
    for (int i = 0; i < n; i++)
      if (lens[i]) sym[offs[lens[i]]++] = (uint16_t)i;
    return true;
  }
  int decode(Bits& b) const {
    int code = 0, first = 0, index = 0;
    for (int l = 1; l < 16; l++) {
      code |= (int)b.get(1);
      const int c = count[l];
      if (code - c < first) return sym[(size_t)(index + (code - first))];
      index += c;
      first += c;
      first <<= 1;
      code <<= 1;
      if (b.bad) return -1;
    }
    return -1;
  }
};

// `limit`: keep at most this many bytes (the image's filtered size: a crafted stream cannot grow the buffer
// past what the header's dimensions use). The rest of the stream is still decoded -- its codes, distances and
// final block validated, its bytes counted and dropped -- as stb_image decodes the whole stream and then
// ignores the surplus: a stream stb refuses (a bad code, no end of block, a truncated tail) is refused here too.
inline bool inflate(const uint8_t* in, size_t n, std::vector<uint8_t>& out, std::string* err,
                    size_t limit = ~size_t(0)) {
  static const uint16_t lbase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                     31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
  static const uint8_t lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
  static const uint16_t dbase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                     193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
  static const uint8_t dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
  auto fail = [&](const char* m) {
    if (err) *err = m;
    return false;
  };
  Bits b{in, n};
  size_t total = out.size();  // bytes decoded, kept or not
  auto put = [&](uint8_t v) {
    if (out.size() < limit) out.push_back(v);
    total++;
  };
  for (;;) {
    const uint32_t last = b.get(1), type = b.get(2);
    if (type == 0) {  // stored
      b.align();
      const uint32_t len = b.get(16), nlen = b.get(16);
      if ((len ^ 0xFFFFu) != nlen) return fail("zlib: stored block length");
      for (uint32_t i = 0; i < len; i++) put((uint8_t)b.get(8));
    } else if (type == 1 || type == 2) {
      Huff lit, dist;
      uint8_t lens[320];
      if (type == 1) {  // fixed codes
        for (int i = 0; i < 144; i++) lens[i] = 8;
        for (int i = 144; i < 256; i++) lens[i] = 9;
        for (int i = 256; i < 280; i++) lens[i] = 7;
        for (int i = 280; i < 288; i++) lens[i] = 8;
        for (int i = 0; i < 30; i++) lens[288 + i] = 5;
        lit.build(lens, 288);
        dist.build(lens + 288, 30);
      } else {  // dynamic codes
        const int hlit = (int)b.get(5) + 257, hdist = (int)b.get(5) + 1, hclen = (int)b.get(4) + 4;
        static const uint8_t ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
        uint8_t cl[19] = {0};
        for (int i = 0; i < hclen; i++) cl[ord[i]] = (uint8_t)b.get(3);
        Huff clh;
        if (!clh.build(cl, 19)) return fail("zlib: code-length code");
        int k = 0;
        while (k < hlit + hdist) {
          const int s = clh.decode(b);
          if (s < 0) return fail("zlib: bad code length");
          if (s < 16) {
            lens[k++] = (uint8_t)s;
          } else {
            int rep, v = 0;
            if (s == 16) {
              if (k == 0) return fail("zlib: repeat without a length");
              v = lens[k - 1];
              rep = 3 + (int)b.get(2);
            } else if (s == 17) {
              rep = 3 + (int)b.get(3);
            } else {
              rep = 11 + (int)b.get(7);
            }
            if (k + rep > hlit + hdist) return fail("zlib: code lengths overflow");
            while (rep--) lens[k++] = (uint8_t)v;
          }
        }
        if (!lit.build(lens, hlit) || !dist.build(lens + hlit, hdist)) return fail("zlib: bad Huffman code");
      }
      for (;;) {
        const int s = lit.decode(b);
        if (s < 0) return fail("zlib: bad literal/length code");
        if (s < 256) {
          put((uint8_t)s);
        } else if (s == 256) {
          break;
        } else {
          const int li = s - 257;
          if (li >= 29) return fail("zlib: bad length symbol");
          const size_t len = lbase[li] + b.get(lext[li]);
          const int ds = dist.decode(b);
          if (ds < 0 || ds >= 30) return fail("zlib: bad distance code");
          const size_t d = dbase[ds] + b.get(dext[ds]);
          if (d > total) return fail("zlib: distance too far back");
          // (while bytes are kept, out holds every byte so far: from + i < out.size())
          const size_t from = total - d;
          for (size_t i = 0; i < len; i++) {
            if (out.size() < limit)
              out.push_back(out[from + i]);
            total++;
          }
        }
        if (b.bad) return fail("zlib: truncated");
      }
    } else {
      return fail("zlib: bad block type");
    }
    if (b.bad) return fail("zlib: truncated");
    if (last) return true;
  }
}

inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

inline int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

}  // namespace detail

inline bool is_png(const std::vector<uint8_t>& d) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
  return d.size() >= 8 && std::memcmp(d.data(), sig, 8) == 0;
}

inline bool decode(const std::vector<uint8_t>& d, Image& im, std::string* err) {
  using namespace detail;
  auto fail = [&](const char* m) {
    if (err) *err = m;
    return false;
  };
  if (!is_png(d)) return fail("not a PNG");
  size_t p = 8;
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> idat, pal;
  bool ihdr = false;
  while (p + 12 <= d.size()) {
    const uint32_t len = be32(&d[p]);
    if (len > d.size() - p - 12) return fail("PNG: chunk past the end");
    const uint8_t* t = &d[p + 4];
    const uint8_t* c = &d[p + 8];
    if (!std::memcmp(t, "IHDR", 4)) {
      if (len < 13) return fail("PNG: short IHDR");
      w = be32(c);
      h = be32(c + 4);
      depth = c[8];
      ctype = c[9];
      interlace = c[12];
      if (c[10] != 0 || c[11] != 0 || interlace > 1) return fail("PNG: unknown compression, filter or interlace");
      ihdr = true;
    } else if (!std::memcmp(t, "PLTE", 4)) {
      pal.assign(c, c + len);
    } else if (!std::memcmp(t, "IDAT", 4)) {
      idat.insert(idat.end(), c, c + len);
    } else if (!std::memcmp(t, "IEND", 4)) {
      break;
    }
    p += 12 + len;
  }
  if (!ihdr || w == 0 || h == 0 || w > (1u << 24) || h > (1u << 24)) return fail("PNG: bad header");
  int ch;
  switch (ctype) {
    case 0: ch = 1; break;
    case 2: ch = 3; break;
    case 3: ch = 1; break;
    case 4: ch = 2; break;
    case 6: ch = 4; break;
    default: return fail("PNG: bad colour type");
  }
  const bool ok_depth = (ctype == 0 && (depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)) ||
                        (ctype == 3 && (depth == 1 || depth == 2 || depth == 4 || depth == 8)) ||
                        ((ctype == 2 || ctype == 4 || ctype == 6) && (depth == 8 || depth == 16));
  if (!ok_depth) return fail("PNG: bad bit depth");
  if (ctype == 3 && pal.size() < 3) return fail("PNG: palette missing");
  if (idat.size() < 2 || (idat[0] & 15) != 8 || ((idat[0] << 8) | idat[1]) % 31 != 0 || (idat[1] & 32))
    return fail("PNG: bad zlib header");
  // stb_image.h:5124-5129 ("Image too large to decode"): refused before anything is allocated
  if ((1u << 30) / w / (uint32_t)(ctype == 3 ? 4 : ch) < h) return fail("PNG: image too large");
  // the filtered size the header implies (every pass's rows, a filter byte each): inflate stops there,
  // and fewer bytes than that is a corrupt image (stb: "not enough pixels") -- checked before the
  // output is allocated
  auto pass_bytes = [&](uint32_t x0, uint32_t y0, uint32_t dx, uint32_t dy) -> uint64_t {
    const uint64_t pw = x0 < w ? (w - x0 + dx - 1) / dx : 0, ph = y0 < h ? (h - y0 + dy - 1) / dy : 0;
    return pw == 0 || ph == 0 ? 0 : ((pw * ch * depth + 7) / 8 + 1) * ph;
  };
  static const uint32_t ax[7] = {0, 4, 0, 2, 0, 1, 0}, ay[7] = {0, 0, 4, 0, 2, 0, 1};
  static const uint32_t adx[7] = {8, 8, 4, 4, 2, 2, 1}, ady[7] = {8, 8, 8, 4, 4, 2, 2};
  uint64_t expect = 0;
  if (!interlace)
    expect = pass_bytes(0, 0, 1, 1);
  else
    for (int k = 0; k < 7; k++) expect += pass_bytes(ax[k], ay[k], adx[k], ady[k]);
  std::vector<uint8_t> raw;
  if (!inflate(idat.data() + 2, idat.size() - 2, raw, err, (size_t)expect)) return false;
  if (raw.size() < expect) return fail("PNG: image data too short");
  const int bpp = (ch * depth + 7) / 8;  // bytes per complete pixel, for the filters (>= 1)
  im.width = (int)w;
  im.height = (int)h;
  im.rgb.assign((size_t)w * h * 3, 0);
  // one pass (the whole image, or one of Adam7's seven) into im.rgb
  auto pass = [&](size_t& off, uint32_t x0, uint32_t y0, uint32_t dx, uint32_t dy) -> bool {
    const uint32_t pw = x0 < w ? (w - x0 + dx - 1) / dx : 0, ph = y0 < h ? (h - y0 + dy - 1) / dy : 0;
    if (pw == 0 || ph == 0) return true;
    const size_t stride = ((size_t)pw * ch * depth + 7) / 8;
    std::vector<uint8_t> prev(stride, 0), cur(stride);
    for (uint32_t y = 0; y < ph; y++) {
      if (off + 1 + stride > raw.size()) return fail("PNG: image data too short");
      const int f = raw[off];
      const uint8_t* src = &raw[off + 1];
      off += 1 + stride;
      for (size_t i = 0; i < stride; i++) {
        const int a = i >= (size_t)bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= (size_t)bpp ? prev[i - bpp] : 0;
        int v = src[i];
        switch (f) {
          case 0: break;
          case 1: v += a; break;
          case 2: v += b; break;
          case 3: v += (a + b) >> 1; break;
          case 4: v += paeth(a, b, c); break;
          default: return fail("PNG: bad filter type");
        }
        cur[i] = (uint8_t)v;
      }
      for (uint32_t x = 0; x < pw; x++) {
        int s[4] = {0, 0, 0, 0};
        for (int k = 0; k < ch; k++) {
          if (depth == 8) {
            s[k] = cur[(size_t)x * ch + k];
          } else if (depth == 16) {
            s[k] = cur[((size_t)x * ch + k) * 2];  // the high byte (stbi__convert_16_to_8)
          } else {
            const size_t bit = (size_t)x * depth;
            s[k] = (cur[bit >> 3] >> (8 - depth - (bit & 7))) & ((1 << depth) - 1);
            if (ctype == 0) s[k] *= depth == 1 ? 0xFF : (depth == 2 ? 0x55 : 0x11);
          }
        }
        uint8_t* o = &im.rgb[3 * ((size_t)(y0 + y * dy) * w + (x0 + x * dx))];
        if (ctype == 3) {
          const size_t i = (size_t)s[0] * 3;
          if (i + 3 > pal.size()) return fail("PNG: palette index out of range");
          o[0] = pal[i], o[1] = pal[i + 1], o[2] = pal[i + 2];
        } else if (ch <= 2) {
          o[0] = o[1] = o[2] = (uint8_t)s[0];
        } else {
          o[0] = (uint8_t)s[0], o[1] = (uint8_t)s[1], o[2] = (uint8_t)s[2];
        }
      }
      prev.swap(cur);
    }
    return true;
  };
  size_t off = 0;
  if (!interlace) return pass(off, 0, 0, 1, 1);
  for (int k = 0; k < 7; k++)
    if (!pass(off, ax[k], ay[k], adx[k], ady[k])) return false;
  return true;
}

}  // namespace rt_png
