// oracle/_ref/stb_decode -- test infrastructure only: decodes an image file with the reference's own
// vendored decoder (/root/reference/src/stb_image.h, stb_image v2.30, compiled where it lies by
// oracle/Makefile's `ref` target) and prints what the reference's image class would hold:
//   line 1: width height
//   line 2: hex of the 8-bit RGB pixels stbi_load returns (the decoder's own output)
//   line 3: hex of float_to_byte(stbi_loadf(...)) (image.h:33-50, 97-101: what picture_texture samples)
// Built only in the container that has /root/reference; its output pins rt/jpeg.h
// (tests/golden/make_jpeg_golden.py, tests/test_jpeg.py). Never linked into the product.
#define STB_IMAGE_IMPLEMENTATION
#include <cstdio>

#include "stb_image.h"

static unsigned char float_to_byte(float v) {
  if (v <= 0.0) return 0;
  if (1.0 <= v) return 255;
  return static_cast<unsigned char>(256.0 * v);
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  int w = 0, h = 0, n = 0;
  unsigned char* b = stbi_load(argv[1], &w, &h, &n, 3);
  float* f = stbi_loadf(argv[1], &w, &h, &n, 3);
  if (!b || !f) return 1;
  std::printf("%d %d\n", w, h);
  for (long i = 0; i < 3L * w * h; i++) std::printf("%02x", b[i]);
  std::printf("\n");
  for (long i = 0; i < 3L * w * h; i++) std::printf("%02x", float_to_byte(f[i]));
  std::printf("\n");
  stbi_image_free(b);
  stbi_image_free(f);
  return 0;
}
