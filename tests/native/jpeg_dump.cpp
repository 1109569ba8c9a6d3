// Decodes an image file with the plugin's loaders and prints, for tests/test_jpeg.py:
//   line 1: width height (0 0 if rt_jpeg::decode refuses it: progressive, 12-bit, ...)
//   line 2: hex of the 8-bit RGB pixels rt_jpeg::decode returns
//   line 3: hex of image::bytes() (what picture_texture samples: float_to_byte(powf(v / 255, 2.2)))
#include <cstdio>
#include <fstream>
#include <iterator>

#include "image.h"

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  rt_jpeg::Image im;
  std::string err;
  if (!rt_jpeg::decode(d, im, &err)) {
    std::printf("0 0\n\n\n");
    return 0;
  }
  std::printf("%d %d\n", im.width, im.height);
  for (uint8_t b : im.rgb) std::printf("%02x", b);
  std::printf("\n");
  image tex(argv[1]);
  for (uint8_t b : tex.bytes()) std::printf("%02x", b);
  std::printf("\n");
  return 0;
}
