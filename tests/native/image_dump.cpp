// Loads an image file through the plugin's image class (rt/image.h: JPEG, PNG, HDR, PPM, PFM) and prints,
// for tests/test_png_hdr.py:
//   line 1: width height (0 0 when the file is refused)
//   line 2: hex of image::bytes() -- what picture_texture samples: float_to_byte of the linear floats
//           (stbi_loadf's, image.h:33-50, 97-101)
#include <cstdio>

#include "image.h"

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  image tex(argv[1]);
  std::printf("%d %d\n", tex.width(), tex.height());
  for (uint8_t b : tex.bytes()) std::printf("%02x", b);
  std::printf("\n");
  return 0;
}
