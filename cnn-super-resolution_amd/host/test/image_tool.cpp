// image_tool -- test driver of the host image codecs (no device needed):
//   image_tool IN OUT        decode IN (JPEG / PNG / PNM, by content) and
//                            write it as OUT (PNG, or PNM for .ppm/.pgm)
// Exit status 1 and the IOException message on unsupported / corrupt input.
#include <iostream>

#include "Image.hpp"

int main(int argc, char** argv) {
  if (argc != 3) {
    std::cerr << "usage: image_tool IN OUT" << std::endl;
    return 2;
  }
  try {
    srcnn::ImageData img;
    srcnn::image::load(argv[1], img);
    srcnn::image::write(argv[2], img);
    std::cout << img.w << " " << img.h << " " << img.bpp << std::endl;
  } catch (const std::exception& e) {
    std::cout << "[ERROR] " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
