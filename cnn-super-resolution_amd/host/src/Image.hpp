// Image files for the `cnn` CLI and the luma helpers.
//
// The reference reads/writes images with the vendored stb_image /
// stb_image_write (src/opencl/UtilsOpenCL.cpp load_image / write_image).
// This is an independent codec set (PNG on the system zlib):
//   JPEG read: baseline / extended / progressive Huffman, 8-bit, gray or
//        YCbCr with whole-ratio sampling factors (Jpeg.cpp) -- the reference's
//        sample pairs and photos are JPEG (src/Main_cl.cpp:267-301)
//   PNG  read: 8-bit gray / gray+alpha / RGB / RGBA / palette, non-interlaced;
//        write: 8-bit gray, RGB or RGBA
//   PNM  read/write: binary P5 (gray) / P6 (RGB)
#ifndef SRCNN_HOST_IMAGE_HPP
#define SRCNN_HOST_IMAGE_HPP

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "Context.hpp"

namespace srcnn {
namespace image {

/** Load a JPEG, PNG or PNM file (by content) into `img`; `channels` 0 keeps
 * the file's channel count, 1/3/4 converts (gray <-> RGB, alpha = 255). */
void load(const std::string& path, ImageData& img, int channels = 0);

/** `load` on an in-memory file image; `name` only labels the error message. */
void decode(const std::vector<unsigned char>& file, ImageData& img, int channels = 0,
            const std::string& name = "<memory>");

/** Largest decoded image, in pixels (and per side): corrupt or hostile
 * headers must not turn into multi-GB allocations (16384 x 16384). */
constexpr size_t kMaxImagePixels = size_t(1) << 28;
constexpr uint32_t kMaxImageSide = 1u << 24;

/** Throw IOException unless a w x h image with `channels` is within the caps. */
void check_dims(uint64_t w, uint64_t h, int channels);

/** Decode a JPEG file image (Jpeg.cpp) to 1 (gray) or 3 (RGB) channels. */
void decode_jpeg(const std::vector<unsigned char>& file, ImageData& img);

/** Write `img` (bpp 1, 3 or 4) as PNG, or PNM when the path ends in
 * .pgm/.ppm/.pnm (RGBA written as RGB there). */
void write(const std::string& path, const ImageData& img);

/** Write a float luma plane (values in [0,1], clamped) as an 8-bit gray PNG. */
void write_luma(const std::string& path, const float* luma, int w, int h);

}  // namespace image
}  // namespace srcnn

#endif  // SRCNN_HOST_IMAGE_HPP
