#include "Image.hpp"

#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <sstream>

namespace srcnn {
namespace image {

namespace {

std::vector<unsigned char> read_all(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) throw IOException("Could not open image file: " + path);
  return std::vector<unsigned char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

uint32_t be32(const unsigned char* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}

void put32(std::string& s, uint32_t v) {
  s += char(v >> 24);
  s += char(v >> 16);
  s += char(v >> 8);
  s += char(v);
}

bool ends_with(const std::string& s, const char* suf) {
  size_t n = std::strlen(suf);
  if (s.size() < n) return false;
  std::string t = s.substr(s.size() - n);
  std::transform(t.begin(), t.end(), t.begin(), ::tolower);
  return t == suf;
}

int paeth(int a, int b, int c) {
  int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

void decode_png(const std::vector<unsigned char>& f, ImageData& img) {
  static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) throw IOException("not a PNG file");
  size_t pos = 8;
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = -1, interlace = 0;
  std::vector<unsigned char> idat, palette, trns;
  while (pos + 8 <= f.size()) {
    uint32_t len = be32(&f[pos]);
    std::string type(reinterpret_cast<const char*>(&f[pos + 4]), 4);
    if (pos + 12 + size_t(len) > f.size()) throw IOException("truncated PNG chunk");
    const unsigned char* d = &f[pos + 8];
    if (type == "IHDR") {
      if (len < 13) throw IOException("short PNG IHDR");
      w = be32(d);
      h = be32(d + 4);
      depth = d[8];
      ctype = d[9];
      interlace = d[12];
    } else if (type == "PLTE") {
      palette.assign(d, d + len);
    } else if (type == "tRNS") {
      trns.assign(d, d + len);
    } else if (type == "IDAT") {
      idat.insert(idat.end(), d, d + len);
    } else if (type == "IEND") {
      break;
    }
    pos += 12 + size_t(len);
  }
  if (!w || !h || ctype < 0) throw IOException("PNG without IHDR");
  if (depth != 8) throw IOException("only 8-bit PNG is supported");
  if (interlace) throw IOException("interlaced PNG is not supported");
  int ch = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
  if (!ch) throw IOException("unsupported PNG color type");
  check_dims(w, h, ch);
  // zlib's deflate ratio is below 1032:1: IDAT data far too short for the
  // raw size cannot inflate to it, so reject before allocating
  if (idat.size() < (size_t(w) * ch + 1) * h / 1032) throw IOException("corrupt PNG image data");
  size_t stride = size_t(w) * ch;
  std::vector<unsigned char> raw((stride + 1) * h);
  uLongf out_len = raw.size();
  if (uncompress(raw.data(), &out_len, idat.data(), idat.size()) != Z_OK || out_len != raw.size())
    throw IOException("corrupt PNG image data");
  std::vector<unsigned char> px(stride * h);
  for (uint32_t y = 0; y < h; ++y) {
    const unsigned char* src = &raw[y * (stride + 1) + 1];
    unsigned char* cur = &px[y * stride];
    const unsigned char* prev = y ? &px[(y - 1) * stride] : nullptr;
    int filter = raw[y * (stride + 1)];
    for (size_t x = 0; x < stride; ++x) {
      int a = x >= size_t(ch) ? cur[x - ch] : 0, b = prev ? prev[x] : 0,
          c = (prev && x >= size_t(ch)) ? prev[x - ch] : 0, v = src[x];
      switch (filter) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) / 2; break;
        case 4: v += paeth(a, b, c); break;
        default: throw IOException("bad PNG filter");
      }
      cur[x] = static_cast<unsigned char>(v);
    }
  }
  if (ctype == 3) {  // palette -> RGB(A)
    bool alpha = !trns.empty();
    img = ImageData(w, h, alpha ? 4 : 3);
    for (size_t i = 0; i < size_t(w) * h; ++i) {
      size_t k = px[i];
      if (3 * k + 2 >= palette.size()) throw IOException("PNG palette index out of range");
      for (int c = 0; c < 3; ++c) img.data[i * img.bpp + c] = palette[3 * k + c];
      if (alpha) img.data[i * 4 + 3] = k < trns.size() ? trns[k] : 255;
    }
  } else if (ctype == 4) {  // gray+alpha -> RGBA
    img = ImageData(w, h, 4);
    for (size_t i = 0; i < size_t(w) * h; ++i) {
      for (int c = 0; c < 3; ++c) img.data[4 * i + c] = px[2 * i];
      img.data[4 * i + 3] = px[2 * i + 1];
    }
  } else {
    img = ImageData(w, h, ch);
    img.data.swap(px);
  }
}

void decode_pnm(const std::vector<unsigned char>& f, ImageData& img) {
  std::string head(f.begin(), f.begin() + std::min<size_t>(f.size(), 512));
  std::istringstream ss(head);
  std::string magic;
  ss >> magic;
  int ch = magic == "P5" ? 1 : magic == "P6" ? 3 : 0;
  if (!ch) throw IOException("unsupported PNM type (P5/P6 only)");
  auto next_int = [&]() {
    std::string tok;
    while (ss >> tok) {
      if (tok[0] == '#') {
        std::string rest;
        std::getline(ss, rest);
        continue;
      }
      return std::atoi(tok.c_str());
    }
    throw IOException("truncated PNM header");
  };
  int w = next_int(), h = next_int(), maxv = next_int();
  if (w <= 0 || h <= 0 || maxv != 255) throw IOException("unsupported PNM header");
  check_dims(w, h, ch);
  const std::streamoff pos = ss.tellg();
  if (pos < 0) throw IOException("truncated PNM header");
  size_t off = size_t(pos) + 1;
  if (off + size_t(w) * h * ch > f.size()) throw IOException("truncated PNM data");
  img = ImageData(w, h, ch, &f[off]);
}

void convert(ImageData& img, int channels) {
  if (!channels || channels == img.bpp) return;
  ImageData out(img.w, img.h, channels);
  for (size_t i = 0, n = size_t(img.w) * img.h; i < n; ++i) {
    const unsigned char* s = &img.data[i * img.bpp];
    unsigned char rgb[4] = {s[0], s[img.bpp >= 3 ? 1 : 0], s[img.bpp >= 3 ? 2 : 0],
                            img.bpp == 4 ? s[3] : (unsigned char)255};
    unsigned char* d = &out.data[i * channels];
    if (channels == 1) {
      d[0] = img.bpp >= 3 ? static_cast<unsigned char>(
                                std::lround(0.299 * rgb[0] + 0.587 * rgb[1] + 0.114 * rgb[2]))
                          : rgb[0];
    } else {
      for (int c = 0; c < std::min(channels, 4); ++c) d[c] = rgb[c];
    }
  }
  img = std::move(out);
}

}  // namespace

void check_dims(uint64_t w, uint64_t h, int channels) {
  if (w == 0 || h == 0 || w > kMaxImageSide || h > kMaxImageSide || w * h > kMaxImagePixels || channels < 1 ||
      channels > 4)
    throw IOException("unsupported image size " + std::to_string(w) + "x" + std::to_string(h));
}

void decode(const std::vector<unsigned char>& f, ImageData& img, int channels, const std::string& name) {
  if (f.size() >= 8 && f[0] == 137 && f[1] == 'P' && f[2] == 'N' && f[3] == 'G')
    decode_png(f, img);
  else if (f.size() >= 2 && f[0] == 'P' && (f[1] == '5' || f[1] == '6'))
    decode_pnm(f, img);
  else if (f.size() >= 3 && f[0] == 0xFF && f[1] == 0xD8 && f[2] == 0xFF)
    decode_jpeg(f, img);
  else
    throw IOException("unsupported image format (JPEG / PNG / PNM only): " + name);
  convert(img, channels);
}

void load(const std::string& path, ImageData& img, int channels) { decode(read_all(path), img, channels, path); }

void write(const std::string& path, const ImageData& img) {
  if (img.w <= 0 || img.h <= 0 || !(img.bpp == 1 || img.bpp == 3 || img.bpp == 4))
    throw std::runtime_error("write_image: expected a non-empty 1/3/4 channel image");
  std::ofstream out(path, std::ios::binary);
  if (!out.is_open()) throw IOException("Could not write image file: " + path);
  if (ends_with(path, ".pgm") || ends_with(path, ".ppm") || ends_with(path, ".pnm")) {
    int ch = img.bpp == 1 ? 1 : 3;
    out << (ch == 1 ? "P5" : "P6") << "\n" << img.w << " " << img.h << "\n255\n";
    for (size_t i = 0, n = size_t(img.w) * img.h; i < n; ++i)
      out.write(reinterpret_cast<const char*>(&img.data[i * img.bpp]), ch);
    return;
  }
  size_t stride = size_t(img.w) * img.bpp;
  std::vector<unsigned char> raw((stride + 1) * img.h);
  for (int y = 0; y < img.h; ++y) {
    raw[y * (stride + 1)] = 0;
    std::memcpy(&raw[y * (stride + 1) + 1], &img.data[y * stride], stride);
  }
  uLongf zlen = compressBound(raw.size());
  std::vector<unsigned char> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), raw.size(), 6) != Z_OK)
    throw std::runtime_error("PNG compression failed");
  auto chunk = [&](const char* type, const unsigned char* d, size_t n) {
    std::string c;
    put32(c, uint32_t(n));
    c.append(type, 4);
    c.append(reinterpret_cast<const char*>(d), n);
    uLong crc = crc32(0L, reinterpret_cast<const Bytef*>(c.data() + 4), uInt(n + 4));
    put32(c, uint32_t(crc));
    out.write(c.data(), std::streamsize(c.size()));
  };
  static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  out.write(reinterpret_cast<const char*>(sig), 8);
  unsigned char ihdr[13];
  std::string hw;
  put32(hw, uint32_t(img.w));
  put32(hw, uint32_t(img.h));
  std::memcpy(ihdr, hw.data(), 8);
  ihdr[8] = 8;
  ihdr[9] = img.bpp == 1 ? 0 : img.bpp == 3 ? 2 : 6;
  ihdr[10] = ihdr[11] = ihdr[12] = 0;
  chunk("IHDR", ihdr, 13);
  chunk("IDAT", z.data(), zlen);
  chunk("IEND", nullptr, 0);
}

void write_luma(const std::string& path, const float* luma, int w, int h) {
  ImageData img(w, h, 1);
  for (size_t i = 0, n = size_t(w) * h; i < n; ++i) {
    float v = std::min(1.0f, std::max(0.0f, luma[i]));
    img.data[i] = static_cast<unsigned char>(std::lround(v * 255.0f));
  }
  write(path, img);
}

}  // namespace image
}  // namespace srcnn
