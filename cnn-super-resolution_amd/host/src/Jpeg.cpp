// JPEG decoder of the cnn_sr host (ITU-T T.81 / JFIF), for the reference's
// image inputs: the reference decodes every image with its vendored
// stb_image (src/opencl/UtilsOpenCL.cpp:88-95 load_image), its training
// sample pairs are `*_large.jpg` / `*_small.jpg` (src/Main_cl.cpp:267-301,
// generate_training_samples.py:36-41) and its SwapLuma spec reads
// test/data/color_grid2.jpg, a progressive JPEG.
//
// An independent implementation of the published algorithms:
//   - baseline and extended sequential Huffman (SOF0 / SOF1) and progressive
//     Huffman (SOF2: spectral selection and successive approximation, DC and
//     AC, first and refinement scans, EOB runs -- T.81 G.1.2), 8-bit samples;
//   - restart intervals (DRI / RSTn), component sampling factors 1..4 in whole ratios;
//   - dequantisation and the 8x8 inverse DCT (T.81 A.3.3) in the published
//     integer Loeffler-Ligtenberg-Moschytz factorisation (the IJG "islow"
//     algorithm), rounded and clamped;
//   - chroma upsampling: the triangle ("fancy") filter for 2:1 ratios --
//     3/4 of the nearer and 1/4 of the farther sample, vertically then
//     horizontally -- replication for the other ratios;
//   - YCbCr -> RGB per JFIF (R = Y + 1.402 Cr', G = Y - 0.34414 Cb' -
//     0.71414 Cr', B = Y + 1.772 Cb') in 16-bit fixed point, or no transform
//     for Adobe RGB.
// Not supported (an IOException says so): arithmetic coding, lossless and
// hierarchical modes, 12-bit samples, CMYK / YCCK.
// The reference's stb_image uses a different fixed-point inverse DCT and
// color conversion, a few LSB apart (tests/test_image_codecs.py measures it
// against the reference's own fixture and against PIL's libjpeg).
#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "Context.hpp"
#include "Image.hpp"

namespace srcnn {
namespace image {

namespace {

const int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                         12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                         35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                         58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

[[noreturn]] void bad(const std::string& why) { throw IOException("JPEG: " + why); }

/** Canonical Huffman table (T.81 C / F.2.2.3), decoded by code length. */
struct Huffman {
  bool present = false;
  // for every code length L: smallest code, count, index of its first value
  int mincode[17] = {0}, maxcode[18] = {0}, valptr[17] = {0};
  std::vector<uint8_t> vals;
  // fast path: the first 9 bits -> (length << 8 | value), 0 = longer code
  uint16_t fast[512] = {0};

  void build(const uint8_t counts[16], const uint8_t* v, int nv) {
    vals.assign(v, v + nv);
    int code = 0, k = 0;
    std::memset(fast, 0, sizeof(fast));
    for (int len = 1; len <= 16; ++len) {
      valptr[len] = k;
      mincode[len] = code;
      for (int i = 0; i < counts[len - 1]; ++i, ++k, ++code) {
        if (code >= (1 << len)) bad("bad Huffman table");  // over-subscribed code lengths
        if (len <= 9) {
          const int shift = 9 - len;
          for (int f = code << shift; f < ((code + 1) << shift); ++f)
            fast[f] = uint16_t((len << 8) | vals[k]);
        }
      }
      maxcode[len] = counts[len - 1] ? code - 1 : -1;
      if (code > (1 << len)) bad("bad Huffman table");
      code <<= 1;
    }
    maxcode[17] = 0x7fffffff;
    present = true;
  }
};

struct Component {
  int id = 0, h = 1, v = 1, tq = 0;
  int bw = 0, bh = 0;      // blocks per row / column in the MCU-padded plane
  int cw = 0, ch = 0;      // component size in samples (unpadded)
  int dc_tab = 0, ac_tab = 0;
  int dc_pred = 0;
  std::vector<int16_t> coef;  // bw * bh blocks of 64 coefficients, natural order
  std::vector<uint8_t> pixels;  // bw*8 x bh*8 after the inverse DCT
};

class Decoder {
 public:
  Decoder(const std::vector<unsigned char>& f) : f_(f) {}

  void decode(ImageData& img) {
    if (f_.size() < 4 || f_[0] != 0xFF || f_[1] != 0xD8) bad("missing SOI marker");
    pos_ = 2;
    bool frame = false, done = false;
    while (!done) {
      const int m = next_marker();
      switch (m) {
        case 0xC0: case 0xC1: read_sof(false); frame = true; break;
        case 0xC2: read_sof(true); frame = true; break;
        case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB:
        case 0xCD: case 0xCE: case 0xCF:
          bad("unsupported coding (lossless / hierarchical / arithmetic)");
        case 0xC4: read_dht(); break;
        case 0xDB: read_dqt(); break;
        case 0xDD: read_dri(); break;
        case 0xDA:
          if (!frame) bad("scan before frame header");
          read_sos();
          break;
        case 0xD9: done = true; break;
        case 0xEE: read_adobe(); break;
        default:
          if ((m >= 0xE0 && m <= 0xEF) || m == 0xFE || m == 0xDC || m == 0xDE || m == 0xDF) skip_segment();
          else if (m >= 0xD0 && m <= 0xD7) { /* stray restart marker */ }
          else bad("unexpected marker");
      }
      if (pos_ >= f_.size()) break;  // tolerate a missing EOI
    }
    if (!frame) bad("no frame");
    finish(img);
  }

 private:
  const std::vector<unsigned char>& f_;
  size_t pos_ = 0;
  int width_ = 0, height_ = 0, hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0;
  bool progressive_ = false;
  int restart_ = 0;
  int adobe_transform_ = -1;
  std::vector<Component> comp_;
  std::array<std::array<uint16_t, 64>, 4> qt_{};
  Huffman dc_[4], ac_[4];
  // bit reader
  uint32_t bits_ = 0;
  int nbits_ = 0;
  bool marker_hit_ = false;
  int eobrun_ = 0;

  int u8() {
    if (pos_ >= f_.size()) bad("truncated file");
    return f_[pos_++];
  }
  int u16() {
    const int a = u8();
    return (a << 8) | u8();
  }
  int next_marker() {
    int c = u8();
    while (c != 0xFF) c = u8();  // skip garbage between segments
    while (c == 0xFF) c = u8();  // fill bytes
    return c;
  }
  void skip_segment() {
    const int len = u16();
    if (len < 2 || pos_ + len - 2 > f_.size()) bad("bad segment length");
    pos_ += len - 2;
  }
  void read_adobe() {
    const size_t start = pos_;
    const int len = u16();
    if (len < 2 || start + len > f_.size()) bad("bad segment length");
    // the transform flag is byte 11 of the payload (start + 13): the whole
    // declared segment is inside the file, and it is long enough to hold it
    if (len >= 14 && std::memcmp(&f_[pos_], "Adobe", 5) == 0) adobe_transform_ = f_[start + 13];
    pos_ = start + len;
  }
  void read_dqt() {
    int len = u16() - 2;
    while (len > 0) {
      const int pq_tq = u8();
      const int pq = pq_tq >> 4, tq = pq_tq & 15;
      if (tq > 3 || pq > 1) bad("bad quantisation table");
      for (int i = 0; i < 64; ++i) qt_[tq][kZigzag[i]] = uint16_t(pq ? u16() : u8());
      len -= 1 + 64 * (pq + 1);
    }
    if (len != 0) bad("bad DQT length");
  }
  void read_dht() {
    int len = u16() - 2;
    while (len > 0) {
      const int tc_th = u8();
      const int tc = tc_th >> 4, th = tc_th & 15;
      if (tc > 1 || th > 3) bad("bad Huffman table id");
      uint8_t counts[16];
      int n = 0;
      for (int i = 0; i < 16; ++i) n += counts[i] = uint8_t(u8());
      if (n > 256 || pos_ + n > f_.size()) bad("bad Huffman table");
      (tc ? ac_[th] : dc_[th]).build(counts, &f_[pos_], n);
      pos_ += n;
      len -= 17 + n;
    }
    if (len != 0) bad("bad DHT length");
  }
  void read_dri() {
    if (u16() != 4) bad("bad DRI length");
    restart_ = u16();
  }
  void read_sof(bool progressive) {
    if (!comp_.empty()) bad("more than one frame");
    progressive_ = progressive;
    const int len = u16();
    if (u8() != 8) bad("only 8-bit samples are supported");
    height_ = u16();
    width_ = u16();
    const int nc = u8();
    if (len != 8 + 3 * nc) bad("bad SOF length");
    if (width_ <= 0 || height_ <= 0) bad("image without size (DNL is not supported)");
    if (nc != 1 && nc != 3) bad("only grayscale and 3-component images are supported");
    comp_.resize(nc);
    for (auto& c : comp_) {
      c.id = u8();
      const int hv = u8();
      c.h = hv >> 4;
      c.v = hv & 15;
      c.tq = u8();
      if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) bad("bad component parameters");
      hmax_ = std::max(hmax_, c.h);
      vmax_ = std::max(vmax_, c.v);
    }
    // upsample() maps luma column x to chroma column x / (hmax / h): only
    // whole sampling ratios are supported (libjpeg's "fancy" ratios are not)
    for (const auto& c : comp_)
      if (hmax_ % c.h != 0 || vmax_ % c.v != 0) bad("unsupported (non-integral) sampling ratio");
    check_dims(width_, height_, nc);
    // every 8x8 luma block costs at least one bit of entropy-coded data (its DC
    // code), so a file much smaller than that cannot hold the image: reject it
    // before allocating the coefficient planes
    if (f_.size() < (size_t(width_) * height_ / 64) / 64) bad("file too small for its frame size");
    mcux_ = (width_ + 8 * hmax_ - 1) / (8 * hmax_);
    mcuy_ = (height_ + 8 * vmax_ - 1) / (8 * vmax_);
    for (auto& c : comp_) {
      c.cw = (width_ * c.h + hmax_ - 1) / hmax_;
      c.ch = (height_ * c.v + vmax_ - 1) / vmax_;
      c.bw = mcux_ * c.h;
      c.bh = mcuy_ * c.v;
      c.coef.assign(size_t(c.bw) * c.bh * 64, 0);
    }
  }

  // ---- entropy-coded data ----
  void reset_bits() {
    bits_ = 0;
    nbits_ = 0;
    marker_hit_ = false;
  }
  void fill() {
    while (nbits_ <= 24) {
      int b = 0;
      if (!marker_hit_ && pos_ < f_.size()) {
        b = f_[pos_];
        if (b == 0xFF) {
          const int nx = pos_ + 1 < f_.size() ? f_[pos_ + 1] : 0xD9;
          if (nx == 0x00) {
            pos_ += 2;  // stuffed zero byte
          } else {
            marker_hit_ = true;  // a marker: feed zeros (T.81 F.2.2.5 note)
            b = 0;
          }
        } else {
          ++pos_;
        }
      }
      bits_ |= uint32_t(b) << (24 - nbits_);
      nbits_ += 8;
    }
  }
  int bit() {
    if (nbits_ < 1) fill();
    const int b = int(bits_ >> 31);
    bits_ <<= 1;
    --nbits_;
    return b;
  }
  int getbits(int n) {
    if (n == 0) return 0;
    if (nbits_ < n) fill();
    const int v = int(bits_ >> (32 - n));
    bits_ <<= n;
    nbits_ -= n;
    return v;
  }
  // value of an n-bit magnitude category (T.81 F.2.2.1 EXTEND)
  int receive_extend(int n) {
    if (n == 0) return 0;
    if (n > 16) bad("bad coefficient size");
    const int v = getbits(n);
    return v < (1 << (n - 1)) ? v - (1 << n) + 1 : v;
  }
  int decode_huff(const Huffman& h) {
    if (!h.present) bad("missing Huffman table");
    if (nbits_ < 16) fill();
    const uint16_t fv = h.fast[bits_ >> 23];
    if (fv) {
      const int len = fv >> 8;
      bits_ <<= len;
      nbits_ -= len;
      return fv & 0xFF;
    }
    int code = 0;
    for (int len = 1; len <= 16; ++len) {
      code = (code << 1) | bit();
      if (code <= h.maxcode[len]) return h.vals[h.valptr[len] + code - h.mincode[len]];
    }
    bad("bad Huffman code");
  }
  void restart_marker() {
    // byte-align, then expect RSTn
    reset_bits();
    while (pos_ + 1 < f_.size() && !(f_[pos_] == 0xFF && f_[pos_ + 1] >= 0xD0 && f_[pos_ + 1] <= 0xD7)) ++pos_;
    if (pos_ + 1 < f_.size()) pos_ += 2;
    for (auto& c : comp_) c.dc_pred = 0;
    eobrun_ = 0;
  }

  // ---- block decoders (coefficients in natural order, quantised) ----
  void block_baseline(Component& c, int16_t* blk) {
    const int t = decode_huff(dc_[c.dc_tab]);
    c.dc_pred = int(uint32_t(c.dc_pred) + uint32_t(receive_extend(t)));  // wraps on corrupt data
    blk[0] = int16_t(c.dc_pred);
    for (int k = 1; k < 64;) {
      const int rs = decode_huff(ac_[c.ac_tab]);
      const int r = rs >> 4, s = rs & 15;
      if (s == 0) {
        if (r != 15) break;  // EOB
        k += 16;
        continue;
      }
      k += r;
      if (k > 63) bad("coefficient index out of range");
      blk[kZigzag[k++]] = int16_t(receive_extend(s));
    }
  }
  void block_dc_first(Component& c, int16_t* blk, int al) {
    const int t = decode_huff(dc_[c.dc_tab]);
    c.dc_pred = int(uint32_t(c.dc_pred) + uint32_t(receive_extend(t)));
    blk[0] = int16_t(int64_t(c.dc_pred) * (int64_t(1) << al));
  }
  void block_dc_refine(int16_t* blk, int al) {
    if (bit()) blk[0] = int16_t(blk[0] | (1 << al));
  }
  void block_ac_first(Component& c, int16_t* blk, int ss, int se, int al) {
    if (eobrun_ > 0) {
      --eobrun_;
      return;
    }
    for (int k = ss; k <= se;) {
      const int rs = decode_huff(ac_[c.ac_tab]);
      const int r = rs >> 4, s = rs & 15;
      if (s == 0) {
        if (r < 15) {  // EOB run of 2^r + extra bits blocks, this one included
          eobrun_ = (1 << r) - 1 + getbits(r);
          break;
        }
        k += 16;
        continue;
      }
      k += r;
      if (k > 63) bad("coefficient index out of range");
      blk[kZigzag[k++]] = int16_t(receive_extend(s) * (1 << al));
    }
  }
  // T.81 G.1.2.3: correction bits for already-nonzero coefficients, new
  // coefficients of magnitude 1 << al placed after `r` zero-history ones
  void block_ac_refine(Component& c, int16_t* blk, int ss, int se, int al) {
    const int p1 = 1 << al, m1 = -p1;
    int k = ss;
    auto refine = [&](int16_t& v) {
      if (bit() && (v & p1) == 0) v = int16_t(v >= 0 ? v + p1 : v + m1);
    };
    if (eobrun_ == 0) {
      for (; k <= se;) {
        const int rs = decode_huff(ac_[c.ac_tab]);
        int r = rs >> 4;
        const int s = rs & 15;
        int value = 0;
        if (s == 0) {
          if (r < 15) {
            eobrun_ = (1 << r) + getbits(r);
            break;  // the rest of this block is refined below as part of the run
          }
          // r == 15: skip 16 zero-history coefficients (refining the nonzero ones)
        } else {
          if (s != 1) bad("bad refinement value");
          value = bit() ? p1 : m1;
        }
        while (k <= se) {
          int16_t& v = blk[kZigzag[k]];
          if (v != 0) {
            refine(v);
          } else {
            if (r == 0) {
              if (value) v = int16_t(value);
              ++k;
              break;
            }
            --r;
          }
          ++k;
        }
      }
    }
    if (eobrun_ > 0) {
      for (; k <= se; ++k) {
        int16_t& v = blk[kZigzag[k]];
        if (v != 0) refine(v);
      }
      --eobrun_;
    }
  }

  void read_sos() {
    const int len = u16();
    const int ns = u8();
    if (ns < 1 || ns > 4 || len != 6 + 2 * ns) bad("bad SOS");
    std::vector<Component*> sc;
    for (int i = 0; i < ns; ++i) {
      const int id = u8(), tab = u8();
      Component* c = nullptr;
      for (auto& cc : comp_)
        if (cc.id == id) c = &cc;
      if (!c) bad("scan of an unknown component");
      c->dc_tab = tab >> 4;
      c->ac_tab = tab & 15;
      if (c->dc_tab > 3 || c->ac_tab > 3) bad("bad Huffman table id");
      sc.push_back(c);
    }
    const int ss = u8(), se = u8(), ahal = u8();
    const int ah = ahal >> 4, al = ahal & 15;
    if (progressive_) {
      if (ss > se || se > 63 || (ss == 0 && se != 0) || (ss > 0 && ns != 1) || al > 13)
        bad("bad progressive scan parameters");
    } else if (ss != 0 || se != 63 || ahal != 0) {
      bad("bad sequential scan parameters");
    }
    reset_bits();
    eobrun_ = 0;
    for (auto* c : sc) c->dc_pred = 0;

    auto do_block = [&](Component& c, int bx, int by) {
      int16_t* blk = &c.coef[(size_t(by) * c.bw + bx) * 64];
      if (!progressive_) block_baseline(c, blk);
      else if (ss == 0) ah == 0 ? block_dc_first(c, blk, al) : block_dc_refine(blk, al);
      else ah == 0 ? block_ac_first(c, blk, ss, se, al) : block_ac_refine(c, blk, ss, se, al);
    };
    int mcu = 0;
    if (ns == 1) {
      // non-interleaved: the component's own block grid (T.81 A.2.2)
      Component& c = *sc[0];
      const int w = (c.cw + 7) / 8, h = (c.ch + 7) / 8;
      for (int by = 0; by < h; ++by)
        for (int bx = 0; bx < w; ++bx) {
          if (restart_ && mcu && mcu % restart_ == 0) restart_marker();
          do_block(c, bx, by);
          ++mcu;
        }
    } else {
      for (int my = 0; my < mcuy_; ++my)
        for (int mx = 0; mx < mcux_; ++mx) {
          if (restart_ && mcu && mcu % restart_ == 0) restart_marker();
          for (auto* c : sc)
            for (int y = 0; y < c->v; ++y)
              for (int x = 0; x < c->h; ++x) do_block(*c, mx * c->h + x, my * c->v + y);
          ++mcu;
        }
    }
    // leave the reader at the next marker
    reset_bits();
    while (pos_ + 1 < f_.size() && !(f_[pos_] == 0xFF && f_[pos_ + 1] != 0x00 &&
                                     !(f_[pos_ + 1] >= 0xD0 && f_[pos_ + 1] <= 0xD7)))
      ++pos_;
  }

  // ---- reconstruction ----
  // Inverse DCT: the integer Loeffler-Ligtenberg-Moschytz factorisation as
  // published with the IJG software ("islow": 13-bit constants, 2 extra bits
  // between the column and the row pass, rounding at the end of each pass),
  // so the pixels are those of libjpeg's default decoder.
  static int fix13(double x) { return int(x * 8192.0 + 0.5); }
  static void idct_block(const int16_t* in, const uint16_t* q, uint8_t* out, int stride) {
    static const int c0298 = fix13(0.298631336), c0390 = fix13(0.390180644),
                     c0541 = fix13(0.541196100), c0765 = fix13(0.765366865),
                     c0899 = fix13(0.899976223), c1175 = fix13(1.175875602),
                     c1501 = fix13(1.501321110), c1847 = fix13(1.847759065),
                     c1961 = fix13(1.961570560), c2053 = fix13(2.053119869),
                     c2562 = fix13(2.562915447), c3072 = fix13(3.072711026);
    constexpr int kConst = 13, kPass1 = 2;
    auto descale = [](int64_t x, int n) { return int((x + (int64_t(1) << (n - 1))) >> n); };
    // one 1-D pass over 8 values v[0..7] at stride `st` of `src`, 8 outputs
    // (before the final descale) into o[]
    auto pass = [&](const int* v, int64_t o[8]) {
      int64_t z2 = v[2], z3 = v[6];
      int64_t z1 = (z2 + z3) * c0541;
      const int64_t t2 = z1 - z3 * c1847;
      const int64_t t3 = z1 + z2 * c0765;
      const int64_t t0 = (int64_t(v[0]) + v[4]) * (int64_t(1) << kConst);
      const int64_t t1 = (int64_t(v[0]) - v[4]) * (int64_t(1) << kConst);
      const int64_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
      int64_t a0 = v[7], a1 = v[5], a2 = v[3], a3 = v[1];
      z1 = a0 + a3;
      z2 = a1 + a2;
      z3 = a0 + a2;
      int64_t z4 = a1 + a3;
      const int64_t z5 = (z3 + z4) * c1175;
      a0 *= c0298;
      a1 *= c2053;
      a2 *= c3072;
      a3 *= c1501;
      z1 *= -c0899;
      z2 *= -c2562;
      z3 = z3 * -c1961 + z5;
      z4 = z4 * -c0390 + z5;
      a0 += z1 + z3;
      a1 += z2 + z4;
      a2 += z2 + z3;
      a3 += z1 + z4;
      o[0] = t10 + a3;
      o[7] = t10 - a3;
      o[1] = t11 + a2;
      o[6] = t11 - a2;
      o[2] = t12 + a1;
      o[5] = t12 - a1;
      o[3] = t13 + a0;
      o[4] = t13 - a0;
    };
    int ws[64];
    for (int x = 0; x < 8; ++x) {  // columns
      int v[8];
      bool ac = false;
      for (int y = 0; y < 8; ++y) {
        v[y] = int(in[y * 8 + x]) * int(q[y * 8 + x]);
        ac |= y > 0 && v[y] != 0;
      }
      if (!ac) {
        for (int y = 0; y < 8; ++y) ws[y * 8 + x] = v[0] * (1 << kPass1);
        continue;
      }
      int64_t o[8];
      pass(v, o);
      for (int y = 0; y < 8; ++y) ws[y * 8 + x] = descale(o[y], kConst - kPass1);
    }
    for (int y = 0; y < 8; ++y) {  // rows
      int64_t o[8];
      pass(&ws[y * 8], o);
      for (int x = 0; x < 8; ++x) {
        const int p = descale(o[x], kConst + kPass1 + 3) + 128;
        out[y * stride + x] = uint8_t(std::min(255, std::max(0, p)));
      }
    }
  }

  // plane of component c upsampled to the full image size
  std::vector<uint8_t> upsample(const Component& c) {
    const int pw = c.bw * 8;
    const int fx = hmax_ / c.h, fy = vmax_ / c.v;
    std::vector<uint8_t> out(size_t(width_) * height_);
    const bool tri_x = fx == 2 && hmax_ % c.h == 0, tri_y = fy == 2 && vmax_ % c.v == 0;
    const int sw = c.cw, sh = c.ch;
    auto S = [&](int x, int y) {
      x = std::min(std::max(x, 0), sw - 1);
      y = std::min(std::max(y, 0), sh - 1);
      return int(c.pixels[size_t(y) * pw + x]);
    };
    for (int y = 0; y < height_; ++y) {
      // vertical: weights 3/4 nearer, 1/4 farther source row (x4 kept)
      const int sy = y / fy;
      const int oy = tri_y ? (y % 2 == 0 ? sy - 1 : sy + 1) : sy;
      for (int x = 0; x < width_; ++x) {
        const int sx = x / fx;
        if (!tri_x && !tri_y && fx * c.h == hmax_ && fy * c.v == vmax_) {
          out[size_t(y) * width_ + x] = uint8_t(S(sx, sy));
          continue;
        }
        auto col = [&](int xx) { return tri_y ? 3 * S(xx, sy) + S(xx, oy) : 4 * S(xx, sy); };
        int v;
        if (tri_x) {
          const int ox = x % 2 == 0 ? sx - 1 : sx + 1;
          // (3 * near + far) of the column sums, /16, the rounding bias
          // alternating between the two outputs of a sample (no drift)
          v = tri_y ? (3 * col(sx) + col(ox) + (x % 2 == 0 ? 8 : 7)) >> 4
                    : (3 * col(sx) + col(ox) + (x % 2 == 0 ? 4 : 8)) >> 4;
        } else {
          v = (col(sx) + (tri_y ? (y % 2 == 0 ? 2 : 1) : 2)) >> 2;
        }
        out[size_t(y) * width_ + x] = uint8_t(std::min(255, std::max(0, v)));
      }
    }
    return out;
  }

  void finish(ImageData& img) {
    for (auto& c : comp_) {
      if (c.coef.empty()) bad("component without data");
      const int pw = c.bw * 8;
      c.pixels.assign(size_t(pw) * c.bh * 8, 0);
      for (int by = 0; by < c.bh; ++by)
        for (int bx = 0; bx < c.bw; ++bx)
          idct_block(&c.coef[(size_t(by) * c.bw + bx) * 64], qt_[c.tq].data(),
                     &c.pixels[size_t(by) * 8 * pw + bx * 8], pw);
    }
    const size_t n = size_t(width_) * height_;
    if (comp_.size() == 1) {
      img = ImageData(width_, height_, 1);
      const Component& c = comp_[0];
      for (int y = 0; y < height_; ++y)
        std::memcpy(&img.data[size_t(y) * width_], &c.pixels[size_t(y) * c.bw * 8], width_);
      return;
    }
    std::vector<uint8_t> planes[3];
    for (int i = 0; i < 3; ++i) planes[i] = upsample(comp_[i]);
    img = ImageData(width_, height_, 3);
    // Adobe transform 0 (or component ids 'R','G','B'): no color transform
    const bool rgb = adobe_transform_ == 0 ||
                     (comp_[0].id == 'R' && comp_[1].id == 'G' && comp_[2].id == 'B');
    // JFIF YCbCr -> RGB in 16-bit fixed point, rounded (IJG jdcolor tables)
    auto fx16 = [](double x) { return int64_t(x * 65536.0 + 0.5); };
    const int64_t kR = fx16(1.40200), kGb = fx16(0.34414), kGr = fx16(0.71414), kB = fx16(1.77200);
    const int64_t half = int64_t(1) << 15;
    auto clamp8 = [](int64_t v) { return uint8_t(std::min<int64_t>(255, std::max<int64_t>(0, v))); };
    for (size_t i = 0; i < n; ++i) {
      if (rgb) {
        for (int k = 0; k < 3; ++k) img.data[3 * i + k] = planes[k][i];
        continue;
      }
      const int64_t Y = planes[0][i], cb = int64_t(planes[1][i]) - 128, cr = int64_t(planes[2][i]) - 128;
      img.data[3 * i + 0] = clamp8(Y + ((kR * cr + half) >> 16));
      img.data[3 * i + 1] = clamp8(Y + ((-kGb * cb - kGr * cr + half) >> 16));
      img.data[3 * i + 2] = clamp8(Y + ((kB * cb + half) >> 16));
    }
  }
};

}  // namespace

void decode_jpeg(const std::vector<unsigned char>& f, ImageData& img) {
  Decoder d(f);
  d.decode(img);
}

}  // namespace image
}  // namespace srcnn
