// Baseline JPEG decoder (see jpeg.h). ITU T.81 Annex F sequential DCT with
// Huffman coding: DQT (8/16-bit), DHT, SOF0/SOF1, SOS, DRI + RSTn, any
// sampling factors up to 4x4, 1 or 3 components. Float separable IDCT,
// centred bilinear chroma upsampling, JFIF YCbCr -> RGB.
#include "jpeg.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <iterator>
#include <stdexcept>

namespace dmlc {

namespace {

const int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                         12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                         35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                         58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
  uint8_t count[17] = {0};
  uint8_t sym[256] = {0};
  int mincode[17], maxcode[18], valptr[17];
  uint8_t lut_len[256];  // 8-bit lookahead: code length (0 = longer than 8)
  uint8_t lut_sym[256];
  bool present = false;
  void build() {
    int code = 0, k = 0;
    for (int l = 1; l <= 16; ++l) {
      valptr[l] = k;
      mincode[l] = code;
      code += count[l];
      k += count[l];
      maxcode[l] = count[l] ? code - 1 : -1;
      code <<= 1;
    }
    maxcode[17] = 0x7fffffff;
    std::memset(lut_len, 0, sizeof(lut_len));
    code = 0;
    k = 0;
    for (int l = 1; l <= 8; ++l) {
      for (int i = 0; i < count[l]; ++i, ++k, ++code) {
        const int shift = 8 - l;
        for (int j = 0; j < (1 << shift); ++j) {
          lut_len[(code << shift) | j] = (uint8_t)l;
          lut_sym[(code << shift) | j] = sym[k];
        }
      }
      code <<= 1;
    }
    present = true;
  }
};

struct Comp {
  int id = 0, h = 1, v = 1, tq = 0;
  int td = 0, ta = 0;
  int bw = 0, bh = 0;  // blocks per line / column in the plane
  std::vector<uint8_t> plane;  // bw*8 x bh*8
  int pred = 0;
};

class BitReader {
 public:
  BitReader(const uint8_t* p, const uint8_t* end) : p_(p), end_(end) {}
  void reset() {
    acc_ = 0;
    nbits_ = 0;
    marker_ = false;
  }
  // Make sure >= n bits (n <= 24) are buffered; past a marker feed zeros.
  void fill(int n) {
    while (nbits_ < n) {
      uint32_t byte = 0;
      if (!marker_ && p_ < end_) {
        byte = *p_;
        if (byte == 0xFF) {
          const uint8_t nx = (p_ + 1 < end_) ? p_[1] : 0;
          if (nx == 0x00) {
            p_ += 2;
          } else {
            marker_ = true;  // leave the marker for the caller
            byte = 0;
          }
        } else {
          ++p_;
        }
      }
      acc_ |= byte << (24 - nbits_);
      nbits_ += 8;
    }
  }
  uint32_t peek(int n) {
    fill(n);
    return acc_ >> (32 - n);
  }
  void skip(int n) {
    acc_ <<= n;
    nbits_ -= n;
  }
  int bits(int n) {
    if (n == 0) return 0;
    uint32_t v = peek(n);
    skip(n);
    return (int)v;
  }
  const uint8_t* pos() const { return p_; }
  void seek(const uint8_t* p) {
    p_ = p;
    reset();
  }

 private:
  const uint8_t* p_;
  const uint8_t* end_;
  uint32_t acc_ = 0;
  int nbits_ = 0;
  bool marker_ = false;
};

int decode_huff(const Huff& h, BitReader& br) {
  const uint32_t look = br.peek(8);
  if (h.lut_len[look]) {
    br.skip(h.lut_len[look]);
    return h.lut_sym[look];
  }
  int code = 0;
  for (int l = 1; l <= 16; ++l) {
    code = (code << 1) | br.bits(1);
    if (h.maxcode[l] >= 0 && code <= h.maxcode[l] && code >= h.mincode[l])
      return h.sym[h.valptr[l] + code - h.mincode[l]];
  }
  throw std::runtime_error("jpeg: bad huffman code");
}

inline int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }

struct IdctTable {
  float c[8][8];
  IdctTable() {
    for (int x = 0; x < 8; ++x)
      for (int u = 0; u < 8; ++u) {
        const double cu = u == 0 ? std::sqrt(0.5) : 1.0;
        c[x][u] = (float)(0.5 * cu * std::cos((2 * x + 1) * u * M_PI / 16.0));
      }
  }
};

void idct8x8(const float* in, uint8_t* out, int stride) {
  static const IdctTable T;
  float tmp[64];
  for (int y = 0; y < 8; ++y)  // rows: over u
    for (int x = 0; x < 8; ++x) {
      float s = 0;
      for (int u = 0; u < 8; ++u) s += T.c[x][u] * in[y * 8 + u];
      tmp[y * 8 + x] = s;
    }
  for (int x = 0; x < 8; ++x)
    for (int y = 0; y < 8; ++y) {
      float s = 0;
      for (int v = 0; v < 8; ++v) s += T.c[y][v] * tmp[v * 8 + x];
      const int val = (int)std::lround(s + 128.f);
      out[y * stride + x] = (uint8_t)std::min(255, std::max(0, val));
    }
}

uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

}  // namespace

Image decode_jpeg(const uint8_t* data, size_t size) {
  const uint8_t* p = data;
  const uint8_t* end = data + size;
  if (size < 4 || p[0] != 0xFF || p[1] != 0xD8) throw std::runtime_error("jpeg: missing SOI");
  p += 2;
  uint16_t qt[4][64] = {};
  Huff dc[4], ac[4];
  std::vector<Comp> comps;
  int W = 0, H = 0, hmax = 1, vmax = 1, restart = 0;
  bool frame = false, scanned = false;
  while (p + 4 <= end) {
    if (p[0] != 0xFF) {
      ++p;
      continue;
    }
    const uint8_t m = p[1];
    p += 2;
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7) || m == 0xFF) continue;
    if (m == 0xD9) break;  // EOI
    if (p + 2 > end) break;
    const int len = be16(p);
    const uint8_t* seg = p + 2;
    const uint8_t* seg_end = p + len;
    if (seg_end > end) throw std::runtime_error("jpeg: truncated segment");
    switch (m) {
      case 0xDB: {  // DQT
        const uint8_t* q = seg;
        while (q < seg_end) {
          const int pq = q[0] >> 4, tq = q[0] & 15;
          ++q;
          if (tq > 3) throw std::runtime_error("jpeg: bad DQT");
          for (int i = 0; i < 64; ++i) {
            qt[tq][i] = pq ? be16(q + 2 * i) : q[i];
          }
          q += pq ? 128 : 64;
        }
        break;
      }
      case 0xC4: {  // DHT
        const uint8_t* q = seg;
        while (q < seg_end) {
          const int tc = q[0] >> 4, th = q[0] & 15;
          if (th > 3 || tc > 1) throw std::runtime_error("jpeg: bad DHT");
          Huff& h = tc ? ac[th] : dc[th];
          int total = 0;
          for (int l = 1; l <= 16; ++l) {
            h.count[l] = q[l];
            total += q[l];
          }
          if (total > 256) throw std::runtime_error("jpeg: bad DHT count");
          std::memcpy(h.sym, q + 17, total);
          h.build();
          q += 17 + total;
        }
        break;
      }
      case 0xC0:
      case 0xC1: {  // SOF0 / SOF1
        if (seg[0] != 8) throw std::runtime_error("jpeg: only 8-bit precision supported");
        H = be16(seg + 1);
        W = be16(seg + 3);
        const int nc = seg[5];
        if (W <= 0 || H <= 0 || (nc != 1 && nc != 3)) throw std::runtime_error("jpeg: unsupported frame");
        comps.resize(nc);
        for (int i = 0; i < nc; ++i) {
          comps[i].id = seg[6 + 3 * i];
          comps[i].h = seg[7 + 3 * i] >> 4;
          comps[i].v = seg[7 + 3 * i] & 15;
          comps[i].tq = seg[8 + 3 * i] & 3;
          if (comps[i].h < 1 || comps[i].h > 4 || comps[i].v < 1 || comps[i].v > 4)
            throw std::runtime_error("jpeg: bad sampling factors");
          hmax = std::max(hmax, comps[i].h);
          vmax = std::max(vmax, comps[i].v);
        }
        const int mcux = (W + 8 * hmax - 1) / (8 * hmax), mcuy = (H + 8 * vmax - 1) / (8 * vmax);
        for (auto& c : comps) {
          c.bw = mcux * c.h;
          c.bh = mcuy * c.v;
          c.plane.assign((size_t)c.bw * 8 * c.bh * 8, 0);
        }
        frame = true;
        break;
      }
      case 0xC2:
      case 0xC3:
      case 0xC5:
      case 0xC6:
      case 0xC7:
      case 0xC9:
      case 0xCA:
      case 0xCB:
      case 0xCD:
      case 0xCE:
      case 0xCF:
        throw std::runtime_error("jpeg: progressive/lossless/arithmetic coding not supported");
      case 0xDD:
        restart = be16(seg);
        break;
      case 0xDA: {  // SOS
        if (!frame) throw std::runtime_error("jpeg: SOS before SOF");
        const int ns = seg[0];
        std::vector<Comp*> sc;
        for (int i = 0; i < ns; ++i) {
          const int cid = seg[1 + 2 * i];
          Comp* c = nullptr;
          for (auto& x : comps)
            if (x.id == cid) c = &x;
          if (!c) throw std::runtime_error("jpeg: bad scan component");
          c->td = seg[2 + 2 * i] >> 4;
          c->ta = seg[2 + 2 * i] & 15;
          if (!dc[c->td & 3].present || !ac[c->ta & 3].present) throw std::runtime_error("jpeg: missing huffman table");
          sc.push_back(c);
        }
        BitReader br(seg_end, end);
        float blk[64];
        int mcus_left = restart;
        auto decode_block = [&](Comp& c, uint8_t* dst, int stride) {
          std::memset(blk, 0, sizeof(blk));
          const uint16_t* q = qt[c.tq];
          const int t = decode_huff(dc[c.td], br);
          c.pred += t ? extend(br.bits(t), t) : 0;
          blk[0] = (float)(c.pred * q[0]);
          for (int k = 1; k < 64;) {
            const int rs = decode_huff(ac[c.ta], br);
            const int r = rs >> 4, s = rs & 15;
            if (s == 0) {
              if (r != 15) break;
              k += 16;
              continue;
            }
            k += r;
            if (k > 63) break;
            blk[kZigzag[k]] = (float)(extend(br.bits(s), s) * q[k]);
            ++k;
          }
          idct8x8(blk, dst, stride);
        };
        auto handle_restart = [&]() {
          if (!restart) return;
          if (mcus_left == 0) {
            // realign to the RSTn marker and reset predictors
            const uint8_t* q = br.pos();
            while (q + 1 < end && !(q[0] == 0xFF && q[1] >= 0xD0 && q[1] <= 0xD7)) ++q;
            if (q + 1 < end) q += 2;
            br.seek(q);
            for (auto* c : sc) c->pred = 0;
            mcus_left = restart;
          }
          --mcus_left;
        };
        if (ns == 1) {  // non-interleaved: blocks cover the component's own size
          Comp& c = *sc[0];
          const int cw = (W * c.h + hmax - 1) / hmax, ch = (H * c.v + vmax - 1) / vmax;
          const int nbx = (cw + 7) / 8, nby = (ch + 7) / 8;
          for (int by = 0; by < nby; ++by)
            for (int bx = 0; bx < nbx; ++bx) {
              handle_restart();
              decode_block(c, c.plane.data() + (size_t)by * 8 * c.bw * 8 + bx * 8, c.bw * 8);
            }
        } else {
          const int mcux = (W + 8 * hmax - 1) / (8 * hmax), mcuy = (H + 8 * vmax - 1) / (8 * vmax);
          for (int my = 0; my < mcuy; ++my)
            for (int mx = 0; mx < mcux; ++mx) {
              handle_restart();
              for (auto* cp : sc) {
                Comp& c = *cp;
                for (int v = 0; v < c.v; ++v)
                  for (int h = 0; h < c.h; ++h) {
                    const int bx = mx * c.h + h, by = my * c.v + v;
                    decode_block(c, c.plane.data() + (size_t)by * 8 * c.bw * 8 + bx * 8, c.bw * 8);
                  }
              }
            }
        }
        scanned = true;
        // continue after the entropy-coded data: find the next marker
        const uint8_t* q = br.pos();
        while (q + 1 < end && !(q[0] == 0xFF && q[1] != 0x00 && !(q[1] >= 0xD0 && q[1] <= 0xD7))) ++q;
        p = q;
        continue;
      }
      default:
        break;  // APPn, COM, ... skipped
    }
    p = seg_end;
  }
  if (!frame || !scanned) throw std::runtime_error("jpeg: no image data");

  Image img;
  img.width = W;
  img.height = H;
  img.rgb.resize((size_t)W * H * 3);
  auto sample = [&](const Comp& c, int x, int y) -> float {
    const int pw = c.bw * 8;
    if (c.h == hmax && c.v == vmax) return c.plane[(size_t)y * pw + x];
    // centred bilinear upsampling of a subsampled plane
    const float sx = (x + 0.5f) * c.h / hmax - 0.5f, sy = (y + 0.5f) * c.v / vmax - 0.5f;
    const int cw = (W * c.h + hmax - 1) / hmax, ch = (H * c.v + vmax - 1) / vmax;
    const float fx = std::min(std::max(sx, 0.f), (float)(cw - 1));
    const float fy = std::min(std::max(sy, 0.f), (float)(ch - 1));
    const int x0 = (int)fx, y0 = (int)fy;
    const int x1 = std::min(x0 + 1, cw - 1), y1 = std::min(y0 + 1, ch - 1);
    const float ax = fx - x0, ay = fy - y0;
    const float a = c.plane[(size_t)y0 * pw + x0], b = c.plane[(size_t)y0 * pw + x1];
    const float d = c.plane[(size_t)y1 * pw + x0], e = c.plane[(size_t)y1 * pw + x1];
    return (a + (b - a) * ax) * (1 - ay) + (d + (e - d) * ax) * ay;
  };
  auto clamp8 = [](float v) { return (uint8_t)std::min(255.f, std::max(0.f, std::round(v))); };
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      uint8_t* o = &img.rgb[((size_t)y * W + x) * 3];
      const float Y = sample(comps[0], x, y);
      if (comps.size() == 1) {
        o[0] = o[1] = o[2] = clamp8(Y);
      } else {
        const float cb = sample(comps[1], x, y) - 128.f, cr = sample(comps[2], x, y) - 128.f;
        o[0] = clamp8(Y + 1.402f * cr);
        o[1] = clamp8(Y - 0.344136f * cb - 0.714136f * cr);
        o[2] = clamp8(Y + 1.772f * cb);
      }
    }
  return img;
}

Image decode_jpeg_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  return decode_jpeg(buf.data(), buf.size());
}

}  // namespace dmlc
