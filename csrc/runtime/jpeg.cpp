// Baseline JPEG decoder (see jpeg.h). ITU T.81 Annex F sequential DCT with
// Huffman coding: DQT (8/16-bit), DHT, SOF0/SOF1, SOS, DRI + RSTn, any
// sampling factors up to 4x4, 1 or 3 components. Float separable IDCT,
// centred bilinear chroma upsampling, JFIF YCbCr -> RGB.
#include "jpeg.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <functional>
#include <immintrin.h>
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
  // AC fast path, kFastBits lookahead: a code AND its value bits resolved in
  // one lookup. Entry = value << 16 | run << 5 | bits consumed; 0 = slow path.
  static constexpr int kFastBits = 10;
  int32_t fast[1 << kFastBits];
  bool present = false;
  void build() {
    int code = 0, k = 0;
    for (int l = 1; l <= 16; ++l) {
      valptr[l] = k;
      mincode[l] = code;
      code += count[l];
      k += count[l];
      // an over-subscribed table (more codes than 2^l) would overflow the
      // lookup tables below (found by tests/test_fuzz_cpu.py)
      if (code > (1 << l)) throw std::runtime_error("jpeg: bad huffman table");
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
    std::memset(fast, 0, sizeof(fast));
    code = 0;
    k = 0;
    for (int l = 1; l <= 16; ++l) {
      for (int i = 0; i < count[l]; ++i, ++k, ++code) {
        const int rs = sym[k], r = rs >> 4, sz = rs & 15;
        if (l > kFastBits || sz == 0 || l + sz > kFastBits) continue;
        for (int v = 0; v < (1 << sz); ++v) {
          const int val = v < (1 << (sz - 1)) ? v - (1 << sz) + 1 : v;
          const int base = ((code << sz) | v) << (kFastBits - l - sz);
          for (int j = 0; j < (1 << (kFastBits - l - sz)); ++j)
            fast[base | j] = (int32_t)((uint32_t)val << 16) | (r << 5) | (l + sz);
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

// Entropy-coded segment reader: a 64-bit accumulator refilled a byte at a
// time up to 56 bits (byte stuffing 0xFF00 -> 0xFF removed; at a marker it
// feeds zeros and leaves the marker in place).
class BitReader {
 public:
  BitReader(const uint8_t* p, const uint8_t* end) : p_(p), end_(end) {}
  void reset() {
    acc_ = 0;
    nbits_ = 0;
    marker_ = false;
  }
  inline void refill() {
    // fast path: the next 8 bytes hold no 0xFF (no stuffing, no marker: ~97%
    // of windows in real entropy-coded data), so every whole byte that fits
    // goes in with one big-endian load
    if (!marker_ && end_ - p_ >= 8) {
      uint64_t w;
      std::memcpy(&w, p_, 8);
      const uint64_t x = ~w;  // a 0xFF byte of w is a zero byte of x
      if (!((x - 0x0101010101010101ULL) & ~x & 0x8080808080808080ULL)) {
        const int nb = (63 - nbits_) >> 3;  // whole bytes that fit
        if (nb > 0) {
          const int keep = nbits_ + 8 * nb;  // <= 64
          const uint64_t v = __builtin_bswap64(w) >> nbits_;
          acc_ |= keep == 64 ? v : v & ~(~0ULL >> keep);
          p_ += nb;
          nbits_ = keep;
        }
      }
    }
    while (nbits_ <= 56) {
      uint64_t byte = 0;
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
      acc_ |= byte << (56 - nbits_);
      nbits_ += 8;
    }
  }
  // n <= 16 bits
  inline uint32_t peek(int n) {
    if (nbits_ < n) refill();
    return (uint32_t)(acc_ >> (64 - n));
  }
  inline void skip(int n) {
    acc_ <<= n;
    nbits_ -= n;
  }
  inline int bits(int n) {
    if (n == 0) return 0;
    const uint32_t v = peek(n);
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
  uint64_t acc_ = 0;
  int nbits_ = 0;
  bool marker_ = false;
};

inline int decode_huff(const Huff& h, BitReader& br) {
  const uint32_t look = br.peek(16);
  const uint32_t l8 = look >> 8;
  if (h.lut_len[l8]) {
    br.skip(h.lut_len[l8]);
    return h.lut_sym[l8];
  }
  // canonical code longer than 8 bits: its top l bits are <= maxcode[l]
  for (int l = 9; l <= 16; ++l) {
    const int code = (int)(look >> (16 - l));
    if (h.maxcode[l] >= 0 && code <= h.maxcode[l]) {
      br.skip(l);
      return h.sym[h.valptr[l] + code - h.mincode[l]];
    }
  }
  throw std::runtime_error("jpeg: bad huffman code");
}

inline int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }

// AAN (Arai-Agui-Nakajima) scaled 8-point IDCT: 5 multiplies per 1-D
// transform; the per-coefficient AAN scale factors and the 1/8 of the 2-D
// transform are folded into the dequantisation table (aan_scale), so a
// block costs ~80 multiplies instead of the 1,024 of a direct separable
// transform. Columns first; a column whose AC terms are all zero (the common
// case after quantisation) is a constant.
struct AanScale {
  float f[64];
  AanScale() {
    double a[8];
    a[0] = 1.0;
    for (int k = 1; k < 8; ++k) a[k] = std::cos(k * M_PI / 16.0) * std::sqrt(2.0);
    for (int v = 0; v < 8; ++v)
      for (int u = 0; u < 8; ++u) f[v * 8 + u] = (float)(a[u] * a[v] / 8.0);
  }
};
const AanScale kAan;

// Eight 1-D transforms at once: lane j of every vector is column j (pass 1)
// or pixel row j (pass 2).
typedef float v8f __attribute__((vector_size(32)));

#define DMLC_IDCT8_LANES(in, o)                                                    \
  do {                                                                             \
    const v8f t10 = in[0] + in[4], t11 = in[0] - in[4];                            \
    const v8f t13 = in[2] + in[6], t12 = (in[2] - in[6]) * 1.414213562f - t13;     \
    const v8f e0 = t10 + t13, e3 = t10 - t13, e1 = t11 + t12, e2 = t11 - t12;      \
    const v8f z13 = in[5] + in[3], z10 = in[5] - in[3];                            \
    const v8f z11 = in[1] + in[7], z12 = in[1] - in[7];                            \
    const v8f o7 = z11 + z13;                                                      \
    const v8f t11b = (z11 - z13) * 1.414213562f;                                   \
    const v8f z5 = (z10 + z12) * 1.847759065f;                                     \
    const v8f t10b = z12 * 1.082392200f - z5;                                      \
    const v8f t12b = z10 * -2.613125930f + z5;                                     \
    const v8f o6 = t12b - o7;                                                      \
    const v8f o5 = t11b - o6;                                                      \
    const v8f o4 = t10b + o5;                                                      \
    o[0] = e0 + o7;                                                                \
    o[7] = e0 - o7;                                                                \
    o[1] = e1 + o6;                                                                \
    o[6] = e1 - o6;                                                                \
    o[2] = e2 + o5;                                                                \
    o[5] = e2 - o5;                                                                \
    o[4] = e3 + o4;                                                                \
    o[3] = e3 - o4;                                                                \
  } while (0)

// AVX2: 8x8 transposes in registers (unpack / shuffle / 128-bit permute),
// saturating pack to bytes.
__attribute__((target("avx2,fma"))) void transpose8_avx(__m256* r) {
  const __m256 t0 = _mm256_unpacklo_ps(r[0], r[1]), t1 = _mm256_unpackhi_ps(r[0], r[1]);
  const __m256 t2 = _mm256_unpacklo_ps(r[2], r[3]), t3 = _mm256_unpackhi_ps(r[2], r[3]);
  const __m256 t4 = _mm256_unpacklo_ps(r[4], r[5]), t5 = _mm256_unpackhi_ps(r[4], r[5]);
  const __m256 t6 = _mm256_unpacklo_ps(r[6], r[7]), t7 = _mm256_unpackhi_ps(r[6], r[7]);
  const __m256 s0 = _mm256_shuffle_ps(t0, t2, _MM_SHUFFLE(1, 0, 1, 0));
  const __m256 s1 = _mm256_shuffle_ps(t0, t2, _MM_SHUFFLE(3, 2, 3, 2));
  const __m256 s2 = _mm256_shuffle_ps(t1, t3, _MM_SHUFFLE(1, 0, 1, 0));
  const __m256 s3 = _mm256_shuffle_ps(t1, t3, _MM_SHUFFLE(3, 2, 3, 2));
  const __m256 s4 = _mm256_shuffle_ps(t4, t6, _MM_SHUFFLE(1, 0, 1, 0));
  const __m256 s5 = _mm256_shuffle_ps(t4, t6, _MM_SHUFFLE(3, 2, 3, 2));
  const __m256 s6 = _mm256_shuffle_ps(t5, t7, _MM_SHUFFLE(1, 0, 1, 0));
  const __m256 s7 = _mm256_shuffle_ps(t5, t7, _MM_SHUFFLE(3, 2, 3, 2));
  r[0] = _mm256_permute2f128_ps(s0, s4, 0x20);
  r[1] = _mm256_permute2f128_ps(s1, s5, 0x20);
  r[2] = _mm256_permute2f128_ps(s2, s6, 0x20);
  r[3] = _mm256_permute2f128_ps(s3, s7, 0x20);
  r[4] = _mm256_permute2f128_ps(s0, s4, 0x31);
  r[5] = _mm256_permute2f128_ps(s1, s5, 0x31);
  r[6] = _mm256_permute2f128_ps(s2, s6, 0x31);
  r[7] = _mm256_permute2f128_ps(s3, s7, 0x31);
}

__attribute__((target("avx2,fma"))) void idct8x8_avx2(const float* in, uint8_t* out, int stride) {
  __m256 a[8], b[8];
  for (int i = 0; i < 8; ++i) a[i] = _mm256_loadu_ps(in + 8 * i);  // a[v]: lane = u
  {
    const v8f* x = (const v8f*)a;
    v8f* y = (v8f*)b;
    DMLC_IDCT8_LANES(x, y);  // b[y]: lane = u
  }
  transpose8_avx(b);  // b[u]: lane = y
  {
    const v8f* x = (const v8f*)b;
    v8f* y = (v8f*)a;
    DMLC_IDCT8_LANES(x, y);  // a[x]: lane = y
  }
  transpose8_avx(a);  // a[y]: lane = x
  const __m256 lo = _mm256_setzero_ps(), hi = _mm256_set1_ps(255.f), half = _mm256_set1_ps(128.5f);
  for (int y = 0; y < 8; ++y) {
    const __m256 f = _mm256_min_ps(_mm256_max_ps(_mm256_add_ps(a[y], half), lo), hi);
    const __m256i i32 = _mm256_cvttps_epi32(f);
    const __m256i i16 = _mm256_packs_epi32(i32, i32);
    const __m256i u8 = _mm256_packus_epi16(i16, i16);
    uint32_t w0 = (uint32_t)_mm256_extract_epi32(u8, 0), w1 = (uint32_t)_mm256_extract_epi32(u8, 4);
    std::memcpy(out + (size_t)y * stride, &w0, 4);
    std::memcpy(out + (size_t)y * stride + 4, &w1, 4);
  }
}

void idct8x8_generic(const float* in, uint8_t* out, int stride) {
  v8f a[8], b[8];
  std::memcpy(a, in, sizeof(a));
  DMLC_IDCT8_LANES(a, b);
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) a[j][i] = b[i][j];
  DMLC_IDCT8_LANES(a, b);
  for (int x = 0; x < 8; ++x)
    for (int y = 0; y < 8; ++y) {
      const float f = b[x][y] + 128.5f;  // round half up; negatives clamp to 0
      const int i = f <= 0.f ? 0 : (int)f;
      out[(size_t)y * stride + x] = (uint8_t)(i > 255 ? 255 : i);
    }
}

bool detect_avx2() {
  __builtin_cpu_init();  // required before __builtin_cpu_supports in a static initialiser
  return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
}
const bool kHasAvx2 = detect_avx2();

// in: dequantised, AAN-prescaled coefficients in natural (row-major) order
inline void idct8x8(const float* in, uint8_t* out, int stride) {
  if (kHasAvx2) idct8x8_avx2(in, out, stride);
  else idct8x8_generic(in, out, stride);
}

uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

// YCbCr -> RGB in 16.16 fixed point (JFIF full-range coefficients, each
// rounded once to a 16.16 constant as libjpeg's FIX() does), e.g.
// R = (Y * 2^16 + kCrR * (Cr - 128) + 2^15) >> 16, clamped to [0, 255]. The
// scalar and AVX2 paths compute exactly this, so they are bit-identical.
constexpr int kCrR = 91881;    // 1.402    * 65536
constexpr int kCbB = 116130;   // 1.772    * 65536
constexpr int kCrG = -46802;   // -0.714136 * 65536
constexpr int kCbG = -22554;   // -0.344136 * 65536

inline uint8_t clamp_fix(int v) {  // 16.16 -> u8, rounded
  v = (v + 32768) >> 16;
  return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

inline void ycc_pixel(int y, int cb, int cr, uint8_t* o) {
  const int Y = y << 16, b = cb - 128, r = cr - 128;
  o[0] = clamp_fix(Y + kCrR * r);
  o[1] = clamp_fix(Y + kCbG * b + kCrG * r);
  o[2] = clamp_fix(Y + kCbB * b);
}

void ycc_row_scalar(const uint8_t* y, const uint8_t* cb, const uint8_t* cr, uint8_t* o, int x0, int W) {
  for (int x = x0; x < W; ++x) ycc_pixel(y[x], cb[x], cr[x], o + 3 * x);
}

// 2 x 8 int32 -> 16 u8 in pixel order, saturating (packs work per 128-bit lane)
__attribute__((target("avx2"))) inline __m128i pack16_avx2(__m256i a, __m256i b) {
  const __m256i w = _mm256_permute4x64_epi64(_mm256_packs_epi32(a, b), 0xD8);  // 16 x i16, in order
  return _mm_packus_epi16(_mm256_castsi256_si128(w), _mm256_extracti128_si256(w, 1));
}

// R, G, B of 16 pixels (bytes of y/cb/cr at p), 32-bit fixed-point lanes
__attribute__((target("avx2"))) inline void ycc16_avx2(const uint8_t* y, const uint8_t* cb, const uint8_t* cr,
                                                       __m128i* R, __m128i* G, __m128i* B) {
  const __m256i c128 = _mm256_set1_epi32(128), half = _mm256_set1_epi32(32768);
  __m256i rr[2], gg[2], bb[2];
  for (int h = 0; h < 2; ++h) {
    const __m256i Y =
        _mm256_add_epi32(_mm256_slli_epi32(_mm256_cvtepu8_epi32(_mm_loadl_epi64((const __m128i*)(y + 8 * h))), 16),
                         half);
    const __m256i b = _mm256_sub_epi32(_mm256_cvtepu8_epi32(_mm_loadl_epi64((const __m128i*)(cb + 8 * h))), c128);
    const __m256i r = _mm256_sub_epi32(_mm256_cvtepu8_epi32(_mm_loadl_epi64((const __m128i*)(cr + 8 * h))), c128);
    rr[h] = _mm256_srai_epi32(_mm256_add_epi32(Y, _mm256_mullo_epi32(r, _mm256_set1_epi32(kCrR))), 16);
    gg[h] = _mm256_srai_epi32(_mm256_add_epi32(Y, _mm256_add_epi32(_mm256_mullo_epi32(b, _mm256_set1_epi32(kCbG)),
                                                                   _mm256_mullo_epi32(r, _mm256_set1_epi32(kCrG)))),
                              16);
    bb[h] = _mm256_srai_epi32(_mm256_add_epi32(Y, _mm256_mullo_epi32(b, _mm256_set1_epi32(kCbB))), 16);
  }
  *R = pack16_avx2(rr[0], rr[1]);
  *G = pack16_avx2(gg[0], gg[1]);
  *B = pack16_avx2(bb[0], bb[1]);
}

// 16 pixels per iteration, the three planar byte vectors interleaved into 48
// RGB bytes with pshufb. Returns the first pixel it did not convert.
__attribute__((target("avx2"))) int ycc_row_avx2(const uint8_t* y, const uint8_t* cb, const uint8_t* cr, uint8_t* o,
                                                 int W) {
  // output byte j of each 16-byte third takes channel j % 3 of pixel j / 3
  alignas(16) static const int8_t m[3][3][16] = {
      {{0, -1, -1, 1, -1, -1, 2, -1, -1, 3, -1, -1, 4, -1, -1, 5},
       {-1, 0, -1, -1, 1, -1, -1, 2, -1, -1, 3, -1, -1, 4, -1, -1},
       {-1, -1, 0, -1, -1, 1, -1, -1, 2, -1, -1, 3, -1, -1, 4, -1}},
      {{-1, -1, 6, -1, -1, 7, -1, -1, 8, -1, -1, 9, -1, -1, 10, -1},
       {5, -1, -1, 6, -1, -1, 7, -1, -1, 8, -1, -1, 9, -1, -1, 10},
       {-1, 5, -1, -1, 6, -1, -1, 7, -1, -1, 8, -1, -1, 9, -1, -1}},
      {{-1, 11, -1, -1, 12, -1, -1, 13, -1, -1, 14, -1, -1, 15, -1, -1},
       {-1, -1, 11, -1, -1, 12, -1, -1, 13, -1, -1, 14, -1, -1, 15, -1},
       {10, -1, -1, 11, -1, -1, 12, -1, -1, 13, -1, -1, 14, -1, -1, 15}}};
  int x = 0;
  for (; x + 16 <= W; x += 16) {
    __m128i R, G, B;
    ycc16_avx2(y + x, cb + x, cr + x, &R, &G, &B);
    for (int k = 0; k < 3; ++k) {
      const __m128i v = _mm_or_si128(_mm_or_si128(_mm_shuffle_epi8(R, _mm_load_si128((const __m128i*)m[k][0])),
                                                  _mm_shuffle_epi8(G, _mm_load_si128((const __m128i*)m[k][1]))),
                                     _mm_shuffle_epi8(B, _mm_load_si128((const __m128i*)m[k][2])));
      _mm_storeu_si128((__m128i*)(o + 3 * x + 16 * k), v);
    }
  }
  return x;
}

void ycc_row(const uint8_t* y, const uint8_t* cb, const uint8_t* cr, uint8_t* o, int W) {
  const int x0 = kHasAvx2 ? ycc_row_avx2(y, cb, cr, o, W) : 0;
  ycc_row_scalar(y, cb, cr, o, x0, W);
}

// Centred (triangle) upsampling of one chroma row by 1 or 2 per axis into
// `out` (W values): vertical blend of rows y0/y1 with weights (wa, wb)/4,
// then horizontal 3:1 blend; result = chroma sample at each output pixel,
// rounded. Same positions as the generic bilinear path ((x+0.5)/f - 0.5,
// clamped to the plane's valid area). The interior loops are branch-free
// (the edge samples are handled apart) so the compiler vectorises them.
void chroma_row(const Comp& c, int hf, int vf, int y, int W, int H, int hmax, int vmax, uint8_t* out,
                std::vector<uint16_t>& tmp) {
  const int pw = c.bw * 8;
  const int cw = (W * c.h + hmax - 1) / hmax, ch = (H * c.v + vmax - 1) / vmax;
  int y0, y1, wa, wb;  // weights of rows y0, y1 (sum 4)
  if (vf == 1) {
    y0 = y1 = y;
    wa = 4;
    wb = 0;
  } else {
    const int i = y >> 1;
    if (y & 1) {
      y0 = i;
      y1 = std::min(i + 1, ch - 1);
    } else {
      y0 = i;
      y1 = std::max(i - 1, 0);
    }
    wa = 3;
    wb = 1;
  }
  const uint8_t* r0 = c.plane.data() + (size_t)y0 * pw;
  const uint8_t* r1 = c.plane.data() + (size_t)y1 * pw;
  tmp.resize((size_t)cw);
  uint16_t* t = tmp.data();
  for (int x = 0; x < cw; ++x) t[x] = (uint16_t)(wa * r0[x] + wb * r1[x]);  // x4
  if (hf == 1) {
    for (int x = 0; x < W; ++x) out[x] = (uint8_t)((t[x] + 2) >> 2);
    return;
  }
  // out[2i] blends t[i] with t[i-1], out[2i+1] with t[i+1] (clamped at the ends)
  auto even = [&](int i) { return (uint8_t)((3 * t[i] + t[std::max(i - 1, 0)] + 8) >> 4); };
  auto odd = [&](int i) { return (uint8_t)((3 * t[i] + t[std::min(i + 1, cw - 1)] + 8) >> 4); };
  const int n = W / 2;  // complete (even, odd) pairs; W odd leaves a last even sample
  if (n >= 2) {
    out[0] = even(0);
    out[1] = odd(0);
    const int last = std::min(n - 1, cw - 2);  // interior pairs: i-1 >= 0 and i+1 <= cw-1
    for (int i = 1; i <= last; ++i) {
      const int m3 = 3 * t[i];
      out[2 * i] = (uint8_t)((m3 + t[i - 1] + 8) >> 4);
      out[2 * i + 1] = (uint8_t)((m3 + t[i + 1] + 8) >> 4);
    }
    for (int i = last + 1; i < n; ++i) {
      out[2 * i] = even(i);
      out[2 * i + 1] = odd(i);
    }
  } else {
    for (int i = 0; i < n; ++i) {
      out[2 * i] = even(i);
      out[2 * i + 1] = odd(i);
    }
  }
  if (W & 1) out[W - 1] = even(n);
}

// Fast colour conversion for 1 or 3 components with chroma subsampled by 1
// or 2 per axis (4:4:4, 4:2:2, 4:2:0, 4:4:0 — essentially every JPEG);
// false for other layouts (the generic float path handles them).
bool convert_fast(const std::vector<Comp>& comps, int hmax, int vmax, int W, int H, uint8_t* rgb) {
  const Comp& Yc = comps[0];
  if (Yc.h != hmax || Yc.v != vmax) return false;
  const int pw = Yc.bw * 8;
  if (comps.size() == 1) {
    for (int y = 0; y < H; ++y) {
      const uint8_t* yr = Yc.plane.data() + (size_t)y * pw;
      uint8_t* o = rgb + (size_t)y * W * 3;
      for (int x = 0; x < W; ++x) o[3 * x] = o[3 * x + 1] = o[3 * x + 2] = yr[x];
    }
    return true;
  }
  int hf[2], vf[2];
  for (int k = 0; k < 2; ++k) {
    const Comp& c = comps[k + 1];
    if (hmax % c.h || vmax % c.v) return false;
    hf[k] = hmax / c.h;
    vf[k] = vmax / c.v;
    if (hf[k] > 2 || vf[k] > 2) return false;
  }
  if (hf[0] == 1 && vf[0] == 1 && hf[1] == 1 && vf[1] == 1) {  // 4:4:4: planes read in place
    const int cpw = comps[1].bw * 8, rpw = comps[2].bw * 8;
    for (int y = 0; y < H; ++y)
      ycc_row(Yc.plane.data() + (size_t)y * pw, comps[1].plane.data() + (size_t)y * cpw,
              comps[2].plane.data() + (size_t)y * rpw, rgb + (size_t)y * W * 3, W);
    return true;
  }
  std::vector<uint8_t> cb((size_t)W), cr((size_t)W);
  std::vector<uint16_t> tmp;
  for (int y = 0; y < H; ++y) {
    chroma_row(comps[1], hf[0], vf[0], y, W, H, hmax, vmax, cb.data(), tmp);
    chroma_row(comps[2], hf[1], vf[1], y, W, H, hmax, vmax, cr.data(), tmp);
    ycc_row(Yc.plane.data() + (size_t)y * pw, cb.data(), cr.data(), rgb + (size_t)y * W * 3, W);
  }
  return true;
}

}  // namespace

// Decodes into the buffer out(W, H) returns (W * H * 3 bytes).
static void decode_jpeg_impl(const uint8_t* data, size_t size, const std::function<uint8_t*(int, int)>& out) {
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
        // a forged frame header must not allocate gigabytes
        if (W > 16384 || H > 16384 || (int64_t)W * H > (int64_t)64 << 20)
          throw std::runtime_error("jpeg: image too large");
        if (frame) throw std::runtime_error("jpeg: second frame header");
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
          if (c->td > 3 || c->ta > 3 || !dc[c->td].present || !ac[c->ta].present)
            throw std::runtime_error("jpeg: missing huffman table");
          sc.push_back(c);
        }
        BitReader br(seg_end, end);
        float blk[64];
        // dequantisation folded with the AAN scale factors, natural order
        float qf[4][64];
        for (int t = 0; t < 4; ++t)
          for (int k = 0; k < 64; ++k) qf[t][kZigzag[k]] = qt[t][k] * kAan.f[kZigzag[k]];
        int mcus_left = restart;
        auto decode_block = [&](Comp& c, uint8_t* dst, int stride) {
          std::memset(blk, 0, sizeof(blk));
          const float* q = qf[c.tq];
          const int t = decode_huff(dc[c.td], br);
          if (t > 15) throw std::runtime_error("jpeg: bad DC magnitude");
          c.pred += t ? extend(br.bits(t), t) : 0;
          blk[0] = (float)c.pred * q[0];
          const Huff& ha = ac[c.ta];
          for (int k = 1; k < 64;) {
            const int32_t fe = ha.fast[br.peek(Huff::kFastBits)];
            if (fe) {
              br.skip(fe & 31);
              k += (fe >> 5) & 15;
              if (k > 63) break;
              const int z = kZigzag[k];
              blk[z] = (float)(fe >> 16) * q[z];
              ++k;
              continue;
            }
            const int rs = decode_huff(ha, br);
            const int r = rs >> 4, s = rs & 15;
            if (s == 0) {
              if (r != 15) break;
              k += 16;
              continue;
            }
            k += r;
            if (k > 63) break;
            const int z = kZigzag[k];
            blk[z] = (float)extend(br.bits(s), s) * q[z];
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

  uint8_t* rgb = out(W, H);
  if (convert_fast(comps, hmax, vmax, W, H, rgb)) return;
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
      uint8_t* o = rgb + ((size_t)y * W + x) * 3;
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
}

Image decode_jpeg(const uint8_t* data, size_t size) {
  Image img;
  decode_jpeg_impl(data, size, [&](int w, int h) {
    img.width = w;
    img.height = h;
    img.rgb.resize((size_t)w * h * 3);
    return img.rgb.data();
  });
  return img;
}

void decode_jpeg_into(const uint8_t* data, size_t size, const std::function<uint8_t*(int, int)>& out) {
  decode_jpeg_impl(data, size, out);
}

Image decode_jpeg_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  return decode_jpeg(buf.data(), buf.size());
}

}  // namespace dmlc
