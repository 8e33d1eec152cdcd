// On-device image preprocessing: u8 HWC -> normalised, zero-padded packed
// RGB bf16 (the conv stem's input layout).
//
// Reference equivalent: tch `imagenet::load_image_and_resize(path, 224, 224)`
// called per query at src/services.rs:492 (decode + resize + /255 + ImageNet
// mean/std normalisation, all on the CPU). Here the host only decodes; the
// resize, crop and normalisation run on the GPU and write [B, S+2p, Wr, 3]
// bf16 with the image at (p, p) and zeros elsewhere, so the stem conv reads
// each kernel row's KW*3 values as contiguous 16-B chunks without bounds
// checks (csrc/kernels/conv_igemm.hip).
//
// Resize rule: resize to (RH, RW) with the short side = S and the long side
// = floor(S * long / short) (aspect preserved), centre-crop SxS at integer
// offsets ((RH-S)/2, (RW-S)/2), bilinear sampling with half-pixel centres
// (= torch interpolate(mode="bilinear", align_corners=False, antialias=False)).
// When the input is already SxS this is an exact per-pixel normalisation.
//
// One thread writes 8 consecutive pixels of an output row = 48 B as three
// 16-B stores (Wr % 8 == 0 keeps every store aligned). In the paired layout
// (input of the fused stem, csrc/kernels/stem_pool.hip) a pixel pair fills a
// 16-B chunk [r g b r g b 0 0] and the 8 pixels are four 16-B stores.
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace dmlc {

namespace {

struct PreParams {
  int B, Hin, Win, S, pad, P, Wr;  // P = S + 2*pad rows, Wr pixels per row
  float sy_scale, sx_scale;
  int oy, ox;
  bool identity;
  bool paired;  // 2 pixels per 16 B: [r g b r g b 0 0]
};

__device__ __forceinline__ void pixel(const uint8_t* __restrict__ img, const PreParams& p, int y, int x,
                                      float* o) {
  if ((unsigned)y >= (unsigned)p.S || (unsigned)x >= (unsigned)p.S) {
    o[0] = o[1] = o[2] = 0.f;
    return;
  }
  float c[3];
  if (p.identity) {
    const uint8_t* q = img + ((long)y * p.Win + x) * 3;
    c[0] = q[0];
    c[1] = q[1];
    c[2] = q[2];
  } else {
    float sy = (y + p.oy + 0.5f) * p.sy_scale - 0.5f;
    float sx = (x + p.ox + 0.5f) * p.sx_scale - 0.5f;
    sy = fminf(fmaxf(sy, 0.f), (float)(p.Hin - 1));
    sx = fminf(fmaxf(sx, 0.f), (float)(p.Win - 1));
    const int y0 = (int)sy, x0 = (int)sx;
    const int y1 = min(y0 + 1, p.Hin - 1), x1 = min(x0 + 1, p.Win - 1);
    const float fy = sy - y0, fx = sx - x0;
    const uint8_t* p00 = img + ((long)y0 * p.Win + x0) * 3;
    const uint8_t* p01 = img + ((long)y0 * p.Win + x1) * 3;
    const uint8_t* p10 = img + ((long)y1 * p.Win + x0) * 3;
    const uint8_t* p11 = img + ((long)y1 * p.Win + x1) * 3;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float top = p00[k] + (p01[k] - (float)p00[k]) * fx;
      const float bot = p10[k] + (p11[k] - (float)p10[k]) * fx;
      c[k] = top + (bot - top) * fy;
    }
  }
  o[0] = imagenet_norm(0, c[0]);
  o[1] = imagenet_norm(1, c[1]);
  o[2] = imagenet_norm(2, c[2]);
}

__global__ __launch_bounds__(256) void preprocess_kernel(const uint8_t* __restrict__ x, bf16* __restrict__ y,
                                                         PreParams p) {
  const int groups = p.Wr / 8;
  const long total = (long)p.B * p.P * groups;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int g = (int)(idx % groups);
    long t = idx / groups;
    const int hy = (int)(t % p.P);
    const int b = (int)(t / p.P);
    const uint8_t* img = x + (long)b * p.Hin * p.Win * 3;
    const int iy = hy - p.pad;
    if (p.paired) {
      float v[32];
#pragma unroll
      for (int i = 0; i < 8; ++i) pixel(img, p, iy, g * 8 + i - p.pad, v + 8 * (i >> 1) + 3 * (i & 1));
      uint4* dst = (uint4*)(y + idx * 32);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[8 * q + 6] = v[8 * q + 7] = 0.f;
        dst[q] = pack8(v + 8 * q);
      }
    } else {
      float v[24];
#pragma unroll
      for (int i = 0; i < 8; ++i) pixel(img, p, iy, g * 8 + i - p.pad, v + 3 * i);
      uint4* dst = (uint4*)(y + idx * 24);
      dst[0] = pack8(v);
      dst[1] = pack8(v + 8);
      dst[2] = pack8(v + 16);
    }
  }
}

}  // namespace

void preprocess_u8(const uint8_t* x, void* y, int B, int Hin, int Win, int S, int pad, int Wr,
                   hipStream_t s, bool paired) {
  if (B <= 0) return;
  if (Hin <= 0 || Win <= 0 || S <= 0 || pad < 0 || Wr < S + 2 * pad || Wr % 8 != 0)
    throw std::invalid_argument("preprocess_u8: bad dims");
  if (!x || !y || ((uintptr_t)y & 15)) throw std::invalid_argument("preprocess_u8: null / misaligned operand");
  PreParams p;
  p.B = B;
  p.Hin = Hin;
  p.Win = Win;
  p.S = S;
  p.pad = pad;
  p.P = S + 2 * pad;
  p.Wr = Wr;
  int RH, RW;
  if (Hin <= Win) {
    RH = S;
    RW = (int)((long)S * Win / Hin);
  } else {
    RW = S;
    RH = (int)((long)S * Hin / Win);
  }
  p.oy = (RH - S) / 2;
  p.ox = (RW - S) / 2;
  p.sy_scale = (float)Hin / RH;
  p.sx_scale = (float)Win / RW;
  p.identity = (Hin == S && Win == S);
  p.paired = paired;
  const long total = (long)B * p.P * (Wr / 8);
  const int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(preprocess_kernel, dim3(blocks), dim3(256), 0, s, x, (bf16*)y, p);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
