// On-device image preprocessing: u8 HWC -> normalised bf16 NHWC4.
//
// Reference equivalent: tch `imagenet::load_image_and_resize(path, 224, 224)`
// called per query at src/services.rs:492 (decode + resize + /255 + ImageNet
// mean/std normalisation, all on the CPU). Here the host only decodes; the
// resize, crop and normalisation run on the GPU and write the 4-channel
// packed layout consumed by the conv stem (channel 3 = 0).
//
// Resize rule: resize to (RH, RW) with the short side = S and the long side
// = floor(S * long / short) (aspect preserved), centre-crop SxS at integer
// offsets ((RH-S)/2, (RW-S)/2), bilinear sampling with half-pixel centres
// (= torch interpolate(mode="bilinear", align_corners=False, antialias=False)).
// When the input is already SxS this is an exact per-pixel normalisation.
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace dmlc {

namespace {

__global__ __launch_bounds__(256) void preprocess_kernel(const uint8_t* __restrict__ x,
                                                         bf16* __restrict__ y, int B, int Hin,
                                                         int Win, int S, float sy_scale,
                                                         float sx_scale, int oy, int ox) {
  const float mean[3] = {0.485f, 0.456f, 0.406f};
  const float istd[3] = {1.f / 0.229f, 1.f / 0.224f, 1.f / 0.225f};
  const long total = (long)B * S * S;
  const bool identity = (Hin == S && Win == S);
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int ox_i = (int)(idx % S);
    long t = idx / S;
    const int oy_i = (int)(t % S);
    const int b = (int)(t / S);
    const uint8_t* img = x + (long)b * Hin * Win * 3;
    float c[3];
    if (identity) {
      const uint8_t* p = img + ((long)oy_i * Win + ox_i) * 3;
      c[0] = p[0];
      c[1] = p[1];
      c[2] = p[2];
    } else {
      // Source coordinate of this output pixel centre in the resized+cropped image.
      float sy = (oy_i + oy + 0.5f) * sy_scale - 0.5f;
      float sx = (ox_i + ox + 0.5f) * sx_scale - 0.5f;
      sy = fminf(fmaxf(sy, 0.f), (float)(Hin - 1));
      sx = fminf(fmaxf(sx, 0.f), (float)(Win - 1));
      const int y0 = (int)sy, x0 = (int)sx;
      const int y1 = min(y0 + 1, Hin - 1), x1 = min(x0 + 1, Win - 1);
      const float fy = sy - y0, fx = sx - x0;
      const uint8_t* p00 = img + ((long)y0 * Win + x0) * 3;
      const uint8_t* p01 = img + ((long)y0 * Win + x1) * 3;
      const uint8_t* p10 = img + ((long)y1 * Win + x0) * 3;
      const uint8_t* p11 = img + ((long)y1 * Win + x1) * 3;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float top = p00[k] + (p01[k] - (float)p00[k]) * fx;
        const float bot = p10[k] + (p11[k] - (float)p10[k]) * fx;
        c[k] = top + (bot - top) * fy;
      }
    }
    float o[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) o[k] = (c[k] * (1.f / 255.f) - mean[k]) * istd[k];
    *(uint2*)(y + idx * 4) = make_uint2(pack2(o[0], o[1]), pack2(o[2], 0.f));
  }
}

}  // namespace

void preprocess_u8(const uint8_t* x, void* y, int B, int Hin, int Win, int S, hipStream_t s) {
  if (B <= 0) return;
  if (Hin <= 0 || Win <= 0 || S <= 0) throw std::invalid_argument("preprocess_u8: bad dims");
  int RH, RW;
  if (Hin <= Win) {
    RH = S;
    RW = (int)((long)S * Win / Hin);
  } else {
    RW = S;
    RH = (int)((long)S * Hin / Win);
  }
  const int oy = (RH - S) / 2, ox = (RW - S) / 2;
  const float sy_scale = (float)Hin / RH, sx_scale = (float)Win / RW;
  const long total = (long)B * S * S;
  const int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(preprocess_kernel, dim3(blocks), dim3(256), 0, s, x, (bf16*)y, B, Hin, Win, S,
                     sy_scale, sx_scale, oy, ox);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
