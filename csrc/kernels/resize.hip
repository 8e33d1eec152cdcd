// Ragged batch resize: differently sized u8 HWC images -> one u8 [B, S, S, 3]
// batch, so a query of mixed-size JPEGs becomes ONE (graph-replayed) forward
// instead of one forward per distinct size.
//
// Reference equivalent: tch `imagenet::load_image_and_resize(path, 224, 224)`
// per query (src/services.rs:492), which resizes the decoded image to u8
// before normalising. Same rule as preprocess.hip (short side -> S, long side
// floor(S*long/short), centre crop, bilinear with half-pixel centres), with the
// result rounded to u8; normalisation then happens inside the fused stem
// (stem_pool.hip) of the forward.
//
// Each image comes from a descriptor {pointer, H, W} in device memory (the
// decoded images live in the executor's HBM cache at their own sizes). One
// thread writes 4 consecutive pixels = 12 B as three dword stores; grid =
// (pixel blocks, B).
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace dmlc {

namespace {

__global__ __launch_bounds__(256) void resize_ragged_kernel(const ImageDesc* __restrict__ descs,
                                                            uint8_t* __restrict__ out, int S) {
  const int b = blockIdx.y;
  const ImageDesc d = descs[b];
  const int q = blockIdx.x * 256 + threadIdx.x;  // quad of pixels
  const int quads = S * S / 4;
  if (q >= quads) return;
  const int p0 = q * 4;
  const int y = p0 / S, x0 = p0 % S;
  uint8_t v[12];
  if (d.h == S && d.w == S) {
    const uint8_t* src = d.ptr + ((long)y * S + x0) * 3;
#pragma unroll
    for (int i = 0; i < 12; ++i) v[i] = src[i];
  } else {
    int RH, RW;
    if (d.h <= d.w) {
      RH = S;
      RW = (int)((long)S * d.w / d.h);
    } else {
      RW = S;
      RH = (int)((long)S * d.h / d.w);
    }
    const float sys = (float)d.h / RH, sxs = (float)d.w / RW;
    const int oy = (RH - S) / 2, ox = (RW - S) / 2;
    float sy = (y + oy + 0.5f) * sys - 0.5f;
    sy = fminf(fmaxf(sy, 0.f), (float)(d.h - 1));
    const int y0 = (int)sy, y1 = min(y0 + 1, d.h - 1);
    const float fy = sy - y0;
    const uint8_t* r0 = d.ptr + (long)y0 * d.w * 3;
    const uint8_t* r1 = d.ptr + (long)y1 * d.w * 3;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float sx = (x0 + i + ox + 0.5f) * sxs - 0.5f;
      sx = fminf(fmaxf(sx, 0.f), (float)(d.w - 1));
      const int xa = (int)sx, xb = min(xa + 1, d.w - 1);
      const float fx = sx - xa;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float a = r0[xa * 3 + k], bb = r0[xb * 3 + k], c = r1[xa * 3 + k], e = r1[xb * 3 + k];
        const float top = a + (bb - a) * fx, bot = c + (e - c) * fx;
        const float val = top + (bot - top) * fy;
        v[i * 3 + k] = (uint8_t)fminf(fmaxf(rintf(val), 0.f), 255.f);
      }
    }
  }
  uint32_t* dst = (uint32_t*)(out + ((long)b * S * S + p0) * 3);
#pragma unroll
  for (int i = 0; i < 3; ++i)
    dst[i] = (uint32_t)v[4 * i] | ((uint32_t)v[4 * i + 1] << 8) | ((uint32_t)v[4 * i + 2] << 16) |
             ((uint32_t)v[4 * i + 3] << 24);
}

}  // namespace

void resize_u8_ragged(const ImageDesc* descs, uint8_t* out, int B, int S, hipStream_t s) {
  if (B <= 0) return;
  if (S <= 0 || S % 4 != 0) throw std::invalid_argument("resize_u8_ragged: S must be a positive multiple of 4");
  if (!descs || !out || ((uintptr_t)out & 3)) throw std::invalid_argument("resize_u8_ragged: null / misaligned operand");
  const int quads = S * S / 4;
  hipLaunchKernelGGL(resize_ragged_kernel, dim3((quads + 255) / 256, B), dim3(256), 0, s, descs, out, S);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
