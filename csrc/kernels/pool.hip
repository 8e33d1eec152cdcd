// NHWC bf16 pooling kernels (max pool, global average pool, adaptive average
// pool). These replace the libtorch max_pool2d / adaptive_avg_pool2d calls
// inside tch-rs resnet18/alexnet `forward_t` (reference: src/services.rs:493).
// Memory-bound: every lane moves 16 B (8 channels) per access.
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace dmlc {

namespace {

__global__ __launch_bounds__(256) void maxpool_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                      int B, int H, int W, int C, int Ho, int Wo,
                                                      int k, int stride, int pad) {
  const int c8 = C / 8;
  const long total = (long)B * Ho * Wo * c8;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int cg = (int)(idx % c8);
    long t = idx / c8;
    const int wo = (int)(t % Wo);
    t /= Wo;
    const int ho = (int)(t % Ho);
    const int b = (int)(t / Ho);
    float m[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = -INFINITY;
    const int h0 = ho * stride - pad, w0 = wo * stride - pad;
    for (int kh = 0; kh < k; ++kh) {
      const int h = h0 + kh;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int w = w0 + kw;
        if ((unsigned)w >= (unsigned)W) continue;
        const uint4 v = *(const uint4*)(x + (((long)b * H + h) * W + w) * C + cg * 8);
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int i = 0; i < 8; ++i) m[i] = fmaxf(m[i], f[i]);
      }
    }
    *(uint4*)(y + idx * 8) = pack8(m);
  }
}

// One thread per (b, 8-channel group); loops over HW. HW <= 64 for ResNet.
// FP8: the input is e4m3 (ResNet50 fp8 path) dequantised by `scale`.
// 8 lanes per (image, 8-channel group): lane `part` sums pixels part,
// part+8, ... with its loads issued together, then a 3-step shuffle reduce
// (one thread walking all HW pixels serially was latency bound: 18.5 us for
// 6.4 MB at ResNet18 layer4, B=256).
template <bool FP8>
__global__ __launch_bounds__(256) void avgpool_global_kernel(const void* __restrict__ xv,
                                                             bf16* __restrict__ y, int B, int HW,
                                                             int C, float scale) {
  const int c8 = C / 8;
  const long total = (long)B * c8 * 8;
  const float inv = (FP8 ? scale : 1.f) / HW;
  for (long t = blockIdx.x * 256L + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const long idx = t >> 3;  // (image, channel group); the 8 lanes of a group share it (256 % 8 == 0)
    const int part = (int)(t & 7);
    const int cg = (int)(idx % c8);
    const int b = (int)(idx / c8);
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const long base = (long)b * HW * C + cg * 8;
    constexpr int U = 8;  // up to U loads in flight per lane
    for (int i0 = part; i0 < HW; i0 += 8 * U) {
      float f[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + 8 * u;
        if (i < HW) {
          if constexpr (FP8) {
            const uint2 q = *(const uint2*)((const uint8_t*)xv + base + (long)i * C);
            e4m3x4_to_f32((uint32_t)q.x, f[u]);
            e4m3x4_to_f32((uint32_t)q.y, f[u] + 4);
          } else {
            unpack8(*(const uint4*)((const bf16*)xv + base + (long)i * C), f[u]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[u][j] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += f[u][j];
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1)
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += __shfl_xor(s[j], o, 64);
    if (part == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] *= inv;
      *(uint4*)(y + idx * 8) = pack8(s);
    }
  }
}

// Same result bit for bit (part p = pixels p, p+8, ... summed in order, the 8
// parts combined in the butterfly order of the shuffle reduce above), with
// a lane owning 8 channels of one image: a wave reads 512 contiguous
// channels of a pixel per load, and a lane keeps all 8 part sums, so no
// shuffles. Loads in blocks of 24 pixels (3 per part) issued together. For
// batches where the 8-lane kernel's scattered 8-B reads ran at ~1 TB/s
// (resnet50_fp8 b256: 23 us for 25.7 MB).
template <bool FP8>
__global__ __launch_bounds__(256) void avgpool_rows_kernel(const void* __restrict__ xv, bf16* __restrict__ y, int HW,
                                                           int C, float scale) {
  const int b = blockIdx.y;
  const int cg = blockIdx.x * blockDim.x + threadIdx.x;  // 8-channel group
  if (cg * 8 >= C) return;
  const float inv = (FP8 ? scale : 1.f) / HW;
  const long base = (long)b * HW * C + cg * 8;
  float s[8][8];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int j = 0; j < 8; ++j) s[p][j] = 0.f;
  constexpr int BLK = 24;
  for (int i0 = 0; i0 < HW; i0 += BLK) {
    uint4 v[BLK];
#pragma unroll
    for (int u = 0; u < BLK; ++u) {
      const int i = i0 + u;
      if (i < HW) {
        if constexpr (FP8) {
          const uint2 q = *(const uint2*)((const uint8_t*)xv + base + (long)i * C);
          v[u] = make_uint4(q.x, q.y, 0u, 0u);
        } else {
          v[u] = *(const uint4*)((const bf16*)xv + base + (long)i * C);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < BLK; ++u) {
      const int i = i0 + u;
      if (i < HW) {
        float f[8];
        if constexpr (FP8) {
          e4m3x4_to_f32((uint32_t)v[u].x, f);
          e4m3x4_to_f32((uint32_t)v[u].y, f + 4);
        } else {
          unpack8(v[u], f);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s[u & 7][j] += f[j];  // (BLK % 8 == 0: part = i % 8 = u % 8)
      }
    }
  }
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    o[j] = (((s[0][j] + s[1][j]) + (s[2][j] + s[3][j])) + ((s[4][j] + s[5][j]) + (s[6][j] + s[7][j]))) * inv;
  *(uint4*)(y + ((long)b * C + cg * 8)) = pack8(o);
}

// torch adaptive_avg_pool2d bin rule: [floor(i*H/Ho), ceil((i+1)*H/Ho)).
__global__ __launch_bounds__(256) void avgpool_adaptive_kernel(const bf16* __restrict__ x,
                                                               bf16* __restrict__ y, int B, int H,
                                                               int W, int C, int Ho, int Wo) {
  const int c8 = C / 8;
  const long total = (long)B * Ho * Wo * c8;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int cg = (int)(idx % c8);
    long t = idx / c8;
    const int wo = (int)(t % Wo);
    t /= Wo;
    const int ho = (int)(t % Ho);
    const int b = (int)(t / Ho);
    const int hs = (ho * H) / Ho, he = ((ho + 1) * H + Ho - 1) / Ho;
    const int ws = (wo * W) / Wo, we = ((wo + 1) * W + Wo - 1) / Wo;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int h = hs; h < he; ++h)
      for (int w = ws; w < we; ++w) {
        float f[8];
        unpack8(*(const uint4*)(x + (((long)b * H + h) * W + w) * C + cg * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += f[j];
      }
    const float inv = 1.f / ((he - hs) * (we - ws));
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] *= inv;
    *(uint4*)(y + idx * 8) = pack8(s);
  }
}

int grid_for(long work) { return (int)std::max<long>(1, std::min<long>((work + 255) / 256, 8192)); }

}  // namespace

void maxpool2d(const void* x, void* y, int B, int H, int W, int C, int Ho, int Wo, int k, int stride,
               int pad, hipStream_t s) {
  if (C % 8 != 0) throw std::invalid_argument("maxpool2d: C % 8 != 0");
  if (Ho != conv_out_dim(H, k, stride, pad) || Wo != conv_out_dim(W, k, stride, pad))
    throw std::invalid_argument("maxpool2d: bad output dims");
  const long work = (long)B * Ho * Wo * (C / 8);
  if (work == 0) return;
  hipLaunchKernelGGL(maxpool_kernel, dim3(grid_for(work)), dim3(256), 0, s, (const bf16*)x, (bf16*)y,
                     B, H, W, C, Ho, Wo, k, stride, pad);
  DMLC_HIP_CHECK(hipGetLastError());
}

void avgpool_global(const void* x, void* y, int B, int HW, int C, hipStream_t s, bool in_fp8, float scale) {
  if (C % 8 != 0) throw std::invalid_argument("avgpool_global: C % 8 != 0");
  const long work = (long)B * (C / 8) * 8;
  if (work == 0) return;
  if (B >= 32 && B <= 65535) {  // (throughput batches: lane per 8 channels, contiguous wave reads)
    const int c8 = C / 8, nt = std::min(c8, 256);
    const dim3 grid((c8 + nt - 1) / nt, B);
    if (in_fp8)
      hipLaunchKernelGGL(avgpool_rows_kernel<true>, grid, dim3(nt), 0, s, x, (bf16*)y, HW, C, scale);
    else
      hipLaunchKernelGGL(avgpool_rows_kernel<false>, grid, dim3(nt), 0, s, x, (bf16*)y, HW, C, 1.f);
  } else if (in_fp8) {
    hipLaunchKernelGGL(avgpool_global_kernel<true>, dim3(grid_for(work)), dim3(256), 0, s, x, (bf16*)y, B, HW, C,
                       scale);
  } else {
    hipLaunchKernelGGL(avgpool_global_kernel<false>, dim3(grid_for(work)), dim3(256), 0, s, x, (bf16*)y, B, HW, C,
                       1.f);
  }
  DMLC_HIP_CHECK(hipGetLastError());
}

void avgpool_adaptive(const void* x, void* y, int B, int H, int W, int C, int Ho, int Wo,
                      hipStream_t s) {
  if (C % 8 != 0) throw std::invalid_argument("avgpool_adaptive: C % 8 != 0");
  const long work = (long)B * Ho * Wo * (C / 8);
  if (work == 0) return;
  hipLaunchKernelGGL(avgpool_adaptive_kernel, dim3(grid_for(work)), dim3(256), 0, s, (const bf16*)x,
                     (bf16*)y, B, H, W, C, Ho, Wo);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
