// Shared device helpers for the gfx950 (CDNA4) kernels.
//
// All activations are bf16 NHWC; all accumulation is fp32 on MFMA.
// Wave = 64 lanes everywhere (CDNA), never 32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dmlc {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));  // v_pk_fma_f32 / v_pk_mul_f32 operands

constexpr int kWave = 64;

// Workgroup start stagger (launch tuning, kernels.h kernel_stagger): a
// workgroup on an odd CU of its XCD (workgroups are dealt to the 8 XCDs
// round-robin, then to CUs in order) starts n x ~2048 cycles late. With one
// workgroup per CU every workgroup otherwise runs its HBM-bound prologue, its
// MFMA loop and its store-bound epilogue in step with all the others; offset
// halves overlap one half's memory phase with the other half's MFMAs.
__device__ __forceinline__ void start_stagger(int n) {
  if (n && ((blockIdx.x >> 3) & 1))  // (a wave-uniform scalar loop)
    for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(32);
}

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }  // v_cvt_pk_bf16_f32 (RNE)

// Unpack / pack 8 bf16 held in a uint4 (16 B) register quad.
// 4 e4m3 bytes -> 4 floats (exact) with the packed converts: two
// v_cvt_pk_f32_fp8 (bytes 0-1, 2-3) instead of four v_cvt_f32_fp8
__device__ __forceinline__ void e4m3x4_to_f32(uint32_t u, float* f) {
  typedef float f32x2v __attribute__((ext_vector_type(2)));
  const f32x2v lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)u, false);
  const f32x2v hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)u, true);
  f[0] = lo.x;
  f[1] = lo.y;
  f[2] = hi.x;
  f[3] = hi.y;
}
__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  bf16 x = f2bf(a), y = f2bf(b);
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

// ImageNet normalisation of a u8-range value of channel c (0=R, 1=G, 2=B):
// (v/255 - mean)/std as ONE fma, v * 1/(255 std) + (-mean/std). Shared by
// preprocess.hip and the u8 stem in stem_pool.hip so both produce the same
// bits (the two-op form costs an extra VALU op per value in the stem's
// VALU-bound u8 conversion).
__device__ __forceinline__ float imagenet_norm(int c, float v) {
  const float sc = c == 0 ? 1.f / (255.f * 0.229f) : c == 1 ? 1.f / (255.f * 0.224f) : 1.f / (255.f * 0.225f);
  const float sh = c == 0 ? -0.485f / 0.229f : c == 1 ? -0.456f / 0.224f : -0.406f / 0.225f;
  return __builtin_fmaf(v, sc, sh);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

// ReLU on 8 packed bf16: max with 0 as int16 (negative bf16 bit patterns are
// negative int16; -0 becomes +0), 4 v_pk_max_i16. Rounding is monotone and
// keeps the sign, so relu-after-rounding equals rounding-after-fmaxf bit for
// bit, at a quarter of the VALU: fmaxf(v, 0) compiles to two v_max_f32 per
// value (a NaN-canonicalising max first), 16 per 8 channels.
__device__ __forceinline__ uint4 relu_bf16x8(uint4 u) {
  typedef short short8v __attribute__((ext_vector_type(8)));
  const short8v z = {0, 0, 0, 0, 0, 0, 0, 0};
  return __builtin_bit_cast(uint4, __builtin_elementwise_max(__builtin_bit_cast(short8v, u), z));
}
__device__ __forceinline__ uint4 pack8_relu(const float* f, bool relu) {
  const uint4 p = pack8(f);
  return relu ? relu_bf16x8(p) : p;
}

// 16-B-per-lane LDS-DMA (global_load_lds_dwordx4: lane l's 16 bytes land at
// lds + 16 l; lds must be wave-uniform), issued as inline asm. With
// __builtin_amdgcn_global_load_lds in flight the compiler's waitcnt pass
// turns every wait on an LDS read into lgkmcnt(0), so a kernel that keeps
// DMA in flight under its MFMAs lost the counted waits that let MFMAs start
// on the first operands to land. The pass does not see these, so every vmcnt
// wait they need is the kernel's own (s_waitcnt vmcnt asm). Compiler-visible
// global loads may still be mixed in: vmcnt retires in issue order, so the
// compiler's counted waits stay correct (they can only wait longer).
__device__ __forceinline__ void dma16(const void* gsrc, const void* lds) {
  const uint32_t l =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds);
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(l), "v"(gsrc) : "memory", "m0");
}
// 4-B-per-lane form (global_load_lds_dword: lane l's 4 bytes land at lds + 4 l).
__device__ __forceinline__ void dma4(const void* gsrc, const void* lds) {
  const uint32_t l =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds);
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, off" ::"s"(l), "v"(gsrc) : "memory", "m0");
}
// Same with a scalar base (saddr form): lane l loads base + voff[l].
__device__ __forceinline__ void dma16s(const void* sbase, uint32_t voff, const void* lds) {
  const uint32_t l =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds);
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(l), "v"(voff), "s"(sbase) : "memory", "m0");
}

// Buffer descriptor from wave-uniform inputs (readfirstlane, else hipcc wraps
// every buffer op in a waterfall loop). Loads through it take a scalar
// offset, so a fully unrolled loop over constant offsets needs no per-load
// address VGPRs.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* p, int bytes) {
  const uint64_t u = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace dmlc
