// Fused classifier head: global average pool + fc (+ bias) + softmax + top-1
// in one launch (ResNet tail: avgpool -> flatten -> fc -> softmax -> top(1)).
//
// Reference: `forward_t` ends in adaptive_avg_pool2d(1) + fc, then
// `.softmax(-1)` and `imagenet::top(output, 1)` per query
// (src/services.rs:493-494). As three launches (avgpool, the fc as a 1x1
// implicit GEMM, softmax_top1) the tail cost ~40 us at B=256, almost all of
// it launch/latency bound; here it is one kernel of B/4 x NS workgroups.
//
// Workgroup (g, s): images 4g..4g+3, classes of split s (NS splits of whole
// 16-class tiles).
//  1. pool its 4 images (8 lanes per (image, 8-channel group), loads in
//     flight, shuffle reduce: the avgpool_global_kernel arithmetic, so the
//     pooled bf16 vector is bit-identical) into LDS;
//  2. each wave takes 16-class tiles: A = fc weight rows from global (16 B
//     per lane), B = pooled^T from LDS (images in MFMA columns 0..3, the
//     other 12 columns are zero registers), v_mfma_f32_16x16x32_bf16 over K;
//  3. logits (+bias) to global fp32 and LDS; per image a wave reduces its
//     split's (max, argmax, sum exp(x - max)) and stores the partial;
//  4. the workgroup that draws the last ticket for group g combines the NS
//     partials (cdna_hip_programming.md §6 Guideline 16 counter recipe:
//     plain stores -> vmcnt(0) -> barrier -> agent release -> vmcnt(0) ->
//     relaxed agent fetch_add; reducer: agent acquire -> vmcnt(0) ->
//     barrier -> loads) and writes (class, prob), then re-arms the counter.
// No workgroup waits on another, so any residency is correct.
#include "common.h"
#include "kernels.h"

namespace dmlc {

namespace {

constexpr int kIPW = 4;  // images per workgroup (one wave each in the softmax)

struct HeadArgs {
  const bf16* x;      // [B, HW, C]
  const bf16* w;      // [Npad, ldw]
  const float* bias;  // [Npad]
  float* logits;      // [B, N]
  int32_t* idx;
  float* prob;
  float4* part;       // [B, NS] (max, argmax bits, sum, -)
  uint32_t* cnt;      // [ceil(B / kIPW)], zero between launches
  int B, HW, C, N, ldw, tiles_per_split, NS;
};

__global__ __launch_bounds__(256) void head_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int C = a.C;
  const int ldp = C + 8;  // pooled row stride (elements): rows 16 B apart in bank space
  bf16* pooled = (bf16*)smem;                                // [kIPW][ldp]
  float* lg = (float*)(smem + kIPW * ldp * 2);               // [kIPW][tiles_per_split*16]
  const int g = blockIdx.x, split = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b0 = g * kIPW;
  const int nimg = min(kIPW, a.B - b0);

  // ---- 1. average pool
  {
    const int c8 = C / 8;
    const int total = nimg * c8 * 8;
    const float inv = 1.f / a.HW;
    for (int t = tid; t < total; t += 256) {
      const int item = t >> 3, part = t & 7;
      const int cg = item % c8, i = item / c8;
      float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      const bf16* base = a.x + ((long)(b0 + i) * a.HW) * C + cg * 8;
      constexpr int U = 8;
      for (int i0 = part; i0 < a.HW; i0 += 8 * U) {
        float f[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int p = i0 + 8 * u;
          if (p < a.HW) {
            unpack8(*(const uint4*)(base + (long)p * C), f[u]);
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
        *(uint4*)(pooled + i * ldp + cg * 8) = pack8(s);
      }
    }
  }
  __syncthreads();

  // ---- 2./3. fc tiles on MFMA: lane holds D[class row (lane>>4)*4 + r][image lane&15]
  const int col = lane & 15, kq = lane >> 4;
  const int nsplit = a.tiles_per_split * 16;
  const int n_begin = split * nsplit;
  for (int t = wave; t < a.tiles_per_split; t += 4) {
    const int n0 = n_begin + t * 16;
    if (n0 >= a.N) break;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    const bf16* wrow = a.w + (long)(n0 + col) * a.ldw + kq * 8;
    const bf16* prow = pooled + col * ldp + kq * 8;
    const bool live = col < nimg;
    for (int k0 = 0; k0 < C; k0 += 32 * 4) {
      bf16x8 wa[4], pb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + 32 * u;
        if (k < C) {
          wa[u] = *(const bf16x8*)(wrow + k);
          pb[u] = live ? *(const bf16x8*)(prow + k) : bf16x8{};
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (k0 + 32 * u < C) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[u], pb[u], acc, 0, 0, 0);
    }
    if (live) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + kq * 4 + r;
        const float v = acc[r] + a.bias[n];
        if (n < a.N) a.logits[(long)(b0 + col) * a.N + n] = v;
        lg[col * nsplit + t * 16 + kq * 4 + r] = v;
      }
    }
  }
  __syncthreads();

  // per image (one wave each): this split's max / argmax / sum exp
  const int n_end = min(a.N, n_begin + nsplit);
  if (wave < nimg) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int n = n_begin + lane; n < n_end; n += 64) {
      const float v = lg[wave * nsplit + (n - n_begin)];
      if (v > best) {
        best = v;
        bi = n;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) {
        best = ov;
        bi = oi;
      }
    }
    float s = 0.f;
    for (int n = n_begin + lane; n < n_end; n += 64) s += __expf(lg[wave * nsplit + (n - n_begin)] - best);
    s = wave_sum(s);
    if (a.NS == 1) {
      if (lane == 0) {
        a.idx[b0 + wave] = bi;
        a.prob[b0 + wave] = 1.f / s;
      }
      return;
    }
    if (lane == 0) a.part[(long)(b0 + wave) * a.NS + split] = make_float4(best, __int_as_float(bi), s, 0.f);
  }
  if (a.NS == 1) return;

  // ---- 4. last arriver of group g combines the NS partials
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = (int*)lg;  // reuse LDS (every wave is past its lg reads: barrier above)
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t ticket = __hip_atomic_fetch_add(&a.cnt[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = ticket == (uint32_t)(a.NS - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&a.cnt[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm (graph replay)
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag || wave >= nimg) return;
  float m = -INFINITY, sum = 0.f;
  int bi = 0x7fffffff;
  const float4* p = a.part + (long)(b0 + wave) * a.NS;
  // every lane walks the NS partials in order (NS is small)
  for (int s = 0; s < a.NS; ++s) {
    const float4 q = p[s];
    if (q.z == 0.f) continue;  // empty split (no classes)
    const int qi = __float_as_int(q.y);
    if (q.x > m || (q.x == m && qi < bi)) {
      sum = sum * __expf(m - q.x) + q.z;
      m = q.x;
      bi = qi;
    } else {
      sum += q.z * __expf(q.x - m);
    }
  }
  if (lane == 0) {
    a.idx[b0 + wave] = bi;
    a.prob[b0 + wave] = 1.f / sum;
  }
}

}  // namespace

int head_splits(int B, int N, int num_cus) {
  const int groups = (B + kIPW - 1) / kIPW;
  const int tiles = (N + 15) / 16;
  int ns = 1;
  while (ns < 8 && (long)groups * ns * 2 <= num_cus && tiles / (ns * 2) >= 4) ns *= 2;
  return ns;
}

size_t head_ws_bytes(int max_batch) {
  // partials for up to 8 splits, then the group counters at the very end
  const size_t groups = (max_batch + kIPW - 1) / kIPW;
  return (size_t)max_batch * 8 * sizeof(float4) + ((groups * sizeof(uint32_t) + 255) & ~(size_t)255);
}

bool head_supported(int C, int N, int ldw, int Npad) {
  return C % 32 == 0 && C >= 32 && ldw >= C && ldw % 8 == 0 && Npad >= ((N + 15) / 16) * 16 && N > 0;
}

void head_fused(const void* x, const void* w, const float* bias, int B, int HW, int C, int N, int ldw, int Npad,
                float* logits, int32_t* idx, float* prob, void* ws, size_t ws_bytes, int num_cus, hipStream_t s) {
  if (B <= 0) return;
  if (!head_supported(C, N, ldw, Npad)) throw std::invalid_argument("head_fused: unsupported C/N/ldw");
  if (!x || !w || !bias || !logits || !idx || !prob || !ws) throw std::invalid_argument("head_fused: null pointer");
  const int groups = (B + kIPW - 1) / kIPW;
  const int tiles = (N + 15) / 16;
  const int ns = head_splits(B, N, num_cus);
  const size_t part_bytes = (size_t)B * ns * sizeof(float4);
  if (part_bytes + groups * sizeof(uint32_t) > ws_bytes) throw std::invalid_argument("head_fused: workspace too small");
  HeadArgs a;
  a.x = (const bf16*)x;
  a.w = (const bf16*)w;
  a.bias = bias;
  a.logits = logits;
  a.idx = idx;
  a.prob = prob;
  a.NS = ns;
  a.tiles_per_split = (tiles + ns - 1) / ns;
  // counters are the last `groups` words (zeroed at allocation, re-armed by each reducer)
  a.part = (float4*)ws;
  a.cnt = (uint32_t*)((uint8_t*)ws + ws_bytes) - groups;
  a.B = B;
  a.HW = HW;
  a.C = C;
  a.N = N;
  a.ldw = ldw;
  const size_t lds = (size_t)kIPW * (C + 8) * 2 + (size_t)kIPW * a.tiles_per_split * 16 * 4;
  if (lds > 160 * 1024) throw std::invalid_argument("head_fused: LDS budget exceeded");
  hipLaunchKernelGGL(head_kernel, dim3(groups, ns), dim3(256), lds, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
