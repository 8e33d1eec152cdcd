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
//  3. logits (+bias) to global fp32 and LDS; 256/IPW threads per image reduce
//     its split's (max, argmax, sum exp(x - max)), all images of the
//     workgroup in one pass, and store the partial;
//  4. the workgroup that draws the last ticket for group g loads all NS
//     partials of its images at once and merges them with a butterfly
//     (fixed order) (cdna_hip_programming.md §6 Guideline 16 counter recipe, sc1
//     form: relaxed agent-scope stores of the partials -> vmcnt(0) ->
//     barrier -> relaxed agent fetch_add; the reducer reads them with relaxed
//     agent-scope loads; no release/acquire fences, which would write back /
//     invalidate the XCD's whole L2 in every workgroup) and writes (class,
//     prob), then re-arms the counter.
// No workgroup waits on another, so any residency is correct.
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdlib>

namespace dmlc {

namespace {

constexpr int kIPW = 4;         // images per workgroup, pooling in the kernel (one wave each in the softmax)
constexpr int kIPWPooled = 16;  // images per workgroup on a pooled input (all 16 MFMA columns)
constexpr int kMaxSplits = 16;  // class splits (workgroups per image group); <= 256 / kIPWPooled

struct HeadArgs {
  const bf16* x;      // [B, HW, C]
  const bf16* pooled;  // POOLED: [B, C] bf16
  const bf16* w;      // [Npad, ldw]
  const float* bias;  // [Npad]
  float* logits;      // [B, N]
  int32_t* idx;
  float* prob;
  float4* part;       // [B, NS] (max, argmax bits, sum, -)
  uint32_t* cnt;      // [ceil(B / kIPW)], zero between launches
  int B, HW, C, N, ldw, tiles_per_split, NS;
  float scale;  // FP8 input: the e4m3 activation's dequantisation scale
  int ko;  // knock-out bits for timing experiments (head_pooled's ko, tools/head_bench.py): 2 = no fc loads
};

// Sum of n (power of two) values in the butterfly order of avgpool_global's
// xor-shuffle reduce: ((v0+v1)+(v2+v3))+((v4+v5)+(v6+v7)).
__device__ __forceinline__ float tree_sum(const float* v, int n) {
  float t[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = i < n ? v[i] : 0.f;
#pragma unroll
  for (int w = 1; w < 8; w <<= 1)
#pragma unroll
    for (int a = 0; a + w < 8; a += 2 * w)
      if (a + w < n) t[a] = t[a] + t[a + w];
  return t[0];
}

template <int TPG, int IPW, bool POOLED, bool FP8 = false>
__global__ __launch_bounds__(256) void head_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int kIPW = IPW;
  const int C = a.C;
  // pooled row stride (elements): C + 16, rows 32 B apart in bank space, so
  // the fc's fragment reads (lane: image lane & 15, 16-B chunk lane >> 4) are
  // conflict free for 4 and for 16 images (C + 8 was 2-way at 16;
  // tests/test_layouts_cpu.py::test_head_lds_layout)
  const int ldp = C + 16;
  bf16* pooled = (bf16*)smem;                                // [kIPW][ldp]
  // logits of the split: row stride nsplit + 4 floats, stored as one 16-B
  // chunk per lane (the 8 lanes of a store group: 8 images at 4-dword steps)
  float* lg = (float*)(smem + kIPW * ldp * 2);  // [kIPW][tiles_per_split*16 + 4]
  float* red = lg;  // pooling partials [TPG][kIPW][C] fp32 (dead before lg is written)
  const int g = blockIdx.x, split = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b0 = g * kIPW;
  const int nimg = min(kIPW, a.B - b0);
  // fc weights of this wave's first tile pair, issued before the pooling so
  // their latency overlaps it (every wave has at most one tile pair when the
  // split is <= 8 tiles, and one 512-deep K chunk when C <= 512): one memory
  // round trip less on the chain pool -> fc -> softmax -> merge
  const int col = lane & 15, kq = lane >> 4;
  const int nsplit = a.tiles_per_split * 16;
  const int lgs = nsplit + 4;
  const int n_begin = split * nsplit;
  // (pooled input: its rows arrive in one batch of loads, and the prefetched
  // weights next to them spilled)
  const bool pre = !POOLED && a.tiles_per_split <= 8 && C <= 512;
  bf16x8 pwa[16], pwb[16];
  float pbv[2][4];
  auto load_tile_pair = [&](int t, bf16x8* wa, bf16x8* wb, float (*bv)[4], int kc) __attribute__((always_inline)) {
    const int n0 = n_begin + t * 16;
    const bool two = t + 4 < a.tiles_per_split && n0 + 64 < a.N;
    // bias of this lane's 4 (+4) classes, in flight with the weight loads
    // (loaded after the MFMAs they cost a dependent round trip per tile)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[h][r] = (h == 0 || two) ? a.bias[n_begin + (t + 4 * h) * 16 + kq * 4 + r] : 0.f;
    const bf16* w0 = a.w + (long)(n0 + col) * a.ldw + kq * 8;
    const bf16* w1 = w0 + 64L * a.ldw;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int k = kc + 32 * u;
      if (k < C) {
        if (a.ko & 2) {
          wa[u] = bf16x8{};
          wb[u] = bf16x8{};
        } else {
          wa[u] = *(const bf16x8*)(w0 + k);
          if (two) wb[u] = *(const bf16x8*)(w1 + k);
        }
      }
    }
  };
  if (pre && wave < a.tiles_per_split && n_begin + wave * 16 < a.N) load_tile_pair(wave, pwa, pwb, pbv, 0);
  if constexpr (POOLED) {  // the last conv already pooled: bf16 [B, C] rows -> LDS
    // rows straight into LDS by LDS-DMA (global_load_lds_dwordx4, 1 KB =
    // 512 channels per wave instruction), all in flight at once: a
    // load-store loop waited a round trip per row (42 us at resnet50_fp8
    // b256, C = 2048)
    const int c8 = C / 8;
    if (C % 512 == 0) {
      const int cpr = C / 512;
      for (int k = wave; k < nimg * cpr; k += 4) {
        const int i = k / cpr, jb = k - i * cpr;
        dma16(a.pooled + (long)(b0 + i) * C + jb * 512 + lane * 8, pooled + i * ldp + jb * 512);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      for (int it = tid; it < nimg * c8; it += 256) {
        const int i = it / c8, cg = it - i * c8;
        *(uint4*)(pooled + i * ldp + cg * 8) = *(const uint4*)(a.pooled + (long)(b0 + i) * C + cg * 8);
      }
    }
    __syncthreads();
  } else {

  // ---- 1. average pool. avgpool_global's arithmetic: part p (0..7) of a
  // channel group sums pixels p, p+8, ... in order; the 8 parts combine in
  // butterfly order. Here TPG threads share a group's 8 parts (PPT each),
  // every thread issues all its loads of an image before adding, and the
  // TPG partials meet in LDS.
  const int c8 = C / 8;
  constexpr int PPT = 8 / TPG;
  constexpr int U = PPT >= 8 ? 2 : PPT >= 4 ? 4 : 8;  // pixels per part in flight
  const float inv = (FP8 ? a.scale : 1.f) / a.HW;  // (avgpool_global's factor)
  for (int it = tid; it < ((a.ko & 1) ? 0 : c8 * TPG); it += 256) {
    const int cg = it % c8, q = it / c8;
    for (int i = 0; i < nimg; ++i) {
      const long eoff = ((long)(b0 + i) * a.HW) * C + cg * 8;  // element offset
      const bf16* base = a.x + eoff;
      const uint8_t* base8 = (const uint8_t*)a.x + eoff;
      float ps[PPT][8];  // [part][channel]
#pragma unroll
      for (int pp = 0; pp < PPT; ++pp)
#pragma unroll
        for (int j = 0; j < 8; ++j) ps[pp][j] = 0.f;
      for (int c0 = 0; c0 < a.HW; c0 += 8 * U) {  // U pixels per part per round
        uint4 v[PPT][U];
#pragma unroll
        for (int pp = 0; pp < PPT; ++pp)
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int pix = c0 + (q * PPT + pp) + 8 * u;
            if constexpr (FP8) {  // 8 e4m3 channels
              const uint2 q8 = pix < a.HW ? *(const uint2*)(base8 + (long)pix * C) : make_uint2(0, 0);
              v[pp][u] = make_uint4(q8.x, q8.y, 0, 0);
            } else {
              v[pp][u] = pix < a.HW ? *(const uint4*)(base + (long)pix * C) : make_uint4(0, 0, 0, 0);
            }
          }
#pragma unroll
        for (int pp = 0; pp < PPT; ++pp)
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int pix = c0 + (q * PPT + pp) + 8 * u;
            if (pix < a.HW) {
              float f[8];
              if constexpr (FP8) {
                const int lo8 = (int)v[pp][u].x, hi8 = (int)v[pp][u].y;
                e4m3x4_to_f32((uint32_t)lo8, f);
                e4m3x4_to_f32((uint32_t)hi8, f + 4);
              } else {
                unpack8(v[pp][u], f);
              }
#pragma unroll
              for (int j = 0; j < 8; ++j) ps[pp][j] += f[j];
            }
          }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float col[8];
#pragma unroll
        for (int pp = 0; pp < 8; ++pp) col[pp] = pp < PPT ? ps[pp][j] : 0.f;
        red[((long)q * kIPW + i) * C + cg * 8 + j] = tree_sum(col, PPT);
      }
    }
  }
  __syncthreads();
  for (int it = tid; it < nimg * c8; it += 256) {
    const int cg = it % c8, i = it / c8;
    float s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float col[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) col[q] = q < TPG ? red[((long)q * kIPW + i) * C + cg * 8 + j] : 0.f;
      s[j] = tree_sum(col, TPG) * inv;
    }
    *(uint4*)(pooled + i * ldp + cg * 8) = pack8(s);
  }
  __syncthreads();
  }  // !POOLED

  // ---- 2./3. fc tiles on MFMA: lane holds D[class row (lane>>4)*4 + r][image lane&15].
  // K in chunks of 512: the chunk's 16 pooled fragments are read once from
  // LDS, then two tiles' 16 weight fragments each are loaded together so a
  // wave waits on global latency once per tile pair.
  const bool live = col < nimg;
  const bf16* prow = pooled + col * ldp + kq * 8;
  for (int t = wave; t < a.tiles_per_split; t += 8) {
    const int n0 = n_begin + t * 16;
    if (n0 >= a.N) break;
    const bool two = t + 4 < a.tiles_per_split && n0 + 64 < a.N;
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    float bv[2][4];
    for (int kc = 0; kc < C; kc += 512) {
      bf16x8 pb[16], wa[16], wb[16];
      if (pre) {  // (t == wave, kc == 0: the prefetched pair)
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          wa[u] = pwa[u];
          wb[u] = pwb[u];
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 4; ++r) bv[h][r] = pbv[h][r];
      } else {
        load_tile_pair(t, wa, wb, bv, kc);
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int k = kc + 32 * u;
        pb[u] = (live && k < C) ? *(const bf16x8*)(prow + k) : bf16x8{};
      }
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (kc + 32 * u < C) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[u], pb[u], acc0, 0, 0, 0);
          if (two) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[u], pb[u], acc1, 0, 0, 0);
        }
    }
    if (live) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !two) break;
        const floatx4 acc = h ? acc1 : acc0;
        const int tt = t + 4 * h;
        floatx4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n_begin + tt * 16 + kq * 4 + r;
          v[r] = acc[r] + bv[h][r];
          if (n < a.N) a.logits[(long)(b0 + col) * a.N + n] = v[r];
        }
        *(floatx4*)(lg + col * lgs + tt * 16 + kq * 4) = v;
      }
    }
  }
  __syncthreads();

  // ---- per image: this split's (max, argmax, sum exp(x - max)). TPI
  // threads per image (16 with 16 images per workgroup, 64 with 4), all
  // images in one pass; ties go to the lower class.
  constexpr int TPI = 256 / kIPW;
  static_assert(TPI <= 64 && 64 % TPI == 0, "an image's threads must sit in one wave");
  const int im = tid / TPI, li = tid % TPI;
  const bool img_live = im < nimg;
  const int n_end = min(a.N, n_begin + nsplit);
  float best = -INFINITY, s = 0.f;
  int bi = 0x7fffffff;
  if (img_live)
    for (int n = n_begin + li; n < n_end; n += TPI) {
      const float v = lg[im * lgs + (n - n_begin)];
      if (v > best) {
        best = v;
        bi = n;
      }
    }
#pragma unroll
  for (int o = TPI / 2; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) {
      best = ov;
      bi = oi;
    }
  }
  if (img_live)
    for (int n = n_begin + li; n < n_end; n += TPI) s += __expf(lg[im * lgs + (n - n_begin)] - best);
#pragma unroll
  for (int o = TPI / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (a.NS == 1) {
    if (img_live && li == 0) {
      a.idx[b0 + im] = bi;
      a.prob[b0 + im] = 1.f / s;
    }
    return;
  }
  if (img_live && li == 0) {  // relaxed agent-scope atomic stores = sc1 write-through: no release fence needed
    float* q = (float*)(a.part + (long)(b0 + im) * a.NS + split);
    __hip_atomic_store(q, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, __int_as_float(bi), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 2, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- 4. last arriver of group g combines the NS partials: lane li of an
  // image's TPI threads loads partial li (all loads of the workgroup in
  // flight together), then a butterfly merge (fixed order: deterministic)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = (int*)lg;  // reuse LDS (every wave is past its lg reads: barrier above)
  if (tid == 0) {
    const uint32_t ticket = __hip_atomic_fetch_add(&a.cnt[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = ticket == (uint32_t)(a.NS - 1);
    if (last) __hip_atomic_store(&a.cnt[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm (graph replay)
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  float m = -INFINITY, sum = 0.f;
  int mi = 0x7fffffff;
  if (img_live && li < a.NS) {
    const float* pq = (const float*)(a.part + (long)(b0 + im) * a.NS + li);  // sc1 loads of the sc1-stored partials
    m = __hip_atomic_load(pq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    mi = __float_as_int(__hip_atomic_load(pq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    sum = __hip_atomic_load(pq + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (sum == 0.f) {  // empty split (no classes)
      m = -INFINITY;
      mi = 0x7fffffff;
    }
  }
#pragma unroll
  for (int o = 1; o < TPI; o <<= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(sum, o, 64);
    const int oi = __shfl_xor(mi, o, 64);
    if (os == 0.f) continue;
    if (sum == 0.f) {
      m = om;
      mi = oi;
      sum = os;
    } else if (om > m || (om == m && oi < mi)) {
      sum = sum * __expf(m - om) + os;
      m = om;
      mi = oi;
    } else {
      sum += os * __expf(om - m);
    }
  }
  if (img_live && li == 0) {
    a.idx[b0 + im] = mi;
    a.prob[b0 + im] = 1.f / sum;
  }
}

}  // namespace

int head_splits_ipw(int B, int N, int num_cus, int ipw) {
  const int groups = (B + ipw - 1) / ipw;
  const int tiles = (N + 15) / 16;
  int ns = 1;
  // (query batches: down to one 16-class tile per wave, 16 splits for 1000
  // classes: the fc is the longest step of the head's chain there)
  const int min_tiles = B <= ipw ? 2 : 4;
  while (ns < kMaxSplits && (long)groups * ns * 2 <= num_cus && tiles / (ns * 2) >= min_tiles) ns *= 2;
  if (B > ipw) ns = std::min(ns, 8);  // (throughput batches: measured with at most 8)
  // pooled head at throughput batches: 16 splits while that stays within one
  // workgroup per CU (B = 256: 16 image groups x 16), each workgroup streaming
  // half the fc weights of an 8-way split: ResNet50 (C = 2048) 18.2 vs 23.4 us,
  // ResNet18 (C = 512) 10.4 vs 11.2 us (tools/head_bench.py, profiles/r5_head_splits.txt)
  if (ipw == kIPWPooled && B > ipw && (long)groups * kMaxSplits <= num_cus && tiles >= 2 * kMaxSplits) ns = kMaxSplits;
  return ns;
}

int head_splits(int B, int N, int num_cus) { return head_splits_ipw(B, N, num_cus, kIPW); }

int head_pooled_splits(int B, int N, int num_cus) { return head_splits_ipw(B, N, num_cus, kIPWPooled); }

size_t head_ws_bytes(int max_batch) {
  // partials for up to kMaxSplits splits, then the group counters at the very end
  const size_t groups = (max_batch + kIPW - 1) / kIPW;
  return (size_t)max_batch * kMaxSplits * sizeof(float4) + ((groups * sizeof(uint32_t) + 255) & ~(size_t)255);
}

bool head_supported(int C, int N, int ldw, int Npad) {
  return C % 32 == 0 && C >= 32 && ldw >= C && ldw % 8 == 0 && Npad >= ((N + 15) / 16) * 16 && N > 0;
}

void head_fused(const void* x, const void* w, const float* bias, int B, int HW, int C, int N, int ldw, int Npad,
                float* logits, int32_t* idx, float* prob, void* ws, size_t ws_bytes, int num_cus, hipStream_t s,
                bool in_fp8, float scale) {
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
  a.ko = 0;
  a.scale = scale;
  const int c8 = C / 8, tpg = c8 >= 256 ? 1 : c8 >= 128 ? 2 : c8 >= 64 ? 4 : 8;
  const size_t lds = (size_t)kIPW * (C + 16) * 2 +
                     std::max((size_t)kIPW * (a.tiles_per_split * 16 + 4) * 4, (size_t)tpg * kIPW * C * 4);
  if (lds > 160 * 1024) throw std::invalid_argument("head_fused: LDS budget exceeded");
  if (in_fp8) {  // ResNet50 e4m3: the last bottleneck's output pooled straight from e4m3
    if (tpg != 1) throw std::invalid_argument("head_fused: e4m3 input needs C >= 2048");
    hipLaunchKernelGGL((head_kernel<1, kIPW, false, true>), dim3(groups, ns), dim3(256), lds, s, a);
    DMLC_HIP_CHECK(hipGetLastError());
    return;
  }
  switch (tpg) {
    case 1: hipLaunchKernelGGL((head_kernel<1, kIPW, false>), dim3(groups, ns), dim3(256), lds, s, a); break;
    case 2: hipLaunchKernelGGL((head_kernel<2, kIPW, false>), dim3(groups, ns), dim3(256), lds, s, a); break;
    case 4: hipLaunchKernelGGL((head_kernel<4, kIPW, false>), dim3(groups, ns), dim3(256), lds, s, a); break;
    default: hipLaunchKernelGGL((head_kernel<8, kIPW, false>), dim3(groups, ns), dim3(256), lds, s, a); break;
  }
  DMLC_HIP_CHECK(hipGetLastError());
}

void head_pooled(const void* pooled, const void* w, const float* bias, int B, int C, int N, int ldw, int Npad,
                 float* logits, int32_t* idx, float* prob, void* ws, size_t ws_bytes, int num_cus, hipStream_t s,
                 int ns_override, int ko) {
  if (B <= 0) return;
  if (!head_supported(C, N, ldw, Npad) || C % 8) throw std::invalid_argument("head_pooled: unsupported C/N/ldw");
  if (!pooled || !w || !bias || !logits || !idx || !prob || !ws || ((uintptr_t)pooled & 15))
    throw std::invalid_argument("head_pooled: null / misaligned pointer");
  constexpr int ipw = kIPWPooled;
  const int groups = (B + ipw - 1) / ipw;
  const int tiles = (N + 15) / 16;
  const int ns = ns_override > 0 ? std::min(ns_override, kMaxSplits) : head_splits_ipw(B, N, num_cus, ipw);
  const size_t part_bytes = (size_t)B * ns * sizeof(float4);
  if (part_bytes + groups * sizeof(uint32_t) > ws_bytes) throw std::invalid_argument("head_pooled: workspace too small");
  HeadArgs a;
  a.x = nullptr;
  a.pooled = (const bf16*)pooled;
  a.w = (const bf16*)w;
  a.bias = bias;
  a.logits = logits;
  a.idx = idx;
  a.prob = prob;
  a.NS = ns;
  a.tiles_per_split = (tiles + ns - 1) / ns;
  a.part = (float4*)ws;
  a.cnt = (uint32_t*)((uint8_t*)ws + ws_bytes) - groups;
  a.B = B;
  a.HW = 1;
  a.C = C;
  a.N = N;
  a.ldw = ldw;
  a.ko = ko;
  const size_t lds = (size_t)ipw * (C + 16) * 2 + (size_t)ipw * (a.tiles_per_split * 16 + 4) * 4;
  if (lds > 160 * 1024) throw std::invalid_argument("head_pooled: LDS budget exceeded");
  hipLaunchKernelGGL((head_kernel<1, kIPWPooled, true>), dim3(groups, ns), dim3(256), lds, s, a);
  DMLC_HIP_CHECK(hipGetLastError());
}

}  // namespace dmlc
