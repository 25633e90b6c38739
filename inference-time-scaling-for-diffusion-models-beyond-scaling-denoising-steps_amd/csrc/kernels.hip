// Non-GEMM kernels of the UNet step (gfx950): GroupNorm(+SiLU) over (dual-source)
// NHWC activations, single-head attention core, head conv, tail conv fused with
// the ancestral-sampler update, timestep/label embedding MLPs, per-candidate
// verifiers, and the counter-based Philox normal generator.
#include <math.h>

#include <algorithm>
#include <type_traits>

#include "common.h"

namespace itsd {

int g_attn_aq = 0;  // attn_mfma_kernel queries per block: 0 auto (32 below 512 blocks), 32, 64
int g_attn_cs = 0;  // attn_mfma_kernel output-channel slices per block row: 0 auto, else forced

// ============================================================================ GroupNorm
// nn.GroupNorm(32, C, eps=1e-5) (Model.py:132,171,180,253) with optional Swish over
// the channel concat of two NHWC sources (the up path's torch.cat, Model.py:280; a
// group may straddle the two sources). The statistics come from the producers'
// channel slabs (conv epilogue / head kernel): per image, the group's sum and sum
// of squares are reduced in fp64 (fixed order: deterministic), mean/biased var ->
// a = rstd*gamma, b = beta - mean*a per channel in LDS; the block then streams its
// pixel range with 16-B loads/stores: y = silu(x*a + b).
template <typename T>
__global__ __launch_bounds__(256) void gn_apply_kernel(GNArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);
  __shared__ float coef[2][2048];
  __shared__ float gst[32][2];
  const int img = blockIdx.y, tid = threadIdx.x;
  const int C = a.C1 + a.C2, gs = C / 32;
  const int spi1 = stat_spi(a.HW, a.spi1), spi2 = stat_spi(a.HW, a.spi2);
  // loads that do not depend on the statistics are issued first (one memory round trip for
  // the whole block instead of three): this block's 4 x 256 data chunks (host:
  // chunks_per_block == 1024) and gamma / beta of the channels this thread finalizes
  const unsigned cpp = C / EPC;  // chunks per pixel
  const unsigned total = (unsigned)a.HW * cpp;
  const unsigned c0 = blockIdx.x * (unsigned)a.chunks_per_block;
  const unsigned c1 = min(total, c0 + (unsigned)a.chunks_per_block);
  const T* s1 = (const T*)a.src1 + (size_t)img * a.HW * a.C1;
  const T* s2 = a.src2 ? (const T*)a.src2 + (size_t)img * a.HW * a.C2 : nullptr;
  T* dst = (T*)a.dst + (size_t)img * a.HW * C;
  u32x4 x[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const unsigned idx = c0 + u * 256 + tid;
    x[u] = u32x4{0u, 0u, 0u, 0u};
    if (idx < c1) {
      const int p = (int)(idx / cpp);
      const int c = (int)(idx - (unsigned)p * cpp) * EPC;
      x[u] = c < a.C1 ? *(const u32x4*)(s1 + (size_t)p * a.C1 + c) : *(const u32x4*)(s2 + (size_t)p * a.C2 + (c - a.C1));
    }
  }
  float gam[8], bet[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int c = tid + 256 * u;
    gam[u] = c < C ? a.gamma[c] : 0.f;
    bet[u] = c < C ? a.beta[c] : 0.f;
  }
  {
    const int g = tid >> 3, l8 = tid & 7;
    // the group's (channel, slot) items: its src1 channels x spi1 slots, then src2 x spi2
    const int c0 = g * gs, nc1 = max(0, min(a.C1 - c0, gs)), n1 = nc1 * spi1, n = n1 + (gs - nc1) * spi2;
    double s = 0.0, q = 0.0;
    for (int k = l8; k < n; k += 8) {
      const bool s1 = k < n1;
      const int spi = s1 ? spi1 : spi2, kk = s1 ? k : k - n1;
      const int c = c0 + (s1 ? 0 : nc1) + kk / spi;
      const long long sl = (long long)img * spi + (kk % spi);
      const float* st = s1 ? a.st1 : a.st2;
      const int Cs = s1 ? a.C1 : a.C2, cc = s1 ? c : c - a.C1;
      s += (double)st[(sl * 2) * Cs + cc];
      q += (double)st[(sl * 2 + 1) * Cs + cc];
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) { s += __shfl_xor(s, o, 64); q += __shfl_xor(q, o, 64); }
    if (l8 == 0) {
      const double E = (double)gs * a.HW;
      const double mean = s / E;
      double var = q / E - mean * mean;
      var = var > 0.0 ? var : 0.0;
      gst[g][0] = (float)mean;
      gst[g][1] = (float)(1.0 / sqrt(var + (double)a.eps));
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int c = tid + 256 * u;
    if (c < C) {
      const int g = c / gs;
      const float sc = gst[g][1] * gam[u];
      coef[0][c] = sc;
      coef[1][c] = bet[u] - gst[g][0] * sc;
    }
  }
  __syncthreads();
  {
    const unsigned i0 = c0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned idx = i0 + u * 256 + tid;
      if (idx >= c1) continue;
      const int p = (int)(idx / cpp);
      const int c = (int)(idx - (unsigned)p * cpp) * EPC;
      const T* xe = (const T*)&x[u];
      u32x4 y;
      T* ye = (T*)&y;
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        float v = Elem<T>::tof(xe[e]) * coef[0][c + e] + coef[1][c + e];
        if (a.silu) v = silu(v);
        ye[e] = Elem<T>::to(v);
      }
      *(u32x4*)(dst + (size_t)p * C + c) = y;
    }
  }
}

template <typename T>
hipError_t launch_groupnorm(const GNArgs& a0, int n, hipStream_t s) {
  constexpr int EPC = 16 / (int)sizeof(T);
  GNArgs a = a0;
  const long long total = (long long)a.HW * ((a.C1 + a.C2) / EPC);
  if (a.C1 + a.C2 > 2048) return hipErrorInvalidValue;  // coefficient table / 8 channels per thread
  a.chunks_per_block = 1024;  // = 4 chunks x 256 threads: the kernel's single batch
  const int bpi = (int)((total + a.chunks_per_block - 1) / a.chunks_per_block);
  ITSD_LAUNCH(gn_apply_kernel<T>, dim3(bpi, n), dim3(256), 0, s, a);
  return hipGetLastError();
}
template hipError_t launch_groupnorm<float>(const GNArgs&, int, hipStream_t);
template hipError_t launch_groupnorm<bf16_t>(const GNArgs&, int, hipStream_t);


// ============================================================================ attention core
// AttnBlock core (Model.py:152-161): w = softmax(q k^T * C^-0.5) ; h = w v, single head,
// S = H*W tokens of width C. Input is the fused q|k|v projection [n][S][3C].
// One block per (32-query chunk, image); the 32 x S score tile lives in LDS (S <= 256).
__host__ __device__ inline int att_qc(int S) { int q = 8192 / S; return q < 1 ? 1 : (q > 32 ? 32 : q); }
template <typename T>
__global__ __launch_bounds__(256) void attn_kernel(AttnArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) float P[];  // [ATT_QC][S]
  const int img = blockIdx.y, q0 = blockIdx.x * att_qc(a.S);
  const int S = a.S, C = a.C, C3 = 3 * a.C;
  const T* base = (const T*)a.qkv + (size_t)img * S * C3;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nq = min(att_qc(S), S - q0);
  // scores
  for (int idx = tid; idx < nq * S; idx += 256) {
    const int r = idx / S, j = idx - r * S;
    const T* qp = base + (size_t)(q0 + r) * C3;
    const T* kp = base + (size_t)j * C3 + C;
    float acc = 0.0f;
    for (int c = 0; c < C; c += EPC) {
      const u32x4 qv = *(const u32x4*)(qp + c);
      const u32x4 kv = *(const u32x4*)(kp + c);
      const T* qe = (const T*)&qv;
      const T* ke = (const T*)&kv;
#pragma unroll
      for (int e = 0; e < EPC; ++e) acc = fmaf(Elem<T>::tof(qe[e]), Elem<T>::tof(ke[e]), acc);
    }
    P[r * S + j] = acc * a.scale;
  }
  __syncthreads();
  // softmax rows (one wave per row)
  for (int r = wid; r < nq; r += 4) {
    float m = -INFINITY;
    for (int j = lane; j < S; j += 64) m = fmaxf(m, P[r * S + j]);
    m = wave_max(m);
    float sum = 0.0f;
    for (int j = lane; j < S; j += 64) { const float e = expf(P[r * S + j] - m); P[r * S + j] = e; sum += e; }
    sum = wave_sum(sum);
    const float inv = 1.0f / sum;
    for (int j = lane; j < S; j += 64) P[r * S + j] *= inv;
  }
  __syncthreads();
  // out = P v
  T* out = (T*)a.out + (size_t)img * S * C;
  for (int idx = tid; idx < nq * C; idx += 256) {
    const int r = idx / C, c = idx - r * C;
    const T* vp = base + 2 * C + c;
    float acc = 0.0f;
    for (int j = 0; j < S; ++j) acc = fmaf(P[r * S + j], Elem<T>::tof(vp[(size_t)j * C3]), acc);
    out[(size_t)(q0 + r) * C + c] = Elem<T>::to(acc);
  }
}

// MFMA attention (bf16 throughput path, S <= 256, S % 16 == 0, C % 32 == 0).
// One block per (64-query chunk, image), 4 waves:
//  1. scores = q k^T * C^-0.5 on v_mfma_f32_32x32x16_bf16, q and k rows read straight
//     from the q|k|v projection (both operands are contiguous 16-B fragments);
//  2. row softmax in fp32 over LDS, P rounded to bf16 in LDS;
//  3. O^T = V^T P^T on MFMA with V^T channel-major (written so by the qkv conv epilogue)
//     -> 4 consecutive channels per lane per store.
// AQ = queries per block (64, or 32 to give small-S launches twice the blocks: at S = 64 one
// block per image left 1 wave per SIMD, 70 % of cycles waiting on memory).
constexpr int ATT_AQ = 64;
template <int AQ>
__global__ __launch_bounds__(256) void attn_mfma_kernel(AttnArgs a) {
  constexpr int NQT = AQ / 32, WPQ = 4 / NQT;  // query tiles; waves per query tile in phase 1
  extern __shared__ __attribute__((aligned(16))) char asm_[];
  const int S = a.S, C = a.C, C3 = 3 * a.C;
  const int Sp = (S + 31) & ~31;
  const int SROW = Sp + 4;            // fp32 score row
  const int PROW = Sp * 2 + 16;       // bf16 P row (bytes), odd 16-B slot stride
  float* Sc = (float*)asm_;
  char* Pm = asm_ + AQ * SROW * 4;
  const int img = blockIdx.y, q0 = blockIdx.x * AQ;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, rl = lane & 31, hh = lane >> 5;
  const bf16_t* base = (const bf16_t*)a.qkv + (size_t)img * S * C3;
  const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
  {
    const int qi = wid / WPQ;
    const int q = q0 + qi * 32 + rl;
    const bool qv = q < S;
    const bf16_t* qp = base + (size_t)(qv ? q : 0) * C3 + 8 * hh;
    for (int kj = wid % WPQ; kj < Sp / 32; kj += WPQ) {
      const int key = kj * 32 + rl;
      const bool kv = key < S;
      const bf16_t* kp = base + (size_t)(kv ? key : 0) * C3 + C + 8 * hh;
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      // q / k fragments straight from the q|k|v rows, 8 k-steps of loads in flight before
      // their MFMAs (one dependent global round trip per 128 channels, not per 16)
      for (int c0 = 0; c0 < C; c0 += 128) {
        bf16x8 af[8], bk[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const bool in = c0 + 16 * i < C;
          af[i] = (qv && in) ? *(const bf16x8*)(qp + c0 + 16 * i) : z8;
          bk[i] = (kv && in) ? *(const bf16x8*)(kp + c0 + 16 * i) : z8;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (c0 + 16 * i < C) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bk[i], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = qi * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        Sc[row * SROW + kj * 32 + rl] = kv ? acc[r] * a.scale : -INFINITY;
      }
    }
  }
  __syncthreads();
  for (int r = wid * (AQ / 4); r < (wid + 1) * (AQ / 4); ++r) {
    float m = -INFINITY;
    for (int j = lane; j < Sp; j += 64) m = fmaxf(m, Sc[r * SROW + j]);
    m = wave_max(m);
    float sum = 0.f;
    for (int j = lane; j < Sp; j += 64) {
      const float e = expf(Sc[r * SROW + j] - m);
      Sc[r * SROW + j] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    const float inv = 1.0f / sum;
    for (int j = lane; j < Sp; j += 64) ((bf16_t*)(Pm + r * PROW))[j] = f2bf(Sc[r * SROW + j] * inv);
  }
  __syncthreads();
  const bf16_t* vt = (const bf16_t*)a.vt + (size_t)img * C * S;
  bf16_t* out = (bf16_t*)a.out + (size_t)img * S * C;
  // O^T tiles (32 channels x 32 queries) t = wid + 4u: four tiles per pass with all their V^T
  // loads of 4 k-steps in flight at once (one dependent global round trip per pass and 64 keys)
  // blockIdx.z splits the output channels (gridDim.z slices of C / 32 / gridDim.z channel tiles;
  // every slice recomputes the block's scores, which are cheap next to the PV loads it spreads)
  const int ctiles = (C / 32) / gridDim.z, cbase = blockIdx.z * ctiles;
  const int ntile = NQT * ctiles;
  for (int t0 = wid; t0 < ntile; t0 += 16) {
    f32x16 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
    for (int k0 = 0; k0 < Sp; k0 += 64) {
      bf16x8 av[4][4], bp[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + 4 * u, ci = cbase + t / NQT, qi = t % NQT;
        const bool tv = t < ntile;
        const bf16_t* vp = vt + (size_t)((tv ? ci : 0) * 32 + rl) * S + 8 * hh;
        const char* pp = Pm + (qi * 32 + rl) * PROW + 16 * hh;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = k0 + 16 * i;
          av[u][i] = (tv && k < Sp && k + 8 * hh < S) ? *(const bf16x8*)(vp + k) : z8;
          bp[u][i] = k < Sp ? *(const bf16x8*)(pp + 2 * k) : z8;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (t0 + 4 * u < ntile && k0 + 16 * i < Sp)
            acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[u][i], bp[u][i], acc[u], 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + 4 * u, ci = cbase + t / NQT, qi = t % NQT;
      const int q = q0 + qi * 32 + rl;
      if (t < ntile && q < S) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = ci * 32 + 8 * g + 4 * hh;
          uint2 w2;
          w2.x = (uint32_t)f2bf(acc[u][4 * g]) | ((uint32_t)f2bf(acc[u][4 * g + 1]) << 16);
          w2.y = (uint32_t)f2bf(acc[u][4 * g + 2]) | ((uint32_t)f2bf(acc[u][4 * g + 3]) << 16);
          *(uint2*)(out + (size_t)q * C + c) = w2;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------- fused AttnBlock, S = 64
// attn_block_kernel<C>: one image's whole AttnBlock (Model.py:145-164) per block -- Arch A's 8x8
// level (S = 64 tokens, C = 384), where the unfused path ran a materialised GroupNorm, the q|k|v
// 1x1 conv (C x 3C over 64 tokens), the attention kernel and the proj conv as four launches with
// three HBM round trips, 2 % of MFMA peak in the attention itself. Here:
//   0. GroupNorm(32, C) of x: group mean / rstd in fp64 from the producer's statistics slab, x
//      staged as hn = bf16(x a + b) in LDS ([token][C], 16-B chunks XOR-swizzled by token & 15);
//   1. V^T = (hn Wv^T + bv)^T -> LDS [C][64] (D[token][c] with Wv fragments as the B operand, so a
//      lane holds 4 consecutive tokens of one channel: 8-B channel-major stores);
//   2. per 128-channel chunk: Q_c, K_c = hn W^T + b (D[c][token]: weights as A) -> LDS [64][128],
//      and the scores S^T[key][query] += K_c Q_c^T accumulate in registers (one 32x32 tile a wave);
//   3. softmax over keys in fp32 (S^T staged through LDS, 4 lanes a query), P [query][key] bf16;
//   4. O^T = V^T P^T (both operands from LDS) -> O [token][C] bf16 in LDS (hn's space);
//   5. out = x + O Wp^T + bp, one bf16 rounding, 16-B stores (permlane32 swap), and the consumer
//      GroupNorm statistics of out (one slot per image) by lane butterflies.
// Roundings as the unfused path: hn, q / k / v, P and O in bf16, fp32 accumulation.
// 8 waves (512 threads, __launch_bounds__(512, 1)): the weight-streaming phases give each wave whole
// 32-channel blocks (V / proj: blocks w, w + 8; q|k: Q on waves 0-3, K on 4-7), the score / softmax / PV
// phases split queries and channel blocks over the waves; weights (fragment-packed [Cout/32][K/16][64][8]
// bf16) stream from L2 into VGPRs with an 8-k-step prefetch; one block per image.

#ifdef ITSD_STAMPS
// Diagnostic build only: attn_block_kernel's phase timeline (s_memrealtime), [block % 1024][wave][slot]
__device__ unsigned long long g_stamps_attn[1024 * 16 * 8];
__device__ __forceinline__ void atl(int slot) {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) g_stamps_attn[((blockIdx.x & 1023) * 16 + (threadIdx.x >> 6)) * 8 + slot] = t;
  __builtin_amdgcn_sched_barrier(0);
}
#define ATL(slot) atl(slot)
#else
#define ATL(slot)
#endif

// (round 4's 4-images-a-block form for the 4x4 middle block, S = 16, measured slower than the unfused ops
// at N = 32 and equal at N = 256, was removed in round 5)
#ifndef ITSD_ATTN_PF
#define ITSD_ATTN_PF 8
#endif
template <int C>
__global__ __launch_bounds__(512, 1) void attn_block_kernel(AttnBlockArgs a) {
  constexpr int S = 64, KS = C / 16, CB = C / 32, CBW = CB / 4, NCH = C / 128, PF = ITSD_ATTN_PF;
  static_assert(C % 128 == 0, "C");
  constexpr int R_VT = S * C * 2, R_QK = R_VT + C * 128, R_GS = R_QK + 2 * S * 256, R_ST = R_GS + 32 * 2 * 4;
  __shared__ __attribute__((aligned(16))) char sm[R_ST + 2 * C * 2 * 4];
  const int tid = threadIdx.x, lane = tid & 63, rl = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wq = w & 3, wt = w >> 2;  // wave = (channel-block group, token block)
  const int img = blockIdx.x;
  ATL(0);
  const bf16_t* x = a.x + (size_t)img * S * C;
  // [row][C] bf16 image, 16-B chunk ch of row r at (ch ^ (r & 15))
  auto rowc = [](int r, int ch, int rowbytes) { return r * rowbytes + ((ch ^ (r & 15)) << 4); };
  // [row][64] bf16 image (128-B rows), chunk ch of row r at ch ^ ((r >> 1) & 7)
  auto row64 = [](int r, int ch) { return r * 128 + ((ch ^ ((r >> 1) & 7)) << 4); };
  auto frag = [&](const bf16_t* W, int cb, int st) -> const bf16x8* {
    return (const bf16x8*)((const char*)W + ((size_t)cb * KS + st) * 1024 + lane * 16);
  };
  // ---- 0. GroupNorm statistics -> (mean, rstd) per group; hn (all x loads issued before any use)
  constexpr int XU = S * (C / 8) / 512;  // 16-B units of x per thread
  u32x4 xv[XU];
#pragma unroll
  for (int i = 0; i < XU; ++i) {
    const int u = tid + 512 * i, t = u / (C / 8), ch = u - t * (C / 8);
    xv[i] = *(const u32x4*)(x + (size_t)t * C + ch * 8);
  }
  // (round 5) every weight stream's first PF fragments are issued ahead of its phase: phase 1's here, behind the
  // x loads (they arrive during the group statistics and hn staging), phase 2's chunk 0 in phase 1's last PF
  // steps and chunk c + 1 after chunk c's Q / K stores, phase 5's before the softmax -- no phase opens with a
  // memory round trip
  constexpr int NBW = (CB + 7) / 8;
  bf16x8 bw[PF][NBW];
#pragma unroll
  for (int p = 0; p < PF; ++p)
#pragma unroll
    for (int b = 0; b < NBW; ++b)
      if (w + 8 * b < CB) bw[p][b] = *frag(a.wqkv, 2 * CB + w + 8 * b, p);
  bf16x8 fa[PF];  // phase 2's ring (Q / K weights of channel block 4 ch + w % 4)
  float* gs = (float*)(sm + R_GS);  // [32 groups][mean, rstd]
  if (tid < 256) {
    const int g = tid >> 3, l8 = tid & 7, gsz = C / 32, n_it = gsz * a.spi;
    double s = 0.0, q = 0.0;
    for (int k = l8; k < n_it; k += 8) {
      const int c = g * gsz + k / a.spi;
      const long long sl = (long long)img * a.spi + k % a.spi;
      s += (double)a.st[(sl * 2) * C + c];
      q += (double)a.st[(sl * 2 + 1) * C + c];
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      s += __shfl_xor(s, o, 64);
      q += __shfl_xor(q, o, 64);
    }
    if (l8 == 0) {
      const double E = (double)gsz * S, mean = s / E;
      double var = q / E - mean * mean;
      var = var > 0.0 ? var : 0.0;
      gs[g * 2] = (float)mean;
      gs[g * 2 + 1] = (float)(1.0 / sqrt(var + 1e-5));
    }
  }
  __syncthreads();
  ATL(1);  // group statistics
#pragma unroll
  for (int i = 0; i < XU; ++i) {
    const int u = tid + 512 * i, t = u / (C / 8), ch = u - t * (C / 8), c0 = ch * 8;
    uint32_t o[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      float y[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int c = c0 + 2 * e2 + h2, g = c / (C / 32);  // (an 8-channel chunk may straddle two groups)
        const float mean = gs[2 * g], rstd = gs[2 * g + 1];
        const float sc = rstd * a.gamma[c];
        const float xf = __uint_as_float(h2 ? (xv[i][e2] & 0xffff0000u) : (xv[i][e2] << 16));
        y[h2] = xf * sc + (a.beta[c] - mean * sc);
      }
      o[e2] = pk_bf16(y[0], y[1]);
    }
    *(u32x4*)(sm + rowc(t, ch, C * 2)) = u32x4{o[0], o[1], o[2], o[3]};
  }
  __syncthreads();
  // hn fragment of (token row r, k-step st): lane (rl, hh) reads channels 16 st + 8 hh ..
  auto hn_frag = [&](int r, int st) { return *(const bf16x8*)(sm + rowc(r, 2 * st + hh, C * 2)); };
  const int tr = 32 * wt + rl;  // this wave's token / query row

  // The weight-streaming phases (1, 2, 5) give each wave whole 32-channel blocks over BOTH token
  // blocks, so every weight fragment is streamed once per block (the two token-block waves of a
  // channel group used to stream the same fragments): V^T and proj -- channel blocks w, w + 8 (NBW a
  // wave at most); q|k -- wave w computes Q (w < 4) or K (w >= 4) of block 4 ch + w % 4. Every
  // output's k order is unchanged.
  // ---- 1. V^T: D[token][c] = hn Wv^T; wave w: channel blocks w + 8 b x both token blocks
  {
    f32x16 acc[2][NBW];
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
      for (int b = 0; b < NBW; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[tb][b][r] = 0.f;
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      bf16x8 cur[NBW];
#pragma unroll
      for (int b = 0; b < NBW; ++b) cur[b] = bw[st % PF][b];
      if (st + PF < KS) {
#pragma unroll
        for (int b = 0; b < NBW; ++b)
          if (w + 8 * b < CB) bw[st % PF][b] = *frag(a.wqkv, 2 * CB + w + 8 * b, st + PF);
      } else {
        fa[st + PF - KS] = *frag(a.wqkv, (w >> 2) * CB + wq, st + PF - KS);
      }
#pragma unroll
      for (int tb = 0; tb < 2; ++tb) {
        const bf16x8 h0 = hn_frag(32 * tb + rl, st);
#pragma unroll
        for (int b = 0; b < NBW; ++b)
          if (w + 8 * b < CB) acc[tb][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(h0, cur[b], acc[tb][b], 0, 0, 0);
      }
    }
    // lane: channel c = 32 cb + rl (column), tokens 32 tb + 8 g + 4 hh + e (rows)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
      for (int b = 0; b < NBW; ++b) {
        if (w + 8 * b >= CB) continue;
        const int c = 32 * (w + 8 * b) + rl;
        const float bv = a.bqkv[2 * C + c];
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *(uint2*)(sm + R_VT + row64(c, 4 * tb + g) + 8 * hh) =
              uint2{pk_bf16(acc[tb][b][4 * g] + bv, acc[tb][b][4 * g + 1] + bv), pk_bf16(acc[tb][b][4 * g + 2] + bv, acc[tb][b][4 * g + 3] + bv)};
      }
  }
  ATL(2);  // hn staged + V^T computed (wave's own)
  // ---- 2. Q_c, K_c per 128-channel chunk; S^T (keys x queries) tile w (waves 0..3) in registers
  f32x16 sacc;
#pragma unroll
  for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
  char* const Qc = sm + R_QK;
  char* const Kc = sm + R_QK + S * 256;
  for (int ch = 0; ch < NCH; ++ch) {
    {  // wave w: Q_c (w < 4) or K_c (w >= 4), channel block 4 ch + w % 4, both token blocks
      const int isk = w >> 2, cb = isk * CB + 4 * ch + wq;
      f32x16 aa[2];
#pragma unroll
      for (int tb = 0; tb < 2; ++tb)
#pragma unroll
        for (int r = 0; r < 16; ++r) aa[tb][r] = 0.f;
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        const bf16x8 w_ = fa[st % PF];
        if (st + PF < KS) fa[st % PF] = *frag(a.wqkv, cb, st + PF);
#pragma unroll
        for (int tb = 0; tb < 2; ++tb) {
          const bf16x8 h0 = hn_frag(32 * tb + rl, st);
          aa[tb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w_, h0, aa[tb], 0, 0, 0);
        }
      }
      // lane: token 32 tb + rl (column), channels 32 wq + 8 g + 4 hh + e of the chunk (rows)
      char* const dstc = isk ? Kc : Qc;
#pragma unroll
      for (int tb = 0; tb < 2; ++tb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int cq = 128 * ch + 32 * wq + 8 * g + 4 * hh, tk = 32 * tb + rl;
          const f32x4 bq = *(const f32x4*)(a.bqkv + isk * C + cq);
          *(uint2*)(dstc + rowc(tk, 4 * wq + g, 256) + 8 * hh) =
              uint2{pk_bf16(aa[tb][4 * g] + bq[0], aa[tb][4 * g + 1] + bq[1]), pk_bf16(aa[tb][4 * g + 2] + bq[2], aa[tb][4 * g + 3] + bq[3])};
        }
      // the next chunk's first PF fragments, in flight through this chunk's barriers and score MFMAs
      if (ch + 1 < NCH)
#pragma unroll
        for (int p = 0; p < PF; ++p) fa[p] = *frag(a.wqkv, cb + 4, p);
    }
    __syncthreads();
    if (w < 4) {
      const int key = 32 * (w >> 1) + rl, qry = 32 * (w & 1) + rl;
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        const bf16x8 kf = *(const bf16x8*)(Kc + rowc(key, 2 * st + hh, 256));
        const bf16x8 qf = *(const bf16x8*)(Qc + rowc(qry, 2 * st + hh, 256));
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf, sacc, 0, 0, 0);
      }
    }
    __syncthreads();  // Q_c / K_c are rewritten by the next chunk
  }
  ATL(3);  // scores done
  // phase 5's first PF weight fragments, in flight through the softmax and PV phases
  bf16x8 aw[PF][NBW];
#pragma unroll
  for (int p = 0; p < PF; ++p)
#pragma unroll
    for (int b = 0; b < NBW; ++b)
      if (w + 8 * b < CB) aw[p][b] = *frag(a.wp, w + 8 * b, p);
  // ---- 3. softmax over keys: S[query][key] fp32 through LDS, P [query][key] bf16
  float* const Sm = (float*)(sm + R_QK);              // [64][64 + 4]
  char* const Pm = sm + R_QK + S * (S + 4) * 4;       // [64][64] bf16, 128-B rows
  if (w < 4) {
    const int qry = 32 * (w & 1) + rl;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) Sm[qry * (S + 4) + 32 * (w >> 1) + 8 * g + 4 * hh + e] = sacc[4 * g + e] * a.scale;
  }
  __syncthreads();
  {
    const int qry = tid >> 3, k0 = (tid & 7) * 8;  // 8 lanes a query, 8 keys a lane
    float v[8], m = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = Sm[qry * (S + 4) + k0 + e];
      m = fmaxf(m, v[e]);
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = expf(v[e] - m);
      sum += v[e];
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) sum += __shfl_xor(sum, o, 64);
    const float inv = 1.0f / sum;
    *(u32x4*)(Pm + row64(qry, tid & 7)) =
        u32x4{pk_bf16(v[0] * inv, v[1] * inv), pk_bf16(v[2] * inv, v[3] * inv), pk_bf16(v[4] * inv, v[5] * inv),
              pk_bf16(v[6] * inv, v[7] * inv)};
  }
  __syncthreads();
  ATL(4);  // softmax done
  // ---- 4. O^T = V^T P^T: D[c][query], wave: channel blocks CBW wq .. x query block wt -> O [token][C]
  {
    f32x16 acc[CBW];
#pragma unroll
    for (int b = 0; b < CBW; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const bf16x8 p0 = *(const bf16x8*)(Pm + row64(tr, 2 * st + hh));
#pragma unroll
      for (int b = 0; b < CBW; ++b) {
        const int c = 32 * (CBW * wq + b) + rl;
        const bf16x8 vf = *(const bf16x8*)(sm + R_VT + row64(c, 2 * st + hh));
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, p0, acc[b], 0, 0, 0);
      }
    }
    // hn is dead since phase 2: O goes to its rows. lane: query tr, channels 32 cb + 8 g + 4 hh + e
#pragma unroll
    for (int b = 0; b < CBW; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *(uint2*)(sm + rowc(tr, 4 * (CBW * wq + b) + g, C * 2) + 8 * hh) =
            uint2{pk_bf16(acc[b][4 * g], acc[b][4 * g + 1]), pk_bf16(acc[b][4 * g + 2], acc[b][4 * g + 3])};
  }
  __syncthreads();
  ATL(5);  // PV done
  // ---- 5. out = x + O Wp^T + bp: D[c'][token], wave w: blocks w + 8 b x both token blocks
  float* const spart = (float*)(sm + R_ST);  // [token block][2][C]: the two token blocks' statistics
  {
    f32x16 acc[2][NBW];
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
      for (int b = 0; b < NBW; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[tb][b][r] = 0.f;
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      bf16x8 cur[NBW];
#pragma unroll
      for (int b = 0; b < NBW; ++b) cur[b] = aw[st % PF][b];
      if (st + PF < KS)
#pragma unroll
        for (int b = 0; b < NBW; ++b)
          if (w + 8 * b < CB) aw[st % PF][b] = *frag(a.wp, w + 8 * b, st + PF);
#pragma unroll
      for (int tb = 0; tb < 2; ++tb) {
        const bf16x8 o0 = hn_frag(32 * tb + rl, st);
#pragma unroll
        for (int b = 0; b < NBW; ++b)
          if (w + 8 * b < CB) acc[tb][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[b], o0, acc[tb][b], 0, 0, 0);
      }
    }
    bf16_t* out = a.out + (size_t)img * S * C;
#pragma unroll
    for (int tb = 0; tb < 2; ++tb) {
      const int tk = 32 * tb + rl;  // this lane's token
#pragma unroll
      for (int b = 0; b < NBW; ++b) {
        if (w + 8 * b >= CB) continue;
        const int cb = w + 8 * b;
        float v[32];
        uint32_t wv[4][2];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = 32 * cb + 8 * g + 4 * hh;
          const f32x4 bb = *(const f32x4*)(a.bp + c);
          const uint2 rr = *(const uint2*)(x + (size_t)tk * C + c);
          const float v0 = acc[tb][b][4 * g + 0] + bb[0] + __uint_as_float(rr.x << 16);
          const float v1 = acc[tb][b][4 * g + 1] + bb[1] + __uint_as_float(rr.x & 0xffff0000u);
          const float v2 = acc[tb][b][4 * g + 2] + bb[2] + __uint_as_float(rr.y << 16);
          const float v3 = acc[tb][b][4 * g + 3] + bb[3] + __uint_as_float(rr.y & 0xffff0000u);
          wv[g][0] = pk_bf16(v0, v1);
          wv[g][1] = pk_bf16(v2, v3);
          const float r0 = __uint_as_float(wv[g][0] << 16), r1 = __uint_as_float(wv[g][0] & 0xffff0000u);
          const float r2 = __uint_as_float(wv[g][1] << 16), r3 = __uint_as_float(wv[g][1] & 0xffff0000u);
          v[4 * g + 0] = r0; v[16 + 4 * g + 0] = r0 * r0;
          v[4 * g + 1] = r1; v[16 + 4 * g + 1] = r1 * r1;
          v[4 * g + 2] = r2; v[16 + 4 * g + 2] = r2 * r2;
          v[4 * g + 3] = r3; v[16 + 4 * g + 3] = r3 * r3;
        }
#pragma unroll
        for (int gp = 0; gp < 4; gp += 2) {
          u32x4 o;
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const auto sw = __builtin_amdgcn_permlane32_swap(wv[gp][d], wv[gp + 1][d], false, false);
            o[d] = sw[0];
            o[2 + d] = sw[1];
          }
          *(u32x4*)(out + (size_t)tk * C + 32 * cb + 8 * (gp + hh)) = o;
        }
        if (a.out_stats) {  // this token block's 32 lanes: butterfly, then the two blocks summed in order
          auto xchg = [](float xf, auto wc) {
            constexpr int wd = decltype(wc)::value;
            const int xi = __builtin_bit_cast(int, xf);
            int r;
            if constexpr (wd == 1) r = __builtin_amdgcn_update_dpp(0, xi, 0xB1, 0xF, 0xF, false);
            else if constexpr (wd == 2) r = __builtin_amdgcn_update_dpp(0, xi, 0x4E, 0xF, 0xF, false);
            else if constexpr (wd == 8) r = __builtin_amdgcn_update_dpp(0, xi, 0x128, 0xF, 0xF, false);
            else r = __builtin_amdgcn_ds_swizzle(xi, 0x1F | (wd << 10));
            return __builtin_bit_cast(float, r);
          };
          auto halve = [&](auto wc) {
            constexpr int wd = decltype(wc)::value;
            const bool up = (rl & wd) != 0;
#pragma unroll
            for (int ii = 0; ii < wd; ++ii) {
              const float lo = v[ii], hi = v[ii + wd];
              v[ii] = (up ? hi : lo) + xchg(up ? lo : hi, wc);
            }
          };
          halve(std::integral_constant<int, 16>{});
          halve(std::integral_constant<int, 8>{});
          halve(std::integral_constant<int, 4>{});
          halve(std::integral_constant<int, 2>{});
          halve(std::integral_constant<int, 1>{});
          const int e = rl & 15, co = 32 * cb + 8 * (e >> 2) + 4 * hh + (e & 3);
          spart[(tb * 2 + (rl >> 4)) * C + co] = v[0];
        }
      }
    }
  }
  ATL(6);  // proj + epilogue (wave's own)
  if (a.out_stats) {
    __syncthreads();
    for (int i = tid; i < 2 * C; i += 512)  // (sum | sum of squares) x channel: token block 0 + block 1
      a.out_stats[(long long)img * 2 * C + i] = spart[i] + spart[2 * C + i];
  }
  ATL(7);
}

// ---------------------------------------------------------------------------- fused AttnBlock over G blocks
// attn_block_split_kernel<C, G>: attn_block_kernel's image spread over G blocks for small batches (the
// 8-GPU shard runs N = 32: one block per image left 224 of 256 CUs idle while every block streamed all
// 1.2 MB of the block's weights). Block (img, g) owns channel blocks [g CBg, (g+1) CBg),
// CBg = C / 32 / G, and streams only those weight rows:
//   0. GroupNorm + hn as attn_block_kernel (every block: hn is the K operand of every projection);
//   1. its V^T, Q, K channel slices (hn W^T + b) -> LDS;
//   2. its partial scores S_g^T = K_g Q_g^T (keys x queries, fp32) -> write-through slab, counter;
//      every block waits for the image's G partials, sums them in g order 0..G-1 (the same bits in every
//      block, whichever arrives last) -> softmax -> P (bf16), as attn_block_kernel;
//   3. O^T of its channels = V_g^T P^T -> write-through slab [img][token][C], counter; waits for all G;
//   4. out = x + O Wp^T + bp for its output channels (full O from the slab), its channels' GroupNorm
//      statistics (per channel: no cross-block sum).
// Roundings as attn_block_kernel (hn, q / k / v, P, O in bf16); only S is summed in another order (G
// partial sums), so it agrees with attn_block_kernel within bf16 tolerance, not bit for bit.
// Hand-offs: MI355X_MICROARCH.md visibility table, row 1 (sc1 stores; every storing wave waits
// vmcnt(0); a workgroup barrier; one agent-scope atomic add per block; one lane polls with sc1 loads
// (s_sleep, bounded); a workgroup barrier; every load of the handed-off bytes an sc1 load). The counters
// only grow, by 12 per launch (12 / G per block), so a block's target -- the next multiple of 12 above the
// value its own add returned -- holds whatever G earlier launches used (launches on a stream never overlap). Waiting blocks need the whole grid resident: the host launches it only when
// n * G <= CUs (one 512-thread block per CU).
#ifndef ITSD_ATTN_SPLIT_PF
#define ITSD_ATTN_SPLIT_PF 8
#endif
template <int C, int G>
__global__ __launch_bounds__(512, 1) void attn_block_split_kernel(AttnBlockArgs a) {
  constexpr int S = 64, KS = C / 16, CB = C / 32, CBg = CB / G, CW = CBg * 32, PF = ITSD_ATTN_SPLIT_PF;
  static_assert(CB % G == 0 && C % 128 == 0 && 12 % G == 0, "G divides the channel blocks and 12");
  constexpr int QROW = CW * 2 + 16;  // Q_g / K_g row (bytes): padded so 16-B reads of 16 rows are conflict-free
  constexpr int R_VT = S * C * 2, R_Q = R_VT + CW * 128, R_K = R_Q + S * QROW, R_SM = R_K + S * QROW;
  constexpr int R_PM = R_SM + S * (S + 4) * 4, R_GS = R_PM + S * 128, R_ST = R_GS + 32 * 2 * 4;
  __shared__ __attribute__((aligned(16))) char sm[R_ST + 2 * 2 * CW * 4];
  const int tid = threadIdx.x, lane = tid & 63, rl = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int img = blockIdx.x / G, g = blockIdx.x - (blockIdx.x / G) * G;
  const bf16_t* x = a.x + (size_t)img * S * C;
  auto rowc = [](int r, int ch, int rowbytes) { return r * rowbytes + ((ch ^ (r & 15)) << 4); };
  auto row64 = [](int r, int ch) { return r * 128 + ((ch ^ ((r >> 1) & 7)) << 4); };
  auto frag = [&](const bf16_t* W, int cb, int st) -> const bf16x8* {
    return (const bf16x8*)((const char*)W + ((size_t)cb * KS + st) * 1024 + lane * 16);
  };
  // projection unit u = kind * CBg + cbl (kind 0 V, 1 Q, 2 K): its fragment row of the packed q|k|v matrix
  auto frow_of = [&](int u) {
    const int kind = u / CBg, cb = g * CBg + u - kind * CBg;
    return kind == 0 ? 2 * CB + cb : (kind - 1) * CB + cb;
  };
  // the first PF weight fragments of this wave's first unit, in flight before anything else (they depend
  // on no earlier kernel: their latency hides behind the x loads and the GroupNorm)
  bf16x8 fw[PF];
  if (w < 3 * CBg) {
#pragma unroll
    for (int p = 0; p < PF; ++p) fw[p] = *frag(a.wqkv, frow_of(w), p);
  }
  // ---- 0. GroupNorm statistics and hn (attn_block_kernel's phase 0)
  constexpr int XU = S * (C / 8) / 512;
  u32x4 xv[XU];
#pragma unroll
  for (int i = 0; i < XU; ++i) {
    const int u = tid + 512 * i, t = u / (C / 8), ch = u - t * (C / 8);
    xv[i] = *(const u32x4*)(x + (size_t)t * C + ch * 8);
  }
  float* gs = (float*)(sm + R_GS);
  if (tid < 256) {
    const int gr = tid >> 3, l8 = tid & 7, gsz = C / 32, n_it = gsz * a.spi;
    double s = 0.0, q = 0.0;
    for (int k = l8; k < n_it; k += 8) {
      const int c = gr * gsz + k / a.spi;
      const long long sl = (long long)img * a.spi + k % a.spi;
      s += (double)a.st[(sl * 2) * C + c];
      q += (double)a.st[(sl * 2 + 1) * C + c];
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      s += __shfl_xor(s, o, 64);
      q += __shfl_xor(q, o, 64);
    }
    if (l8 == 0) {
      const double E = (double)gsz * S, mean = s / E;
      double var = q / E - mean * mean;
      var = var > 0.0 ? var : 0.0;
      gs[2 * gr] = (float)mean;
      gs[2 * gr + 1] = (float)(1.0 / sqrt(var + 1e-5));
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < XU; ++i) {
    const int u = tid + 512 * i, t = u / (C / 8), ch = u - t * (C / 8), c0 = ch * 8;
    uint32_t o[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      float y[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int c = c0 + 2 * e2 + h2, gg = c / (C / 32);
        const float mean = gs[2 * gg], rstd = gs[2 * gg + 1];
        const float sc = rstd * a.gamma[c];
        const float xf = __uint_as_float(h2 ? (xv[i][e2] & 0xffff0000u) : (xv[i][e2] << 16));
        y[h2] = xf * sc + (a.beta[c] - mean * sc);
      }
      o[e2] = pk_bf16(y[0], y[1]);
    }
    *(u32x4*)(sm + rowc(t, ch, C * 2)) = u32x4{o[0], o[1], o[2], o[3]};
  }
  __syncthreads();
  auto hn_frag = [&](int r, int st) { return *(const bf16x8*)(sm + rowc(r, 2 * st + hh, C * 2)); };
  // weight-stream unit: one 32-channel block of a projection over both token blocks (fragments loaded once);
  // fw holds the unit's first PF fragments when it is called
  auto unit = [&](const bf16_t* W, int frow, f32x16 (&acc)[2], auto vform) __attribute__((always_inline)) {
    constexpr bool VF = decltype(vform)::value;  // true: D[token][c] (A = hn); false: D[c][token] (A = W)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tb][r] = 0.f;
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const bf16x8 cur = fw[st % PF];
      if (st + PF < KS) fw[st % PF] = *frag(W, frow, st + PF);
#pragma unroll
      for (int tb = 0; tb < 2; ++tb) {
        const bf16x8 h0 = hn_frag(32 * tb + rl, st);
        if constexpr (VF) acc[tb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(h0, cur, acc[tb], 0, 0, 0);
        else acc[tb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, h0, acc[tb], 0, 0, 0);
      }
    }
  };
  // ---- 1. this block's V^T, Q, K slices: units u = kind * CBg + cbl (kind 0 V, 1 Q, 2 K)
  for (int u = w; u < 3 * CBg; u += 8) {
    const int kind = u / CBg, cbl = u - kind * CBg, cb = g * CBg + cbl;
    f32x16 acc[2];
    if (u != w) {  // a wave's later units (G <= 4): their first fragments now
#pragma unroll
      for (int p = 0; p < PF; ++p) fw[p] = *frag(a.wqkv, frow_of(u), p);
    }
    if (kind == 0) {
      unit(a.wqkv, 2 * CB + cb, acc, std::true_type{});
      // lane: channel 32 cb + rl, tokens 32 tb + 8 q + 4 hh + e -> V^T row (local channel), 4 tokens a store
      const float bv = a.bqkv[2 * C + 32 * cb + rl];
#pragma unroll
      for (int tb = 0; tb < 2; ++tb)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *(uint2*)(sm + R_VT + row64(32 * cbl + rl, 4 * tb + q) + 8 * hh) =
              uint2{pk_bf16(acc[tb][4 * q] + bv, acc[tb][4 * q + 1] + bv), pk_bf16(acc[tb][4 * q + 2] + bv, acc[tb][4 * q + 3] + bv)};
    } else {
      unit(a.wqkv, (kind - 1) * CB + cb, acc, std::false_type{});
      // lane: token 32 tb + rl, channels 32 cb + 8 q + 4 hh + e -> Q_g / K_g [token][local channel]
      char* dst = sm + (kind == 1 ? R_Q : R_K);
#pragma unroll
      for (int tb = 0; tb < 2; ++tb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cl = 32 * cbl + 8 * q + 4 * hh;
          const f32x4 bq = *(const f32x4*)(a.bqkv + (kind - 1) * C + g * CW + cl);
          *(uint2*)(dst + (32 * tb + rl) * QROW + cl * 2) =
              uint2{pk_bf16(acc[tb][4 * q] + bq[0], acc[tb][4 * q + 1] + bq[1]), pk_bf16(acc[tb][4 * q + 2] + bq[2], acc[tb][4 * q + 3] + bq[3])};
        }
    }
  }
  __syncthreads();
  // ---- 2. partial scores S_g^T[key][query] over this block's channels (waves 0..3: tile w), write-through
  const uint32_t sp_bytes = (uint32_t)std::min<long long>((long long)a.n * G * 4 * 1024 * 4, 0x7fffffffLL);
  const __amdgpu_buffer_rsrc_t sp = __builtin_amdgcn_make_buffer_rsrc(a.spart, (short)0, (int)sp_bytes, 0x00020000);
  if (w < 4) {
    const int key = 32 * (w >> 1) + rl, qry = 32 * (w & 1) + rl;
    f32x16 sacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
#pragma unroll
    for (int st = 0; st < CW / 16; ++st) {
      const bf16x8 kf = *(const bf16x8*)(sm + R_K + key * QROW + (2 * st + hh) * 16);
      const bf16x8 qf = *(const bf16x8*)(sm + R_Q + qry * QROW + (2 * st + hh) * 16);
      sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf, sacc, 0, 0, 0);
    }
    const uint32_t off = (uint32_t)((((size_t)img * G + g) * 4 + w) * 1024 + lane * 16) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(sacc[4 * q]), __float_as_uint(sacc[4 * q + 1]),
                                                   __float_as_uint(sacc[4 * q + 2]), __float_as_uint(sacc[4 * q + 3])},
                                             sp, off + q * 16, 0, 16);
  }
  // hand-off: this block's stores drained, one add, one lane polls until the image's G blocks have added
  // Every launch adds exactly 12 to each counter (12 / G per block; G in {2, 4, 6}), so between launches a
  // counter is a multiple of 12 whatever G earlier launches used, and a block's target is the next one.
  // `during` runs between the barriers while lane 0 of wave 0 polls (work that needs no handed-off byte)
  // Fail loudly: a wait that exhausts its poll bound (a grid that is not co-resident -- another process on
  // the GPU, a CU mask) would read partial slabs; the block then keeps the counter protocol (every block
  // still adds, so later launches' targets hold), sets bit 0 of the status word *a.err (the sampler / forward
  // report ITSD_ERR_HANDOFF) and writes NaN to its output channels (the NaN check of Diffusion.py:100 fires too)
  __shared__ int hbad;
  if (tid == 0) hbad = 0;
  auto handoff = [&](int* cnt, auto during) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    during();
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(cnt, 12 / G, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int target = (old / 12 + 1) * 12;
      int v = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int it = 0; v < target && it < a.spin_bound; ++it) {  // bounded: a grid that is not co-resident cannot hang the GPU
        __builtin_amdgcn_s_sleep(2);
        v = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (v < target) {
        hbad = 1;
        __hip_atomic_fetch_or(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
  };
  handoff(a.sync + 2 * img, [] {});
  // every block: S = sum of the G partials in g order (waves 0..3, their tile), scaled -> Sm [query][key]
  float* const Sm = (float*)(sm + R_SM);
  char* const Pm = sm + R_PM;
  if (w < 4) {
    f32x16 sacc;
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      const uint32_t off = (uint32_t)((((size_t)img * G + gg) * 4 + w) * 1024 + lane * 16) * 4;
      u32x4 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = __builtin_amdgcn_raw_buffer_load_b128(sp, off + q * 16, 0, 16);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          sacc[4 * q + e] = gg == 0 ? __uint_as_float(v[q][e]) : sacc[4 * q + e] + __uint_as_float(v[q][e]);
    }
    const int qry = 32 * (w & 1) + rl;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) Sm[qry * (S + 4) + 32 * (w >> 1) + 8 * q + 4 * hh + e] = sacc[4 * q + e] * a.scale;
  }
  __syncthreads();
  {  // ---- softmax over keys (attn_block_kernel's phase 3): 8 lanes a query, 8 keys a lane
    const int qry = tid >> 3, k0 = (tid & 7) * 8;
    float v[8], m = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = Sm[qry * (S + 4) + k0 + e];
      m = fmaxf(m, v[e]);
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = expf(v[e] - m);
      sum += v[e];
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) sum += __shfl_xor(sum, o, 64);
    const float inv = 1.0f / sum;
    *(u32x4*)(Pm + row64(qry, tid & 7)) =
        u32x4{pk_bf16(v[0] * inv, v[1] * inv), pk_bf16(v[2] * inv, v[3] * inv), pk_bf16(v[4] * inv, v[5] * inv),
              pk_bf16(v[6] * inv, v[7] * inv)};
  }
  __syncthreads();
  // ---- 3. O^T of this block's channels = V_g^T P^T: tiles (local channel block, query block) -> O slab
  const uint32_t o_bytes = (uint32_t)std::min<long long>((long long)a.n * S * C * 2, 0x7fffffffLL);
  const __amdgpu_buffer_rsrc_t osl = __builtin_amdgcn_make_buffer_rsrc(a.oslab, (short)0, (int)o_bytes, 0x00020000);
  for (int tile = w; tile < 2 * CBg; tile += 8) {
    const int cbl = tile >> 1, q = 32 * (tile & 1) + rl;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const bf16x8 p0 = *(const bf16x8*)(Pm + row64(q, 2 * st + hh));
      const bf16x8 vf = *(const bf16x8*)(sm + R_VT + row64(32 * cbl + rl, 2 * st + hh));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, p0, acc, 0, 0, 0);
    }
    // lane: query q, channels g CW + 32 cbl + 8 r4 + 4 hh + e (4 consecutive: one 8-B store)
    typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
      const int c = g * CW + 32 * cbl + 8 * r4 + 4 * hh;
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{pk_bf16(acc[4 * r4], acc[4 * r4 + 1]), pk_bf16(acc[4 * r4 + 2], acc[4 * r4 + 3])},
                                            osl, (uint32_t)((((size_t)img * S + q) * C + c) * 2), 0, 16);
    }
  }
  // (the proj unit's first fragments go out while the block waits for the other slices)
  handoff(a.sync + 2 * img + 1, [&] {
    if (w < CBg) {
#pragma unroll
      for (int p = 0; p < PF; ++p) fw[p] = *frag(a.wp, g * CBg + w, p);
    }
  });
  // the full O [token][C] (every block's slice) -> hn's rows (hn is dead since phase 1)
  for (int i = tid; i < S * (C / 8); i += 512) {
    const int t = i / (C / 8), ch = i - t * (C / 8);
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(osl, (uint32_t)((((size_t)img * S + t) * C + ch * 8) * 2), 0, 16);
    *(u32x4*)(sm + rowc(t, ch, C * 2)) = v;
  }
  __syncthreads();
  // ---- 4. out = x + O Wp^T + bp for this block's output channels; statistics of its channels
  float* const spart = (float*)(sm + R_ST);  // [token block][2][CW]
  bf16_t* out = a.out + (size_t)img * S * C;
  const bool hb = hbad != 0;  // (a failed hand-off, see handoff: NaN outputs)
  for (int cbl = w; cbl < CBg; cbl += 8) {  // (CBg <= 6: one unit a wave, its fragments loaded above)
    const int cb = g * CBg + cbl;
    f32x16 acc[2];
    unit(a.wp, cb, acc, std::false_type{});  // D[c'][token]
#pragma unroll
    for (int tb = 0; tb < 2; ++tb) {
      const int tk = 32 * tb + rl;
      float v[32];
      uint32_t wv[4][2];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 32 * cb + 8 * q + 4 * hh;
        const f32x4 bb = *(const f32x4*)(a.bp + c);
        const uint2 rr = *(const uint2*)(x + (size_t)tk * C + c);
        const float nan = __builtin_nanf("");  // (a failed hand-off: every output channel NaN)
        const float v0 = hb ? nan : acc[tb][4 * q + 0] + bb[0] + __uint_as_float(rr.x << 16);
        const float v1 = hb ? nan : acc[tb][4 * q + 1] + bb[1] + __uint_as_float(rr.x & 0xffff0000u);
        const float v2 = hb ? nan : acc[tb][4 * q + 2] + bb[2] + __uint_as_float(rr.y << 16);
        const float v3 = hb ? nan : acc[tb][4 * q + 3] + bb[3] + __uint_as_float(rr.y & 0xffff0000u);
        wv[q][0] = pk_bf16(v0, v1);
        wv[q][1] = pk_bf16(v2, v3);
        const float r0 = __uint_as_float(wv[q][0] << 16), r1 = __uint_as_float(wv[q][0] & 0xffff0000u);
        const float r2 = __uint_as_float(wv[q][1] << 16), r3 = __uint_as_float(wv[q][1] & 0xffff0000u);
        v[4 * q + 0] = r0; v[16 + 4 * q + 0] = r0 * r0;
        v[4 * q + 1] = r1; v[16 + 4 * q + 1] = r1 * r1;
        v[4 * q + 2] = r2; v[16 + 4 * q + 2] = r2 * r2;
        v[4 * q + 3] = r3; v[16 + 4 * q + 3] = r3 * r3;
      }
#pragma unroll
      for (int gp = 0; gp < 4; gp += 2) {
        u32x4 o;
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto swp = __builtin_amdgcn_permlane32_swap(wv[gp][d], wv[gp + 1][d], false, false);
          o[d] = swp[0];
          o[2 + d] = swp[1];
        }
        *(u32x4*)(out + (size_t)tk * C + 32 * cb + 8 * (gp + hh)) = o;
      }
      if (a.out_stats) {
        auto xchg = [](float xf, auto wc) {
          constexpr int wd = decltype(wc)::value;
          const int xi = __builtin_bit_cast(int, xf);
          int r;
          if constexpr (wd == 1) r = __builtin_amdgcn_update_dpp(0, xi, 0xB1, 0xF, 0xF, false);
          else if constexpr (wd == 2) r = __builtin_amdgcn_update_dpp(0, xi, 0x4E, 0xF, 0xF, false);
          else if constexpr (wd == 8) r = __builtin_amdgcn_update_dpp(0, xi, 0x128, 0xF, 0xF, false);
          else r = __builtin_amdgcn_ds_swizzle(xi, 0x1F | (wd << 10));
          return __builtin_bit_cast(float, r);
        };
        auto halve = [&](auto wc) {
          constexpr int wd = decltype(wc)::value;
          const bool up = (rl & wd) != 0;
#pragma unroll
          for (int ii = 0; ii < wd; ++ii) {
            const float lo = v[ii], hi = v[ii + wd];
            v[ii] = (up ? hi : lo) + xchg(up ? lo : hi, wc);
          }
        };
        halve(std::integral_constant<int, 16>{});
        halve(std::integral_constant<int, 8>{});
        halve(std::integral_constant<int, 4>{});
        halve(std::integral_constant<int, 2>{});
        halve(std::integral_constant<int, 1>{});
        const int e = rl & 15, col = 32 * cbl + 8 * (e >> 2) + 4 * hh + (e & 3);
        spart[(tb * 2 + (rl >> 4)) * CW + col] = v[0];
      }
    }
  }
  if (a.out_stats) {
    __syncthreads();
    for (int i = tid; i < 2 * CW; i += 512) {  // (sum | sum of squares) x local channel: token block 0 + block 1
      const int half = i / CW, cl = i - half * CW;
      a.out_stats[(long long)img * 2 * C + half * C + g * CW + cl] = spart[i] + spart[2 * CW + i];
    }
  }
}

#ifdef ITSD_STAMPS
extern "C" int itsd_debug_stamps_attn(unsigned long long* host) {
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(itsd::g_stamps_attn), sizeof(unsigned long long) * 1024 * 128) == hipSuccess ? 0 : 1;
}
#endif

int g_attn_wide_nq = 1;  // its query groups a block: 0 auto, 1 / 2 forced (2 measured equal at C3, slower at C4) (itsd_set_option "attn_wide_nq")
int g_attn_wide = 1;   // channel-split attention: 0 off, 1 auto (C >= 384, S >= 256), 2 wherever attn_cs_ok (itsd_set_option "attn_wide")
int g_spin_bound = 1 << 22;  // polls before an in-kernel hand-off wait fails (itsd_set_option "spin_bound", diagnostic)
int g_attn_split = 1;  // attn_block_split_kernel for small batches: 0 off, 1 auto, 2/4/6 forced G (itsd_set_option "attn_split")
// G blocks per image for attn_block_split_kernel at batch n (0: one block per image, attn_block_kernel):
// the largest of 6 / 4 / 2 that keeps the grid co-resident (n * G <= CUs, one block per CU)
int attn_split_g(int n, int C) {
  if (C != 384 || !g_attn_split) return 0;
  const int opts[3] = {6, 4, 2};
  for (int G : opts)
    // (co-resident grid: one 512-thread block a CU; the partial-score slab holds 4 MB = 256 x 16 KB)
    if ((g_attn_split == 1 || g_attn_split == G) && (long long)n * G <= g_num_cus && (long long)n * G * 16384 <= (4ll << 20))
      return G;
  return 0;
}

hipError_t launch_attn_block(const AttnBlockArgs& a, int C, hipStream_t s) {
  if (a.spart && a.oslab && a.sync && a.S == 64) {
    const int G = attn_split_g(a.n, C);
    if (G == 6) ITSD_LAUNCH((attn_block_split_kernel<384, 6>), dim3(a.n * 6), dim3(512), 0, s, a);
    else if (G == 4) ITSD_LAUNCH((attn_block_split_kernel<384, 4>), dim3(a.n * 4), dim3(512), 0, s, a);
    else if (G == 2) ITSD_LAUNCH((attn_block_split_kernel<384, 2>), dim3(a.n * 2), dim3(512), 0, s, a);
    if (G) return hipGetLastError();
  }
  if (a.S != 64) return hipErrorInvalidValue;
  if (C == 384) ITSD_LAUNCH((attn_block_kernel<384>), dim3(a.n), dim3(512), 0, s, a);
  else if (C == 256) ITSD_LAUNCH((attn_block_kernel<256>), dim3(a.n), dim3(512), 0, s, a);
  else if (C == 128) ITSD_LAUNCH((attn_block_kernel<128>), dim3(a.n), dim3(512), 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
// S = 64: one image a block (LDS: C <= 384). (The 4x4 middle block's 4-images-a-block form measured slower at N = 32
// and was removed in round 5: that AttnBlock runs the unfused GroupNorm / q|k|v / attention / proj launches.)
bool attn_block_ok(int S, int C) {
  return S == 64 && (C == 128 || C == 256 || C == 384);
}

// Flash-style MFMA attention for long sequences (S > 256: the CFG UNet's 32x32 level,
// S = 1024, C = 128, ModelCondition.py:98-118; Arch A at 64/256 px). No S x S tile is
// materialised: each wave owns 32 queries, and the block's 4 waves (128 queries) stream
// 32-key tiles of K and V^T through LDS with an online softmax.
//  - K / V^T tiles are double-buffered in LDS with one barrier a tile (the next tile's global
//    loads are in flight while the current one is consumed): each K / V byte is fetched from
//    L2 once per block, not once per wave (the per-wave form was bound by those loads);
//  - blocks run XCD-major (block b on XCD b % 8 takes logical tile (b % 8) * nb/8 + b / 8), so the
//    query tiles of one image share one XCD's L2 for that image's K / V;
//  - scores are computed transposed, s^T = K q^T (A = 32 keys x 16 ch, B = q^T), so every lane
//    holds 16 keys of ONE query: the row max / row sum is a register reduction plus one xor-32
//    shuffle, and the rescale of O is one factor/lane;
//  - O^T = V^T P^T with P^T straight from the score registers (bf16): the MFMA B operand of lane
//    (query, hi) is its 8 score registers r = 8j..8j+7, i.e. keys {16j+4hi+0..3, 16j+8+4hi+0..3};
//    V^T rows sit in LDS with each 16-key group stored in the order 0-3, 8-11, 4-7, 12-15, so the
//    A operand of lane (channel, hi) is ONE 16-byte LDS read at position 16j + 8hi.
// CB = C / 32 channel blocks (C <= 256: q fragment and O accumulators stay in registers).
template <int CB>
__global__ __launch_bounds__(256) void attn_flash_kernel(AttnArgs a) {
  constexpr int C = CB * 32, C3 = 3 * C, QS = C / 16, KP = C + 8, VP = 40, NSEG = CB / 2;
  static_assert(CB % 2 == 0, "two 16-byte segments of K and of V^T per thread per 64 channels");
  __shared__ __attribute__((aligned(16))) bf16_t Ks[2][32 * KP];  // [key][channel] (+8 pad)
  __shared__ __attribute__((aligned(16))) bf16_t Vs[2][C * VP];   // [channel][permuted key] (+8 pad)
  const int S = a.S, QT = (S + 127) / 128;
  const int nb = gridDim.x, bx = blockIdx.x;
  const int L = (nb & 7) ? bx : (bx & 7) * (nb >> 3) + (bx >> 3);
  const int img = L / QT, qt = L - img * QT;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, rl = lane & 31, hh = lane >> 5;
  const int q = qt * 128 + wid * 32 + rl;
  const bool qv = q < S;
  const bf16_t* base = (const bf16_t*)a.qkv + (size_t)img * S * C3;
  const bf16_t* vt = (const bf16_t*)a.vt + (size_t)img * C * S;
  bf16x8 qf[QS];  // (a query past S reads row 0; its output is not stored)
  {
    const bf16_t* qp = base + (size_t)(qv ? q : 0) * C3 + 8 * hh;
#pragma unroll
    for (int i = 0; i < QS; ++i) qf[i] = *(const bf16x8*)(qp + 16 * i);
  }
  f32x16 o[CB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[cb][r] = 0.f;
  const float sl2 = a.scale * 1.4426950408889634f;  // softmax via exp2
  float m = -INFINITY, l = 0.f;
  // staging: thread tid moves 16-byte segments g = tid + 256 r of the K tile (key g / (C/8),
  // channels 8 (g % (C/8)) ..) and of the V^T tile (channel g / 4, keys 8 (g % 4) ..); S % 8 == 0
  // (S % 32 == 0, attn_flash_ok: every key of every tile exists, no masks)
  u32x4 kr[NSEG], vr[NSEG];
#define ITSD_FLASH_GLOAD(kt)                                                                 \
  _Pragma("unroll") for (int r = 0; r < NSEG; ++r) {                                         \
    const int g = tid + 256 * r;                                                             \
    kr[r] = *(const u32x4*)(base + (size_t)((kt) + g / (C / 8)) * C3 + C + 8 * (g % (C / 8))); \
    vr[r] = *(const u32x4*)(vt + (size_t)(g >> 2) * S + (kt) + 8 * (g & 3));                 \
  }
#define ITSD_FLASH_LSTORE(buf)                                                               \
  _Pragma("unroll") for (int r = 0; r < NSEG; ++r) {                                         \
    const int g = tid + 256 * r, sg = g & 3;                                                 \
    *(u32x4*)&Ks[buf][(g / (C / 8)) * KP + 8 * (g % (C / 8))] = kr[r];                       \
    bf16_t* vp = &Vs[buf][(g >> 2) * VP + 16 * (sg >> 1) + 4 * (sg & 1)];                    \
    *(uint2*)vp = make_uint2(vr[r][0], vr[r][1]);       /* keys 8sg+0..3 */                    \
    *(uint2*)(vp + 8) = make_uint2(vr[r][2], vr[r][3]); /* keys 8sg+4..7 */                    \
  }
  ITSD_FLASH_GLOAD(0)
  ITSD_FLASH_LSTORE(0)
  __syncthreads();
  const int nt = (S + 31) / 32;
  for (int t = 0; t < nt; ++t) {
    const int kt = t * 32, buf = t & 1;
    if (t + 1 < nt) { ITSD_FLASH_GLOAD(kt + 32) }
    const bf16_t* ks = Ks[buf] + rl * KP + 8 * hh;
    f32x16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
    for (int i = 0; i < QS; ++i)
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(ks + 16 * i), qf[i], s, 0, 0, 0);
    // s[r] = score(query rl, key kt + (r&3) + 8(r>>2) + 4hh) (unscaled)
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] *= sl2;
      mx = fmaxf(mx, s[r]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    // lazy rescale: the running max moves (and O, l are rescaled) only when some query of the wave
    // gains more than 8 (log2 units) on it; otherwise P = 2^(s - m) <= 256 against the stale max,
    // the same quotient O / l (wave-uniform branch; the first tile always takes it, m = -inf)
    if (__ballot(mx > m + 8.0f) != 0ull) {
      const float mn = fmaxf(m, mx);
      const float alpha = exp2f(m - mn);
      l *= alpha;
      m = mn;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[cb][r] *= alpha;
    }
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = exp2f(s[r] - m);
      rs += s[r];
    }
    rs += __shfl_xor(rs, 32, 64);
    l += rs;
    const bf16_t* vs = Vs[buf] + rl * VP + 8 * hh;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bf16x8 bp;
#pragma unroll
      for (int i = 0; i < 8; ++i) bp[i] = (short)f2bf(s[8 * j + i]);
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
        o[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(vs + cb * 32 * VP + 16 * j), bp, o[cb], 0,
                                                        0, 0);
    }
    if (t + 1 < nt) { ITSD_FLASH_LSTORE(buf ^ 1) }  // (buf ^ 1 was last read in tile t - 1, before the barrier)
    __syncthreads();
  }
  if (!qv) return;
  const float inv = 1.0f / l;
  bf16_t* out = (bf16_t*)a.out + ((size_t)img * S + q) * C;
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = cb * 32 + 8 * g + 4 * hh;
      uint2 w2;
      w2.x = (uint32_t)f2bf(o[cb][4 * g] * inv) | ((uint32_t)f2bf(o[cb][4 * g + 1] * inv) << 16);
      w2.y = (uint32_t)f2bf(o[cb][4 * g + 2] * inv) | ((uint32_t)f2bf(o[cb][4 * g + 3] * inv) << 16);
      *(uint2*)(out + c) = w2;
    }
#undef ITSD_FLASH_GLOAD
#undef ITSD_FLASH_LSTORE
}

// Channel-split attention for wide channels (C = 256 .. 1024, S % 64 == 0: Arch A's 16x16 level at
// 64 px (S = 256, C = 384), the CFG model's 16x16 level (S = 256, C = 512) and 8x8 level (S = 64,
// C = 1024, NW = 8 waves a query group)), where one wave cannot hold q and O for all C channels.
// A block takes 32 queries per group; wave w owns channels [w C/NW, (w+1) C/NW) for
// BOTH products, so every K / V byte is read once per block with no LDS staging:
//  - per 32-key tile each wave computes a partial s^T = K_w q_w^T over its channels (C/64 MFMAs,
//    K fragments prefetched a tile ahead), writes it to LDS, and after one barrier every wave sums
//    the NW partials in wave order (identical scores in all waves: deterministic), runs the online
//    softmax and O_w^T += V_w^T P^T on its own C/128 channel blocks (V^T fragments prefetched a tile
//    ahead, the flash kernel's key permutation);
//  - the partial-score buffer is double-buffered by tile parity: one barrier a tile.
template <int C, int NQ, int NW = 4>
__global__ __launch_bounds__(64 * NW * NQ) void attn_cs_kernel(AttnArgs a) {
  constexpr int CQ = C / NW, QS = CQ / 16, CB = CQ / 32, C3 = 3 * C;
  static_assert(CQ % 32 == 0, "whole 32-channel blocks a wave");
  // [tile parity][query group][wave of the group][r / 4][lane][r % 4]
  __shared__ __attribute__((aligned(16))) float Sp[2][NQ][NW][4][64][4];
  const int S = a.S, QT = S / (32 * NQ);
  const int nb = gridDim.x, bx = blockIdx.x;
  const int L = (nb & 7) ? bx : (bx & 7) * (nb >> 3) + (bx >> 3);  // XCD-major: an image's tiles on one XCD
  const int img = L / QT, qt = L - img * QT;
  const int tid = threadIdx.x, lane = tid & 63, wid = (tid >> 6) % NW, qg = (tid >> 6) / NW, rl = lane & 31, hh = lane >> 5;
  const int q = (qt * NQ + qg) * 32 + rl, ch0 = wid * CQ;
  const bf16_t* base = (const bf16_t*)a.qkv + (size_t)img * S * C3;
  const bf16_t* vt = (const bf16_t*)a.vt + (size_t)img * C * S;
  bf16x8 qf[QS], kf[QS];
  {
    const bf16_t* qp = base + (size_t)q * C3 + ch0 + 8 * hh;
#pragma unroll
    for (int i = 0; i < QS; ++i) qf[i] = *(const bf16x8*)(qp + 16 * i);
    const bf16_t* kp = base + (size_t)rl * C3 + C + ch0 + 8 * hh;
#pragma unroll
    for (int i = 0; i < QS; ++i) kf[i] = *(const bf16x8*)(kp + 16 * i);
  }
  // V^T fragments of tile kt: lane (channel rl of block cb, hi) keys {16j+4hi+0..3, 16j+8+4hi+0..3}
  u32x4 vf[CB][2];
  auto load_v = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const bf16_t* vp = vt + (size_t)(ch0 + cb * 32 + rl) * S + kt + 4 * hh;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint2 lo = *(const uint2*)(vp + 16 * j), hi = *(const uint2*)(vp + 16 * j + 8);
        vf[cb][j] = u32x4{lo.x, lo.y, hi.x, hi.y};
      }
    }
  };
  load_v(0);
  f32x16 o[CB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[cb][r] = 0.f;
  const float sl2 = a.scale * 1.4426950408889634f;  // softmax via exp2
  float m = -INFINITY, l = 0.f;
  const int nt = S / 32;
  for (int t = 0; t < nt; ++t) {
    const int kt = t * 32, par = t & 1;
    f32x16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
    for (int i = 0; i < QS; ++i) s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[i], qf[i], s, 0, 0, 0);
    if (t + 1 < nt) {  // next tile's K fragments (their latency behind the exchange, softmax and PV)
      const bf16_t* kp = base + (size_t)(kt + 32 + rl) * C3 + C + ch0 + 8 * hh;
#pragma unroll
      for (int i = 0; i < QS; ++i) kf[i] = *(const bf16x8*)(kp + 16 * i);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *(f32x4*)&Sp[par][qg][wid][g][lane][0] = f32x4{s[4 * g], s[4 * g + 1], s[4 * g + 2], s[4 * g + 3]};
    __syncthreads();  // (Sp[par] of tile t - 2 was read before this barrier's predecessor)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 v = *(const f32x4*)&Sp[par][qg][0][g][lane][0];
#pragma unroll
      for (int w = 1; w < NW; ++w) v += *(const f32x4*)&Sp[par][qg][w][g][lane][0];
#pragma unroll
      for (int e = 0; e < 4; ++e) s[4 * g + e] = v[e] * sl2;
    }
    // s[r] = scaled score(query rl, key kt + (r&3) + 8(r>>2) + 4hh)
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    // lazy rescale: the running max moves (and O, l are rescaled) only when some query of the wave
    // gains more than 8 (log2 units) on it; otherwise P = 2^(s - m) <= 256 against the stale max,
    // the same quotient O / l (wave-uniform branch; the first tile always takes it, m = -inf)
    if (__ballot(mx > m + 8.0f) != 0ull) {
      const float mn = fmaxf(m, mx);
      const float alpha = exp2f(m - mn);
      l *= alpha;
      m = mn;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[cb][r] *= alpha;
    }
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = exp2f(s[r] - m);
      rs += s[r];
    }
    rs += __shfl_xor(rs, 32, 64);
    l += rs;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bf16x8 bp;
#pragma unroll
      for (int i = 0; i < 8; ++i) bp[i] = (short)f2bf(s[8 * j + i]);
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
        o[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vf[cb][j]), bp, o[cb], 0, 0, 0);
    }
    if (t + 1 < nt) load_v(kt + 32);
  }
  const float inv = 1.0f / l;
  bf16_t* out = (bf16_t*)a.out + ((size_t)img * S + q) * C + ch0;
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = cb * 32 + 8 * g + 4 * hh;
      uint2 w2;
      w2.x = (uint32_t)f2bf(o[cb][4 * g] * inv) | ((uint32_t)f2bf(o[cb][4 * g + 1] * inv) << 16);
      w2.y = (uint32_t)f2bf(o[cb][4 * g + 2] * inv) | ((uint32_t)f2bf(o[cb][4 * g + 3] * inv) << 16);
      *(uint2*)(out + c) = w2;
    }
}
bool attn_cs_ok(int S, int C) { return S % 64 == 0 && (C == 256 || C == 384 || C == 512 || C == 1024); }

bool attn_flash_ok(int S, int C) { return S % 32 == 0 && (C == 64 || C == 128 || C == 256); }

size_t attn_mfma_smem(int S) {
  const int Sp = (S + 31) & ~31;
  return (size_t)64 * (Sp + 4) * 4 + (size_t)64 * (Sp * 2 + 16);
}

template <typename T>
hipError_t launch_attn(const AttnArgs& a, int n, hipStream_t s) {
  if constexpr (sizeof(T) == 2) {
    // channel-split attention: auto (g_attn_wide = 1) for C >= 384 at S >= 256; 2 = wherever it applies
    // (C = 1024, the CFG 8x8 level at S = 64: 8 waves of 128 channels a query group)
    if (a.vt && g_attn_wide && attn_cs_ok(a.S, a.C) && a.C == 1024) {
      ITSD_LAUNCH((attn_cs_kernel<1024, 1, 8>), dim3((unsigned)((a.S / 32) * n)), dim3(512), 0, s, a);
      return hipGetLastError();
    }
    if (a.vt && g_attn_wide && attn_cs_ok(a.S, a.C) && (g_attn_wide == 2 || (a.C >= 384 && a.S >= 256))) {
      // 64 queries (two groups of 4 waves) a block; 32 when the query tiles of 64 leave CUs idle
      if (g_attn_wide_nq == 2 || (g_attn_wide_nq == 0 && (long long)(a.S / 64) * n >= g_num_cus)) {
        const dim3 grid((unsigned)((a.S / 64) * n));
        if (a.C == 512) ITSD_LAUNCH((attn_cs_kernel<512, 2>), grid, dim3(512), 0, s, a);
        else if (a.C == 384) ITSD_LAUNCH((attn_cs_kernel<384, 2>), grid, dim3(512), 0, s, a);
        else ITSD_LAUNCH((attn_cs_kernel<256, 2>), grid, dim3(512), 0, s, a);
      } else {
        const dim3 grid((unsigned)((a.S / 32) * n));
        if (a.C == 512) ITSD_LAUNCH((attn_cs_kernel<512, 1>), grid, dim3(256), 0, s, a);
        else if (a.C == 384) ITSD_LAUNCH((attn_cs_kernel<384, 1>), grid, dim3(256), 0, s, a);
        else ITSD_LAUNCH((attn_cs_kernel<256, 1>), grid, dim3(256), 0, s, a);
      }
      return hipGetLastError();
    }
    if (a.vt && a.S > 256) {
      if (!attn_flash_ok(a.S, a.C)) return hipErrorInvalidValue;
      const dim3 grid((unsigned)(((a.S + 127) / 128) * n));
      if (a.C == 64) ITSD_LAUNCH(attn_flash_kernel<2>, grid, dim3(256), 0, s, a);
      else if (a.C == 128) ITSD_LAUNCH(attn_flash_kernel<4>, grid, dim3(256), 0, s, a);
      else ITSD_LAUNCH(attn_flash_kernel<8>, grid, dim3(256), 0, s, a);
      return hipGetLastError();
    }
    if (a.vt) {
      static bool attr = false;
      const size_t sm = attn_mfma_smem(a.S);
      if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)attn_mfma_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)attn_mfma_smem(256));
        if (e != hipSuccess) return e;
        e = hipFuncSetAttribute((const void*)attn_mfma_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)attn_mfma_smem(256));
        if (e != hipSuccess) return e;
        attr = true;
      }
      // output-channel slices (attn_cs): measured slower at every split (each slice repeats the
      // score phase, which dominates: 26 -> 38 / 66 us at S = 64 for 2 / 4 slices), so 1 by default
      const bool q32 = g_attn_aq == 32 || (g_attn_aq == 0 && (long long)n * ((a.S + 63) / 64) < 512);
      const int cs = g_attn_cs > 0 ? g_attn_cs : 1;
      if ((a.C / 32) % cs) return hipErrorInvalidValue;
      if (q32) ITSD_LAUNCH(attn_mfma_kernel<32>, dim3((a.S + 31) / 32, n, cs), dim3(256), sm, s, a);
      else ITSD_LAUNCH(attn_mfma_kernel<64>, dim3((a.S + 63) / 64, n, cs), dim3(256), sm, s, a);
      return hipGetLastError();
    }
  }
  const int qc = att_qc(a.S);
  dim3 grid((a.S + qc - 1) / qc, n);
  ITSD_LAUNCH(attn_kernel<T>, grid, dim3(256), qc * a.S * sizeof(float), s, a);
  return hipGetLastError();
}
template hipError_t launch_attn<float>(const AttnArgs&, int, hipStream_t);
template hipError_t launch_attn<bf16_t>(const AttnArgs&, int, hipStream_t);

// ============================================================================ head conv
// head = Conv2d(3, ch, 3, padding=1) (Model.py:219) from the NCHW fp32 sampler state
// to NHWC activations. A block covers one GroupNorm statistics slot (128 pixels);
// threads are (pixel lane, 16-B chunk of output channels), consecutive threads one
// pixel's channel row (coalesced stores), weights in LDS. The block also writes the
// slot's channel sums / sums of squares for the first ResBlock's GroupNorm.
template <typename T>
__global__ __launch_bounds__(256) void head_kernel(HeadArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) float hw[];  // [27][Cout] (k-major: 16-B reads) then bias [Cout]
  float* red = hw + 28 * a.Cout;                              // [256 / cq][Cout][2] statistics partials
  // fill in destination order: conflict-free LDS stores, gathered (L2-resident) reads
  for (int d = threadIdx.x; d < a.Cout * 27; d += 256) {
    const int k = d / a.Cout, co = d - k * a.Cout;
    hw[d] = a.w[co * 27 + k];
  }
  for (int i = threadIdx.x; i < a.Cout; i += 256) hw[a.Cout * 27 + i] = a.b[i];
  __syncthreads();
  // block = one statistics slot of G pixels; thread = (pixel lane, 16-B chunk of couts)
  const int HW = a.H * a.W, G = stat_slot_px(HW);
  const int cq = a.Cout / EPC, plan = 256 / cq;
  const int ch = threadIdx.x % cq, pl = threadIdx.x / cq, c0 = ch * EPC;
  const long long pbase = (long long)blockIdx.x * G;
  // the block's input window (3 channels, 1-pixel border) staged in LDS: whole rows
  // when W <= G, else a G-wide row segment (host: G % W == 0 or W % G == 0)
  const int img = (int)(pbase / HW), r0 = (int)(pbase - (long long)img * HW);
  const int y0 = r0 / a.W, x0 = r0 - y0 * a.W;
  const int TW = (a.W <= G ? a.W : G) + 2, TR = (a.W <= G ? G / a.W : 1) + 2;
  float* tin = red + (size_t)plan * a.Cout * 2;  // [3][TR][TW]
  {
    const float* xs = a.x + (size_t)(img % a.x_img_mod) * 3 * HW;
    for (int i = threadIdx.x; i < 3 * TR * TW; i += 256) {
      const int ci = i / (TR * TW), r = i - ci * TR * TW, ty = r / TW, tx = r - ty * TW;
      const int iy = y0 - 1 + ty, ix = x0 - 1 + tx;
      tin[i] = (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) ? xs[ci * HW + iy * a.W + ix] : 0.0f;
    }
  }
  __syncthreads();
  float ssum[EPC], ssq[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) ssum[e] = ssq[e] = 0.f;
  if (pl < plan) {
    for (int p = pl; p < G; p += plan) {
      const long long pix = pbase + p;
      const int ly = a.W <= G ? p / a.W : 0, lx = a.W <= G ? p - ly * a.W : p;
      float in[27];
#pragma unroll
      for (int ci = 0; ci < 3; ++ci)
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) in[ci * 9 + ky * 3 + kx] = tin[(ci * TR + ly + ky) * TW + lx + kx];
      float acc[EPC];
#pragma unroll
      for (int e = 0; e < EPC; ++e) acc[e] = 0.0f;
#pragma unroll
      for (int k = 0; k < 27; ++k) {
#pragma unroll
        for (int q = 0; q < EPC / 4; ++q) {
          const f32x4 w4 = *(const f32x4*)(hw + k * a.Cout + c0 + 4 * q);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[4 * q + e] = fmaf(w4[e], in[k], acc[4 * q + e]);
        }
      }
      u32x4 w;
      T* we = (T*)&w;
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        we[e] = Elem<T>::to(acc[e] + hw[a.Cout * 27 + c0 + e]);
        const float v = Elem<T>::tof(we[e]);  // statistics of the stored (rounded) tensor
        ssum[e] += v;
        ssq[e] += v * v;
      }
      *(u32x4*)((T*)a.out + (size_t)pix * a.Cout + c0) = w;
    }
  }
  if (!a.stats) return;
  // GroupNorm statistics slab of the head output: stats[slot][0|1][c] (fixed-order sums)
  if (pl < plan) {
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      red[(pl * a.Cout + c0 + e) * 2] = ssum[e];
      red[(pl * a.Cout + c0 + e) * 2 + 1] = ssq[e];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < a.Cout; c += 256) {
    float s = 0.f, q = 0.f;
    for (int l = 0; l < plan; ++l) {
      s += red[(l * a.Cout + c) * 2];
      q += red[(l * a.Cout + c) * 2 + 1];
    }
    a.stats[((size_t)blockIdx.x * 2) * a.Cout + c] = s;
    a.stats[((size_t)blockIdx.x * 2 + 1) * a.Cout + c] = q;
  }
}

template <typename T>
hipError_t launch_head(const HeadArgs& a, hipStream_t s) {
  constexpr int EPC = 16 / (int)sizeof(T);
  const int HW = a.H * a.W, G = stat_slot_px(HW), cq = a.Cout / EPC;
  if (a.Cout % EPC || cq > 256 || 256 % cq || HW % G || (G % a.W && a.W % G)) return hipErrorInvalidValue;
  const int TW = (a.W <= G ? a.W : G) + 2, TR = (a.W <= G ? G / a.W : 1) + 2;
  const size_t smem = ((size_t)a.Cout * 28 + (size_t)(256 / cq) * a.Cout * 2 + 3 * TR * TW) * sizeof(float);
  ITSD_LAUNCH(head_kernel<T>, dim3((unsigned)((long long)a.n * HW / G)), dim3(256), smem, s, a);
  return hipGetLastError();
}
template hipError_t launch_head<float>(const HeadArgs&, hipStream_t);
template hipError_t launch_head<bf16_t>(const HeadArgs&, hipStream_t);

// ============================================================================ Philox
// Philox4x32-10 (Salmon et al., SC'11); normal via Box-Muller on the first two words.
__device__ __forceinline__ float philox_normal(unsigned long long seed, unsigned step, unsigned long long idx) {
  uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32), c2 = step, c3 = 0x1d5a1u;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  const float u1 = ((float)(c0 >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
  const float u2 = (float)(c1 >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// ============================================================================ tail conv + sampler step
// tail = GN -> Swish -> Conv2d(C, 3, 3, padding=1) (Model.py:252-256, 282). The GN+Swish
// output g is produced by groupnorm_kernel; this kernel does the 3-output conv per
// pixel with the weights in LDS and then either writes eps (forward API) or applies
// the ancestral update of Diffusion.py:67-71,96-100 in place on x:
//   mean = coeff1[t]*x - coeff2[t]*eps ;  x = mean + sqrt(var[t]) * z  (z = 0 at t = 0)
// CFG: eps = (1+w) eps_c - w eps_u (DiffusionCondition.py:85) with the unconditional
// branch at image index img + n of g.
template <typename T>
__global__ __launch_bounds__(256) void tail_kernel(TailArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) float wl[];  // [9][C][3]
  const int C = a.C;
  for (int i = threadIdx.x; i < 27 * C; i += 256) {
    // reference layout w[co][ci][ky][kx] -> wl[(tap*C + ci)*3 + co]
    const int co = i / (C * 9);
    const int r = i - co * C * 9;
    const int ci = r / 9, tap = r - ci * 9;
    wl[(tap * C + ci) * 3 + co] = a.w[i];
  }
  __syncthreads();
  const int HW = a.H * a.W;
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  if (pix >= (long long)a.n * HW) return;
  const int img = (int)(pix / HW);
  const int rem = (int)(pix - (long long)img * HW);
  const int y = rem / a.W, x = rem - y * a.W;
  auto conv3 = [&](int im, float& e0, float& e1, float& e2) {
    const T* gb = (const T*)a.g + (size_t)im * HW * C;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = y + ky - 1;
      if (iy < 0 || iy >= a.H) continue;
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = x + kx - 1;
        if (ix < 0 || ix >= a.W) continue;
        const T* gp = gb + (size_t)(iy * a.W + ix) * C;
        const float* wp = wl + (ky * 3 + kx) * C * 3;
        for (int c = 0; c < C; c += EPC) {
          const u32x4 v = *(const u32x4*)(gp + c);
          const T* ve = (const T*)&v;
#pragma unroll
          for (int e = 0; e < EPC; ++e) {
            const float gv = Elem<T>::tof(ve[e]);
            s0 = fmaf(gv, wp[(c + e) * 3 + 0], s0);
            s1 = fmaf(gv, wp[(c + e) * 3 + 1], s1);
            s2 = fmaf(gv, wp[(c + e) * 3 + 2], s2);
          }
        }
      }
    }
    e0 = s0 + a.b[0]; e1 = s1 + a.b[1]; e2 = s2 + a.b[2];
  };
  float eps[3];
  conv3(img, eps[0], eps[1], eps[2]);
  if (a.cfg) {
#pragma clang fp contract(off)
    float u[3];
    conv3(img + a.n, u[0], u[1], u[2]);
    const float w1 = a.guide_w1;
#pragma unroll
    for (int c = 0; c < 3; ++c) eps[c] = w1 * eps[c] - a.guide_w * u[c];
  }
  if (!a.step_mode) {
#pragma unroll
    for (int c = 0; c < 3; ++c) a.eps_out[((size_t)img * 3 + c) * HW + rem] = eps[c];
    return;
  }
  {
#pragma clang fp contract(off)
    const int t = *a.tsel;
    const float c1 = a.coeff1[t], c2 = a.coeff2[t], sv = a.sqrt_var[t];
    bool bad = false;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const size_t o = ((size_t)img * 3 + c) * HW + rem;
      const float xv = a.x[o];
      const float mean = c1 * xv - c2 * eps[c];
      float xn = mean;
      if (t > 0) {
        const float z = a.noise ? a.noise[(size_t)t * a.n * 3 * HW + o] : philox_normal(a.run->seed, (unsigned)t, (unsigned long long)(a.run->noise_offset + (long long)o));
        xn = mean + sv * z;
      }
      bad |= (xn != xn);
      if (t == a.run->clip_at) xn = fminf(fmaxf(xn, -1.0f), 1.0f);
      a.x[o] = xn;
    }
    if (bad) atomicOr(a.nan_flag, 1);
  }
}

// Tiled tail: one block per 64 output pixels (64/W full rows of one image); the input
// halo rows are staged once in LDS (coalesced 16-B loads, padded pixel stride: no bank
// conflicts) and 4 threads per pixel split the channels, reduced by lane shuffles.
template <typename T>
__global__ __launch_bounds__(256) void tail2_kernel(TailArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) char tsm[];
  const int C = a.C, W = a.W, H = a.H;
  const int rpb = 64 / W;
  const int HW = H * W;
  const int PST = C * (int)sizeof(T) + 16;
  float* wl = (float*)tsm;           // [9][C][3]
  char* halo = tsm + 27 * C * 4;     // [(rpb+2)*(W+2)] pixels of PST bytes
  for (int i = threadIdx.x; i < 27 * C; i += 256) {
    const int co = i / (C * 9);
    const int r = i - co * C * 9;
    const int ci = r / 9, tap = r - ci * 9;
    wl[(tap * C + ci) * 3 + co] = a.w[i];
  }
  const int bpi = H / rpb;
  const int img = blockIdx.x / bpi, y0 = (blockIdx.x % bpi) * rpb;
  // wave = channel quarter (its weight reads are wave-uniform LDS broadcasts),
  // lane = output pixel (halo reads at a conflict-free padded pixel stride)
  const int tid = threadIdx.x, pl = tid & 63, cq = tid >> 6;
  const int py = pl / W, px = pl - (pl / W) * W;
  const int cpq = C / 4;
  float* red = (float*)(halo + (rpb + 2) * (W + 2) * PST);  // [2 passes][4 waves][64 px][3]
  for (int pass = 0; pass < (a.cfg ? 2 : 1); ++pass) {
    const int im = img + pass * a.n;
    __syncthreads();
    const T* gb = (const T*)a.g + (size_t)im * HW * C;
    const int cpp = C / EPC, npx = (rpb + 2) * (W + 2);
    for (int i = tid; i < npx * cpp; i += 256) {
      const int hp = i / cpp, ch = i - hp * cpp;
      const int hy = hp / (W + 2), hx = hp - hy * (W + 2);
      const int gy = y0 - 1 + hy, gx = hx - 1;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (gy >= 0 && gy < H && gx >= 0 && gx < W) v = *(const u32x4*)(gb + ((size_t)gy * W + gx) * C + ch * EPC);
      *(u32x4*)(halo + hp * PST + ch * 16) = v;
    }
    __syncthreads();
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int ky = 0; ky < 3; ++ky)
      for (int kx = 0; kx < 3; ++kx) {
        const char* hpix = halo + ((py + ky) * (W + 2) + px + kx) * PST;
        const float* wp = wl + (ky * 3 + kx) * C * 3;
        for (int c = cq * cpq; c < (cq + 1) * cpq; c += EPC) {
          const u32x4 v = *(const u32x4*)(hpix + c * (int)sizeof(T));
          const T* ve = (const T*)&v;
#pragma unroll
          for (int e0 = 0; e0 < EPC; e0 += 4) {
            const f32x4 w0 = *(const f32x4*)(wp + (c + e0) * 3);      // 12 consecutive weights:
            const f32x4 w1 = *(const f32x4*)(wp + (c + e0) * 3 + 4);  // 4 channels x 3 outputs
            const f32x4 w2 = *(const f32x4*)(wp + (c + e0) * 3 + 8);
            const float g0 = Elem<T>::tof(ve[e0]), g1 = Elem<T>::tof(ve[e0 + 1]);
            const float g2 = Elem<T>::tof(ve[e0 + 2]), g3 = Elem<T>::tof(ve[e0 + 3]);
            s0 = fmaf(g0, w0[0], s0); s1 = fmaf(g0, w0[1], s1); s2 = fmaf(g0, w0[2], s2);
            s0 = fmaf(g1, w0[3], s0); s1 = fmaf(g1, w1[0], s1); s2 = fmaf(g1, w1[1], s2);
            s0 = fmaf(g2, w1[2], s0); s1 = fmaf(g2, w1[3], s1); s2 = fmaf(g2, w2[0], s2);
            s0 = fmaf(g3, w2[1], s0); s1 = fmaf(g3, w2[2], s1); s2 = fmaf(g3, w2[3], s2);
          }
        }
      }
    float* rp = red + ((pass * 4 + cq) * 64 + pl) * 3;
    rp[0] = s0; rp[1] = s1; rp[2] = s2;
  }
  __syncthreads();
  if (tid >= 192) return;
  const int opx = tid / 3, oc = tid - opx * 3;  // (pixel, output channel), channel quarters summed in order
  float e = a.b[oc];
  {
    float s = 0.f;
    for (int w = 0; w < 4; ++w) s += red[(w * 64 + opx) * 3 + oc];
    e += s;
  }
  if (a.cfg) {
#pragma clang fp contract(off)
    float s = 0.f;
    for (int w = 0; w < 4; ++w) s += red[((4 + w) * 64 + opx) * 3 + oc];
    const float u = a.b[oc] + s;
    e = a.guide_w1 * e - a.guide_w * u;
  }
  const int rem = (y0 + opx / W) * W + (opx - (opx / W) * W);
  const size_t o = ((size_t)img * 3 + oc) * HW + rem;
  if (!a.step_mode) {
    a.eps_out[o] = e;
    return;
  }
  {
#pragma clang fp contract(off)
    const int t = *a.tsel;
    const float xv = a.x[o];
    const float mean = a.coeff1[t] * xv - a.coeff2[t] * e;
    float xn = mean;
    if (t > 0) {
      const float z = a.noise ? a.noise[(size_t)t * a.n * 3 * HW + o]
                              : philox_normal(a.run->seed, (unsigned)t, (unsigned long long)(a.run->noise_offset + (long long)o));
      xn = mean + a.sqrt_var[t] * z;
    }
    if (xn != xn) atomicOr(a.nan_flag, 1);
    if (t == a.run->clip_at) xn = fminf(fmaxf(xn, -1.0f), 1.0f);
    a.x[o] = xn;
  }
}

// bf16 tail on MFMA with the tail GroupNorm+SiLU fused (Model.py:252-256 / 282, then the
// sampler step as tail2_kernel). Block = 128 output pixels (128/W rows) of one image; the
// raw input halo ((128/W + 2) x (W + 2) pixels x C) is staged once in LDS with
// y = silu(x*a + b) applied (padding stays 0), at a padded pixel stride (tail_pst: conflict-free
// 16-B fragment reads); the staging issues 8 loads per thread before transforming any
// (HBM latency once per batch, not per chunk). Each wave owns 2 x 16 pixels:
// eps[pixel][co] = sum_k patch[pixel][k] W[co][k] on v_mfma_f32_16x16x32_bf16
// (k = tap*C + ci; 9C/32 k-steps; B columns 3..15 are zero).
// TM_PX output pixels per block: 128 (64 -- a smaller halo, 3 blocks a CU -- measured +0.3 %, removed in round 5);
// NTH threads: 512 (round 5: 8 waves, one 16-pixel group each -- twice the waves a CU for the halo transform's
// latency: 71.1 -> 65.5 us a launch at N = 256 against 256 threads, profiles/r05/tail_512_vs_256_r05x.txt)
// Halo pixel stride (bytes): 2C + 32 = (C / 8 + 2) x 16 B, == 2 (mod 4) 16-B units for C % 32 == 0. An A-fragment
// ds_read_b128 group ({0-3, 12-15, 20-27}, ...: 8 pixels of one k-group + 8 of the next) then lands on 16 distinct
// 16-B slots, the two k-groups on opposite slot parities (2C + 16, one unit odd, put pixel m + 1 of one k-group on
// pixel m's slot of the other: 6.8e6 bank-conflict cycles a launch at N = 256, profiles/r05/pmc_dispatch_table_r05ae.txt)
#ifndef ITSD_TAIL_PAD32
#define ITSD_TAIL_PAD32 1  // (0: 2C + 16, A/B builds)
#endif
__host__ __device__ constexpr int tail_pst(int C) { return 2 * C + (ITSD_TAIL_PAD32 ? 32 : 16); }

template <int TM_PX, int NTH>
__global__ __launch_bounds__(NTH, 2) void tail_mfma_kernel(TailArgs a) {
  constexpr int NW = NTH / 64, GPW = TM_PX / 16 / NW;  // waves; 16-pixel MFMA groups a wave
  static_assert(GPW >= 1 && GPW * 16 * NW == TM_PX, "tail geometry");
  extern __shared__ __attribute__((aligned(16))) char tsm[];
  const int C = a.C, W = a.W, H = a.H, HW = H * W;
  const int rpb = TM_PX / W, bpi = H / rpb, PST = tail_pst(C), NKS = 9 * C / 32;
  const int img = blockIdx.x / bpi, y0 = (blockIdx.x % bpi) * rpb;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  bf16x8* wl = (bf16x8*)tsm;                                   // [NKS][4][3]
  char* halo = tsm + NKS * 12 * 16;                            // [(rpb+2)*(W+2)][PST]
  float* red = (float*)(halo + (rpb + 2) * (W + 2) * PST);     // [2 passes][TM_PX][3]
  float* cfl = red + 2 * TM_PX * 3;                            // [4][C/8][4] this pass's GN coefficients
  const int m = lane & 15, kg = lane >> 4;
  int hbase[GPW];
#pragma unroll
  for (int gi = 0; gi < GPW; ++gi) {
    const int pl = wid * 16 * GPW + gi * 16 + m, py = pl / W, px = pl - py * W;
    hbase[gi] = (py * (W + 2) + px) * PST + 16 * kg;
  }
  const bf16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
  const int cpp = C / 8, npx = (rpb + 2) * (W + 2), total = npx * cpp;
  // the sampler step's operands of this thread's output items (it = tid, tid + NTH, ..), loaded now: their
  // latency hides behind the halo staging and the MFMAs
  constexpr int TIT = (TM_PX * 3 + NTH - 1) / NTH;
  float xpre[TIT];
  int tpre = 0;
  float c1pre = 0.f, c2pre = 0.f, svpre = 0.f;
  unsigned long long seedpre = 0;
  long long noffpre = 0;
  int clippre = -1;
  if (a.step_mode) {
    tpre = *a.tsel;
    seedpre = a.run->seed;
    noffpre = a.run->noise_offset;
    clippre = a.run->clip_at;
    c1pre = a.coeff1[tpre];
    c2pre = a.coeff2[tpre];
    svpre = a.sqrt_var[tpre];
#pragma unroll
    for (int k = 0; k < TIT; ++k) {
      const int it = tid + NTH * k, opx = it < TM_PX * 3 ? it / 3 : 0, oc = it < TM_PX * 3 ? it - opx * 3 : 0;
      const int rem = (y0 + opx / W) * W + (opx - (opx / W) * W);
      xpre[k] = a.x[((size_t)img * 3 + oc) * HW + rem];
    }
  }
  constexpr int TB = 4096 / NTH;  // halo items a thread per batch (C = 128, 32 x 32: the whole halo in one batch)
  for (int pass = 0; pass < (a.cfg ? 2 : 1); ++pass) {
    const int im = img + pass * a.n;
    __syncthreads();
    const bf16_t* gb = (const bf16_t*)a.g + (size_t)im * HW * C;
    for (int i0 = 0; i0 < total; i0 += TB * NTH) {
      u32x4 v[TB];
      int dst[TB];
#pragma unroll
      for (int u = 0; u < TB; ++u) {  // all loads of the batch first
        const int i = i0 + u * NTH + tid;
        const int hp = i / cpp, ch = i - hp * cpp;
        const int hy = hp / (W + 2), hx = hp - hy * (W + 2);
        const int gy = y0 - 1 + hy, gx = hx - 1;
        const bool ok = i < total && gy >= 0 && gy < H && gx >= 0 && gx < W;
        dst[u] = i < total ? hp * PST + ch * 16 : -1;
        v[u] = ok ? *(const u32x4*)(gb + ((size_t)gy * W + gx) * C + ch * 8) : u32x4{0u, 0u, 0u, 0u};
        if (!ok) dst[u] = i < total ? -2 - dst[u] : -1;  // padding: store zeros at -2 - dst
      }
      if (i0 == 0) {  // the image's GroupNorm coefficients (and, first pass, the weights) into LDS, their
                      // loads behind the batch's: one memory round trip for all of them
        // (coef[img][C/8][a0..a7, b0..b7] -> quarter q of chunk ch at (q C/8 + ch) x 16 B: the 16 chunks a 16-lane
        // read group stages are then 256 contiguous bytes, not 64-B strided -- a 4-way conflict on every read)
        for (int i = tid; i < cpp * 16; i += NTH) {
          const int ch = i >> 4, e = i & 15;
          cfl[((e >> 2) * cpp + ch) * 4 + (e & 3)] = a.coef[(size_t)im * cpp * 16 + i];
        }
        if (pass == 0)
          for (int i = tid; i < NKS * 12; i += NTH) wl[i] = *(const bf16x8*)(a.wmf + (size_t)i * 8);
        __syncthreads();
      }
#pragma unroll
      for (int u = 0; u < TB; ++u) {
        if (dst[u] == -1) continue;
        u32x4 y = {0u, 0u, 0u, 0u};
        int d = dst[u];
        if (d >= 0) {
          const int ch = (d % PST) / 16;
          const f32x4* cp = (const f32x4*)cfl + ch;
          const f32x4 a0 = cp[0], a1 = cp[cpp], b0 = cp[2 * cpp], b1 = cp[3 * cpp];
          // silu(v) = v / (1 + 2^(-v log2 e)): one exp2 and one rcp (the result is rounded to bf16)
          auto fsilu = [](float v) { return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v * -1.4426950408889634f)); };
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const float x0 = __uint_as_float(v[u][w] << 16), x1 = __uint_as_float(v[u][w] & 0xffff0000u);
            const float s0 = w < 2 ? a0[2 * w] : a1[2 * w - 4], s1 = w < 2 ? a0[2 * w + 1] : a1[2 * w - 3];
            const float t0 = w < 2 ? b0[2 * w] : b1[2 * w - 4], t1 = w < 2 ? b0[2 * w + 1] : b1[2 * w - 3];
            y[w] = pk_bf16(fsilu(x0 * s0 + t0), fsilu(x1 * s1 + t1));
          }
        } else {
          d = -2 - d;
        }
        *(u32x4*)(halo + d) = y;
      }
    }
    __syncthreads();
    f32x4 acc[GPW];
#pragma unroll
    for (int gi = 0; gi < GPW; ++gi) acc[gi] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int cpt = C / 32;
    {
#pragma unroll 4
    for (int ks = 0; ks < NKS; ++ks) {
      const int tap = ks / cpt, ci0 = (ks - tap * cpt) * 32;
      const int ky = tap / 3, kx = tap - ky * 3;
      const int toff = (ky * (W + 2) + kx) * PST + ci0 * 2;
      const bf16x8 bw = m < 3 ? wl[(ks * 4 + kg) * 3 + m] : z8;
#pragma unroll
      for (int gi = 0; gi < GPW; ++gi) {
        const bf16x8 af = *(const bf16x8*)(halo + hbase[gi] + toff);
        acc[gi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw, acc[gi], 0, 0, 0);
      }
    }
    // D[pixel 4*kg + i][co = m] of this wave's two 16-pixel groups
    if (m < 3) {
#pragma unroll
      for (int gi = 0; gi < GPW; ++gi)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[(pass * TM_PX + wid * 16 * GPW + gi * 16 + 4 * kg + i) * 3 + m] = acc[gi][i];
    }
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < TIT; ++k) {
    const int it = tid + NTH * k;
    if (it >= TM_PX * 3) break;
    const int opx = it / 3, oc = it - opx * 3;
    float e = red[opx * 3 + oc] + a.b[oc];
    if (a.cfg) {
#pragma clang fp contract(off)
      const float u = red[(TM_PX + opx) * 3 + oc] + a.b[oc];
      e = a.guide_w1 * e - a.guide_w * u;
    }
    const int rem = (y0 + opx / W) * W + (opx - (opx / W) * W);
    const size_t o = ((size_t)img * 3 + oc) * HW + rem;
    if (!a.step_mode) {
      a.eps_out[o] = e;
      continue;
    }
    {
#pragma clang fp contract(off)
      const int t = tpre;
      const float xv = xpre[k];
      const float mean = c1pre * xv - c2pre * e;
      float xn = mean;
      if (t > 0) {
        const float z = a.noise ? a.noise[(size_t)t * a.n * 3 * HW + o]
                                : philox_normal(seedpre, (unsigned)t, (unsigned long long)(noffpre + (long long)o));
        xn = mean + svpre * z;
      }
      if (xn != xn) atomicOr(a.nan_flag, 1);
      if (t == clippre) xn = fminf(fmaxf(xn, -1.0f), 1.0f);
      a.x[o] = xn;
    }
  }
}

static size_t tail_mfma_smem_px(int px, int H, int W, int C) {
  return (size_t)(9 * C / 32) * 12 * 16 + (size_t)(px / W + 2) * (W + 2) * tail_pst(C) + 2 * px * 3 * 4 +
         (size_t)C * 2 * 4;
}
static bool tail_mfma_ok_px(int px, int H, int W, int C) {
  return W <= px && px % W == 0 && px / W <= H && H % (px / W) == 0 && C % 32 == 0 &&
         tail_mfma_smem_px(px, H, W, C) <= 160 * 1024;
}
size_t tail_mfma_smem(int H, int W, int C) { return tail_mfma_smem_px(128, H, W, C); }
bool tail_mfma_ok(int H, int W, int C) { return tail_mfma_ok_px(128, H, W, C); }

hipError_t launch_tail_mfma(const TailArgs& a, hipStream_t s) {
  if (!a.coef || !a.wmf || !tail_mfma_ok(a.H, a.W, a.C)) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    for (const void* f : {(const void*)tail_mfma_kernel<128, 512>}) {
      hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e != hipSuccess) return e;
    }
    attr = true;
  }
  ITSD_LAUNCH((tail_mfma_kernel<128, 512>), dim3(a.n * (a.H / (128 / a.W))), dim3(512),
              tail_mfma_smem_px(128, a.H, a.W, a.C), s, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_tail(const TailArgs& a, hipStream_t s) {
  if (a.W <= 64 && 64 % a.W == 0 && a.H % (64 / a.W) == 0 && a.C % 32 == 0) {
    const size_t sm = 27 * a.C * 4 + (size_t)(64 / a.W + 2) * (a.W + 2) * (a.C * sizeof(T) + 16) + 2 * 4 * 64 * 3 * 4;
    if (sm > 160 * 1024) return hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
      hipError_t e = hipFuncSetAttribute((const void*)tail2_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         160 * 1024);
      if (e != hipSuccess) return e;
      attr = true;
    }
    ITSD_LAUNCH(tail2_kernel<T>, dim3(a.n * (a.H / (64 / a.W))), dim3(256), sm, s, a);
    return hipGetLastError();
  }
  const long long total = (long long)a.n * a.H * a.W;
  ITSD_LAUNCH(tail_kernel<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 27 * a.C * sizeof(float), s, a);
  return hipGetLastError();
}
template hipError_t launch_tail<float>(const TailArgs&, hipStream_t);
template hipError_t launch_tail<bf16_t>(const TailArgs&, hipStream_t);

// ============================================================================ embeddings
// DDPM functional sinusoid (Model.py:74-88): e = interleave(sin(t f), cos(t f)).
// CFG: row of a table (nn.Embedding, ModelCondition.py:38,54) selected by idx.
__global__ void emb_input_kernel(const int* idx, int M, const float* freq, const float* table, int d, float* out,
                                 int idx_offset) {
  const int m = blockIdx.x;
  if (m >= M) return;
  const int t = idx ? idx[m] : (m + idx_offset);
  for (int i = threadIdx.x; i < d; i += blockDim.x) {
    float v;
    if (table) v = table[(size_t)t * d + i];
    else {
      const float e = (float)t * freq[i >> 1];
      v = (i & 1) ? cosf(e) : sinf(e);
    }
    out[(size_t)m * d + i] = v;
  }
}

// out[m][j] = act_out( sum_i act_in(in[m][i]) * Wt[i][j] + b[j] ), Wt = W^T [Nin][Nout] fp32.
__global__ __launch_bounds__(256) void linear_kernel(const float* in, int M, int Nin, const float* Wt, const float* b,
                                                     int Nout, int silu_in, float* out) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int m = blockIdx.y;
  extern __shared__ float xin[];
  for (int i = threadIdx.x; i < Nin; i += 256) {
    float v = in[(size_t)m * Nin + i];
    xin[i] = silu_in ? silu(v) : v;
  }
  __syncthreads();
  if (j >= Nout) return;
  float acc = 0.0f;
  for (int i = 0; i < Nin; ++i) acc = fmaf(xin[i], Wt[(size_t)i * Nout + j], acc);
  out[(size_t)m * Nout + j] = acc + b[j];
}

hipError_t launch_emb_input(const int* idx, int M, const float* freq, const float* table, int d, float* out,
                            int idx_offset, hipStream_t s) {
  ITSD_LAUNCH(emb_input_kernel, dim3(M), dim3(128), 0, s, idx, M, freq, table, d, out, idx_offset);
  return hipGetLastError();
}
hipError_t launch_linear(const float* in, int M, int Nin, const float* Wt, const float* b, int Nout, int silu_in,
                         float* out, hipStream_t s) {
  ITSD_LAUNCH(linear_kernel, dim3((Nout + 255) / 256, M), dim3(256), Nin * sizeof(float), s, in, M, Nin, Wt,
                     b, Nout, silu_in, out);
  return hipGetLastError();
}

// ============================================================================ verifiers
// One block per candidate (b images of c*h*w). Reductions in fp64, then the fp32
// roundings the reference performs (torch fp32 tensors, .item() to Python float).
//  ORACLE    verifier.py:62-63   1/(1 + mean_b var_unbiased(x_b))
//  AESTHETIC verifier.py:277-286 if min<0: x=(x+1)/2 ; 2 * mean_b std_unbiased(x_b)
//  SELFSUP   verifier.py:219-246 avgpool 8x8 -> L2 normalise -> mean off-diagonal cosine
__global__ __launch_bounds__(256) void verify_kernel(int kind, const float* images, int b, int c, int h, int w,
                                                     double* scores, const float* ref) {
  const int cand = blockIdx.x;
  const int D = c * h * w;
  const float* base = images + (size_t)cand * b * D;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ double red[4];
  __shared__ double bc;
  __shared__ float feat[64][192];  // selfsup: up to 64 images x (c*8*8 <= 192)
  auto block_sum = [&](double v) -> double {
    v = wave_sum_d(v);
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
  };
  if (kind == 3) {  // OracleVerifier with dataset stats (verifier.py:66): mean of the candidate's images
    double s = 0.0;
    for (long long i = tid; i < (long long)b * D; i += 256) s += base[i];
    s = block_sum(s);
    if (tid == 0) scores[cand] = (double)(float)(s / ((double)b * D));
    return;
  }
  if (kind == 0 || kind == 2) {
    bool shift = false;
    if (kind == 2) {
      float mn = INFINITY;
      for (int i = tid; i < b * D; i += 256) mn = fminf(mn, base[i]);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mn = fminf(mn, __shfl_xor(mn, o, 64));
      __syncthreads();
      if (lane == 0) red[wid] = mn;
      __syncthreads();
      shift = fminf(fminf((float)red[0], (float)red[1]), fminf((float)red[2], (float)red[3])) < 0.0f;
    }
    float accum = 0.0f;  // fp32 mean over images, like a torch fp32 .mean()
    for (int im = 0; im < b; ++im) {
      const float* xb = base + (size_t)im * D;
      double s = 0.0;
      for (int i = tid; i < D; i += 256) {
        float v = xb[i];
        if (shift) v = (v + 1.0f) / 2.0f;
        s += v;
      }
      const double mean = block_sum(s) / D;
      double q = 0.0;
      for (int i = tid; i < D; i += 256) {
        float v = xb[i];
        if (shift) v = (v + 1.0f) / 2.0f;
        const double d = (double)v - mean;
        q += d * d;
      }
      const double var = block_sum(q) / (D - 1);
      accum += (kind == 0) ? (float)var : (float)sqrt(var);
    }
    if (tid == 0) {
      const float m = accum / (float)b;
      scores[cand] = (kind == 0) ? 1.0 / (1.0 + (double)m) : (double)(m + m);
    }
    return;
  }
  // SELFSUP: adaptive_avg_pool2d to 8x8 (h, w divisible by 8 here)
  const int F = c * 64;
  const int ph = h / 8, pw = w / 8;
  for (int im = 0; im < b && im < 64; ++im) {
    const float* xb = base + (size_t)im * D;
    for (int f = tid; f < F; f += 256) {
      const int ch = f / 64, cell = f % 64, cy = cell / 8, cx = cell % 8;
      float s = 0.0f;
      for (int yy = 0; yy < ph; ++yy)
        for (int xx = 0; xx < pw; ++xx) s += xb[(size_t)ch * h * w + (cy * ph + yy) * w + cx * pw + xx];
      feat[im][f] = s / (float)(ph * pw);
    }
  }
  __syncthreads();
  if (tid < 64 && tid < b) {
    double nn = 0.0;
    for (int f = 0; f < F; ++f) nn += (double)feat[tid][f] * feat[tid][f];
    const float nrm = fmaxf((float)sqrt(nn), 1e-12f);
    for (int f = 0; f < F; ++f) feat[tid][f] = feat[tid][f] / nrm;
  }
  __syncthreads();
  if (kind == 4) {  // paired mode (verifier.py:237-240): cosine of image i with reference row i
    // one candidate = one image (the reference's .item() of a b-vector needs b == 1)
    const float* r = ref + (size_t)cand * F;
    double rr = 0.0, fr = 0.0;
    for (int f = tid; f < F; f += 256) {
      rr += (double)r[f] * r[f];
      fr += (double)feat[0][f] * r[f];
    }
    rr = block_sum(rr);
    fr = block_sum(fr);
    if (tid == 0) scores[cand] = (double)(float)(fr / fmax(sqrt(rr), 1e-12));
    return;
  }
  double s = 0.0;
  for (int pr = tid; pr < b * b; pr += 256) {
    const int i = pr / b, j = pr % b;
    if (i == j) continue;
    double d = 0.0;
    for (int f = 0; f < F; ++f) d += (double)feat[i][f] * feat[j][f];
    s += (double)(float)d;
  }
  s = block_sum(s);
  if (tid == 0) {
    const long long cnt = (long long)b * b - b;
    bc = cnt > 0 ? s / (double)cnt : NAN;
    scores[cand] = (double)(float)bc;
  }
}

hipError_t launch_verify(int kind, const float* images, int n_cand, int b, int c, int h, int w, double* scores,
                         const float* ref, hipStream_t s) {
  ITSD_LAUNCH(verify_kernel, dim3(n_cand), dim3(256), 0, s, kind, images, b, c, h, w, scores, ref);
  return hipGetLastError();
}

// out[c][e] = pivot[e] + scale * z(seed, stream_id, (cand_offset + c) * per_cand + e)
__global__ __launch_bounds__(256) void noise_kernel(float* out, const float* pivot, long long total, long long per_cand,
                                                    float scale, unsigned long long seed, unsigned stream_id,
                                                    long long base) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const float z = philox_normal(seed, stream_id, (unsigned long long)(base + i));
  out[i] = (pivot ? pivot[i % per_cand] : 0.0f) + scale * z;
}
hipError_t launch_noise(float* out, const float* pivot, int n_cand, long long per_cand, float scale,
                        unsigned long long seed, unsigned stream_id, long long cand_offset, hipStream_t s) {
  const long long total = (long long)n_cand * per_cand;
  ITSD_LAUNCH(noise_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, out, pivot, total, per_cand,
                     scale, seed, stream_id, cand_offset * per_cand);
  return hipGetLastError();
}

// ============================================================================ representation
// The pre-tail activation (NHWC, bf16 or fp32) of image img -> NCHW fp32 (ModelCondition.py:225-235's
// last_representation): 64 pixels x 64 channels per block through LDS, coalesced on both sides.
template <typename T>
__global__ __launch_bounds__(256) void nhwc_to_nchw_kernel(const T* in, float* out, int HW, int C) {
  __shared__ float tile[64][65];
  const int img = blockIdx.z, p0 = blockIdx.x * 64, c0 = blockIdx.y * 64, tid = threadIdx.x;
  const T* src = in + (size_t)img * HW * C;
  for (int i = tid; i < 64 * 64; i += 256) {
    const int p = i >> 6, c = i & 63;
    tile[p][c] = (p0 + p < HW && c0 + c < C) ? Elem<T>::tof(src[(size_t)(p0 + p) * C + c0 + c]) : 0.f;
  }
  __syncthreads();
  float* dst = out + (size_t)img * C * HW;
  for (int i = tid; i < 64 * 64; i += 256) {
    const int c = i >> 6, p = i & 63;
    if (p0 + p < HW && c0 + c < C) dst[(size_t)(c0 + c) * HW + p0 + p] = tile[p][c];
  }
}
template <typename T>
hipError_t launch_nhwc_to_nchw(const void* in, float* out, int n, int HW, int C, hipStream_t s) {
  ITSD_LAUNCH(nhwc_to_nchw_kernel<T>, dim3((HW + 63) / 64, (C + 63) / 64, n), dim3(256), 0, s, (const T*)in, out, HW, C);
  return hipGetLastError();
}
template hipError_t launch_nhwc_to_nchw<float>(const void*, float*, int, int, int, hipStream_t);
template hipError_t launch_nhwc_to_nchw<bf16_t>(const void*, float*, int, int, int, hipStream_t);

// ============================================================================ small utilities
__global__ void set_int_kernel(int* p, int v) { *p = v; }
// start of a sampler run: step counter, NaN flag and the run's parameters (one launch, outside
// the replayed step graph)
__global__ void run_begin_kernel(int* t, int t_begin, int* nan_flag, RunParams* run, RunParams v) {
  *t = t_begin;
  nan_flag[0] = 0;  // the NaN flag (Diffusion.py:100)
  nan_flag[1] = 0;  // the in-kernel hand-off status word (AttnBlockArgs::err)
  *run = v;
}
hipError_t launch_run_begin(int* t, int t_begin, int* nan_flag, RunParams* run, const RunParams& v, hipStream_t s) {
  ITSD_LAUNCH(run_begin_kernel, dim3(1), dim3(1), 0, s, t, t_begin, nan_flag, run, v);
  return hipGetLastError();
}
__global__ void add_int_kernel(int* p, int v) { *p += v; }
hipError_t launch_set_int(int* p, int v, hipStream_t s) {
  ITSD_LAUNCH(set_int_kernel, dim3(1), dim3(1), 0, s, p, v);
  return hipGetLastError();
}
hipError_t launch_add_int(int* p, int v, hipStream_t s) {
  ITSD_LAUNCH(add_int_kernel, dim3(1), dim3(1), 0, s, p, v);
  return hipGetLastError();
}

}  // namespace itsd
