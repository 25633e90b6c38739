// Implicit-GEMM convolution on MFMA for gfx950 (the UNet's nn.Conv2d sites:
// ResBlock block1/block2 3x3 (Diffusion/Model.py:173,183), shortcut 1x1 (:186),
// AttnBlock q/k/v/proj 1x1 (:133-136, fused q|k|v), DownSample 3x3 s2 (:99),
// UpSample nearest-x2 + 3x3 (:114,123)).
//
// GEMM view (operands swapped so the epilogue writes rows of couts per pixel):
//   D[cout][pixel] = sum_k W[cout][k] * X[pixel][k],  k = (ky*ks + kx)*Cin + ci
// A operand = packed weights [Cout][K], B operand = gathered NHWC activations.
// Block tile 128 couts x 128 pixels, 4 waves in 2x2, each wave 64x64 =
// 2x2 tiles of 32x32 MFMA (bf16: v_mfma_f32_32x32x16_bf16; fp32 parity mode:
// v_mfma_f32_32x32x2_f32, exact fp32 products).
// Both LDS images are [128 rows][128 B] with the 16-B chunk index XOR-swizzled by
// (row>>1)&7, which makes the per-lane ds_read_b128 fragment reads conflict-free.
// K loop: register-staged double buffer (global loads of stage k+1 are in flight
// while stage k's MFMAs run), one barrier per stage.
// Epilogue (LDS-staged) fuses + bias + temb_proj row (+ CFG cond_proj row) + residual,
// stores coalesced 16-B chunks and emits the consumer GroupNorm's channel statistics.
#include "common.h"

namespace itsd {

constexpr int CONV_BM = 128;  // couts per block
constexpr int CONV_BN = 128;  // pixels per block
constexpr int ROWB = 128;     // bytes per LDS row
constexpr int TILEB = 128 * ROWB;
constexpr int EROW = 132;  // epilogue LDS row (floats)
constexpr int SMEM_BYTES = (2 * 2 * TILEB > 128 * EROW * 4) ? 2 * 2 * TILEB : 128 * EROW * 4;

__device__ __forceinline__ int swz(int r, int c) { return r * ROWB + ((c ^ ((r >> 1) & 7)) << 4); }

template <typename T>
__global__ __launch_bounds__(256, 2) void conv_igemm(ConvArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);  // elements per 16-B chunk
  constexpr int BK = 8 * EPC;               // k per stage
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tileP = blockIdx.x * CONV_BN, tileC = blockIdx.y * CONV_BM;
  const int c16 = tid & 7, r0 = tid >> 3;
  const int Cin = a.C1 + a.C2;
  const int HWo = a.Hout * a.Wout;
  const int Hv = a.upsample ? 2 * a.Hin : (a.zins ? 2 * a.Hin - 1 : a.Hin);
  const int Wv = a.upsample ? 2 * a.Win : (a.zins ? 2 * a.Win - 1 : a.Win);
  const T* src1 = (const T*)a.src1;
  const T* src2 = (const T*)a.src2;
  const T* wt = (const T*)a.wt;

  int pimg[4], piy[4], pix[4];
  bool pval[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = tileP + r0 + 32 * i;
    pval[i] = p < a.M;
    const int img = p / HWo;
    const int rem = p - img * HWo;
    const int oy = rem / a.Wout;
    const int ox = rem - oy * a.Wout;
    pimg[i] = img;
    piy[i] = oy * a.stride - a.pad;
    pix[i] = ox * a.stride - a.pad;
  }

  u32x4 ra[4], rb[4];
  auto gload = [&](int kc) {
    const int k0 = kc * BK + c16 * EPC;
    const bool kval = k0 < a.K;
    const int tap = k0 / Cin;
    const int ci = k0 - tap * Cin;
    const int ky = tap / a.ksize;
    const int kx = tap - ky * a.ksize;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = tileC + r0 + 32 * i;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (kval && co < a.Cout) v = *(const u32x4*)(wt + (size_t)co * a.K + k0);
      ra[i] = v;
    }
    const T* src;
    int Cs, cs;
    if (ci < a.C1) { src = src1; Cs = a.C1; cs = ci; }
    else { src = src2; Cs = a.C2; cs = ci - a.C1; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int iy = piy[i] + ky, ix = pix[i] + kx;
      bool ok = kval && pval[i] && iy >= 0 && iy < Hv && ix >= 0 && ix < Wv;
      if (a.zins) ok = ok && !((iy | ix) & 1);
      if (a.upsample | a.zins) { iy >>= 1; ix >>= 1; }
      u32x4 v = {0u, 0u, 0u, 0u};
      if (ok) v = *(const u32x4*)(src + (((size_t)pimg[i] * a.Hin + iy) * a.Win + ix) * Cs + cs);
      rb[i] = v;
    }
  };
  auto sstore = [&](int s) {
    char* A = smem + s * 2 * TILEB;
    char* B = A + TILEB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = r0 + 32 * i;
      *(u32x4*)(A + swz(r, c16)) = ra[i];
      *(u32x4*)(B + swz(r, c16)) = rb[i];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  const int rl = lane & 31, hh = lane >> 5;
  auto compute = [&](int s) {
    const char* A = smem + s * 2 * TILEB;
    const char* B = A + TILEB;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        bf16x8 af[2], bfg[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = *(const bf16x8*)(A + swz(wm * 64 + i * 32 + rl, 2 * kk + hh));
#pragma unroll
        for (int j = 0; j < 2; ++j) bfg[j] = *(const bf16x8*)(B + swz(wn * 64 + j * 32 + rl, 2 * kk + hh));
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
      }
    } else {
      // k mapping for the f32 MFMA: step s, lane half h -> k = 16h + s (A and B alike).
      f32x4 af[2][4], bfg[2][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i][q] = *(const f32x4*)(A + swz(wm * 64 + i * 32 + rl, 4 * hh + q));
#pragma unroll
        for (int j = 0; j < 2; ++j) bfg[j][q] = *(const f32x4*)(B + swz(wn * 64 + j * 32 + rl, 4 * hh + q));
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][q][e], bfg[j][q][e], acc[i][j], 0, 0, 0);
    }
  };

  const int nK = (a.K + BK - 1) / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kc = 0; kc < nK; ++kc) {
    const int s = kc & 1;
    if (kc + 1 < nK) gload(kc + 1);
    compute(s);
    if (kc + 1 < nK) sstore(s ^ 1);
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  // 1. accumulators -> fp32 tile in LDS [pixel][cout] (row pad 4 floats: conflict-free)
  // 2. fused bias + temb/cemb rows + residual, rounded and stored as full 16-B chunks
  //    (coalesced rows of the NHWC output), rounded values written back to LDS
  // 3. per-channel (sum, sum of squares) over each pixel slot of the tile: the
  //    GroupNorm statistics of the consumer (Model.py:171,180), written as a
  //    deterministic partial slab stats[slot][2][Cout] (no atomics).
  float* E = (float*)smem;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 v4 = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        *(f32x4*)(E + (wn * 64 + j * 32 + rl) * EROW + wm * 64 + i * 32 + 8 * g + 4 * hh) = v4;
      }
  __syncthreads();
  const long long trow = a.temb ? (a.temb_tsel ? (long long)(*a.temb_tsel) * a.temb_row_stride : 0) : 0;
  constexpr int CPR = 128 / EPC;  // 16-B output chunks per tile row
  for (int it = tid; it < 128 * CPR; it += 256) {
    const int pl = it / CPR, cl = (it - pl * CPR) * EPC;
    const int p = tileP + pl, co = tileC + cl;
    if (p >= a.M || co >= a.Cout) continue;
    const int img = p / HWo;
    float v[EPC];
#pragma unroll
    for (int q = 0; q < EPC / 4; ++q) {
      const f32x4 e4 = *(const f32x4*)(E + pl * EROW + cl + 4 * q);
      const f32x4 b4 = *(const f32x4*)(a.bias + co + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * q + e] = e4[e] + b4[e];
    }
    if (a.temb) {
      const float* tb = a.temb + trow + (long long)img * a.temb_img_stride + co;
#pragma unroll
      for (int q = 0; q < EPC / 4; ++q) {
        const f32x4 t4 = *(const f32x4*)(tb + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] += t4[e];
      }
    }
    if (a.cemb) {
      int lab = 0;
      if (a.cemb_uncond_from < 0 || img < a.cemb_uncond_from) lab = a.cemb_labels[img % a.cemb_label_mod];
      const float* cb = a.cemb + (long long)lab * a.cemb_row_stride + co;
#pragma unroll
      for (int q = 0; q < EPC / 4; ++q) {
        const f32x4 c4 = *(const f32x4*)(cb + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] += c4[e];
      }
    }
    const size_t o = (size_t)p * a.Cout + co;
    if (a.resid) {
      const u32x4 r = *(const u32x4*)((const T*)a.resid + o);
      const T* re = (const T*)&r;
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[e] += Elem<T>::tof(re[e]);
    }
    u32x4 w;
    T* we = (T*)&w;
#pragma unroll
    for (int e = 0; e < EPC; ++e) we[e] = Elem<T>::to(v[e]);
    *(u32x4*)((T*)a.out + o) = w;
    if (a.stats) {
#pragma unroll
      for (int q = 0; q < EPC / 4; ++q) {
        f32x4 s4;
#pragma unroll
        for (int e = 0; e < 4; ++e) s4[e] = Elem<T>::tof(we[4 * q + e]);
        *(f32x4*)(E + pl * EROW + cl + 4 * q) = s4;
      }
    }
  }
  if (a.stats) {
    __syncthreads();
    const int Gt = HWo < 128 ? HWo : 128;  // pixels per slot (host guarantees 128 % HWo == 0 or HWo % 128 == 0)
    const int S = 128 / Gt;
    for (int item = tid; item < S * 128; item += 256) {
      const int s = item >> 7, cl = item & 127;
      const int co = tileC + cl, p0 = tileP + s * Gt;
      if (co >= a.Cout || p0 >= a.M) continue;
      float sum = 0.f, sq = 0.f;
      for (int k = 0; k < Gt; ++k) {
        const float v = E[(s * Gt + k) * EROW + cl];
        sum += v;
        sq = fmaf(v, v, sq);
      }
      const long long slot = p0 / Gt;
      a.stats[(slot * 2) * a.Cout + co] = sum;
      a.stats[(slot * 2 + 1) * a.Cout + co] = sq;
    }
  }
}

template <typename T>
hipError_t launch_conv(const ConvArgs& a, hipStream_t s) {
  dim3 grid((a.M + CONV_BN - 1) / CONV_BN, (a.Cout + CONV_BM - 1) / CONV_BM);
  hipLaunchKernelGGL(conv_igemm<T>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

template hipError_t launch_conv<float>(const ConvArgs&, hipStream_t);
template hipError_t launch_conv<bf16_t>(const ConvArgs&, hipStream_t);

}  // namespace itsd
