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
// Epilogue fuses + bias + temb_proj row (+ CFG cond_proj row) + residual.
#include "common.h"

namespace itsd {

constexpr int CONV_BM = 128;  // couts per block
constexpr int CONV_BN = 128;  // pixels per block
constexpr int ROWB = 128;     // bytes per LDS row
constexpr int TILEB = 128 * ROWB;

__device__ __forceinline__ int swz(int r, int c) { return r * ROWB + ((c ^ ((r >> 1) & 7)) << 4); }

template <typename T>
__global__ __launch_bounds__(256, 2) void conv_igemm(ConvArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);  // elements per 16-B chunk
  constexpr int BK = 8 * EPC;               // k per stage
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILEB];

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
  const long long trow = a.temb ? (a.temb_tsel ? (long long)(*a.temb_tsel) * a.temb_row_stride : 0) : 0;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int p = tileP + wn * 64 + j * 32 + rl;
    if (p >= a.M) continue;
    const int img = p / HWo;
    const float* tb = a.temb ? a.temb + trow + (long long)img * a.temb_img_stride : nullptr;
    const float* cb = nullptr;
    if (a.cemb) {
      int lab = 0;
      if (a.cemb_uncond_from < 0 || img < a.cemb_uncond_from) lab = a.cemb_labels[img % a.cemb_label_mod];
      cb = a.cemb + (long long)lab * a.cemb_row_stride;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int co = tileC + wm * 64 + i * 32 + 8 * g + 4 * hh;
        if (co >= a.Cout) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * g + e];
        const f32x4 bb = *(const f32x4*)(a.bias + co);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bb[e];
        if (tb) {
          const f32x4 t4 = *(const f32x4*)(tb + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += t4[e];
        }
        if (cb) {
          const f32x4 c4 = *(const f32x4*)(cb + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += c4[e];
        }
        const size_t o = (size_t)p * a.Cout + co;
        if constexpr (sizeof(T) == 2) {
          if (a.resid) {
            const uint2 r2 = *(const uint2*)((const bf16_t*)a.resid + o);
            v[0] += bf2f((bf16_t)(r2.x & 0xffff)); v[1] += bf2f((bf16_t)(r2.x >> 16));
            v[2] += bf2f((bf16_t)(r2.y & 0xffff)); v[3] += bf2f((bf16_t)(r2.y >> 16));
          }
          uint2 w2;
          w2.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          w2.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          *(uint2*)((bf16_t*)a.out + o) = w2;
        } else {
          if (a.resid) {
            const f32x4 r4 = *(const f32x4*)((const float*)a.resid + o);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += r4[e];
          }
          f32x4 w4 = {v[0], v[1], v[2], v[3]};
          *(f32x4*)((float*)a.out + o) = w4;
        }
      }
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
