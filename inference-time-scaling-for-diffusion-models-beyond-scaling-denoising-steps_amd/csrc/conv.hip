// Implicit-GEMM convolution on MFMA for gfx950 (the UNet's nn.Conv2d sites:
// ResBlock block1/block2 3x3 (Diffusion/Model.py:173,183), shortcut 1x1 (:186),
// AttnBlock q/k/v/proj 1x1 (:133-136, fused q|k|v), DownSample 3x3 s2 (:99),
// UpSample nearest-x2 + 3x3 (:114,123); CFG 5x5 s2 and ConvTranspose2d as a
// zero-insertion gather conv (ModelCondition.py:69,80)).
//
// GEMM view (operands swapped so the epilogue writes rows of couts per pixel):
//   D[cout][pixel] = sum_k W[cout][k] * X[pixel][k],  k = (ky*ks + kx)*Cin + ci
// A operand = packed weights [Cout][K], B operand = gathered NHWC activations.
// Block tile 128 couts x 128 pixels, 4 waves in 2x2, each wave 64x64 =
// 2x2 tiles of 32x32 MFMA (bf16: v_mfma_f32_32x32x16_bf16; fp32 parity mode:
// v_mfma_f32_32x32x2_f32, exact fp32 products).
// Both LDS images are [128 rows][128 B] with the 16-B chunk index XOR-swizzled by
// (row>>1)&7, which makes the per-lane ds_read_b128 fragment reads conflict-free.
//
// Two main loops:
//  * conv_pipe (every shape whose input channels split into whole 128-B K-chunks,
//    i.e. all Arch A/C layers): a 4-stage LDS ring filled by global_load_lds
//    (HBM/L2 -> LDS DMA, 1 KiB per wave-instruction, inverse-swizzled per-lane
//    source address; padded / out-of-range rows read a zero page), counted
//    s_waitcnt vmcnt + raw s_barrier so three stages stay in flight while one is
//    consumed -- the loop is otherwise load-latency bound.
//  * conv_igemm (generic fallback): register-staged double buffer.
// Epilogue (shared, LDS-staged): + bias + temb_proj row (+ CFG cond_proj row) +
// residual, coalesced 16-B stores, and the consumer GroupNorm's channel statistics.
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace itsd {

constexpr int CONV_BM = 128;  // couts per block
constexpr int CONV_BN = 128;  // pixels per block
constexpr int ROWB = 128;     // bytes per LDS row
constexpr int TILEB = 128 * ROWB;
constexpr int EROW = 132;  // epilogue LDS row (floats)
constexpr int EPI_BYTES = 128 * EROW * 4 + 8 * 2 * 128 * 4;  // fp32 tile + statistics partials
constexpr int SMEM_BYTES = (2 * 2 * TILEB > EPI_BYTES) ? 2 * 2 * TILEB : EPI_BYTES;
int g_fuse_gn = 1;
int g_conv_dbg = 0;
int g_conv_variant = 2;  // 2 conv_pipe (2-stage LDS-DMA ring), 1 conv_igemm (register-staged)
int g_small_conv = 1;    // 64x64-tile conv for the small levels: 0 off, 1 auto, 2 whenever eligible
int g_conv1x1 = 1;       // streaming 1x1 kernel for statistics-free 1x1 convs of large pixel counts: 0 off,
                         // 1 on (4-stage ring), 2 on (7-stage ring) ("conv1x1")
int g_small_8x8 = 1;     // ... and for the 8x8 level's convs when the 128x128 grid under-fills the chip ("small_8x8")
int g_small_wide = 1;    // ... also for statistics-free convs of larger images (64-pixel tiles inside one image)
                         // whose 128x128 conv_pipe grid under-fills the chip (small batches) ("small_wide")
int g_splitk = 1;        // split-K for under-filled grids (variant 2): 0 off, 1 auto, >= 2 forced slices
int g_gn_wide = 1;       // 256-pixel fused GroupNorm conv: 0 off, 1 auto, 2 whenever eligible
int g_p4_w = 7;          // levels conv3x3_gn_p4_kernel takes: bit 0 W = 8, 1 W = 16, 2 W = 32 (64x64 runs p5: p4 there
                         // measured 34.8 vs 33.0 us a launch at C4's N = 16, profiles/r04/census_c4_p4_64*; removed in round 5)
int g_num_cus = 256;     // compute units of the device (set at itsd_unet_create): persistent grids
int g_splitk_inl = 1;     // conv_pipe split-K combined in-launch (ticket) instead of splitk_epilogue_kernel
int g_p4_plain = 1;      // plain 3x3 stride-1 convs (the CFG upsample's conv) on conv3x3_gn_p4_kernel<W, 2>
int g_small_minks = 8;    // conv_small split K: >= this many K-chunks a slice (itsd_set_option "small_minks"; 8 against
                          // 2: N=32 step -2.3 %, N=64 -0.9 %, N=256 / C3 / C4 equal, profiles/r04/small_minks_ab.txt)
int g_convt_prune = 1;    // ConvTranspose2d sub-pixel phases skip their all-zero taps (itsd_set_option "convt_prune")
int g_subpix_split = 1;   // under-filled sub-pixel conv_pipe launches split K in-launch (itsd_set_option "subpix_split")
int g_p4_xcd = 2;        // conv3x3_gn_p4_kernel: each XCD a contiguous range of tiles (ConvArgs::xcd): 0 off, 1 every
                         // level (measured -2 % at N = 256), 2 the 8x8 level only (a pixel tile's cout tiles on one
                         // XCD: its input read once per L2; 8x8 HBM traffic 98.5 -> 65.1 MB a launch at equal step
                         // time, profiles/r05/p4_xcd8_traffic_r05s.txt)
int g_p4_c96 = 1;        // 8x8 p4 on 96-cout tiles where they fill the CUs better: 0 off, 1 auto, 2 always (conv_p4_c96)
int g_p4_sub = 1;        // nearest-x2 upsample convs on conv3x3_gn_p4_kernel's sub-pixel form (AB = 128)
int g_p5 = 1;            // conv3x3_gn_p5_kernel at 8x8: 0 off, 1 auto (where p4 has < 192 tiles), 2 always (4x4: always)
int g_p5_split = 0;      // its K slices: 0 auto, >= 1 forced
int g_p5_sc = 1;         // the ResBlock's 1x1 shortcut folded into its block2 p5 conv: 0 off, 1 auto (cost model), 2 always
int g_p5_xl = 3;    // p5's split-K partials exchanged through one XCD's L2 (ConvArgs::kxl): 0 off, 1 the shared combine at
                    // W >= 8, 2 every eligible form, 3 (shipped) 1 + the two-slice form at 8x8 / 16x16 where K <= 3456
int g_p5_pub = 1;   // p5's two-slice last-arriver combine: only the first arriver stores its partial (0: both, round 5)
int g_p5_dist = 1;       // p5's split-K combine shared by every slice of a tile where all items are co-resident (2: the
                         // same plans, combined by the last arriver)
int g_gn_fold = 1;       // p5 finalizes its input GroupNorm itself (no gn_coef launch): 0 off, 1 on

__device__ __forceinline__ int swz(int r, int c) { return r * ROWB + ((c ^ ((r >> 1) & 7)) << 4); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// One BK-deep stage of MFMAs for a wave's 64x64 sub-tile.
template <typename T>
__device__ __forceinline__ void mma_stage(const char* A, const char* B, f32x16 (&acc)[2][2], int wm, int wn, int rl,
                                          int hh) {
  if constexpr (sizeof(T) == 2) {
    // fragment reads two k-steps ahead of their MFMAs (two buffers, order pinned: the
    // scheduler otherwise reads each k-step right before its MFMAs behind an lgkmcnt(0))
    bf16x8 fa[2][2], fb[2][2];
    auto rd = [&](int kk, int buf) {
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[buf][i] = *(const bf16x8*)(A + swz(wm * 64 + i * 32 + rl, 2 * kk + hh));
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[buf][j] = *(const bf16x8*)(B + swz(wn * 64 + j * 32 + rl, 2 * kk + hh));
    };
    rd(0, 0);
    rd(1, 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int b = kk & 1;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[b][i], fb[b][j], acc[i][j], 0, 0, 0);
      if (kk + 2 < 4) rd(kk + 2, b);
      __builtin_amdgcn_sched_barrier(0);
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
}

// Shared epilogue. Precondition: every wave is done reading smem (barrier passed).
// 1. accumulators -> fp32 tile in LDS [pixel][cout] (row pad 4 floats: conflict-free)
// 2. fused bias + temb/cemb rows + residual, rounded and stored as full 16-B chunks
//    (coalesced rows of the NHWC output), rounded values written back to LDS
// 3. per-channel (sum, sum of squares) over each pixel slot of the tile: the
//    GroupNorm statistics of the consumer (Model.py:171,180), written as a
//    deterministic partial slab stats[slot][2][Cout] (no atomics).
// Additive values (bias + temb row + CFG cond row) of UB tile entries it0 + u * step (image
// img0 + it / BM, cout tileC + it % BM), all loads of the batch issued before the first use: the
// labels first, then the rows (the cond row's address depends on the label).
template <int BM, int UB>
__device__ __forceinline__ void addv_batch(const ConvArgs& a, int tileC, int img0, int HWo, int nent, long long trow,
                                           int it0, int step, float (&v)[UB]) {
  int lab[UB];
#pragma unroll
  for (int u = 0; u < UB; ++u) {
    const int it = it0 + u * step, img = img0 + it / BM;
    lab[u] = 0;
    if (a.cemb && it < nent && (long long)img * HWo < a.M && (a.cemb_uncond_from < 0 || img < a.cemb_uncond_from))
      lab[u] = a.cemb_labels[img % a.cemb_label_mod];
  }
#pragma unroll
  for (int u = 0; u < UB; ++u) {
    const int it = it0 + u * step, co = tileC + it % BM, img = img0 + it / BM;
    float x = 0.f;
    if (it < nent && co < a.Cout && (long long)img * HWo < a.M) {
      x = a.bias[co];
      if (a.temb) x += a.temb[trow + (long long)img * a.temb_img_stride + co];
      if (a.cemb) x += a.cemb[(long long)lab[u] * a.cemb_row_stride + co];
    }
    v[u] = x;
  }
}
__device__ __forceinline__ long long temb_row_of(const ConvArgs& a) {
  return a.temb ? (a.temb_tsel ? (long long)(*a.temb_tsel) * a.temb_row_stride : 0) : 0;
}

// ADDV: floats of LDS after the fp32 tile for the staged additive rows (EPI_BYTES: 16 images of 128
// couts); a tile holding more images (the 2x2 / 1x1 levels: 32 / 128 images per 128-pixel tile)
// reads its rows from global memory per output chunk instead.
// PRE: the caller has already written the additive rows to LDS (E + BN * ER).
// GNO: the kernel may carry a fused consumer GroupNorm (ConvArgs gn_out; conv_small only).
template <typename T, int BM = 128, int BN = 128, int NTH = 256, int ADDV = (EPI_BYTES - 128 * EROW * 4) / 4,
          bool PRE = false, bool GNO = false>
__device__ __forceinline__ void epilogue_from_E(const ConvArgs& a, char* smem, int tileP, int tileC, int phase,
                                                const f32x4* gn_affine = nullptr);

// accumulators (waves 0..3, 2x2 of 64x64) -> fp32 tile E[pixel][cout] in LDS
__device__ __forceinline__ void acc_to_E(f32x16 (&acc)[2][2], float* E, int pbase) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = (wid >> 1) & 1, wn = wid & 1, rl = lane & 31, hh = lane >> 5;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 v4 = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        *(f32x4*)(E + (pbase + wn * 64 + j * 32 + rl) * EROW + wm * 64 + i * 32 + 8 * g + 4 * hh) = v4;
      }
}

// gamma / beta of the 8 output channels thread tid stores in gn_out_from_E (BM / 8 chunks a row)
template <int BM>
__device__ __forceinline__ void gn_affine_of(const ConvArgs& a, int tileC, f32x4 (&gam)[2], f32x4 (&bet)[2]) {
  const int co = tileC + (threadIdx.x % (BM / 8)) * 8;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const bool ok = a.gn_out && co < a.Cout;
    gam[q] = ok ? *(const f32x4*)(a.go_gamma + co + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    bet[q] = ok ? *(const f32x4*)(a.go_beta + co + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// The consumer GroupNorm(+SiLU) of a whole-image tile (ConvArgs gn_out: HWo <= 16, one statistics slot an image, every
// group's gs = Cout / 32 channels inside the tile), from E holding the rounded outputs (the statistics pass ran). The
// (image, group) statistics are gn_apply_kernel's to the bit: the per-channel slot sums in the statistics pass's order
// (float sum, fmaf square sum over the slot's pixels), eight fp64 partials -- partial l adds channels l, l + 8, .. in
// order, as lane l8 = l of gn_apply's 8-lane group -- combined in its xor-butterfly's tree ((p0+p1)+(p2+p3)) +
// ((p4+p5)+(p6+p7)), mean / rstd rounded to float; here one thread per (image, group), so the finalize is one short
// pass instead of gn_apply's shuffle rounds. The outputs get gn_apply's coefficient expressions: silu(x (rstd gamma) +
// (beta - mean rstd gamma)), one bf16 rounding. gst: 2 floats a pair of LDS (free: the additive rows are dead after
// the output pass).
template <typename T, int BM, int BN>
__device__ __forceinline__ void gn_out_from_E(const ConvArgs& a, const float* E, float* gst, int tileP, int tileC,
                                              const f32x4 (&gam)[2], const f32x4 (&bet)[2]) {
  constexpr int ER = BM + 4, EPC = 16 / (int)sizeof(T), CPR = BM / EPC;
  static_assert(EPC == 8, "bf16 chunks");
  const int tid = threadIdx.x, NT = blockDim.x;
  const int HWo = a.Hout * a.Wout, gs = a.Cout / 32;
  const int nimg = BN / HWo, ngrp = BM / gs, npairs = nimg * ngrp;
  const int img0 = tileP / HWo;
  // this thread's output chunk columns (the same for every row it stores: NT % CPR == 0), whose gamma / beta the
  // kernel loaded before its K loop (gn_affine_of)
  const int cl = (tid % CPR) * EPC, co = tileC + cl;
  // (no barrier here: the statistics pass's own barrier -- host: a.stats -- already follows the output pass's last
  // reads of the additive rows)
  for (int pr = tid; pr < npairs; pr += NT) {
    const int il = pr / ngrp, gl = pr - il * ngrp;
    if ((img0 + il) * HWo >= a.M) continue;
    double ps[8], pq[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      ps[l] = 0.0;
      pq[l] = 0.0;
      for (int k = l; k < gs; k += 8) {
        const int c = gl * gs + k;
        float sum = 0.f, sq = 0.f;
        for (int j = 0; j < HWo; ++j) {
          const float v = E[(il * HWo + j) * ER + c];
          sum += v;
          sq = fmaf(v, v, sq);
        }
        ps[l] += (double)sum;
        pq[l] += (double)sq;
      }
    }
    const double sd = ((ps[0] + ps[1]) + (ps[2] + ps[3])) + ((ps[4] + ps[5]) + (ps[6] + ps[7]));
    const double qd = ((pq[0] + pq[1]) + (pq[2] + pq[3])) + ((pq[4] + pq[5]) + (pq[6] + pq[7]));
    const double En = (double)gs * HWo;
    const double mean = sd / En;
    double var = qd / En - mean * mean;
    var = var > 0.0 ? var : 0.0;
    gst[2 * pr] = (float)mean;
    gst[2 * pr + 1] = (float)(1.0 / sqrt(var + (double)1e-5f));
  }
  // LDS writes drained, then the block barrier alone (a __syncthreads would also wait for the gamma / beta loads)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // (keeps the gst reads below the barrier)
  if (co >= a.Cout) return;
  for (int pl = tid / CPR; pl < BN; pl += NT / CPR) {
    const int p = tileP + pl;
    if (p >= a.M) break;
    const int il = pl / HWo;
    u32x4 y;
    T* ye = (T*)&y;
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      const int pr = il * ngrp + (cl + e) / gs;
      const float sc = gst[2 * pr + 1] * gam[e >> 2][e & 3];
      const float c0 = sc, c1 = bet[e >> 2][e & 3] - gst[2 * pr] * sc;
      float v = E[pl * ER + cl + e] * c0 + c1;  // (E: the rounded outputs, host: a.stats)
      if (a.go_silu) v = silu(v);
      ye[e] = Elem<T>::to(v);
    }
    *(u32x4*)((T*)a.gn_out + (size_t)p * a.Cout + co) = y;
  }
}

template <typename T>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x16 (&acc)[2][2], char* smem, int tileP,
                                              int tileC, int phase = -1) {
  if (threadIdx.x < 256) acc_to_E(acc, (float*)smem, 0);
  __syncthreads();
  epilogue_from_E<T>(a, smem, tileP, tileC, phase);
}

// E (128 pixels x 128 couts, fp32, barrier passed) -> outputs (+ bias/temb/cemb/resid),
// and the consumer GroupNorm's statistics slab.
template <typename T, int BM, int BN, int NTH, int ADDV, bool PRE, bool GNO>
__device__ __forceinline__ void epilogue_from_E(const ConvArgs& a, char* smem, int tileP, int tileC, int phase,
                                                const f32x4* gn_affine) {
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int ER = BM + 4;  // E row (floats): 128x128 tile -> EROW
  const int NT = blockDim.x;
  const int tid = threadIdx.x;
  const int HWo = a.Hout * a.Wout;
  float* E = (float*)smem;
  // output row of tile-space pixel p (sub-pixel phase convs write a 2x grid)
  auto orow = [&](int p) -> size_t {
    if (phase < 0) return (size_t)p;
    const int img = p / HWo, rem = p - img * HWo, i = rem / a.Wout, j = rem - i * a.Wout;
    return ((size_t)img * 2 * a.Hout + 2 * i + (phase >> 1)) * (2 * a.Wout) + 2 * j + (phase & 1);
  };
  if (a.vt_out && tileC >= a.vt_from) {
    // channel-major store of this (whole-V) tile: vt[img][c][pixel], 16-B chunks of
    // consecutive pixels of one image (host: HWo % EPC == 0, vt_from % 128 == 0); + bias only.
    // lanes take consecutive channels (the 8 column reads of a chunk hit 64 banks once: the
    // pixel-major order read 8 lanes per bank); each lane stores 8 consecutive pixels of its channel
    const int Cv = a.Cout - a.vt_from;
    for (int it = tid; it < BM * (BN / EPC); it += NT) {
      const int cl = it % BM, pl = (it / BM) * EPC;
      const int co = tileC + cl, p = tileP + pl;
      if (co >= a.Cout || p >= a.M) continue;
      const int img = p / HWo, pi = p - img * HWo;
      const float bb = a.bias[co];
      u32x4 w;
      T* we = (T*)&w;
#pragma unroll
      for (int e = 0; e < EPC; ++e) we[e] = Elem<T>::to(E[(pl + e) * ER + cl] + bb);
      *(u32x4*)((T*)a.vt_out + ((size_t)img * Cv + (co - a.vt_from)) * HWo + pi) = w;
    }
    return;
  }
  // Additive vectors bias + temb row + CFG cond row per (image of the tile, cout),
  // staged once in LDS (the statistics scratch R, free until the statistics pass).
  // Host: the tile's pixels span whole images (HWo % 128 == 0) or 128 % HWo == 0.
  float* addv = E + BN * ER;  // [images of the tile][BM]
  const int img0 = tileP / HWo;
  const int nimt = HWo >= BN ? 1 : BN / HWo;
  const bool staged = nimt * BM <= ADDV;
  const long long trow0 = temb_row_of(a);
  if (staged && !PRE) {
    // 8 entries per thread per batch, every load of a batch issued before the first use (the
    // CFG model's 2x2 / 1x1 tiles hold 32 / 64 images: one dependent label -> cond-row round trip
    // per entry in a plain loop was ~12 us of a ~15 us conv)
    constexpr int UB = 8;
    const int nent = nimt * BM;
    for (int it0 = tid; it0 < nent; it0 += UB * NT) {
      float v[UB];
      addv_batch<BM, UB>(a, tileC, img0, HWo, nent, trow0, it0, NT, v);
#pragma unroll
      for (int u = 0; u < UB; ++u)
        if (it0 + u * NT < nent) addv[it0 + u * NT] = v[u];
    }
  }
  constexpr int CPR = BM / EPC;  // 16-B output chunks per tile row
  const int cl = (tid % CPR) * EPC, co = tileC + cl;
  const int RPI = NT / CPR;       // rows per pass
  constexpr int MAXR = (BN * CPR + NTH - 1) / NTH;  // NTH = blockDim.x
  // residual rows first: all loads in flight before the first use
  u32x4 rres[MAXR];
  if (a.resid) {
#pragma unroll
    for (int k = 0; k < MAXR; ++k) {
      const int pl = tid / CPR + k * RPI;
      const int p = tileP + pl;
      rres[k] = (pl < BN && p < a.M && co < a.Cout && !(a.dbg & 256))
                    ? *(const u32x4*)((const T*)a.resid + orow(p) * a.Cout + co)
                    : u32x4{0u, 0u, 0u, 0u};
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < MAXR; ++k) {
    const int pl = tid / CPR + k * RPI;
    const int p = tileP + pl;
    if (pl >= BN || p >= a.M || co >= a.Cout) continue;
    float v[EPC];
    if (staged) {
      const float* av = addv + (HWo >= BN ? 0 : pl / HWo) * BM + cl;
#pragma unroll
      for (int q = 0; q < EPC / 4; ++q) {
        const f32x4 e4 = *(const f32x4*)(E + pl * ER + cl + 4 * q);
        const f32x4 b4 = *(const f32x4*)(av + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = e4[e] + b4[e];
      }
    } else {  // the chunk's EPC additive values straight from the bias / temb / cond rows
      const int img = p / HWo;
      int lab = 0;
      if (a.cemb && (a.cemb_uncond_from < 0 || img < a.cemb_uncond_from)) lab = a.cemb_labels[img % a.cemb_label_mod];
#pragma unroll
      for (int q = 0; q < EPC / 4; ++q) {
        const f32x4 e4 = *(const f32x4*)(E + pl * ER + cl + 4 * q);
        f32x4 b4 = *(const f32x4*)(a.bias + co + 4 * q);
        if (a.temb) b4 += *(const f32x4*)(a.temb + trow0 + (long long)img * a.temb_img_stride + co + 4 * q);
        if (a.cemb) b4 += *(const f32x4*)(a.cemb + (long long)lab * a.cemb_row_stride + co + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = e4[e] + b4[e];
      }
    }
    if (a.resid) {
      const T* re = (const T*)&rres[k];
#pragma unroll
      for (int e = 0; e < EPC; ++e) v[e] += Elem<T>::tof(re[e]);
    }
    u32x4 w;
    T* we = (T*)&w;
#pragma unroll
    for (int e = 0; e < EPC; ++e) we[e] = Elem<T>::to(v[e]);
    if (!(a.dbg & 32)) *(u32x4*)((T*)a.out + orow(p) * a.Cout + co) = w;
    if (a.stats) {
#pragma unroll
      for (int q = 0; q < EPC / 4; ++q) {
        f32x4 s4;
#pragma unroll
        for (int e = 0; e < 4; ++e) s4[e] = Elem<T>::tof(we[4 * q + e]);
        *(f32x4*)(E + pl * ER + cl + 4 * q) = s4;
      }
    }
  }
  if (a.stats && !(a.dbg & 128)) {
    __syncthreads();
    const int Gt = stat_slot_px(HWo);  // host guarantees 128 % HWo == 0 or HWo % 128 == 0
    const int S = BN / Gt;
    if (Gt >= 16) {
      // pass 1: BN/16 groups of 16 pixel rows x BM/4 channel quads, 16-B LDS reads
      float* R = E + BN * ER;  // [BN/16 groups][2][BM]
      if (tid < (BN / 16) * (BM / 4)) {
        const int cq = tid % (BM / 4), pg = tid / (BM / 4);
        f32x4 s4 = {0.f, 0.f, 0.f, 0.f}, q4 = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < 16; ++k) {
          const int pl = pg * 16 + k;
          if (tileP + pl < a.M) {
            const f32x4 v = *(const f32x4*)(E + pl * ER + 4 * cq);
            s4 += v;
            q4 += v * v;
          }
        }
        *(f32x4*)(R + (pg * 2) * BM + 4 * cq) = s4;
        *(f32x4*)(R + (pg * 2 + 1) * BM + 4 * cq) = q4;
      }
      __syncthreads();
      // pass 2: groups -> slots in fixed order (deterministic); an item = 4 consecutive couts of a slot
      // (16-B reads and stores, the per-channel sums unchanged; host: Cout % 4 == 0)
      const int gps = Gt / 16;
      for (int item = tid; item < S * (BM / 4); item += NT) {
        const int s = item / (BM / 4), cl = (item % (BM / 4)) * 4;
        const int co = tileC + cl, p0 = tileP + s * Gt;
        if (co >= a.Cout || p0 >= a.M) continue;
        f32x4 sum = {0.f, 0.f, 0.f, 0.f}, sq = {0.f, 0.f, 0.f, 0.f};
        for (int g = s * gps; g < (s + 1) * gps; ++g) {
          sum += *(const f32x4*)(R + (g * 2) * BM + cl);
          sq += *(const f32x4*)(R + (g * 2 + 1) * BM + cl);
        }
        // sub-pixel phases: spp slots per phase image (one when the phase image is below a slot)
        const int spp = HWo >= 128 ? HWo / 128 : 1;
        const long long slot = phase < 0 ? p0 / Gt : (long long)(p0 / HWo) * 4 * spp + phase * spp + (p0 % HWo) / Gt;
        *(f32x4*)(a.stats + (slot * 2) * a.Cout + co) = sum;
        *(f32x4*)(a.stats + (slot * 2 + 1) * a.Cout + co) = sq;
      }
    } else {
      // items (slot, 4 consecutive couts): 16-B column reads of E and 16-B stores of the 4 sums and the
      // 4 square sums (the per-channel arithmetic of one item per cout; host: Cout % 4 == 0)
      for (int item = tid; item < S * (BM / 4); item += NT) {
        const int s = item / (BM / 4), cl = (item % (BM / 4)) * 4;
        const int co = tileC + cl, p0 = tileP + s * Gt;
        if (co >= a.Cout || p0 >= a.M) continue;
        f32x4 sum = {0.f, 0.f, 0.f, 0.f}, sq = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < Gt; ++k) {
          const f32x4 v = *(const f32x4*)(E + (s * Gt + k) * ER + cl);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sum[e] += v[e];
            sq[e] = fmaf(v[e], v[e], sq[e]);
          }
        }
        const int spp = HWo >= 128 ? HWo / 128 : 1;
        const long long slot = phase < 0 ? p0 / Gt : (long long)(p0 / HWo) * 4 * spp + phase * spp + (p0 % HWo) / Gt;
        *(f32x4*)(a.stats + (slot * 2) * a.Cout + co) = sum;
        *(f32x4*)(a.stats + (slot * 2 + 1) * a.Cout + co) = sq;
      }
    }
  }
  if constexpr (GNO) {  // (gn_affine: gamma[0..1], beta[2..3] of the thread's 8 channels, gn_affine_of)
    if (a.gn_out)
      gn_out_from_E<T, BM, BN>(a, E, E + BN * ER, tileP, tileC, *(const f32x4(*)[2])gn_affine,
                               *(const f32x4(*)[2])(gn_affine + 2));
  }
}

__device__ __forceinline__ void zero_acc(f32x16 (&acc)[2][2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
}

// ---------------------------------------------------------------------------- split-K
// In-launch split-K combine (MI355X guide, "In-launch split-K reduction"): every slice
// writes its fp32 partial tile (thread-native layout, 16-B stores), drains, and one
// lane releases (agent scope) then takes a ticket; the block drawing S-1 acquires,
// resets the ticket for the next launch, and sums all partials in slice order 0..S-1
// (its own from registers) -- bit-identical whichever slice arrives last -- then runs
// the fused epilogue. Correct for any placement of the slices over XCDs.
struct TileId {
  int x, y, z;
};

// Bijective XCD-aware remap (MI355X guide T1): the dispatcher deals linear block ids
// round-robin over the 8 XCDs, so XCD (b % 8) is given the contiguous tile-id range
// [start, start + count) of the cout-major order t = (z*gy + y)*gx + x. Blocks that
// share a cout tile (its weights) then share one L2 -- at the 8x8 / 4x4 levels the
// weight matrices (up to 9.4 MB) do not fit one 4 MB L2 if every XCD needs all of them.
// Speed only: correctness never depends on placement.
// (A cout-major order -- an XCD's range = a band of cout tiles x every pixel tile -- for the weight-heavy
// CFG 4x4 / 8x8 conv_pipe launches measured no faster: profiles/r04/census_archC_2N64_wmajor.txt)
__device__ __forceinline__ TileId tile_of_block(bool pixel_major = false) {
  const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  const int B = gx * gy * gz;
  const int b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int xcd = b & 7, q = B >> 3, r = B & 7;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  TileId id;
  if (pixel_major) {  // t = (x * gz + z) * gy + y: an XCD's range = a band of pixel tiles x every (cout, z)
    id.y = t % gy;
    id.z = (t / gy) % gz;
    id.x = t / (gy * gz);
  } else {
    id.x = t % gx;
    id.y = (t / gx) % gy;
    id.z = t / (gx * gy);
  }
  return id;
}

// Padding rows are DMA'd from a zero region. One shared 16-B source would put every
// padded row of every CU on the same L2 channel (at the 4x4 level ~1/3 of all taps are
// padding); each block reads its own 4-KiB-spaced slot of a 256-KiB region instead.
template <typename T>
__device__ __forceinline__ const T* zero_of_block(const ConvArgs& a) {
  const int b = blockIdx.x + 7 * blockIdx.y + 13 * blockIdx.z;
  return (const T*)((const char*)a.zero + (b & 63) * 4096);
}

// Split-K (under-filled grids): slice z of a tile writes its raw fp32 accumulators to
// slab[tile][z][thread][64] and exits; splitk_epilogue_kernel (next launch on the stream,
// so no cross-XCD fences) sums the slices in slice order -- deterministic -- and runs
// the shared epilogue. Slab index of a tile: y * gridDim.x + x.
__device__ __forceinline__ void splitk_store(const ConvArgs& a, f32x16 (&acc)[2][2], int z, int S, const TileId& bt,
                                             int gx) {
  const long long tile = (long long)bt.y * gx + bt.x;
  float* mine = a.splitk_ws + ((size_t)tile * S + z) * 16384 + threadIdx.x * 64;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        *(f32x4*)(mine + (i * 2 + j) * 16 + 4 * g) = v;
      }
}

// ---------------------------------------------------------------------------- pipelined
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Same wait as a real S_WAITCNT the compiler sees (it then knows which loads retired and
// needs no conservative vmcnt(0) of its own). gfx9 encoding: vmcnt[3:0|15:14],
// expcnt[6:4] = 7, lgkmcnt[11:8] = 15 (no wait on those).
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

template <typename T, int NS, bool LIN>
__global__ __launch_bounds__(256, (NS <= 2 ? 2 : 1)) void conv_pipe(ConvArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int BK = 8 * EPC;
  constexpr int STAGE = 2 * TILEB;
  __shared__ __attribute__((aligned(16))) char smem[(NS * STAGE > EPI_BYTES) ? NS * STAGE : EPI_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1, rl = lane & 31, hh = lane >> 5;
  // pixel-tile-major over the XCDs: each XCD's L2 keeps its band of input rows for every cout tile and
  // sub-pixel phase / K slice (measured: 16x16-level plain convs -5 %, N = 256 forward -1.2 %)
  const TileId bt = tile_of_block(true);
  const int tileP = bt.x * CONV_BN, tileC = bt.y * CONV_BM;
  const int Cin = a.C1 + a.C2;
  const int cpt = Cin / BK;  // K-chunks per tap
  const int nK = a.ksize * a.ksize * cpt;
  const int HWo = a.Hout * a.Wout;
  // sub-pixel phase: (subpix 1, nearest-x2 upsample convs) 2x2 taps at input offsets (dy + py - 1,
  // dx + px - 1); (subpix 2, CFG ConvTranspose2d(5, 2, 2, 1)) 3x3 taps at (dy - 1, dx - 1) for every phase
  // (sub-pixel launches: z = phase + 4 x K slice)
  const int phase = a.subpix ? (bt.z & 3) : -1;
  const int padY = a.subpix == 1 ? 1 - (phase >> 1) : a.pad, padX = a.subpix == 1 ? 1 - (phase & 1) : a.pad;
  const T* wbase = (const T*)a.wt + (a.subpix ? (size_t)phase * a.Cout * a.K : 0);
  const int Hv = a.upsample ? 2 * a.Hin : (a.zins ? 2 * a.Hin - 1 : a.Hin);
  const int Wv = a.upsample ? 2 * a.Win : (a.zins ? 2 * a.Win - 1 : a.Win);
  const T* zero = zero_of_block<T>(a);

  // This lane's DMA rows: instruction q of wave w fills rows 8*(4w+q) .. +7 (1 KiB);
  // lane L lands at row 8*(4w+q) + L/8, slot L%8, so it must fetch logical chunk
  // (L%8) ^ ((row>>1)&7) (the read-side swizzle applied to the source).
  // Per-lane gather state, computed once: the weight row pointer, and for the pixel
  // row a bitmask of the taps that land inside the (virtual) input plus, per tap, a
  // 32-bit element offset = pixel term (per lane) + tap term (per stage, scalar).
  // Nearest-x2 upsample / zero-insertion make the pixel term tap-dependent, so those
  // layers keep a per-tap row/column table instead (rowt/colt: -1 = padding).
  const T* arow[4];
  int pix1[4], pix2[4];  // element offset of (iy0, ix0) in src1 / src2, + chunk
  unsigned tmask[4];
  int rowt[4][5], colt[4][5], chk[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 8 * (4 * wid + q) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int co = tileC + r;
    arow[q] = wbase + (size_t)(co < a.Cout ? co : 0) * a.K + c * EPC;
    if (co >= a.Cout) arow[q] = nullptr;
    const int p = tileP + r;
    const bool pv = p < a.M;
    const int img = p / HWo;
    const int rem = p - img * HWo;
    const int oy = rem / a.Wout;
    const int iy0 = oy * a.stride - padY;
    const int ix0 = (rem - oy * a.Wout) * a.stride - padX;
    const int pl = (img * a.Hin + iy0) * a.Win + ix0;
    pix1[q] = pl * a.C1 + c * EPC;
    pix2[q] = pl * a.C2 + c * EPC;
    unsigned m = 0;
    for (int ky = 0; ky < a.ksize; ++ky)
      for (int kx = 0; kx < a.ksize; ++kx) {
        const int iy = iy0 + ky, ix = ix0 + kx;
        bool ok = pv && iy >= 0 && iy < Hv && ix >= 0 && ix < Wv;
        if (a.zins) ok = ok && !((iy | ix) & 1);
        if (ok) m |= 1u << (ky * a.ksize + kx);
      }
    tmask[q] = m;
    chk[q] = c * EPC;
    if constexpr (!LIN) {
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        rowt[q][k] = (img * a.Hin + ((iy0 + k) >> 1)) * a.Win;
        colt[q][k] = (ix0 + k) >> 1;
      }
    }
  }

  auto issue = [&](int kc) {
    const int tap = kc / cpt;
    const int ci0 = (kc - tap * cpt) * BK;
    const int ky = tap / a.ksize, kx = tap - (tap / a.ksize) * a.ksize;
    char* sA = smem + (kc % NS) * STAGE;
    char* sB = sA + TILEB;
    const bool s1 = ci0 < a.C1;
    const T* src = s1 ? (const T*)a.src1 : (const T*)a.src2;
    const int Cs = s1 ? a.C1 : a.C2;
    const int cs0 = s1 ? ci0 : ci0 - a.C1;
    const int toff = (ky * a.Win + kx) * Cs + cs0;  // scalar tap term
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const T* ga = arow[q] ? arow[q] + (size_t)kc * BK : zero;
      __builtin_amdgcn_global_load_lds((const void*)ga, (lds_ptr_t)(sA + (4 * wid + q) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int off;
      if constexpr (LIN) off = (s1 ? pix1[q] : pix2[q]) + toff;
      else off = (rowt[q][ky] + colt[q][kx]) * Cs + cs0 + chk[q];
      const T* gb = ((tmask[q] >> tap) & 1u) ? src + off : zero;
      __builtin_amdgcn_global_load_lds((const void*)gb, (lds_ptr_t)(sB + (4 * wid + q) * 1024), 16, 0, 0);
    }
  };

  f32x16 acc[2][2];
  zero_acc(acc);
  // split-K: slice z covers K-stages [k0, k1) (sub-pixel launches: gridDim.z = 4 phases x S slices)
  const int S = a.subpix ? (int)(gridDim.z >> 2) : (int)gridDim.z, z = a.subpix ? (bt.z >> 2) : bt.z;
  const int k0 = (int)((long long)nK * z / S), k1 = (int)((long long)nK * (z + 1) / S);
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (k0 + s < k1) issue(k0 + s);
  for (int kc = k0; kc < k1; ++kc) {
    // stage kc must have landed: keep the younger in-flight stages (8 DMA each) pending
    const int ahead = min(NS - 2, k1 - 1 - kc);
    if (ahead >= 2) wait_vmcnt<16>();
    else if (ahead == 1) wait_vmcnt<8>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (kc + NS - 1 < k1 && !(a.dbg & 1)) issue(kc + NS - 1);
    const char* A = smem + (kc % NS) * STAGE;
    if (!(a.dbg & 2)) mma_stage<T>(A, A + TILEB, acc, wm, wn, rl, hh);
  }
  wait_vmcnt<0>();
  __syncthreads();
  if (S > 1) {
    if (!a.tickets) {  // (host: tile count above the ticket capacity) splitk_epilogue_kernel combines
      splitk_store(a, acc, z, S, bt, gridDim.x);
      return;
    }
    // in-launch combine (conv_small's hand-off): write-through partial [tile][z][16 x 4 KB rows],
    // drained by every wave; the slice drawing ticket S-1 sums slices 0..S-1 in order
    const __amdgpu_buffer_rsrc_t slab = __builtin_amdgcn_make_buffer_rsrc(
        a.splitk_ws, (short)0, (int)std::min<long long>(a.splitk_cap * 4, 0x7fffffffLL), 0x00020000);
    const int tile = ((a.subpix ? phase : 0) * gridDim.y + bt.y) * gridDim.x + bt.x;  // (host: tickets for all)
    const uint32_t base = (uint32_t)((size_t)tile * S * 65536) + threadIdx.x * 16;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const f32x16& v = acc[q >> 3][(q >> 2) & 1];
      const int g = q & 3;
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{__float_as_uint(v[4 * g]), __float_as_uint(v[4 * g + 1]), __float_as_uint(v[4 * g + 2]),
                __float_as_uint(v[4 * g + 3])},
          slab, base + z * 65536 + q * 4096, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = (int*)smem;
    if (threadIdx.x == 0)
      flag[0] = __hip_atomic_fetch_add(a.tickets + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (flag[0] != S - 1) return;  // another slice finishes this tile (uniform over the block)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // (no instruction: keeps the loads below the ticket)
    if (threadIdx.x == 0) __hip_atomic_store(a.tickets + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int sl = 0; sl < S; ++sl) {  // (one slice's 16 loads in flight: registers beside acc)
      u32x4 w[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) w[q] = __builtin_amdgcn_raw_buffer_load_b128(slab, base + sl * 65536 + q * 4096, 0, 16);
#pragma unroll
      for (int q = 0; q < 16; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = acc[q >> 3][(q >> 2) & 1][4 * (q & 3) + e];
          acc[q >> 3][(q >> 2) & 1][4 * (q & 3) + e] = sl == 0 ? __uint_as_float(w[q][e]) : d + __uint_as_float(w[q][e]);
        }
    }
    __syncthreads();  // flag read by every wave before the epilogue reuses the LDS
  }
  if (a.dbg & 16) return;
  conv_epilogue<T>(a, acc, smem, tileP, tileC, phase);
}

// ---------------------------------------------------------------------------- small tiles
// The 8x8 / 4x4 / 2x2 / 1x1 levels (M = n * HWo <= 64 n): 128 x 128 tiles leave most of
// the 256 CUs idle (4x4 level, n = 256: 128 tiles), and split-K buys the parallelism
// back with an fp32 partial round trip and a second launch. A 64 couts x 64 pixels tile
// gives 4x the blocks with the whole K in one block: 4 waves in 2x2, each one 32x32
// v_mfma_f32_32x32x16_bf16 accumulator; LDS images [64 rows][128 B] (same swizzle), a
// 4-deep global_load_lds ring (16 KB per stage, 3 stages in flight), 2 blocks per CU.
// The epilogue is the shared one at 64 x 64 (host: 64 % HWo == 0, so a tile holds whole
// images and whole GroupNorm statistics slots).
// Split K (gridDim.z = S > 1: the 2x2 / 1x1 levels and small batches, where M / 64 x Cout / 64
// is a handful of tiles streaming megabytes of weights): slice z runs K-chunks
// [z nK / S, (z+1) nK / S) and hands its 64 x 64 fp32 partial to the last-arriving slice of
// the tile (the p5 hand-off: sc1 stores, drain, ticket), which sums the S partials in slice
// order -- bit-identical whichever slice arrives last -- and runs the epilogue.
constexpr int SM_B = 64;                    // couts and pixels per small tile
constexpr int SM_TILEB = SM_B * ROWB;       // 8 KB
constexpr int SM_NS = 4;
constexpr int SM_EPI = SM_B * (SM_B + 4) * 4 + SM_B * SM_B * 4;  // E + (addv | statistics groups)
constexpr int SM_SMEM = (SM_NS * 2 * SM_TILEB > SM_EPI) ? SM_NS * 2 * SM_TILEB : SM_EPI;

// TAPIN: the K loop runs the taps inside each 64-channel chunk (K-chunk kc = chunk * taps + tap)
// instead of the weight layout's tap-major order: a chunk's input rows are re-read by the 9 taps
// in 9 consecutive stages (L2 / L1 hits) instead of once per tap sweep over the whole Cin (a reuse
// distance of Cin/64 stages x every resident block's rows: ~4 MiB per XCD at the 4x4 level, N = 256)
template <bool TAPIN>
__global__ __launch_bounds__(256, 2) void conv_small(ConvArgs a) {
  typedef bf16_t T;
  constexpr int BK = 64, STAGE = 2 * SM_TILEB;
  __shared__ __attribute__((aligned(16))) char smem[SM_SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1, rl = lane & 31, hh = lane >> 5;
  const TileId bt = tile_of_block();
  const int tileP = bt.x * SM_B, tileC = bt.y * SM_B;
  const int Cin = a.C1 + a.C2, cpt = Cin / BK, nK = a.ksize * a.ksize * cpt;
  const int HWo = a.Hout * a.Wout;
  const T* zero = zero_of_block<T>(a);
  // DMA rows: instruction q of wave w fills rows 8*(2w+q) .. +7 of the A and B images
  const T* arow[2];
  int pix1[2], pix2[2];
  unsigned tmask[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 8 * (2 * wid + q) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int co = tileC + r;
    arow[q] = co < a.Cout ? (const T*)a.wt + (size_t)co * a.K + c * 8 : nullptr;
    const int p = tileP + r;
    const bool pv = p < a.M;
    const int img = p / HWo, rem = p - img * HWo, oy = rem / a.Wout;
    const int iy0 = oy * a.stride - a.pad, ix0 = (rem - oy * a.Wout) * a.stride - a.pad;
    const int pl = (img * a.Hin + iy0) * a.Win + ix0;
    pix1[q] = pl * a.C1 + c * 8;
    pix2[q] = pl * a.C2 + c * 8;
    unsigned m = 0;
    for (int ky = 0; ky < a.ksize; ++ky)
      for (int kx = 0; kx < a.ksize; ++kx) {
        const int iy = iy0 + ky, ix = ix0 + kx;
        if (pv && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win) m |= 1u << (ky * a.ksize + kx);
      }
    tmask[q] = m;
  }
  // the tile's additive rows (<= 64 images x 64 couts: <= 16 entries a thread), loaded before the K
  // loop so their label -> cond-row round trips overlap it (the 2x2 / 1x1 levels' tiles hold 16-64
  // images); written to LDS after the loop (epilogue_from_E<..., PRE>)
  float pre[16];
  {
    const int nent = (HWo >= SM_B ? 1 : SM_B / HWo) * SM_B;
    const long long trow = temb_row_of(a);
    float v0[8], v1[8];
    addv_batch<SM_B, 8>(a, tileC, tileP / HWo, HWo, nent, trow, tid, 256, v0);
    addv_batch<SM_B, 8>(a, tileC, tileP / HWo, HWo, nent, trow, tid + 2048, 256, v1);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      pre[u] = v0[u];
      pre[8 + u] = v1[u];
    }
  }
  // the fused consumer GroupNorm's affine (gn_out), loaded with the additive rows
  f32x4 gnab[4];
  gn_affine_of<SM_B>(a, tileC, *(f32x4(*)[2])gnab, *(f32x4(*)[2])(gnab + 2));
  const int ntap = a.ksize * a.ksize;
  const int S = gridDim.z, kc0 = bt.z * nK / S, nKs = (bt.z + 1) * nK / S - kc0;
  auto issue = [&](int kc, int slot) {
    int tap, ci0;
    if constexpr (TAPIN) {
      const int cc = kc / ntap;
      tap = kc - cc * ntap;
      ci0 = cc * BK;
    } else {
      tap = kc / cpt;
      ci0 = (kc - tap * cpt) * BK;
    }
    const int ky = tap / a.ksize, kx = tap - ky * a.ksize;
    char* sA = smem + slot * STAGE;
    char* sB = sA + SM_TILEB;
    const bool s1 = ci0 < a.C1;
    const T* src = s1 ? (const T*)a.src1 : (const T*)a.src2;
    const int toff = (ky * a.Win + kx) * (s1 ? a.C1 : a.C2) + (s1 ? ci0 : ci0 - a.C1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const T* ga = arow[q] ? arow[q] + (size_t)(tap * Cin + ci0) : zero;
      __builtin_amdgcn_global_load_lds((const void*)ga, (lds_ptr_t)(sA + (2 * wid + q) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const T* gb = ((tmask[q] >> tap) & 1u) ? src + (s1 ? pix1[q] : pix2[q]) + toff : zero;
      __builtin_amdgcn_global_load_lds((const void*)gb, (lds_ptr_t)(sB + (2 * wid + q) * 1024), 16, 0, 0);
    }
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int s = 0; s < SM_NS - 1; ++s)
    if (s < nKs) issue(kc0 + s, s);
  for (int kc = 0; kc < nKs; ++kc) {
    const int ahead = min(SM_NS - 2, nKs - 1 - kc);  // younger stages kept in flight (4 DMA each)
    if (ahead >= 2) wait_vmcnt<8>();
    else if (ahead == 1) wait_vmcnt<4>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (kc + SM_NS - 1 < nKs) issue(kc0 + kc + SM_NS - 1, (kc + SM_NS - 1) % SM_NS);
    const char* A = smem + (kc % SM_NS) * STAGE;
    const char* B = A + SM_TILEB;
    bf16x8 af[4], bf[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      af[kk] = *(const bf16x8*)(A + swz(wm * 32 + rl, 2 * kk + hh));
      bf[kk] = *(const bf16x8*)(B + swz(wn * 32 + rl, 2 * kk + hh));
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the MFMAs
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kk], bf[kk], acc, 0, 0, 0);
  }
  wait_vmcnt<0>();
  __syncthreads();
  if (S > 1) {
    // partial out (slab[tile][z][g][thread] as 16-B rows), drained by every wave before thread 0
    // takes the tile's ticket; the slice drawing S-1 resets it and sums slices 0..S-1
    const __amdgpu_buffer_rsrc_t slab = __builtin_amdgcn_make_buffer_rsrc(
        a.splitk_ws, (short)0, (int)std::min<long long>(a.splitk_cap * 4, 0x7fffffffLL), 0x00020000);
    const int tile = bt.y * gridDim.x + bt.x;
    const uint32_t base = (uint32_t)((size_t)tile * S * 16384) + tid * 16;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{__float_as_uint(acc[4 * g]), __float_as_uint(acc[4 * g + 1]), __float_as_uint(acc[4 * g + 2]),
                __float_as_uint(acc[4 * g + 3])},
          slab, base + bt.z * 16384 + g * 4096, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = (int*)smem;
    if (tid == 0) flag[0] = __hip_atomic_fetch_add(a.tickets + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (flag[0] != S - 1) return;  // another slice finishes this tile (uniform over the block)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // (no instruction: keeps the loads below the ticket)
    if (tid == 0) __hip_atomic_store(a.tickets + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // 8 slices' loads in flight per batch (one memory round trip each), summed in slice order
    for (int sl0 = 0; sl0 < S; sl0 += 8) {
      u32x4 v[8][4];
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          v[j][g] = __builtin_amdgcn_raw_buffer_load_b128(slab, base + min(sl0 + j, S - 1) * 16384 + g * 4096, 0, 16);
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (sl0 + j < S)
              acc[4 * g + e] = sl0 + j == 0 ? __uint_as_float(v[j][g][e]) : acc[4 * g + e] + __uint_as_float(v[j][g][e]);
    }
    __syncthreads();  // flag read by every wave before E overwrites it
  }
  // accumulators -> E[pixel][cout] (row SM_B + 4 floats); the additive rows after it
  float* E = (float*)smem;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    f32x4 v4 = {acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
    *(f32x4*)(E + (wn * 32 + rl) * (SM_B + 4) + wm * 32 + 8 * g + 4 * hh) = v4;
  }
  {
    const int nent = (HWo >= SM_B ? 1 : SM_B / HWo) * SM_B;
    float* addv = E + SM_B * (SM_B + 4);
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (tid + 256 * u < nent) addv[tid + 256 * u] = pre[u];
  }
  __syncthreads();
  epilogue_from_E<T, SM_B, SM_B, 256, (SM_SMEM - SM_B * (SM_B + 4) * 4) / 4, true, true>(a, smem, tileP, tileC, -1,
                                                                                          gnab);
}

// ---------------------------------------------------------------------------- streaming 1x1
// Statistics-free 1x1 convs of large pixel counts (the ResBlock shortcuts at the 32x32 / 16x16 levels
// at N = 256: K = 256..640, Cout = 128 / 256) are HBM streams (2 Cout = 256 flops per input byte,
// below the bf16 ridge): conv_pipe reloads the weights per 128x128 tile and drains its pipeline per
// tile (~45 % of HBM bandwidth). Here a persistent block keeps one 128-cout tile's weights in
// VGPRs for the whole launch (wave w: couts 32w..32w+31, all CIN as CIN/16 A fragments straight from
// the [Cout][K] rows) and streams 128-pixel tiles through an NS-stage global_load_lds ring of 64-channel
// chunks that runs across tile boundaries (the next tile's loads fly during the epilogue); the
// epilogue rounds acc + bias into an LDS tile and stores it as coalesced 16-B rows. Blocks are dealt
// XCD-major: the blocks of the cout tiles of one pixel tile share an XCD (its L2 serves the second read).
// NS ring stages (64-channel chunks of 128 pixels, 16 KB each; NS = 7: 96 KB in flight a CU)
constexpr int S1_OROW = 272;                // out-tile row bytes (128 couts bf16 + 16 B pad: 16-B aligned)
// s_waitcnt vmcnt(n) for a run-time n in {0, 4, .., N} (wave-uniform)
template <int N>
__device__ __forceinline__ void s1_wait_from(int n) {
  if constexpr (N < 0) {
    wait_vmcnt<0>();
  } else {
    if (n >= N) wait_vmcnt<N>();
    else s1_wait_from<N - 4>(n);
  }
}

template <int CIN, int S1_NS>
__global__ __launch_bounds__(256, 1) void conv1x1_stream_kernel(ConvArgs a) {
  typedef bf16_t T;
  constexpr int NK = CIN / 16, NCH = CIN / 64;
  __shared__ __attribute__((aligned(16))) char smem[S1_NS * TILEB + 128 * S1_OROW];
  char* const otile = smem + S1_NS * TILEB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, rl = lane & 31, hh = lane >> 5;
  const int nTC = a.Cout / CONV_BM, nTP = a.M / CONV_BN;
  const int G = gridDim.x, b = blockIdx.x;  // host: G % (8 nTC) == 0
  const int xcd = b & 7, j = b >> 3, tc = j % nTC, slot = (j / nTC) * 8 + xcd, GS = G / nTC;
  const int ntile = slot < nTP ? (nTP - 1 - slot) / GS + 1 : 0;
  if (ntile == 0) return;
  const int co0 = tc * CONV_BM + 32 * wid;
  // weights: A fragment of k-step s = W[co0 + rl][16 s + 8 hh .. +7]
  bf16x8 wa[NK];
#pragma unroll
  for (int s = 0; s < NK; ++s) wa[s] = *(const bf16x8*)((const T*)a.wt + (size_t)(co0 + rl) * a.K + 16 * s + 8 * hh);
  float bias[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[g][e] = a.bias[co0 + 8 * g + 4 * hh + e];
  // DMA rows: instruction q of wave w fills rows 8 (4w + q) .. +7 of a stage (lane -> row + lane / 8,
  // slot lane % 8 <- logical 16-B chunk (lane % 8) ^ ((row >> 1) & 7): swz's image)
  int roff[4], coff[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 8 * (4 * wid + q) + (lane >> 3);
    roff[q] = r;
    coff[q] = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
  }
  const int nst = ntile * NCH;  // the block's chunk sequence: tile i = slot + i GS, chunk cc
  auto issue = [&](int st) __attribute__((always_inline)) {
    const int i = st / NCH, cc = st - i * NCH, tp = slot + i * GS;
    const int ci0 = cc * 64;
    const bool s1 = ci0 < a.C1;
    const T* src = s1 ? (const T*)a.src1 : (const T*)a.src2;
    const int Cs = s1 ? a.C1 : a.C2, cs0 = s1 ? ci0 : ci0 - a.C1;
    char* dst = smem + (st % S1_NS) * TILEB;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const T* g = src + (size_t)(tp * CONV_BN + roff[q]) * Cs + cs0 + coff[q];
      __builtin_amdgcn_global_load_lds((const void*)g, (lds_ptr_t)(dst + (4 * wid + q) * 1024), 16, 0, 0);
    }
  };
#pragma unroll
  for (int st = 0; st < S1_NS - 1; ++st)
    if (st < nst) issue(st);
  f32x16 acc[4];
  for (int i = 0; i < ntile; ++i) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[jj][r] = 0.f;
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) {  // (unrolled: the weight fragments are indexed at compile time)
      const int st = i * NCH + cc;
      // stage st landed: the younger stages (4 DMA each) and, after a tile's end, its 8 output stores
      // (younger than that step's DMA) may still fly
      const int ahead = min(S1_NS - 2, nst - 1 - st);
      s1_wait_from<4 * (S1_NS - 2) + 8>(4 * ahead + (cc == 0 && i > 0 ? 8 : 0));
      __builtin_amdgcn_s_barrier();
      if (st + S1_NS - 1 < nst) issue(st + S1_NS - 1);  // (its slot was read in step st - 1)
      const char* B = smem + (st % S1_NS) * TILEB;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bf16x8 bf[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) bf[jj] = *(const bf16x8*)(B + swz(32 * jj + rl, 2 * ks + hh));
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          acc[jj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[cc * 4 + ks], bf[jj], acc[jj], 0, 0, 0);
      }
    }
    // acc (+ bias) -> bf16 out tile [pixel][128 couts]: lane (pixel 32 jj + rl), couts 8 g + 4 hh .. +3
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 w2;
        w2.x = (uint32_t)f2bf(acc[jj][4 * g] + bias[g][0]) | ((uint32_t)f2bf(acc[jj][4 * g + 1] + bias[g][1]) << 16);
        w2.y = (uint32_t)f2bf(acc[jj][4 * g + 2] + bias[g][2]) | ((uint32_t)f2bf(acc[jj][4 * g + 3] + bias[g][3]) << 16);
        *(uint2*)(otile + (32 * jj + rl) * S1_OROW + (32 * wid + 8 * g + 4 * hh) * 2) = w2;
      }
    __syncthreads();
    const int tp = slot + i * GS;
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // 128 pixels x 16 chunks of 16 B
      const int u = tid + 256 * k, pr = u >> 4, ch = u & 15;
      const u32x4 v = *(const u32x4*)(otile + pr * S1_OROW + ch * 16);
      *(u32x4*)((T*)a.out + (size_t)(tp * CONV_BN + pr) * a.Cout + tc * CONV_BM + ch * 8) = v;
    }
    // (the next tile's epilogue writes the out tile only after >= 1 more ring barrier)
  }
}
bool conv1x1_stream_ok(const ConvArgs& a);
// conv1x1_stream_kernel's grid for this conv (whole XCD rounds of every cout tile), 0 where it does not run it: >= 4
// pixel tiles a block, or (round 6) >= 1 where the 128-tile grid fills the chip by itself (N = 256's 8x8 shortcuts,
// 384 tiles on 240 blocks: 19.7 -> 15.2 us a launch, step -0.5 %, profiles/r06/stepab_s1_mint_r06aa.txt); smaller
// grids stay on conv_small's split-K path (small_wide)
static int conv1x1_stream_grid(const ConvArgs& a) {
  if (!g_conv1x1 || !conv1x1_stream_ok(a)) return 0;
  const int nTC = a.Cout / CONV_BM, nTP = a.M / CONV_BN;
  const int G = (g_num_cus / (8 * nTC)) * 8 * nTC;
  const long long tiles = (long long)nTP * nTC;
  return G > 0 && (tiles >= 4LL * G || (tiles >= G && tiles >= 256)) ? G : 0;
}
bool conv1x1_stream_ok(const ConvArgs& a) {
  const int Cin = a.C1 + a.C2;
  return a.zero && a.ksize == 1 && a.stride == 1 && a.pad == 0 && !a.subpix && !a.upsample && !a.zins && !a.gn_coef &&
         !a.stats && !a.temb && !a.cemb && !a.resid && !a.vt_out && a.C1 % 64 == 0 && a.C2 % 64 == 0 &&
         (Cin == 128 || Cin == 256 || Cin == 384 || Cin == 512 || Cin == 640) && a.K == Cin && a.Cout % CONV_BM == 0 &&
         a.M % CONV_BN == 0;
}

// Host-side eligibility of conv_small (bf16, whole 128-B K-chunks, plain stride/pad addressing).
bool conv_small_ok(const ConvArgs& a) {
  const int HWo = a.Hout * a.Wout, Cin = a.C1 + a.C2;
  // (tiles of whole images -- their statistics slots and additive rows -- or, without a consumer
  // GroupNorm, 64-pixel tiles inside one image)
  return a.zero && !a.subpix && !a.upsample && !a.zins && !a.gn_coef && Cin % 64 == 0 && a.C1 % 64 == 0 &&
         a.K == a.ksize * a.ksize * Cin && a.ksize <= 5 &&
         ((HWo <= SM_B && SM_B % HWo == 0) || (g_small_wide && !a.stats && HWo % SM_B == 0)) &&
         (!a.vt_out || HWo % 8 == 0);
}

template <typename T>
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(ConvArgs a, int S) {
  __shared__ __attribute__((aligned(16))) char smem[EPI_BYTES];
  const int tileP = blockIdx.x * CONV_BN, tileC = blockIdx.y * CONV_BM;
  const float* src = a.splitk_ws + (size_t)(blockIdx.y * gridDim.x + blockIdx.x) * S * 16384 + threadIdx.x * 64;
  f32x16 acc[2][2];
  zero_acc(acc);
  for (int z = 0; z < S; ++z, src += 16384) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = *(const f32x4*)(src + (i * 2 + j) * 16 + 4 * g);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][4 * g + e] += v[e];
        }
  }
  conv_epilogue<T>(a, acc, smem, tileP, tileC);
}

// ---------------------------------------------------------------------------- generic
template <typename T>
__global__ __launch_bounds__(256, 2) void conv_igemm(ConvArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);  // elements per 16-B chunk
  constexpr int BK = 8 * EPC;               // k per stage
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const TileId bt = tile_of_block();
  const int tileP = bt.x * CONV_BN, tileC = bt.y * CONV_BM;
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
  zero_acc(acc);
  const int rl = lane & 31, hh = lane >> 5;
  const int nK = (a.K + BK - 1) / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kc = 0; kc < nK; ++kc) {
    const int s = kc & 1;
    if (kc + 1 < nK) gload(kc + 1);
    mma_stage<T>(smem + s * 2 * TILEB, smem + s * 2 * TILEB + TILEB, acc, wm, wn, rl, hh);
    if (kc + 1 < nK) sstore(s ^ 1);
    __syncthreads();
  }
  conv_epilogue<T>(a, acc, smem, tileP, tileC);
}

// ---------------------------------------------------------------------------- fused GN + SiLU + conv3x3
// ResBlock block1/block2 (Model.py:170-174,179-184): conv3x3(silu(groupnorm(x))) with the
// GroupNorm applied while the input tile is staged, so the normalised tensor never
// exists in HBM. bf16, stride 1, pad 1, 64-channel K-chunks.
//
// Block = 4 waves (2x2 of 64x64, as conv_pipe), output tile 128 couts x 128 pixels
// (whole image rows; two 8x8 images per tile at the 8x8 level), 2 blocks per CU.
//   * prologue: the group statistics (mean, rstd) of the tile's images are reduced in
//     fp64 from the producers' statistics slabs (the finalize step of gn_apply_kernel,
//     per block: no separate launch);
//   * weights: 9 taps x (Cin/64) stages of [128 couts][64 k] (16 KB) through a 3-deep
//     global_load_lds ring (counted vmcnt + raw barrier, as conv_pipe);
//   * input: a HALO image in LDS holding the tile's rows plus a 1-pixel border,
//     [halo pixel][64 ch] bf16 with the (row>>1)&7 chunk swizzle. The 9 taps are 9
//     shifted windows of it, so each input element is loaded once per chunk instead
//     of 9 times (implicit im2col from LDS). The next chunk's halo is loaded to
//     registers at tap 0 (covered by the vmcnt budget of taps 1-2), and after tap 8
//     transformed y = silu(x*a + b) -> bf16 into the single halo buffer (padding stays
//     exactly 0: the conv pads the activated tensor). The transform is branch-free
//     (every lane writes its 7 rows; rows past the halo are scratch), which keeps the
//     compiler's own vmcnt bookkeeping exact across the chunk loop.
constexpr int GNC_ITEMS = 7;                    // halo pixels per thread (32 pixels x 8 chunks per pass)
constexpr int GNC_HALO_ROWS = GNC_ITEMS * 32;  // 224: 32x32 6x34, 16x16 10x18, 8x8 2 x 10x10 (+ scratch rows)
constexpr int GNC_NS = 3;                       // weight ring depth
constexpr int GNC_SMEM = GNC_HALO_ROWS * ROWB + GNC_NS * TILEB;
static_assert(GNC_SMEM >= EPI_BYTES, "epilogue reuses the fused conv's LDS");
static_assert(2 * GNC_SMEM <= 160 * 1024, "two blocks per CU");

// x*a + b then SiLU on two lanes of packed fp32 (v_pk_fma / v_pk_add / v_pk_mul), the
// exp and reciprocal per element (bf16 output: fast reciprocal is below its rounding)
typedef __attribute__((ext_vector_type(2))) float f32x2;
__device__ __forceinline__ f32x2 gn_silu2(f32x2 x, f32x2 sc, f32x2 sh) {
  const f32x2 y = x * sc + sh;
  f32x2 e;
  e.x = __expf(-y.x);
  e.y = __expf(-y.y);
  const f32x2 d = e + 1.0f;
  f32x2 r;
  r.x = __builtin_amdgcn_rcpf(d.x);
  r.y = __builtin_amdgcn_rcpf(d.y);
  return y * r;
}

// NSEG = images per tile (1: 16x16 and larger, 2: 8x8).
template <int NSEG>
__global__ __launch_bounds__(256, 2) void conv3x3_gn_kernel(ConvArgs a) {
  typedef bf16_t T;
  __shared__ __attribute__((aligned(16))) char smem[GNC_SMEM];
  char* halo = smem;
  char* wring = smem + GNC_HALO_ROWS * ROWB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1, rl = lane & 31, hh = lane >> 5;
  const TileId bt = tile_of_block();
  const int tileP = bt.x * CONV_BN, tileC = bt.y * CONV_BM;
  const int H = a.Hout, W = a.Wout, HW = H * W, W2 = W + 2;
  const int Cin = a.C1 + a.C2, ncc = Cin / 64, nS = 9 * ncc;
  const int THs = min(H, 128 / W), HS = (THs + 2) * W2, NH = NSEG * HS;
  const int nimg = a.M / HW;
  const int img0 = tileP / HW, y0 = (tileP - img0 * HW) / W;
  const T* zero = zero_of_block<T>(a);

  // ---- per-lane addressing
  int hb[2];  // halo pixel of this lane's B columns at tap (0,0)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int pl = wn * 64 + j * 32 + rl;
    const int seg = pl / (THs * W), rem = pl - seg * THs * W, oy = rem / W;
    hb[j] = seg * HS + oy * W2 + (rem - oy * W);
  }
  int arow[4];  // element offset of this lane's weight row chunk, -1 past Cout
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 8 * (4 * wid + q) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int co = tileC + r;
    arow[q] = co < a.Cout ? co * a.K + c * 8 : -1;
  }
  const int lch = tid & 7;
  int poff[GNC_ITEMS];  // input pixel (img*H + iy)*W + ix of halo row j, or -1 (padding / scratch row)
  int hseg = 0;         // bit j: halo row j belongs to the tile's second image
#pragma unroll
  for (int j = 0; j < GNC_ITEMS; ++j) {
    const int h = (tid >> 3) + 32 * j;
    int po = -1;
    if (h < NH) {
      const int seg = h / HS, r = h - seg * HS, hy = r / W2, hx = r - hy * W2;
      const int img = img0 + seg, iy = y0 + hy - 1, ix = hx - 1;
      if (img < nimg && iy >= 0 && iy < H && ix >= 0 && ix < W) po = (img * H + iy) * W + ix;
      hseg |= (seg & 1) << j;
    }
    poff[j] = po;
  }

  // Every step issues exactly 4 weight DMAs (past the last stage: zero page into the
  // retired slot), so the vmcnt budget is the same at every step.
  auto issue_w = [&](int s) {
    const int cc = s / 9, tap = s - cc * 9;
    const int k0 = tap * Cin + cc * 64;
    char* dst = wring + (s % GNC_NS) * TILEB;
    const bool live = s < nS && (s < 2 || !(a.dbg & 1));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const T* ga = (arow[q] >= 0 && live) ? (const T*)a.wt + (unsigned)(arow[q] + k0) : zero;
      __builtin_amdgcn_global_load_lds((const void*)ga, (lds_ptr_t)(dst + (4 * wid + q) * 1024), 16, 0, 0);
    }
  };
  f32x16 acc[2][2];
  u32x4 hreg[GNC_ITEMS];
  f32x4 cf0[4], cf1[4];  // per image of the tile: a[8], b[8] of this lane's 8 channels
  // 7 + 4*NSEG vector loads per lane: the halo chunks and the lane's GN coefficients.
  // Issued as inline asm: the compiler does not count the weight DMAs (LDS-direct
  // loads) in its vmcnt scoreboard and would drain them with vmcnt(0) before the first
  // use; the explicit counted waits of the tap loop retire these loads by tap 3.
  constexpr int LPC = GNC_ITEMS + 4 * NSEG;
  auto load_chunk = [&](int cc) {
    const int ci0 = cc * 64;
    const bool s1 = ci0 < a.C1;
    const T* src = s1 ? (const T*)a.src1 : (const T*)a.src2;
    const int Cs = s1 ? a.C1 : a.C2;
    const int cs0 = (s1 ? ci0 : ci0 - a.C1) + lch * 8;
#pragma unroll
    for (int j = 0; j < GNC_ITEMS; ++j) {
      const T* p = src + (unsigned)(poff[j] * Cs + cs0);
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(hreg[j]) : "v"(poff[j] >= 0 && !(a.dbg & 64) ? p : zero) : "memory");
    }
    const f32x4* cp0 = (const f32x4*)(a.gn_coef + ((size_t)img0 * (Cin / 8) + cc * 8 + lch) * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(cf0[q]) : "v"(cp0 + q) : "memory");
    if constexpr (NSEG == 2) {
      const int img1 = min(img0 + 1, nimg - 1);
      const f32x4* cp1 = (const f32x4*)(a.gn_coef + ((size_t)img1 * (Cin / 8) + cc * 8 + lch) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(cf1[q]) : "v"(cp1 + q) : "memory");
    }
  };
  // y = silu(x*a + b); branch-free (scratch rows past the halo are written too) so
  // every loaded register is consumed here
  auto write_halo = [&]() {
#pragma unroll
    for (int j = 0; j < GNC_ITEMS; ++j) {
      const int h = (tid >> 3) + 32 * j;
      f32x4 c[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) c[q] = (NSEG == 2 && ((hseg >> j) & 1)) ? cf1[q] : cf0[q];
      u32x4 y;
      if (a.dbg & 8) {
        y = hreg[j];
      } else {
        const uint32_t* xw = (const uint32_t*)&hreg[j];
#pragma unroll
        for (int w = 0; w < 4; ++w) {  // bf16 pair -> fp32 pair -> transform -> bf16 pair
          const f32x2 x = {__uint_as_float(xw[w] << 16), __uint_as_float(xw[w] & 0xffff0000u)};
          const f32x4 av = c[w >> 1], bv = c[2 + (w >> 1)];
          const f32x2 sc = (w & 1) ? f32x2{av[2], av[3]} : f32x2{av[0], av[1]};
          const f32x2 sh = (w & 1) ? f32x2{bv[2], bv[3]} : f32x2{bv[0], bv[1]};
          const f32x2 r = gn_silu2(x, sc, sh);
          y[w] = (uint32_t)f2bf(r.x) | ((uint32_t)f2bf(r.y) << 16);
        }
      }
      const bool pad = poff[j] < 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = pad ? 0u : y[e];
      *(u32x4*)(halo + h * ROWB + ((lch ^ ((h >> 1) & 7)) << 4)) = y;
    }
  };
  auto mma_tap = [&](int s, int tap) {
    if (a.dbg & 2) return;
    const int ky = tap / 3, kx = tap - ky * 3, toff = ky * W2 + kx;
    const char* A = wring + (s % GNC_NS) * TILEB;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      bf16x8 af[2], bfg[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = *(const bf16x8*)(A + swz(wm * 64 + i * 32 + rl, 2 * kk + hh));
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int h = hb[j] + toff;
        bfg[j] = *(const bf16x8*)(halo + h * ROWB + (((2 * kk + hh) ^ ((h >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
    }
  };

  zero_acc(acc);
  load_chunk(0);
  issue_w(0);
  issue_w(1);
  wait_vmcnt<8>();  // the chunk-0 loads (older than the 8 weight DMAs)
  write_halo();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // One chunk = 9 taps. STAGE: also load + transform the next chunk's halo. The
  // staging variant runs for every chunk but the last, so along each instantiation
  // the loaded registers are consumed exactly once per iteration and the compiler's
  // own vmcnt bookkeeping stays exact (no conservative drains of the weight ring).
  auto run_chunk = [&](int cc, auto stage) {
    constexpr bool ST = decltype(stage)::value;
    const int s0 = cc * 9;
    // tap 0 (peeled): the next chunk's loads go out behind w(s0+2)
    wait_vmcnt<4>();
    __builtin_amdgcn_s_barrier();
    issue_w(s0 + 2);
    if constexpr (ST) {
      asm volatile("" ::: "memory");
      load_chunk(cc + 1);
      asm volatile("" ::: "memory");
    }
    mma_tap(s0, 0);
    // taps 1-7 as a runtime loop; loads issued after stage s: w(s+1) (4), plus the
    // next chunk's LPC while they sit in between (taps 1, 2)
#pragma unroll 1
    for (int tap = 1; tap < 8; ++tap) {
      if (ST && tap <= 2) wait_vmcnt<4 + LPC>();
      else wait_vmcnt<4>();
      __builtin_amdgcn_s_barrier();
      issue_w(s0 + tap + 2);
      mma_tap(s0 + tap, tap);
    }
    // tap 8 (peeled): its DMA is the one op the compiler can count after the chunk loads
    wait_vmcnt<4>();
    __builtin_amdgcn_s_barrier();
    issue_w(s0 + 10);
    mma_tap(s0 + 8, 8);
    if constexpr (ST) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave is done reading this chunk's halo
      write_halo();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };
  for (int cc = 0; cc + 1 < ncc; ++cc) run_chunk(cc, std::true_type{});
  run_chunk(ncc - 1, std::false_type{});
  wait_vmcnt<0>();
  __syncthreads();
  if (a.dbg & 16) return;
  conv_epilogue<T>(a, acc, smem, tileP, tileC);
}

// ---------------------------------------------------------------------------- 256-pixel tiles (persistent)
#ifdef ITSD_STAMPS
// Diagnostic build only (hipcc -DITSD_STAMPS): per-wave cycle shares of the wide fused conv's
// phases, [block % 1024][wave][phase] (the last launch to touch a slot wins). Never shipped.
__device__ unsigned long long g_stamps[1024 * 16 * 8];  // [block % 1024][wave (<16)][slot]
__device__ __forceinline__ unsigned long long stamp() {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define STAMP(var) const unsigned long long var = stamp()
#define STAMP_ADD(slot, d) st[slot] += (d)
// timeline stamps (s_memrealtime, 100 MHz, one clock for every block and launch): slot s of wave w
// (wave 1 records s_memtime instead: the shader clock over a span = its delta / wave 0's delta x 100 MHz)
__device__ __forceinline__ void tl_stamp(int slot) {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = (threadIdx.x >> 6) == 1 ? __builtin_amdgcn_s_memtime() : __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) g_stamps[((blockIdx.x & 1023) * 16 + (threadIdx.x >> 6)) * 8 + slot] = t;
  __builtin_amdgcn_sched_barrier(0);
}
#define TL(slot) tl_stamp(slot)
#else
#define TL(slot)
#define STAMP(var)
#define STAMP_ADD(slot, d)
#endif
constexpr int GNW_BN = 256;                                                   // pixels per tile
constexpr int GNW_EPI = GNW_BN * EROW * 4 + (GNW_BN / 16) * 2 * CONV_BM * 4;  // E tile + statistics groups
constexpr int GNW_SMEM = 160 * 1024;
static_assert(GNW_EPI <= GNW_SMEM, "epilogue tile");

// GroupNorm+SiLU for the halo waves (conv3x3_gn_p4_kernel; diagnostic builds: also the earlier 256-pixel kernels)
// silu(x*a + b) from coefficients prescaled by -log2(e) (a' = -a log2e, b' = -b log2e):
// t = x a' + b' = -y log2e, 2^t = e^-y, and silu(y) = y / (1 + e^-y) = t / ((1 + 2^t)(-1/ln2))
// -- fma, exp2, fma, rcp, mul: one VALU op fewer than fma, mul, exp2, add, rcp, mul
constexpr float GN_L2E = -1.44269504f;
__device__ __forceinline__ float gn_silu_l2(float x, float a2, float b2) {
  const float t = __builtin_fmaf(x, a2, b2);
  return t * __builtin_amdgcn_rcpf(__builtin_fmaf(__builtin_amdgcn_exp2f(t), GN_L2E, GN_L2E));
}
// Two packed bf16 pairs (4 channels) through gn_silu_l2, rounded back to bf16 pairs and masked
// (zm: 0 zeroes a padding row) -- the halo waves' transform as one fixed instruction stream: four
// independent chains interleaved, so no transcendental's consumer follows it directly (no
// hazard s_nop) and exp / rcp latency overlaps. The compiler, at this kernel's register
// pressure, scheduled the same work one chain at a time with a nop after every v_exp / v_rcp.
__device__ __forceinline__ void gn_silu_x4(uint32_t xa, uint32_t xb, float a0, float a1, float a2, float a3,
                                           float b0, float b1, float b2, float b3, uint32_t zm, uint32_t& ya,
                                           uint32_t& yb) {
  float t0, t1, t2, t3, e0, e1, e2, e3;
  asm volatile(
      "v_lshlrev_b32 %2, 16, %10\n\t"
      "v_and_b32 %3, 0xffff0000, %10\n\t"
      "v_lshlrev_b32 %4, 16, %11\n\t"
      "v_and_b32 %5, 0xffff0000, %11\n\t"
      "v_fma_f32 %2, %2, %12, %16\n\t"
      "v_fma_f32 %3, %3, %13, %17\n\t"
      "v_fma_f32 %4, %4, %14, %18\n\t"
      "v_fma_f32 %5, %5, %15, %19\n\t"
      "v_exp_f32 %6, %2\n\t"
      "v_exp_f32 %7, %3\n\t"
      "v_exp_f32 %8, %4\n\t"
      "v_exp_f32 %9, %5\n\t"
      "v_fma_f32 %6, %6, %21, %21\n\t"
      "v_fma_f32 %7, %7, %21, %21\n\t"
      "v_fma_f32 %8, %8, %21, %21\n\t"
      "v_fma_f32 %9, %9, %21, %21\n\t"
      "v_rcp_f32 %6, %6\n\t"
      "v_rcp_f32 %7, %7\n\t"
      "v_rcp_f32 %8, %8\n\t"
      "v_rcp_f32 %9, %9\n\t"
      "v_mul_f32 %2, %2, %6\n\t"
      "v_mul_f32 %3, %3, %7\n\t"
      "v_mul_f32 %4, %4, %8\n\t"
      "v_mul_f32 %5, %5, %9\n\t"
      "v_cvt_pk_bf16_f32 %0, %2, %3\n\t"
      "v_cvt_pk_bf16_f32 %1, %4, %5\n\t"
      "v_and_b32 %0, %0, %20\n\t"
      "v_and_b32 %1, %1, %20"
      : "=&v"(ya), "=&v"(yb), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(e0), "=&v"(e1), "=&v"(e2),
        "=&v"(e3)
      : "v"(xa), "v"(xb), "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(zm),
        "s"(GN_L2E));
}

// ---------------------------------------------------------------------------- persistent, warp-specialized
// conv3x3_gn_ws_kernel's stamps (profiles/r02_ws_stamps.txt): the MFMA waves keep the matrix pipe
// ~88 % busy while they compute, but per 64-channel chunk they then wait ~5k cycles for the halo
// waves (staging 14.5k cycles vs 10.5k of MFMA work: its 11 loads per lane are issued only when
// the chunk starts), every tile begins with a ~10k-cycle exposed first-chunk staging, and ends with
// a ~7k-cycle epilogue through a 128 KiB fp32 LDS tile. This kernel removes all three:
//   * persistent: one block per CU walks the tiles t = blockIdx.x + k * gridDim.x; the 64-channel
//     chunks of all its tiles form one stage sequence, double-buffered in LDS by stage parity;
//   * halo waves (8..11) software-pipeline the stages as conv3x3_gn_ws_kernel's do: while
//     transforming stage p they reload each item's register with stage p+1's item right after its
//     transform, so HBM latency hides behind a whole chunk; during a tile's last chunk they stage
//     the NEXT tile's first chunk and LDS-DMA this tile's residual rows into LDS (16-B units
//     XOR-swizzled by row: conflict-free 8-B reads in the accumulator layout), and with its first
//     chunk write its bias/temb rows;
//   * MFMA waves (0..7) run the epilogue straight from their accumulators: + addv + residual,
//     one rounding, 8-B stores, and the consumer GroupNorm statistics by a butterfly over the 32
//     pixel lanes -- each wave's 128 pixels are whole statistics slots and its 32 couts are its
//     own, so the statistics go straight to the slab: no LDS tile, no block barrier. Meanwhile
//     the halo waves already stage the next tile's second chunk.
// A fragments are prefetched across chunk and tile boundaries (the 6-slot ring never drains).
// Per output the MFMA sequence is conv3x3_gn_reg_kernel's.
template <int W> struct GnpCfg;
template <> struct GnpCfg<32> { static constexpr int NSEG = 1, ITEMS = 11, RES = 1; };
template <> struct GnpCfg<16> { static constexpr int NSEG = 1, ITEMS = 11, RES = 1; };
template <> struct GnpCfg<8> { static constexpr int NSEG = 4, ITEMS = 13, RES = 0; };  // LDS: residual from HBM


// ---------------------------------------------------------------------------- persistent, one MFMA wave per SIMD
// conv3x3_gn_pws_kernel's ablations (profiles/r02_pws_ablations.txt): without the B-fragment LDS
// reads a launch takes 21 % less time, without the A-fragment loads 16 % less -- the two MFMA
// waves per SIMD each read all 128 pixels' fragments of every k-step (1 KiB of LDS per MFMA)
// and hide load latency only one k-step (B) / five k-steps (A) ahead inside a 168-register
// budget. Here a 512-thread block runs 4 MFMA waves (one per SIMD, 64 couts x 128 pixels each:
// 8 MFMAs per k-step, half the B reads per MFMA, 128 accumulators in AGPRs) beside the same 4
// halo waves: 2 waves per SIMD, 256 registers each.
#ifndef ITSD_P4_M16
#define ITSD_P4_M16 2
#endif
#ifndef ITSD_P4_ZR8
#define ITSD_P4_ZR8 1  // COMPACT 16x16x32 forms: 8 zero rows (a padding lane keeps its bank slot; 0: one, A/B builds)
#endif
#ifndef ITSD_P5_SC_LAUNCH
#define ITSD_P5_SC_LAUNCH 7.5  // the standalone 1x1 launch a folded shortcut saves, in p5 chunk-times: round 5's 5 (3:
                               // r05aq A/B) + the 2.4 by which round 6 re-priced a 2-slice combine (0.6 -> 3.0), so
                               // that the folds round 5 measured faster stay chosen
#endif
#ifndef ITSD_P5_SWZ
#define ITSD_P5_SWZ 1  // conv3x3_gn_p5_kernel's per-level halo swizzle at W <= 16 (0: (h >> 1) & 7; A/B builds)
#endif
#ifndef ITSD_P4_SUBSWZ
#define ITSD_P4_SUBSWZ 1  // p4's non-compact 8x8 / 16x16 halo (sub-pixel forms) swizzled by halo coordinates (0: (h >> 1) & 7)
#endif
#ifndef ITSD_P4_HSWZ
#define ITSD_P4_HSWZ 1  // the 16x16x32 forms' halo swizzle h & 6 (0: (h >> 1) & 7, as the 32x32x16 forms; A/B builds)
#endif
constexpr int P4_RING = 6;  // A k-step slots (prefetch distance 5 k-steps = 40 MFMAs); divides the 36 k-steps
                            // of a chunk, so the slots of the next chunk's prefetched steps line up
constexpr int P4_BD = 2;    // B fragment buffers (reads P4_BD - 1 k-steps = 8 MFMAs ahead)
// AB: bit 1 (value 2) = plain conv3x3 (no GroupNorm+SiLU: the halo waves copy the input; shipped, the
// CFG UpSample's 3x3 conv, conv_p4_plain_selected); bit 7 (value 128) = a sub-pixel phase conv (plain):
// W is the INPUT grid, a tile is (phase, 256 input-grid pixels, 128 couts) with the phase's weights
// (wfrag [4 phases][Cout/32][K/16]), outputs scattered to (2i + py, 2j + px) of the 2x grid and the
// statistics slots of each (image, phase) -- 4 taps at halo offsets (dy + py, dx + px) for a nearest-x2
// upsample + conv3x3 (Model.py:121-126, the phase's 2x2 folded taps), or with bit 8 (value 256) the 9
// taps of a 3x3 window for ConvTranspose2d(5, 2, 2, 1) (ModelCondition.py:80, the phase's taps of the 5x5
// kernel) (conv_p4_sub_selected); the other bits are diagnostic ablations (ITSD_DIAG).
template <int W, int AB = 0>
__global__ __launch_bounds__(512, 1) void conv3x3_gn_p4_kernel(ConvArgs a) {
  typedef bf16_t T;
  constexpr bool SUB = (AB & 128) != 0, PLAIN = SUB || (AB & 2) != 0;
  constexpr bool SUB4 = SUB && (AB & 256) == 0;      // upsample phases: 2x2 taps; else 3x3 windows
  constexpr int NTAP = SUB4 ? 4 : 9, KST = 4 * NTAP;  // taps and 16-deep k-steps of a 64-channel chunk
  // COMPACT (round 5; tiles of whole images: the 16x16 level's one image, the 8x8 level's four, non-sub-pixel
  // forms): the halo holds only the tile's 256 interior pixels, row = tile pixel, plus one zero row that every
  // tap reading outside its image is pointed at -- 256 rows staged a stage instead of 324 / 400 (the padding
  // frame is never loaded, transformed or written), 33 KB a buffer instead of 44 / 53 KB, so the 8x8 level
  // has room for the LDS residual / output tile (RES) and its halo-wave drain instead of the register epilogue
  constexpr bool COMPACT = !SUB && (W == 8 || W == 16);
  constexpr int NSEG = GnpCfg<W>::NSEG, ITEMS = COMPACT ? 8 : GnpCfg<W>::ITEMS, RES = COMPACT ? 1 : GnpCfg<W>::RES;
  constexpr int W2 = W + 2;
  constexpr int THs = NSEG == 1 ? GNW_BN / W : W;
  constexpr int HS = (THs + 2) * W2;
  constexpr int HWs = THs * W;  // pixels of one image segment
  constexpr int TPS = 256 / NSEG, RPP = TPS / 8;
  constexpr int ZROW = GNW_BN;  // COMPACT: the zero row
  // M16: the MFMA waves on v_mfma_f32_16x16x32_bf16 (the LDS residual / output tile forms; the sub-pixel and
  // register-epilogue forms stay on 32x32x16). ITSD_P4_M16: 0 none, 1 the 32x32 level, 2 every RES form
  constexpr bool M16 = ITSD_P4_M16 >= 1 && RES && !SUB && (AB & 1) == 0 && (W == 32 || ITSD_P4_M16 >= 2);
  // (COMPACT + M16: 8 zero rows, a lane whose tap falls outside its image reads the one with its own row's residue
  // mod 8 -- its own bank slot under hswz, so the zero reads do not collide with the group's real rows -- and 8 more
  // 64 rows past them, read at the +64-row immediate offset of pixel blocks 4..7)
  constexpr int ZROWS = COMPACT ? (M16 ? (ITSD_P4_ZR8 ? 72 : 65) : 1) : 0;
  // halo row h's 16-B units are stored XOR-permuted by hswz(h). ds_read_b128 serves a wave in four 16-lane groups
  // ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, +32: MI355X_MICROARCH.md, LDS) over 16 slots of 16 B (row parity x
  // unit). The 32x32x16 B reads (lane = 32 rows x 2 halves) are conflict-free for any tap offset with
  // (h >> 1) & 7; the 16x16x32 ones (lane = 16 rows x 4 k-groups: a group holds rows +0-3 / +12-15 of one k-group
  // and +4-11 of the other) were 2-way at 3 of every 4 row offsets with it (the round-5 7x rise of
  // SQ_LDS_BANK_CONFLICT, profiles/r05/p4_lds_conflicts_r05ab.txt), and are conflict-free at every offset with
  // h & 6 (exhaustive check over offsets, groups and both half-steps: tools/halo_swizzle.py)
  auto hswz = [](int h) { return M16 && ITSD_P4_HSWZ ? (h & 6) : ((h >> 1) & 7); };
  // The non-compact halo at 8x8 / 16x16 (the sub-pixel forms' input grids): a 32-pixel block spans image rows of
  // W + 2-row pitch, so (h >> 1) & 7 left 37 % / 12 % of the 32x32x16 B reads' lanes on a taken bank slot (9.4e6
  // conflict cycles a <8, 128> / <16, 128> launch at N = 256); halo coordinates instead: unit ^ (hy + SC2 hx) & 7
  // (as conv3x3_gn_p5_kernel's halo; tools/halo_swizzle.py --p5 geometry)
  constexpr bool CSWZ = ITSD_P4_SUBSWZ && !COMPACT && !M16 && W <= 16;
  constexpr int SC1 = 1, SC2 = W <= 8 ? 2 : 1;
  // C96 (AB bit 512, 8x8 only): 96-cout tiles -- Cout = 384 gives 4 cout tiles, so N = 256's 64 pixel tiles make
  // 256 tiles for the 256 CUs instead of 192 with 128 couts (a quarter of the chip idle). Each MFMA wave holds 48
  // couts (3 16x16 blocks); the LDS output tile keeps its 64-cout halves (48 used: units 0..5 of 8)
  constexpr bool C96 = (AB & 512) != 0;
  constexpr int BM = C96 ? 96 : CONV_BM, HB = BM / 2, NCI = HB / 16;
  static_assert(!C96 || (M16 && COMPACT), "96-cout tiles: the 16x16x32 compact forms");
  constexpr int HALO = COMPACT ? (((GNW_BN + ZROWS) * ROWB + 1023) & ~1023) : NSEG * ITEMS * RPP * ROWB;
  constexpr int RESB = RES ? GNW_BN * CONV_BM * 2 : 0;  // residual tile, bf16 [256 px][128 couts]
  static_assert(COMPACT ? ITEMS * RPP == HWs : ITEMS * RPP >= HS, "halo items cover the segment");
  // (sub-pixel forms: 4 slots, dividing every phase's k-step count: 16, or 36 / 24 / 24 / 16 live)
  // (diagnostic AB bits: 64 a 4-slot A ring, 32 three B buffers; round 5 also measured the B reads in a step's first
  // four MFMA gaps and a 9-slot A ring: +1.5 / -0.7 %, both spilling, profiles/r05/p4_sched_variants.txt)
  constexpr int RING = ((AB & 64) || SUB) ? 4 : P4_RING, BD = (AB & 32) ? P4_BD + 1 : P4_BD;
  static_assert(KST % RING == 0, "ring slots repeat per chunk");
  // + gn_fold: per halo wave, the group mean / rstd of the image it stages [32 groups][2]
  __shared__ __attribute__((aligned(16))) char smem[2 * HALO + RESB + 2 * NSEG * CONV_BM * 4 + 4 * 64 * 4];
  char* const rlds = smem + 2 * HALO;
  float* const addv = (float*)(smem + 2 * HALO + RESB);  // [2 tile parities][NSEG][128]
#ifdef ITSD_STAMPS
  {  // the SIMD each wave runs on (HW_ID.SIMD_ID) -> stamp slot [block][8 + wave][1]
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (4 << 6) | (1 << 11));
    if ((threadIdx.x & 63) == 0) g_stamps[((blockIdx.x & 1023) * 16 + 8 + (threadIdx.x >> 6)) * 8 + 1] = hw;
  }
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.Hout;
  const int Cin = a.C1 + a.C2, ncc = Cin / 64, kpt = Cin >> 4;
  const int nTC = a.Cout / BM, nPT = a.M / GNW_BN, NT = (SUB ? 4 : 1) * nPT * nTC;
  // xcd: blocks are dealt round-robin over the 8 XCDs (blocks b and b + 8 share one; speed only), so logical
  // block (b % 8) * G/8 + b / 8 gives each XCD a contiguous eighth of the tile sequence: the cout tiles of a
  // pixel tile (8x8: 3 blocks) read its input through one L2 instead of three
  const int G = gridDim.x;
  const int b = (a.xcd && (G & 7) == 0) ? (int)(blockIdx.x & 7) * (G >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  // block b walks the contiguous tile range [tb0, tb0 + ntiles) (cout tile fastest): its tiles share
  // pixel tiles and images, so a gn_fold block reduces an image's statistics once for all of them
  const int tb0 = (int)(((long long)b * NT) / G);
  const int ntiles = (int)(((long long)(b + 1) * NT) / G) - tb0;
  const int nstages = ntiles * ncc;
  // tile t = ((phase * nPT) + pixel tile) * nTC + cout tile (SUB: phase slowest, so a block's contiguous
  // range keeps one phase's weights). ConvTranspose2d phases with tap_live cost 9 / 6 / 6 / 4 taps: the
  // first half of the sequence alternates phases 0 and 3 (same pixel / cout tile), the second 1 and 2, so
  // that a block's contiguous pair of tiles costs 13 or 12 taps (phase-major: 18 .. 8)
  constexpr bool CT = SUB && !SUB4;
  const int Q = nPT * nTC;
  auto tile_r = [&](int k) -> int {  // (SUB: the tile within its phase)
    const int t = tb0 + k;
    if constexpr (!SUB) return t;
    if (CT && a.tap_live) return (t - (t >= 2 * Q ? 2 * Q : 0)) >> 1;
    return t % Q;
  };
  auto tile_p = [&](int k) { return (tile_r(k) / nTC) * GNW_BN; };
  auto tile_c = [&](int k) { return (tile_r(k) % nTC) * BM; };
  auto tile_ph = [&](int k) -> int {
    const int t = tb0 + k;
    if constexpr (!SUB) return 0;
    if (CT && a.tap_live) return t >= 2 * Q ? 1 + ((t - 2 * Q) & 1) : 3 * (t & 1);
    return t / Q;
  };
  // SUB: output NHWC row of input-grid pixel p of phase ph: (img, 2i + py, 2j + px) of the 2x grid
  auto orow = [&](int p, int ph) -> size_t {
    if constexpr (!SUB) return (size_t)p;
    const int HWi = H * W, img = p / HWi, rem = p - img * HWi, i = rem / W, j = rem - i * W;
    return ((size_t)img * 2 * H + 2 * i + (ph >> 1)) * (2 * W) + 2 * j + (ph & 1);
  };
#ifdef ITSD_STAMPS
  // MFMA waves: 0 chunk compute, 1 barrier wait, 6 epilogues, 7 total; halo waves: 3 stage
  // transforms (incl. next-stage load issue), 1 barrier wait, 5 prologue (stage 0), 7 total
  unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long t_begin = stamp();
  auto stamps_out = [&]() {
    st[7] = stamp() - t_begin;
    if (lane == 0) {
      const int bb = blockIdx.x & 1023;
#pragma unroll
      for (int qq = 0; qq < 8; ++qq) g_stamps[(bb * 16 + wid) * 8 + qq] = st[qq];
    }
  };
#define P4_STAMP_OUT() stamps_out()
#else
#define P4_STAMP_OUT()
#endif
  auto block_sync = [&]() {
    STAMP(b0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    STAMP(b1);
    STAMP_ADD(1, b1 - b0);
  };
  if (ntiles == 0) return;  // (the host launches gridDim.x <= tiles)
  // bias (+ time / class embedding) of tile k's couts (and image segments) -> addv[k & 1]
  auto stage_addv = [&](int k, int t0) {  // threads t0 .. t0+255
    const int tileP = tile_p(k), tileC = tile_c(k), img0 = tileP / (H * W);
    const long long trow = a.temb ? (a.temb_tsel ? (long long)(*a.temb_tsel) * a.temb_row_stride : 0) : 0;
    for (int it = t0; it < NSEG * BM; it += 256) {
      const int il = it / BM, cl = it - il * BM, co = tileC + cl, img = img0 + il;
      float v = a.bias[co];
      if (a.temb) v += a.temb[trow + (long long)img * a.temb_img_stride + co];
      if (a.cemb) {
        int lab = 0;
        if (a.cemb_uncond_from < 0 || img < a.cemb_uncond_from) lab = a.cemb_labels[img % a.cemb_label_mod];
        v += a.cemb[(long long)lab * a.cemb_row_stride + co];
      }
      addv[(k & 1) * NSEG * BM + it] = v;
    }
  };

  if (wid < 4) {
    if constexpr (M16) {
    // ================================================================ MFMA waves, v_mfma_f32_16x16x32_bf16
    // The same wave tiles (wave w: couts 64*(w & 1) .. +63, pixels 128*(w >> 1) .. +127) as 4 x 8 16x16
    // accumulators (f32x4: couts 16 ci + 4 kg .. +3 of pixel 16 pj + m, lane = 16 kg + m), 32 MFMAs per
    // 32-deep k-step, run as two half-steps of 16 (pixel blocks 0-3, 4-7) so that the B buffers stay 4
    // fragments. Equal cycles per FLOP to 32x32x16, but the chip holds a higher clock under this shape
    // (MI355X_MICROARCH.md DVFS item 7; the calibration loops of calib.hip measure both on the box).
    // A fragments come from the 32x32x16 fragment array unchanged: a 16-cout fragment of k32-step s is
    // lane 16 (ci & 1) + m + 32 (kg & 1) of 32-cout block 2 wm + (ci >> 1), k16-step 2 s + (kg >> 1).
    const int wm = wid & 1, wn = wid >> 1, m = lane & 15, kg = lane >> 4;
    static_assert(COMPACT || (W == 32 && NSEG == 1), "halo rows of the 16-pixel blocks from one base");
    // pixel block j of this lane: COMPACT the tile pixel hb0 + 16 j (column m % W, row hb0 / W + 16 j / W of its
    // image); else (32 x 32) halo row hb0 + (j >> 1) * W2 + 16 (j & 1) at tap (0, 0) -- one register
    const int hb0 = COMPACT ? wn * 128 + m : wn * 4 * W2 + m;
    const uint32_t ablk = (uint32_t)(NTAP * kpt) * 1024;
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.wfrag, (short)0, 0x7fffffff, 0x00020000);
    const uint32_t avo0 = (uint32_t)((kg >> 1) * 1024 + (m + 32 * (kg & 1)) * 16) + 2 * wm * ablk, avo1 = avo0 + ablk;
    auto abase_of = [&](int k) -> uint32_t { return (uint32_t)(tile_c(k) >> 5) * ablk; };
    constexpr int KS2 = 2 * NTAP, RING2 = 3;  // k32-steps a chunk; A ring slots (prefetch 2 k32-steps = 64 MFMAs)
    static_assert(KS2 % RING2 == 0, "ring slots repeat per chunk");
    f32x4 acc[NCI][8];
#pragma unroll
    for (int i = 0; i < NCI; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 ra[RING2][NCI];
    // C96: the wave's 16-cout block b is block 3 wm + b of the tile -- 32-cout block (3 wm + b) >> 1, half
    // (3 wm + b) & 1: a wave-uniform part of the offset, added to soffset
    const uint32_t avl = (uint32_t)((kg >> 1) * 1024 + (m + 32 * (kg & 1)) * 16);
    auto fo96 = [&](int b) -> uint32_t { return (uint32_t)((3 * wm + b) >> 1) * ablk + (uint32_t)((3 * wm + b) & 1) * 256; };
    // half hf of k32-step s's A fragments (ci = 2 hf, 2 hf + 1): tap s >> 1, k16-steps 2 (s & 1) + (kg >> 1)
    auto load_a = [&](uint32_t base, int st, u32x4 (&dst)[NCI], int hf) __attribute__((always_inline)) {
      const uint32_t off = base + (uint32_t)((st >> 1) * kpt + 2 * (st & 1)) * 1024;
      if constexpr ((AB & 8) != 0) {
#pragma unroll
        for (int b = 2 * hf; b < 2 * hf + 2; ++b)
          if (b < NCI) dst[b] = u32x4{(uint32_t)st, (uint32_t)b, 0u, 0u};
      } else if constexpr (C96) {
#pragma unroll
        for (int b = 2 * hf; b < 2 * hf + 2; ++b)
          if (b < NCI) dst[b] = __builtin_amdgcn_raw_buffer_load_b128(wrs, avl, off + fo96(b), 0);
      } else {
        const uint32_t vo = hf ? avo1 : avo0;
        dst[2 * hf] = __builtin_amdgcn_raw_buffer_load_b128(wrs, vo, off, 0);
        dst[2 * hf + 1] = __builtin_amdgcn_raw_buffer_load_b128(wrs, vo + 256, off, 0);
      }
    };
    {
      const uint32_t ab0 = abase_of(0);
#pragma unroll
      for (int s0 = 0; s0 < RING2 - 1; ++s0) {
        load_a(ab0, s0, ra[s0], 0);
        load_a(ab0, s0, ra[s0], 1);
      }
    }
    auto init_acc = [&](int kk) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int seg = NSEG == 1 ? 0 : (wn * 128 + j * 16) / HWs;
#pragma unroll
        for (int i = 0; i < NCI; ++i)
          acc[i][j] = *(const f32x4*)(addv + ((kk & 1) * NSEG + seg) * BM + wm * HB + 16 * i + 4 * kg);
      }
    };
    stage_addv(0, tid);
    block_sync();  // B0: stage 0 staged
    init_acc(0);
    int q = 0;
    for (int k = 0; k < ntiles; ++k) {
      const uint32_t ab = abase_of(k);
      const uint32_t abn = k + 1 < ntiles ? abase_of(k + 1) : ab;
      for (int cc = 0; cc < ncc; ++cc, ++q) {
        const char* hcur = smem + (q & 1) * HALO;
        const uint32_t nb = cc + 1 < ncc ? ab + (uint32_t)(cc + 1) * 4 * 1024 : abn;
        const uint32_t cb = ab + (uint32_t)cc * 4 * 1024;
        STAMP(c0);
        // a half-step: 16 MFMAs; its 2 A loads, 4 B reads and address VALU in the first gaps
        auto half_sched = [&]() __attribute__((always_inline)) {
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
#pragma unroll
          for (int g = 0; g < 10; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        };
        int tb[4];
        int zad = 0;  // (W = 16: this lane's zero-row address, for the two pixel blocks a wave-uniform tap row leaves)
        bf16x8 fb[BD][4];
        // B unit u = (k32-step u >> 1, pixel blocks 4 (u & 1) .. +3): byte (h * 128 + ((kg ^ hswz(h)) << 4)) ^ (s2 << 6),
        // s2 = the step's half of the tap's 64 channels. Four address registers a tap, rebuilt at its first unit:
        // a pixel block 16 rows (32x32: block 2t + 1 of block 2t) or 64 rows (COMPACT: block j + 4 of block j) on has
        // the same swizzle (hswz has period 8 rows), so it is an immediate offset (2048 / 8192 B) of its partner's address.
        // COMPACT: a tap reading outside its image reads a zero row (x: per lane, all blocks -- the zero rows 256 and
        // 320; y at 16x16: rows -1 / 16 are wave-uniform, block 0 at ky = 0 of wave row 0, block 7 at ky = 2 of wave
        // row 1 -- those two reads take the zero-row address; their partners are in range)
        auto rd = [&](int u, int buf) __attribute__((always_inline)) {
          const int st = u >> 1, hf = u & 1, tap = st >> 1, s2 = st & 1;
          const int ky = tap / 3, kx = tap - (tap / 3) * 3;
          if (s2 == 0 && hf == 0) {
            int p0 = hb0;
            asm volatile("" : "+v"(p0));  // (rebuilt per tap, not hoisted out of the chunk loop)
            const int hoff = (int)(hcur - smem);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              int h;
              if constexpr (COMPACT) {
                // block t: x = column, y = row in its image (y range checked at 8x8 only: 16x16 rows are wave-uniform)
                const int x = (p0 & (W - 1)) + kx - 1, y = (((p0 / W) + t * (16 / W)) & (W - 1)) + ky - 1;
                const bool ok = (unsigned)x < (unsigned)W && (W == 16 || (unsigned)y < (unsigned)W);
                const int hw = p0 + 16 * t + (ky - 1) * W + (kx - 1);
                h = ok ? hw : ZROW + (ITSD_P4_ZR8 && W == 8 ? (hw & 7) : 0);  // (16x16: one zero row; 8 rows by residue spilled)
              } else {
                h = p0 + t * W2 + ky * W2 + kx;  // block 2t
              }
              if constexpr (COMPACT) tb[t] = hoff + h * ROWB + ((kg ^ hswz(h)) << 4);
              else tb[t] = (hoff + h * ROWB + (hswz(h) << 4)) ^ (kg << 4);  // (the same bits; fewer registers at 32x32)
            }
            if constexpr (COMPACT && W == 16)
              if (ky != 1) zad = hoff + ZROW * ROWB + ((kg ^ hswz(ZROW)) << 4);
          }
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * hf + jj;
            int ad;
            if constexpr (COMPACT) {
              ad = (tb[jj] ^ (s2 << 6)) + hf * 8192;
              if constexpr (W == 16) {
                if (ky == 0 && j == 0 && wn == 0) ad = zad ^ (s2 << 6);
                if (ky == 2 && j == 7 && wn == 1) ad = zad ^ (s2 << 6);
              }
            } else {
              ad = (tb[j >> 1] ^ (s2 << 6)) + (j & 1) * 2048;
            }
            if constexpr ((AB & 16) != 0) fb[buf][jj] = bf16x8{(short)(u + jj), 0, 0, 0, 0, 0, 0, 1};
            else fb[buf][jj] = *(const bf16x8*)(smem + ad);
          }
        };
#pragma unroll
        for (int u0 = 0; u0 < BD - 1; ++u0) rd(u0, u0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 2 * KS2; ++u) {
          const int st = u >> 1, hf = u & 1, pf = st + RING2 - 1;
          if (pf < KS2) load_a(cb, pf, ra[pf % RING2], hf);
          else load_a(nb, pf - KS2, ra[pf % RING2], hf);
          if (u + BD - 1 < 2 * KS2) rd(u + BD - 1, (u + BD - 1) % BD);
#pragma unroll
          for (int i = 0; i < NCI; ++i) {
            const bf16x8 af = __builtin_bit_cast(bf16x8, ra[st % RING2][i]);
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][4 * hf + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, fb[u % BD][j], acc[i][4 * hf + j], 0, 0, 0);
          }
          half_sched();
        }
        STAMP(c1);
        STAMP_ADD(0, c1 - c0);
        block_sync();  // end of stage q: its buffer is free, stage q+1 is published
      }
      STAMP(e0);
      if constexpr ((AB & 4) == 0) {
        // epilogue of tile k into the LDS residual / output tile (the 32x32x16 path's layout: row p, 16-B group
        // cout / 8 ^ sw(p), 8-B half (cout / 4) & 1); the halo waves store it and sum its statistics
        auto epi = [&](auto hr) __attribute__((always_inline)) {
          constexpr bool HR = decltype(hr)::value;
          uint2 rr[2][NCI];
          int pb = wn * 128 + m, kgo = kg;
          asm volatile("" : "+v"(pb), "+v"(kgo));  // (the 32 addresses are rebuilt here, not held through the chunk loop)
          auto addr = [&](int i, int j) {
            const int p = pb + j * 16;
            return rlds + wm * 32768 + p * 128 + (((2 * i + (kgo >> 1)) ^ ((p >> 1) & 7)) << 4) + 8 * (kgo & 1);
          };
          auto rdr = [&](int j, uint2 (&d)[NCI]) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < NCI; ++i) d[i] = HR ? *(const uint2*)addr(i, j) : uint2{0u, 0u};
          };
          rdr(0, rr[0]);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if (j + 1 < 8) rdr(j + 1, rr[(j + 1) & 1]);
#pragma unroll
            for (int i = 0; i < NCI; ++i) {
              const uint2 r = rr[j & 1][i];
              const float v0 = acc[i][j][0] + __uint_as_float(r.x << 16);
              const float v1 = acc[i][j][1] + __uint_as_float(r.x & 0xffff0000u);
              const float v2 = acc[i][j][2] + __uint_as_float(r.y << 16);
              const float v3 = acc[i][j][3] + __uint_as_float(r.y & 0xffff0000u);
              *(uint2*)addr(i, j) = uint2{pk_bf16(v0, v1), pk_bf16(v2, v3)};
            }
          }
        };
        if (a.resid) epi(std::true_type{});
        else epi(std::false_type{});
      } else {  // keep the accumulators alive
        float sm = 0.f;
#pragma unroll
        for (int i = 0; i < NCI; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) sm += acc[i][j][r];
        if (sm == 1.2345f) ((float*)a.out)[0] = sm;
      }
      if (k + 1 < ntiles) init_acc(k + 1);
      STAMP(e1);
      STAMP_ADD(6, e1 - e0);
    }
    block_sync();  // the last tile's output is in LDS
    P4_STAMP_OUT();
    return;
    } else {
    // ================================================================ MFMA waves (one per SIMD)
    // wave w: couts 64*(w & 1) .. +63 (two 32-cout A fragments per k-step), pixels 128*(w >> 1) ..
    // +127 (four B fragments): 8 MFMAs per k-step on 128 accumulator registers (AGPRs)
    const int wm = wid & 1, wn = wid >> 1, rl = lane & 31, hh = lane >> 5;
    int hb[4];  // halo row of this lane's pixel at tap (0, 0) (COMPACT: the tile pixel itself)
    int hq[4];  // (CSWZ) its coordinate swizzle base SC1 oy + SC2 ox
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pl = wn * 128 + j * 32 + rl;
      const int seg = pl / (THs * W), rem = pl - seg * THs * W, oy = rem / W;
      hb[j] = COMPACT ? pl : seg * HS + oy * W2 + (rem - oy * W);
      hq[j] = SC1 * oy + SC2 * (rem - oy * W);
    }
    const uint32_t ablk = (uint32_t)(NTAP * kpt) * 1024;  // one 32-cout block of fragments
    // A fragments by buffer loads: resource = the whole wfrag array, voffset = this lane's 16 B of the wave's
    // two 32-cout blocks, soffset = the tile's fragment block + the k-step (uniform: scalar arithmetic, no
    // 64-bit address VGPRs, no per-step 64-bit SGPR offsets held across the chunk loop)
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.wfrag, (short)0, 0x7fffffff, 0x00020000);
    const uint32_t avo0 = (uint32_t)lane * 16 + 2 * wm * ablk, avo1 = avo0 + ablk;
    auto abase_of = [&](int k) -> uint32_t {
      return (uint32_t)(tile_ph(k) * (a.Cout >> 5) + (tile_c(k) >> 5)) * ablk;
    };
    f32x16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    u32x4 ra[RING][2];
    auto load_a = [&](uint32_t base, int st, u32x4 (&dst)[2]) __attribute__((always_inline)) {
      const uint32_t off = base + (uint32_t)((st >> 2) * kpt + (st & 3)) * 1024;
      if constexpr ((AB & 8) != 0) {
        dst[0] = u32x4{(uint32_t)st, 0u, 0u, 0u};
        dst[1] = u32x4{(uint32_t)st, 1u, 0u, 0u};
      } else {
        dst[0] = __builtin_amdgcn_raw_buffer_load_b128(wrs, avo0, off, 0);
        dst[1] = __builtin_amdgcn_raw_buffer_load_b128(wrs, avo1, off, 0);
      }
    };
    // ConvTranspose2d phases with tap_live: a chunk runs only its phase's live taps; the A prefetch that
    // crosses into the next chunk / tile starts at that chunk's first live tap (tap0_off)
    auto tap0_off = [&](int k) -> uint32_t {
      if constexpr (CT) {
        if (a.tap_live) {
          const int ph = tile_ph(k);
          return (uint32_t)(((ph >> 1) * 3 + (ph & 1)) * kpt) * 1024;
        }
      }
      return 0;
    };
    {
      const uint32_t ab0 = abase_of(0) + tap0_off(0);
#pragma unroll
      for (int s0 = 0; s0 < RING - 1; ++s0) load_a(ab0, s0, ra[s0]);
    }
    // RES: the accumulators start from tile k's bias (+ time / class embedding), staged by the halo
    // waves in LDS before the barrier that precedes the tile (tile 0: B0)
    auto init_acc = [&](int kk) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            // (the image segment of pixel block j: NSEG = 4 -- 64-pixel images -- has two a wave)
            const int seg = NSEG == 1 ? 0 : (wn * 128 + j * 32) / HWs;
            const f32x4 ad = *(const f32x4*)(addv + ((kk & 1) * NSEG + seg) * BM + (2 * wm + i) * 32 + 8 * g + 4 * hh);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[i][j][4 * g + e] = ad[e];
          }
        }
    };
    stage_addv(0, tid);  // (off the halo waves' stage-0 critical path)
    block_sync();  // B0: stage 0 staged
    if constexpr (RES) init_acc(0);
    int q = 0;     // stage (chunk) counter of this block
    for (int k = 0; k < ntiles; ++k) {
      const int tileP = tile_p(k), tileC = tile_c(k), tph = tile_ph(k);
      const uint32_t ab = abase_of(k);
      const uint32_t abn = k + 1 < ntiles ? abase_of(k + 1) + tap0_off(k + 1) : ab;
      const uint32_t t0k = tap0_off(k);
      for (int cc = 0; cc < ncc; ++cc, ++q) {
        const char* hcur = smem + (q & 1) * HALO;
        const uint32_t nb = cc + 1 < ncc ? ab + (uint32_t)(cc + 1) * 4 * 1024 + t0k : (k + 1 < ntiles ? abn : ab);
        const uint32_t cb = ab + (uint32_t)cc * 4 * 1024;
        STAMP(c0);
        // the step's A loads, B reads and address VALU spread over its 8 MFMA gaps (measured against all of
        // them ahead of the MFMAs in one gap: 32x32 -1 %, 16x16 -3 %, 8x8 -1.5 %, profiles/r03b/p4_sgb_ab.txt)
        auto step_sched = [&]() __attribute__((always_inline)) {
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
          }
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
          }
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        };
        auto mfma_step = [&](const u32x4 (&af2)[2], const bf16x8 (&fbs)[4]) __attribute__((always_inline)) {
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const bf16x8 af = __builtin_bit_cast(bf16x8, af2[i]);
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if constexpr ((AB & 1) != 0) acc[i][j][0] += __builtin_bit_cast(float, (uint32_t)fbs[j][0] << 16) + (float)af[0];
              else acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, fbs[j], acc[i][j], 0, 0, 0);
          }
        };
        // B fragment j of k-step kk of the tap at halo offset (ky, kx): byte (h * 128 + ((hh ^ sw(h)) << 4))
        // ^ (kk << 5), h = the pixel's halo row for the tap: the tap's 4 row addresses are rebuilt (from an
        // opaque copy, so they are not hoisted out of the chunk loop: 36 registers) at its first k-step
        int tb[4];
        bf16x8 fb[BD][4];
        auto rd_tap = [&](int ky, int kx, int kk, int buf) __attribute__((always_inline)) {
          if (kk == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              int h;
              if constexpr (COMPACT) {  // the tap's pixel inside the image, else the zero row
                int p = hb[j];
                asm volatile("" : "+v"(p));
                const int x = (p & (W - 1)) + kx - 1, y = ((p / W) & (W - 1)) + ky - 1;
                h = ((unsigned)x < (unsigned)W && (unsigned)y < (unsigned)W) ? p + (ky - 1) * W + (kx - 1) : ZROW;
              } else {
                h = hb[j] + ky * W2 + kx;
                asm volatile("" : "+v"(h));
              }
              const int sw = CSWZ ? (hq[j] + SC1 * ky + SC2 * kx) & 7 : (h >> 1) & 7;
              tb[j] = (int)(hcur - smem) + h * ROWB + ((hh ^ sw) << 4);
            }
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if constexpr ((AB & 16) != 0) fb[buf][j] = bf16x8{(short)(kk + j), 0, 0, 0, 0, 0, 0, 1};
            else fb[buf][j] = *(const bf16x8*)(smem + (tb[j] ^ (kk << 5)));
          }
        };
        if constexpr (CT) {
          static_assert(RING == 4 && BD == 2, "one tap's 4 k-steps per ring turn");
          // ConvTranspose2d phases: a run-time loop over the phase's live taps (window rows ry..2 x
          // columns rx..2 with tap_live; all 9 otherwise), 4 unrolled k-steps a tap: step kk of every tap
          // uses ring slot kk and B buffer kk & 1; the A prefetch 3 steps ahead reaches into the next
          // live tap (or the next chunk, nb, at the last one)
          const int ry = a.tap_live ? (tph >> 1) : 0, rx = a.tap_live ? (tph & 1) : 0;
          const int ntl = (3 - ry) * (3 - rx);
          int ky = ry, kx = rx;
          rd_tap(ky, kx, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          for (int ti = 0; ti < ntl; ++ti) {
            const bool last = ti + 1 == ntl;
            const int nky = kx == 2 ? ky + 1 : ky, nkx = kx == 2 ? rx : kx + 1;
            const int rky = last ? ky : nky, rkx = last ? kx : nkx;  // (the last tap re-reads its own rows)
            const uint32_t tcur = cb + (uint32_t)((ky * 3 + kx) * kpt) * 1024;
            const uint32_t tnxt = last ? nb : cb + (uint32_t)((nky * 3 + nkx) * kpt) * 1024;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
              if (kk == 0) load_a(tcur, 3, ra[3]);
              else load_a(tnxt, kk - 1, ra[kk - 1]);
              if (kk < 3) rd_tap(ky, kx, kk + 1, (kk + 1) & 1);
              else rd_tap(rky, rkx, 0, 0);
              mfma_step(ra[kk], fb[kk & 1]);
              step_sched();
            }
            ky = nky;
            kx = nkx;
          }
        } else {
          // 36 (9 taps x 4) or 16 (4 taps x 4) k-steps, fully unrolled; B fragments BD - 1 k-steps ahead,
          // across tap boundaries
          auto rd = [&](int st, int buf) __attribute__((always_inline)) {
            const int tap = st >> 2;
            // SUB4: tap (dy, dx) of phase (py, px) reads input offset (dy + py - 1, dx + px - 1)
            const int ky = SUB4 ? (tap >> 1) + (tph >> 1) : tap / 3, kx = SUB4 ? (tap & 1) + (tph & 1) : tap - (tap / 3) * 3;
            rd_tap(ky, kx, st & 3, buf);
          };
#pragma unroll
          for (int s0 = 0; s0 < BD - 1; ++s0) rd(s0, s0);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int step = 0; step < KST; ++step) {
            const int pf = step + RING - 1;
            if (pf < KST) load_a(cb, pf, ra[pf % RING]);
            else load_a(nb, pf - KST, ra[pf % RING]);
            if (step + BD - 1 < KST) rd(step + BD - 1, (step + BD - 1) % BD);
            mfma_step(ra[step % RING], fb[step % BD]);
            step_sched();
          }
        }
        STAMP(c1);
        STAMP_ADD(0, c1 - c0);
        block_sync();  // end of stage q: its buffer is free, stage q+1 is published
      }
      STAMP(e0);
      if constexpr ((AB & 4) == 0 && RES) {
      // ---- epilogue of tile k, first half: out = acc (which started from addv) + residual, rounded
      // to bf16 in place of the residual in LDS (8 B per lane and register group, the layout below);
      // the halo waves store the tile and sum its GroupNorm statistics during the next tile's second
      // stage. The reads of pixel block j+1 are issued before the writes of block j.
      auto epi = [&](auto hr) __attribute__((always_inline)) {
        constexpr bool HR = decltype(hr)::value;
        uint2 rr[2][4];
        auto rd = [&](int i, int j, uint2 (&d)[4]) __attribute__((always_inline)) {
          const int p = wn * 128 + j * 32 + rl;
#pragma unroll
          for (int g = 0; g < 4; ++g)
            d[g] = HR ? *(const uint2*)(rlds + wm * 32768 + p * 128 + (((4 * i + g) ^ ((p >> 1) & 7)) << 4) + 8 * hh)
                      : uint2{0u, 0u};
        };
        rd(0, 0, rr[0]);
#pragma unroll
        for (int ij = 0; ij < 8; ++ij) {
          const int i = ij >> 2, j = ij & 3, p = wn * 128 + j * 32 + rl;
          if (ij + 1 < 8) rd((ij + 1) >> 2, (ij + 1) & 3, rr[(ij + 1) & 1]);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const uint2 r = rr[ij & 1][g];
            const float v0 = acc[i][j][4 * g + 0] + __uint_as_float(r.x << 16);
            const float v1 = acc[i][j][4 * g + 1] + __uint_as_float(r.x & 0xffff0000u);
            const float v2 = acc[i][j][4 * g + 2] + __uint_as_float(r.y << 16);
            const float v3 = acc[i][j][4 * g + 3] + __uint_as_float(r.y & 0xffff0000u);
            *(uint2*)(rlds + wm * 32768 + p * 128 + (((4 * i + g) ^ ((p >> 1) & 7)) << 4) + 8 * hh) =
                uint2{pk_bf16(v0, v1), pk_bf16(v2, v3)};
          }
        }
      };
      if (a.resid) epi(std::true_type{});
      else epi(std::false_type{});
      } else if constexpr ((AB & 4) == 0) {
      // ---- epilogue of tile k from the accumulators (no LDS tile, no barrier)
      // lane (rl, hh): pixels p_j = wn*128 + 32j + rl, couts c = wmi*32 + 8g + 4hh + e, wmi = 2wm + i
      const bool has_res = a.resid != nullptr;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
      const int wmi = 2 * wm + i;
      const float* av = addv + (k & 1) * NSEG * BM + wmi * 32 + 4 * hh;
      float s16[16], q16[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) s16[e] = q16[e] = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = wn * 128 + j * 32 + rl;
        const float* avj = av + (NSEG == 1 ? 0 : (wn * 2 + (j >> 1))) * BM;
        uint32_t wv[4][2];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = wmi * 32 + 8 * g + 4 * hh;
          const f32x4 ad = *(const f32x4*)(avj + 8 * g);
          const T* rp = has_res ? (const T*)a.resid + (size_t)(tileP + p) * a.Cout + tileC + c
                                : (const T*)zero_of_block<T>(a);
          uint2 rr = *(const uint2*)rp;
          if (!has_res) rr = uint2{0u, 0u};  // select, not a branch
          float v[4];
          v[0] = acc[i][j][4 * g + 0] + ad[0] + __uint_as_float(rr.x << 16);
          v[1] = acc[i][j][4 * g + 1] + ad[1] + __uint_as_float(rr.x & 0xffff0000u);
          v[2] = acc[i][j][4 * g + 2] + ad[2] + __uint_as_float(rr.y << 16);
          v[3] = acc[i][j][4 * g + 3] + ad[3] + __uint_as_float(rr.y & 0xffff0000u);
          const T b0 = f2bf(v[0]), b1 = f2bf(v[1]), b2 = f2bf(v[2]), b3 = f2bf(v[3]);
          wv[g][0] = (uint32_t)b0 | ((uint32_t)b1 << 16);
          wv[g][1] = (uint32_t)b2 | ((uint32_t)b3 << 16);
          const float r0 = bf2f(b0), r1 = bf2f(b1), r2 = bf2f(b2), r3 = bf2f(b3);
          s16[4 * g + 0] += r0; q16[4 * g + 0] = fmaf(r0, r0, q16[4 * g + 0]);
          s16[4 * g + 1] += r1; q16[4 * g + 1] = fmaf(r1, r1, q16[4 * g + 1]);
          s16[4 * g + 2] += r2; q16[4 * g + 2] = fmaf(r2, r2, q16[4 * g + 2]);
          s16[4 * g + 3] += r3; q16[4 * g + 3] = fmaf(r3, r3, q16[4 * g + 3]);
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
          const int c8 = wmi * 32 + 8 * (gp + hh);
          *(u32x4*)((T*)a.out + orow(tileP + p, tph) * a.Cout + tileC + c8) = o;
        }
        if (a.stats && ((NSEG == 1 && j == 3) || (NSEG != 1 && (j & 1)))) {
          float v[32];
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            v[e] = s16[e];
            v[16 + e] = q16[e];
          }
          auto xchg = [](float x, auto wc) {
            constexpr int w = decltype(wc)::value;
            const int xi = __builtin_bit_cast(int, x);
            int r;
            if constexpr (w == 1) r = __builtin_amdgcn_update_dpp(0, xi, 0xB1, 0xF, 0xF, false);
            else if constexpr (w == 2) r = __builtin_amdgcn_update_dpp(0, xi, 0x4E, 0xF, 0xF, false);
            else if constexpr (w == 8) r = __builtin_amdgcn_update_dpp(0, xi, 0x128, 0xF, 0xF, false);
            else r = __builtin_amdgcn_ds_swizzle(xi, 0x1F | (w << 10));
            return __builtin_bit_cast(float, r);
          };
          auto halve = [&](auto wc) {
            constexpr int w = decltype(wc)::value;
            const bool up = (rl & w) != 0;
#pragma unroll
            for (int ii = 0; ii < w; ++ii) {
              const float lo = v[ii], hi = v[ii + w];
              v[ii] = (up ? hi : lo) + xchg(up ? lo : hi, wc);
            }
          };
          halve(std::integral_constant<int, 16>{});
          halve(std::integral_constant<int, 8>{});
          halve(std::integral_constant<int, 4>{});
          halve(std::integral_constant<int, 2>{});
          halve(std::integral_constant<int, 1>{});
          {
            constexpr int SLOT = NSEG == 1 ? 128 : 64;
            long long slot = (long long)(tileP + wn * 128 + (NSEG == 1 ? 0 : (j >> 1) * 64)) / SLOT;
            // SUB (W = 8: 64-pixel phase images): one statistics slot per (image, phase)
            if constexpr (SUB) slot = slot * 4 + tph;
            const int e = rl & 15, co = wmi * 32 + 8 * (e >> 2) + 4 * hh + (e & 3);
            a.stats[(slot * 2 + (rl >> 4)) * a.Cout + tileC + co] = v[0];
          }
#pragma unroll
          for (int e = 0; e < 16; ++e) s16[e] = q16[e] = 0.f;
        }
      }
      }
      } else {  // keep the accumulators alive
        float sm = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) sm += acc[i][j][r];
        if (sm == 1.2345f) ((float*)a.out)[0] = sm;
      }
      if constexpr (RES) {
        if (k + 1 < ntiles) init_acc(k + 1);
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
      }
      STAMP(e1);
      STAMP_ADD(6, e1 - e0);
    }
    if constexpr (RES) block_sync();  // the last tile's output is in LDS
    P4_STAMP_OUT();
    return;
    }  // (!M16)
  }

  // ================================================================== halo waves
  // (conv3x3_gn_ws_kernel's halo pipeline, over the block's whole stage sequence.) Item j of this
  // thread = halo row (lt >> 3) + RPP * j of its image segment, 8 channels (lch). Per tile, for
  // the loads: the input pixel of each item (0 for padding / scratch rows: a valid address,
  // never used); for the LDS writes: each item's address (its halo row, or a dump row past the
  // segments for scratch rows) and a mask that zeroes padding rows (rewritten every stage: the
  // padding rows differ between tiles). Stage and tile indices advance by counters (no divides).
  const int tt = tid - 256, lch = tt & 7, sg = tt / TPS, lt = tt - sg * TPS;
  static_assert(COMPACT || NSEG * ITEMS * RPP > NSEG * HS, "a scratch row exists");
  if (a.dbg & (1 << 20)) __builtin_amdgcn_s_setprio(1);  // measurement switches, as in the ws kernel
  if (a.dbg & (1 << 21)) __builtin_amdgcn_s_setprio(2);
  const int dump = NSEG * HS * ROWB + (lch << 4);  // (not COMPACT: the scratch rows' write target)
  const int hrow0 = (COMPACT ? sg * HWs : sg * HS) + (lt >> 3), hrow1 = hrow0 + RPP;
  const int lds0 = hrow0 * ROWB + ((lch ^ hswz(hrow0)) << 4);
  const int lds1 = hrow1 * ROWB + ((lch ^ hswz(hrow1)) << 4);
  auto item_lds = [&](int j) {
    if constexpr (CSWZ) {  // (halo coordinates of the item's row; the scratch rows past HS go to dump)
      const int r = (lt >> 3) + RPP * j, hy = r / W2, hx = r - hy * W2;
      return (sg * HS + r) * ROWB + ((lch ^ ((SC1 * hy + SC2 * hx) & 7)) << 4);
    }
    return ((j & 1) ? lds1 : lds0) + (j >> 1) * (2 * RPP * ROWB);
  };
  auto tile_y0img = [&](int k, int& img0, int& y0) {
    const int tileP = tile_p(k);
    img0 = tileP / (H * W);
    y0 = (tileP - img0 * H * W) / W;
  };
  int ipix[ITEMS];
  const float* cbase;  // GroupNorm coefficients of the loading tile's image, this lane's 8 channels
  int simg = 0;        // (gn_fold) the loading tile's image of this thread's segment
  int gimg = -1;       // (gn_fold) the image whose statistics gsw holds
  float* const gsw = (float*)(smem + 2 * HALO + RESB + 2 * NSEG * CONV_BM * 4) + (wid - 4) * 64;
  // gn_fold (conv3x3_gn_p5_kernel's reduction): group mean / rstd of image img from the producers'
  // statistics slabs, fp64, this wave's 32 groups -> gsw. Lane = (group lane & 31, half lane >> 5);
  // its (channel pair, slot) items in batches of 8 with all 16 loads in flight before the first sum
  auto group_stats = [&](int img) __attribute__((always_inline)) {
    const int g = lane & 31, hf = Cin / 64, c0 = g * 2 * hf + (lane >> 5) * hf;
    const int HWi = H * W;
    const int sp1 = stat_spi(HWi, a.gn_spi1), sp2 = a.C2 ? stat_spi(HWi, a.gn_spi2) : 0;
    const int spm = sp1 > sp2 ? sp1 : sp2, np = hf >> 1, m = np * spm;
    double sm = 0.0, sq = 0.0;
    for (int b0 = 0; b0 < m; b0 += 8) {
      float2 vs[8], vq[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int it = b0 + i, q = it / np, cr = c0 + 2 * (it - q * np);
        const bool s1 = cr < a.C1;
        const bool ok = it < m && q < (s1 ? sp1 : sp2);
        const int c = ok ? cr : c0, qq = ok ? q : 0;
        const bool t1 = c < a.C1;
        const float* st = t1 ? a.gn_st1 : a.gn_st2;
        const int Cs = t1 ? a.C1 : a.C2, cs = t1 ? c : c - a.C1, sp = t1 ? sp1 : sp2;
        const long long slot = (long long)img * sp + qq;
        const float2 u0 = *(const float2*)(st + (slot * 2) * Cs + cs);
        const float2 u1 = *(const float2*)(st + (slot * 2 + 1) * Cs + cs);
        vs[i] = ok ? u0 : float2{0.f, 0.f};
        vq[i] = ok ? u1 : float2{0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sm += (double)vs[i].x + (double)vs[i].y;
        sq += (double)vq[i].x + (double)vq[i].y;
      }
    }
    sm += __shfl_xor(sm, 32, 64);
    sq += __shfl_xor(sq, 32, 64);
    const double E = (double)(Cin / 32) * HWi, mean = sm / E;
    double var = sq / E - mean * mean;
    var = var > 0.0 ? var : 0.0;
    if (lane < 32) {
      gsw[2 * g] = (float)mean;
      gsw[2 * g + 1] = (float)(1.0 / sqrt(var + 1e-5));
    }
  };
  auto geometry_pix = [&](int k) __attribute__((always_inline)) {
    int img0, y0;
    tile_y0img(k, img0, y0);
    // the item geometry from an opaque copy of lt: hoisted out of the stage loop (it is tile-
    // invariant), it would hold ~30 registers for good and starve the transform of temporaries
    int ltv = lt;
    asm volatile("" : "+v"(ltv));
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int r = (ltv >> 3) + RPP * j;
      if constexpr (COMPACT) {  // every item an interior pixel of image img0 + sg
        ipix[j] = (img0 + sg) * HWs + r;
      } else {
        const int hy = r / W2, hx = r - hy * W2, iy = y0 + hy - 1, ix = hx - 1;
        const bool ok = r < HS && iy >= 0 && iy < H && ix >= 0 && ix < W;
        ipix[j] = ok ? ((img0 + sg) * H + iy) * W + ix : 0;
      }
    }
    if constexpr (!PLAIN) cbase = a.gn_coef + ((size_t)(img0 + sg) * (Cin / 8) + lch) * 16;
    simg = img0 + sg;
  };
  // Only the last item can hold scratch rows (ITEMS * RPP - HS < RPP for every W): its write
  // address is chosen once; the other items' addresses are lds0/lds1 plus constants.
  static_assert(COMPACT || ITEMS * RPP - HS < RPP, "scratch rows only in the last item");
  const int waddr_last = (COMPACT || ((lt >> 3) + RPP * (ITEMS - 1)) < HS) ? item_lds(ITEMS - 1) : dump;
  auto waddr = [&](int j) { return j == ITEMS - 1 ? waddr_last : item_lds(j); };
  int inm = 0;  // bit j: item j's row is real input (or scratch) -- else zero padding
  auto geometry_emit = [&](int k) __attribute__((always_inline)) {
    int img0, y0;
    tile_y0img(k, img0, y0);
    int ltv = lt;
    asm volatile("" : "+v"(ltv));
    inm = 0;
    if constexpr (COMPACT) {
      inm = (1 << ITEMS) - 1;  // (no padding rows)
      return;
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int r = (ltv >> 3) + RPP * j;
      const int hy = r / W2, hx = r - hy * W2, iy = y0 + hy - 1, ix = hx - 1;
      const bool in = r >= HS || (iy >= 0 && iy < H && ix >= 0 && ix < W);
      inm |= (int)in << j;
    }
  };
  // stage loads: buffer loads (32-bit byte offset into src1, or src2 = the concatenated skip
  // input; the chunk's channel offset in soffset); past the last stage a zero-record descriptor,
  // so every reload is unconditional (a conditional one keeps the old value alive beside the new
  // one: a second register set the compiler rotates with waiting copies)
  const int nrec1 = (int)std::min<long long>((long long)a.M * a.C1 * 2, 0x7fffffffLL);
  const int nrec2 = (int)std::min<long long>((long long)a.M * a.C2 * 2, 0x7fffffffLL);
  struct Src {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t rowb, so;
  };
  auto src_of = [&](int cc, bool live) __attribute__((always_inline)) {  // scalar selects only (uniform)
    const int ci0 = cc * 64;
    const bool s1 = ci0 < a.C1;
    Src c;
    c.rs = __builtin_amdgcn_make_buffer_rsrc(s1 ? (void*)a.src1 : (void*)a.src2, (short)0,
                                             live ? (s1 ? nrec1 : nrec2) : 0, 0x00020000);
    c.rowb = (uint32_t)(s1 ? a.C1 : a.C2) * 2;
    c.so = (uint32_t)(s1 ? ci0 : ci0 - a.C1) * 2;
    return c;
  };
  // Output tile in LDS (RES): [cout half][256 px][128 B]; 16-B unit u (couts 8u .. 8u+7 of the
  // half) of pixel p at unit u ^ ((p >> 1) & 7): the MFMA waves' 8-B accesses in the accumulator
  // layout (32 pixels x 2) and the halo waves' 16-B row accesses (8 rows) both spread over all
  // banks. Halo wave hw owns cout half hw & 1 of statistics slot hw >> 1 (pixels 128 (hw >> 1) ..
  // +127): it loads the residual there and drains the output from there, so the LDS-DMA of tile
  // k's residual follows the drain of tile k-1 in the same wave (no cross-wave hazard).
  const int dh = (wid - 4) & 1, ds = (wid - 4) >> 1;
  auto res_dma = [&](int k) __attribute__((always_inline)) {
    if constexpr (RES) {
      const int tileP = tile_p(k), tileC = tile_c(k);
#pragma unroll
      for (int i = 0; i < 16; ++i) {  // rows 128 ds + 8 i + lane / 8; LDS unit lane % 8 <- source unit u
        const int row = 128 * ds + 8 * i + (lane >> 3), u = (lane & 7) ^ ((row >> 1) & 7);
        // (C96: units 6, 7 of a half are past its 48 couts -- those lanes load unit 0 again, never read)
        const int us = (C96 && u >= HB / 8) ? 0 : u;
        const T* src = (const T*)a.resid + (size_t)(tileP + row) * a.Cout + tileC + dh * HB + us * 8;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(rlds + dh * 32768 + (128 * ds + 8 * i) * 128), 16, 0, 0);
      }
    }
  };
  // tile kd's output: LDS -> HBM (16 B a lane), and its GroupNorm statistics: lane (r = lane / 8,
  // u = lane % 8) sums couts 8u .. 8u+7 over rows r, r+8, .., then the 8 lanes of a unit halve
  // their 16 sums three times (fixed order: deterministic); lane (b3, b4, b5) = bits 3..5 keeps
  // sum (b3 = 0) or sum of squares of couts 8u + 4 b4 + 2 b5 + {0, 1}
  auto drain = [&](int kd) __attribute__((always_inline)) {
    if constexpr (RES) {
      // (lane from an opaque copy: the row / unit addresses are rebuilt per call, not held in registers
      // across the whole stage loop for the final drain -- they spilled to scratch)
      int lane = tid & 63;
      asm volatile("" : "+v"(lane));
      const int tileP = tile_p(kd), tileC = tile_c(kd), u = lane & 7, dph = tile_ph(kd);
      // statistics slots: 128 pixels (one a wave half), or 64 at the 8x8 level (COMPACT RES: two a wave half)
      constexpr int NH = NSEG == 4 ? 2 : 1;
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) {
        float v[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = 0.f;
#pragma unroll
        for (int i = hf * 16 / NH; i < (hf + 1) * 16 / NH; ++i) {
          const int row = 128 * ds + 8 * i + (lane >> 3);
          u32x4 d = *(const u32x4*)(rlds + dh * 32768 + row * 128 + ((u ^ ((row >> 1) & 7)) << 4));
          if (!C96 || u < HB / 8) *(u32x4*)((T*)a.out + orow(tileP + row, dph) * a.Cout + tileC + dh * HB + u * 8) = d;
          else d = u32x4{0u, 0u, 0u, 0u};  // (C96: no such couts; zeros through the statistics butterfly)
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const float lo = __uint_as_float(d[w] << 16), hi = __uint_as_float(d[w] & 0xffff0000u);
            v[2 * w] += lo;
            v[2 * w + 1] += hi;
            v[8 + 2 * w] = fmaf(lo, lo, v[8 + 2 * w]);
            v[8 + 2 * w + 1] = fmaf(hi, hi, v[8 + 2 * w + 1]);
          }
        }
        if (a.stats) {
          auto xchg = [&](float x, auto wc) {
            constexpr int w = decltype(wc)::value;
            const int xi = __builtin_bit_cast(int, x);
            int r;
            if constexpr (w == 8) r = __builtin_amdgcn_update_dpp(0, xi, 0x128, 0xF, 0xF, false);  // row_ror:8
            else if constexpr (w == 16) r = __builtin_amdgcn_ds_swizzle(xi, 0x1F | (16 << 10));
            else r = __builtin_amdgcn_ds_bpermute((lane ^ 32) << 2, xi);
            return __builtin_bit_cast(float, r);
          };
          auto halve = [&](auto wc, int n) {
            const bool up = (lane & decltype(wc)::value) != 0;
#pragma unroll
            for (int ii = 0; ii < 8; ++ii) {
              if (ii < n) {
                const float lo = v[ii], hi = v[ii + n];
                v[ii] = (up ? hi : lo) + xchg(up ? lo : hi, wc);
              }
            }
          };
          halve(std::integral_constant<int, 8>{}, 8);
          halve(std::integral_constant<int, 16>{}, 4);
          halve(std::integral_constant<int, 32>{}, 2);
          long long slot = NH == 1 ? (long long)tileP / 128 + ds : ((long long)tileP + 128 * ds + 64 * hf) / 64;
          if constexpr (SUB) {  // (image, phase, 128-pixel slot of the phase image): the 2x grid has 4x the slots
            const int HWi = H * W, spp = HWi / 128, img = tileP / HWi;
            slot = (long long)img * 4 * spp + dph * spp + (tileP - img * HWi) / 128 + ds;
          }
          const int co = dh * HB + 8 * u + 4 * ((lane >> 4) & 1) + 2 * (lane >> 5);
          if (!C96 || u < HB / 8) *(float2*)(a.stats + (slot * 2 + ((lane >> 3) & 1)) * a.Cout + tileC + co) = float2{v[0], v[1]};
        }
      }
    }
  };
  // the stage being loaded: tile kL, chunk ccL (the emitted stage is the one before it)
  int kL = 0, ccL = 0;
  u32x4 h[ITEMS];
  f32x4 c[4], cn[4];
  // the loaded stage's coefficients c from cn: gn_coef rows (a0..a7, b0..b7), or (gn_fold) gamma0..7,
  // beta0..7 with the group statistics in gsw: a = rstd gamma, b = beta - mean a (gn_coef_kernel's formula)
  auto prescale = [&]() __attribute__((always_inline)) {  // scalar multiplies (packed f32 is costly here)
    if constexpr (PLAIN) return;  // plain conv: no GroupNorm coefficients
    if (a.gn_fold) {
      // group of channel c = floor((c + 0.5) / gsz) by a reciprocal (exact: c < 2^11, gsz <= 64)
      const int c0 = ccL * 64 + 8 * lch;
      const float rg = 32.0f / (float)Cin;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int g = (int)(((float)(c0 + e) + 0.5f) * rg);
        const float mean = gsw[2 * g], rstd = gsw[2 * g + 1];
        const float sc = rstd * cn[e >> 2][e & 3];
        c[e >> 2][e & 3] = sc * GN_L2E;
        c[2 + (e >> 2)][e & 3] = (cn[2 + (e >> 2)][e & 3] - mean * sc) * GN_L2E;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) c[q][e] = cn[q][e] * GN_L2E;
    }
  };
  auto load_cn = [&](int ccx) __attribute__((always_inline)) {  // (stage coefficients or affine, as above)
    if constexpr (PLAIN) return;
    if (a.gn_fold) {
      const int c0 = ccx * 64 + 8 * lch;
      cn[0] = *(const f32x4*)(a.gn_gamma + c0);
      cn[1] = *(const f32x4*)(a.gn_gamma + c0 + 4);
      cn[2] = *(const f32x4*)(a.gn_beta + c0);
      cn[3] = *(const f32x4*)(a.gn_beta + c0 + 4);
    } else {
      const f32x4* cp = (const f32x4*)(cbase + ccx * 128);
#pragma unroll
      for (int q = 0; q < 4; ++q) cn[q] = cp[q];
    }
  };
  // transform the emitted stage (items in h, coefficients in c) into hbuf; each item's register
  // is reloaded with the loaded stage's item right after its transform; that stage's
  // coefficients go to cn first (older than every item reload: waiting for them never waits for
  // an item).
  auto emit = [&](char* hbuf) __attribute__((always_inline)) {
    if (ccL == 0) geometry_emit(kL);  // the emitted stage opens tile kL
    bool opened = false;
    if (++ccL == ncc) {
      ccL = 0;
      if (++kL < ntiles) {
        geometry_pix(kL);
        opened = true;
      }
    }
    const bool live = kL < ntiles;
    load_cn(live ? ccL : 0);
    const Src nx = src_of(ccL, live);
    typedef __attribute__((ext_vector_type(2))) float f32x2;
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t zm = (uint32_t)__builtin_amdgcn_sbfe(inm, j, 1);  // 0 (padding) or ~0
      uint32_t yw[4];
      if constexpr (PLAIN) {
#pragma unroll
        for (int w = 0; w < 4; ++w) yw[w] = h[j][w] & zm;
      } else
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)  // channels 4hf .. 4hf+3: words 2hf, 2hf+1
        gn_silu_x4(h[j][2 * hf], h[j][2 * hf + 1], c[hf][0], c[hf][1], c[hf][2], c[hf][3], c[2 + hf][0],
                   c[2 + hf][1], c[2 + hf][2], c[2 + hf][3], zm, yw[2 * hf], yw[2 * hf + 1]);
      const u32x4 y = {yw[0], yw[1], yw[2], yw[3]};
      *(u32x4*)(hbuf + waddr(j)) = y;
      __builtin_amdgcn_sched_barrier(0);
      h[j] = __builtin_amdgcn_raw_buffer_load_b128(nx.rs, __umul24((uint32_t)ipix[j], nx.rowb) + lch * 16, nx.so, 0);
    }
    // gn_fold: a tile opened -- its image's group statistics (loads issued after the item reloads; the
    // wait also covers those, inside the current MFMA stage)
    if (a.gn_fold && opened && simg != gimg) {
      group_stats(simg);
      gimg = simg;
    }
    prescale();
  };
  // prologue: stage 0 (and tile 0's addv)
  geometry_pix(0);
  {
    load_cn(0);
    const Src s0 = src_of(0, true);
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      h[j] = __builtin_amdgcn_raw_buffer_load_b128(s0.rs, __umul24((uint32_t)ipix[j], s0.rowb) + lch * 16, s0.so, 0);
    if (a.gn_fold) group_stats(simg);  // (its loads in flight with stage 0's)
    gimg = simg;
    prescale();
  }
  if constexpr (COMPACT) {  // the zero row of both halo buffers (no stage writes it; read after B0)
    if (tt < 16) *(u32x4*)(smem + (tt >> 3) * HALO + ZROW * ROWB + ((tt & 7) << 4)) = u32x4{0u, 0u, 0u, 0u};
    if (M16 && ITSD_P4_ZR8) {  // rows ZROW + 0..7 and + 64..71 of both buffers: one 16-B unit a thread
      const int r = (tt >> 3) & 15;
      *(u32x4*)(smem + (tt >> 7) * HALO + (ZROW + (r & 7) + (r >> 3) * 64) * ROWB + ((tt & 7) << 4)) = u32x4{0u, 0u, 0u, 0u};
    } else if (M16 && tt >= 16 && tt < 32) {
      *(u32x4*)(smem + ((tt >> 3) & 1) * HALO + (ZROW + 64) * ROWB + ((tt & 7) << 4)) = u32x4{0u, 0u, 0u, 0u};
    }
  }
  emit(smem);
#ifdef ITSD_STAMPS
  st[5] = stamp() - t_begin;
#endif
  block_sync();  // B0
  for (int q = 0, k = 0, cc = 0; q < nstages; ++q) {  // during MFMA stage q = (tile k, chunk cc)
    STAMP(h0);
    // tile k's residual, during its last chunk (issued before the item reloads: the wait below
    // for it leaves them in flight); tile k+1's addv with its first chunk
    if (RES && cc == 1 && k > 0) {  // tile k-1's output (written before MFMA stage (k, 0))
      drain(k - 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read out before the residual DMA lands
    }
    const bool res = RES && a.resid && cc == ncc - 1;
    if (res) res_dma(k);
    // tile k+1's addv: RES tiles seed their accumulators from it after tile k (its other parity
    // was last read when tile k-1 started), so it is staged with tile k's FIRST chunk, away from
    // the last chunk's residual DMA and drain (at two chunks per tile that stage carried them all);
    // the register epilogue (8x8) still reads parity k+1 = k-1 during chunk 0, so it waits for the last
    const int addv_cc = RES ? 0 : ncc - 1;
    if (cc == addv_cc && k + 1 < ntiles) stage_addv(k + 1, tt);
    if (q + 1 < nstages) emit(smem + ((q + 1) & 1) * HALO);
    // the residual DMA has landed (only the next stage's coefficient loads and item reloads, all
    // issued after it, may still be in flight)
    if (res) {  // (last stage: nothing was issued after the DMA)
      if (q + 1 < nstages) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ITEMS + 4) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#ifdef ITSD_STAMPS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
    STAMP(h1);
    STAMP_ADD(3, h1 - h0);
    block_sync();  // end of MFMA stage q
    if (++cc == ncc) {
      cc = 0;
      ++k;
    }
  }
  if constexpr (RES) {
    block_sync();  // the last tile's output is in LDS
    drain(ntiles - 1);
  }
  P4_STAMP_OUT();
}

// ---------------------------------------------------------------------------- small levels, split-K persistent
// conv3x3_gn_p5_kernel<W>: the fused GroupNorm+SiLU+conv3x3 (Model.py:170-174,179-184) of the 8x8
// and 4x4 levels (W = 8, 4), whose tiles hold whole images. At N = 256 the 4x4 level has only
// 4096 pixels: 128-pixel x 64-cout tiles with the whole K per block (conv_small) spend their time
// in a 72..144-stage K loop at 9-14 % MFMA busy, and with p4's 256 x 128 tiles only 64 tiles exist.
// Here a work item is (128-pixel tile = 8 / 2 whole images, 128 couts, K slice):
//   * 4 MFMA waves, wave w = couts 32w .. 32w+31 x all 128 pixels (one A fragment and four B
//     fragments per k-step: 4 v_mfma_f32_32x32x16_bf16), A streamed from wfrag into a 9-slot
//     register ring across chunk and item boundaries, B from a double-buffered LDS halo;
//   * 4 halo waves stage the next 64-channel chunk while the MFMA waves compute the current one
//     (p4's software pipeline): only the tile's INTERIOR pixels are loaded (16 B a lane, one
//     image's GroupNorm coefficients per lane), GroupNorm+SiLU'd and written; the padding rows of
//     both halo buffers are zeroed once per launch (whole-image tiles: the same rows every item);
//   * K split into S slices (items = tiles x S, S from a cost model so the items fill the 256
//     CUs): each MFMA wave of a slice stores its fp32 partial (64 accumulators a lane) to a slab,
//     releases it at agent scope and takes a ticket on a per-(tile, wave) counter; the wave that
//     draws S-1 acquires, sums the partials in slice order 0..S-1 (deterministic whichever slice
//     arrives last, correct for any placement over XCDs), resets the counter and runs the epilogue;
//   * register epilogue: + bias/temb (+ CFG cond) rows staged in LDS by the halo waves + residual
//     from HBM, one bf16 rounding, 16-B stores (permlane32 swap), and the consumer GroupNorm's
//     statistics slots (one per image at 4x4, one per image at 8x8) by lane butterflies;
//   * ragged batches: images past the batch load zeros (buffer-descriptor bound) and store nothing.
// Tiles of whole images (W <= 8: NSEG = 128 / HW images, "interior" halo mode: only the images'
// own pixels are loaded, the padding ring is zeroed once) or of TH = 128 / W rows of one image
// (W = 16 / 32, "rows" mode: the rows above and below the tile are loaded too, masked to zero where
// they fall outside the image; the padding columns are zeroed once).
template <int W> struct Gp5Cfg {
  static constexpr int HW = W * W;
  static constexpr bool ROWS = HW > 128;
  static constexpr int TH = ROWS ? 128 / W : W, NSEG = ROWS ? 1 : 128 / HW, W2 = W + 2, HS = (TH + 2) * W2;
  static constexpr int HY0 = ROWS ? 0 : 1, NHY = ROWS ? TH + 2 : TH;  // halo rows loaded per segment
  static constexpr int TPS = 256 / NSEG, RPP = TPS / 8, ITEMS = NHY * W / RPP;
  static constexpr int HALO = ((NSEG * HS * ROWB) + 1023) & ~1023;  // one halo buffer (bytes)
};
#ifndef ITSD_P5_RING
#define ITSD_P5_RING 9
#endif
#ifndef ITSD_P5_BD
#define ITSD_P5_BD 3
#endif
constexpr int P5_RING = ITSD_P5_RING;  // A k-step slots (prefetch distance 8 k-steps = 32 MFMAs); divides 36
                            // (12 and 18 measured equal at N = 32 and 256)
constexpr int P5_BD = ITSD_P5_BD;    // B fragment buffers (reads two k-steps = 8 MFMAs ahead)
// (round 5: the MFMA waves on v_mfma_f32_16x16x32_bf16 as in p4 -- 2 x 8 f32x4 accumulators, 6-slot k32 A ring, 8-B
// stores, per-slot butterflies over the 16 pixel lanes -- measured N = 256 equal, N = 32 +2.3 %, N = 64 +0.7 %, C4
// +0.7 % step time against this form, profiles/r05/step_p5_m16_vs_m32.txt: removed)

// CB (round 6): couts per item, 128 or 64 (W <= 8: a statistics slot never spans the two pixel halves). With 64-cout
// items waves w and w + 2 share a 32-cout block and each takes two of the four 32-pixel blocks: the same k order per
// output and the same statistics tree, so the forward is bit-identical to 128-cout items; twice the items at the same
// K slices -- the 4x4 level at N = 256 fills the 256 CUs without splitting K (128 tiles of 128 couts)
// DIST (round 6): the split-K combine shared by every slice (ConvArgs::kdist; a separate instantiation, so the
// last-arriver form's code is the round-5 kernel's: sharing one body cost its launches 5 % at N = 256,
// profiles/r06/census_r05lib_vs_r06_r06k.txt)
template <int W, int CB = 128, bool DIST = false>
__global__ __launch_bounds__(512, 1) void conv3x3_gn_p5_kernel(ConvArgs a) {
  typedef bf16_t T;
  using Cf = Gp5Cfg<W>;
  static_assert(CB == 128 || (CB == 64 && W <= 8), "p5 cout tile");
  static_assert(!DIST || CB == 128, "shared combine: 128-cout items");
  constexpr int CWB = CB / 32, NJW = CWB;  // 32-cout blocks a tile; 32-pixel blocks a wave (4 waves: CWB x 4 / CWB)
  constexpr int HW = Cf::HW, NSEG = Cf::NSEG, W2 = Cf::W2, HS = Cf::HS, TPS = Cf::TPS, RPP = Cf::RPP;
  constexpr int ITEMS = Cf::ITEMS, HALO = Cf::HALO, TH = Cf::TH, HY0 = Cf::HY0, NHY = Cf::NHY;
  constexpr int SPX = TH * W;  // pixels of one segment
  // halo row (hy, hx) -> its 16-B units XOR-permuted by swz: ds_read_b128 serves the MFMA waves' B reads in 16-lane
  // groups ({0-3, 12-15, 20-27}, ...) of 16 pixels, which at W <= 16 span 2-4 image rows of a segment, non-contiguous
  // halo rows; (h >> 1) & 7 left 37 % (W = 4 / 8) and 12 % (W = 16) of those lanes on a taken bank slot -- the p5<4>
  // launch's 4.8e6 conflict cycles (profiles/r05/pmc_dispatch_table_r05ae.txt). A slot is (hx & 1, swz) (W2 even);
  // these keep every group of every tap on 16 distinct slots (exhaustive check: tools/halo_swizzle.py --p5)
  constexpr int SC1 = 1, SC2 = W <= 8 ? 2 : 1;
  auto swz = [](int hy, int hx, int h) { return W <= 16 && ITSD_P5_SWZ ? (SC1 * hy + SC2 * hx) & 7 : (h >> 1) & 7; };
  static_assert(NSEG * SPX == 128 && ITEMS * RPP == NHY * W && ITEMS <= 31 && 36 % P5_RING == 0, "p5 geometry");
  constexpr int SEGW = 64 / TPS > 0 ? 64 / TPS : 1;  // image segments one halo wave covers (W = 4: 2)
  // + the residual tiles of two items [item parity][128 px][128 couts] bf16 (LDS-DMA'd by the halo waves
  // during an item's last stage; 16-B unit u of pixel p at u ^ (p & 15))
  constexpr int RTILE = 128 * CONV_BM * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * HALO + 2 * NSEG * CONV_BM * 4 + 4 * 2 * SEGW * 64 * 4 + 2 * RTILE];
  float* const addv = (float*)(smem + 2 * HALO);  // [item parity][image of the tile][128 couts]
  char* const rres = smem + 2 * HALO + 2 * NSEG * CONV_BM * 4 + 4 * 2 * SEGW * 64 * 4;
  // gn_fold: per halo wave, [item parity][segment of the wave][32 groups][mean, rstd]
  float* const gsw_all = (float*)(smem + 2 * HALO + 2 * NSEG * CONV_BM * 4);
  TL(0);
#ifdef ITSD_STAMPS
  {  // timeline: the SIMD each wave runs on (HW_ID.SIMD_ID) -> stamp slot [block][8 + wave][0]
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (4 << 6) | (1 << 11));
    if ((threadIdx.x & 63) == 0) g_stamps[((blockIdx.x & 1023) * 16 + 8 + (threadIdx.x >> 6)) * 8] = hw;
  }
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Cin = a.C1 + a.C2, nch = Cin / 64, kpt = Cin >> 4;
  const int nimg = a.M / HW, nTP = Cf::ROWS ? a.M / 128 : (nimg + NSEG - 1) / NSEG;
  const int nTC = a.Cout / CB, S = a.ksplit;
  // (folded 1x1 shortcut: slices S .. ST-1 run the shortcut's K over its own input, nchx 64-channel chunks)
  const int S2 = a.sc_split, ST = S + S2, nchx = (a.sc_C1 + a.sc_C2) / 64;
  const int NI = nTP * nTC * ST;
  const int G = gridDim.x, b = blockIdx.x;
  // XCD-aware: the dispatcher deals block ids round-robin over the 8 XCDs; XCD x takes the
  // contiguous logical range, in which items sharing a (cout tile, slice) -- its weights -- are adjacent
  const int bl = (G & 7) ? b : (b & 7) * (G >> 3) + (b >> 3);
  const int nit = bl < NI ? (NI - 1 - bl) / G + 1 : 0;
  if (nit == 0) return;  // (the host launches gridDim.x <= items)
  // item k of this block -> pixel tile tp (fastest), K slice z, cout tile tc; XCD-local exchange (kxl): K slice
  // fastest, so that a tile's slices are adjacent items on one XCD
  const bool xl = a.kxl != 0;
  const int d1 = xl ? ST : nTP, d2 = xl ? nTP : ST;  // the fastest index's extent, then the next one's
  auto item_of = [&](int k, int& tp, int& tc, int& z) {
    const int L = bl + k * G;
    const int i1 = L % d1, r = L / d1, i2 = r % d2;
    tp = xl ? i2 : i1;
    z = xl ? i1 : i2;
    tc = r / d2;
  };
  // chunk range [lo, hi) of slice z: the 3x3 conv's Cin / 64 chunks over slices 0 .. S-1, the shortcut's over S ..
  auto chunk_lo = [&](int z) { return z < S ? (nch * z) / S : (nchx * (z - S)) / S2; };
  auto chunk_hi = [&](int z) { return z < S ? (nch * (z + 1)) / S : (nchx * (z + 1 - S)) / S2; };
  auto block_sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  if (wid < 4) {
    // ================================================================ MFMA waves
    const int rl = lane & 31, hh = lane >> 5;
    const int cw = CB == 128 ? wid : wid % CWB, jb0 = CB == 128 ? 0 : (wid / CWB) * NJW;  // its 32-cout block, first px block
    int hb[NJW];  // halo row of this lane's pixel (tap 0, 0) in each of its 32-pixel blocks
    int hq[NJW];  // its swz coordinates SC1 y + SC2 x (W <= 16)
#pragma unroll
    for (int j = 0; j < NJW; ++j) {
      const int pl = (jb0 + j) * 32 + rl, seg = pl / SPX, rem = pl - seg * SPX, y = rem / W;
      hb[j] = seg * HS + y * W2 + (rem - y * W);
      hq[j] = SC1 * y + SC2 * (rem - y * W);
    }
    // B unit of pixel block j at tap (ky, kx): halo row h = hb[j] + ky W2 + kx, hy = y + ky, hx = x + kx
    auto bunit = [&](int j, int h, int ky, int kx) {
      return W <= 16 && ITSD_P5_SWZ ? (hq[j] + SC1 * ky + SC2 * kx) & 7 : (h >> 1) & 7;
    };
    const uint32_t ablk = (uint32_t)(9 * kpt) * 1024;  // one 32-cout block of fragments
    // A fragments by buffer loads (conv3x3_gn_p4_kernel's scheme): voffset = this lane's 16 B of the wave's
    // 32-cout block, soffset = the tile's fragment block + chunk + k-step (uniform scalar arithmetic)
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.wfrag, (short)0, 0x7fffffff, 0x00020000);
    const uint32_t avo = (uint32_t)lane * 16 + (uint32_t)cw * ablk;
    auto abase = [&](int tc, int cc) -> uint32_t { return (uint32_t)(tc * CWB) * ablk + (uint32_t)cc * 4 * 1024; };
    auto load_a = [&](uint32_t base, int st, u32x4& dst) __attribute__((always_inline)) {
#if defined(ITSD_DIAG) && defined(P5_AB)
      if constexpr ((P5_AB & 8) != 0) {  // ablation: no A loads
        dst = u32x4{(uint32_t)st, 0u, 0u, 0u};
        return;
      }
#endif
      dst = __builtin_amdgcn_raw_buffer_load_b128(wrs, avo, base + (uint32_t)((st >> 2) * kpt + (st & 3)) * 1024, 0);
    };
    f32x16 acc[NJW];
    u32x4 ra[P5_RING];
    // the folded shortcut's A fragments: voffset = this lane's 16 B, soffset = the wave's 32-cout block + chunk + k-step
    const __amdgpu_buffer_rsrc_t wrx = __builtin_amdgcn_make_buffer_rsrc((void*)a.sc_wfrag, (short)0, 0x7fffffff, 0x00020000);
    const uint32_t ablkx = (uint32_t)(nchx * 4) * 1024;
    auto load_ax = [&](int tc, int cc, int st, u32x4& dst) __attribute__((always_inline)) {
      dst = __builtin_amdgcn_raw_buffer_load_b128(wrx, (uint32_t)lane * 16,
                                                  (uint32_t)(tc * CWB + cw) * ablkx + (uint32_t)(cc * 4 + st) * 1024, 0);
    };
    bool ring = false;  // ra[0 .. P5_RING-2] hold the next 3x3 item's first k-steps
    {
      int tp, tc, z;
      item_of(0, tp, tc, z);
      if (z < S) {
        const uint32_t ab0 = abase(tc, chunk_lo(z));
#pragma unroll
        for (int s0 = 0; s0 < P5_RING - 1; ++s0) load_a(ab0, s0, ra[s0]);
        ring = true;
      }
    }
    block_sync();  // B0: stage 0 staged
    TL(1);
    int q = 0;
    for (int k = 0; k < nit; ++k) {
      int tp, tc, z;
      item_of(k, tp, tc, z);
      const int c0 = chunk_lo(z), c1 = chunk_hi(z);
#pragma unroll
      for (int j = 0; j < NJW; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
#if defined(ITSD_DIAG) && defined(P5_CHAINS2)  // diagnostic: 8 accumulation chains (odd k-steps apart)
      f32x16 acc2[NJW];
#pragma unroll
      for (int j = 0; j < NJW; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc2[j][r] = 0.0f;
#endif
      if (z >= S) {
        // ---- a folded-shortcut slice: the centre tap of the raw input chunks the halo waves stage, 4 k-steps
        // a chunk; chunk cc + 1's A fragments load during chunk cc (ra[0..3] / ra[4..7] by chunk parity)
#pragma unroll
        for (int st = 0; st < 4; ++st) load_ax(tc, c0, st, ra[st]);
        auto chunk1 = [&](auto pc, int cc) __attribute__((always_inline)) {
          constexpr int P = decltype(pc)::value;
          if (cc + 1 < c1) {
#pragma unroll
            for (int st = 0; st < 4; ++st) load_ax(tc, cc + 1, st, ra[4 * (1 - P) + st]);
          }
          int tx[NJW];
#pragma unroll
          for (int j = 0; j < NJW; ++j) {
            const int h = hb[j] + W2 + 1;
            tx[j] = (q & 1) * HALO + h * ROWB + ((hh ^ bunit(j, h, 1, 1)) << 4);
          }
#pragma unroll
          for (int st = 0; st < 4; ++st) {
            bf16x8 fx[NJW];
#pragma unroll
            for (int j = 0; j < NJW; ++j) fx[j] = *(const bf16x8*)(smem + (tx[j] ^ (st << 5)));
            const bf16x8 af = __builtin_bit_cast(bf16x8, ra[4 * P + st]);
#pragma unroll
            for (int j = 0; j < NJW; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, fx[j], acc[j], 0, 0, 0);
          }
          block_sync();  // end of stage q: its halo buffer is free, stage q+1 is published
          ++q;
        };
        for (int cc = c0; cc < c1; cc += 2) {
          chunk1(std::integral_constant<int, 0>{}, cc);
          if (cc + 1 < c1) chunk1(std::integral_constant<int, 1>{}, cc + 1);
        }
        ring = false;
      } else {
      if (!ring) {  // (after a shortcut slice) the ring's first k-steps
        const uint32_t ab0 = abase(tc, c0);
#pragma unroll
        for (int s0 = 0; s0 < P5_RING - 1; ++s0) load_a(ab0, s0, ra[s0]);
      }
      uint32_t nitem = abase(tc, c1 - 1);  // the next item's first chunk (A prefetch across the item boundary)
      ring = false;
      if (k + 1 < nit) {
        int tp2, tc2, z2;
        item_of(k + 1, tp2, tc2, z2);
        if (z2 < S) {
          nitem = abase(tc2, chunk_lo(z2));
          ring = true;
        }
      }
      for (int cc = c0; cc < c1; ++cc, ++q) {
        const char* hcur = smem + (q & 1) * HALO;
        const uint32_t cb = abase(tc, cc);
        const uint32_t nb = cc + 1 < c1 ? abase(tc, cc + 1) : nitem;
        int tb[NJW];
        bf16x8 fb[P5_BD][NJW];
        auto rd = [&](int st, int buf) __attribute__((always_inline)) {
          if ((st & 3) == 0) {
            const int tap = st >> 2, ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
            for (int j = 0; j < NJW; ++j) {
              int h = hb[j] + ky * W2 + kx;
              asm volatile("" : "+v"(h));  // rebuilt per tap, not hoisted out of the chunk loop
              tb[j] = (int)(hcur - smem) + h * ROWB + ((hh ^ bunit(j, h, ky, kx)) << 4);
            }
          }
#if defined(ITSD_DIAG) && defined(P5_AB)
          if constexpr ((P5_AB & 16) != 0) {  // ablation: no B reads
#pragma unroll
            for (int j = 0; j < NJW; ++j) fb[buf][j] = bf16x8{(short)(st + j), 0, 0, 0, 0, 0, 0, 1};
            return;
          }
#endif
#pragma unroll
          for (int j = 0; j < NJW; ++j) fb[buf][j] = *(const bf16x8*)(smem + (tb[j] ^ ((st & 3) << 5)));
        };
#pragma unroll
        for (int s0 = 0; s0 < P5_BD - 1; ++s0) rd(s0, s0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int step = 0; step < 36; ++step) {
          const int pf = step + P5_RING - 1;
          if (pf < 36) load_a(cb, pf, ra[pf % P5_RING]);
          else load_a(nb, pf - 36, ra[pf % P5_RING]);
          if (step + P5_BD - 1 < 36) rd(step + P5_BD - 1, (step + P5_BD - 1) % P5_BD);
          const bf16x8 af = __builtin_bit_cast(bf16x8, ra[step % P5_RING]);
#pragma unroll
          for (int j = 0; j < NJW; ++j)
#if defined(ITSD_DIAG) && defined(P5_CHAINS2)
            if (step & 1) acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, fb[step % P5_BD][j], acc2[j], 0, 0, 0);
            else
#endif
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, fb[step % P5_BD][j], acc[j], 0, 0, 0);
          // (round 5) the step's A load, B reads and address VALU spread over its 4 MFMA gaps, as in
          // conv3x3_gn_p4_kernel, instead of all of them ahead of the MFMAs: the tap-boundary address
          // rebuilds no longer stall the matrix pipe
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (q == 0) TL(6);
        block_sync();  // end of stage q: its halo buffer is free, stage q+1 is published
        if (q == 0) TL(7);
      }
      }  // (3x3 slice)
#if defined(ITSD_DIAG) && defined(P5_CHAINS2)
#pragma unroll
      for (int j = 0; j < NJW; ++j) acc[j] += acc2[j];
#endif
      TL(2);
      // ---- split-K: partial out, ticket; the last slice of this (tile, wave) combines (or every slice its own units)
      const int tile = tc * nTP + tp;
      if (ST > 1) {
        // Guideline 16's R1 hand-off, per wave: the partial is stored write-through (sc1), the wave
        // drains its stores, then adds to its (tile, wave) counter; the wave whose add returns S-1 reads
        // every partial with sc1 loads (past its own L1) -- no release / acquire fence, whose L2
        // write-back / L1 invalidate cost ~2-7 us per episode (MI355X_MICROARCH.md, visibility table)
        const __amdgpu_buffer_rsrc_t slab = __builtin_amdgcn_make_buffer_rsrc(
            a.splitk_ws, (short)0, (int)std::min<long long>(a.splitk_cap * 4, 0x7fffffffLL), 0x00020000);
        // slab [tile][slice][wave][NJW x 4 KB] (a wave's NJW pixel blocks x 4 cout groups of 1 KB)
        const uint32_t wbase = (uint32_t)(((size_t)tile * ST * 4 + wid) * NJW * 4096) + lane * 16;
        const uint32_t zstride = 4 * NJW * 4096;  // bytes between the slices of one (tile, wave)
        auto store_partial = [&]() __attribute__((always_inline)) {
          if (xl) {  // (into this XCD's L2)
#pragma unroll
            for (int j = 0; j < NJW; ++j)
#pragma unroll
              for (int g = 0; g < 4; ++g)
                __builtin_amdgcn_raw_buffer_store_b128(
                    u32x4{__float_as_uint(acc[j][4 * g]), __float_as_uint(acc[j][4 * g + 1]),
                          __float_as_uint(acc[j][4 * g + 2]), __float_as_uint(acc[j][4 * g + 3])},
                    slab, wbase + z * zstride + (j * 4 + g) * 1024, 0, 0);
          } else {  // (sc1: through to memory)
#pragma unroll
            for (int j = 0; j < NJW; ++j)
#pragma unroll
              for (int g = 0; g < 4; ++g)
                __builtin_amdgcn_raw_buffer_store_b128(
                    u32x4{__float_as_uint(acc[j][4 * g]), __float_as_uint(acc[j][4 * g + 1]),
                          __float_as_uint(acc[j][4 * g + 2]), __float_as_uint(acc[j][4 * g + 3])},
                    slab, wbase + z * zstride + (j * 4 + g) * 1024, 0, 16);
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        };
        // a partial of this tile: sc0 (past L1, from this XCD's L2) under kxl, else sc1
        auto load_partial = [&](uint32_t o) __attribute__((always_inline)) {
          return xl ? __builtin_amdgcn_raw_buffer_load_b128(slab, o, 0, 1) : __builtin_amdgcn_raw_buffer_load_b128(slab, o, 0, 16);
        };
        // this wave's XCC_ID (HW_REG_XCC_ID bits 3:0): reported with the arrival under kxl
        const int xcc = xl ? (int)(__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)) & 7) : 0;
        // (round 6) two slices, last-arriver form: arrival first; only the FIRST arriver stores its partial, the
        // last one adds it to its own from registers (p0 + p1 == p1 + p0 in IEEE arithmetic: bit-identical to the
        // slice-order sum). At N = 256's 4x4 level (256 items, S = 2) every block's combine runs at once and is
        // bound by the slab bytes (16.8 MB written + 16.8 MB read a launch, ~7.5 us of the 45 us launch,
        // profiles/r05/p5_timeline_n256_r05am.txt op 36): half of each
        const bool pub2 = !DIST && a.kpub && ST == 2;  // (option p5_pub; 0: both slices publish, round 5)
        if (!pub2) store_partial();
        if constexpr (DIST) {
          // ---- the combine shared by all ST slices (every block runs one item: the grid is co-resident). The wave's
          // 16 (pixel block j, cout group g) units of 32 px x 8 couts form NU statistics units of NJ pixel blocks (one
          // consumer GroupNorm slot each: W = 4 a half block, W = 8 a pair, W >= 16 the tile); slice z finishes units
          // u = z, z + ST, ... (u = jg * 4 + g, j = jg NJ + jj): it waits until all ST partials of its (tile, wave) are
          // stored, sums each unit's ST partials in slice order and runs the epilogue for those units. Counter (one
          // 128-B line per (tile, wave): 512 waves polling a few shared lines serialise at their memory channel):
          // arrivals in the low 16 bits, departures in the high ones; the last departure resets it to 0 (the tickets
          // are zero between launches, as with the last-arriver form). One slab round trip per 8 KB instead of ST
          // serial ones in one block (30 us of a 56 us 4x4 launch at N = 32, ST = 8: profiles/r05/
          // p5_timeline_n32_r05am.txt). Bit-identical to the last-arriver combine: the same slice order, the same
          // statistics tree (per lane over j, then lane pairs by bits 16 / 8 / 4 / 2 / 1 of the pixel lane). (The
          // unrolled epilogue below with per-unit store / statistics masks instead measured slower: its register
          // pressure spilled the staging, profiles/r06/p5_timeline_n32_shared_r06c.txt.)
          constexpr int NJ = W == 4 ? 1 : W == 8 ? 2 : 4, NU = 16 / NJ;
          int* const tk = a.tickets + (tile * 4 + wid) * 32;  // (tiles x 4 x 32 <= kTicketCap: p5_dist)
          const int nown = z < NU ? (NU - 1 - z) / ST + 1 : 0;
          if (xl && lane == 0) {  // this slice's XCD into the tile's mask (tk[1]) before its arrival
            __hip_atomic_fetch_or(tk + 1, 1 << xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
          if (nown == 0) {  // (ST > NU: no unit of its own) arrive and depart at once
            if (lane == 0) __hip_atomic_fetch_add(tk, 0x10001, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            TL(3);
            return;  // (the block's only item: nothing, such as the A ring, stays live)
          }
          int bad = 0;
          if (lane == 0) {
            int v = (__hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xffff) + 1;
            TL(3);
            for (int it = 0; v < ST && it < a.spin_bound; ++it) {  // bounded: a grid that is not co-resident cannot hang
              __builtin_amdgcn_s_sleep(2);
              v = __hip_atomic_load(tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xffff;
            }
            bad = v < ST;
            if (xl && !bad) {  // every slice on this wave's XCD (else its partial is not in this L2)
              const int msk = __hip_atomic_load(tk + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              bad = msk != (1 << xcc);
            }
            if (bad) __hip_atomic_fetch_or(a.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          bad = __builtin_amdgcn_readfirstlane(bad);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the poll)
          TL(4);  // (timeline, shared combine: 3 partial drained + arrived, 4 every slice arrived, 5 done)
          // staging: the slab loads land in registers (sc1) and go through this wave's 16 KB of free LDS (halo buffers
          // for waves 0 / 1, the unused residual tile for 2 / 3), so that runtime (fragment, slice) slots map to
          // static registers
          char* const stg = wid < 2 ? smem + wid * 16384 : rres + RTILE + (wid - 2) * 16384;
          static_assert(2 * HALO >= 2 * 16384, "p5 combine staging");
          const int tileP = tp * 128, tileC = tc * CONV_BM;
          const int nfrag = nown * NJ, F = 16 / ST;  // fragments (unit, jj) of this wave; a batch of F x ST slots
          f32x4 s4 = {0.f, 0.f, 0.f, 0.f}, q4 = {0.f, 0.f, 0.f, 0.f};
          // lane exchange with lane ^ w (as the last-arriver epilogue's statistics: DPP within a row, else swizzle)
          auto xchg = [](float x, auto wc) {
            constexpr int w = decltype(wc)::value;
            const int xi = __builtin_bit_cast(int, x);
            int r;
            if constexpr (w == 1) r = __builtin_amdgcn_update_dpp(0, xi, 0xB1, 0xF, 0xF, false);
            else if constexpr (w == 2) r = __builtin_amdgcn_update_dpp(0, xi, 0x4E, 0xF, 0xF, false);
            else if constexpr (w == 8) r = __builtin_amdgcn_update_dpp(0, xi, 0x128, 0xF, 0xF, false);
            else r = __builtin_amdgcn_ds_swizzle(xi, 0x1F | (w << 10));
            return __builtin_bit_cast(float, r);
          };
          auto bfly = [&](auto wc) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              s4[e] += xchg(s4[e], wc);
              q4[e] += xchg(q4[e], wc);
            }
          };
          for (int f0 = 0; f0 < nfrag; f0 += F) {
            const int nl = std::min(F, nfrag - f0) * ST;
            int fr = f0, sl = 0;  // the next slot's fragment and slice (uniform, advanced slot by slot)
            auto slot_off = [&]() __attribute__((always_inline)) {
              const int u = z + ST * (fr / NJ), jj = fr - (fr / NJ) * NJ;
              const int j = (u >> 2) * NJ + jj, g = u & 3;
              const uint32_t o = wbase + sl * zstride + (uint32_t)(j * 4 + g) * 1024;
              if (++sl == ST) { sl = 0; ++fr; }
              return o;
            };
            // 8 registers: the second 8 slots' loads go out as the first 8 are written (two overlapped round trips;
            // 16 registers spilled the kernel)
            u32x4 vv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i)
              if (i < nl) vv[i] = load_partial(slot_off());
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              if (i < nl) *(u32x4*)(stg + i * 1024 + lane * 16) = vv[i];
              if (i + 8 < nl) vv[i] = load_partial(slot_off());
            }
#pragma unroll
            for (int i = 0; i < 8; ++i)
              if (i + 8 < nl) *(u32x4*)(stg + (i + 8) * 1024 + lane * 16) = vv[i];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            for (int f = 0; f < nl / ST; ++f) {
              const int frg = f0 + f, u = z + ST * (frg / NJ), jj = frg - (frg / NJ) * NJ;
              const int j = (u >> 2) * NJ + jj, g = u & 3;
              const char* p = stg + (f * ST) * 1024 + lane * 16;
              f32x4 x = *(const f32x4*)p;
              for (int s2 = 1; s2 < ST; ++s2) x += *(const f32x4*)(p + s2 * 1024);
              // epilogue of fragment (j, g): lane = pixel 32 j + rl, couts c .. c + 3
              const int pl = j * 32 + rl, seg = pl / SPX, c = wid * 32 + 8 * g + 4 * hh;
              const bool live = Cf::ROWS ? tp * 128 < a.M : tp * NSEG + seg < nimg;
              const f32x4 ad = *(const f32x4*)(addv + seg * CONV_BM + c);
              uint2 rr = *(const uint2*)(rres + pl * 256 + ((((c >> 3) ^ pl) & 15) << 4) + 8 * hh);
              if (a.resid == nullptr) rr = uint2{0u, 0u};
              const float nan = __builtin_nanf("");
              const T b0 = f2bf(bad ? nan : x[0] + ad[0] + __uint_as_float(rr.x << 16));
              const T b1 = f2bf(bad ? nan : x[1] + ad[1] + __uint_as_float(rr.x & 0xffff0000u));
              const T b2 = f2bf(bad ? nan : x[2] + ad[2] + __uint_as_float(rr.y << 16));
              const T b3 = f2bf(bad ? nan : x[3] + ad[3] + __uint_as_float(rr.y & 0xffff0000u));
              if (live)
                *(uint2*)((T*)a.out + (size_t)(tileP + pl) * a.Cout + tileC + c) =
                    uint2{(uint32_t)b0 | ((uint32_t)b1 << 16), (uint32_t)b2 | ((uint32_t)b3 << 16)};
              const float m = live ? 1.0f : 0.0f;
              const float r0 = bf2f(b0) * m, r1 = bf2f(b1) * m, r2 = bf2f(b2) * m, r3 = bf2f(b3) * m;
              s4[0] += r0; q4[0] = fmaf(r0, r0, q4[0]);
              s4[1] += r1; q4[1] = fmaf(r1, r1, q4[1]);
              s4[2] += r2; q4[2] = fmaf(r2, r2, q4[2]);
              s4[3] += r3; q4[3] = fmaf(r3, r3, q4[3]);
              if (jj == NJ - 1) {  // the unit's statistics slot is complete: lane pairs by bits (16) 8 4 2 1 of rl
                if (a.stats) {
                  if constexpr (W != 4) bfly(std::integral_constant<int, 16>{});
                  bfly(std::integral_constant<int, 8>{});
                  bfly(std::integral_constant<int, 4>{});
                  bfly(std::integral_constant<int, 2>{});
                  bfly(std::integral_constant<int, 1>{});
                  if (W == 4) {
                    const int img = tp * NSEG + 2 * j + (rl >> 4);
                    if ((rl & 15) == 0 && img < nimg) {
                      *(f32x4*)(a.stats + ((long long)img * 2) * a.Cout + tileC + c) = s4;
                      *(f32x4*)(a.stats + ((long long)img * 2 + 1) * a.Cout + tileC + c) = q4;
                    }
                  } else {
                    const long long slot = W == 8 ? tp * NSEG + (j >> 1) : tp;
                    if (rl == 0 && slot * (W == 8 ? 64 : 128) < a.M) {
                      *(f32x4*)(a.stats + (slot * 2) * a.Cout + tileC + c) = s4;
                      *(f32x4*)(a.stats + (slot * 2 + 1) * a.Cout + tileC + c) = q4;
                    }
                  }
                }
                s4 = f32x4{0.f, 0.f, 0.f, 0.f};
                q4 = f32x4{0.f, 0.f, 0.f, 0.f};
              }
            }
          }
          if (lane == 0) {  // depart; the last one resets the counter
            const int old = __hip_atomic_fetch_add(tk, 0x10000, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((old >> 16) == ST - 1) {
              if (xl) __hip_atomic_store(tk + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          TL(5);
          return;
        } else if (pub2) {
          // counter per (tile, wave): arrivals in bits 0-7, the last arriver's give-up in bit 8, the first arriver's
          // publication in bits 16+; whoever sees the other's final event resets it to 0 (the last arriver after the
          // publication, or the publisher after a give-up), so the counter is 0 between launches on every path
          // (kxl: the arrival carries this slice's XCC_ID in bits 9-11; the last arriver compares the first's with its own)
          int* const tk = a.tickets + tile * 4 + wid;
          int old = 0;
          if (lane == 0) old = __hip_atomic_fetch_add(tk, 1 + (xcc << 9), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          old = __builtin_amdgcn_readfirstlane(old);
          if ((old & 0xff) == 0) {  // first: publish (R1: sc1 stores, drained, then the add) and go on
            store_partial();
            if (lane == 0) {
              const int o2 = __hip_atomic_fetch_add(tk, 0x10000, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if (o2 & 0x100) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            continue;
          }
          // last: wait for the publication (the first arriver is resident -- it took its ticket -- and waits on
          // nothing, so this cannot hang on a grid larger than the chip; bounded anyway: a wait that runs out sets
          // status bit 1 and poisons the tile with NaN, ITSD_ERR_HANDOFF)
          int bad = 0;
          if (lane == 0) {
            int v = old + 1;
            for (int it = 0; (v >> 16) == 0 && it < a.spin_bound; ++it) {
              __builtin_amdgcn_s_sleep(1);
              v = __hip_atomic_load(tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if ((v >> 16) == 0) v = __hip_atomic_fetch_add(tk, 0x100, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bad = (v >> 16) == 0;  // (published meanwhile: the give-up's own return says so)
            if (bad) __hip_atomic_fetch_or(a.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (xl && !bad && ((old >> 9) & 7) != xcc) {  // the publisher ran on another XCD: its partial is not here
              bad = 1;
              __hip_atomic_fetch_or(a.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          bad = __builtin_amdgcn_readfirstlane(bad);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the poll)
          auto add_other = [&](auto cp) __attribute__((always_inline)) {  // cp: the loads' cache policy
#pragma unroll
            for (int j = 0; j < NJW; ++j) {
              u32x4 v[4];
#pragma unroll
              for (int g = 0; g < 4; ++g)
                v[g] = __builtin_amdgcn_raw_buffer_load_b128(slab, wbase + (1 - z) * zstride + (j * 4 + g) * 1024, 0,
                                                             decltype(cp)::value);
#pragma unroll
              for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[j][4 * g + e] += __uint_as_float(v[g][e]);
              __builtin_amdgcn_sched_barrier(0);
            }
          };
          if (xl) add_other(std::integral_constant<int, 1>{});
          else add_other(std::integral_constant<int, 16>{});
          if (bad) {
#pragma unroll
            for (int j = 0; j < NJW; ++j)
#pragma unroll
              for (int r = 0; r < 16; ++r) acc[j][r] = __builtin_nanf("");
          }
        } else {
        int old = 0;
        if (lane == 0) old = __hip_atomic_fetch_add(a.tickets + tile * 4 + wid, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        old = __builtin_amdgcn_readfirstlane(old);
        if (old != ST - 1) continue;  // another slice finishes this tile
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the add)
        if (lane == 0) __hip_atomic_store(a.tickets + tile * 4 + wid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // every slice's partial (this one's included), summed in slice order
        for (int sl = 0; sl < ST; ++sl) {
#pragma unroll
          for (int j = 0; j < NJW; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(slab, wbase + sl * zstride + (j * 4 + g) * 1024, 0, 16);
#pragma unroll
              for (int e = 0; e < 4; ++e)
                acc[j][4 * g + e] = sl == 0 ? __uint_as_float(v[e]) : acc[j][4 * g + e] + __uint_as_float(v[e]);
            }
        }
        }  // (last arriver)
      }
      if constexpr (!DIST) TL(3);
      // ---- epilogue: out = acc + addv + residual (lane: pixel 32j + rl, couts 32w + 8g + 4hh + e)
      const int tileP = tp * 128, tileC = tc * CB;
      const float* av = addv + (k & 1) * NSEG * CONV_BM + cw * 32 + 4 * hh;
      const bool has_res = a.resid != nullptr;
      float s16[16], q16[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) s16[e] = q16[e] = 0.f;
      const char* rk = rres + (k & 1) * RTILE;  // this item's residual tile (halo waves, before the last barrier)
      int rlo = rl;
      asm volatile("" : "+v"(rlo));  // (the per-lane epilogue offsets rebuilt per item, not hoisted and spilled)
#pragma unroll
      for (int j = 0; j < NJW; ++j) {
        const int pl = (jb0 + j) * 32 + rlo, seg = pl / SPX;
        const bool live = Cf::ROWS ? tp * 128 < a.M : tp * NSEG + seg < nimg;
        const float* avj = av + seg * CB;
        uint32_t wv[4][2];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = cw * 32 + 8 * g + 4 * hh;
          const f32x4 ad = *(const f32x4*)(avj + 8 * g);
          uint2 rr = *(const uint2*)(rk + pl * 256 + ((((c >> 3) ^ pl) & 15) << 4) + 8 * hh);
          if (!has_res) rr = uint2{0u, 0u};
          float v[4];
          v[0] = acc[j][4 * g + 0] + ad[0] + __uint_as_float(rr.x << 16);
          v[1] = acc[j][4 * g + 1] + ad[1] + __uint_as_float(rr.x & 0xffff0000u);
          v[2] = acc[j][4 * g + 2] + ad[2] + __uint_as_float(rr.y << 16);
          v[3] = acc[j][4 * g + 3] + ad[3] + __uint_as_float(rr.y & 0xffff0000u);
          const T b0 = f2bf(v[0]), b1 = f2bf(v[1]), b2 = f2bf(v[2]), b3 = f2bf(v[3]);
          wv[g][0] = (uint32_t)b0 | ((uint32_t)b1 << 16);
          wv[g][1] = (uint32_t)b2 | ((uint32_t)b3 << 16);
          const float m = live ? 1.0f : 0.0f;
          const float r0 = bf2f(b0) * m, r1 = bf2f(b1) * m, r2 = bf2f(b2) * m, r3 = bf2f(b3) * m;
          s16[4 * g + 0] += r0; q16[4 * g + 0] = fmaf(r0, r0, q16[4 * g + 0]);
          s16[4 * g + 1] += r1; q16[4 * g + 1] = fmaf(r1, r1, q16[4 * g + 1]);
          s16[4 * g + 2] += r2; q16[4 * g + 2] = fmaf(r2, r2, q16[4 * g + 2]);
          s16[4 * g + 3] += r3; q16[4 * g + 3] = fmaf(r3, r3, q16[4 * g + 3]);
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
          const int c8 = cw * 32 + 8 * (gp + hh);
          if (live) *(u32x4*)((T*)a.out + (size_t)(tileP + pl) * a.Cout + tileC + c8) = o;
        }
        // consumer GroupNorm statistics: one slot per image (W = 8: j-blocks {0,1} / {2,3};
        // W = 4: lanes 0-15 / 16-31 of each j-block), one per 128-pixel tile (W >= 16: all four)
        if (a.stats && (W == 4 || (W == 8 && (j & 1)) || j == 3)) {
          float v[32];
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            v[e] = s16[e];
            v[16 + e] = q16[e];
          }
          auto xchg = [](float x, auto wc) {
            constexpr int w = decltype(wc)::value;
            const int xi = __builtin_bit_cast(int, x);
            int r;
            if constexpr (w == 1) r = __builtin_amdgcn_update_dpp(0, xi, 0xB1, 0xF, 0xF, false);
            else if constexpr (w == 2) r = __builtin_amdgcn_update_dpp(0, xi, 0x4E, 0xF, 0xF, false);
            else if constexpr (w == 8) r = __builtin_amdgcn_update_dpp(0, xi, 0x128, 0xF, 0xF, false);
            else r = __builtin_amdgcn_ds_swizzle(xi, 0x1F | (w << 10));
            return __builtin_bit_cast(float, r);
          };
          // halve(d, n): lanes with bit d of rl keep the upper n/2 values, each summed with its partner's
          auto halve = [&](auto wc, auto nc) {
            constexpr int d = decltype(wc)::value, n = decltype(nc)::value;
            const bool up = (rl & d) != 0;
#pragma unroll
            for (int ii = 0; ii < n / 2; ++ii) {
              const float lo = v[ii], hi = v[ii + n / 2];
              v[ii] = (up ? hi : lo) + xchg(up ? lo : hi, wc);
            }
          };
          if constexpr (W >= 8) {  // 64-pixel slot (W = 8: 2 j-blocks) / 128-pixel slot: one value a lane
            halve(std::integral_constant<int, 16>{}, std::integral_constant<int, 32>{});
            halve(std::integral_constant<int, 8>{}, std::integral_constant<int, 16>{});
            halve(std::integral_constant<int, 4>{}, std::integral_constant<int, 8>{});
            halve(std::integral_constant<int, 2>{}, std::integral_constant<int, 4>{});
            halve(std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{});
            const long long slot = W == 8 ? tp * NSEG + ((jb0 + j) >> 1) : tp;  // = global pixel / stat_slot_px
            const int e = rl & 15, co = cw * 32 + 8 * (e >> 2) + 4 * hh + (e & 3);
            if (slot * (W == 8 ? 64 : 128) < a.M) a.stats[(slot * 2 + (rl >> 4)) * a.Cout + tileC + co] = v[0];
          } else {  // 16-pixel slot = 16 lanes: two values a lane, idx = 2 (rl & 15) + {0, 1}
            halve(std::integral_constant<int, 8>{}, std::integral_constant<int, 32>{});
            halve(std::integral_constant<int, 4>{}, std::integral_constant<int, 16>{});
            halve(std::integral_constant<int, 2>{}, std::integral_constant<int, 8>{});
            halve(std::integral_constant<int, 1>{}, std::integral_constant<int, 4>{});
            const int img = tp * NSEG + 2 * (jb0 + j) + (rl >> 4);
            const int m = rl & 7, co = cw * 32 + 8 * (m >> 1) + 4 * hh + 2 * (m & 1);
            if (img < nimg) *(float2*)(a.stats + ((long long)img * 2 + ((rl >> 3) & 1)) * a.Cout + tileC + co) = float2{v[0], v[1]};
          }
#pragma unroll
          for (int e = 0; e < 16; ++e) s16[e] = q16[e] = 0.f;
        }
      }
      if constexpr (!DIST) TL(4);
    }
    TL(5);
    return;
  }

  // ================================================================== halo waves
#if defined(ITSD_DIAG) && defined(P5_NOHALO)
  return;  // diagnostic: the MFMA waves alone on their SIMDs (with P5_AB = 24: no operand traffic either)
#endif
  // thread tt: 8 channels (16 B unit lch) of interior pixels (lt >> 3) + RPP j of image segment sg
  const int tt = tid - 256, lch = tt & 7, sg = tt / TPS, lt = tt - sg * TPS;
  int lds[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int r = (lt >> 3) + RPP * j, hy = HY0 + r / W, x = r - (r / W) * W;
    const int hrow = sg * HS + hy * W2 + (x + 1);
    lds[j] = hrow * ROWB + ((lch ^ swz(hy, x + 1, hrow)) << 4);
  }
#ifdef ITSD_STAMPS
  {  // timeline: the kernel arguments are in SGPRs (a first dependent use)
    int m = a.M;
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(m));
    if (m == -1) g_stamps[0] = 0;
    TL(7);
  }
#endif
  struct Src {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t rowb, so;
  };
  // chunk cc of the 3x3 conv's input (src1 ++ src2) or, raw, of the folded shortcut's (sc_src1 ++ sc_src2); every
  // operand of the selects a prvalue (a conditional over the argument block's lvalues selects between field
  // ADDRESSES: the block could no longer live in registers and went to scratch)
  auto src_of = [&](int cc, bool raw) __attribute__((always_inline)) {
    const int ci0 = cc * 64;
    const int C1 = raw ? static_cast<int>(a.sc_C1) : static_cast<int>(a.C1);
    const int C2 = raw ? static_cast<int>(a.sc_C2) : static_cast<int>(a.C2);
    const bool s1 = ci0 < C1;
    const void* p = raw ? (s1 ? static_cast<const void*>(a.sc_src1) : static_cast<const void*>(a.sc_src2))
                        : (s1 ? static_cast<const void*>(a.src1) : static_cast<const void*>(a.src2));
    const int nrec = (int)std::min<long long>((long long)a.M * (s1 ? C1 : C2) * 2, 0x7fffffffLL);
    Src c;
    c.rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, nrec, 0x00020000);
    c.rowb = (uint32_t)(s1 ? C1 : C2) * 2;
    c.so = (uint32_t)(s1 ? ci0 : ci0 - C1) * 2;
    return c;
  };
  // the stage sequence of this block: (item k, chunk cc); E = the next stage to emit (its data in
  // h, its prescaled coefficients in c, its image mask in zm), L = the stage after it
  u32x4 h[ITEMS];
  f32x4 c[4], cn[4];
  uint32_t zm = 0, zmn = 0;      // bit j: item j of the emitted / loaded stage is real input (else zero)
  bool rawE = false, rawL = false;  // the emitted / loaded stage is a folded-shortcut chunk (copied, no GroupNorm+SiLU)
  int kL = 0, ccL = 0, c1L = 0;  // the stage being loaded and its item's chunk end
  int pix0 = 0;                  // global pixel of this thread's item 0 of the loaded stage (r = lt >> 3)
  const float* cbase = a.gn_coef;
  const int hw = (tid >> 6) - 4, sw0 = (64 * hw) / TPS, sl = sg - sw0;  // this wave's first segment; mine in it
  float* const gsw = gsw_all + hw * 2 * SEGW * 64;
  // gn_fold: group mean / rstd (fp64 sums of the producers' slabs, as gn_coef_kernel) of the images of
  // item k that this wave stages -> gsw[k & 1]. Lane = (group lane & 31, half lane >> 5): half a
  // group's channels, 2 at a time, every load of a slot issued before any is used (unconditional
  // loads from clamped addresses, then a select: no branch / wait per element)
  auto group_stats = [&](int k) {
    int tp, tc, z;
    item_of(k, tp, tc, z);
    const int g = lane & 31, hf = Cin / 64, c0 = g * 2 * hf + (lane >> 5) * hf;  // (Cin / 32 channels a group)
    const int sp1 = stat_spi(HW, a.gn_spi1), sp2 = a.C2 ? stat_spi(HW, a.gn_spi2) : 0;
    const int spm = sp1 > sp2 ? sp1 : sp2;
    // this lane's (segment, slot q, channel pair p) items, it = (segl * spm + q) * np + p, in batches of 8
    // whose 16 loads are all in flight before the first is summed (one memory round trip per batch: 1 at
    // the 16x16 and smaller levels, both 4x4 segments included; 1-3 at 32x32)
    static_assert(SEGW <= 2, "two segments a wave at most");
    const int np = hf >> 1, m = np * spm, mt = SEGW * m;
    int img[SEGW];
#pragma unroll
    for (int segl = 0; segl < SEGW; ++segl) {
      const int im = Cf::ROWS ? (tp * 128) / HW : tp * NSEG + sw0 + segl;
      img[segl] = im < nimg ? im : nimg - 1;
    }
    double sm0 = 0.0, sq0 = 0.0, sm1 = 0.0, sq1 = 0.0;
    for (int b0 = 0; b0 < mt; b0 += 8) {
      float2 vs[8], vq[8];
      bool hi[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int it = b0 + i;
        hi[i] = SEGW > 1 && it >= m;
        const int r = hi[i] ? it - m : it, q = r / np, cr = c0 + 2 * (r - q * np);
        const bool s1 = cr < a.C1;
        const bool ok = it < mt && q < (s1 ? sp1 : sp2);
        const int c = ok ? cr : c0, qq = ok ? q : 0;
        const bool t1 = c < a.C1;
        const float* st = t1 ? a.gn_st1 : a.gn_st2;
        const int Cs = t1 ? a.C1 : a.C2, cs = t1 ? c : c - a.C1, sp = t1 ? sp1 : sp2;
        const long long slot = (long long)(hi[i] ? img[SEGW - 1] : img[0]) * sp + qq;
        const float2 u0 = *(const float2*)(st + (slot * 2) * Cs + cs);
        const float2 u1 = *(const float2*)(st + (slot * 2 + 1) * Cs + cs);
        vs[i] = ok ? u0 : float2{0.f, 0.f};
        vq[i] = ok ? u1 : float2{0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const double ds = (double)vs[i].x + (double)vs[i].y, dq = (double)vq[i].x + (double)vq[i].y;
        if (hi[i]) {
          sm1 += ds;
          sq1 += dq;
        } else {
          sm0 += ds;
          sq0 += dq;
        }
      }
    }
#pragma unroll
    for (int segl = 0; segl < SEGW; ++segl) {
      double sm = segl ? sm1 : sm0, sq = segl ? sq1 : sq0;
      sm += __shfl_xor(sm, 32, 64);
      sq += __shfl_xor(sq, 32, 64);
      const double E = (double)(Cin / 32) * HW, mean = sm / E;
      double var = sq / E - mean * mean;
      var = var > 0.0 ? var : 0.0;
      if (lane < 32) {
        float* d = gsw + ((k & 1) * SEGW + segl) * 64 + 2 * g;
        d[0] = (float)mean;
        d[1] = (float)(1.0 / sqrt(var + 1e-5));
      }
    }
  };
  auto open_item = [&](int k) __attribute__((always_inline)) {  // geometry of item k (as the loaded stage)
    int tp, tc, z;
    item_of(k, tp, tc, z);
    ccL = chunk_lo(z);
    c1L = chunk_hi(z);
    rawL = z >= S;
    const int img = Cf::ROWS ? (tp * 128) / HW : tp * NSEG + sg;
    const int y0 = Cf::ROWS ? ((tp * 128) % HW) / W : 0;  // the tile's first image row
    const int imgc = img < nimg ? img : nimg - 1;
    pix0 = img * HW + (y0 - 1 + HY0) * W + (lt >> 3);
    zmn = 0;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int y = y0 - 1 + HY0 + ((lt >> 3) + RPP * j) / W;
      zmn |= (uint32_t)(img < nimg && y >= 0 && y < W) << j;  // (square images: H = W)
    }
    cbase = a.gn_coef + ((size_t)imgc * (Cin / 8) + lch) * 16;
  };
  // stage L's GroupNorm+SiLU coefficients of this lane's 8 channels (gn_fold: gamma / beta, turned
  // into a, b by prescale from the wave's group statistics)
  auto load_stage = [&]() __attribute__((always_inline)) {
    if (rawL) return;
    if (a.gn_fold) {
      const int c0 = ccL * 64 + 8 * lch;
      cn[0] = *(const f32x4*)(a.gn_gamma + c0);
      cn[1] = *(const f32x4*)(a.gn_gamma + c0 + 4);
      cn[2] = *(const f32x4*)(a.gn_beta + c0);
      cn[3] = *(const f32x4*)(a.gn_beta + c0 + 4);
    } else {
      const f32x4* cp = (const f32x4*)(cbase + ccL * 128);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) cn[qq] = cp[qq];
    }
  };
  auto prescale = [&]() __attribute__((always_inline)) {
    rawE = rawL;
    if (rawL) {
      zm = zmn;
      return;
    }
    if (a.gn_fold) {  // a = rstd gamma, b = beta - mean a (gn_coef_kernel's formula), per channel's group
      const int c0 = ccL * 64 + 8 * lch;
      const float rg = 32.0f / (float)Cin;  // group = floor((c + 0.5) / gsz) (exact: c < 2^11, gsz <= 64)
      const float* gs = gsw + ((kL & 1) * SEGW + sl) * 64;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int g = (int)(((float)(c0 + e) + 0.5f) * rg);
        const float mean = gs[2 * g], rstd = gs[2 * g + 1];
        const float sc = rstd * cn[e >> 2][e & 3];
        c[e >> 2][e & 3] = sc * GN_L2E;
        c[2 + (e >> 2)][e & 3] = (cn[2 + (e >> 2)][e & 3] - mean * sc) * GN_L2E;
      }
    } else {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
#pragma unroll
        for (int e = 0; e < 4; ++e) c[qq][e] = cn[qq][e] * GN_L2E;
    }
    zm = zmn;
  };
  bool more = true;  // a stage L exists
  auto advance = [&]() __attribute__((always_inline)) {  // L <- the stage after L
    if (++ccL == c1L) {
      if (++kL < nit) {
        open_item(kL);
        if (a.gn_fold && !rawL) group_stats(kL);
      } else {
        more = false;
      }
    }
  };
  // emit: transform stage E (h, c, zm) into hbuf, reloading each item's register with stage L's
  auto emit = [&](char* hbuf) __attribute__((always_inline)) {
    const bool live = more;
    if (live) load_stage();
    const Src nx = src_of(live ? ccL : 0, live && rawL);
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      uint32_t yw[4];
      const uint32_t zj = (uint32_t)__builtin_amdgcn_sbfe((int)zm, j, 1);  // 0 (padding) or ~0
      if (rawE) {
#pragma unroll
        for (int e = 0; e < 4; ++e) yw[e] = h[j][e] & zj;
      } else {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
          gn_silu_x4(h[j][2 * hf], h[j][2 * hf + 1], c[hf][0], c[hf][1], c[hf][2], c[hf][3], c[2 + hf][0],
                     c[2 + hf][1], c[2 + hf][2], c[2 + hf][3], zj, yw[2 * hf], yw[2 * hf + 1]);
      }
      *(u32x4*)(hbuf + lds[j]) = u32x4{yw[0], yw[1], yw[2], yw[3]};
      __builtin_amdgcn_sched_barrier(0);
      const uint32_t pix = live && ((zmn >> j) & 1) ? (uint32_t)(pix0 + RPP * j) : 0u;
      h[j] = __builtin_amdgcn_raw_buffer_load_b128(nx.rs, __umul24(pix, nx.rowb) + lch * 16, nx.so, 0);
    }
    prescale();
    if (live) advance();
  };
  auto stage_addv = [&](int k) {  // bias (+ time / class embedding) of item k's images x couts
    int tp, tc, z;
    item_of(k, tp, tc, z);
    const long long trow = a.temb ? (a.temb_tsel ? (long long)(*a.temb_tsel) * a.temb_row_stride : 0) : 0;
    for (int it = tt; it < NSEG * CB; it += 256) {  // [image of the tile][CB couts]
      const int il = it / CB, cl = it % CB, co = tc * CB + cl;
      const int img = min(Cf::ROWS ? (tp * 128) / HW : tp * NSEG + il, nimg - 1);
      float v = a.bias[co];
      if (a.temb) v += a.temb[trow + (long long)img * a.temb_img_stride + co];
      if (a.cemb) {
        int lab = 0;
        if (a.cemb_uncond_from < 0 || img < a.cemb_uncond_from) lab = a.cemb_labels[img % a.cemb_label_mod];
        v += a.cemb[(long long)lab * a.cemb_row_stride + co];
      }
      addv[(k & 1) * NSEG * CONV_BM + it] = v;
    }
  };
  // prologue: stage 0 into buffer 0 (stage 1 loading)
  // item k's residual tile -> rres[k & 1] by LDS-DMA: wave hw, instruction i covers tile rows
  // 4 (8 hw + i) .. +3, lane l -> row + l / 16, LDS unit l % 16 <- source unit (l % 16) ^ (row & 15)
  auto res_dma = [&](int k) __attribute__((always_inline)) {
    int tp, tc, z;
    item_of(k, tp, tc, z);
    const int hw = (tid >> 6) - 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r0 = 4 * (8 * hw + i), r = r0 + (lane >> 4), u = (lane & 15) ^ (r & 15), p = tp * 128 + r;
      // (64-cout items: units 8..15 of a row are not the tile's: the zero page)
      const T* src = p < a.M && u * 8 < CB ? (const T*)a.resid + (size_t)p * a.Cout + tc * CB + u * 8
                                           : (const T*)zero_of_block<T>(a);
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(rres + (k & 1) * RTILE + r0 * 256), 16, 0, 0);
    }
  };
  // prologue: stage 0's input and affine loads are in flight before the first item's statistics
  // loads (one memory round trip for all of them)
  open_item(0);
  load_stage();
  {
    const Src s0 = src_of(ccL, rawL);
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      h[j] = __builtin_amdgcn_raw_buffer_load_b128(
          s0.rs, __umul24(((zmn >> j) & 1) ? (uint32_t)(pix0 + RPP * j) : 0u, s0.rowb) + lch * 16, s0.so, 0);
  }
  // (after stage 0's loads are issued) the halo rows no item writes (the padding columns; interior mode: also the top and bottom rows)
  // of both buffers: zeroed once (item writes never touch them, so no ordering against the first
  // emit is needed; the MFMA waves read after B0)
  for (int u = tt; u < 2 * NSEG * HS * 8; u += 256) {
    const int row = (u >> 3) % (NSEG * HS), buf = (u >> 3) / (NSEG * HS), r = row % HS, y = r / W2, x = r - y * W2;
    if (x == 0 || x == W2 - 1 || (!Cf::ROWS && (y == 0 || y == TH + 1)))
      *(u32x4*)(smem + buf * HALO + row * ROWB + ((u & 7) << 4)) = u32x4{0u, 0u, 0u, 0u};
  }
  if (a.gn_fold && !rawL) group_stats(0);
  TL(1);
  prescale();
  advance();
  emit(smem);
  TL(2);
  block_sync();  // B0
  TL(3);
  // during MFMA stage q (item k, chunk cc): stage item k's addv with its first chunk, emit stage q+1
  int q = 0;
  for (int k = 0; k < nit; ++k) {
    int tp, tc, z;
    item_of(k, tp, tc, z);
    const int c0 = chunk_lo(z), c1 = chunk_hi(z);
    for (int cc = c0; cc < c1; ++cc, ++q) {
      if (cc == c0) stage_addv(k);
      // the item's residual, during its last stage; landed before that stage's barrier (only the next
      // stage's ITEMS item reloads, issued after it, may still be in flight: loads retire in order)
      const bool rdma = a.resid && cc + 1 == c1;
      if (rdma) res_dma(k);
      const bool em = !(k + 1 == nit && cc + 1 == c1);
      if (em) emit(smem + ((q + 1) & 1) * HALO);
      if (rdma) {
        if (em) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ITEMS) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (q == 0) TL(4);
      block_sync();  // end of MFMA stage q
      if (q == 0) TL(6);
    }
  }
  TL(5);
}

// GroupNorm finalize for the fused conv (the statistics half of gn_apply_kernel): per
// image the group mean / rstd in fp64 from the producers' slabs, then per channel
// a = rstd*gamma, b = beta - mean*a as coef[img][C/8][a0..a7, b0..b7].
__global__ __launch_bounds__(256) void gn_coef_kernel(GNArgs g, float* coef) {
  __shared__ float gst[32][2];
  const int img = blockIdx.x, tid = threadIdx.x;
  const int C = g.C1 + g.C2, gsz = C / 32;
  const int spi1 = stat_spi(g.HW, g.spi1), spi2 = stat_spi(g.HW, g.spi2);
  // gamma / beta of this thread's channels, in flight beside the statistics loads
  float gam[8], bet[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int c = tid + 256 * u;
    gam[u] = c < C ? g.gamma[c] : 0.f;
    bet[u] = c < C ? g.beta[c] : 0.f;
  }
  {
    const int grp = tid >> 3, l8 = tid & 7;
    // the group's (channel, slot) items: its src1 channels x spi1 slots, then src2 x spi2 (with
    // equal slot counts the order of a single spi, c = grp*gsz + k/spi). (Round 5: the same items in batches
    // of 8 loads measured C4 +2.5 %, C3 +0.3 % step time -- profiles/r05/step_gn_batched_r05q.txt -- kept as is.)
    const int c0 = grp * gsz, nc1 = max(0, min(g.C1 - c0, gsz)), n1 = nc1 * spi1, n = n1 + (gsz - nc1) * spi2;
    double s = 0.0, q = 0.0;
    for (int k = l8; k < n; k += 8) {
      const bool s1 = k < n1;
      const int spi = s1 ? spi1 : spi2, kk = s1 ? k : k - n1;
      const int c = c0 + (s1 ? 0 : nc1) + kk / spi;
      const long long sl = (long long)img * spi + (kk % spi);
      const float* st = s1 ? g.st1 : g.st2;
      const int Cs = s1 ? g.C1 : g.C2, cs = s1 ? c : c - g.C1;
      s += (double)st[(sl * 2) * Cs + cs];
      q += (double)st[(sl * 2 + 1) * Cs + cs];
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      s += __shfl_xor(s, o, 64);
      q += __shfl_xor(q, o, 64);
    }
    if (l8 == 0) {
      const double E = (double)gsz * g.HW;
      const double mean = s / E;
      double var = q / E - mean * mean;
      var = var > 0.0 ? var : 0.0;
      gst[grp][0] = (float)mean;
      gst[grp][1] = (float)(1.0 / sqrt(var + (double)g.eps));
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int c = tid + 256 * u;
    if (c < C) {
      const int grp = c / gsz;
      const float sc = gst[grp][1] * gam[u];
      float* o = coef + ((size_t)img * (C / 8) + c / 8) * 16 + (c & 7);
      o[0] = sc;
      o[8] = bet[u] - gst[grp][0] * sc;
    }
  }
}

hipError_t launch_gn_coef(const GNArgs& g, int n, float* coef, hipStream_t s) {
  if (g.C1 + g.C2 > 2048) return hipErrorInvalidValue;  // 8 channels per thread
  ITSD_LAUNCH(gn_coef_kernel, dim3(n), dim3(256), 0, s, g, coef);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- head on MFMA
// head = Conv2d(3, ch, 3, padding=1) (Model.py:219, ModelCondition.py:170) in bf16 mode as
// an MFMA GEMM with K = 27 zero-padded to 32: D[cout][pixel] = W[cout][k] x patch[k][pixel],
// k = ci*9 + ky*3 + kx. Block = 128 pixels (whole image rows: one GroupNorm statistics slot)
// x 128 couts; the 3-channel input window sits in LDS as fp32. (Round 5) wave w owns couts
// 32w .. 32w+31 over all 128 pixels (4 accumulators, one per 32-pixel block; each lane builds the
// k-fragments of its pixel in every block from the window) and finishes in registers -- + bias, one
// bf16 rounding, 16-B NHWC stores (permlane32 swap), the slot's statistics by lane butterflies -- so
// the block needs 2.4 KB of LDS instead of the 67 KB fp32 output tile of the shared epilogue, and a CU
// holds 4 blocks (register-bound, 121 VGPRs) instead of 2 (the launch is store- and latency-bound: 67 MB
// of bf16 out at N = 256).
__global__ __launch_bounds__(256, 4) void head_mfma_kernel(HeadArgs h) {
  typedef bf16_t T;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, rl = lane & 31, hh = lane >> 5;
  const int HW = h.H * h.W, W = h.W;
  const long long tileP = (long long)blockIdx.x * 128;
  const int tileC = blockIdx.y * 128;
  // input window: the tile's 128 / W rows (+1 border) of its image
  const int img0 = (int)(tileP / HW), r0 = (int)(tileP - (long long)img0 * HW);
  const int rows = 128 / W, y0 = r0 / W, TR = rows + 2, TW = W + 2;
  __shared__ float tin[3 * 6 * 34 + 3 * 10 * 18];  // [3][TR][TW] (W = 32: 3 x 6 x 34; W <= 16 fits too)
  const int tot = 3 * TR * TW;
  for (int i0 = tid; i0 < tot; i0 += 4 * 256) {
    float v[4];
    bool ok[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + 256 * u;
      const int ci = i / (TR * TW), q = i - ci * TR * TW, ty = q / TW, tx = q - ty * TW;
      const int iy = y0 - 1 + ty, ix = tx - 1;
      ok[u] = i < tot && img0 < h.n && iy >= 0 && iy < h.H && ix >= 0 && ix < W;
      v[u] = h.x[ok[u] ? ((size_t)(img0 % h.x_img_mod) * 3 + ci) * HW + iy * W + ix : 0];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + 256 * u < tot) tin[i0 + 256 * u] = ok[u] ? v[u] : 0.0f;
  }
  // A fragments (weights) of this wave's 32 couts straight from the prepacked [Cout][32] bf16 matrix
  bf16x8 af[2];
  {
    const int co = tileC + wid * 32 + rl;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      af[s2] = co < h.Cout ? *(const bf16x8*)(h.wmf + (size_t)co * 32 + 16 * s2 + 8 * hh) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  __syncthreads();
  f32x16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int pl = j * 32 + rl, ly = pl / W, lx = pl - ly * W;
    bf16x8 bfr[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 16 * s2 + 8 * hh + e;
        float v = 0.0f;
        if (k < 27) {
          const int ci = k / 9, tap = k - ci * 9, ky = tap / 3, kx = tap - ky * 3;
          v = tin[(ci * TR + ly + ky) * TW + lx + kx];
        }
        bfr[s2][e] = (short)f2bf(v);
      }
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s2], bfr[s2], acc[j], 0, 0, 0);
  }
  // epilogue: lane (rl, hh) holds pixel 32 j + rl, couts 32 w + 8 g + 4 hh + e (a wave past Cout: nothing)
  const bool live = img0 < h.n && tileC + wid * 32 < h.Cout;
  float s16[16], q16[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) s16[e] = q16[e] = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int pl = j * 32 + rl;
    uint32_t wv[4][2];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = tileC + wid * 32 + 8 * g + 4 * hh;
      const f32x4 bb = *(const f32x4*)(h.b + c);
      const T b0 = f2bf(acc[j][4 * g] + bb[0]), b1 = f2bf(acc[j][4 * g + 1] + bb[1]);
      const T b2 = f2bf(acc[j][4 * g + 2] + bb[2]), b3 = f2bf(acc[j][4 * g + 3] + bb[3]);
      wv[g][0] = (uint32_t)b0 | ((uint32_t)b1 << 16);
      wv[g][1] = (uint32_t)b2 | ((uint32_t)b3 << 16);
      const float r0 = bf2f(b0), r1 = bf2f(b1), r2 = bf2f(b2), r3 = bf2f(b3);
      s16[4 * g + 0] += r0; q16[4 * g + 0] = fmaf(r0, r0, q16[4 * g + 0]);
      s16[4 * g + 1] += r1; q16[4 * g + 1] = fmaf(r1, r1, q16[4 * g + 1]);
      s16[4 * g + 2] += r2; q16[4 * g + 2] = fmaf(r2, r2, q16[4 * g + 2]);
      s16[4 * g + 3] += r3; q16[4 * g + 3] = fmaf(r3, r3, q16[4 * g + 3]);
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
      const int c8 = tileC + wid * 32 + 8 * (gp + hh);
      if (live) *(u32x4*)((T*)h.out + (size_t)(tileP + pl) * h.Cout + c8) = o;
    }
  }
  if (h.stats && live) {  // the tile's 128 pixels = one slot: 32 values a lane -> one (p5's W >= 16 butterfly)
    float v[32];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      v[e] = s16[e];
      v[16 + e] = q16[e];
    }
    auto xchg = [](float x, auto wc) {
      constexpr int w = decltype(wc)::value;
      const int xi = __builtin_bit_cast(int, x);
      int r;
      if constexpr (w == 1) r = __builtin_amdgcn_update_dpp(0, xi, 0xB1, 0xF, 0xF, false);
      else if constexpr (w == 2) r = __builtin_amdgcn_update_dpp(0, xi, 0x4E, 0xF, 0xF, false);
      else if constexpr (w == 8) r = __builtin_amdgcn_update_dpp(0, xi, 0x128, 0xF, 0xF, false);
      else r = __builtin_amdgcn_ds_swizzle(xi, 0x1F | (w << 10));
      return __builtin_bit_cast(float, r);
    };
    auto halve = [&](auto wc) {
      constexpr int d = decltype(wc)::value;
      const bool up = (rl & d) != 0;
#pragma unroll
      for (int ii = 0; ii < d; ++ii) {
        const float lo = v[ii], hi = v[ii + d];
        v[ii] = (up ? hi : lo) + xchg(up ? lo : hi, wc);
      }
    };
    halve(std::integral_constant<int, 16>{});
    halve(std::integral_constant<int, 8>{});
    halve(std::integral_constant<int, 4>{});
    halve(std::integral_constant<int, 2>{});
    halve(std::integral_constant<int, 1>{});
    const long long slot = tileP / 128;
    const int e = rl & 15, co = wid * 32 + 8 * (e >> 2) + 4 * hh + (e & 3);
    h.stats[(slot * 2 + (rl >> 4)) * h.Cout + tileC + co] = v[0];
  }
}

hipError_t launch_head_mfma(const HeadArgs& h, hipStream_t s) {
  const int HW = h.H * h.W;
  // (128-pixel tiles of whole rows: one statistics slot each; the window fits tin)
  if (!h.wmf || HW % 128 || 128 % h.W || h.Cout % 32 || 3 * (128 / h.W + 2) * (h.W + 2) > 3 * 6 * 34 + 3 * 10 * 18)
    return hipErrorInvalidValue;
  ITSD_LAUNCH(head_mfma_kernel, dim3((unsigned)(((long long)h.n * HW + 127) / 128), (h.Cout + 127) / 128), dim3(256), 0,
              s, h);
  return hipGetLastError();
}

// Host-side eligibility of the fused kernel at an HxW level (the builder decides per conv).
bool conv_gn_eligible(int H, int W) {
  if (W > 128 || 128 % W) return false;
  const int THs = std::min(H, 128 / W);
  if (THs * W == 0 || 128 % (THs * W) || H % THs) return false;
  const int segs = 128 / (THs * W);
  return segs <= 2 && segs * (THs + 2) * (W + 2) <= GNC_HALO_ROWS;
}

// Which fused GroupNorm conv launch_conv runs at this shape: 0 = conv3x3_gn_kernel (128 x 128),
// 1 / 4 = conv3x3_gn_wide_kernel<1 | 4> (256 pixels = rows of one image | four 8x8 images).
int conv_gn_wide_segs(int H, int W, int M, int Cout, bool any_tiles = false) {
  if (!g_gn_wide || W > GNW_BN || GNW_BN % W || M % GNW_BN) return 0;
  int segs = 0;
  if (GNW_BN / W <= H) {
    const int THs = GNW_BN / W;
    const int items = GnpCfg<32>::ITEMS;  // p4's halo items (32 rows each)
    if (H % THs == 0 && (THs + 2) * (W + 2) <= items * 32) segs = 1;
  } else if (GNW_BN == 4 * H * W && (H + 2) * (W + 2) <= GnpCfg<8>::ITEMS * 8) {
    segs = 4;
  }
  const long long blocks = (long long)(M / GNW_BN) * ((Cout + CONV_BM - 1) / CONV_BM);
  return segs && (g_gn_wide == 2 || any_tiles || blocks >= 192) ? segs : 0;
}


// conv3x3_gn_p5_kernel: levels whose 128-pixel tiles hold whole images
bool p5_eligible(int H, int W) { return H == W && (W == 4 || W == 8 || W == 16 || W == 32 || W == 64); }

// The split-K combine shared by every slice (ConvArgs::kdist): where every item has a block of its own (the grid
// co-resident), 3 to 16 slices (arrival count in 16 bits, one 16-slot staging batch a fragment; at 2 slices it measured
// +1 % at N = 256, whose 4x4 launches move 2 x 8 MB of partials: the last arriver's two serial reads cost no more than
// the shared form's poll and staging, profiles/r06/stepab_a256_r06b.txt). g_p5_dist 2: planned
// as shared, combined by the last arriver (the parity tests' bit-identity reference for the same plan)
// (not at the 64x64 level: its instantiation stays the last-arriver form, and the C4 shard's 512+ tiles are not co-resident)
static bool p5_dist(int tiles, int st, int W) {
  return g_p5_dist && W <= 32 && st > 2 && st <= 16 && (long long)tiles * st <= g_num_cus && (long long)tiles * 4 * 32 <= kTicketCap;
}
// its cost in chunk-times (a 64-channel chunk ~4.1 us at N <= 64), fitted to the per-op sweeps of forced slice counts
// (tools/p5_split_sweep.py, profiles/r06/p5_split_n*_r06f.txt, sweep256_r06m.txt): the last item's combine is
// exposed at the end of the launch -- the partial's write-through and drain, the arrival, the slab reads, then the
// epilogue: shared ~2.5 (one poll, two overlapped slab round trips), the last arriver ~2 + 0.5 a slice (its serial
// slice reads). (Round 5 priced 0.3 a slice: it ran the 16x16 level at N = 32 on 2 slices, 25 us a launch where 1
// takes 18; amortising it over a block's items instead ran N = 256's 4x4 level on 4 slices, 50-55 us against 36.)
static double p5_combine_cost(int tiles, int st, int cb, int W) {
  if (st <= 1) return 0.0;
  return cb == 128 && p5_dist(tiles, st, W) ? 2.5 : 2.0 + 0.5 * st;
}
// 64-cout items (CB = 64, W <= 8): a chunk's MFMA work halves, its staging does not -- ITSD_P5_C64_CHUNK chunk-times
#ifndef ITSD_P5_C64_CHUNK
#define ITSD_P5_C64_CHUNK 0.6
#endif

// K slices of a p5 launch at cout tile cb: the S minimising ceil(items / CUs) x (chunks per slice x chunk cost + ~1.5
// chunks of prologue / epilogue) + the combine, bounded by the slab and ticket capacities
static int p5_split(const ConvArgs& a, int tiles, int nch, int cb, double fc) {
  int S = 1;
  if (g_p5_split > 0) {
    S = std::min(g_p5_split, nch);
  } else {
    double best = 1e30;
    for (int s = 1; s <= std::min(nch, 16); ++s) {
      const double waves = std::ceil((double)tiles * s / g_num_cus);
      const double cost = waves * (std::ceil((double)nch / s) * fc + 1.5) + p5_combine_cost(tiles, s, cb, a.Wout);
      if (cost < best - 1e-9) { best = cost; S = s; }
    }
  }
  while (S > 1 && ((long long)tiles * S * 128 * cb > a.splitk_cap || (long long)tiles * 4 > kTicketCap)) --S;
  return S;
}

bool conv_p5_selected(const ConvArgs& a);
// launch_conv's kernel choice for a fused GroupNorm conv: conv3x3_gn_p4_kernel (any form)?
// 96-cout tiles of conv3x3_gn_p4_kernel<8> (AB 512)? Where the 128-cout tile count leaves CUs idle and 96-cout
// tiles need fewer tile-rounds x tile cost (ceil(NT / CUs) x BM / 128), e.g. N = 256: 192 -> 256 tiles
bool conv_p4_c96(const ConvArgs& a) {
  if (!g_p4_c96 || a.Wout != 8 || a.Cout % 96 || a.M % GNW_BN || ITSD_P4_M16 < 2) return false;
  const long long npt = a.M / GNW_BN, G = g_num_cus;
  const long long t96 = npt * (a.Cout / 96), r96 = (t96 + G - 1) / G;
  if (a.Cout % CONV_BM) return true;
  const long long t128 = npt * (a.Cout / CONV_BM), r128 = (t128 + G - 1) / G;
  return g_p4_c96 == 2 || 3 * r96 * 100 < 4 * r128 * 97;  // 0.75 r96 < 0.97 r128
}
bool conv_p4_selected(const ConvArgs& a) {
  if (!a.gn_coef || conv_p5_selected(a) || !conv_gn_wide_segs(a.Hout, a.Wout, a.M, a.Cout)) return false;
  if (conv_p4_c96(a)) return a.wfrag && a.Hout == a.Wout && a.C1 + a.C2 >= 128 && (g_p4_w & 1);
  return a.wfrag && a.Cout % CONV_BM == 0 && a.Hout == a.Wout && a.C1 + a.C2 >= 128 &&
         ((a.Wout == 32 && (g_p4_w & 4)) || (a.Wout == 16 && (g_p4_w & 2)) || (a.Wout == 8 && (g_p4_w & 1)));
}

// A plain (no GroupNorm) 3x3 stride-1 conv on conv3x3_gn_p4_kernel<W, 2>? (the CFG UpSample's conv
// after its ConvTranspose2d: 32x32 / 16x16 / 8x8, ModelCondition.py UpSample)
bool conv_p4_plain_selected(const ConvArgs& a) {
  if (!g_p4_plain || a.gn_coef || !a.wfrag || a.ksize != 3 || a.stride != 1 || a.pad != 1 || a.subpix || a.upsample ||
      a.zins || a.vt_out || !a.zero || a.K != 9 * (a.C1 + a.C2) || a.C1 % 64 || a.C2 % 64)
    return false;
  // (down to 128 tiles, half the CUs: the CFG 8x8 UpSample conv at 2N = 64, 145 -> 113 us against conv_pipe,
  // profiles/r04/census_archC_2N64_p4_plain_128.txt; p4_plain = 2: any tile count)
  const long long tiles = (a.M % GNW_BN) ? 0 : (long long)(a.M / GNW_BN) * (a.Cout / CONV_BM);
  if (!conv_gn_wide_segs(a.Hout, a.Wout, a.M, a.Cout, g_p4_plain == 2 || tiles >= 128)) return false;
  return a.Cout % CONV_BM == 0 && a.Hout == a.Wout && a.Hin == a.Hout && a.C1 + a.C2 >= 128 &&
         (a.Wout == 32 || a.Wout == 16 || a.Wout == 8);
}

// A sub-pixel phase conv on conv3x3_gn_p4_kernel<W, 128 | 256 x (ConvTranspose2d)>? subpix 1: the 2x2-tap
// phases of a nearest-x2 upsample conv; subpix 2: the 3x3-tap phases of ConvTranspose2d(5, 2, 2, 1). W = the
// input grid (8 / 16 / 32); auto from 64 tiles of 4 phases x 256 pixels x 128 couts (192 until round 6)
bool conv_p4_sub_selected(const ConvArgs& a) {
  const int taps = a.subpix == 1 ? 4 : 9;
  if (!g_p4_sub || !a.subpix || !a.wfrag || a.ksize * a.ksize != taps || a.resid || a.vt_out || !a.zero ||
      a.gn_coef || a.Hout != a.Wout || !(a.Wout == 8 || a.Wout == 16 || a.Wout == 32) || a.Cout % CONV_BM ||
      a.C1 % 64 || a.C2 % 64 || a.C1 + a.C2 < 128 || a.K != taps * (a.C1 + a.C2) || a.M % GNW_BN)
    return false;
  // (round 6: from 64 tiles -- N = 32's 8x8 -> 16x16 upsample, 96 tiles, ran 43 us on split-K conv_pipe; was 192)
  return 4LL * (a.M / GNW_BN) * (a.Cout / CONV_BM) >= 64;
}

// launch_conv's kernel choice for a fused GroupNorm conv: conv3x3_gn_p5_kernel?
bool conv_p5_selected(const ConvArgs& a) {
  if (!a.gn_coef || !a.wfrag || a.Cout % CONV_BM || a.C1 % 64 || a.C2 % 64 || !p5_eligible(a.Hout, a.Wout)) return false;
  const int p4_tiles = (a.M % GNW_BN) ? 0 : (a.M / GNW_BN) * (a.Cout / CONV_BM);
  // (4x4: no other persistent fused kernel holds it; 64x64 on p5 unless p4_w bit 3 is set)
  return a.Wout == 4 || a.Wout == 64 || g_p5 == 2 || (g_p5 == 1 && p4_tiles < 192);
}

// The ResBlock's 1x1 shortcut as extra K slices of its block2 conv on p5 (ConvArgs sc_*): the (S, S2) 3x3 /
// shortcut slice counts minimising ceil(items / CUs) x the slower slice + the combine, in chunk-times (a 3x3
// chunk = 1; a shortcut chunk ~0.4: 4 of its 36 k-steps, the same staging; prologue / epilogue 1.5); folded
// where that beats the unfolded plan plus the standalone 1x1 launch it replaces (ITSD_P5_SC_LAUNCH = 5 chunk-times: a
// 10-20 us launch with its gap; 3 left the 32x32 shortcuts at N = 32, the 8x8 ones at N = 64 and the 4x4 ones at N = 256
// unfolded, 0.5-1.1 % slower steps, profiles/r05/p5_sc_launch_cost_r05aq.txt), or always with g_p5_sc = 2. Returns S2
// (0: not folded) and the S to run with.
struct P5Plan {
  int cb = 128, s = 1, s2 = 0;  // cout tile, 3x3 K slices, folded-shortcut K slices (0: not folded)
  double cost = 0.0;
};
// 64-cout p5 items at W <= 8: 0 off (shipped), 1 auto (cost model), 2 always ("p5_c64", diagnostic builds). Measured and
// dropped in round 6: bit-identical to 128-cout items, per-op steady state -8 % at N = 256's 4x4 level, but the
// graph-replayed step equal at N = 256 (4.005 vs 4.001 ms) and 4-7 % slower at N = 64 / 32 (twice the items' prologues
// and staging), profiles/r06/stepab_p5_c64_n*_r06h.txt, p5c64_*_r06h.txt
int g_p5_c64 = 0;
// Also the cout tile: 128, or 64 at W <= 8 (option p5_c64) where twice the tiles without a split cost less.
static P5Plan p5_plan(const ConvArgs& a) {
  const int HW = a.Hout * a.Wout, nimg = a.M / HW;
  const int ptiles = HW > 128 ? a.M / 128 : (nimg + 128 / HW - 1) / (128 / HW);
  const int nch = (a.C1 + a.C2) / 64, nchx = (a.sc_C1 + a.sc_C2) / 64;
  const bool ws = a.splitk_ws && a.tickets;
  const bool sc = ws && g_p5_sc && a.sc_wfrag && nchx > 0 && a.sc_C1 % 64 == 0 && a.sc_C2 % 64 == 0;
  P5Plan best;
  best.cost = 1e30;
  for (int cb : {128, 64}) {
    if (cb == 64 && (!g_p5_c64 || a.Wout > 8 || a.Cout % 64)) continue;
    if (cb == 128 && g_p5_c64 == 2 && a.Wout <= 8 && a.Cout % 64 == 0) continue;
    const int tiles = ptiles * (a.Cout / cb);
    const double fc = cb == 128 ? 1.0 : ITSD_P5_C64_CHUNK;
    auto cost = [&](int s, int s2) {
      const double waves = std::ceil((double)tiles * (s + s2) / g_num_cus);
      const double c3 = std::ceil((double)nch / s) * fc + 1.5, c1 = s2 ? 0.4 * std::ceil((double)nchx / s2) + 1.5 : 0.0;
      return waves * std::max(c3, c1) + p5_combine_cost(tiles, s + s2, cb, a.Wout);
    };
    P5Plan p;
    p.cb = cb;
    p.s = ws ? p5_split(a, tiles, nch, cb, fc) : 1;
    p.cost = cost(p.s, 0) + (sc ? ITSD_P5_SC_LAUNCH : 0.0);  // (unfolded: the shortcut's own launch besides)
    if (sc && (long long)tiles * 4 <= kTicketCap) {
      double bf = 1e30;
      int bs = 0, bs2 = 0;
      const int slo = g_p5_split > 0 ? p.s : 1, shi = g_p5_split > 0 ? p.s : std::min(nch, 16);
      for (int s1 = slo; s1 <= shi; ++s1)
        for (int s2 = 1; s2 <= std::min(nchx, 16); ++s2) {
          if ((long long)tiles * (s1 + s2) * 128 * cb > a.splitk_cap) break;
          const double c = cost(s1, s2);
          if (c < bf - 1e-9) { bf = c; bs = s1; bs2 = s2; }
        }
      if (bs2 && (g_p5_sc == 2 || bf < p.cost)) {
        p.s = bs;
        p.s2 = bs2;
        p.cost = bf;
      }
    }
    if (p.cost < best.cost - 1e-9) best = p;
  }
  return best;
}

// launch_conv's shortcut fold for a p5 conv carrying sc_* candidates: folded?
bool conv_p5_sc_fold(const ConvArgs& a) { return conv_p5_selected(a) && p5_plan(a).s2 > 0; }

static hipError_t launch_p5(const ConvArgs& a0, hipStream_t s) {
  ConvArgs a = a0;
  const int HW = a.Hout * a.Wout, nimg = a.M / HW;
  const int ptiles = HW > 128 ? a.M / 128 : (nimg + 128 / HW - 1) / (128 / HW);
  const P5Plan p = p5_plan(a);
  if (a.sc_C1 + a.sc_C2 && !p.s2) return hipErrorInvalidValue;  // (the caller folds only what p5_plan accepts)
  const int tiles = ptiles * (a.Cout / p.cb);
  a.ksplit = p.s;
  a.sc_split = p.s2;
  const int items = tiles * (p.s + p.s2);
  a.kdist = g_p5_dist == 1 && p.cb == 128 && p5_dist(tiles, p.s + p.s2, a.Wout);
  a.kpub = g_p5_pub;
  const dim3 g(std::min(items, g_num_cus));
  {  // XCD-local exchange: the ST slices of a tile are adjacent items; every XCD's contiguous range of G / 8 blocks
     // (and so of each item round) holds whole tiles when ST divides G / 8
    const int ST = p.s + p.s2, G = (int)g.x;
    // 1: the shared combine at the 8x8 / 16x16 levels (N = 16 step -1.2..2.4 %, N = 32 -0.1..0.9 %); the other forms
    // mostly lose more to the slice-major order's weight re-reads than the L2 exchange saves (the 4x4 level, the
    // two-slice form at K >= 4608 and at 32x32: N = 256 +1.1 % with every form, profiles/r06/p5_xl_ops_r06as.txt);
    // 2 takes every eligible form (A/B); 3 (shipped) adds the two-slice form where K <= 3456 at 8x8 / 16x16
    // (N = 32 -1.0 % against 1, N = 16 / 64 / 256 equal: profiles/r06/stepab_p5_xl3_r06ax.txt)
    // (3: K <= 3456 -- a cout tile's whole K of weights, <= 885 KB, per XCD)
    const bool pub = a.kpub && ST == 2, dist8 = a.kdist && a.Wout >= 8;
    const bool form = g_p5_xl == 2 ? (a.kdist || pub)
                      : g_p5_xl == 3 ? (dist8 || (pub && (a.Wout == 8 || a.Wout == 16) && a.K <= 3456))
                                     : dist8;
    a.kxl = g_p5_xl && ST > 1 && form && G % 8 == 0 && (G / 8) % ST == 0;
  }
  if (a.kdist) {  // (items <= CUs: 128-cout tiles at W <= 32)
    if (a.Wout == 32) ITSD_LAUNCH((conv3x3_gn_p5_kernel<32, 128, true>), g, dim3(512), 0, s, a);
    else if (a.Wout == 16) ITSD_LAUNCH((conv3x3_gn_p5_kernel<16, 128, true>), g, dim3(512), 0, s, a);
    else if (a.Wout == 8) ITSD_LAUNCH((conv3x3_gn_p5_kernel<8, 128, true>), g, dim3(512), 0, s, a);
    else if (a.Wout == 4) ITSD_LAUNCH((conv3x3_gn_p5_kernel<4, 128, true>), g, dim3(512), 0, s, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (a.Wout == 64) ITSD_LAUNCH(conv3x3_gn_p5_kernel<64>, g, dim3(512), 0, s, a);
  else if (a.Wout == 32) ITSD_LAUNCH(conv3x3_gn_p5_kernel<32>, g, dim3(512), 0, s, a);
  else if (a.Wout == 16) ITSD_LAUNCH(conv3x3_gn_p5_kernel<16>, g, dim3(512), 0, s, a);
#ifdef ITSD_DIAG
  else if (a.Wout == 8 && p.cb == 64) ITSD_LAUNCH((conv3x3_gn_p5_kernel<8, 64>), g, dim3(512), 0, s, a);
  else if (p.cb == 64) ITSD_LAUNCH((conv3x3_gn_p5_kernel<4, 64>), g, dim3(512), 0, s, a);
#endif
  else if (a.Wout == 8) ITSD_LAUNCH(conv3x3_gn_p5_kernel<8>, g, dim3(512), 0, s, a);
  else ITSD_LAUNCH(conv3x3_gn_p5_kernel<4>, g, dim3(512), 0, s, a);
  return hipGetLastError();
}

#ifdef ITSD_DIAG
// Diagnostic builds: the compile-time ablations of conv3x3_gn_p4_kernel<32> (conv_dbg 4096 | AB << 13)
static hipError_t launch_p4_ablation(const ConvArgs& a, dim3 gp, hipStream_t s) {
  switch ((g_conv_dbg >> 13) & 127) {
    case 2: ITSD_LAUNCH((conv3x3_gn_p4_kernel<32, 2>), gp, dim3(512), 0, s, a); break;
    case 4: ITSD_LAUNCH((conv3x3_gn_p4_kernel<32, 4>), gp, dim3(512), 0, s, a); break;
    case 8: ITSD_LAUNCH((conv3x3_gn_p4_kernel<32, 8>), gp, dim3(512), 0, s, a); break;
    case 16: ITSD_LAUNCH((conv3x3_gn_p4_kernel<32, 16>), gp, dim3(512), 0, s, a); break;
    case 24: ITSD_LAUNCH((conv3x3_gn_p4_kernel<32, 24>), gp, dim3(512), 0, s, a); break;
    case 10: ITSD_LAUNCH((conv3x3_gn_p4_kernel<32, 10>), gp, dim3(512), 0, s, a); break;
    case 32: ITSD_LAUNCH((conv3x3_gn_p4_kernel<32, 32>), gp, dim3(512), 0, s, a); break;
    case 64: ITSD_LAUNCH((conv3x3_gn_p4_kernel<32, 64>), gp, dim3(512), 0, s, a); break;
    case 18: ITSD_LAUNCH((conv3x3_gn_p4_kernel<32, 18>), gp, dim3(512), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

#endif

// conv_small's K slices when launch_conv runs this (bf16, statistics-free or whole-image) conv on it, else 0 (shared
// by launch_conv and the host's GroupNorm-output fusion, api.hip conv_args, so that both see one decision).
int conv_small_split(const ConvArgs& a) {
  if (a.gn_coef || conv_p4_plain_selected(a)) return 0;
  if (conv1x1_stream_grid(a)) return 0;
  const dim3 grid((a.M + CONV_BN - 1) / CONV_BN, (a.Cout + CONV_BM - 1) / CONV_BM);
  // small levels: 64 x 64 tiles, whole K per block (auto: the 4x4 level and below, where
  // 128 x 128 tiles need split-K; measured slower than conv_pipe at 8x8)
  // (auto: not for K >= 7168 or Cout >= 1536, where the 128-tile pipe with split-K measured
  // 12-18 % faster at N = 256, profiles/r02_small_level_ab.txt; round 6: Cout >= 1536 only where the pipe's grid
  // fills the chip -- the 4x4 q|k|v conv at N = 32 ran 48 pipe blocks without a K split)
  // Under ~one block per CU (the 2x2 / 1x1 levels, small batches) conv_small splits K itself
  // (in-launch combine), up to ~2 blocks per CU with >= 2 K-chunks a slice.
  const dim3 gs((a.M + SM_B - 1) / SM_B, (a.Cout + SM_B - 1) / SM_B);
  int S = 1;
  // (wide: a statistics-free conv of larger images whose 128x128 grid under-fills the chip)
  // (small8: the 8x8 level's convs -- down, shortcuts -- when the 128x128 grid under-fills the chip; not
  // for K >= 7168: the CFG's merged 5x5 DownSample into 8x8, K = 12800 at 2N = 64, measured 156 us on
  // conv_small's 64x64 tiles vs 97 us on the 128-tile pipe, profiles/r04/census_archC_2N64_small8_k.txt)
  const bool wide = g_small_wide && a.Hout * a.Wout > SM_B && grid.x * grid.y < (g_small_wide == 2 ? 512u : 256u);
  // (round 5: also where the 128-tile grid's last round is part-empty -- N = 256's 8x8 shortcuts, 384 tiles --
  // measured 31 -> 48 us a launch, N = 256 step +0.8 %, profiles/r05/small8_part_round_r05t.txt: not taken)
  const bool small8 = g_small_8x8 && a.Hout * a.Wout > 16 && a.Hout * a.Wout <= SM_B && grid.x * grid.y < 256 &&
                      a.K < 7168;
  if (g_small_conv && conv_small_ok(a) && a.splitk_ws && a.tickets && g_splitk &&
      (a.Hout * a.Wout <= 16 || wide || small8) &&
      gs.x * gs.y < 256 && gs.x * gs.y <= kTicketCap) {
    const int blocks = (int)(gs.x * gs.y), nK = a.ksize * a.ksize * ((a.C1 + a.C2) / 64);
    S = std::min(std::min((512 + blocks - 1) / blocks, nK / g_small_minks), 16);  // <= 2 combine batches
    while (S > 1 && (long long)blocks * S * 4096 > a.splitk_cap) --S;
    if (S < 1) S = 1;
  }
  if (g_small_conv && conv_small_ok(a) &&
      (g_small_conv == 2 || S > 1 || wide || small8 ||
       (a.Hout * a.Wout <= 16 && grid.x * grid.y < 1024 &&
        !(a.splitk_ws && g_splitk && (a.K >= 7168 || (a.Cout >= 1536 && grid.x * grid.y >= 256)))))) {
    return S;
  }
  return 0;
}

template <typename T>
hipError_t launch_conv(const ConvArgs& a, hipStream_t s) {
  // (the consumer GroupNorm's output is written by conv_small's epilogue only: host sets gn_out where it runs)
  if (a.gn_out && (sizeof(T) != 2 || !conv_small_split(a))) return hipErrorInvalidValue;
  if constexpr (sizeof(T) == 2) {
    if (a.gn_coef) {
      // the 4x4 level always (no other fused kernel holds it); the others where p4 under-fills the chip
      if (conv_p5_selected(a)) return launch_p5(a, s);
      if (const int segs = conv_gn_wide_segs(a.Hout, a.Wout, a.M, a.Cout)) {
        if (conv_p4_selected(a)) {
          // persistent, one MFMA wave per SIMD (512 threads, 256 registers a wave)
          const bool c96 = conv_p4_c96(a);
          const int tiles = (a.M / GNW_BN) * (a.Cout / (c96 ? 96 : CONV_BM));
          const dim3 gp(std::min(tiles, g_num_cus));
#ifdef ITSD_DIAG
          if ((g_conv_dbg & 4096) && a.Wout == 32) return launch_p4_ablation(a, gp, s);
#endif
          if (a.Wout == 32) ITSD_LAUNCH(conv3x3_gn_p4_kernel<32>, gp, dim3(512), 0, s, a);
          else if (a.Wout == 16) ITSD_LAUNCH(conv3x3_gn_p4_kernel<16>, gp, dim3(512), 0, s, a);
          else if (c96) ITSD_LAUNCH((conv3x3_gn_p4_kernel<8, 512>), gp, dim3(512), 0, s, a);
          else ITSD_LAUNCH(conv3x3_gn_p4_kernel<8>, gp, dim3(512), 0, s, a);
          return hipGetLastError();
        }
      }
      dim3 grid((a.M + CONV_BN - 1) / CONV_BN, (a.Cout + CONV_BM - 1) / CONV_BM);
      const int THs = std::min(a.Hout, 128 / a.Wout), segs = 128 / (THs * a.Wout);
      if (segs == 1) ITSD_LAUNCH(conv3x3_gn_kernel<1>, grid, dim3(256), 0, s, a);
      else ITSD_LAUNCH(conv3x3_gn_kernel<2>, grid, dim3(256), 0, s, a);
      return hipGetLastError();
    }
  }
  constexpr int BK = 8 * (16 / (int)sizeof(T));
  dim3 grid((a.M + CONV_BN - 1) / CONV_BN, (a.Cout + CONV_BM - 1) / CONV_BM);
  if constexpr (sizeof(T) == 2) {
    if (conv_p4_plain_selected(a)) {
      const dim3 gp(std::min((a.M / GNW_BN) * (a.Cout / CONV_BM), g_num_cus));
      if (a.Wout == 32) ITSD_LAUNCH((conv3x3_gn_p4_kernel<32, 2>), gp, dim3(512), 0, s, a);
      else if (a.Wout == 16) ITSD_LAUNCH((conv3x3_gn_p4_kernel<16, 2>), gp, dim3(512), 0, s, a);
      else ITSD_LAUNCH((conv3x3_gn_p4_kernel<8, 2>), gp, dim3(512), 0, s, a);
      return hipGetLastError();
    }
  }
  if constexpr (sizeof(T) == 2) {
    // streaming 1x1 convs: >= 4 pixel tiles per persistent block (large pixel counts, N = 256)
    if (const int G = conv1x1_stream_grid(a)) {
      {
        const int Cin = a.C1 + a.C2;
#define ITSD_S1(NS)                                                                          \
  if (Cin == 128) ITSD_LAUNCH((conv1x1_stream_kernel<128, NS>), dim3(G), dim3(256), 0, s, a);      \
  else if (Cin == 256) ITSD_LAUNCH((conv1x1_stream_kernel<256, NS>), dim3(G), dim3(256), 0, s, a); \
  else if (Cin == 384) ITSD_LAUNCH((conv1x1_stream_kernel<384, NS>), dim3(G), dim3(256), 0, s, a); \
  else if (Cin == 512) ITSD_LAUNCH((conv1x1_stream_kernel<512, NS>), dim3(G), dim3(256), 0, s, a); \
  else ITSD_LAUNCH((conv1x1_stream_kernel<640, NS>), dim3(G), dim3(256), 0, s, a);
        if (g_conv1x1 == 2) {
          ITSD_S1(7)
        } else {
          ITSD_S1(4)
        }
#undef ITSD_S1
        return hipGetLastError();
      }
    }
    if (const int S = conv_small_split(a)) {
      const dim3 gs((a.M + SM_B - 1) / SM_B, (a.Cout + SM_B - 1) / SM_B, S);
      ITSD_LAUNCH(conv_small<false>, gs, dim3(256), 0, s, a);
      return hipGetLastError();
    }
  }
  const int Cin = a.C1 + a.C2;
  const bool pipe = a.zero && Cin % BK == 0 && a.C1 % BK == 0 && a.K == a.ksize * a.ksize * Cin;
  const int v = g_conv_variant;
  const bool lin = !(a.upsample | a.zins);
  if (a.subpix) {
    if (!pipe || !lin || (a.subpix == 2 ? (a.ksize != 3 && !(a.ksize == 1 && a.Hout * a.Wout == 1)) : a.ksize != 2) ||
        ((a.Hout * a.Wout) % 128 && 128 % (a.Hout * a.Wout)))
      return hipErrorInvalidValue;
    if constexpr (sizeof(T) == 2) {
      if (conv_p4_sub_selected(a)) {  // 4 phases x pixel tiles x cout tiles, persistent
        const dim3 gp(std::min(4 * (a.M / GNW_BN) * (a.Cout / CONV_BM), g_num_cus));
        if (a.subpix == 1) {
          if (a.Wout == 32) ITSD_LAUNCH((conv3x3_gn_p4_kernel<32, 128>), gp, dim3(512), 0, s, a);
          else if (a.Wout == 16) ITSD_LAUNCH((conv3x3_gn_p4_kernel<16, 128>), gp, dim3(512), 0, s, a);
          else ITSD_LAUNCH((conv3x3_gn_p4_kernel<8, 128>), gp, dim3(512), 0, s, a);
        } else {
          if (a.Wout == 32) ITSD_LAUNCH((conv3x3_gn_p4_kernel<32, 384>), gp, dim3(512), 0, s, a);
          else if (a.Wout == 16) ITSD_LAUNCH((conv3x3_gn_p4_kernel<16, 384>), gp, dim3(512), 0, s, a);
          else ITSD_LAUNCH((conv3x3_gn_p4_kernel<8, 384>), gp, dim3(512), 0, s, a);
        }
        return hipGetLastError();
      }
    }
    grid.z = 4;
    // under-filled grids (the 4x4 -> 8x8 upsample at small batches, the CFG ConvTranspose2d from the 2x2
    // grid: 32-64 blocks): split K with the in-launch combine, the tiles' tickets per (phase, tile)
    if (a.splitk_ws && a.tickets && g_splitk && g_splitk_inl && g_subpix_split) {
      const int blocks = (int)(grid.x * grid.y) * 4;
      const int nK = a.ksize * a.ksize * (Cin / BK);
      int S = 1;
      if (blocks < 256 && blocks <= kTicketCap) S = std::min((512 + blocks - 1) / blocks, nK / 8);
      while (S > 1 && (long long)blocks * S * 16384 > a.splitk_cap) --S;
      if (S > 1) grid.z = 4 * S;
    }
    // (3- / 4-stage rings at one block a CU measured 8-30 % slower here and were removed in round 5,
    // profiles/r04/census_archC_2N64_conv_variant*.txt)
    ITSD_LAUNCH((conv_pipe<T, 2, true>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
  }
  ConvArgs b = a;  // (conv_pipe's split-K: in-launch combine unless the tiles outnumber the tickets)
  if (pipe && v != 1 && a.splitk_ws && g_splitk) {
    // under-filled grids (the 8x8 / 4x4 levels): split K so that >= ~2 blocks per CU exist,
    // keeping >= 8 K-stages per slice
    const int blocks = (int)(grid.x * grid.y);
    if (blocks > kTicketCap || !g_splitk_inl) b.tickets = nullptr;
    const int nK = a.ksize * a.ksize * (Cin / BK);
    int S = 1;
    if (g_splitk >= 2) S = std::min(g_splitk, nK / 4);  // forced slice count (measurements)
    else if (blocks < 256) S = std::min((512 + blocks - 1) / blocks, nK / 8);  // measured: helps only < 1 block/CU
    while (S > 1 && (long long)blocks * S * 16384 > a.splitk_cap) --S;
    grid.z = S < 1 ? 1 : S;
  }
  if (!pipe || v == 1) ITSD_LAUNCH(conv_igemm<T>, grid, dim3(256), 0, s, a);
  else if (lin) ITSD_LAUNCH((conv_pipe<T, 2, true>), grid, dim3(256), 0, s, b);
  else ITSD_LAUNCH((conv_pipe<T, 2, false>), grid, dim3(256), 0, s, b);
  if (grid.z > 1 && pipe && v != 1 && !b.tickets) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    ITSD_LAUNCH(splitk_epilogue_kernel<T>, dim3(grid.x, grid.y), dim3(256), 0, s, a, (int)grid.z);
  }
  return hipGetLastError();
}

template hipError_t launch_conv<float>(const ConvArgs&, hipStream_t);
template hipError_t launch_conv<bf16_t>(const ConvArgs&, hipStream_t);

}  // namespace itsd

#ifdef ITSD_STAMPS
// diagnostic builds only: copy the wide fused conv's per-wave phase cycles out
extern "C" int itsd_debug_stamps(unsigned long long* host) {
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(itsd::g_stamps), sizeof(unsigned long long) * 1024 * 128) == hipSuccess ? 0 : 1;
}
#endif
