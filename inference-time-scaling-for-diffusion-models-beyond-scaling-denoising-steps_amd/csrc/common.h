// Shared device helpers and kernel argument structs for libitsd_hip (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace itsd {

extern int g_conv_variant;  // kernel-variant switch for A/B measurements (itsd_set_option)
extern int g_small_conv;   // 64x64-tile conv_small for small levels (itsd_set_option "small_conv")
extern int g_splitk;        // split-K on/off (itsd_set_option "splitk")
extern int g_conv_dbg;      // measurement-only conv switches (itsd_set_option "conv_dbg")
extern int g_gn_wide;       // 256-pixel fused GroupNorm conv (itsd_set_option "gn_wide")
extern int g_attn_cs;       // attention output-channel slices (itsd_set_option "attn_cs")
extern int g_attn_aq;       // attention queries per block (itsd_set_option "attn_aq")
extern int g_p4_w;          // conv3x3_gn_p4_kernel level mask (itsd_set_option "p4_w")
extern int g_num_cus;       // compute units of the device (persistent grids)
extern int g_splitk_inl;     // conv_pipe split-K combined in-launch: 0 off (second launch), 1 on (itsd_set_option "splitk_inl")
extern int g_p4_plain;      // plain (no GroupNorm) 3x3 stride-1 convs on conv3x3_gn_p4_kernel<W, 2>: 0 off, 1 on (itsd_set_option "p4_plain")
extern int g_conv1x1;        // streaming 1x1 conv kernel: 0 off, 1 on ("conv1x1")
extern int g_small_8x8;      // conv_small (split K) for under-filled 8x8-level convs ("small_8x8")
extern int g_small_wide;     // conv_small for under-filled statistics-free convs of larger images ("small_wide")
extern int g_attn_wide_nq;   // its query groups a block: 0 auto, 1 / 2 forced ("attn_wide_nq")
extern int g_attn_wide;      // channel-split attention: 0 off, 1 auto, 2 wherever it applies ("attn_wide")
extern int g_small_minks;  // conv_small split K: >= this many K-chunks a slice ("small_minks")
extern int g_convt_prune;  // ConvTranspose2d sub-pixel phases skip their all-zero taps: 0 off, 1 on ("convt_prune")
extern int g_subpix_split;  // under-filled sub-pixel conv_pipe launches split K in-launch: 0 off, 1 on ("subpix_split")
extern int g_p4_xcd;        // persistent fused convs: contiguous tile ranges per XCD ("p4_xcd")
extern int g_p4_c96;        // 8x8 conv3x3_gn_p4_kernel<8, 512> (96-cout tiles): 0 off, 1 auto, 2 always (itsd_set_option "p4_c96")
extern int g_p4_sub;        // nearest-x2 upsample convs on conv3x3_gn_p4_kernel<W, 128>: 0 off, 1 on (itsd_set_option "p4_sub")
extern int g_p5;            // small-level fused conv conv3x3_gn_p5_kernel: 0 off (W = 8), 1 auto, 2 forced (itsd_set_option "p5")
extern int g_p5_split;      // its K slices: 0 auto (cost model), >= 1 forced (itsd_set_option "p5_split")
extern int g_p5_sc;         // 1x1 shortcut folded into the block2 p5 conv: 0 off, 1 auto, 2 always ("p5_sc")
extern int g_p5_xl;         // p5's split-K partials exchanged through one XCD's L2 (ConvArgs::kxl): 0 off, 1 / 2 / 3 (shipped) forms ("p5_xl")
extern int g_p5_pub;        // p5's two-slice combine: only the first arriver stores its partial: 0 off, 1 on ("p5_pub")
extern int g_p5_dist;       // p5 split-K combine by every slice where the grid is co-resident: 0 off, 1 on ("p5_dist")
extern int g_p5_c64;        // 64-cout p5 items at the 8x8 / 4x4 levels: 0 off, 1 auto, 2 always ("p5_c64", diagnostic)
extern int g_spin_bound;     // polls before an in-kernel hand-off wait fails: ITSD_ERR_HANDOFF ("spin_bound", diagnostic)
extern int g_attn_split;     // attn_block_split_kernel at small batches: 0 off, 1 auto, 2/4/6 forced G (itsd_set_option "attn_split")
extern int g_gn_fold;       // GroupNorm finalize inside p4 / p5 instead of a gn_coef launch (itsd_set_option "gn_fold")
extern int g_fuse_gn;       // fused GroupNorm+SiLU+conv3x3 in ResBlocks (itsd_set_option "fuse_gn", read at create)
// Census (itsd_profile_ops): the first kernel an op launches. Every launch site goes through
// ITSD_LAUNCH, which records the kernel expression's name if none is recorded yet; the census
// clears it before each op and maps the name to a small id (kernel_id, itsd_kernel_name).
// Per thread (a census on one thread never reads another thread's launches); kernel_id's
// registry is guarded by a mutex.
extern thread_local const char* g_last_kernel;
int kernel_id(const char* name);
#define ITSD_LAUNCH(K, ...)                                    \
  do {                                                         \
    if (!::itsd::g_last_kernel) ::itsd::g_last_kernel = #K;    \
    hipLaunchKernelGGL(K, __VA_ARGS__);                        \
  } while (0)

typedef uint16_t bf16_t;  // storage type for bf16 activations / weights

// In-launch split-K tickets per UNet handle: the hipMalloc'd counter array (api.hip itsd_unet::tickets)
// and every launch-side bound on ticket indices (conv.hip: conv_pipe / conv_small tile, p5 tile * 4 + wave)
// use this one constant.
constexpr long long kTicketCap = 16384;

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: RNE, NaN stays NaN
  return __builtin_bit_cast(bf16_t, b);
}

// two floats -> one word of two bf16 (lo in the low half): one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  typedef float f2v __attribute__((ext_vector_type(2)));
  typedef __bf16 b2v __attribute__((ext_vector_type(2)));
  const b2v r = __builtin_convertvector((f2v){lo, hi}, b2v);
  return __builtin_bit_cast(uint32_t, r);
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  static __device__ __forceinline__ float load(const float* p) { return *p; }
  static __device__ __forceinline__ float to(float v) { return v; }
  static __device__ __forceinline__ float tof(float v) { return v; }
};
template <> struct Elem<bf16_t> {
  static __device__ __forceinline__ float load(const bf16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ bf16_t to(float v) { return f2bf(v); }
  static __device__ __forceinline__ float tof(bf16_t v) { return bf2f(v); }
};

__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }

// Wave64 reductions.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ----------------------------------------------------------------------------- args
// Implicit-GEMM convolution over NHWC activations (see conv.hip).
struct ConvArgs {
  const void* src1;  // [n][Hin][Win][C1]
  const void* src2;  // [n][Hin][Win][C2] (channel-concat second source, Model.py:280) or null
  int C1, C2;
  int Hin, Win, Hout, Wout;
  int ksize, stride, pad, upsample;  // upsample: nearest x2 folded into addressing (Model.py:123)
  int zins;                          // zero-insertion (ConvTranspose2d s2 as a gather conv, ModelCondition.py:80)
  const void* wt;                    // packed [Cout][K], K = ksize*ksize*(C1+C2), k=(ky*ks+kx)*Cin+ci
  const void* wfrag;                 // the same weights in MFMA A-fragment order [Cout/32][K/16][64][8]
  int Cout, K;
  const float* bias;                 // [Cout]
  // epilogue additive vectors (ResBlock temb_proj, Model.py:204; CFG cond_proj ModelCondition.py:156)
  const float* temb;                 // temb[(tsel? *tsel*row : 0) + img*img_stride + co]
  const int* temb_tsel;
  long long temb_row_stride, temb_img_stride;
  const float* cemb;                 // cemb[labels[img]*row + co]
  const int* cemb_labels;
  long long cemb_row_stride;
  int cemb_label_mod;                // labels index = img % mod (CFG cond||uncond batch)
  int cemb_uncond_from;              // images >= this use label 0 (uncond half); <0 disables
  const void* resid;                 // [M][Cout] same layout as out, or null
  void* out;                         // [M][Cout]
  int M;                             // n * Hout * Wout
  float* stats;                      // channel-statistics slab [slot][2][Cout] for the consumer GN, or null
  const void* zero;                  // >= 16 zero bytes: DMA source for padded / out-of-range rows
  void* vt_out;                      // couts >= vt_from go channel-major to vt_out[img][co-vt_from][HWo]
  int vt_from;                       // (the V of a fused q|k|v projection, for the MFMA attention)
  float* splitk_ws;                  // split-K partial tiles (capacity splitk_cap floats) or null
  long long splitk_cap;
  // fused GroupNorm+SiLU of the input (bf16 3x3, conv3x3_gn_kernel): per-image channel
  // coefficients coef[img][Cin/8][a0..a7, b0..b7] (gn_coef_kernel); null = plain conv
  const float* gn_coef;
  int subpix;                        // 1: nearest-x2 upsample + 3x3 conv run as 4 phase-wise 2x2 convs;
                                     // 2: ConvTranspose2d(5, 2, 2, 1) as 4 phase-wise 3x3 convs (pad 1)
                                     // (grid.z = phase py*2+px): Hout/Wout/M/ksize/K describe the
                                     // input-grid GEMM; output rows are (2i+py, 2j+px) of a 2x grid
  int dbg;                           // g_conv_dbg (measurements only)
  int xcd;                           // persistent fused convs: deal each XCD a contiguous range of tiles (speed only)
  int tap_live;                      // subpix 2 on conv3x3_gn_p4_kernel: skip each phase's all-zero taps
                                     // (conv_pipe runs all 9: measured no faster with live taps)
  // conv3x3_gn_p5_kernel (the fused conv of the 8x8 / 4x4 levels): K split into ksplit slices
  // (>= 1) combined in-launch by the last-arriving slice of each (tile, MFMA wave); tickets[]
  // are zero between launches (zeroed at create, reset by each last arriver)
  int ksplit;
  int* tickets;
  // the GroupNorm finalize folded into conv3x3_gn_p4 / p5_kernel (gn_fold != 0: the gn_coef launch is
  // skipped and the halo waves reduce the input's statistics slabs to group mean / rstd themselves)
  int gn_fold;
  const float* gn_st1;
  const float* gn_st2;
  int gn_spi1, gn_spi2;
  const float* gn_gamma;
  const float* gn_beta;
  // conv3x3_gn_p5_kernel with the ResBlock's 1x1 shortcut folded in (Model.py:200-205, h + shortcut(x)):
  // sc_split more K slices after the ksplit 3x3 ones, over x = sc_src1 ++ sc_src2 (raw, no GroupNorm) with the
  // shortcut's fragment-ordered weights sc_wfrag [Cout/32][(sc_C1+sc_C2)/16][64][8]; bias = both biases summed,
  // resid = null. sc_split == 0: no shortcut slices
  const void* sc_src1;
  const void* sc_src2;
  int sc_C1, sc_C2, sc_split;
  const void* sc_wfrag;
  // conv3x3_gn_p5_kernel's split-K combine shared by all slices (kdist != 0: every block runs one item, so the
  // grid is co-resident): each slice waits for the tile's other slices and finishes its own share of the tile's
  // units; a wait that exhausts spin_bound polls sets bit 1 of *err and writes NaN (ITSD_ERR_HANDOFF)
  int kdist;
  // two slices, last-arriver form (kdist == 0, ST == 2): kpub != 0 -- arrival first, only the first arriver stores its
  // partial (sc1, drained, then publishes on the same counter), the last one adds it to its own from registers
  int kpub;
  // XCD-local split-K exchange (kdist or the two-slice kpub form): the slices of a tile are adjacent items, so they
  // run on blocks of one XCD (the dispatcher deals block b to XCD b % 8) and exchange partials through that XCD's
  // L2 -- plain stores, L1-bypassing (sc0) loads -- instead of writing through to memory (sc1). Each slice reports
  // its XCC_ID with its arrival; a tile whose slices ran on different XCDs is poisoned with NaN and sets bit 1 of
  // *err (ITSD_ERR_HANDOFF): never a silent stale read
  int kxl;
  int* err;
  int spin_bound;
  // conv_small (whole-image tiles, HWo <= 16) with its consumer GroupNorm(+SiLU) fused into the epilogue: the next op
  // (gn_apply_kernel over this output alone) is skipped and the epilogue writes silu(GN(out)) to gn_out as well, from
  // the same per-channel slot sums and the same fp64 group finalize (bit-identical); a group's channels lie inside
  // one 64-cout tile (host: 64 % (Cout / 32) == 0). Null: no fused GroupNorm
  void* gn_out;
  const float* go_gamma;
  const float* go_beta;
  int go_silu;
};

// Channel-statistics slab of an NHWC tensor (written by its producer): slots of
// Gt = min(HW, 128) consecutive pixels; stats[slot][0][c] = sum, [slot][1][c] = sum of squares.
__host__ __device__ inline int stat_slot_px(int HW) { return HW < 128 ? HW : 128; }
// Statistics slots per image of a tensor: HW / stat_slot_px(HW), except the output of a sub-pixel
// upsample conv whose phase images are smaller than a slot: one slot per (image, phase).
__host__ __device__ inline int stat_spi(int HW, int spi) { return spi > 0 ? spi : HW / stat_slot_px(HW); }

struct GNArgs {
  const void* src1; const void* src2;  // NHWC, C1 (+ C2) channels
  const float* st1; const float* st2;  // their statistics slabs
  int C1, C2, HW;
  int spi1, spi2;                      // statistics slots per image of src1 / src2 (0: HW / stat_slot_px(HW))
  const float* gamma; const float* beta;
  float eps;
  int silu;
  void* dst;                           // NHWC, C1+C2 channels
  int chunks_per_block;                // 16-B chunks of one image handled per block
};

struct AttnArgs {
  const void* qkv;  // [n][S][3C]  (q | k | v per token; v unused when vt != null)
  const void* vt;   // [n][C][S]   channel-major v (MFMA path) or null
  void* out;        // [n][S][C]
  int S, C;
  float scale;
};

// Fused AttnBlock at S = 64 (kernels.hip attn_block_kernel).
struct AttnBlockArgs {
  const bf16_t* x;        // [n][S][C] NHWC (the ResBlock output)
  const float* st;        // its GroupNorm statistics slab [n * spi][2][C]
  int spi;                // statistics slots per image
  const float* gamma; const float* beta;
  const bf16_t* wqkv;     // [3C/32][C/16][64][8]: q rows, k rows, v rows
  const float* bqkv;      // [3C]
  const bf16_t* wp;       // [C/32][C/16][64][8]
  const float* bp;        // [C]
  bf16_t* out;            // [n][S][C]
  float* out_stats;       // [n][2][C] (one slot per image) or null
  float scale;            // C^-0.5
  int n;
  int S;                  // tokens an image: 64 (one image a block) or 16 (4 images a block)
  // attn_block_split_kernel (an image's work over G blocks, small batches): partial-score and O slabs
  // (write-through hand-offs) and two monotonic counters per image
  float* spart;           // [n][G][4 tiles][64 lanes][16] fp32
  bf16_t* oslab;          // [n][64][C] bf16
  int* sync;              // [n][2], never reset (targets from each block's own add)
  int* err;               // device status word: bit 0 set when a hand-off wait exhausted its poll bound
  int spin_bound;         // polls before a hand-off wait gives up (itsd_set_option "spin_bound", diagnostic)
};

struct HeadArgs {
  const float* x;       // NCHW fp32 [n][3][H][W]
  const float* w;       // [Cout][3][3][3] fp32 (reference layout)
  const float* b;
  void* out;            // NHWC [n][H][W][Cout]
  int H, W, Cout, n;
  int x_img_mod;        // image i reads x[i % x_img_mod] (CFG cond||uncond batch)
  float* stats;         // GroupNorm statistics slab of the output [slot][2][Cout], or null
  const bf16_t* wmf;    // bf16 MFMA weights [Cout][32] (k = ci*9 + tap, zero-padded 27..31), or null
};

// Per-run sampler parameters, kept in device memory so that one captured step graph serves
// every run of a search (only the values change between rounds, never the graph).
struct RunParams {
  unsigned long long seed;  // Philox key of the per-step noise z
  long long noise_offset;   // Philox element offset (global candidate index * per-candidate elements)
  int clip_at;              // clip when t == clip_at (-1: never)
  int pad_;
};

struct TailArgs {
  const void* g;        // NHWC [nb][H][W][C] : silu(gn(h))
  const float* w;       // [3][C][3][3] fp32 (reference layout)
  const float* b;       // [3]
  int H, W, C, n;       // n = output images
  int cfg;              // eps = (1+w) eps(img) - w eps(img+n)  (DiffusionCondition.py:85)
  float guide_w;        // w (fp32 cast of the Python float)
  float guide_w1;       // (1 + w) computed in double then cast, as the reference's scalar
  // mode
  int step_mode;        // 0: write eps NCHW; 1: sampler update of x in place
  float* eps_out;       // NCHW [n][3][H][W]
  float* x;             // NCHW [n][3][H][W]
  const int* tsel;      // current step t (device)
  const float* coeff1; const float* coeff2; const float* sqrt_var;
  const float* noise;   // [T][n][3][H][W] or null
  const RunParams* run; // seed / noise offset / clip step of this run (device)
  int* nan_flag;
  // bf16 MFMA tail (tail_mfma_kernel): g is the RAW last ResBlock output and the tail
  // GroupNorm+SiLU is applied while staging it, with per-image coefficients
  // coef[img][C/8][a0..a7, b0..b7] (gn_coef_kernel); wmf = bf16 weights [9C/32][4][3][8]
  // (k = tap*C + ci; k-step ks, lane group kg, output channel, 8 consecutive k)
  const float* coef;
  const bf16_t* wmf;
};

}  // namespace itsd
