// libitsd_hip runtime: the C ABI of include/itsd.h.
//
// Builds the UNet op program natively from the reference constructor arguments
// (Diffusion/Model.py:212-262, DiffusionFreeGuidence/ModelCondition.py:164-203),
// repacks the state_dict into MFMA-friendly layouts, owns one activation arena
// sized for max_batch (288 GB of HBM makes a dedicated buffer per op affordable),
// and drives the ancestral sampler loop (Diffusion.py:84-102) as one hipGraph
// replayed T times; the timestep lives in device memory so the graph is
// step-invariant and no host sync happens inside the loop.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "itsd.h"

namespace itsd {
template <typename T> hipError_t launch_conv(const ConvArgs&, hipStream_t);
template <typename T> hipError_t launch_groupnorm(const GNArgs&, int, hipStream_t);
template <typename T> hipError_t launch_attn(const AttnArgs&, int, hipStream_t);
bool attn_flash_ok(int S, int C);
bool attn_cs_ok(int S, int C);
bool attn_block_ok(int S, int C);
hipError_t launch_attn_block(const AttnBlockArgs&, int, hipStream_t);
int g_attn_fuse = 1;  // fused AttnBlock kernel at S = 64 (Arch A's 8x8 level): 0 off, 1 on (itsd_set_option "attn_fuse", read at create)
int g_tap_prune = 1;   // drop conv taps that read only padding for every output pixel ("tap_prune", read at create)
int g_down_merge = 1;  // CFG DownSample c1 (3x3) + c2 (5x5) as one 5x5 conv ("down_merge", read at create)
int g_attn_s1 = 1;    // one-token AttnBlock (the CFG 1x1 level) as GroupNorm + one folded 1x1 conv ("attn_s1", read at create)
template <typename T> hipError_t launch_head(const HeadArgs&, hipStream_t);
template <typename T> hipError_t launch_tail(const TailArgs&, hipStream_t);
hipError_t launch_emb_input(const int*, int, const float*, const float*, int, float*, int, hipStream_t);
hipError_t launch_linear(const float*, int, int, const float*, const float*, int, int, float*, hipStream_t);
hipError_t launch_verify(int, const float*, int, int, int, int, int, double*, const float*, hipStream_t);
hipError_t launch_set_int(int*, int, hipStream_t);
hipError_t launch_add_int(int*, int, hipStream_t);
int calibrate_run(int what, double* value, hipStream_t s);
hipError_t launch_run_begin(int*, int, int*, RunParams*, const RunParams&, hipStream_t);
int g_option_gen = 0;  // bumped by every itsd_set_option: part of the step-graph cache key
bool conv_gn_eligible(int H, int W);
bool p5_eligible(int H, int W);
bool conv_p5_selected(const ConvArgs& a);
bool conv_p4_selected(const ConvArgs& a);
bool conv_p5_sc_fold(const ConvArgs& a);
int conv_small_split(const ConvArgs& a);
int conv_gn_wide_segs(int H, int W, int M, int Cout, bool any_tiles = false);
hipError_t launch_gn_coef(const GNArgs&, int, float*, hipStream_t);
hipError_t launch_head_mfma(const HeadArgs&, hipStream_t);
hipError_t launch_tail_mfma(const TailArgs&, hipStream_t);
bool tail_mfma_ok(int H, int W, int C);
int g_io_mfma = 1;  // bf16 head / tail on MFMA (itsd_set_option "io_mfma", read at create)
int g_small_gn = 1;  // conv_small writes its consumer GroupNorm's output (itsd_set_option "small_gn"): 0 off, 1 on
hipError_t launch_noise(float*, const float*, int, long long, float, unsigned long long, unsigned, long long,
                        hipStream_t);
template <typename T> hipError_t launch_nhwc_to_nchw(const void*, float*, int, int, int, hipStream_t);
}  // namespace itsd

using namespace itsd;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                           \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) return fail(ITSD_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define CHK(x)                  \
  do {                          \
    int r_ = (x);               \
    if (r_ != ITSD_OK) return r_; \
  } while (0)

// ITSD_ERR_HANDOFF's message from the status word's bits (AttnBlockArgs::err)
std::string handoff_msg(int bits) {
  std::string m = "in-kernel hand-off wait exhausted its poll bound (grid not co-resident?):";
  if (bits & 1) m += " attn_block_split_kernel";
  if (bits & 2) m += " conv3x3_gn_p5_kernel (split-K combine)";
  return m;
}

uint16_t host_f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// NHWC activation buffer (capacity = max batch), located at ws + off.
struct Act {
  size_t off;
  int H, W, C;
  size_t stats = SIZE_MAX;  // ws offset of the channel-statistics slab (consumed by a GroupNorm), or none
  int spi = 0;              // its slots per image (0: H*W / stat_slot_px(H*W); sub-pixel outputs: stat_spi)
};

enum OpKind { OP_GN, OP_CONV, OP_ATTN, OP_GNCOEF, OP_ATTNBLOCK };
constexpr int kCensusAttnBlock = 7;  // census kind of OP_ATTNBLOCK (runtime.py "attnblock")
constexpr int kCensusConvGN = 4;  // census kind of a fused GroupNorm+SiLU conv (conv3x3_gn_kernel)
constexpr int kCensusConvGNW = 5;   // ... run as conv3x3_gn_wide_kernel<1>
constexpr int kCensusConvGNW4 = 6;  // ... run as conv3x3_gn_wide_kernel<4>

struct Op {
  OpKind kind;
  int src1 = -1, src2 = -1, dst = -1;
  // GN
  size_t gamma = 0, beta = 0;  // fp32 offsets in the weight arena
  int silu = 0;
  // CONV
  int ksize = 3, stride = 1, pad = 1, upsample = 0, zins = 0;
  int subpix = 0;  // upsample conv as 4 phase-wise 2x2 convs (conv.hip conv_pipe)
  size_t wt = 0, bias = 0;
  size_t wfrag = SIZE_MAX;  // fragment-ordered copy of wt (fused GroupNorm convs: conv3x3_gn_p4 / p5_kernel)
  int Cout = 0, K = 0;
  int temb_col = -1;
  int resid = -1;
  // ATTN
  int S = 0, C = 0;
  int vt = -1, vt_from = 0;  // channel-major V buffer (conv: couts >= vt_from go there; attn: reads it)
  size_t coef = SIZE_MAX;    // GNCOEF: output; CONV: GroupNorm+SiLU coefficients of the input (fused conv)
  size_t wt2 = 0, bias2 = 0;  // ATTNBLOCK: the proj matrix (fragment-packed) and bias; wt / bias: q|k|v
  size_t gn_gamma = SIZE_MAX, gn_beta = SIZE_MAX;  // CONV with coef: its input GroupNorm's affine (gn_fold)
  // a ResBlock's block2 conv and its 1x1 shortcut (conv3x3_gn_p5_kernel folds the shortcut in as K slices, ConvArgs
  // sc_*): on block2, the shortcut op, its weights in fragment order and the two biases summed; on the shortcut, block2
  int sc_op = -1, sc_into = -1;
  size_t sc_wfrag = SIZE_MAX, bias_sc = SIZE_MAX;
  // a conv and the GroupNorm op right after it over its output alone (conv_small writes the GroupNorm's output in its
  // epilogue, ConvArgs gn_out): on the conv, the GN op; on the GN op, the conv
  int gn_next = -1, gn_from = -1;
};

// Host staging for the weight arena: fp32 params and packed conv weights.
struct Arena {
  std::vector<char> host;
  size_t add(const void* p, size_t bytes) {
    size_t off = (host.size() + 255) & ~(size_t)255;
    host.resize(off + bytes);
    if (p) std::memcpy(host.data() + off, p, bytes);
    return off;
  }
};

// A captured denoising step is keyed by what its launches bake in: the batch, whether labels
// are used, the injected-noise pointer and the kernel-selection options. x and labels are
// staged through handle-owned buffers and the seed, noise offset and clip step live in device
// memory (RunParams), so every round of a search replays one graph.
struct GraphEntry {
  std::tuple<int, bool, const float*, int> key;
  hipGraphExec_t exec = nullptr;
};

}  // namespace

struct itsd_unet {
  itsd_unet_desc d{};
  int device = 0;
  bool bf16 = false;
  size_t esz = 4;
  bool cfg = false;
  int H = 32, ch = 128, tdim = 512, sumC = 0;
  int nb_max = 0;  // capacity in images (CFG: 2 * max_batch)
  int last_forward_n = 0;  // batch of the last itsd_unet_forward (itsd_unet_representation reads its tail input)

  char* wdev = nullptr;
  char* ws = nullptr;
  size_t ws_bytes = 0;
  std::vector<Act> acts;
  std::vector<Op> ops;
  int head_out = -1, tail_g = -1, tail_in = -1;
  size_t tail_gn_g = 0, tail_gn_b = 0;

  // fp32 params (arena offsets)
  size_t head_w = 0, head_b = 0, tail_w = 0, tail_b = 0;
  size_t head_wmf = SIZE_MAX, tail_wmf = SIZE_MAX, tail_coef = SIZE_MAX;  // bf16 MFMA head / tail (+ tail GN coefficients)
  size_t freq = 0, ttable = 0, W0t = 0, b0 = 0, W2t = 0, b2 = 0, Wpt = 0, bp = 0;
  size_t ctable = 0, C1t = 0, cb1 = 0, C3t = 0, cb3 = 0, Wct = 0, bc = 0;

  // scratch (separate allocation)
  float* emb_buf = nullptr;   // [rows][ch]
  float* h1_buf = nullptr;    // [rows][tdim]
  float* te_buf = nullptr;    // [rows][tdim]
  float* proj_buf = nullptr;  // [max_batch][sumC]
  int rows_cap = 0;
  float* cemb_table = nullptr;  // [num_labels+1][sumC] (CFG)
  // sampler
  int T_sched = 0;
  float* coeff1 = nullptr;
  float* coeff2 = nullptr;
  float* sqrt_var = nullptr;
  float* temb_table = nullptr;  // [T_sched][sumC]
  float guide_w = 0.f, guide_w1 = 1.f;
  int* d_t = nullptr;
  int* d_nan = nullptr;
  RunParams* d_run = nullptr;
  float* x_state = nullptr;     // [max_batch][3][H][W]: the sampler's x between the caller's copies
  int32_t* lab_state = nullptr; // [max_batch] labels of the guided sampler
  long long graph_captures = 0;  // step graphs captured + instantiated (itsd_unet_query)
  void* zero_page = nullptr;  // 256 KiB of zeros (conv DMA source for padding, conv.hip zero_of_block)
  float* splitk_ws = nullptr;  // split-K partial tiles (shared by all convs: they run in stream order)
  int* tickets = nullptr;      // in-launch split-K counters (conv3x3_gn_p5_kernel), zero between launches
  int* attn_sync = nullptr;    // attn_block_split_kernel's per-image hand-off counters [nb_max][2] (monotonic)
  static constexpr long long kSplitkCap = 16ll << 20;  // floats (64 MB)

  hipStream_t stream = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  std::vector<GraphEntry> graphs;

  template <typename P = float>
  P* wp(size_t off) const { return (P*)(wdev + off); }
  void* ap(int id) const { return ws + acts[id].off; }
};

namespace {

struct Builder {
  itsd_unet* u;
  Arena ar;
  std::unordered_map<std::string, std::pair<const float*, int64_t>> w;
  size_t used = 0;
  size_t ws_off = 0;
  std::string err;
  std::vector<std::pair<std::string, size_t>> temb_cols;  // resblock prefix -> column

  const float* get(const std::string& name, int64_t numel) {
    auto it = w.find(name);
    if (it == w.end()) {
      if (err.empty()) err = "missing key in state_dict: " + name;
      return nullptr;
    }
    if (it->second.second != numel) {
      if (err.empty())
        err = "size mismatch for " + name + ": got " + std::to_string(it->second.second) + " elements, expected " +
              std::to_string(numel);
      return nullptr;
    }
    ++used;
    return it->second.first;
  }
  // a second view of an entry already consumed by get/f32 (not counted again)
  const float* peek(const std::string& name, int64_t numel) {
    auto it = w.find(name);
    return (it == w.end() || it->second.second != numel) ? nullptr : it->second.first;
  }
  size_t f32(const std::string& name, int64_t numel) {
    const float* p = get(name, numel);
    return ar.add(p, numel * 4);
  }
  int act(int H, int W, int C) {
    Act a{ws_off, H, W, C};
    size_t bytes = (size_t)u->nb_max * H * W * C * u->esz;
    ws_off = (ws_off + bytes + 255) & ~(size_t)255;
    u->acts.push_back(a);
    return (int)u->acts.size() - 1;
  }
  // Packs conv weight(s) [Cout][Cin][k][k] into [Cout][K] with k = (ky*ks+kx)*Cin + ci.
  // flip_t: source is ConvTranspose2d [Cin][Cout][k][k]; use the flipped kernel.
  size_t pack(const std::vector<const float*>& parts, int Cpart, int Cin, int ks, bool flip_t = false) {
    const int Cout = Cpart * (int)parts.size();
    const int K = ks * ks * Cin;
    std::vector<float> tmp((size_t)Cout * K, 0.f);
    for (size_t pi = 0; pi < parts.size(); ++pi) {
      const float* src = parts[pi];
      if (!src) continue;
      for (int co = 0; co < Cpart; ++co)
        for (int ci = 0; ci < Cin; ++ci)
          for (int ky = 0; ky < ks; ++ky)
            for (int kx = 0; kx < ks; ++kx) {
              float v;
              if (!flip_t) v = src[(((size_t)co * Cin + ci) * ks + ky) * ks + kx];
              else v = src[(((size_t)ci * Cpart + co) * ks + (ks - 1 - ky)) * ks + (ks - 1 - kx)];
              tmp[((size_t)pi * Cpart + co) * K + (ky * ks + kx) * Cin + ci] = v;
            }
    }
    if (u->bf16) {
      std::vector<uint16_t> b(tmp.size());
      for (size_t i = 0; i < tmp.size(); ++i) b[i] = host_f2bf(tmp[i]);
      return ar.add(b.data(), b.size() * 2);
    }
    return ar.add(tmp.data(), tmp.size() * 4);
  }
  // [Cout][K] bf16 (k = (ky*ks+kx)*Cin + ci) -> MFMA A-fragment order [Cout/32][K/16][64][8]:
  // lane L of k-step s holds W[32*cb + (L & 31)][16*s + 8*(L >> 5) + e] (v_mfma_f32_32x32x16_bf16).
  size_t pack_frag(const float* Wsrc, int Cout, int Cin, int ks) {
    const int K = ks * ks * Cin, nks = K / 16;
    std::vector<uint16_t> b((size_t)Cout * K, 0);
    if (Wsrc)
      for (int cb = 0; cb < Cout / 32; ++cb)
        for (int st = 0; st < nks; ++st)
          for (int L = 0; L < 64; ++L)
            for (int e = 0; e < 8; ++e) {
              const int co = 32 * cb + (L & 31), k = 16 * st + 8 * (L >> 5) + e;
              const int tap = k / Cin, ci = k - tap * Cin, ky = tap / ks, kx = tap - ky * ks;
              b[(((size_t)cb * nks + st) * 64 + L) * 8 + e] =
                  host_f2bf(Wsrc[(((size_t)co * Cin + ci) * ks + ky) * ks + kx]);
            }
    return ar.add(b.data(), b.size() * 2);
  }
  // Phase weights [4][Cout][K] (fp32) in MFMA A-fragment order per phase, [4][Cout/32][K/16][64][8]
  // (conv3x3_gn_p4_kernel's sub-pixel form): lane L of k-step st holds W'[ph][32 cb + L % 32][16 st + 8 (L / 32) + e].
  // SIZE_MAX unless bf16 with Cout % 32 == 0 and K % 16 == 0.
  size_t frag4(const std::vector<float>& tmp, int Cout, int K) {
    if (!u->bf16 || Cout % 32 || K % 16) return SIZE_MAX;
    const int nks = K / 16;
    std::vector<uint16_t> f(tmp.size());
    for (int ph = 0; ph < 4; ++ph)
      for (int cb = 0; cb < Cout / 32; ++cb)
        for (int st = 0; st < nks; ++st)
          for (int L = 0; L < 64; ++L)
            for (int e = 0; e < 8; ++e)
              f[((((size_t)ph * (Cout / 32) + cb) * nks + st) * 64 + L) * 8 + e] =
                  host_f2bf(tmp[((size_t)ph * Cout + 32 * cb + (L & 31)) * K + 16 * st + 8 * (L >> 5) + e]);
    return ar.add(f.data(), f.size() * 2);
  }
  // Nearest-x2 upsample + 3x3 conv (Model.py:123-125) as 4 sub-pixel phases: output
  // (2i+py, 2j+px) sees input rows i+dy+py-1 (dy in {0,1}) with the 3x3 taps folded
  // onto them: W'[ph][co][dy][dx][ci] = sum over ky in R(py,dy), kx in R(px,dx) of
  // W[co][ci][ky][kx], R(0,0)={0}, R(0,1)={1,2}, R(1,0)={0,1}, R(1,1)={2}. Sums in fp64.
  size_t pack_subpix(const float* W, int Cout, int Cin, size_t* wfrag = nullptr) {
    static const int lo[2][2] = {{0, 1}, {0, 2}}, hi[2][2] = {{0, 2}, {1, 2}};  // [p][d] -> k range
    const int K = 4 * Cin;
    std::vector<float> tmp((size_t)4 * Cout * K, 0.f);
    for (int ph = 0; ph < 4; ++ph) {
      const int py = ph >> 1, px = ph & 1;
      for (int co = 0; co < Cout; ++co)
        for (int dy = 0; dy < 2; ++dy)
          for (int dx = 0; dx < 2; ++dx)
            for (int ci = 0; ci < Cin; ++ci) {
              double acc = 0.0;
              for (int ky = lo[py][dy]; ky <= hi[py][dy]; ++ky)
                for (int kx = lo[px][dx]; kx <= hi[px][dx]; ++kx)
                  acc += W ? (double)W[(((size_t)co * Cin + ci) * 3 + ky) * 3 + kx] : 0.0;
              tmp[((size_t)ph * Cout + co) * K + (dy * 2 + dx) * Cin + ci] = (float)acc;
            }
    }
    if (wfrag) *wfrag = frag4(tmp, Cout, K);
    if (u->bf16) {
      std::vector<uint16_t> b(tmp.size());
      for (size_t i = 0; i < tmp.size(); ++i) b[i] = host_f2bf(tmp[i]);
      return ar.add(b.data(), b.size() * 2);
    }
    return ar.add(tmp.data(), tmp.size() * 4);
  }
  // ConvTranspose2d(Cin, Cout, 5, stride 2, padding 2, output_padding 1) (ModelCondition.py:80) as 4
  // sub-pixel phases: output (2m+ry, 2n+rx) = sum over input (m+dy, n+dx), dy, dx in {-1, 0, 1}, of
  // x * w[ci][co][k(ry, dy)][k(rx, dx)] with k(0, d) = 2 - 2d, k(1, d) = 3 - 2d (none for d = -1):
  // W'[ph][co][((dy+1)*3 + dx+1)*Cin + ci] (transposed-conv weight layout [Cin][Cout][5][5])
  // centre_only (a 1x1 input grid, where the d = +-1 taps read only padding): the d = 0 tap alone,
  // W'[ph][co][ci] (K = Cin, ksize 1, pad 0).
  size_t pack_convt_subpix(const float* W, int Cout, int Cin, size_t* wfrag = nullptr, bool centre_only = false) {
    auto kk = [](int r, int d) { return r == 0 ? 2 - 2 * d : (d < 0 ? -1 : 3 - 2 * d); };
    const int rd = centre_only ? 0 : 1, kw = 2 * rd + 1, K = kw * kw * Cin;
    std::vector<float> tmp((size_t)4 * Cout * K, 0.f);
    for (int ph = 0; ph < 4; ++ph) {
      const int ry = ph >> 1, rx = ph & 1;
      for (int co = 0; co < Cout; ++co)
        for (int dy = -rd; dy <= rd; ++dy)
          for (int dx = -rd; dx <= rd; ++dx) {
            const int ky = kk(ry, dy), kx = kk(rx, dx);
            if (ky < 0 || kx < 0 || !W) continue;
            for (int ci = 0; ci < Cin; ++ci)
              tmp[((size_t)ph * Cout + co) * K + ((dy + rd) * kw + dx + rd) * Cin + ci] =
                  W[(((size_t)ci * Cout + co) * 5 + ky) * 5 + kx];
          }
    }
    if (wfrag) *wfrag = frag4(tmp, Cout, K);
    if (u->bf16) {
      std::vector<uint16_t> b(tmp.size());
      for (size_t i = 0; i < tmp.size(); ++i) b[i] = host_f2bf(tmp[i]);
      return ar.add(b.data(), b.size() * 2);
    }
    return ar.add(tmp.data(), tmp.size() * 4);
  }
  int upconv(int s1, const std::string& name, int Cout, int Hout) {
    const Act& A = u->acts[s1];
    const int Cin = A.C, epc = u->bf16 ? 8 : 4;
    // sub-pixel tiles hold whole phase images or lie inside one (128-pixel tiles)
    if (((A.H * A.W) % 128 && 128 % (A.H * A.W)) || Cin % (8 * epc))
      return conv_layer(s1, -1, name, Cout, 3, 1, 1, 1, Hout, Hout);
    const float* W = get(name + ".weight", (int64_t)Cout * Cin * 9);
    size_t wf = SIZE_MAX;
    // fragment-ordered copy for conv3x3_gn_p4_kernel's sub-pixel form (input grids 8x8 / 16x16 / 32x32)
    const bool p4sub = Cout % 128 == 0 && Cin % 64 == 0 && Cin >= 128 && A.H == A.W && (A.W == 8 || A.W == 16 || A.W == 32);
    size_t wt = pack_subpix(W, Cout, Cin, p4sub ? &wf : nullptr);
    size_t b = f32(name + ".bias", Cout);
    int dst = act(Hout, Hout, Cout);
    if (A.H * A.W < 128) u->acts[dst].spi = 4;  // one statistics slot per (image, phase)
    conv(s1, -1, dst, wt, b, Cout, 3, 1, 1, 1);
    Op& o = u->ops.back();
    o.subpix = 1;
    o.wfrag = wf;
    return dst;
  }
  size_t concat_f32(const std::vector<const float*>& parts, int n) {
    std::vector<float> tmp((size_t)n * parts.size(), 0.f);
    for (size_t i = 0; i < parts.size(); ++i)
      if (parts[i]) std::memcpy(tmp.data() + i * n, parts[i], n * 4);
    return ar.add(tmp.data(), tmp.size() * 4);
  }
  // W [out][in] -> W^T [in][out] fp32
  size_t transposed(const float* W, int out, int in) {
    std::vector<float> tmp((size_t)out * in, 0.f);
    if (W)
      for (int o = 0; o < out; ++o)
        for (int i = 0; i < in; ++i) tmp[(size_t)i * out + o] = W[(size_t)o * in + i];
    return ar.add(tmp.data(), tmp.size() * 4);
  }

  void gn(int s1, int s2, int dst, const std::string& p, int C, int silu) {
    Op o;
    o.kind = OP_GN;
    o.src1 = s1; o.src2 = s2; o.dst = dst;
    o.gamma = f32(p + ".weight", C);
    o.beta = f32(p + ".bias", C);
    o.silu = silu;
    u->ops.push_back(o);
  }
  void conv(int s1, int s2, int dst, size_t wt, size_t bias, int Cout, int ks, int stride, int pad, int ups,
            int temb_col = -1, int resid = -1, int zins = 0) {
    Op o;
    o.kind = OP_CONV;
    o.src1 = s1; o.src2 = s2; o.dst = dst;
    o.wt = wt; o.bias = bias; o.Cout = Cout;
    const int Cin = u->acts[s1].C + (s2 >= 0 ? u->acts[s2].C : 0);
    o.K = ks * ks * Cin;
    o.ksize = ks; o.stride = stride; o.pad = pad; o.upsample = ups; o.zins = zins;
    o.temb_col = temb_col; o.resid = resid;
    u->ops.push_back(o);
  }
  // (Wx / bx: weights [Cout][Cin][ks][ks] and bias built by the caller instead of name's)
  int conv_layer(int s1, int s2, const std::string& name, int Cout, int ks, int stride, int pad, int ups, int Hout,
                 int Wout, int temb_col = -1, int resid = -1, const std::string& gn = "", const float* Wx = nullptr,
                 const float* bx = nullptr) {
    const int Cin = u->acts[s1].C + (s2 >= 0 ? u->acts[s2].C : 0);
    size_t coef = SIZE_MAX;
    if (!gn.empty()) {  // GN coefficient op feeding the fused conv
      Op g;
      g.kind = OP_GNCOEF;
      g.src1 = s1; g.src2 = s2;
      g.gamma = f32(gn + ".weight", Cin);
      g.beta = f32(gn + ".bias", Cin);
      g.coef = coef = ws_off;
      ws_off = (ws_off + (size_t)u->nb_max * Cin * 2 * 4 + 255) & ~(size_t)255;
      u->ops.push_back(g);
    }
    const float* W = Wx ? Wx : get(name + ".weight", (int64_t)Cout * Cin * ks * ks);
    // Taps that read only padding for EVERY output pixel (the 1x1 / 2x2 levels of Arch C: a 3x3
    // conv on a 1x1 image uses its centre tap alone; a stride-2 3x3 / 5x5 conv 2x2 -> 1x1 uses a
    // 2x2 window) are dropped: the conv runs as the ks' x ks' window with pad' = pad - k0.
    // Tap ky is live iff some output row reads an in-range input row:
    // pad - (Hout-1)*stride <= ky <= Hin + pad - 1. Exact (the dropped taps multiply zeros).
    std::vector<float> wwin;
    {
      const Act& A = u->acts[s1];
      const int k0 = std::max(0, pad - (Hout - 1) * stride), k1 = std::min(ks - 1, A.H + pad - 1);
      const int x0 = std::max(0, pad - (Wout - 1) * stride), x1 = std::min(ks - 1, A.W + pad - 1);
      if (itsd::g_tap_prune && gn.empty() && !ups && W && (k0 > 0 || k1 < ks - 1) && k0 == x0 && k1 == x1 && k1 >= k0) {
        const int ks2 = k1 - k0 + 1;
        wwin.resize((size_t)Cout * Cin * ks2 * ks2);
        for (size_t oc = 0; oc < (size_t)Cout * Cin; ++oc)
          for (int ky = 0; ky < ks2; ++ky)
            for (int kx = 0; kx < ks2; ++kx)
              wwin[(oc * ks2 + ky) * ks2 + kx] = W[(oc * ks + k0 + ky) * ks + k0 + kx];
        W = wwin.data();
        ks = ks2;
        pad -= k0;
      }
    }
    size_t wt = pack({W}, Cout, Cin, ks);
    size_t b = bx ? ar.add(bx, (size_t)Cout * 4) : f32(name + ".bias", Cout);
    int dst = act(Hout, Wout, Cout);
    conv(s1, s2, dst, wt, b, Cout, ks, stride, pad, ups, temb_col, resid);
    u->ops.back().coef = coef;
    if (coef != SIZE_MAX) {  // (the GNCOEF op pushed just before this conv)
      u->ops.back().gn_gamma = u->ops[u->ops.size() - 2].gamma;
      u->ops.back().gn_beta = u->ops[u->ops.size() - 2].beta;
    }
    // (plain 3x3 stride-1 convs too: conv3x3_gn_p4_kernel's plain form, conv_p4_plain_selected)
    const bool plain3 = coef == SIZE_MAX && ks == 3 && stride == 1 && pad == 1 && !ups && Cout % 128 == 0 &&
                        Cin % 128 == 0 && Hout == Wout && (Hout == 32 || Hout == 16 || Hout == 8);
    if ((coef != SIZE_MAX || plain3) && u->bf16 && Cout % 32 == 0 && (ks * ks * Cin) % 16 == 0)
      u->ops.back().wfrag = pack_frag(W, Cout, Cin, ks);
    return dst;
  }
  // conv3x3(silu(GroupNorm(s1 ++ s2))) can run as one fused launch (conv3x3_gn_kernel)
  bool fusable(int s1, int s2, int Cout) const {
    const Act& A = u->acts[s1];
    return u->bf16 && itsd::g_fuse_gn && A.C % 64 == 0 && (s2 < 0 || u->acts[s2].C % 64 == 0) &&
           Cout % 128 == 0 && (conv_gn_eligible(A.H, A.W) || p5_eligible(A.H, A.W));
  }

  int resblock(int x1, int x2, const std::string& p, int in_ch, int out_ch, bool attn) {
    const int H = u->acts[x1].H, W = u->acts[x1].W;
    const int col = u->sumC;
    u->sumC += out_ch;
    temb_cols.push_back({p, (size_t)col});
    // GroupNorm+SiLU either fused into the conv's input staging (conv3x3_gn_kernel) or
    // materialised by gn_apply_kernel
    int h1, o;
    int resid = x1;
    if (fusable(x1, x2, out_ch)) {
      h1 = conv_layer(x1, x2, p + ".block1.2", out_ch, 3, 1, 1, 0, H, W, col, -1, p + ".block1.0");
    } else {
      int g1 = act(H, W, in_ch);
      gn(x1, x2, g1, p + ".block1.0", in_ch, 1);
      h1 = conv_layer(g1, -1, p + ".block1.2", out_ch, 3, 1, 1, 0, H, W, col);
    }
    const bool f2 = fusable(h1, -1, out_ch);
    int g2 = -1;
    if (!f2) {
      g2 = act(H, W, out_ch);
      gn(h1, -1, g2, p + ".block2.0", out_ch, 1);
    }
    int isc = -1;
    if (in_ch != out_ch) {
      resid = conv_layer(x1, x2, p + ".shortcut", out_ch, 1, 1, 0, 0, H, W);
      isc = (int)u->ops.size() - 1;
    }
    if (f2) o = conv_layer(h1, -1, p + ".block2.3", out_ch, 3, 1, 1, 0, H, W, -1, resid, p + ".block2.0");
    else o = conv_layer(g2, -1, p + ".block2.3", out_ch, 3, 1, 1, 0, H, W, -1, resid);
    if (f2 && isc >= 0 && u->bf16 && out_ch % 32 == 0 && u->acts[x1].C % 64 == 0 && (x2 < 0 || u->acts[x2].C % 64 == 0)) {
      // the shortcut as extra K slices of block2 where block2 runs on conv3x3_gn_p5_kernel (run time: conv_args)
      const float* wsc = peek(p + ".shortcut.weight", (int64_t)out_ch * in_ch);
      const float* bsc = peek(p + ".shortcut.bias", out_ch);
      const float* bb2 = peek(p + ".block2.3.bias", out_ch);
      if (wsc && bsc && bb2) {
        std::vector<float> bs((size_t)out_ch);
        for (int c = 0; c < out_ch; ++c) bs[c] = bb2[c] + bsc[c];
        Op& c2 = u->ops.back();
        c2.sc_wfrag = pack_frag(wsc, out_ch, in_ch, 1);
        c2.bias_sc = ar.add(bs.data(), (size_t)out_ch * 4);
        c2.sc_op = isc;
        u->ops[isc].sc_into = (int)u->ops.size() - 1;
      }
    }
    if (attn && H * W == 1 && itsd::g_attn_s1) {
      // AttnBlock over ONE token (ModelCondition.py's 1x1 level; Model.py:145-164): the softmax over a single key
      // is exp(0) / exp(0) = 1 exactly, so h = v and the block is x + proj(v(GN(x))) = x + Wf GN(x) + bf with
      // Wf = Wp Wv, bf = Wp bv + bp (folded here in fp64): one GroupNorm and one 1x1 conv instead of GroupNorm,
      // the q|k|v conv, the attention kernel and the proj conv (q and k never reach the output)
      const std::string a = p + ".attn";
      const int64_t cc = (int64_t)out_ch * out_ch;
      const float* wv = get(a + ".proj_v.weight", cc);
      const float* bv = get(a + ".proj_v.bias", out_ch);
      const float* wp = get(a + ".proj.weight", cc);
      const float* bp = get(a + ".proj.bias", out_ch);
      // (q / k: validated and counted as the reference's keys, never read)
      const bool qk = get(a + ".proj_q.weight", cc) && get(a + ".proj_q.bias", out_ch) && get(a + ".proj_k.weight", cc) &&
                      get(a + ".proj_k.bias", out_ch);
      if (wv && bv && wp && bp && qk) {
        std::vector<float> wf((size_t)cc), bf((size_t)out_ch);
        std::vector<double> row((size_t)out_ch);
        for (int oc = 0; oc < out_ch; ++oc) {
          std::fill(row.begin(), row.end(), 0.0);
          double bacc = (double)bp[oc];
          for (int c = 0; c < out_ch; ++c) {
            const double w = (double)wp[(size_t)oc * out_ch + c];
            const float* vr = wv + (size_t)c * out_ch;
            for (int ic = 0; ic < out_ch; ++ic) row[ic] += w * (double)vr[ic];
            bacc += w * (double)bv[c];
          }
          for (int ic = 0; ic < out_ch; ++ic) wf[(size_t)oc * out_ch + ic] = (float)row[ic];
          bf[oc] = (float)bacc;
        }
        int ga = act(H, W, out_ch);
        gn(o, -1, ga, a + ".group_norm", out_ch, 0);
        return conv_layer(ga, -1, a + ".proj", out_ch, 1, 1, 0, 0, H, W, -1, o, "", wf.data(), bf.data());
      }
    }
    if (attn && u->bf16 && itsd::g_attn_fuse && attn_block_ok(H * W, out_ch)) {
      // the whole AttnBlock in one launch (kernels.hip attn_block_kernel)
      const std::string a = p + ".attn";
      const int64_t cc = (int64_t)out_ch * out_ch;
      std::vector<float> wcat((size_t)3 * cc, 0.f);
      const float* wq = get(a + ".proj_q.weight", cc);
      const float* wk = get(a + ".proj_k.weight", cc);
      const float* wv = get(a + ".proj_v.weight", cc);
      if (wq && wk && wv) {
        std::memcpy(wcat.data(), wq, cc * 4);
        std::memcpy(wcat.data() + cc, wk, cc * 4);
        std::memcpy(wcat.data() + 2 * cc, wv, cc * 4);
      }
      Op ab;
      ab.kind = OP_ATTNBLOCK;
      ab.src1 = o;
      ab.gamma = f32(a + ".group_norm.weight", out_ch);
      ab.beta = f32(a + ".group_norm.bias", out_ch);
      ab.wt = pack_frag(wcat.data(), 3 * out_ch, out_ch, 1);
      ab.bias = concat_f32({get(a + ".proj_q.bias", out_ch), get(a + ".proj_k.bias", out_ch),
                            get(a + ".proj_v.bias", out_ch)}, out_ch);
      ab.wt2 = pack_frag(get(a + ".proj.weight", cc), out_ch, out_ch, 1);
      ab.bias2 = f32(a + ".proj.bias", out_ch);
      ab.S = H * W;
      ab.C = out_ch;
      ab.dst = act(H, W, out_ch);
      u->ops.push_back(ab);
      return ab.dst;
    }
    if (attn) {
      const std::string a = p + ".attn";
      int ga = act(H, W, out_ch);
      gn(o, -1, ga, a + ".group_norm", out_ch, 0);
      const int64_t cc = (int64_t)out_ch * out_ch;
      size_t wqkv = pack({get(a + ".proj_q.weight", cc), get(a + ".proj_k.weight", cc), get(a + ".proj_v.weight", cc)},
                         out_ch, out_ch, 1);
      size_t bqkv = concat_f32({get(a + ".proj_q.bias", out_ch), get(a + ".proj_k.bias", out_ch),
                                get(a + ".proj_v.bias", out_ch)}, out_ch);
      int qkv = act(H, W, 3 * out_ch);
      conv(ga, -1, qkv, wqkv, bqkv, 3 * out_ch, 1, 1, 0, 0);
      // MFMA attention (bf16): V goes channel-major to its own buffer from the conv epilogue
      const int S = H * W;
      int vt = -1;
      // (S <= 256: whole-row MFMA kernel; longer sequences: flash kernel, C <= 256)
      if (u->bf16 && S % 16 == 0 && out_ch % 64 == 0 && (S <= 256 || attn_flash_ok(S, out_ch) || attn_cs_ok(S, out_ch))) {
        vt = act(out_ch, S, 1);
        u->ops.back().vt = vt;
        u->ops.back().vt_from = 2 * out_ch;
      }
      int ao = act(H, W, out_ch);
      Op at;
      at.kind = OP_ATTN;
      at.src1 = qkv; at.dst = ao; at.S = H * W; at.C = out_ch; at.vt = vt;
      u->ops.push_back(at);
      o = conv_layer(ao, -1, a + ".proj", out_ch, 1, 1, 0, 0, H, W, -1, o);
    }
    return o;
  }
};

int build(itsd_unet* u, const itsd_tensor_view* views, int nviews) {
  Builder b;
  b.u = u;
  for (int i = 0; i < nviews; ++i) b.w[views[i].name] = {views[i].data, views[i].numel};
  const itsd_unet_desc& d = u->d;
  const int ch = d.ch, tdim = 4 * ch, H = d.img_size;
  u->ch = ch; u->tdim = tdim; u->H = H;

  // embeddings
  if (!u->cfg) {
    u->freq = b.f32("time_embedding.freq_coeffs", ch / 2);
    u->W0t = b.transposed(b.get("time_embedding.timembedding.0.weight", (int64_t)tdim * ch), tdim, ch);
    u->b0 = b.f32("time_embedding.timembedding.0.bias", tdim);
    u->W2t = b.transposed(b.get("time_embedding.timembedding.2.weight", (int64_t)tdim * tdim), tdim, tdim);
    u->b2 = b.f32("time_embedding.timembedding.2.bias", tdim);
  } else {
    u->ttable = b.f32("time_embedding.timembedding.0.weight", (int64_t)d.T * ch);
    u->W0t = b.transposed(b.get("time_embedding.timembedding.1.weight", (int64_t)tdim * ch), tdim, ch);
    u->b0 = b.f32("time_embedding.timembedding.1.bias", tdim);
    u->W2t = b.transposed(b.get("time_embedding.timembedding.3.weight", (int64_t)tdim * tdim), tdim, tdim);
    u->b2 = b.f32("time_embedding.timembedding.3.bias", tdim);
    u->ctable = b.f32("cond_embedding.condEmbedding.0.weight", (int64_t)(d.num_labels + 1) * ch);
    u->C1t = b.transposed(b.get("cond_embedding.condEmbedding.1.weight", (int64_t)tdim * ch), tdim, ch);
    u->cb1 = b.f32("cond_embedding.condEmbedding.1.bias", tdim);
    u->C3t = b.transposed(b.get("cond_embedding.condEmbedding.3.weight", (int64_t)tdim * tdim), tdim, tdim);
    u->cb3 = b.f32("cond_embedding.condEmbedding.3.bias", tdim);
  }
  u->head_w = b.f32("head.weight", (int64_t)ch * 27);
  u->head_b = b.f32("head.bias", ch);
  u->head_out = b.act(H, H, ch);
  // (head_mfma_kernel: 128-pixel tiles of whole rows, couts in 32-blocks; else the plain head kernel)
  if (u->bf16 && itsd::g_io_mfma && ch % 32 == 0 && (H * H) % 128 == 0 && 128 % H == 0) {
    // [Cout][32] bf16, k = ci*9 + tap (the reference's flat per-cout order), zero-padded
    const float* hw = b.peek("head.weight", (int64_t)ch * 27);
    if (hw) {
      std::vector<uint16_t> wm((size_t)ch * 32, 0);
      for (int co = 0; co < ch; ++co)
        for (int k = 0; k < 27; ++k) wm[(size_t)co * 32 + k] = host_f2bf(hw[(size_t)co * 27 + k]);
      u->head_wmf = b.ar.add(wm.data(), wm.size() * 2);
    }
  }

  std::vector<int> hs{u->head_out};
  int cur = u->head_out;
  int now = ch;
  int ndown = 0;
  auto P = [](const char* s, int i) { return std::string(s) + "." + std::to_string(i); };
  for (int i = 0; i < d.n_mult; ++i) {
    const int out = ch * d.ch_mult[i];
    bool at = false;
    for (int k = 0; k < d.n_attn; ++k) at |= (d.attn[k] == i);
    if (u->cfg) at = true;
    for (int r = 0; r < d.num_res_blocks; ++r) {
      cur = b.resblock(cur, -1, P("downblocks", ndown++), now, out, at);
      now = out;
      hs.push_back(cur);
    }
    if (i != d.n_mult - 1) {
      const std::string p = P("downblocks", ndown++);
      const int Hc = b.u->acts[cur].H;
      if (!u->cfg) {
        cur = b.conv_layer(cur, -1, p + ".main", now, 3, 2, 1, 0, Hc / 2, Hc / 2);
      } else if (!itsd::g_down_merge) {  // c1(x) + c2(x), ModelCondition.py:71-73, as two convs
        int t1 = b.conv_layer(cur, -1, p + ".c1", now, 3, 2, 1, 0, Hc / 2, Hc / 2);
        cur = b.conv_layer(cur, -1, p + ".c2", now, 5, 2, 2, 0, Hc / 2, Hc / 2, -1, t1);
      } else {  // c1(x) + c2(x), ModelCondition.py:71-73: both stride 2 and centred on the same input
        // pixel (3x3 pad 1, 5x5 pad 2), so the sum is ONE 5x5 conv with c1's taps added onto c2's
        // inner 3x3 (summed in fp32 before packing) and bias b1 + b2: 25 Cin of K instead of 34 Cin,
        // one launch and no intermediate tensor
        const int Cin = b.u->acts[cur].C;
        const float* W1 = b.get(p + ".c1.weight", (int64_t)now * Cin * 9);
        const float* W2 = b.get(p + ".c2.weight", (int64_t)now * Cin * 25);
        const float* b1 = b.get(p + ".c1.bias", now);
        const float* b2 = b.get(p + ".c2.bias", now);
        std::vector<float> wm((size_t)now * Cin * 25, 0.f), bm(now, 0.f);
        if (W2) std::memcpy(wm.data(), W2, wm.size() * 4);
        if (W1)
          for (size_t oc = 0; oc < (size_t)now * Cin; ++oc)
            for (int ky = 0; ky < 3; ++ky)
              for (int kx = 0; kx < 3; ++kx) wm[(oc * 5 + ky + 1) * 5 + kx + 1] += W1[(oc * 3 + ky) * 3 + kx];
        for (int c = 0; c < now; ++c) bm[c] = (b1 ? b1[c] : 0.f) + (b2 ? b2[c] : 0.f);
        cur = b.conv_layer(cur, -1, p + ".c12", now, 5, 2, 2, 0, Hc / 2, Hc / 2, -1, -1, "", wm.data(), bm.data());
      }
      hs.push_back(cur);
    }
  }
  cur = b.resblock(cur, -1, "middleblocks.0", now, now, true);
  cur = b.resblock(cur, -1, "middleblocks.1", now, now, false);
  int nup = 0;
  for (int i = d.n_mult - 1; i >= 0; --i) {
    const int out = ch * d.ch_mult[i];
    bool at = false;
    for (int k = 0; k < d.n_attn; ++k) at |= (d.attn[k] == i);
    if (u->cfg) at = false;
    for (int r = 0; r < d.num_res_blocks + 1; ++r) {
      int skip = hs.back();
      hs.pop_back();
      cur = b.resblock(cur, skip, P("upblocks", nup++), now + u->acts[skip].C, out, at);
      now = out;
    }
    if (i != 0) {
      const std::string p = P("upblocks", nup++);
      const int Hc = b.u->acts[cur].H;
      if (!u->cfg) {
        cur = b.upconv(cur, p + ".main", now, 2 * Hc);
      } else {  // ConvTranspose2d(5, 2, 2, 1) then Conv 3x3, ModelCondition.py:83-85
        const float* Wt = b.get(p + ".t.weight", (int64_t)now * now * 25);
        size_t bt = b.f32(p + ".t.bias", now);
        int tmp = b.act(2 * Hc, 2 * Hc, now);
        const int epc = u->bf16 ? 8 : 4;
        if (((Hc * Hc) % 128 == 0 || 128 % (Hc * Hc) == 0) && now % (8 * epc) == 0) {
          // sub-pixel form: 4 phase-wise 3x3 convs over the input grid (9 of the 25 taps a phase,
          // against 25 per output of the zero-insertion form)
          // (+ the fragment-ordered phase weights for conv3x3_gn_p4_kernel's sub-pixel form at 8x8 .. 32x32 inputs)
          size_t wf = SIZE_MAX;
          const bool p4sub = now % 128 == 0 && now >= 128 && (Hc == 8 || Hc == 16 || Hc == 32);
          // (a 1x1 input grid: the centre tap alone, K = Cin instead of 9 Cin)
          const bool c1 = Hc == 1 && itsd::g_tap_prune;
          size_t wt = b.pack_convt_subpix(Wt, now, now, p4sub ? &wf : nullptr, c1);
          if (Hc * Hc < 128) u->acts[tmp].spi = 4;  // one statistics slot per (image, phase)
          b.conv(cur, -1, tmp, wt, bt, now, c1 ? 1 : 3, 1, c1 ? 0 : 1, 0);
          u->ops.back().subpix = 2;
          u->ops.back().wfrag = wf;
        } else {
          size_t wt = b.pack({Wt}, now, now, 5, true);
          b.conv(cur, -1, tmp, wt, bt, now, 5, 1, 2, 0, -1, -1, 1);
        }
        cur = b.conv_layer(tmp, -1, p + ".c", now, 3, 1, 1, 0, 2 * Hc, 2 * Hc);
      }
    }
  }
  if (!hs.empty()) return fail(ITSD_ERR_INVALID, "internal: skip stack not empty");
  u->tail_in = cur;
  u->tail_gn_g = b.f32("tail.0.weight", now);
  u->tail_gn_b = b.f32("tail.0.bias", now);
  u->tail_w = b.f32("tail.2.weight", (int64_t)3 * now * 9);
  u->tail_b = b.f32("tail.2.bias", 3);
  if (u->bf16 && itsd::g_io_mfma && tail_mfma_ok(H, H, now)) {
    // GroupNorm+SiLU fused into the MFMA tail: coefficients instead of a normalised copy;
    // weights as [9C/32 k-steps][4 lane groups][3 couts][8 k] bf16, k = tap*C + ci
    const float* tw = b.peek("tail.2.weight", (int64_t)3 * now * 9);
    if (tw) {
      const int nks = 9 * now / 32;
      std::vector<uint16_t> wm((size_t)nks * 4 * 3 * 8);
      for (int ks = 0; ks < nks; ++ks)
        for (int kg = 0; kg < 4; ++kg)
          for (int co = 0; co < 3; ++co)
            for (int j = 0; j < 8; ++j) {
              const int k = 32 * ks + 8 * kg + j, tap = k / now, ci = k - tap * now;
              wm[(((size_t)ks * 4 + kg) * 3 + co) * 8 + j] = host_f2bf(tw[((size_t)co * now + ci) * 9 + tap]);
            }
      u->tail_wmf = b.ar.add(wm.data(), wm.size() * 2);
    }
    u->tail_coef = b.ws_off;
    b.ws_off = (b.ws_off + (size_t)u->nb_max * now * 2 * 4 + 255) & ~(size_t)255;
  } else {
    u->tail_g = b.act(H, H, now);
  }

  // all ResBlock temb_proj (and cond_proj) Linears as one [tdim][sumC] matrix
  {
    std::vector<float> Wp((size_t)u->sumC * tdim), bpv(u->sumC), Wc, bcv;
    if (u->cfg) { Wc.resize(Wp.size()); bcv.resize(u->sumC); }
    for (size_t k = 0; k < b.temb_cols.size(); ++k) {
      const std::string& p = b.temb_cols[k].first;
      const size_t col = b.temb_cols[k].second;
      const size_t next = (k + 1 < b.temb_cols.size()) ? b.temb_cols[k + 1].second : (size_t)u->sumC;
      const int oc = (int)(next - col);
      auto fill = [&](const std::string& nm, std::vector<float>& Wd, std::vector<float>& bd) {
        const float* W = b.get(nm + ".weight", (int64_t)oc * tdim);
        const float* bb = b.get(nm + ".bias", oc);
        if (!W || !bb) return;
        for (int o = 0; o < oc; ++o) {
          for (int i = 0; i < tdim; ++i) Wd[(size_t)i * u->sumC + col + o] = W[(size_t)o * tdim + i];
          bd[col + o] = bb[o];
        }
      };
      fill(p + ".temb_proj.1", Wp, bpv);
      if (u->cfg) fill(p + ".cond_proj.1", Wc, bcv);
    }
    u->Wpt = b.ar.add(Wp.data(), Wp.size() * 4);
    u->bp = b.ar.add(bpv.data(), bpv.size() * 4);
    if (u->cfg) {
      u->Wct = b.ar.add(Wc.data(), Wc.size() * 4);
      u->bc = b.ar.add(bcv.data(), bcv.size() * 4);
    }
  }
  if (!b.err.empty()) return fail(ITSD_ERR_WEIGHTS, b.err);
  if ((int)b.used != nviews) {
    return fail(ITSD_ERR_WEIGHTS, "state_dict has " + std::to_string(nviews) + " entries, model uses " +
                                      std::to_string(b.used) + " (unexpected keys present)");
  }
  // a GroupNorm op over the output of the conv right before it (and nothing else): a candidate for conv_small's fused
  // GroupNorm output (conv_args decides per launch; every activation has its own buffer, so the GroupNorm's output
  // never aliases the conv's operands)
  for (size_t i = 1; i < u->ops.size(); ++i) {
    Op& g = u->ops[i];
    Op& p = u->ops[i - 1];
    if (g.kind == OP_GN && g.src2 < 0 && p.kind == OP_CONV && p.dst == g.src1 && p.sc_into < 0 && p.vt < 0) {
      p.gn_next = (int)i;
      g.gn_from = (int)i - 1;
    }
  }
  // channel-statistics slabs for every tensor a GroupNorm reads (written by its producer)
  {
    std::vector<int> need;
    for (const Op& o : u->ops)
      if (o.kind == OP_GN || o.kind == OP_GNCOEF || o.kind == OP_ATTNBLOCK) {
        need.push_back(o.src1);
        if (o.src2 >= 0) need.push_back(o.src2);
      }
    need.push_back(u->tail_in);
    for (int id : need) {
      Act& A = u->acts[id];
      if (A.stats != SIZE_MAX) continue;
      const int HW = A.H * A.W;
      if (!(128 % HW == 0 || HW % 128 == 0))
        return fail(ITSD_ERR_INVALID, "spatial size " + std::to_string(HW) + " not supported by the GN statistics slots");
      const size_t slots = (size_t)u->nb_max * stat_spi(HW, A.spi);
      A.stats = b.ws_off;
      b.ws_off = (b.ws_off + slots * 2 * A.C * 4 + 255) & ~(size_t)255;
      bool produced = (id == u->head_out);
      for (const Op& o : u->ops) produced |= ((o.kind == OP_CONV || o.kind == OP_ATTNBLOCK) && o.dst == id);
      if (!produced) return fail(ITSD_ERR_INVALID, "internal: GroupNorm input without a statistics producer");
    }
  }
  // device arenas
  HIPCHK(hipMalloc(&u->wdev, b.ar.host.size()));
  HIPCHK(hipMemcpy(u->wdev, b.ar.host.data(), b.ar.host.size(), hipMemcpyHostToDevice));
  u->ws_bytes = b.ws_off;
  HIPCHK(hipMalloc(&u->ws, u->ws_bytes));
  return ITSD_OK;
}

// ------------------------------------------------------------------------- program execution
struct RunCtx {
  int nb;                // images in the UNet batch
  const float* x;        // head input NCHW
  int x_mod;             // head reads x[img % x_mod]
  const float* temb;     // temb rows/table base
  const int* tsel;       // device t (table mode) or null
  long long temb_img_stride;
  const int32_t* labels; // CFG labels
  int label_mod;
  int uncond_from;
  TailArgs tail;
  // census
  bool census = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>>* evs = nullptr;
  std::vector<int>* ev_kind = nullptr;
  std::vector<double>* ev_flops = nullptr;
  std::vector<int>* ev_kid = nullptr;  // kernel_id of the op's first launch (itsd_kernel_name)
  std::vector<int>* ev_op = nullptr;   // program op index (1-based; 0 = head / tail) of each launch
};

// The launch arguments of a conv op (shared by launch_op and run_program's gn_fold decision).
int conv_args(itsd_unet* u, const Op& o, const RunCtx& c, ConvArgs& a) {
    const Act& in = u->acts[o.src1];
    const Act& out = u->acts[o.dst];
    a.src1 = u->ap(o.src1);
    a.src2 = o.src2 >= 0 ? u->ap(o.src2) : nullptr;
    a.C1 = in.C;
    a.C2 = o.src2 >= 0 ? u->acts[o.src2].C : 0;
    a.Hin = in.H; a.Win = in.W; a.Hout = out.H; a.Wout = out.W;
    a.ksize = o.ksize; a.stride = o.stride; a.pad = o.pad; a.upsample = o.upsample;
    a.wt = u->wdev + o.wt;
    a.wfrag = o.wfrag != SIZE_MAX ? u->wdev + o.wfrag : nullptr;
    a.Cout = o.Cout; a.K = o.K;
    a.bias = u->wp(o.bias);
    if (o.temb_col >= 0) {
      a.temb = c.temb + o.temb_col;
      a.temb_tsel = c.tsel;
      a.temb_row_stride = u->sumC;
      a.temb_img_stride = c.temb_img_stride;
      if (u->cfg) {
        a.cemb = u->cemb_table + o.temb_col;
        a.cemb_labels = (const int*)c.labels;
        a.cemb_row_stride = u->sumC;
        a.cemb_label_mod = c.label_mod;
        a.cemb_uncond_from = c.uncond_from;
      }
    }
    a.resid = o.resid >= 0 ? u->ap(o.resid) : nullptr;
    a.out = u->ap(o.dst);
    a.M = c.nb * out.H * out.W;
    a.stats = out.stats != SIZE_MAX ? (float*)(u->ws + out.stats) : nullptr;
    a.zero = u->zero_page;
    a.splitk_ws = u->splitk_ws;
    a.splitk_cap = itsd_unet::kSplitkCap;
    a.tickets = u->tickets;
    a.err = u->d_nan + 1;
    a.spin_bound = itsd::g_spin_bound;
    if (o.vt >= 0) {
      if (o.vt_from % 128 || (out.H * out.W) % 8) return fail(ITSD_ERR_INVALID, "internal: bad channel-major V split");
      a.vt_out = u->ap(o.vt);
      a.vt_from = o.vt_from;
    }
    a.zins = o.zins;
    a.dbg = itsd::g_conv_dbg;
    a.xcd = itsd::g_p4_xcd == 1 || (itsd::g_p4_xcd == 2 && a.Wout == 8);
    if (o.subpix) {  // input-grid GEMM with 2x2 (upsample) / 3x3 (ConvTranspose2d) taps per phase (conv.hip)
      a.subpix = o.subpix;
      a.Hout = in.H; a.Wout = in.W;
      a.M = c.nb * in.H * in.W;
      a.ksize = o.subpix == 2 ? o.ksize : 2; a.pad = o.subpix == 2 ? o.pad : 0; a.upsample = 0; a.zins = 0;
      a.K = a.ksize * a.ksize * (a.C1 + a.C2);
      a.tap_live = o.subpix == 2 && a.ksize == 3 && itsd::g_convt_prune;  // (p4: skip the zero taps)
    }
    if (o.coef != SIZE_MAX) {
      if (!u->bf16 || o.ksize != 3 || o.stride != 1 || o.pad != 1 || o.upsample || o.zins ||
          !(conv_gn_eligible(in.H, in.W) || p5_eligible(in.H, in.W)) || a.C1 % 64 || a.C2 % 64 || a.Cout % 128)
        return fail(ITSD_ERR_INVALID, "internal: fused GroupNorm conv on an unsupported shape");
      a.gn_coef = (const float*)(u->ws + o.coef);
    }
    {  // the kernel moves 16-B chunks: every chunk must sit inside one source and one tap
      const int epc = u->bf16 ? 8 : 4;
      if (a.C1 % epc || a.C2 % epc || a.Cout % 4 || a.K % epc)
        return fail(ITSD_ERR_INVALID, "conv channels must be multiples of " + std::to_string(epc));
    }
  // gn_fold: conv3x3_gn_p5_kernel / conv3x3_gn_p4_kernel reduce the input's statistics slabs themselves
  // (run_program then skips the op's gn_coef launch); up to 8 slots an image (32x32): the 32 slots of a
  // 64x64 image made the in-kernel reduction 4-12 dependent load batches (measured: the 64x64 level
  // 0.90 ms folded vs 0.55 ms with its gn_coef launches, C4 at N = 16)
  if (a.gn_coef && o.gn_gamma != SIZE_MAX && itsd::g_gn_fold && (a.C1 + a.C2) % 128 == 0 && in.H * in.W <= 1024 &&
      (conv_p5_selected(a) || conv_p4_selected(a))) {
    a.gn_fold = 1;
    a.gn_st1 = (const float*)(u->ws + u->acts[o.src1].stats);
    a.gn_st2 = o.src2 >= 0 ? (const float*)(u->ws + u->acts[o.src2].stats) : nullptr;
    a.gn_spi1 = u->acts[o.src1].spi;
    a.gn_spi2 = o.src2 >= 0 ? u->acts[o.src2].spi : 0;
    a.gn_gamma = u->wp(o.gn_gamma);
    a.gn_beta = u->wp(o.gn_beta);
  }
  // (round 6) the consumer GroupNorm(+SiLU) in conv_small's epilogue (run_program then skips the GN op): whole-image
  // tiles with one statistics slot an image (HWo <= 16: the CFG model's 2x2 / 1x1 levels), a group's gs = Cout / 32
  // channels inside one 64-cout tile
  if (o.gn_next >= 0 && itsd::g_small_gn && u->bf16 && a.stats && !a.gn_coef && !o.subpix && !a.vt_out &&
      u->acts[o.dst].spi == 0) {
    const int HWo = a.Hout * a.Wout, gs = a.Cout / 32;
    if (HWo <= 16 && 64 % HWo == 0 && a.Cout % 64 == 0 && gs >= 2 && 64 % gs == 0 && conv_small_split(a)) {
      const Op& g = u->ops[o.gn_next];
      a.gn_out = u->ap(g.dst);
      a.go_gamma = u->wp(g.gamma);
      a.go_beta = u->wp(g.beta);
      a.go_silu = g.silu;
    }
  }
  if (o.sc_op >= 0 && itsd::g_p5_sc) {  // the shortcut folded in (run_program then skips the shortcut's launch)
    const Op& sc = u->ops[o.sc_op];
    ConvArgs t = a;
    t.sc_src1 = u->ap(sc.src1);
    t.sc_src2 = sc.src2 >= 0 ? u->ap(sc.src2) : nullptr;
    t.sc_C1 = u->acts[sc.src1].C;
    t.sc_C2 = sc.src2 >= 0 ? u->acts[sc.src2].C : 0;
    t.sc_wfrag = u->wdev + o.sc_wfrag;
    if (conv_p5_sc_fold(t)) {
      a = t;
      a.bias = u->wp(o.bias_sc);
      a.resid = nullptr;
    }
  }
  return ITSD_OK;
}

int launch_op(itsd_unet* u, const Op& o, const RunCtx& c, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (o.kind == OP_GNCOEF) {
    GNArgs g{};
    g.C1 = u->acts[o.src1].C;
    g.C2 = o.src2 >= 0 ? u->acts[o.src2].C : 0;
    g.HW = u->acts[o.src1].H * u->acts[o.src1].W;
    g.gamma = u->wp(o.gamma);
    g.beta = u->wp(o.beta);
    g.eps = 1e-5f;
    g.st1 = (const float*)(u->ws + u->acts[o.src1].stats);
    g.st2 = o.src2 >= 0 ? (const float*)(u->ws + u->acts[o.src2].stats) : nullptr;
    g.spi1 = u->acts[o.src1].spi;
    g.spi2 = o.src2 >= 0 ? u->acts[o.src2].spi : 0;
    e = launch_gn_coef(g, c.nb, (float*)(u->ws + o.coef), s);
  } else if (o.kind == OP_GN) {
    GNArgs a{};
    a.src1 = u->ap(o.src1);
    a.src2 = o.src2 >= 0 ? u->ap(o.src2) : nullptr;
    a.C1 = u->acts[o.src1].C;
    a.C2 = o.src2 >= 0 ? u->acts[o.src2].C : 0;
    a.HW = u->acts[o.src1].H * u->acts[o.src1].W;
    a.gamma = u->wp(o.gamma);
    a.beta = u->wp(o.beta);
    a.eps = 1e-5f;
    a.silu = o.silu;
    a.dst = u->ap(o.dst);
    a.st1 = (const float*)(u->ws + u->acts[o.src1].stats);
    a.st2 = o.src2 >= 0 ? (const float*)(u->ws + u->acts[o.src2].stats) : nullptr;
    a.spi1 = u->acts[o.src1].spi;
    a.spi2 = o.src2 >= 0 ? u->acts[o.src2].spi : 0;
    e = u->bf16 ? launch_groupnorm<bf16_t>(a, c.nb, s) : launch_groupnorm<float>(a, c.nb, s);
  } else if (o.kind == OP_CONV) {
    ConvArgs a{};
    CHK(conv_args(u, o, c, a));
    e = u->bf16 ? launch_conv<bf16_t>(a, s) : launch_conv<float>(a, s);
  } else if (o.kind == OP_ATTNBLOCK) {
    AttnBlockArgs a{};
    const Act& in = u->acts[o.src1];
    const Act& out = u->acts[o.dst];
    a.x = (const bf16_t*)u->ap(o.src1);
    a.st = (const float*)(u->ws + in.stats);
    a.spi = stat_spi(in.H * in.W, in.spi);
    a.gamma = u->wp(o.gamma);
    a.beta = u->wp(o.beta);
    a.wqkv = (const bf16_t*)(u->wdev + o.wt);
    a.bqkv = u->wp(o.bias);
    a.wp = (const bf16_t*)(u->wdev + o.wt2);
    a.bp = u->wp(o.bias2);
    a.out = (bf16_t*)u->ap(o.dst);
    a.out_stats = out.stats != SIZE_MAX ? (float*)(u->ws + out.stats) : nullptr;
    a.scale = (float)std::pow((double)o.C, -0.5);
    a.n = c.nb;
    a.S = o.S;
    // attn_block_split_kernel's slabs in the split-K workspace (ops run in stream order; <= 4 MB of
    // partial scores at n * G <= 256, then the O slab)
    if ((long long)c.nb * 64 * o.C * 2 / 4 + (4ll << 20) / 4 <= itsd_unet::kSplitkCap) {
      a.spart = u->splitk_ws;
      a.oslab = (bf16_t*)(u->splitk_ws + (4ll << 20) / 4);
      a.sync = u->attn_sync;
    }
    a.err = u->d_nan + 1;
    a.spin_bound = itsd::g_spin_bound;
    e = launch_attn_block(a, o.C, s);
  } else {
    AttnArgs a{};
    a.qkv = u->ap(o.src1);
    a.vt = o.vt >= 0 ? u->ap(o.vt) : nullptr;
    a.out = u->ap(o.dst);
    a.S = o.S; a.C = o.C;
    a.scale = (float)std::pow((double)o.C, -0.5);
    e = u->bf16 ? launch_attn<bf16_t>(a, c.nb, s) : launch_attn<float>(a, c.nb, s);
  }
  if (e != hipSuccess) return fail(ITSD_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
  return ITSD_OK;
}

double op_flops(const itsd_unet* u, const Op& o, int nb) {
  if (o.kind == OP_CONV) {  // executed MFMA work (sub-pixel upsample convs: 4 of the 9 taps)
    const Act& out = u->acts[o.dst];
    // (executed: nearest-x2 upsample convs 4 of their 9 taps per output; the sub-pixel ConvTranspose2d's
    // K is already its 9 taps per output)
    return 2.0 * nb * out.H * out.W * (double)o.Cout * (o.subpix == 1 ? o.K * 4 / 9 : o.K);
  }
  if (o.kind == OP_ATTN) return 2.0 * 2.0 * nb * (double)o.S * o.S * o.C;
  if (o.kind == OP_ATTNBLOCK)  // q|k|v and proj projections + the two attention products
    return 2.0 * nb * (double)o.S * (4.0 * o.C * o.C) + 2.0 * 2.0 * nb * (double)o.S * o.S * o.C;
  return 0.0;
}

int run_program(itsd_unet* u, const RunCtx& c, hipStream_t s) {
  int cur_op = 0;  // program op being launched (census: 1-based, 0 head / tail)
  auto mark = [&](int kind, double fl, const std::function<int()>& fn) -> int {
    if (!c.census) return fn();
    if (c.ev_op) c.ev_op->push_back(cur_op);
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    HIPCHK(hipEventRecord(a, s));
    itsd::g_last_kernel = nullptr;
    int r = fn();
    HIPCHK(hipEventRecord(b, s));
    c.evs->push_back({a, b});
    c.ev_kind->push_back(kind);
    c.ev_flops->push_back(fl);
    if (c.ev_kid) c.ev_kid->push_back(itsd::kernel_id(itsd::g_last_kernel));
    return r;
  };
  // head
  CHK(mark(-1, 2.0 * c.nb * u->H * u->H * 27.0 * u->ch, [&]() -> int {
    HeadArgs h{};
    h.x = c.x;
    h.w = u->wp(u->head_w);
    h.b = u->wp(u->head_b);
    h.out = u->ap(u->head_out);
    h.H = u->H; h.W = u->H; h.Cout = u->ch; h.n = c.nb; h.x_img_mod = c.x_mod;
    const Act& ho = u->acts[u->head_out];
    h.stats = ho.stats != SIZE_MAX ? (float*)(u->ws + ho.stats) : nullptr;
    hipError_t e;
    if (u->head_wmf != SIZE_MAX) {
      h.wmf = (const bf16_t*)(u->wdev + u->head_wmf);
      e = launch_head_mfma(h, s);
    } else {
      e = u->bf16 ? launch_head<bf16_t>(h, s) : launch_head<float>(h, s);
    }
    return e == hipSuccess ? ITSD_OK : fail(ITSD_ERR_HIP, hipGetErrorString(e));
  }));
  // census kinds: OpKind, and kCensusConvGN for the fused GroupNorm+SiLU convs
  for (size_t oi = 0; oi < u->ops.size(); ++oi) {
    const Op& o = u->ops[oi];
    if (o.kind == OP_GNCOEF && oi + 1 < u->ops.size() && u->ops[oi + 1].kind == OP_CONV) {
      ConvArgs na{};  // gn_fold: the consumer conv finalizes this GroupNorm itself
      if (conv_args(u, u->ops[oi + 1], c, na) == ITSD_OK && na.gn_fold) continue;
    }
    if (o.kind == OP_GN && o.gn_from >= 0) {
      ConvArgs na{};  // a GroupNorm its producer conv wrote in its epilogue
      if (conv_args(u, u->ops[o.gn_from], c, na) == ITSD_OK && na.gn_out) continue;
    }
    if (o.kind == OP_CONV && o.sc_into >= 0) {
      ConvArgs na{};  // a shortcut its block2 conv runs as K slices
      if (conv_args(u, u->ops[o.sc_into], c, na) == ITSD_OK && na.sc_C1 + na.sc_C2 > 0) continue;
    }
    int kind = o.kind == OP_ATTNBLOCK ? kCensusAttnBlock : (int)o.kind;
    cur_op = (int)oi + 1;
    if (o.kind == OP_CONV && o.coef != SIZE_MAX) {
      const Act& out = u->acts[o.dst];
      const int segs = u->bf16 ? conv_gn_wide_segs(out.H, out.W, c.nb * out.H * out.W, o.Cout) : 0;
      kind = segs == 1 ? kCensusConvGNW : segs == 4 ? kCensusConvGNW4 : kCensusConvGN;
    }
    double fl = op_flops(u, o, c.nb);
    if (c.census && o.kind == OP_CONV && o.sc_op >= 0) {  // + the folded shortcut's K slices (1x1, its Cin)
      ConvArgs na{};
      if (conv_args(u, o, c, na) == ITSD_OK && na.sc_C1 + na.sc_C2 > 0) fl += 2.0 * na.M * (double)o.Cout * (na.sc_C1 + na.sc_C2);
    }
    CHK(mark(kind, fl, [&]() { return launch_op(u, o, c, s); }));
  }
  // tail GN + conv (+ sampler update); bf16 MFMA tail: GN coefficients, then one fused launch
  cur_op = 0;
  Op g;
  g.src1 = u->tail_in; g.gamma = u->tail_gn_g; g.beta = u->tail_gn_b; g.silu = 1;
  if (u->tail_wmf != SIZE_MAX) {
    g.kind = OP_GNCOEF;
    g.coef = u->tail_coef;
  } else {
    g.kind = OP_GN;
    g.dst = u->tail_g;
  }
  CHK(mark((int)g.kind, 0.0, [&]() { return launch_op(u, g, c, s); }));
  CHK(mark(-2, 2.0 * c.tail.n * (c.tail.cfg ? 2 : 1) * u->H * u->H * 27.0 * u->acts[u->tail_in].C, [&]() -> int {
    TailArgs t = c.tail;
    t.w = u->wp(u->tail_w);
    t.b = u->wp(u->tail_b);
    t.H = u->H; t.W = u->H; t.C = u->acts[u->tail_in].C;
    hipError_t e;
    if (u->tail_wmf != SIZE_MAX) {
      t.g = u->ap(u->tail_in);
      t.coef = (const float*)(u->ws + u->tail_coef);
      t.wmf = (const bf16_t*)(u->wdev + u->tail_wmf);
      e = launch_tail_mfma(t, s);
    } else {
      t.g = u->ap(u->tail_g);
      e = u->bf16 ? launch_tail<bf16_t>(t, s) : launch_tail<float>(t, s);
    }
    return e == hipSuccess ? ITSD_OK : fail(ITSD_ERR_HIP, hipGetErrorString(e));
  }));
  return ITSD_OK;
}

// temb rows: out[m][sumC] = Wp^T silu(MLP(emb(idx[m]))) + bp (Model.py:51-93 then each
// ResBlock's temb_proj, :175-178); cond=true uses the label table / cond MLP.
int temb_rows(itsd_unet* u, const int* idx, int M, int offset, bool cond, float* out, hipStream_t s) {
  if (M > u->rows_cap) return fail(ITSD_ERR_INVALID, "temb rows exceed capacity");
  const int ch = u->ch, td = u->tdim;
  hipError_t e;
  if (!cond) {
    e = launch_emb_input(idx, M, u->cfg ? nullptr : u->wp(u->freq), u->cfg ? u->wp(u->ttable) : nullptr, ch,
                         u->emb_buf, offset, s);
  } else {
    e = launch_emb_input(idx, M, nullptr, u->wp(u->ctable), ch, u->emb_buf, offset, s);
  }
  if (e != hipSuccess) return fail(ITSD_ERR_HIP, hipGetErrorString(e));
  const float* W0 = u->wp(cond ? u->C1t : u->W0t);
  const float* b0 = u->wp(cond ? u->cb1 : u->b0);
  const float* W2 = u->wp(cond ? u->C3t : u->W2t);
  const float* b2 = u->wp(cond ? u->cb3 : u->b2);
  HIPCHK(launch_linear(u->emb_buf, M, ch, W0, b0, td, 0, u->h1_buf, s));
  HIPCHK(launch_linear(u->h1_buf, M, td, W2, b2, td, 1, u->te_buf, s));
  HIPCHK(launch_linear(u->te_buf, M, td, u->wp(cond ? u->Wct : u->Wpt), u->wp(cond ? u->bc : u->bp), u->sumC, 1,
                       out, s));
  return ITSD_OK;
}

int alloc_rows(itsd_unet* u, int rows) {
  if (rows <= u->rows_cap) return ITSD_OK;
  hipFree(u->emb_buf); hipFree(u->h1_buf); hipFree(u->te_buf);
  HIPCHK(hipMalloc(&u->emb_buf, (size_t)rows * u->ch * 4));
  HIPCHK(hipMalloc(&u->h1_buf, (size_t)rows * u->tdim * 4));
  HIPCHK(hipMalloc(&u->te_buf, (size_t)rows * u->tdim * 4));
  u->rows_cap = rows;
  return ITSD_OK;
}

void clear_graphs(itsd_unet* u) {
  for (auto& g : u->graphs)
    if (g.exec) hipGraphExecDestroy(g.exec);
  u->graphs.clear();
}

int check_batch(itsd_unet* u, int n) {
  if (n <= 0 || n > u->d.max_batch)
    return fail(ITSD_ERR_INVALID, "batch " + std::to_string(n) + " outside [1, max_batch=" +
                                      std::to_string(u->d.max_batch) + "]");
  return ITSD_OK;
}

}  // namespace

// ============================================================================ C ABI
namespace itsd {
thread_local const char* g_last_kernel = nullptr;
std::mutex& kernel_names_mu() {
  static std::mutex m;
  return m;
}
std::vector<const char*>& kernel_names() {
  static std::vector<const char*> v;
  return v;
}
// ids of launch-site names: 0 = none recorded, else 1 + index in kernel_names() (the names are
// the ITSD_LAUNCH string literals, so equal sites compare equal by content)
int kernel_id(const char* name) {
  if (!name) return 0;
  std::lock_guard<std::mutex> lk(kernel_names_mu());
  auto& v = kernel_names();
  for (size_t i = 0; i < v.size(); ++i)
    if (v[i] == name || !std::strcmp(v[i], name)) return (int)i + 1;
  v.push_back(name);
  return (int)v.size();
}
}  // namespace itsd

extern "C" {

int itsd_version(void) { return 1; }

const char* itsd_kernel_name(int id) {
  std::lock_guard<std::mutex> lk(itsd::kernel_names_mu());
  return id > 0 && id <= (int)itsd::kernel_names().size() ? itsd::kernel_names()[id - 1] : "";
}

int itsd_set_option(const char* key, int value) {
  if (!key) return fail(ITSD_ERR_INVALID, "null key");
#ifndef ITSD_DIAG
  // (round 6) measurement switches -- the conv_dbg ablations, forced attention tilings, the XCD tile
  // order at every level, conv_small's slice floor, forced split-K slice counts and the 7-stage 1x1 ring -- select
  // measured-and-dropped variants: diagnostic builds only (tools/build_diag.sh). The shipped library takes the
  // shipped choices below (auto / off / forced forms of the paths it ships, each A/B'd by a parity test).
  for (const char* dk : {"conv_dbg", "attn_cs", "attn_aq", "p4_xcd", "small_minks", "p5_c64"})
    if (!std::strcmp(key, dk)) return fail(ITSD_ERR_INVALID, std::string(key) + ": diagnostic builds only (tools/build_diag.sh)");
  if (!std::strcmp(key, "splitk") && value > 1) return fail(ITSD_ERR_INVALID, "splitk in [0,1] (forced slice counts: diagnostic builds)");
  if (!std::strcmp(key, "conv1x1") && value > 1) return fail(ITSD_ERR_INVALID, "conv1x1 in [0,1] (the 7-stage ring: diagnostic builds)");
#endif
  ++itsd::g_option_gen;  // cached step graphs baked in the previous kernel choices
  if (!std::strcmp(key, "conv_variant")) {  // 2: conv_pipe (shipped); 1: conv_igemm (register-staged, parity checks)
    if (value < 1 || value > 2) return fail(ITSD_ERR_INVALID, "conv_variant in [1,2]");
    itsd::g_conv_variant = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "splitk")) {
    if (value < 0 || value > 64) return fail(ITSD_ERR_INVALID, "splitk in [0,64]");
    itsd::g_splitk = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "io_mfma")) {  // takes effect for UNets created afterwards
    itsd::g_io_mfma = value ? 1 : 0;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "conv1x1")) {  // streaming 1x1 conv kernel for statistics-free 1x1 convs of large pixel counts
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "conv1x1 in [0,2]");
    itsd::g_conv1x1 = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "small_8x8")) {  // conv_small (split K) for under-filled 8x8-level convs
    if (value < 0 || value > 1) return fail(ITSD_ERR_INVALID, "small_8x8 in [0,1]");
    itsd::g_small_8x8 = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "small_wide")) {  // conv_small for under-filled statistics-free convs of larger images
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "small_wide in [0,2]");
    itsd::g_small_wide = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "small_conv")) {
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "small_conv in [0,2]");
    itsd::g_small_conv = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "conv_dbg")) {  // measurements only (results are wrong when set): 1 no
    // in-loop loads (zero-page sources), 2 no MFMA, 8 no GN transform, 16 no epilogue,
    // 32 no epilogue output stores, 64 fused-conv halo loads from the zero page, 128 no
    // GN statistics pass, 256 no residual loads, 512 (wide fused
    // conv) s_setprio 1 for waves 4-7 (results unchanged), 1024 / 2048 (wide
    // fused conv) every lane reads the same B / A fragment row (LDS broadcast). (Never skip an issued load's wait: an
    // in-flight load landing in a reused register faults.)
    // 4096 | (mask << 13): compile-time ablations of conv3x3_gn_p4_kernel<32> (conv.hip, diagnostic builds)
    // (1 << 20) / (1 << 21): s_setprio 1 / 2 for the halo waves of the fused GroupNorm conv
    const int v = value & (1 | 2 | 8 | 16 | 32 | 64 | 128 | 256 | 512 | 1024 | 2048 | 4096 | (127 << 13) | (3 << 20));
#ifndef ITSD_DIAG
    // validated before it is stored: a refused call leaves the previous setting in place
    if (v & 4096) return fail(ITSD_ERR_INVALID, "conv_dbg 4096 (compile-time ablations): diagnostic builds only (tools/build_diag.sh)");
#endif
    itsd::g_conv_dbg = v;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "gn_wide")) {  // the persistent 256-pixel fused conv: 0 off, 1 auto, 2 whenever eligible
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "gn_wide in [0,2]");
    itsd::g_gn_wide = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "attn_cs")) {  // attn_mfma_kernel output-channel slices: 0 auto, 1..8 forced
    if (value < 0 || value > 8) return fail(ITSD_ERR_INVALID, "attn_cs in [0,8]");
    itsd::g_attn_cs = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "attn_aq")) {  // attn_mfma_kernel queries per block: 0 auto, 32, 64
    if (value != 0 && value != 32 && value != 64) return fail(ITSD_ERR_INVALID, "attn_aq in {0,32,64}");
    itsd::g_attn_aq = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "p4_w")) {  // levels conv3x3_gn_p4_kernel takes (bit 0 W = 8, 1 W = 16, 2 W = 32); others p5 / 128-px
    if (value < 0 || value > 7) return fail(ITSD_ERR_INVALID, "p4_w in [0,7]");
    itsd::g_p4_w = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "splitk_inl")) {  // conv_pipe split-K: 1 in-launch ticket combine, 0 splitk_epilogue_kernel
    if (value < 0 || value > 1) return fail(ITSD_ERR_INVALID, "splitk_inl in [0,1]");
    itsd::g_splitk_inl = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "spin_bound")) {  // diagnostic: polls before an in-kernel hand-off wait fails (shipped 1 << 22)
    if (value < 0) return fail(ITSD_ERR_INVALID, "spin_bound >= 0");
    itsd::g_spin_bound = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "p4_xcd")) {  // conv3x3_gn_p4_kernel: deal each XCD a contiguous range of tiles (0 off, 1 on,
                                       // 2 the 8x8 level only)
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "p4_xcd in [0,2]");
    itsd::g_p4_xcd = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "p4_c96")) {  // 8x8 conv3x3_gn_p4_kernel on 96-cout tiles: 0 off, 1 auto, 2 always (Cout % 96 == 0)
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "p4_c96 in [0,2]");
    itsd::g_p4_c96 = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "p4_sub")) {  // nearest-x2 upsample convs on conv3x3_gn_p4_kernel's sub-pixel form: 0 off, 1 on
    if (value < 0 || value > 1) return fail(ITSD_ERR_INVALID, "p4_sub in [0,1]");
    itsd::g_p4_sub = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "small_minks")) {  // conv_small split K: at least this many 64-channel K-chunks a slice
    if (value < 1 || value > 64) return fail(ITSD_ERR_INVALID, "small_minks in [1,64]");
    itsd::g_small_minks = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "convt_prune")) {  // ConvTranspose2d sub-pixel phases skip their all-zero taps (p4 / conv_pipe)
    if (value < 0 || value > 1) return fail(ITSD_ERR_INVALID, "convt_prune in [0,1]");
    itsd::g_convt_prune = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "subpix_split")) {  // under-filled sub-pixel conv_pipe launches split K in-launch
    if (value < 0 || value > 1) return fail(ITSD_ERR_INVALID, "subpix_split in [0,1]");
    itsd::g_subpix_split = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "p4_plain")) {  // plain 3x3 stride-1 convs on conv3x3_gn_p4_kernel (halo copies the input)
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "p4_plain in [0,2]");
    itsd::g_p4_plain = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "p5")) {  // conv3x3_gn_p5_kernel at 8x8: 0 off, 1 auto, 2 always (4x4: always)
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "p5 in [0,2]");
    itsd::g_p5 = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "p5_split")) {  // its K slices: 0 auto (cost model), 1..16 forced
    if (value < 0 || value > 16) return fail(ITSD_ERR_INVALID, "p5_split in [0,16]");
    itsd::g_p5_split = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "p5_sc")) {  // ResBlock 1x1 shortcuts as K slices of their block2 p5 conv: 0 off, 1 auto, 2 always
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "p5_sc in [0,2]");
    itsd::g_p5_sc = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "small_gn")) {  // conv_small writes its consumer GroupNorm's output (the GN launch skipped): 0 off, 1 on
    if (value < 0 || value > 1) return fail(ITSD_ERR_INVALID, "small_gn in [0,1]");
    itsd::g_small_gn = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "p5_pub")) {  // p5's two-slice last-arriver combine: 1 only the first arriver stores its partial,
                                      // 0 both slices store theirs (round 5; bit-identity checks)
    if (value < 0 || value > 1) return fail(ITSD_ERR_INVALID, "p5_pub in [0,1]");
    itsd::g_p5_pub = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "p5_xl")) {  // p5's split-K partials through one XCD's L2 (slices of a tile on one XCD): 0 off,
                                     // 1 the shared combine at 8x8 / 16x16, 2 every eligible form (A/B), 3 (shipped)
                                     // 1 + the two-slice form at 8x8 / 16x16 where K <= 3456
    if (value < 0 || value > 3) return fail(ITSD_ERR_INVALID, "p5_xl in [0,3]");
    itsd::g_p5_xl = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "p5_dist")) {  // p5's split-K combine shared by every slice (co-resident grids): 0 off (last arriver),
                                       // 1 on, 2 the same plans as 1 combined by the last arriver (bit-identity checks)
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "p5_dist in [0,2]");
    itsd::g_p5_dist = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "p5_c64")) {  // (diagnostic) 64-cout conv3x3_gn_p5_kernel items at 8x8 / 4x4: 0 off, 1 auto, 2 always
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "p5_c64 in [0,2]");
    itsd::g_p5_c64 = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "gn_fold")) {  // GroupNorm finalize inside conv3x3_gn_p4 / p5_kernel: 0 off, 1 on
    itsd::g_gn_fold = value ? 1 : 0;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "attn_split")) {  // attn_block_split_kernel (an image over G blocks): 0 off, 1 auto, 2 / 4 / 6 forced
    if (value != 0 && value != 1 && value != 2 && value != 4 && value != 6)
      return fail(ITSD_ERR_INVALID, "attn_split in {0, 1, 2, 4, 6}");
    itsd::g_attn_split = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "tap_prune")) {  // drop all-padding conv taps at build time (UNets created afterwards)
    itsd::g_tap_prune = value ? 1 : 0;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "down_merge")) {  // CFG DownSample c1 + c2 as one 5x5 conv (UNets created afterwards)
    itsd::g_down_merge = value ? 1 : 0;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "attn_wide_nq")) {  // channel-split attention: query groups a block (0 auto, 1, 2)
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "attn_wide_nq in [0,2]");
    itsd::g_attn_wide_nq = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "attn_wide")) {  // channel-split attention (attn_cs_kernel): 0 off, 1 auto (C >= 384 at S >= 256; C = 1024), 2 wherever it applies
    if (value < 0 || value > 2) return fail(ITSD_ERR_INVALID, "attn_wide in [0,2]");
    itsd::g_attn_wide = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "attn_s1")) {  // one-token AttnBlock folded to GroupNorm + one 1x1 conv (UNets created afterwards)
    if (value < 0 || value > 1) return fail(ITSD_ERR_INVALID, "attn_s1 in [0,1]");
    itsd::g_attn_s1 = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "attn_fuse")) {  // fused AttnBlock kernel (S = 64): 0 off, 1 on (UNets created afterwards)
    if (value < 0 || value > 1) return fail(ITSD_ERR_INVALID, "attn_fuse in [0,1] (the 16-token form was removed)");
    itsd::g_attn_fuse = value;
    return ITSD_OK;
  }
  if (!std::strcmp(key, "fuse_gn")) {  // takes effect for UNets created afterwards
    itsd::g_fuse_gn = value ? 1 : 0;
    return ITSD_OK;
  }
  return fail(ITSD_ERR_INVALID, std::string("unknown option ") + key);
}

const char* itsd_last_error(void) { return g_err.c_str(); }

int itsd_calibrate(int what, double* value, void* stream) {
  if (!value) return fail(ITSD_ERR_INVALID, "null argument");
  if (what != ITSD_CALIB_MFMA_BF16 && what != ITSD_CALIB_HBM_COPY && what != ITSD_CALIB_MFMA_BF16_16X16) return fail(ITSD_ERR_INVALID, "unknown calibration");
  const int rc = calibrate_run(what, value, (hipStream_t)stream);
  if (rc == ITSD_ERR_OOM) return fail(rc, "calibration buffers (2 x 1 GiB)");
  if (rc != ITSD_OK) return fail(rc, "calibration kernel");
  return ITSD_OK;
}

int itsd_unet_query(const itsd_unet* u, const char* key, int64_t* value) {
  if (!u || !key || !value) return fail(ITSD_ERR_INVALID, "null argument");
  if (!std::strcmp(key, "graph_captures")) *value = u->graph_captures;
  else if (!std::strcmp(key, "max_batch")) *value = u->d.max_batch;
  else if (!std::strcmp(key, "T_sched")) *value = u->T_sched;
  else if (!std::strcmp(key, "ws_bytes")) *value = (int64_t)u->ws_bytes;
  else if (!std::strcmp(key, "ops")) *value = (int64_t)u->ops.size();
  else if (!std::strcmp(key, "status")) {  // synchronous: the in-kernel hand-off status word of the last forward / run
    if (hipStreamSynchronize(u->stream) != hipSuccess) return fail(ITSD_ERR_HIP, "status: stream synchronize");
    int flag = 0;
    if (hipMemcpy(&flag, u->d_nan + 1, 4, hipMemcpyDeviceToHost) != hipSuccess) return fail(ITSD_ERR_HIP, "status: copy");
    *value = flag;
  }
  else return fail(ITSD_ERR_INVALID, std::string("unknown query key ") + key);
  return ITSD_OK;
}

int itsd_unet_create(const itsd_unet_desc* desc, const itsd_tensor_view* weights, int n_weights, int device,
                     itsd_unet** out) {
  if (!desc || !out || (!weights && n_weights)) return fail(ITSD_ERR_INVALID, "null argument");
  const itsd_unet_desc& d = *desc;
  if (d.arch != ITSD_ARCH_DDPM && d.arch != ITSD_ARCH_CFG) return fail(ITSD_ERR_INVALID, "unknown arch");
  if (d.ch <= 0 || d.ch % 32 || d.n_mult < 1 || d.n_mult > 8 || d.n_attn < 0 || d.n_attn > 8 ||
      d.num_res_blocks < 1 || d.max_batch < 1 || d.img_size < 8)
    return fail(ITSD_ERR_INVALID, "invalid UNet descriptor");
  if (d.img_size % (1 << (d.n_mult - 1))) return fail(ITSD_ERR_INVALID, "img_size not divisible by the down path");
  for (int k = 0; k < d.n_attn; ++k)
    if (d.attn[k] < 0 || d.attn[k] >= d.n_mult) return fail(ITSD_ERR_INVALID, "attn index out of bound");
  if (d.precision != ITSD_PREC_FP32 && d.precision != ITSD_PREC_BF16) return fail(ITSD_ERR_INVALID, "precision");
  HIPCHK(hipSetDevice(device));
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
      itsd::g_num_cus = cus;
  }
  std::unique_ptr<itsd_unet> u(new itsd_unet());
  u->d = d;
  u->device = device;
  u->bf16 = d.precision == ITSD_PREC_BF16;
  u->esz = u->bf16 ? 2 : 4;
  u->cfg = d.arch == ITSD_ARCH_CFG;
  u->nb_max = d.max_batch * (u->cfg ? 2 : 1);
  CHK(build(u.get(), weights, n_weights));
  HIPCHK(hipStreamCreateWithFlags(&u->stream, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&u->ev_in, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&u->ev_out, hipEventDisableTiming));
  HIPCHK(hipMalloc(&u->d_t, 64));
  HIPCHK(hipMalloc(&u->d_nan, 64));
  HIPCHK(hipMalloc(&u->d_run, sizeof(RunParams)));
  HIPCHK(hipMemset(u->d_run, 0, sizeof(RunParams)));
  HIPCHK(hipMalloc(&u->x_state, (size_t)d.max_batch * 3 * d.img_size * d.img_size * 4));
  HIPCHK(hipMalloc(&u->lab_state, (size_t)d.max_batch * 4));
  HIPCHK(hipMalloc(&u->zero_page, 64 * 4096 + 1024));
  HIPCHK(hipMemset(u->zero_page, 0, 64 * 4096 + 1024));
  HIPCHK(hipMalloc(&u->splitk_ws, itsd_unet::kSplitkCap * 4));
  HIPCHK(hipMalloc(&u->tickets, itsd::kTicketCap * 4));
  HIPCHK(hipMemset(u->tickets, 0, itsd::kTicketCap * 4));
  HIPCHK(hipMalloc(&u->attn_sync, (size_t)u->nb_max * 2 * 4));
  HIPCHK(hipMemset(u->attn_sync, 0, (size_t)u->nb_max * 2 * 4));
  HIPCHK(hipMalloc(&u->proj_buf, (size_t)d.max_batch * u->sumC * 4));
  CHK(alloc_rows(u.get(), std::max(d.max_batch, d.num_labels + 1)));
  if (u->cfg) {
    HIPCHK(hipMalloc(&u->cemb_table, (size_t)(d.num_labels + 1) * u->sumC * 4));
    CHK(temb_rows(u.get(), nullptr, d.num_labels + 1, 0, true, u->cemb_table, u->stream));
    HIPCHK(hipStreamSynchronize(u->stream));
  }
  *out = u.release();
  return ITSD_OK;
}

int itsd_unet_destroy(itsd_unet* u) {
  if (!u) return ITSD_OK;
  hipSetDevice(u->device);
  clear_graphs(u);
  hipFree(u->wdev); hipFree(u->ws); hipFree(u->emb_buf); hipFree(u->h1_buf); hipFree(u->te_buf);
  hipFree(u->proj_buf); hipFree(u->cemb_table); hipFree(u->coeff1); hipFree(u->coeff2); hipFree(u->sqrt_var);
  hipFree(u->temb_table); hipFree(u->d_t); hipFree(u->d_nan); hipFree(u->d_run); hipFree(u->x_state); hipFree(u->lab_state); hipFree(u->zero_page);
  hipFree(u->splitk_ws);
  hipFree(u->tickets);
  hipFree(u->attn_sync);
  if (u->stream) hipStreamDestroy(u->stream);
  if (u->ev_in) hipEventDestroy(u->ev_in);
  if (u->ev_out) hipEventDestroy(u->ev_out);
  delete u;
  return ITSD_OK;
}

int itsd_unet_forward(itsd_unet* u, const float* x, const int32_t* t, const int32_t* labels, float* eps, int n,
                      void* stream) {
  if (!u || !x || !t || !eps) return fail(ITSD_ERR_INVALID, "null argument");
  if (u->cfg && !labels) return fail(ITSD_ERR_INVALID, "CFG UNet needs labels");
  CHK(check_batch(u, n));
  hipStream_t cs = (hipStream_t)stream;
  hipStream_t s = u->stream;
  HIPCHK(hipEventRecord(u->ev_in, cs));
  HIPCHK(hipStreamWaitEvent(s, u->ev_in, 0));
  CHK(temb_rows(u, t, n, 0, false, u->proj_buf, s));
  RunCtx c{};
  c.nb = n; c.x = x; c.x_mod = n;
  c.temb = u->proj_buf; c.tsel = nullptr; c.temb_img_stride = u->sumC;
  c.labels = labels; c.label_mod = n; c.uncond_from = -1;
  c.tail.n = n; c.tail.cfg = 0; c.tail.step_mode = 0; c.tail.eps_out = eps;
  HIPCHK(hipMemsetAsync(u->d_nan + 1, 0, 4, s));  // this forward's hand-off status (itsd_unet_query "status")
  CHK(run_program(u, c, s));
  u->last_forward_n = n;
  HIPCHK(hipEventRecord(u->ev_out, s));
  HIPCHK(hipStreamWaitEvent(cs, u->ev_out, 0));
  return ITSD_OK;
}

int itsd_unet_representation(itsd_unet* u, float* repr, int n, void* stream) {
  if (!u || !repr) return fail(ITSD_ERR_INVALID, "null argument");
  if (u->last_forward_n == 0) return fail(ITSD_ERR_INVALID, "itsd_unet_representation: no itsd_unet_forward on this handle yet");
  if (n < 1 || n > u->last_forward_n)
    return fail(ITSD_ERR_INVALID, "itsd_unet_representation: n outside [1, last forward's batch]");
  HIPCHK(hipSetDevice(u->device));
  const Act& A = u->acts[u->tail_in];
  hipStream_t cs = (hipStream_t)stream;
  hipStream_t s = u->stream;
  HIPCHK(hipEventRecord(u->ev_in, cs));
  HIPCHK(hipStreamWaitEvent(s, u->ev_in, 0));
  HIPCHK(u->bf16 ? launch_nhwc_to_nchw<bf16_t>(u->ap(u->tail_in), repr, n, A.H * A.W, A.C, s)
                 : launch_nhwc_to_nchw<float>(u->ap(u->tail_in), repr, n, A.H * A.W, A.C, s));
  HIPCHK(hipEventRecord(u->ev_out, s));
  HIPCHK(hipStreamWaitEvent(cs, u->ev_out, 0));
  return ITSD_OK;
}

int itsd_set_schedule(itsd_unet* u, int T, const float* coeff1, const float* coeff2, const float* sqrt_var, float w) {
  if (!u || T < 1 || !coeff1 || !coeff2 || !sqrt_var) return fail(ITSD_ERR_INVALID, "bad schedule");
  if (u->cfg && T > u->d.T)
    return fail(ITSD_ERR_INVALID, "CFG time-embedding table has " + std::to_string(u->d.T) + " rows < sampler T");
  HIPCHK(hipSetDevice(u->device));
  clear_graphs(u);
  hipFree(u->coeff1); hipFree(u->coeff2); hipFree(u->sqrt_var); hipFree(u->temb_table);
  u->coeff1 = u->coeff2 = u->sqrt_var = u->temb_table = nullptr;
  HIPCHK(hipMalloc(&u->coeff1, T * 4));
  HIPCHK(hipMalloc(&u->coeff2, T * 4));
  HIPCHK(hipMalloc(&u->sqrt_var, T * 4));
  HIPCHK(hipMemcpy(u->coeff1, coeff1, T * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(u->coeff2, coeff2, T * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(u->sqrt_var, sqrt_var, T * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&u->temb_table, (size_t)T * u->sumC * 4));
  CHK(alloc_rows(u, T));
  CHK(temb_rows(u, nullptr, T, 0, false, u->temb_table, u->stream));
  HIPCHK(hipStreamSynchronize(u->stream));
  u->T_sched = T;
  u->guide_w = w;
  u->guide_w1 = (float)(1.0 + (double)w);
  return ITSD_OK;
}

int itsd_sampler_run(itsd_unet* u, float* x, const int32_t* labels, int n, int t_begin, int t_end, uint64_t seed,
                     int64_t noise_offset, const float* noise, uint32_t flags, void* stream) {
  if (!u || !x) return fail(ITSD_ERR_INVALID, "null argument");
  if (!u->T_sched) return fail(ITSD_ERR_INVALID, "itsd_set_schedule not called");
  if (u->cfg && !labels) return fail(ITSD_ERR_INVALID, "CFG sampler needs labels");
  CHK(check_batch(u, n));
  if (t_begin >= u->T_sched || t_end < 0 || t_end > t_begin) return fail(ITSD_ERR_INVALID, "bad step range");
  HIPCHK(hipSetDevice(u->device));
  u->last_forward_n = 0;  // (the tail input is overwritten: itsd_unet_representation refuses until the next forward)
  hipStream_t cs = (hipStream_t)stream;
  hipStream_t s = u->stream;
  HIPCHK(hipEventRecord(u->ev_in, cs));
  HIPCHK(hipStreamWaitEvent(s, u->ev_in, 0));
  const int clip_at = (flags & ITSD_RUN_CLIP) ? t_end : -1;
  const size_t xbytes = (size_t)n * 3 * u->H * u->H * 4;
  HIPCHK(hipMemcpyAsync(u->x_state, x, xbytes, hipMemcpyDeviceToDevice, s));
  if (labels) HIPCHK(hipMemcpyAsync(u->lab_state, labels, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
  float* xs = u->x_state;
  const int32_t* ls = labels ? u->lab_state : nullptr;

  RunCtx c{};
  c.nb = u->cfg ? 2 * n : n;
  c.x = xs; c.x_mod = n;
  c.temb = u->temb_table; c.tsel = u->d_t; c.temb_img_stride = 0;
  c.labels = ls; c.label_mod = n; c.uncond_from = u->cfg ? n : -1;
  TailArgs& t = c.tail;
  t.n = n; t.cfg = u->cfg ? 1 : 0; t.guide_w = u->guide_w; t.guide_w1 = u->guide_w1;
  t.step_mode = 1; t.x = xs; t.tsel = u->d_t;
  t.coeff1 = u->coeff1; t.coeff2 = u->coeff2; t.sqrt_var = u->sqrt_var;
  t.noise = noise; t.run = u->d_run; t.nan_flag = u->d_nan;

  RunParams rp{};
  rp.seed = seed; rp.noise_offset = noise_offset; rp.clip_at = clip_at;
  HIPCHK(launch_run_begin(u->d_t, t_begin, u->d_nan, u->d_run, rp, s));
  const int steps = t_begin - t_end + 1;
  if (flags & ITSD_RUN_GRAPH) {
    auto key = std::make_tuple(n, labels != nullptr, noise, itsd::g_option_gen);
    hipGraphExec_t exec = nullptr;
    for (auto& g : u->graphs)
      if (g.key == key) exec = g.exec;
    if (!exec) {
      HIPCHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      int r = run_program(u, c, s);
      if (r == ITSD_OK && launch_add_int(u->d_t, -1, s) != hipSuccess) r = fail(ITSD_ERR_HIP, "add_int");
      hipGraph_t graph = nullptr;
      hipError_t e = hipStreamEndCapture(s, &graph);
      if (r != ITSD_OK) { if (graph) hipGraphDestroy(graph); return r; }
      if (e != hipSuccess) return fail(ITSD_ERR_HIP, std::string("capture: ") + hipGetErrorString(e));
      e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
      hipGraphDestroy(graph);
      if (e != hipSuccess) return fail(ITSD_ERR_HIP, std::string("instantiate: ") + hipGetErrorString(e));
      if (u->graphs.size() >= 4) { hipGraphExecDestroy(u->graphs.front().exec); u->graphs.erase(u->graphs.begin()); }
      u->graphs.push_back({key, exec});
      ++u->graph_captures;
    }
    for (int i = 0; i < steps; ++i) HIPCHK(hipGraphLaunch(exec, s));
  } else {
    for (int i = 0; i < steps; ++i) {
      CHK(run_program(u, c, s));
      HIPCHK(launch_add_int(u->d_t, -1, s));
    }
  }
  HIPCHK(hipMemcpyAsync(x, u->x_state, xbytes, hipMemcpyDeviceToDevice, s));
  HIPCHK(hipEventRecord(u->ev_out, s));
  HIPCHK(hipStreamWaitEvent(cs, u->ev_out, 0));
  if (flags & ITSD_RUN_SYNC) {
    HIPCHK(hipStreamSynchronize(s));
    int flag[2] = {0, 0};
    HIPCHK(hipMemcpy(flag, u->d_nan, 8, hipMemcpyDeviceToHost));
    if (flag[1]) return fail(ITSD_ERR_HANDOFF, handoff_msg(flag[1]));
    if (flag[0]) return fail(ITSD_ERR_NAN, "nan in tensor.");
  }
  return ITSD_OK;
}

int itsd_verify(int kind, const float* images, int n_cand, int b, int c, int h, int w, double* scores, void* stream) {
  if (!images || !scores || n_cand < 1 || b < 1) return fail(ITSD_ERR_INVALID, "bad verify arguments");
  if (kind < 0 || kind > 3) return fail(ITSD_ERR_INVALID, "unknown verifier kind");
  if (kind == ITSD_VERIFY_SELFSUP && (c * 64 > 192 || h % 8 || w % 8 || b > 64))
    return fail(ITSD_ERR_INVALID, "selfsup verifier needs c<=3, h,w divisible by 8, b<=64");
  HIPCHK(launch_verify(kind, images, n_cand, b, c, h, w, scores, nullptr, (hipStream_t)stream));
  return ITSD_OK;
}

int itsd_verify_paired(const float* images, const float* ref_features, int n_cand, int c, int h, int w,
                       double* scores, void* stream) {
  if (!images || !ref_features || !scores || n_cand < 1) return fail(ITSD_ERR_INVALID, "bad verify arguments");
  if (c * 64 > 192 || h % 8 || w % 8) return fail(ITSD_ERR_INVALID, "paired selfsup needs c<=3, h,w divisible by 8");
  HIPCHK(launch_verify(4, images, n_cand, 1, c, h, w, scores, ref_features, (hipStream_t)stream));
  return ITSD_OK;
}

int itsd_attention(const void* qkv, const void* vt, void* out, int n, int S, int C, int precision, void* stream) {
  if (!qkv || !out || n < 1 || S < 1 || C < 1) return fail(ITSD_ERR_INVALID, "bad attention arguments");
  if (precision != ITSD_PREC_FP32 && precision != ITSD_PREC_BF16) return fail(ITSD_ERR_INVALID, "precision");
  AttnArgs a{};
  a.qkv = qkv; a.out = out; a.S = S; a.C = C;
  a.scale = (float)std::pow((double)C, -0.5);
  if (precision == ITSD_PREC_BF16) {
    if (C % 8) return fail(ITSD_ERR_INVALID, "C must be a multiple of 8");
    if (vt) {
      if (S % 16 || C % 64 || (S > 256 && !attn_flash_ok(S, C) && !attn_cs_ok(S, C)))
        return fail(ITSD_ERR_INVALID, "MFMA attention needs S % 16 == 0, C % 64 == 0 (S > 256: S % 32 == 0 with C in "
                                      "{64,128,256}, or S % 64 == 0 with C in {256,384,512,1024})");
      a.vt = vt;
    }
    HIPCHK(launch_attn<bf16_t>(a, n, (hipStream_t)stream));
  } else {
    if (C % 4) return fail(ITSD_ERR_INVALID, "C must be a multiple of 4");
    HIPCHK(launch_attn<float>(a, n, (hipStream_t)stream));
  }
  return ITSD_OK;
}

int itsd_noise(float* out, const float* pivot, int n_cand, int64_t per_cand, float scale, uint64_t seed,
               uint32_t stream_id, int64_t cand_offset, void* stream) {
  if (!out || n_cand < 0 || per_cand < 1) return fail(ITSD_ERR_INVALID, "bad noise arguments");
  if (n_cand == 0) return ITSD_OK;
  HIPCHK(launch_noise(out, pivot, n_cand, per_cand, scale, seed, stream_id, cand_offset, (hipStream_t)stream));
  return ITSD_OK;
}

int itsd_profile_forward(itsd_unet* u, const float* x, const int32_t* t, int n, double* conv_ms, double* conv_flops,
                         int* conv_launches, double* total_ms, void* stream) {
  if (!u || !x || !t) return fail(ITSD_ERR_INVALID, "null argument");
  if (u->cfg) return fail(ITSD_ERR_INVALID, "profile_forward: DDPM only");
  CHK(check_batch(u, n));
  HIPCHK(hipSetDevice(u->device));
  u->last_forward_n = 0;  // (the tail input is overwritten: itsd_unet_representation refuses until the next forward)
  hipStream_t s = u->stream;
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  float* eps = nullptr;
  HIPCHK(hipMalloc(&eps, (size_t)n * 3 * u->H * u->H * 4));
  CHK(temb_rows(u, t, n, 0, false, u->proj_buf, s));
  std::vector<std::pair<hipEvent_t, hipEvent_t>> evs;
  std::vector<int> kinds;
  std::vector<double> fl;
  RunCtx c{};
  c.nb = n; c.x = x; c.x_mod = n;
  c.temb = u->proj_buf; c.temb_img_stride = u->sumC;
  c.label_mod = n; c.uncond_from = -1;
  c.tail.n = n; c.tail.step_mode = 0; c.tail.eps_out = eps;
  c.census = true; c.evs = &evs; c.ev_kind = &kinds; c.ev_flops = &fl;
  int r = run_program(u, c, s);
  hipError_t e = hipStreamSynchronize(s);
  double cm = 0, cf = 0, tm = 0;
  int cl = 0;
  for (size_t i = 0; i < evs.size(); ++i) {
    float ms = 0.f;
    if (r == ITSD_OK && e == hipSuccess) hipEventElapsedTime(&ms, evs[i].first, evs[i].second);
    tm += ms;
    if (kinds[i] == OP_CONV || kinds[i] == kCensusConvGN || kinds[i] == kCensusConvGNW ||
        kinds[i] == kCensusConvGNW4) {
      cm += ms; cf += fl[i]; ++cl;
    }
    hipEventDestroy(evs[i].first);
    hipEventDestroy(evs[i].second);
  }
  hipFree(eps);
  CHK(r);
  HIPCHK(e);
  if (conv_ms) *conv_ms = cm;
  if (conv_flops) *conv_flops = cf;
  if (conv_launches) *conv_launches = cl;
  if (total_ms) *total_ms = tm;
  return ITSD_OK;
}

int itsd_profile_op(itsd_unet* u, const float* x, const int32_t* t, int n, int op_index, int reps, double* ms,
                    void* stream) {
  if (!u || !x || !t || !ms || reps < 1) return fail(ITSD_ERR_INVALID, "null argument or reps < 1");
  if (op_index < 1 || op_index > (int)u->ops.size()) return fail(ITSD_ERR_INVALID, "profile_op: op_index out of range");
  CHK(check_batch(u, n));
  HIPCHK(hipSetDevice(u->device));
  u->last_forward_n = 0;  // (the tail input is overwritten: itsd_unet_representation refuses until the next forward)
  hipStream_t s = u->stream;
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  float* eps = nullptr;
  HIPCHK(hipMalloc(&eps, (size_t)n * 3 * u->H * u->H * 4));
  // CFG: label 0 (the unconditional row) for every image -- the guided batch's launches, shapes
  // and FLOPs
  int32_t* lab0 = nullptr;
  if (u->cfg) {
    HIPCHK(hipMalloc(&lab0, (size_t)n * 4));
    HIPCHK(hipMemsetAsync(lab0, 0, (size_t)n * 4, s));
  }
  int r = temb_rows(u, t, n, 0, false, u->proj_buf, s);
  RunCtx c{};
  c.nb = n; c.x = x; c.x_mod = n;
  c.temb = u->proj_buf; c.temb_img_stride = u->sumC;
  c.labels = lab0; c.label_mod = n; c.uncond_from = -1;
  c.tail.n = n; c.tail.step_mode = 0; c.tail.eps_out = eps;
  if (r == ITSD_OK) r = run_program(u, c, s);  // every op's inputs in place
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipError_t e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  const Op& o = u->ops[op_index - 1];
  if (r == ITSD_OK && e == hipSuccess) r = launch_op(u, o, c, s);  // warm
  if (r == ITSD_OK && e == hipSuccess) e = hipEventRecord(e0, s);
  for (int i = 0; i < reps && r == ITSD_OK && e == hipSuccess; ++i) r = launch_op(u, o, c, s);
  if (r == ITSD_OK && e == hipSuccess) e = hipEventRecord(e1, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  float m = 0.f;
  if (r == ITSD_OK && e == hipSuccess) e = hipEventElapsedTime(&m, e0, e1);
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  hipFree(eps);
  if (lab0) hipFree(lab0);
  CHK(r);
  HIPCHK(e);
  *ms = (double)m / reps;
  return ITSD_OK;
}

int itsd_profile_ops(itsd_unet* u, const float* x, const int32_t* t, int n, int max_ops, int* kinds, double* ms,
                     double* flops, int* shapes, int* n_ops, void* stream) {
  if (!u || !x || !t || !n_ops) return fail(ITSD_ERR_INVALID, "null argument");
  CHK(check_batch(u, n));
  HIPCHK(hipSetDevice(u->device));
  u->last_forward_n = 0;  // (the tail input is overwritten: itsd_unet_representation refuses until the next forward)
  hipStream_t s = u->stream;
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  float* eps = nullptr;
  HIPCHK(hipMalloc(&eps, (size_t)n * 3 * u->H * u->H * 4));
  int32_t* lab0 = nullptr;  // CFG: label 0 for every image (as itsd_profile_op)
  if (u->cfg) {
    HIPCHK(hipMalloc(&lab0, (size_t)n * 4));
    HIPCHK(hipMemsetAsync(lab0, 0, (size_t)n * 4, s));
  }
  CHK(temb_rows(u, t, n, 0, false, u->proj_buf, s));
  std::vector<std::pair<hipEvent_t, hipEvent_t>> evs;
  std::vector<int> kd, kid, eop;
  std::vector<double> fl;
  RunCtx c{};
  c.nb = n; c.x = x; c.x_mod = n;
  c.temb = u->proj_buf; c.temb_img_stride = u->sumC;
  c.labels = lab0; c.label_mod = n; c.uncond_from = -1;
  c.tail.n = n; c.tail.step_mode = 0; c.tail.eps_out = eps;
  c.census = true; c.evs = &evs; c.ev_kind = &kd; c.ev_flops = &fl; c.ev_kid = &kid; c.ev_op = &eop;
  int r = run_program(u, c, s);
  hipError_t e = hipStreamSynchronize(s);
  // launch order: head, ops..., tail GN, tail
  int k = 0;
  for (size_t i = 0; i < evs.size(); ++i) {
    float m = 0.f;
    if (r == ITSD_OK && e == hipSuccess) hipEventElapsedTime(&m, evs[i].first, evs[i].second);
    hipEventDestroy(evs[i].first);
    hipEventDestroy(evs[i].second);
    if (k >= max_ops) continue;
    if (kinds) kinds[k] = (kid[i] << 8) | (kd[i] & 0xff);
    if (ms) ms[k] = m;
    if (flops) flops[k] = fl[i];
    if (shapes) {
      int* sh = shapes + 8 * k;
      for (int q = 0; q < 8; ++q) sh[q] = 0;
      sh[6] = eop[i];
      if (eop[i] >= 1) {
        const Op& o = u->ops[eop[i] - 1];
        const Act& out = u->acts[o.dst >= 0 ? o.dst : o.src1];
        const Act& in = u->acts[o.src1];
        sh[0] = n * out.H * out.W;
        sh[1] = o.kind == OP_CONV ? o.Cout : out.C;
        sh[2] = o.kind == OP_CONV ? o.K : in.C + (o.src2 >= 0 ? u->acts[o.src2].C : 0);
        sh[3] = out.H;
        sh[4] = o.ksize;
        sh[5] = o.stride * 10 + o.upsample;
        // flags for the algorithmic-bytes count (bench.py conv_alg_bytes): bit 0 a residual operand, bit 1 the
        // output's GroupNorm statistics written, bit 2 the input GroupNorm(+SiLU) fused (its statistics read)
        sh[7] = (o.resid >= 0 ? 1 : 0) | (out.stats != SIZE_MAX ? 2 : 0) | (o.coef != SIZE_MAX ? 4 : 0);
        if (o.kind == OP_CONV && o.sc_op >= 0) {  // a block2 conv with its 1x1 shortcut folded in as K slices: no
          ConvArgs na{};                          // residual operand; the shortcut's input channels in bits 8..
          if (conv_args(u, o, c, na) == ITSD_OK && na.sc_C1 + na.sc_C2 > 0) sh[7] = (sh[7] & ~1) | ((na.sc_C1 + na.sc_C2) << 8);
        }
      }
    }
    ++k;
  }
  *n_ops = k;
  hipFree(eps);
  if (lab0) hipFree(lab0);
  CHK(r);
  HIPCHK(e);
  return ITSD_OK;
}

}  // extern "C"
