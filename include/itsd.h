/*
 * itsd.h — C ABI of libitsd_hip.so, the MI355X (gfx950) search-over-noise sampler.
 *
 * The reference exposes this path as Python duck-typed objects;
 * each entry point below replaces one of them:
 *
 *   itsd_unet_create / _destroy  <- UNet(T, ch, ch_mult, attn, num_res_blocks, dropout)
 *                                   + load_state_dict   (Diffusion/Model.py:213,
 *                                   DiffusionFreeGuidence/ModelCondition.py:165,
 *                                   Diffusion/Train.py:814-818)
 *   itsd_unet_forward            <- UNet.forward(x, t[, labels])   (Model.py:265,
 *                                   ModelCondition.py:206)
 *   itsd_unet_representation     <- UNet.forward(..., return_representation=True)'s second
 *                                   output, the pre-tail h (ModelCondition.py:206,225-235)
 *   itsd_set_schedule            <- GaussianDiffusionSampler.__init__ tables
 *                                   (Diffusion/Diffusion.py:51-65, DiffusionCondition.py:57-73)
 *   itsd_sampler_run             <- GaussianDiffusionSampler.forward loop
 *                                   (Diffusion.py:84-102, DiffusionCondition.py:89-105)
 *   itsd_verify                  <- OracleVerifier / SelfSupervisedVerifier /
 *                                   AestheticPredictor .score (search/verifier.py:45-66,
 *                                   223-248, 262-287), batched per candidate
 *   itsd_verify_paired           <- SelfSupervisedVerifier.score(images, reference_features)
 *                                   (search/verifier.py:235-240)
 *   itsd_attention               <- AttnBlock core softmax(q k^T C^-0.5) v
 *                                   (Diffusion/Model.py:152-161, ModelCondition.py:105-115)
 *   itsd_profile_forward / _ops / _op, itsd_unet_query, itsd_set_option
 *                                <- (no reference counterpart) per-kernel census used by
 *                                   bench.py for the roofline line, introspection, A/B switches
 *
 * Conventions
 *  - Every tensor argument is a DEVICE pointer owned by the caller; the library
 *    borrows it for the stream-ordered duration of the call. Weights passed to
 *    itsd_unet_create are HOST fp32 pointers (a state_dict on CPU); they are
 *    repacked and copied, and may be freed after the call returns.
 *  - Layouts at the boundary are the reference's: images NCHW fp32, timesteps and
 *    labels int32 per sample. Internally activations are NHWC (bf16 or fp32).
 *  - Every function returns ITSD_OK (0) or an error code; no exception or abort
 *    crosses the ABI. itsd_last_error() returns a thread-local message.
 *  - Calls are asynchronous on the given stream (a hipStream_t passed as void*;
 *    NULL = the default stream) unless documented otherwise. One handle per
 *    device/process; a handle is not thread-safe.
 */
#ifndef ITSD_H
#define ITSD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ITSD_OK 0
#define ITSD_ERR_INVALID 1   /* bad argument / shape / unsupported configuration */
#define ITSD_ERR_HIP 2       /* a HIP runtime call failed */
#define ITSD_ERR_WEIGHTS 3   /* state_dict key or shape mismatch (load_state_dict strict) */
#define ITSD_ERR_NAN 4       /* the sampler produced a NaN (Diffusion.py:100 assert) */
#define ITSD_ERR_OOM 5
#define ITSD_ERR_HANDOFF 6   /* an in-kernel cross-block hand-off wait exhausted its poll bound (the grid was not
                                co-resident); its outputs are NaN. Reported by itsd_sampler_run with ITSD_RUN_SYNC
                                and by itsd_unet_query(u, "status", ...) after itsd_unet_forward */

enum { ITSD_ARCH_DDPM = 0, ITSD_ARCH_CFG = 1 };
enum { ITSD_PREC_FP32 = 0, ITSD_PREC_BF16 = 1 };
enum { ITSD_VERIFY_ORACLE = 0, ITSD_VERIFY_SELFSUP = 1, ITSD_VERIFY_AESTHETIC = 2, ITSD_VERIFY_MEAN = 3 };

/* itsd_sampler_run flags */
#define ITSD_RUN_GRAPH 1u   /* capture one denoising step in a hipGraph and replay it */
#define ITSD_RUN_CLIP 2u    /* clip(x, -1, 1) after the last step (Diffusion.py:102) */
#define ITSD_RUN_SYNC 4u    /* synchronise at the end and report ITSD_ERR_NAN */

typedef struct itsd_unet itsd_unet;

/* Constructor arguments of the reference UNets plus sizing. */
typedef struct {
  int32_t arch;            /* ITSD_ARCH_DDPM (Model.py) or ITSD_ARCH_CFG (ModelCondition.py) */
  int32_t T;               /* model T (CFG: rows of the time-embedding table) */
  int32_t ch;              /* 'channel' */
  int32_t n_mult;
  int32_t ch_mult[8];      /* 'channel_mult' */
  int32_t n_attn;
  int32_t attn[8];         /* 'attn' level indices (DDPM only) */
  int32_t num_res_blocks;
  int32_t img_size;        /* H = W */
  int32_t num_labels;      /* CFG only */
  int32_t max_batch;       /* largest n passed to forward/sampler (CFG: per-branch n) */
  int32_t precision;       /* ITSD_PREC_FP32 (parity) or ITSD_PREC_BF16 (throughput) */
} itsd_unet_desc;

/* One state_dict entry (host fp32, contiguous, reference key name). */
typedef struct {
  const char* name;
  const float* data;
  int64_t numel;
} itsd_tensor_view;

int itsd_unet_create(const itsd_unet_desc* desc, const itsd_tensor_view* weights, int n_weights,
                     int device, itsd_unet** out);
int itsd_unet_destroy(itsd_unet* u);

/* eps[n,3,H,W] = UNet(x[n,3,H,W], t[n]) (DDPM) or UNet(x, t, labels[n]) (CFG). */
int itsd_unet_forward(itsd_unet* u, const float* x, const int32_t* t, const int32_t* labels,
                      float* eps, int n, void* stream);

/* repr[n,C,H,W] (NCHW fp32) = the pre-tail activation h of the LAST itsd_unet_forward on this handle
 * (ModelCondition.py:225-235: last_representation = h before self.tail), C = ch * ch_mult[0];
 * stream-ordered after that forward (same stream, or synchronised); n <= that forward's n. */
int itsd_unet_representation(itsd_unet* u, float* repr, int n, void* stream);

/* Host fp32 tables of length T: coeff1, coeff2 and sqrt(var) (the fp32 casts the
 * reference's extract() produces, Diffusion.py:9-16), plus the CFG weight w. */
int itsd_set_schedule(itsd_unet* u, int T, const float* coeff1, const float* coeff2,
                      const float* sqrt_var, float w);

/* Run steps t_begin..t_end (inclusive, descending) of the ancestral sampler in
 * place on x[n,3,H,W]. With ITSD_RUN_GRAPH one denoising step is captured per
 * (n, x, labels, noise, option state) and replayed: seed, noise_offset and the clip
 * step are device-side run parameters, so rounds that differ only in them reuse it. noise == NULL: z ~ N(0,1) from counter-based Philox keyed
 * (seed, step, noise_offset + element); otherwise noise is [T][n][3][H][W] fp32 and
 * step t uses noise[t] (t >= 1; the reference draws no noise at t = 0). labels: CFG only. */
int itsd_sampler_run(itsd_unet* u, float* x, const int32_t* labels, int n, int t_begin, int t_end,
                     uint64_t seed, int64_t noise_offset, const float* noise, uint32_t flags, void* stream);

/* out[c][e] = (pivot ? pivot[e] : 0) + scale * z, z ~ N(0,1) from Philox keyed
 * (seed, stream_id, (cand_offset + c) * per_cand + e), for c < n_cand, e < per_cand.
 * Candidate noises are thus a function of their GLOBAL index, so every rank can
 * regenerate any candidate (search_algorithm.py:67 randn, :225 pivot + randn*(1-lambda)). */
int itsd_noise(float* out, const float* pivot, int n_cand, int64_t per_cand, float scale, uint64_t seed,
               uint32_t stream_id, int64_t cand_offset, void* stream);

/* scores[c] = verifier(images[c*b:(c+1)*b]) for c < n_cand; images NCHW fp32.
 * ITSD_VERIFY_MEAN is OracleVerifier.score with dataset_stats (search/verifier.py:66: mean). */
int itsd_verify(int kind, const float* images, int n_cand, int b, int c, int h, int w,
                double* scores, void* stream);

/* SelfSupervisedVerifier.score(images, reference_features) (search/verifier.py:235-240):
 * scores[i] = cos(pool8x8(images[i]), ref_features[i]) for i < n_cand (one image per
 * candidate: the reference's .item() of the per-image vector needs a single image);
 * ref_features [n_cand][c*64] fp32. */
int itsd_verify_paired(const float* images, const float* ref_features, int n_cand, int c, int h, int w,
                       double* scores, void* stream);

/* AttnBlock core on n images of S tokens, width C (single head):
 *   out[i][s][:] = softmax_j(q_s . k_j * C^-0.5) v_j
 * qkv: [n][S][3C] (q | k | v per token, the fused projection the UNet produces);
 * precision ITSD_PREC_FP32: fp32 tensors; ITSD_PREC_BF16: bf16 tensors and vt, the
 * channel-major V [n][C][S] (the MFMA kernels read V^T; S <= 256: whole-row kernel,
 * S > 256: the flash kernel, S % 32 == 0 and C in {64,128,256}, or the channel-split kernel,
 * S % 64 == 0 and C in {256,384,512,1024}), out [n][S][C]. */
int itsd_attention(const void* qkv, const void* vt, void* out, int n, int S, int C, int precision, void* stream);

/* Census of one forward at batch n (synchronous): runs the op program eagerly with
 * HIP events around every launch. Outputs (any may be NULL):
 *   conv_ms / conv_flops / conv_launches : the implicit-GEMM conv kernel
 *   total_ms                              : the whole forward (sum of launches) */
int itsd_profile_forward(itsd_unet* u, const float* x, const int32_t* t, int n, double* conv_ms,
                         double* conv_flops, int* conv_launches, double* total_ms, void* stream);

/* Per-launch census of one forward (synchronous, eager, HIP events): for launch i
 * (head, program ops in order, tail GN, tail) kinds[i] = (kernel << 8) | (kind & 0xff) with
 * kind the op class (0 GN, 1 conv, 2 attention, 3 GN finalize, 4/5/6 fused GroupNorm conv
 * 128 px / 256 px / 8x8 level; -1 head, -2 tail, as a signed byte) and kernel the id of
 * the first kernel the launch ran (itsd_kernel_name), ms[i], flops[i] and shapes[8*i..] =
 * {M, Cout, K or Cin, Hout, ksize, 10*stride+upsample, op, flags} with op the program op index
 * (1-based, itsd_profile_op's numbering; 0 = head / tail). Ops whose launch is folded into the
 * next one (a GroupNorm finalize done by conv3x3_gn_p5_kernel) have no entry. kind 7 = the fused
 * AttnBlock. flags: bit 0 the op adds a residual, bit 1 it writes its output's GroupNorm statistics, bit 2
 * its input GroupNorm(+SiLU) is fused (statistics read). CFG UNets run with label 0.
 * At most max_ops entries; *n_ops = entries written. */
int itsd_profile_ops(itsd_unet* u, const float* x, const int32_t* t, int n, int max_ops, int* kinds,
                     double* ms, double* flops, int* shapes, int* n_ops, void* stream);

/* Steady-state duration of one program op (synchronous): runs one forward at batch n to set up
 * its inputs, then launches op `op_index` (census numbering of itsd_profile_ops: 1 = first
 * program op) `reps` times back to back between two HIP events on the UNet's stream;
 * *ms = elapsed / reps. The per-launch time a replayed step graph sees, without the eager
 * census's per-launch event overhead. */
int itsd_profile_op(itsd_unet* u, const float* x, const int32_t* t, int n, int op_index, int reps, double* ms,
                    void* stream);

/* Process-wide choices between the shipped paths (api.hip lists every key and its range): kernel and tile
 * choices ("conv_variant", "splitk" 0/1, "splitk_inl", "small_conv", "gn_wide", "fuse_gn", "io_mfma", "p4_w",
 * "p4_sub", "p4_plain", "p4_c96", "p5", "p5_split", "p5_sc", "p5_pub", "p5_dist", "p5_xl", "gn_fold", "attn_split", "attn_wide",
 * "attn_wide_nq", "conv1x1" 0/1, "small_wide", "small_8x8", "subpix_split", "convt_prune"), the in-kernel hand-off
 * poll bound ("spin_bound"), and build-time choices read at create ("attn_fuse", "attn_s1", "tap_prune",
 * "down_merge"). Defaults are the shipped choices; every alternative is covered by a parity test. Measurement
 * switches of measured-and-dropped variants ("conv_dbg", "attn_cs", "attn_aq", "p4_xcd", "small_minks", forced
 * "splitk" slice counts, "conv1x1" 2) exist in diagnostic builds only (tools/build_diag.sh): this library returns
 * ITSD_ERR_INVALID for them. */
int itsd_set_option(const char* key, int value);

/* Introspection of a handle (no device work): "graph_captures" (step graphs captured and
 * instantiated so far; a search replays one graph across all its rounds), "max_batch",
 * "T_sched", "ws_bytes" (activation arena), "ops" (program length); and, synchronising the
 * handle's stream, "status" = the in-kernel hand-off status word of the last forward / sampler run
 * (0 ok; bit 0: attn_block_split_kernel's wait exhausted its bound, bit 1: conv3x3_gn_p5_kernel's shared split-K
 * combine -- ITSD_ERR_HANDOFF). */
int itsd_unet_query(const itsd_unet* u, const char* key, int64_t* value);

/* Name of census kernel id `id` (itsd_profile_ops): the launch site's kernel expression,
 * e.g. "conv3x3_gn_p4_kernel<32>"; "" for 0 / unknown ids. */
const char* itsd_kernel_name(int id);

/* On-box peak calibration (synchronous on stream; measurement only, no reference counterpart):
 * ITSD_CALIB_MFMA_BF16 -> *value = the achievable dense bf16 MFMA rate in TFLOP/s (v_mfma_f32_32x32x16_bf16
 * chains on random operands, every CU, 2 waves per SIMD); ITSD_CALIB_HBM_COPY -> *value = the achievable
 * HBM streaming rate in GB/s (a 1 GiB 16-B-per-lane copy, bytes read + written); ITSD_CALIB_MFMA_BF16_16X16
 * -> the ITSD_CALIB_MFMA_BF16 loop on v_mfma_f32_16x16x32_bf16 (the chip holds another clock under that shape).
 * bench.py reports its roofline fractions against these as well as against the datasheet peaks. */
enum { ITSD_CALIB_MFMA_BF16 = 0, ITSD_CALIB_HBM_COPY = 1, ITSD_CALIB_MFMA_BF16_16X16 = 2 };
int itsd_calibrate(int what, double* value, void* stream);

const char* itsd_last_error(void);
int itsd_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ITSD_H */
