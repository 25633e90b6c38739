// On-box peak calibration ("re-measure both on the box"): the achievable bf16 MFMA
// rate and the achievable HBM streaming rate of THIS device, so that bench.py can report its roofline
// fractions against the box as well as against the datasheet (boxes of one pool differ by +-5-8 %;
// MI355X_MICROARCH.md, DVFS item 5). Measurement only: no reference counterpart.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "common.h"
#include "itsd.h"

namespace itsd {

// bf16 MFMA loop: every CU runs 2 blocks of 4 waves (2 waves per SIMD, as the fused convs), each wave
// 8 independent v_mfma_f32_32x32x16_bf16 chains on RANDOM operands (the clock the chip holds under load
// depends on the data: zero operands clock higher, MI355X_MICROARCH.md DVFS item 1); the sum of the
// accumulators is stored so nothing is dead.
__global__ __launch_bounds__(256, 2) void calib_mfma_kernel(float* out, int iters, uint32_t seed) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  auto hash = [](uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
  };
  // bf16 operands of magnitude [0.5, 1) with random sign and mantissa
  auto rnd8 = [&](uint32_t k) {
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (short)((hash(seed ^ (gid * 64 + k * 8 + e)) & 0x807F) | 0x3F00);
    return v;
  };
  bf16x8 av[4], bv[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) av[i] = rnd8(i);
#pragma unroll
  for (int j = 0; j < 2; ++j) bv[j] = rnd8(4 + j);
  f32x16 acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.0f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c & 3], bv[c >> 2], acc[c], 0, 0, 0);
  }
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[gid] = s;
}

// the same loop on v_mfma_f32_16x16x32_bf16 (16 independent chains a wave, equal FLOP per chain step x 1/2):
// the chip holds a different clock under the two shapes (MI355X_MICROARCH.md DVFS item 7)
__global__ __launch_bounds__(256, 2) void calib_mfma16_kernel(float* out, int iters, uint32_t seed) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  auto hash = [](uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
  };
  auto rnd8 = [&](uint32_t k) {
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (short)((hash(seed ^ (gid * 64 + k * 8 + e)) & 0x807F) | 0x3F00);
    return v;
  };
  bf16x8 av[4], bv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) av[i] = rnd8(i);
#pragma unroll
  for (int j = 0; j < 4; ++j) bv[j] = rnd8(4 + j);
  f32x4 acc[16];
#pragma unroll
  for (int c = 0; c < 16; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[c][r] = 0.0f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < 16; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c & 3], bv[c >> 2], acc[c], 0, 0, 0);
  }
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < 16; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) s += acc[c][r];
  out[gid] = s;
}

// HBM streaming copy: 16 B a lane loads and stores, 4 independent loads in flight per lane before their
// stores (a grid-stride loop of single loads leaves each wave one load deep), nontemporal stores
// (MI355X_MICROARCH.md: float4 copy measured 6.29 TB/s of the 8 TB/s spec); bytes counted = read + written.
// n is a multiple of 4 * gridDim.x * blockDim.x (the host sizes it so).
__global__ __launch_bounds__(256) void calib_copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v[u], dst + i + u * stride);
  }
}

// what: ITSD_CALIB_MFMA_BF16 (ITSD_CALIB_MFMA_BF16_16X16) -> TFLOP/s, ITSD_CALIB_HBM_COPY -> GB/s (read + written); synchronous on s.
// Returns ITSD_OK, ITSD_ERR_OOM (buffers) or ITSD_ERR_HIP.
int calibrate_run(int what, double* value, hipStream_t s) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess) return ITSD_ERR_HIP;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return ITSD_ERR_HIP;
  double best = 0.0;
  int rc = 0;
  if (what == ITSD_CALIB_MFMA_BF16 || what == ITSD_CALIB_MFMA_BF16_16X16) {
    const bool m16 = what == ITSD_CALIB_MFMA_BF16_16X16;
    const int blocks = 2 * cus, iters = 1 << 15;  // ~8.6e13 FLOP: tens of ms at ~2 PFLOP/s
    float* out = nullptr;
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) rc = ITSD_ERR_OOM;
    for (int r = 0; r < 4 && !rc; ++r) {  // the first launch warms the clock; the best of the rest
      hipEventRecord(e0, s);
      if (m16) hipLaunchKernelGGL(calib_mfma16_kernel, dim3(blocks), dim3(256), 0, s, out, iters, 0x9e3779b9u + r);
      else hipLaunchKernelGGL(calib_mfma_kernel, dim3(blocks), dim3(256), 0, s, out, iters, 0x9e3779b9u + r);
      hipEventRecord(e1, s);
      if (hipEventSynchronize(e1) != hipSuccess) { rc = ITSD_ERR_HIP; break; }
      float ms = 0.0f;
      hipEventElapsedTime(&ms, e0, e1);
      // (8 MFMAs of 32x32x16 or 16 of 16x16x32 a wave per iteration: 2^18 FLOP either way)
      const double flops = (double)blocks * 4 /* waves */ * iters * 8 * 32768.0;
      if (r > 0) best = std::max(best, flops / (ms * 1e-3) / 1e12);  // TFLOP/s
    }
    hipFree(out);
  } else {
    const long long bytes = 1ll << 30;  // 1 GiB each way: far past the 256 MiB Infinity Cache
    void *src = nullptr, *dst = nullptr;
    if (hipMalloc(&src, bytes) != hipSuccess || hipMalloc(&dst, bytes) != hipSuccess) rc = ITSD_ERR_OOM;
    if (!rc && hipMemsetAsync(src, 1, bytes, s) != hipSuccess) rc = ITSD_ERR_HIP;
    for (int r = 0; r < 4 && !rc; ++r) {
      hipEventRecord(e0, s);
      // (1 GiB / 16 B = 2^26 units, a multiple of 4 x the 2^12 blocks x 256 threads: every index in range)
      hipLaunchKernelGGL(calib_copy_kernel, dim3(4096), dim3(256), 0, s, (const u32x4*)src, (u32x4*)dst, bytes / 16);
      hipEventRecord(e1, s);
      if (hipEventSynchronize(e1) != hipSuccess) { rc = ITSD_ERR_HIP; break; }
      float ms = 0.0f;
      hipEventElapsedTime(&ms, e0, e1);
      if (r > 0) best = std::max(best, 2.0 * (double)bytes / (ms * 1e-3) / 1e9);  // GB/s, read + write
    }
    hipFree(src);
    hipFree(dst);
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  // (read and cleared on every path: a failed hipMalloc leaves hipErrorOutOfMemory as this thread's last error, which
  // the next launch_* helper would report as its own kernel-launch failure)
  const hipError_t last = hipGetLastError();
  if (!rc && last != hipSuccess) rc = ITSD_ERR_HIP;
  *value = best;
  return rc;
}

}  // namespace itsd
