// Host AddressSanitizer driver for the C ABI's argument validation (SURVEY.md §5 "race detection /
// sanitizers"): every entry point of include/itsd.h is called with each class of invalid argument it
// rejects, and the calls that pass validation on a machine without a GPU must fail cleanly with
// ITSD_ERR_HIP (no leak, no use-after-free, no overflow in the error paths). Built by
// tools/asan_build.sh with api.hip compiled under -Xarch_host -fsanitize=address; run by
// tests/test_asan_abi.py (CPU). Exit status 0 = every expectation held.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "itsd.h"

static int g_fail = 0;

static void expect(const char* what, int got, int want) {
  const char* msg = itsd_last_error();
  if (got != want) {
    std::printf("FAIL %s: got %d want %d (%s)\n", what, got, want, msg ? msg : "(null)");
    ++g_fail;
    return;
  }
  if (want != ITSD_OK && (!msg || !*msg)) {
    std::printf("FAIL %s: error %d without a message\n", what, got);
    ++g_fail;
    return;
  }
  std::printf("ok   %s -> %d (%s)\n", what, got, want == ITSD_OK ? "" : msg);
}

static itsd_unet_desc arch_a() {
  itsd_unet_desc d;
  std::memset(&d, 0, sizeof(d));
  d.arch = ITSD_ARCH_DDPM;
  d.T = 1000;
  d.ch = 128;
  d.n_mult = 4;
  d.ch_mult[0] = 1; d.ch_mult[1] = 2; d.ch_mult[2] = 3; d.ch_mult[3] = 4;
  d.n_attn = 1;
  d.attn[0] = 2;
  d.num_res_blocks = 2;
  d.img_size = 32;
  d.max_batch = 4;
  d.precision = ITSD_PREC_BF16;
  return d;
}

int main() {
  expect("itsd_version", itsd_version() >= 1 ? ITSD_OK : 1, ITSD_OK);

  // ---- itsd_calibrate: argument checks (no device here: a valid request fails in HIP)
  {
    double v = 0.0;
    expect("calibrate null value", itsd_calibrate(ITSD_CALIB_MFMA_BF16, nullptr, nullptr), ITSD_ERR_INVALID);
    expect("calibrate what=7", itsd_calibrate(7, &v, nullptr), ITSD_ERR_INVALID);
    expect("calibrate mfma, no GPU", itsd_calibrate(ITSD_CALIB_MFMA_BF16, &v, nullptr), ITSD_ERR_HIP);
  }

  // ---- itsd_set_option: null / unknown key, out-of-range values, valid values restored
  expect("set_option null key", itsd_set_option(nullptr, 0), ITSD_ERR_INVALID);
  expect("set_option unknown key", itsd_set_option("no_such_option", 1), ITSD_ERR_INVALID);
  expect("set_option conv_variant=9", itsd_set_option("conv_variant", 9), ITSD_ERR_INVALID);
  expect("set_option splitk=-1", itsd_set_option("splitk", -1), ITSD_ERR_INVALID);
  expect("set_option small_conv=3", itsd_set_option("small_conv", 3), ITSD_ERR_INVALID);
  expect("set_option gn_wide=7", itsd_set_option("gn_wide", 7), ITSD_ERR_INVALID);
  expect("set_option gn_reg=4 (removed)", itsd_set_option("gn_reg", 4), ITSD_ERR_INVALID);
  expect("set_option conv_wide=0 (removed)", itsd_set_option("conv_wide", 0), ITSD_ERR_INVALID);
  expect("set_option p4_m16=1 (removed)", itsd_set_option("p4_m16", 1), ITSD_ERR_INVALID);
  // round 6: measurement switches are diagnostic-build only
  expect("set_option conv_dbg=1 (diagnostic)", itsd_set_option("conv_dbg", 1), ITSD_ERR_INVALID);
  expect("set_option attn_cs=2 (diagnostic)", itsd_set_option("attn_cs", 2), ITSD_ERR_INVALID);
  expect("set_option attn_aq=32 (diagnostic)", itsd_set_option("attn_aq", 32), ITSD_ERR_INVALID);
  expect("set_option p4_xcd=1 (diagnostic)", itsd_set_option("p4_xcd", 1), ITSD_ERR_INVALID);
  expect("set_option small_minks=2 (diagnostic)", itsd_set_option("small_minks", 2), ITSD_ERR_INVALID);
  expect("set_option splitk=2 (diagnostic)", itsd_set_option("splitk", 2), ITSD_ERR_INVALID);
  expect("set_option conv1x1=2 (diagnostic)", itsd_set_option("conv1x1", 2), ITSD_ERR_INVALID);
  expect("set_option p5_c64=2 (diagnostic)", itsd_set_option("p5_c64", 2), ITSD_ERR_INVALID);
  expect("set_option p5_dist=3", itsd_set_option("p5_dist", 3), ITSD_ERR_INVALID);
  expect("set_option p5_dist=1", itsd_set_option("p5_dist", 1), ITSD_OK);
  expect("set_option p5_pub=2", itsd_set_option("p5_pub", 2), ITSD_ERR_INVALID);
  expect("set_option p5_pub=1", itsd_set_option("p5_pub", 1), ITSD_OK);
  expect("set_option conv_variant=3 (removed)", itsd_set_option("conv_variant", 3), ITSD_ERR_INVALID);
  expect("set_option conv_variant=2 (default)", itsd_set_option("conv_variant", 2), ITSD_OK);
  expect("set_option spin_bound=-1", itsd_set_option("spin_bound", -1), ITSD_ERR_INVALID);
  expect("set_option spin_bound=4194304 (default)", itsd_set_option("spin_bound", 1 << 22), ITSD_OK);
  expect("set_option p4_xcd=3", itsd_set_option("p4_xcd", 3), ITSD_ERR_INVALID);
  expect("set_option attn_aq=48", itsd_set_option("attn_aq", 48), ITSD_ERR_INVALID);
  expect("set_option p4_w=8 (64x64 removed)", itsd_set_option("p4_w", 8), ITSD_ERR_INVALID);
  expect("set_option convt_prune=2", itsd_set_option("convt_prune", 2), ITSD_ERR_INVALID);
  expect("set_option convt_prune=1 (default)", itsd_set_option("convt_prune", 1), ITSD_OK);
  expect("set_option attn_wide=3", itsd_set_option("attn_wide", 3), ITSD_ERR_INVALID);
  expect("set_option tail_px=64 (removed)", itsd_set_option("tail_px", 64), ITSD_ERR_INVALID);
  expect("set_option small_minks=0", itsd_set_option("small_minks", 0), ITSD_ERR_INVALID);
  expect("set_option attn_fuse=2 (removed)", itsd_set_option("attn_fuse", 2), ITSD_ERR_INVALID);
  expect("set_option attn_fuse=1 (default)", itsd_set_option("attn_fuse", 1), ITSD_OK);
  expect("set_option small_minks=8 (diagnostic)", itsd_set_option("small_minks", 8), ITSD_ERR_INVALID);
  expect("set_option conv_dbg=0 (diagnostic)", itsd_set_option("conv_dbg", 0), ITSD_ERR_INVALID);
  {  // a long key: the error message copies it
    std::string k(4096, 'k');
    expect("set_option 4 KiB key", itsd_set_option(k.c_str(), 0), ITSD_ERR_INVALID);
  }

  // ---- itsd_unet_create: every descriptor check, then the HIP failure path (no device here)
  itsd_unet* u = nullptr;
  itsd_unet_desc d = arch_a();
  expect("create null desc", itsd_unet_create(nullptr, nullptr, 0, 0, &u), ITSD_ERR_INVALID);
  expect("create null out", itsd_unet_create(&d, nullptr, 0, 0, nullptr), ITSD_ERR_INVALID);
  expect("create weights null, n>0", itsd_unet_create(&d, nullptr, 3, 0, &u), ITSD_ERR_INVALID);
  struct Bad {
    const char* what;
    void (*mut)(itsd_unet_desc&);
  } bad[] = {
      {"arch=7", [](itsd_unet_desc& x) { x.arch = 7; }},
      {"ch=0", [](itsd_unet_desc& x) { x.ch = 0; }},
      {"ch=100 (not /32)", [](itsd_unet_desc& x) { x.ch = 100; }},
      {"n_mult=0", [](itsd_unet_desc& x) { x.n_mult = 0; }},
      {"n_mult=9", [](itsd_unet_desc& x) { x.n_mult = 9; }},
      {"n_attn=-1", [](itsd_unet_desc& x) { x.n_attn = -1; }},
      {"n_attn=9", [](itsd_unet_desc& x) { x.n_attn = 9; }},
      {"num_res_blocks=0", [](itsd_unet_desc& x) { x.num_res_blocks = 0; }},
      {"max_batch=0", [](itsd_unet_desc& x) { x.max_batch = 0; }},
      {"img_size=4", [](itsd_unet_desc& x) { x.img_size = 4; }},
      {"img_size=36 (down path)", [](itsd_unet_desc& x) { x.img_size = 36; }},
      {"attn level 4 of 4", [](itsd_unet_desc& x) { x.attn[0] = 4; }},
      {"attn level -1", [](itsd_unet_desc& x) { x.attn[0] = -1; }},
      {"precision=5", [](itsd_unet_desc& x) { x.precision = 5; }},
  };
  for (const Bad& b : bad) {
    itsd_unet_desc x = arch_a();
    b.mut(x);
    u = nullptr;
    expect((std::string("create ") + b.what).c_str(), itsd_unet_create(&x, nullptr, 0, 0, &u), ITSD_ERR_INVALID);
    if (u) {
      std::printf("FAIL create %s: handle written on error\n", b.what);
      ++g_fail;
    }
  }
  {
    std::vector<float> w(16, 0.f);
    itsd_tensor_view tv{"head.weight", w.data(), (int64_t)w.size()};
    u = nullptr;
    const int rc = itsd_unet_create(&d, &tv, 1, 0, &u);
    expect("create valid desc, no GPU", rc, ITSD_ERR_HIP);
    if (u) {
      std::printf("FAIL create: handle written on error\n");
      ++g_fail;
    }
  }
  expect("destroy null", itsd_unet_destroy(nullptr), ITSD_OK);

  // ---- handle-taking entry points with a null handle
  float f[16] = {0};
  int32_t ti[4] = {0};
  double dd[4] = {0};
  int ki[4] = {0};
  int64_t q = 0;
  expect("forward null handle", itsd_unet_forward(nullptr, f, ti, nullptr, f, 1, nullptr), ITSD_ERR_INVALID);
  expect("representation null handle", itsd_unet_representation(nullptr, f, 1, nullptr), ITSD_ERR_INVALID);
  expect("set_schedule null handle", itsd_set_schedule(nullptr, 4, f, f, f, 0.f), ITSD_ERR_INVALID);
  expect("sampler_run null handle", itsd_sampler_run(nullptr, f, nullptr, 1, 3, 0, 1, 0, nullptr, 0, nullptr),
         ITSD_ERR_INVALID);
  expect("query null handle", itsd_unet_query(nullptr, "ops", &q), ITSD_ERR_INVALID);
  expect("profile_forward null handle",
         itsd_profile_forward(nullptr, f, ti, 1, dd, dd, ki, dd, nullptr), ITSD_ERR_INVALID);
  expect("profile_ops null handle", itsd_profile_ops(nullptr, f, ti, 1, 4, ki, dd, dd, ki, ki, nullptr),
         ITSD_ERR_INVALID);
  expect("profile_op null handle", itsd_profile_op(nullptr, f, ti, 1, 1, 1, dd, nullptr), ITSD_ERR_INVALID);

  // ---- itsd_verify
  expect("verify null images", itsd_verify(0, nullptr, 1, 1, 3, 32, 32, dd, nullptr), ITSD_ERR_INVALID);
  expect("verify null scores", itsd_verify(0, f, 1, 1, 3, 32, 32, nullptr, nullptr), ITSD_ERR_INVALID);
  expect("verify n_cand=0", itsd_verify(0, f, 0, 1, 3, 32, 32, dd, nullptr), ITSD_ERR_INVALID);
  expect("verify b=0", itsd_verify(0, f, 1, 0, 3, 32, 32, dd, nullptr), ITSD_ERR_INVALID);
  expect("verify kind=4", itsd_verify(4, f, 1, 1, 3, 32, 32, dd, nullptr), ITSD_ERR_INVALID);
  expect("verify kind=-1", itsd_verify(-1, f, 1, 1, 3, 32, 32, dd, nullptr), ITSD_ERR_INVALID);
  expect("verify selfsup c=4", itsd_verify(1, f, 1, 2, 4, 32, 32, dd, nullptr), ITSD_ERR_INVALID);
  expect("verify selfsup h=30", itsd_verify(1, f, 1, 2, 3, 30, 32, dd, nullptr), ITSD_ERR_INVALID);
  expect("verify selfsup b=65", itsd_verify(1, f, 1, 65, 3, 32, 32, dd, nullptr), ITSD_ERR_INVALID);
  // ---- itsd_verify_paired
  expect("verify_paired null images", itsd_verify_paired(nullptr, f, 1, 3, 32, 32, dd, nullptr), ITSD_ERR_INVALID);
  expect("verify_paired null ref", itsd_verify_paired(f, nullptr, 1, 3, 32, 32, dd, nullptr), ITSD_ERR_INVALID);
  expect("verify_paired null scores", itsd_verify_paired(f, f, 1, 3, 32, 32, nullptr, nullptr), ITSD_ERR_INVALID);
  expect("verify_paired n_cand=0", itsd_verify_paired(f, f, 0, 3, 32, 32, dd, nullptr), ITSD_ERR_INVALID);
  expect("verify_paired c=4", itsd_verify_paired(f, f, 1, 4, 32, 32, dd, nullptr), ITSD_ERR_INVALID);
  expect("verify_paired w=30", itsd_verify_paired(f, f, 1, 3, 32, 30, dd, nullptr), ITSD_ERR_INVALID);

  // ---- itsd_attention
  expect("attention null qkv", itsd_attention(nullptr, nullptr, f, 1, 16, 64, 1, nullptr), ITSD_ERR_INVALID);
  expect("attention null out", itsd_attention(f, nullptr, nullptr, 1, 16, 64, 1, nullptr), ITSD_ERR_INVALID);
  expect("attention n=0", itsd_attention(f, nullptr, f, 0, 16, 64, 1, nullptr), ITSD_ERR_INVALID);
  expect("attention precision=2", itsd_attention(f, nullptr, f, 1, 16, 64, 2, nullptr), ITSD_ERR_INVALID);
  expect("attention bf16 C=12", itsd_attention(f, nullptr, f, 1, 16, 12, 1, nullptr), ITSD_ERR_INVALID);
  expect("attention bf16+vt S=20", itsd_attention(f, f, f, 1, 20, 64, 1, nullptr), ITSD_ERR_INVALID);
  expect("attention bf16+vt C=96", itsd_attention(f, f, f, 1, 16, 96, 1, nullptr), ITSD_ERR_INVALID);
  expect("attention wide S=1056 C=512 (S % 64)", itsd_attention(f, f, f, 1, 1056, 512, 1, nullptr), ITSD_ERR_INVALID);
  expect("attention S=1024 C=768", itsd_attention(f, f, f, 1, 1024, 768, 1, nullptr), ITSD_ERR_INVALID);
  expect("attention fp32 C=6", itsd_attention(f, nullptr, f, 1, 16, 6, 0, nullptr), ITSD_ERR_INVALID);

  // ---- itsd_noise
  expect("noise null out", itsd_noise(nullptr, nullptr, 1, 16, 1.f, 0, 0, 0, nullptr), ITSD_ERR_INVALID);
  expect("noise n_cand=-1", itsd_noise(f, nullptr, -1, 16, 1.f, 0, 0, 0, nullptr), ITSD_ERR_INVALID);
  expect("noise per_cand=0", itsd_noise(f, nullptr, 1, 0, 1.f, 0, 0, 0, nullptr), ITSD_ERR_INVALID);
  expect("noise n_cand=0 (no-op)", itsd_noise(f, nullptr, 0, 16, 1.f, 0, 0, 0, nullptr), ITSD_OK);

  std::printf("%s (%d failures)\n", g_fail ? "FAILED" : "PASSED", g_fail);
  return g_fail ? 1 : 0;
}
