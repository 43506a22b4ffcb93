// Per-op host-pointer entry points shared by the two drop-in ABIs (include/dnn_hip.h,
// include/dnn_hip_avx.h).  The reference's per-op contract: caller-owned
// host NHWC fp32 buffers, synchronous, result valid on return.  Each call stages its
// operands in a grow-only device arena (no per-call hipMalloc, unlike dnn_cuda.cu:193-210
// and dnn_cublas.cu:149-169), runs the gfx950 kernels, and copies the result back.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <algorithm>
#include <mutex>
#include <vector>
#include "dnn_common.h"
#include "legacy.h"

namespace dnnhip {

namespace {
std::mutex g_mu;
constexpr int kSlots = 8;
void* g_slot[kSlots];
size_t g_size[kSlots];
int g_device = -1;

float* slot(int i, size_t floats) {
  size_t bytes = std::max<size_t>(floats, 1) * sizeof(float);
  if (g_size[i] < bytes) {
    if (g_slot[i]) (void)hipFree(g_slot[i]);
    g_slot[i] = nullptr;
    g_size[i] = 0;
    if (hipMalloc(&g_slot[i], bytes) != hipSuccess) {
      set_error("device arena: hipMalloc(%zu) failed", bytes);
      return nullptr;
    }
    g_size[i] = bytes;
  }
  return static_cast<float*>(g_slot[i]);
}

int ensure_device() {
  int dev = 0;
  DNN_HIP_TRY(hipGetDevice(&dev));
  if (g_device != dev) {  // arena belongs to one device; drop it on a device switch
    for (int i = 0; i < kSlots; ++i) {
      if (g_slot[i]) (void)hipFree(g_slot[i]);
      g_slot[i] = nullptr;
      g_size[i] = 0;
    }
    g_device = dev;
  }
  return 0;
}

#define SLOT(var, i, n)                 \
  float* var = slot((i), (n));          \
  if (!(var)) return -1

int h2d(float* d, const float* h, size_t n) {
  if (n) DNN_HIP_TRY(hipMemcpy(d, h, n * sizeof(float), hipMemcpyHostToDevice));
  return 0;
}
int d2h(float* h, const float* d, size_t n) {
  if (n) DNN_HIP_TRY(hipMemcpy(h, d, n * sizeof(float), hipMemcpyDeviceToHost));
  return 0;
}
}  // namespace

void legacy_begin() { set_error("%s", ""); }

void legacy_report(const char* fn, int rc) {
  if (rc) fprintf(stderr, "dnn_hip: %s failed: %s\n", fn, last_error());
}

int legacy_conv(const float* in, const float* w, int order, float* out, int B, int oh, int ow, int od, int ih,
                int iw, int ic, int kh, int kw, int sh, int sw) {
  DNN_REQUIRE(B >= 0 && oh > 0 && ow > 0 && od > 0 && ih > 0 && iw > 0 && ic > 0 && kh > 0 && kw > 0 && sh > 0 &&
                  sw > 0,
              "conv: bad shape");
  DNN_REQUIRE((oh - 1) * sh + kh <= ih && (ow - 1) * sw + kw <= iw,
              "conv: output %dx%d does not fit the padded input %dx%d", oh, ow, ih, iw);
  if (B == 0) return 0;
  std::lock_guard<std::mutex> lk(g_mu);
  if (int rc = ensure_device()) return rc;
  const long long M = (long long)B * oh * ow;
  const int K = kh * kw * ic;
  const int cfg = choose_gemm_cfg(M, od, K);
  const int Kpad = (K + gemm_cfg_bk(cfg) - 1) / gemm_cfg_bk(cfg) * gemm_cfg_bk(cfg);
  const int Npad = (od + gemm_cfg_bn(cfg) - 1) / gemm_cfg_bn(cfg) * gemm_cfg_bn(cfg);
  const size_t n_in = (size_t)B * ih * iw * ic, n_out = (size_t)M * od;
  SLOT(d_in, 0, n_in);
  SLOT(d_w, 1, (size_t)K * od);
  SLOT(d_bt, 2, (size_t)Npad * Kpad);
  SLOT(d_col, 3, (size_t)M * Kpad);
  SLOT(d_out, 4, n_out);
  if (int rc = h2d(d_in, in, n_in)) return rc;
  if (int rc = h2d(d_w, w, (size_t)K * od)) return rc;
  if (int rc = launch_pack_weights(d_w, d_bt, K, od, Kpad, Npad, order, kh, kw, ic, 0)) return rc;
  ConvGeom g{B, ih, iw, ic, oh, ow, kh, kw, sh, sw, 0, 0, K, Kpad};
  if (int rc = launch_im2col(d_in, d_col, g, 0)) return rc;
  EpiParams epi{nullptr, nullptr, nullptr, nullptr, 0};
  // same split-K rule as the plan, so per-op and fused results agree bit for bit
  const int splits = (cfg >= GEMM_128x128_K32 && Kpad == K) ? choose_splitk(od, K) : 1;
  float* d_slab = nullptr;
  if (splits > 1) {
    d_slab = slot(5, (size_t)splits * M * od);
    if (!d_slab) return -1;
  }
  if (int rc = launch_gemm(cfg, d_col, Kpad, d_bt, Kpad, d_out, od, M, od, Kpad, epi, 0, splits, d_slab)) return rc;
  if (splits > 1)
    if (int rc = launch_splitk_reduce(d_slab, splits, M, od, d_out, od, epi, 0)) return rc;
  return d2h(out, d_out, n_out);
}

int legacy_im2col(const float* imb, float* colb, int oh, int ow, int ih, int iw, int ic, int kh, int kw, int sh,
                  int sw) {
  // K order (ic, kh, kw) as dnn_openblas.c:135-158, gathered in that order on the device
  // (im2col_ckk_kernel).  Diagnostic entry point only: the plan uses implicit GEMM.
  DNN_REQUIRE(oh > 0 && ow > 0 && ic > 0 && kh > 0 && kw > 0 && sh > 0 && sw > 0, "im2col: bad shape");
  DNN_REQUIRE((oh - 1) * sh + kh <= ih && (ow - 1) * sw + kw <= iw, "im2col: window exceeds input");
  std::lock_guard<std::mutex> lk(g_mu);
  if (int rc = ensure_device()) return rc;
  const int K = kh * kw * ic;
  const size_t M = (size_t)oh * ow, n_in = (size_t)ih * iw * ic;
  SLOT(d_in, 0, n_in);
  SLOT(d_col, 3, M * K);
  if (int rc = h2d(d_in, imb, n_in)) return rc;
  ConvGeom g{1, ih, iw, ic, oh, ow, kh, kw, sh, sw, 0, 0, K, K};
  if (int rc = launch_im2col_ckk(d_in, d_col, g, 0)) return rc;
  return d2h(colb, d_col, M * K);
}

int legacy_pool(const float* in, float* out, int B, int oh, int ow, int od, int ih, int iw, int ic, int kh, int kw,
                int sh, int sw, int gt_below) {
  DNN_REQUIRE(B >= 0 && oh > 0 && ow > 0 && od > 0 && kh > 0 && kw > 0 && sh > 0 && sw > 0, "max_pool2d: bad shape");
  DNN_REQUIRE(od == ic, "max_pool2d: od (%d) != ic (%d)", od, ic);
  DNN_REQUIRE((oh - 1) * sh + kh <= ih && (ow - 1) * sw + kw <= iw, "max_pool2d: window exceeds input");
  if (B == 0) return 0;
  std::lock_guard<std::mutex> lk(g_mu);
  if (int rc = ensure_device()) return rc;
  const size_t n_in = (size_t)B * ih * iw * ic, n_out = (size_t)B * oh * ow * od;
  SLOT(d_in, 0, n_in);
  SLOT(d_out, 4, n_out);
  if (int rc = h2d(d_in, in, n_in)) return rc;
  PoolGeom g{B, ih, iw, ic, oh, ow, kh, kw, sh, sw, 0, 0, gt_below};
  if (int rc = launch_maxpool(d_in, d_out, g, 0)) return rc;
  return d2h(out, d_out, n_out);
}

int legacy_bias_add(const float* in, const float* b, float* out, int B, int H, int W, int C) {
  DNN_REQUIRE(B >= 0 && H >= 0 && W >= 0 && C > 0, "bias_add: bad shape");
  const size_t n = (size_t)B * H * W * C;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> lk(g_mu);
  if (int rc = ensure_device()) return rc;
  SLOT(d_in, 0, n);
  SLOT(d_out, 4, n);
  SLOT(d_b, 5, C);
  if (int rc = h2d(d_in, in, n)) return rc;
  if (int rc = h2d(d_b, b, C)) return rc;
  if (int rc = launch_bias_add(d_in, d_b, d_out, (long long)n, C, 0)) return rc;
  return d2h(out, d_out, n);
}

int legacy_bn_mvg(const float* in, const float* mean, const float* var, const float* gamma, float eps, float* out,
                  int B, int H, int W, int C) {
  DNN_REQUIRE(B >= 0 && H >= 0 && W >= 0 && C > 0, "batch_norm: bad shape");
  const size_t n = (size_t)B * H * W * C;
  if (n == 0) return 0;
  std::vector<float> sq(C);
  for (int d = 0; d < C; ++d) {
    volatile float s = var[d] + eps;  // fp32 add, then sqrt (dnn_openblas.c:48-50)
    sq[d] = sqrtf(s);
  }
  std::lock_guard<std::mutex> lk(g_mu);
  if (int rc = ensure_device()) return rc;
  SLOT(d_in, 0, n);
  SLOT(d_out, 4, n);
  SLOT(d_m, 5, C);
  SLOT(d_s, 6, C);
  SLOT(d_g, 7, C);
  if (int rc = h2d(d_in, in, n)) return rc;
  if (int rc = h2d(d_m, mean, C)) return rc;
  if (int rc = h2d(d_s, sq.data(), C)) return rc;
  if (int rc = h2d(d_g, gamma, C)) return rc;
  if (int rc = launch_bn_mvg(d_in, d_m, d_s, d_g, d_out, (long long)n, C, 0)) return rc;
  return d2h(out, d_out, n);
}

int legacy_bn_ab(const float* in, const float* alpha, const float* beta, float* out, int B, int H, int W, int C) {
  DNN_REQUIRE(B >= 0 && H >= 0 && W >= 0 && C > 0, "batch_norm: bad shape");
  const size_t n = (size_t)B * H * W * C;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> lk(g_mu);
  if (int rc = ensure_device()) return rc;
  SLOT(d_in, 0, n);
  SLOT(d_out, 4, n);
  SLOT(d_a, 5, C);
  SLOT(d_b, 6, C);
  if (int rc = h2d(d_in, in, n)) return rc;
  if (int rc = h2d(d_a, alpha, C)) return rc;
  if (int rc = h2d(d_b, beta, C)) return rc;
  if (int rc = launch_bn_ab(d_in, d_a, d_b, d_out, (long long)n, C, 0)) return rc;
  return d2h(out, d_out, n);
}

int legacy_leaky(const float* in, float* out, int B, int H, int W, int C, int f32_variant) {
  DNN_REQUIRE(B >= 0 && H >= 0 && W >= 0 && C >= 0, "leaky_relu: bad shape");
  const size_t n = (size_t)B * H * W * C;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> lk(g_mu);
  if (int rc = ensure_device()) return rc;
  SLOT(d_in, 0, n);
  SLOT(d_out, 4, n);
  if (int rc = h2d(d_in, in, n)) return rc;
  if (int rc = launch_leaky(d_in, d_out, (long long)n, f32_variant, 0)) return rc;
  return d2h(out, d_out, n);
}

}  // namespace dnnhip
