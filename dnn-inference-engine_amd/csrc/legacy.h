// Internal per-op helpers behind the two drop-in ABIs (abi_openblas.cpp, abi_avx.cpp).
#pragma once
#include <vector>

namespace dnnhip {
void legacy_begin();                          // clear the thread's last error
void legacy_report(const char* fn, int rc);  // print a failure to stderr
// order 0: w rows (kh, kw, ic) [HWIO]; order 1: w rows (ic, kh, kw) [kernel_r]
int legacy_conv(const float* in, const float* w, int order, float* out, int B, int oh, int ow, int od, int ih,
                int iw, int ic, int kh, int kw, int sh, int sw);
int legacy_im2col(const float* imb, float* colb, int oh, int ow, int ih, int iw, int ic, int kh, int kw, int sh,
                  int sw);
int legacy_pool(const float* in, float* out, int B, int oh, int ow, int od, int ih, int iw, int ic, int kh, int kw,
                int sh, int sw, int gt_below);
int legacy_bias_add(const float* in, const float* b, float* out, int B, int H, int W, int C);
int legacy_bn_mvg(const float* in, const float* mean, const float* var, const float* gamma, float eps, float* out,
                  int B, int H, int W, int C);
int legacy_bn_ab(const float* in, const float* alpha, const float* beta, float* out, int B, int H, int W, int C);
int legacy_leaky(const float* in, float* out, int B, int H, int W, int C, int f32_variant);
}  // namespace dnnhip
