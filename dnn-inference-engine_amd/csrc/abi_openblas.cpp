// libdnn_hip.so front-end: the OpenBLAS / cuBLAS engine ABI (include/dnn_hip.h).
// Symbol-for-symbol what proj3/dnn_openblas.py:180-284 and proj3/dnn_cublas.py:183-295 bind.
#include "../../include/dnn_hip.h"
#include "legacy.h"

using namespace dnnhip;

extern "C" {

void conv2d_mul(float* in_layer, float* col, float* kernel_r, float* result, int batch, int oh, int ow, int od,
                int ih, int iw, int ic, int kh, int kw, int sh, int sw) {
  (void)col;  // scratch of the host im2col; the device im2col buffer replaces it
  legacy_begin();
  legacy_report("conv2d_mul",
                legacy_conv(in_layer, kernel_r, 1, result, batch, oh, ow, od, ih, iw, ic, kh, kw, sh, sw));
}

void conv2d_cublas(float* in_layer, float* col, float* kernel_r, float* result, int batch, int oh, int ow, int od,
                   int ih, int iw, int ic, int kh, int kw, int sh, int sw) {
  (void)col;
  legacy_begin();
  legacy_report("conv2d_cublas",
                legacy_conv(in_layer, kernel_r, 1, result, batch, oh, ow, od, ih, iw, ic, kh, kw, sh, sw));
}

void im2col(float* imb, float* colb, int oh, int ow, int ih, int iw, int ic, int kh, int kw, int sh, int sw) {
  legacy_begin();
  legacy_report("im2col", legacy_im2col(imb, colb, oh, ow, ih, iw, ic, kh, kw, sh, sw));
}

void bias_add(float* in_layer, float* biases, float* result, int batch, int h, int w, int c) {
  legacy_begin();
  legacy_report("bias_add", legacy_bias_add(in_layer, biases, result, batch, h, w, c));
}

void batch_norm(float* in_layer, float* mean, float* variance, float* gamma, float epsilon, float* result,
                int batch, int oh, int ow, int od) {
  legacy_begin();
  legacy_report("batch_norm", legacy_bn_mvg(in_layer, mean, variance, gamma, epsilon, result, batch, oh, ow, od));
}

void max_pool2d(float* in_layer, float* result, int batch, int oh, int ow, int od, int ih, int iw, int ic, int kh,
                int kw, int sh, int sw) {
  legacy_begin();
  legacy_report("max_pool2d",
                legacy_pool(in_layer, result, batch, oh, ow, od, ih, iw, ic, kh, kw, sh, sw, /*gt_below=*/0));
}

void leaky_relu(float* in_layer, float* result, int batch, int oh, int ow, int od) {
  legacy_begin();
  legacy_report("leaky_relu", legacy_leaky(in_layer, result, batch, oh, ow, od, /*f32_variant=*/0));
}

}  // extern "C"
