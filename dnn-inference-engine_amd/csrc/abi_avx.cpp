// libdnn_hip_avx.so front-end: the AVX/pthread and CUDA engine ABI (include/dnn_hip_avx.h).
// Symbol-for-symbol what proj3/dnn_avx.py:202-335 and proj3/dnn_cuda.py:215-320 bind.
#include "../../include/dnn_hip_avx.h"
#include "legacy.h"

using namespace dnnhip;

namespace {
// int32[10] shape block {oh, ow, od, ih, iw, ic, kh, kw, sh, sw} (dnn_avx.c:15-20)
struct ShapeArgs {
  int oh, ow, od, ih, iw, ic, kh, kw, sh, sw;
};
}  // namespace

extern "C" {

void conv2d_pthread(float* in_layer, float* kernel, float* result, int batch, int* args) {
  legacy_begin();
  const ShapeArgs* a = reinterpret_cast<const ShapeArgs*>(args);
  legacy_report("conv2d_pthread", legacy_conv(in_layer, kernel, 0, result, batch, a->oh, a->ow, a->od, a->ih,
                                              a->iw, a->ic, a->kh, a->kw, a->sh, a->sw));
}

void conv2d_cuda_pthread(float* in_layer, float* col, float* kernel_r, float* result, int batch, int* args) {
  (void)col;
  legacy_begin();
  const ShapeArgs* a = reinterpret_cast<const ShapeArgs*>(args);
  legacy_report("conv2d_cuda_pthread", legacy_conv(in_layer, kernel_r, 1, result, batch, a->oh, a->ow, a->od, a->ih,
                                                   a->iw, a->ic, a->kh, a->kw, a->sh, a->sw));
}

void bias_add_pthread(float* in_layer, float* biases, float* result, int batch, int oh, int ow, int od) {
  legacy_begin();
  legacy_report("bias_add_pthread", legacy_bias_add(in_layer, biases, result, batch, oh, ow, od));
}

void max_pool2d_pthread(float* in_layer, float* result, int batch, int* args) {
  legacy_begin();
  const ShapeArgs* a = reinterpret_cast<const ShapeArgs*>(args);
  // 8-wide _mm256_max_ps for channels < od - od%8, scalar MAX for the tail (dnn_avx.c:374-420)
  legacy_report("max_pool2d_pthread", legacy_pool(in_layer, result, batch, a->oh, a->ow, a->od, a->ih, a->iw, a->ic,
                                                  a->kh, a->kw, a->sh, a->sw, a->od - a->od % 8));
}

void max_pool2d_avx(float* in_layer, float* result, int batch, int oh, int ow, int od, int ih, int iw, int ic,
                    int kh, int kw, int sh, int sw) {
  legacy_begin();
  legacy_report("max_pool2d_avx",
                legacy_pool(in_layer, result, batch, oh, ow, od, ih, iw, ic, kh, kw, sh, sw, od - od % 8));
}

void batch_norm(float* in_layer, float* alpha, float* beta, float* result, int batch, int oh, int ow, int od) {
  legacy_begin();
  legacy_report("batch_norm", legacy_bn_ab(in_layer, alpha, beta, result, batch, oh, ow, od));
}

void batch_norm_cuda(float* in_layer, float* alpha, float* beta, float* result, int batch, int oh, int ow,
                     int od) {
  legacy_begin();
  legacy_report("batch_norm_cuda", legacy_bn_ab(in_layer, alpha, beta, result, batch, oh, ow, od));
}

void leaky_relu(float* in_layer, float* result, int batch, int oh, int ow, int od) {
  legacy_begin();
  legacy_report("leaky_relu", legacy_leaky(in_layer, result, batch, oh, ow, od, /*f32_variant=*/1));
}

}  // extern "C"
