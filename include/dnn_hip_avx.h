/* dnn_hip_avx.h — libdnn_hip_avx.so: drop-in replacement for the proj3 AVX/pthread and
 * CUDA engines (ctypes.cdll.LoadLibrary('./libdnn_avx.so'), proj3/dnn_avx.py:10, and
 * './libdnn_cuda.so', proj3/dnn_cuda.py:10).  These two ABIs cannot share one .so with
 * dnn_hip.h because both define `batch_norm` and `leaky_relu` with other semantics.
 *
 * `args` is the int32[10] shape block {oh, ow, od, ih, iw, ic, kh, kw, sh, sw} the wrappers
 * pack (proj3/dnn_avx.py:174-179, 262-267).  Host pointers, synchronous, void, as in the
 * reference; errors via dnn_last_error() (dnn_hip_plan.h).  Correct batched semantics
 * (the reference's batch_norm has no batch offset, dnn_avx.c:501, and conv2d_pthread's
 * od%8 tail accumulates across runs, dnn_avx.c:63-68).
 */
#ifndef DNN_HIP_AVX_H
#define DNN_HIP_AVX_H
#include "dnn_hip_plan.h"

#ifdef __cplusplus
extern "C" {
#endif
#pragma GCC visibility push(default)

/* proj3/dnn_avx.c:79-126 (dnn_avx.py:202-207): direct conv, pre-padded input, HWIO kernel. */
void conv2d_pthread(float* in_layer, float* kernel, float* result, int batch, int* args);

/* proj3/dnn_cuda.cu:134-213 (dnn_cuda.py:215-221): im2col + GEMM, kernel_r K order (ic,kh,kw). */
void conv2d_cuda_pthread(float* in_layer, float* col, float* kernel_r, float* result, int batch, int* args);

/* proj3/dnn_avx.c:231-274 (dnn_avx.py:234-238, dnn_cuda.py:239-243): result = in + biases[c]. */
void bias_add_pthread(float* in_layer, float* biases, float* result, int batch, int oh, int ow, int od);

/* proj3/dnn_avx.c:374-420 (dnn_avx.py:285-288): max pool of a -FLT_MAX pre-padded input. */
void max_pool2d_pthread(float* in_layer, float* result, int batch, int* args);

/* proj3/dnn_cuda.cu:639 (dnn_cuda.py:271-277): same argument list as max_pool2d. */
void max_pool2d_avx(float* in_layer, float* result, int batch, int oh, int ow, int od, int ih, int iw, int ic,
                    int kh, int kw, int sh, int sw);

/* proj3/dnn_avx.c:483-518 (dnn_avx.py:312-317): result = in * alpha[c] - beta[c]
 * with alpha = gamma / sqrt(var + eps), beta = alpha * mean folded by the wrapper
 * (dnn_avx.py:301-303). */
void batch_norm(float* in_layer, float* alpha, float* beta, float* result, int batch, int oh, int ow, int od);

/* proj3/dnn_cuda.cu:724-755 (dnn_cuda.py:300-305): same contract as batch_norm above. */
void batch_norm_cuda(float* in_layer, float* alpha, float* beta, float* result, int batch, int oh, int ow,
                     int od);

/* proj3/dnn_avx.c:525-553 (dnn_avx.py:333-335): max(t, 0.1f * t).  dnn_cuda.py:318-320
 * binds the same name to dnn_cuda.cu:801-818, which rounds 0.1*t in double; the two
 * differ by at most 1 ulp on negative inputs (use libdnn_hip.so's leaky_relu for that form). */
void leaky_relu(float* in_layer, float* result, int batch, int oh, int ow, int od);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif
