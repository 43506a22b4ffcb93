/* dnn_hip.h — libdnn_hip.so: drop-in replacement for the proj3 OpenBLAS and cuBLAS engines.
 *
 * Exports exactly the symbols and argument lists that the reference's ctypes wrappers bind
 * (ctypes.cdll.LoadLibrary('./libdnn_openblas.so'), proj3/dnn_openblas.py:9, and
 * './libdnn_cublas.so', proj3/dnn_cublas.py:9).  All pointers are HOST pointers to NHWC
 * fp32 contiguous arrays owned by the caller; calls are synchronous (the result is valid
 * on return) and return void, as in the reference.  Internally every call copies its
 * inputs to a grow-only device arena, runs the gfx950 kernels and copies the result back.
 * A failure is reported through dnn_last_error() (declared in dnn_hip_plan.h) and on
 * stderr; the Python mirror (dnn_hip.py) turns it into an exception.
 *
 * Semantics are the reference's CORRECT ones: batched inputs are strided
 * by ih*iw*ic (the reference's conv2d_mul strides by oh*ow*od, dnn_openblas.c:170), and
 * batch_norm neither mutates `variance` (dnn_openblas.c:48-50) nor skips images >= 1
 * (dnn_openblas.c:56-58).
 */
#ifndef DNN_HIP_H
#define DNN_HIP_H
#include "dnn_hip_plan.h"

#ifdef __cplusplus
extern "C" {
#endif
#pragma GCC visibility push(default)

/* proj3/dnn_openblas.c:160-194 (called from dnn_openblas.py:180-188).
 * in_layer: pre-padded [B][ih][iw][ic]; col: caller scratch [B][oh*ow][ic*kh*kw] (not
 * touched: the device im2col replaces it); kernel_r: [ic*kh*kw][od] with K order
 * (ic, kh, kw) (dnn_openblas.py:166-167); result: [B][oh][ow][od], fully overwritten. */
void conv2d_mul(float* in_layer, float* col, float* kernel_r, float* result, int batch, int oh, int ow,
                int od, int ih, int iw, int ic, int kh, int kw, int sh, int sw);

/* proj3/dnn_cublas.cu:114-174 (called from dnn_cublas.py:183-191); same contract. */
void conv2d_cublas(float* in_layer, float* col, float* kernel_r, float* result, int batch, int oh, int ow,
                   int od, int ih, int iw, int ic, int kh, int kw, int sh, int sw);

/* proj3/dnn_openblas.c:135-158: im2col of ONE pre-padded image, K order (ic, kh, kw),
 * colb [oh*ow][ic*kh*kw]. */
void im2col(float* imb, float* colb, int oh, int ow, int ih, int iw, int ic, int kh, int kw, int sh, int sw);

/* proj3/dnn_openblas.c:9-38 (dnn_openblas.py:205-209, dnn_cublas.py:210-214):
 * result = in + biases[c]. */
void bias_add(float* in_layer, float* biases, float* result, int batch, int h, int w, int c);

/* proj3/dnn_openblas.c:40-65 (dnn_openblas.py:263-270, dnn_cublas.py:272-279):
 * result = ((in - mean) / sqrtf(var + eps)) * gamma.  `variance` is read only. */
void batch_norm(float* in_layer, float* mean, float* variance, float* gamma, float epsilon, float* result,
                int batch, int oh, int ow, int od);

/* proj3/dnn_openblas.c:196-234 (dnn_openblas.py:236-242): max over kh x kw windows at
 * stride (sh, sw) of a pre-padded input.  The wrapper's 4 trailing pad ints are ignored
 * by cdecl, as in the reference. */
void max_pool2d(float* in_layer, float* result, int batch, int oh, int ow, int od, int ih, int iw, int ic,
                int kh, int kw, int sh, int sw);

/* proj3/dnn_openblas.c:236-254 (dnn_openblas.py:282-284): t < 0 ? 0.1*t (double) : t. */
void leaky_relu(float* in_layer, float* result, int batch, int oh, int ow, int od);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif
