/* dnn_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement (plain C, gcc) of the
 * reference's proj3 C engines, used as the parity checker and as bench.py's CPU baseline.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product path (libdnn_hip*.so) never does.
 *
 * Pinned by: tests/golden/ fixtures generated from the reference's own numpy engine
 * (cs492-projects/proj3/dnn.py) by tests/golden/make_golden.py.  The reference's C files
 * (dnn_openblas.c, dnn_avx.c) include "cblas.h", which this image does not ship, so they
 * are unbuildable here; this file restates their algorithms with the
 * reference's CORRECT semantics (batch strides fixed, no in-place variance update, no
 * cross-run accumulation — SURVEY.md §8a lists the bugs).
 *
 * Each function cites the reference code it restates.
 */
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define CMAX(x, y) ((x) >= (y) ? (x) : (y)) /* dnn_openblas.c:8 */

/* proj3/dnn_openblas.c:135-158: col[i*ow+j][c*kh*kw + di*kw + dj] = im[i*sh+di][j*sw+dj][c] */
void oracle_im2col(const float* imb, float* colb, int oh, int ow, int ih, int iw, int ic, int kh, int kw, int sh,
                   int sw) {
  const int K = ic * kh * kw;
  (void)ih;
  for (int i = 0; i < oh; ++i)
    for (int j = 0; j < ow; ++j)
      for (int c = 0; c < ic; ++c)
        for (int k = 0; k < kh * kw; ++k)
          colb[(size_t)(i * ow + j) * K + c * kh * kw + k] =
              imb[((size_t)(i * sh + k / kw) * iw + (j * sw + k % kw)) * ic + c];
}

/* proj3/dnn_openblas.c:160-194 with the batch stride fixed to ih*iw*ic: per image im2col,
 * then C = col * kernel_r (RowMajor NN, beta = 0), fp32 accumulation in ascending k. */
void oracle_conv2d_mul(const float* in, const float* kernel_r, float* out, int batch, int oh, int ow, int od,
                       int ih, int iw, int ic, int kh, int kw, int sh, int sw) {
  const int K = ic * kh * kw, M = oh * ow;
  float* col = (float*)malloc((size_t)M * K * sizeof(float));
  for (int b = 0; b < batch; ++b) {
    const float* imb = in + (size_t)b * ih * iw * ic;
    float* ob = out + (size_t)b * M * od;
    oracle_im2col(imb, col, oh, ow, ih, iw, ic, kh, kw, sh, sw);
    for (int i = 0; i < M; ++i) {
      float* orow = ob + (size_t)i * od;
      for (int n = 0; n < od; ++n) orow[n] = 0.f;
      for (int k = 0; k < K; ++k) {
        const float a = col[(size_t)i * K + k];
        const float* wrow = kernel_r + (size_t)k * od;
        for (int n = 0; n < od; ++n) orow[n] += a * wrow[n];
      }
    }
  }
  free(col);
}

/* proj3/dnn_openblas.c:160-194 as the OpenBLAS engine runs it (BASELINE config 1): per image
 * single-thread im2col into a col buffer, then one cblas_sgemm(RowMajor, NoTrans, NoTrans,
 * M, od, K, 1, col, K, kernel_r, od, 0, out, od).  The sgemm is OpenBLAS itself, reached
 * through a function pointer the caller resolves in the OpenBLAS build numpy/scipy ship
 * (oracle_c.openblas_sgemm: scipy_cblas_sgemm, 32-bit ints); no cblas.h is needed. */
typedef void (*cblas_sgemm_fn)(int order, int ta, int tb, int m, int n, int k, float alpha, const float* a,
                               int lda, const float* b, int ldb, float beta, float* c, int ldc);

void oracle_conv2d_sgemm(const float* in, const float* kernel_r, float* out, int batch, int oh, int ow, int od,
                         int ih, int iw, int ic, int kh, int kw, int sh, int sw, void* sgemm) {
  const int K = ic * kh * kw, M = oh * ow;
  float* col = (float*)malloc((size_t)M * K * sizeof(float));
  for (int b = 0; b < batch; ++b) {
    oracle_im2col(in + (size_t)b * ih * iw * ic, col, oh, ow, ih, iw, ic, kh, kw, sh, sw);
    ((cblas_sgemm_fn)sgemm)(101 /* RowMajor */, 111 /* NoTrans */, 111, M, od, K, 1.0f, col, K, kernel_r, od, 0.0f,
                            out + (size_t)b * M * od, od);
  }
  free(col);
}

/* ---- AVX-engine-equivalent direct conv (proj3/dnn_avx.c:33-126): output rows split over
 * nthreads pthreads (P_THREADS = 4 in the reference, dnn_avx.c:13), accumulation order
 * (c, di, dj) per output pixel, vectorisable over od. */
struct direct_arg {
  const float* in;
  const float* k;
  float* out;
  const int* a; /* {oh, ow, od, ih, iw, ic, kh, kw, sh, sw} */
  int r0, r1;
};

static void* direct_rows(void* p) {
  struct direct_arg* d = (struct direct_arg*)p;
  const int* a = d->a;
  const int ow = a[1], od = a[2], iw = a[4], ic = a[5], kh = a[6], kw = a[7], sh = a[8], sw = a[9];
  float* acc = (float*)malloc((size_t)od * sizeof(float));
  for (int i = d->r0; i < d->r1; ++i)
    for (int j = 0; j < ow; ++j) {
      for (int n = 0; n < od; ++n) acc[n] = 0.f;
      for (int c = 0; c < ic; ++c)
        for (int di = 0; di < kh; ++di)
          for (int dj = 0; dj < kw; ++dj) {
            const float x = d->in[((size_t)(sh * i + di) * iw + (sw * j + dj)) * ic + c];
            const float* w = d->k + (((size_t)di * kw + dj) * ic + c) * od;
            for (int n = 0; n < od; ++n) acc[n] += x * w[n];
          }
      memcpy(d->out + ((size_t)i * ow + j) * od, acc, (size_t)od * sizeof(float));
    }
  free(acc);
  return NULL;
}

void oracle_conv2d_direct(const float* in, const float* kernel_hwio, float* out, int batch, const int* args,
                          int nthreads) {
  const int oh = args[0], ow = args[1], od = args[2], ih = args[3], iw = args[4], ic = args[5];
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  if (nthreads > oh) nthreads = oh;
  pthread_t th[256];
  struct direct_arg da[256];
  for (int b = 0; b < batch; ++b) {
    const int part = oh / nthreads;
    for (int t = 0; t < nthreads; ++t) {
      da[t].in = in + (size_t)b * ih * iw * ic;
      da[t].k = kernel_hwio;
      da[t].out = out + (size_t)b * oh * ow * od;
      da[t].a = args;
      da[t].r0 = part * t;
      da[t].r1 = t < nthreads - 1 ? part * (t + 1) : oh;
      pthread_create(&th[t], NULL, direct_rows, &da[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  }
}

/* proj3/dnn_openblas.c:9-38: result = in + biases[d] */
void oracle_bias_add(const float* in, const float* b, float* out, int batch, int h, int w, int c) {
  const size_t n = (size_t)batch * h * w * c;
  for (size_t i = 0; i < n; ++i) out[i] = in[i] + b[i % c];
}

/* proj3/dnn_openblas.c:40-65 without the in-place variance update and with the batch
 * offset: ((in - mean) / sqrtf(var + eps)) * gamma, every step in fp32. */
void oracle_batch_norm(const float* in, const float* mean, const float* var, const float* gamma, float eps,
                       float* out, int batch, int h, int w, int c) {
  float* sq = (float*)malloc((size_t)c * sizeof(float));
  for (int d = 0; d < c; ++d) {
    volatile float s = var[d] + eps;
    sq[d] = (float)sqrt((double)s);
  }
  const size_t n = (size_t)batch * h * w * c;
  for (size_t i = 0; i < n; ++i) {
    const int d = (int)(i % c);
    out[i] = ((in[i] - mean[d]) / sq[d]) * gamma[d];
  }
  free(sq);
}

/* proj3/dnn_avx.c:483-518 (batched): in * alpha - beta, two fp32 roundings */
void oracle_batch_norm_ab(const float* in, const float* alpha, const float* beta, float* out, int batch, int h,
                          int w, int c) {
  const size_t n = (size_t)batch * h * w * c;
  for (size_t i = 0; i < n; ++i) {
    const int d = (int)(i % c);
    volatile float r = in[i] * alpha[d];
    out[i] = r - beta[d];
  }
}

/* f32_variant 0: proj3/dnn_openblas.c:236-254  t < 0 ? 0.1 * t (double) : t
 * f32_variant 1: proj3/dnn_avx.c:525-553        max_ps(t, 0.1f * t) = t > s ? t : s */
void oracle_leaky_relu(const float* in, float* out, int batch, int h, int w, int c, int f32_variant) {
  const size_t n = (size_t)batch * h * w * c;
  for (size_t i = 0; i < n; ++i) {
    const float t = in[i];
    if (f32_variant) {
      volatile float s = t * 0.1f;
      out[i] = t > s ? t : s;
    } else {
      out[i] = t < 0 ? (float)(0.1 * (double)t) : t;
    }
  }
}

/* proj3/dnn_openblas.c:196-234 on an UNPADDED input with the wrapper's -FLT_MAX padding
 * (dnn_openblas.py:232-235) applied on the fly; pt/pl are the front pads.  Channels
 * c < gt_below compare with `>` (the AVX engine's _mm256_max_ps), the rest with CMAX. */
void oracle_max_pool2d(const float* in, float* out, int batch, int h, int w, int c, int oh, int ow, int kh, int kw,
                       int sh, int sw, int pt, int pl, int gt_below) {
  for (int b = 0; b < batch; ++b)
    for (int i = 0; i < oh; ++i)
      for (int j = 0; j < ow; ++j)
        for (int d = 0; d < c; ++d) {
          const int y0 = i * sh - pt, x0 = j * sw - pl;
#define PIX(y, x)                                                            \
  (((y) >= 0 && (y) < h && (x) >= 0 && (x) < w)                              \
       ? in[(((size_t)b * h + (y)) * w + (x)) * c + d]                       \
       : -FLT_MAX)
          float m = PIX(y0, x0);
          for (int di = 0; di < kh; ++di)
            for (int dj = 0; dj < kw; ++dj) {
              const float v = PIX(y0 + di, x0 + dj);
              m = d < gt_below ? (m > v ? m : v) : CMAX(m, v);
            }
#undef PIX
          out[(((size_t)b * oh + i) * ow + j) * c + d] = m;
        }
}
