// YOLOv2 postprocessing on the GPU (include/dnn_hip_post.h): the reference's host-side
// decode + threshold + sort + greedy NMS (cs492-projects/proj3/yolov2tiny.py:94-234) as one
// workgroup per image, so a batch leaves the GPU as a few kB of detections instead of
// 84.5 kB of raw predictions per image.
//
//   phase 1  thread per box (845): fp32 decode exactly as the reference evaluates it under
//            numpy (weak Python scalars: everything stays fp32; softmax sum in numpy's
//            8-accumulator pairwise order); every box's corners are truncated to int64
//            (non-finite / huge -> the image is flagged, as int() raises in the reference);
//            boxes above the threshold append a sort key to LDS
//   phase 2  bitonic sort of the keys (score descending, then box index = Python's stable
//            sort of the (row, col, anchor)-ordered list)
//   phase 3  greedy NMS as a bitmask: every wave fills rows of S[i][j] = IoU(i, j) > 0.3 for
//            j < i (64 pairs per wave step, ballot into one word), then one wave walks the
//            candidates in order with the keep mask in registers (lane w holds word w):
//            candidate i is dropped iff S[i] & keep != 0 — the reference's "IoU with ANY kept
//            box" (yolov2tiny.py:197-226).  IoU is the reference's integer formula (+1 widths,
//            negative overlaps not clamped) in exact 64/128-bit integers, converted to double
//            with correct rounding like Python's int -> float.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "dnn_common.h"
#include "../../include/dnn_hip_post.h"

namespace dnnhip {

constexpr int PP_THREADS = 512;
constexpr int PP_WAVES = PP_THREADS / 64;
constexpr int PP_WORDS = (DNN_YOLO_BOXES + 63) / 64;  // 14 keep / suppression words
constexpr int PP_SORT = 1024;  // >= DNN_YOLO_BOXES, power of two

__constant__ float kAnchorsF32[10] = {1.08f, 1.19f, 3.42f, 4.41f, 6.63f, 11.38f, 9.42f, 5.11f, 16.62f, 10.52f};

// numpy 2.x float32 exp (the AVX512F / AVX2 loop numpy dispatches to on x86, its
// loops_exponent_log "simd_exp_f32" algorithm restated): Cody-Waite reduction by
// rint(x * log2 e) (magic-number rounding), a 5th/2nd-order rational minimax, scale by 2^k.
// Matches np.exp bit for bit on all 2^32 float32 inputs (checked on x86 against numpy 2.2).
__device__ __forceinline__ float np_expf(float x) {
  if (x != x) return x;
  if (x >= 88.72283935546875f) return __builtin_inff();
  if (x <= -103.97208404541015625f) return 0.0f;
  const float magic = 12582912.0f;  // 0x1.8p+23
  float q = x * 1.442695040888963407359924681001892137f;
  q = (q + magic) - magic;
  float r = __builtin_fmaf(q, -6.93145752e-1f, x);
  r = __builtin_fmaf(q, -1.42860677e-6f, r);
  r = __builtin_fmaf(q, 0.0f, r);
  float num = __builtin_fmaf(5.082762527590693718096e-04f, r, 6.757896990527504603057e-03f);
  num = __builtin_fmaf(num, r, 5.114512081637298353406e-02f);
  num = __builtin_fmaf(num, r, 2.473615434895520810817e-01f);
  num = __builtin_fmaf(num, r, 7.257664613233124478488e-01f);
  num = __builtin_fmaf(num, r, 9.999999999980870924916e-01f);
  float den = __builtin_fmaf(2.159509375685829852307e-02f, r, -2.742335390411667452936e-01f);
  den = __builtin_fmaf(den, r, 1.0f);
  return ldexpf(num / den, (int)q);
}

// 1 / (1 + float32(e) ** -x)  (yolov2tiny.py:229-230 with numpy 2 fp32 scalar semantics: the
// power is libm powf).  e32 ** y is evaluated as exp2(y * log2(e32)) in double and rounded
// once: equal to glibc 2.35 powf(e32, y) on all but 0.004 % of float32 y (1 ulp apart there).
__device__ __forceinline__ float sigmoid_ref(float x) {
  const double log2_e32 = 0x1.715475968cddcp+0;  // log2((double)float32(np.e)) = 1.4426949970774023
  const float pw = (float)exp2((double)(-x) * log2_e32);
  return 1.0f / (1.0f + pw);
}

// numpy's float32 add.reduce of a contiguous 20-vector: 8 partial sums over the first 16,
// combined pairwise, then the 4 tail elements in order
__device__ __forceinline__ float pairwise_sum20(const float* e) {
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = e[j] + e[8 + j];
  float s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
  for (int j = 16; j < 20; ++j) s = s + e[j];
  return s;
}

// int(float32) with the reference's failure cases flagged: truncation toward zero
__device__ __forceinline__ bool trunc_i64(float v, long long* out) {
  const float lim = 2305843009213693952.0f;  // 2^61: keeps every +1 width / difference in int64
  if (!(v > -lim && v < lim)) return false;   // also NaN
  *out = (long long)v;                        // fp -> int conversion truncates
  return true;
}

__device__ __forceinline__ double u64_to_f64(unsigned long long x) {
  // both terms exact, one rounding of the exact sum = correctly rounded
  return (double)(unsigned)(x >> 32) * 4294967296.0 + (double)(unsigned)x;
}

// correctly rounded (nearest-even) |v| -> double for |v| < 2^127, as Python's int -> float
__device__ __forceinline__ double i128_to_f64(__int128 v) {
  const bool neg = v < 0;
  const unsigned __int128 u = neg ? (unsigned __int128)(-v) : (unsigned __int128)v;
  const unsigned long long hi = (unsigned long long)(u >> 64), lo = (unsigned long long)u;
  double d;
  if (hi == 0) {
    d = u64_to_f64(lo);
  } else {
    const int s = 64 - __clzll((long long)hi);  // 1..63
    unsigned long long top = (unsigned long long)(u >> s);
    top |= (lo & ((1ull << s) - 1)) != 0 ? 1ull : 0ull;  // sticky bit: round-to-odd below
    d = ldexp(u64_to_f64(top), s);
  }
  return neg ? -d : d;
}

// yolov2tiny.py:179-195: iou(a, b) > thr on integer corners [l, t, r, b].  A zero
// denominator (possible: overlaps are not clamped) raises ZeroDivisionError in the reference;
// it sets *zero_den here.
__device__ __forceinline__ bool iou_gt(const long long* a, const long long* b, double thr, bool* zero_den) {
  const long long xa = a[0] > b[0] ? a[0] : b[0], ya = a[1] > b[1] ? a[1] : b[1];
  const long long xb = a[2] < b[2] ? a[2] : b[2], yb = a[3] < b[3] ? a[3] : b[3];
  // fast path: every width below 2^25 -> every product and sum below 2^53, exact in int64 and
  // in double, so the double division is the reference's int / float(int) exactly
  const long long w0 = xb - xa + 1, h0 = yb - ya + 1, wa = a[2] - a[0] + 1, ha = a[3] - a[1] + 1,
                  wb = b[2] - b[0] + 1, hb = b[3] - b[1] + 1;
  const long long lim = 1ll << 25;
  if (w0 > -lim && w0 < lim && h0 > -lim && h0 < lim && wa > -lim && wa < lim && ha > -lim && ha < lim &&
      wb > -lim && wb < lim && hb > -lim && hb < lim) {
    const long long inter = w0 * h0, den = wa * ha + wb * hb - inter;
    if (den == 0) {
      *zero_den = true;
      return false;
    }
    return (double)inter / (double)den > thr;
  }
  const __int128 inter = (__int128)(xb - xa + 1) * (__int128)(yb - ya + 1);
  const __int128 area_a = (__int128)(a[2] - a[0] + 1) * (__int128)(a[3] - a[1] + 1);
  const __int128 area_b = (__int128)(b[2] - b[0] + 1) * (__int128)(b[3] - b[1] + 1);
  const __int128 den = area_a + area_b - inter;
  if (den == 0) {
    *zero_den = true;
    return false;
  }
  return i128_to_f64(inter) / i128_to_f64(den) > thr;
}

__global__ void __launch_bounds__(PP_THREADS)
yolo_postprocess_kernel(const float* __restrict__ pred, dnn_detection* __restrict__ dets, int max_det,
                        int* __restrict__ counts) {
  __shared__ unsigned long long keys[PP_SORT];
  __shared__ long long box[DNN_YOLO_BOXES][4];
  __shared__ float score_of[DNN_YOLO_BOXES];
  __shared__ int cls_of[DNN_YOLO_BOXES];
  __shared__ unsigned long long sup[DNN_YOLO_BOXES][PP_WORDS];  // S[i][w]: bits j = 64w.. < i
  __shared__ unsigned char zrow[DNN_YOLO_BOXES];               // row i has a zero IoU denominator
  __shared__ int n_cand, bad;

  const int img = blockIdx.x, tid = threadIdx.x;
  const float* p = pred + (size_t)img * DNN_YOLO_BOXES * 25;
  if (tid == 0) {
    n_cand = 0;
    bad = 0;
  }
  for (int i = tid; i < PP_SORT; i += PP_THREADS) keys[i] = ~0ull;
  __syncthreads();

  // ---- phase 1: decode (yolov2tiny.py:113-143)
  for (int k = tid; k < DNN_YOLO_BOXES; k += PP_THREADS) {
    const float* q = p + k * 25;
    const int b = k % 5, cell = k / 5, col = cell % 13, row = cell / 13;
    const float cx = ((float)col + sigmoid_ref(q[0])) * 32.0f;
    const float cy = ((float)row + sigmoid_ref(q[1])) * 32.0f;
    const float rw = (np_expf(q[2]) * kAnchorsF32[2 * b]) * 32.0f;
    const float rh = (np_expf(q[3]) * kAnchorsF32[2 * b + 1]) * 32.0f;
    const float conf = sigmoid_ref(q[4]);
    float m = q[5];
#pragma unroll
    for (int c = 1; c < 20; ++c) m = q[5 + c] > m ? q[5 + c] : m;
    float e[20];
#pragma unroll
    for (int c = 0; c < 20; ++c) e[c] = np_expf(q[5 + c] - m);
    const float s = pairwise_sum20(e);
    int best = 0;
    float bp = e[0] / s;
#pragma unroll
    for (int c = 1; c < 20; ++c) {
      const float pc = e[c] / s;
      if (pc > bp) {  // first index of the max
        bp = pc;
        best = c;
      }
    }
    const float hw = rw / 2.0f, hh = rh / 2.0f;
    long long l = 0, t = 0, r = 0, bt = 0;
    const bool ok = trunc_i64(cx - hw, &l) && trunc_i64(cx + hw, &r) && trunc_i64(cy - hh, &t) &&
                    trunc_i64(cy + hh, &bt);
    if (!ok) bad = 1;
    box[k][0] = l;
    box[k][1] = t;
    box[k][2] = r;
    box[k][3] = bt;
    const float sc = conf * bp;
    score_of[k] = sc;
    cls_of[k] = best;
    if (sc > 0.3f) {  // float32 comparison, as numpy compares a float32 with a Python float
      const int pos = atomicAdd(&n_cand, 1);
      // positive scores: larger float bits = larger score; ~bits sorts descending
      keys[pos] = ((unsigned long long)(~__float_as_uint(sc)) << 32) | (unsigned)k;
    }
  }
  __syncthreads();
  const int n = n_cand;
  if (bad) {
    if (tid == 0) counts[img] = -1;
    return;
  }

  // ---- phase 2: bitonic sort of the first pow2 >= n keys (yolov2tiny.py:146)
  int ns = 1;
  while (ns < n) ns <<= 1;
  for (int kk = 2; kk <= ns; kk <<= 1) {
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < ns; i += PP_THREADS) {
        const int ij = i ^ j;
        if (ij > i) {
          const unsigned long long a = keys[i], c = keys[ij];
          if (((i & kk) == 0) == (a > c)) {
            keys[i] = c;
            keys[ij] = a;
          }
        }
      }
      __syncthreads();
    }
  }

  // ---- phase 3a: suppression bitmask, all waves (yolov2tiny.py:197-216 evaluates every pair
  // (candidate i, kept j < i); here every pair j < i, the keep mask selects below)
  const int lane = tid & 63, wid = tid >> 6;
  for (int i = wid; i < n; i += PP_WAVES) {
    const int ki = (int)(keys[i] & 0xffffffffu);
    const long long bi[4] = {box[ki][0], box[ki][1], box[ki][2], box[ki][3]};
    bool zany = false;
    for (int w = 0; w * 64 < i; ++w) {
      const int j = w * 64 + lane;
      bool hit = false;
      if (j < i) hit = iou_gt(bi, box[(int)(keys[j] & 0xffffffffu)], 0.3, &zany);
      const unsigned long long m = __ballot(hit);
      if (lane == 0) sup[i][w] = m;
    }
    const bool z = __any(zany);
    if (lane == 0) zrow[i] = z ? 1 : 0;
  }
  __syncthreads();

  // ---- phase 3b: greedy walk in wave 0, keep word w in lane w
  if (tid < 64) {
    unsigned long long kw = 0;
    bool zero_hit = false;
    for (int i = 0; i < n; ++i) {
      const int nwi = (i + 63) >> 6;  // words holding j < i
      const unsigned long long row = lane < nwi ? sup[i][lane] : 0ull;
      const bool drop = __any((row & kw) != 0ull);
      if (zrow[i]) {  // rare: a zero IoU denominator against a KEPT box raises in the reference
        const int ki = (int)(keys[i] & 0xffffffffu);
        bool zd = false;
        for (unsigned long long bits = lane < nwi ? kw : 0ull; bits; bits &= bits - 1) {
          const int j = lane * 64 + __builtin_ctzll(bits);
          (void)iou_gt(box[ki], box[(int)(keys[j] & 0xffffffffu)], 0.3, &zd);
        }
        zero_hit |= zd;
      }
      if (!drop && lane == (i >> 6)) kw |= 1ull << (i & 63);
    }
    if (__any(zero_hit)) {
      if (lane == 0) counts[img] = -2;
      return;
    }
    // output in candidate order: exclusive prefix of the per-word popcounts
    const int cnt = __popcll(kw);
    int incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    const int nk = __shfl(incl, 63);
    int r = incl - cnt;
    for (unsigned long long bits = kw; bits; bits &= bits - 1, ++r) {
      const int i = lane * 64 + __builtin_ctzll(bits);
      if (r >= max_det) break;
      const int k = (int)(keys[i] & 0xffffffffu);
      dnn_detection d;
      d.cls = cls_of[k];
      d.score = score_of[k];
      d.left = box[k][0];
      d.top = box[k][1];
      d.right = box[k][2];
      d.bottom = box[k][3];
      dets[(size_t)img * max_det + r] = d;
    }
    if (lane == 0) counts[img] = nk;
  }
}

// Image-major compaction of the per-image detection lists: packed = concat_i dets[i][:counts[i]]
// (error images contribute nothing), total[0] = rows written.  One workgroup: a serial
// prefix over the counts in LDS chunks, then all threads copy rows.
__global__ void __launch_bounds__(PP_THREADS)
yolo_pack_kernel(const dnn_detection* __restrict__ dets, const int* __restrict__ counts, int n, int max_det,
                 dnn_detection* __restrict__ packed, int* __restrict__ total) {
  __shared__ int off[PP_THREADS + 1];
  int base = 0;
  for (int c0 = 0; c0 < n; c0 += PP_THREADS) {
    const int i = c0 + threadIdx.x;
    int c = i < n ? counts[i] : 0;
    c = c < 0 ? 0 : (c > max_det ? max_det : c);
    off[threadIdx.x + 1] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      off[0] = base;
      for (int k = 1; k <= PP_THREADS; ++k) off[k] += off[k - 1];
    }
    __syncthreads();
    const int lo = off[0], hi = off[PP_THREADS];
    // row r of this chunk's output belongs to the image whose [off[t], off[t+1]) holds it
    for (int r = lo + threadIdx.x; r < hi; r += PP_THREADS) {
      int t = 0, h = PP_THREADS;  // binary search: last t with off[t] <= r
      while (h - t > 1) {
        const int m = (t + h) >> 1;
        if (off[m] <= r) t = m; else h = m;
      }
      packed[r] = dets[(size_t)(c0 + t) * max_det + (r - off[t])];
    }
    base = hi;
    __syncthreads();
  }
  if (threadIdx.x == 0) total[0] = base;
}

int launch_yolo_pack(const dnn_detection* dets, const int* counts, int n, int max_det, dnn_detection* packed,
                     int* total, hipStream_t stream) {
  if (n < 0 || max_det < 0 || !total || (n > 0 && (!counts || (max_det > 0 && (!dets || !packed))))) {
    set_error("dnn_yolo_pack_detections: bad arguments (n=%d max_det=%d)", n, max_det);
    return -2;
  }
  hipLaunchKernelGGL(yolo_pack_kernel, dim3(1), dim3(PP_THREADS), 0, stream, dets, counts, n, max_det, packed,
                     total);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("launch yolo_pack: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int launch_yolo_postprocess(const float* pred, int n_images, dnn_detection* dets, int max_det, int* counts,
                            hipStream_t stream) {
  if (n_images == 0) return 0;
  if (n_images < 0 || max_det < 0 || !pred || !counts || (max_det > 0 && !dets)) {
    set_error("dnn_yolo_postprocess: bad arguments (n_images=%d max_det=%d)", n_images, max_det);
    return -2;
  }
  hipLaunchKernelGGL(yolo_postprocess_kernel, dim3(n_images), dim3(PP_THREADS), 0, stream, pred, dets, max_det,
                     counts);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("launch yolo_postprocess: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

}  // namespace dnnhip

extern "C" {

int dnn_yolo_postprocess(const float* pred, int n_images, dnn_detection* dets, int max_det, int* counts,
                         void* stream) {
  return dnnhip::launch_yolo_postprocess(pred, n_images, dets, max_det, counts, static_cast<hipStream_t>(stream));
}

int dnn_yolo_pack_detections(const dnn_detection* dets, const int* counts, int n_images, int max_det,
                             dnn_detection* packed, int* total, void* stream) {
  return dnnhip::launch_yolo_pack(dets, counts, n_images, max_det, packed, total, static_cast<hipStream_t>(stream));
}

int dnn_yolo_postprocess_host(const float* pred, int n_images, dnn_detection* dets, int max_det, int* counts) {
  DNN_REQUIRE(n_images >= 0 && max_det >= 0, "dnn_yolo_postprocess_host: bad arguments");
  if (n_images == 0) return 0;
  DNN_REQUIRE(pred && counts && (max_det == 0 || dets), "dnn_yolo_postprocess_host: NULL pointer");
  const size_t pb = (size_t)n_images * DNN_YOLO_BOXES * 25 * sizeof(float);
  const size_t db = (size_t)n_images * max_det * sizeof(dnn_detection), cb = (size_t)n_images * sizeof(int);
  char* buf = nullptr;
  DNN_HIP_TRY(hipMalloc(&buf, pb + db + cb));
  float* d_pred = reinterpret_cast<float*>(buf);
  dnn_detection* d_dets = reinterpret_cast<dnn_detection*>(buf + pb);
  int* d_counts = reinterpret_cast<int*>(buf + pb + db);
  int rc = 0;
  if (hipMemcpy(d_pred, pred, pb, hipMemcpyHostToDevice) != hipSuccess) {
    dnnhip::set_error("dnn_yolo_postprocess_host: copy in failed");
    rc = -1;
  }
  if (!rc) rc = dnnhip::launch_yolo_postprocess(d_pred, n_images, d_dets, max_det, d_counts, nullptr);
  if (!rc && (hipMemcpy(counts, d_counts, cb, hipMemcpyDeviceToHost) != hipSuccess ||
              (db && hipMemcpy(dets, d_dets, db, hipMemcpyDeviceToHost) != hipSuccess))) {
    dnnhip::set_error("dnn_yolo_postprocess_host: copy out failed");
    rc = -1;
  }
  (void)hipFree(buf);
  return rc;
}

}  // extern "C"
