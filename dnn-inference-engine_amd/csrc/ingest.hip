// Frame ingest on the GPU (include/dnn_hip_ingest.h): the reference's host preprocessing
// `resize_input` (cs492-projects/proj3/__init__.py:8-12)
//     imsz = cv2.resize(im, (416, 416))          # uint8 BGR, INTER_LINEAR
//     imsz = imsz / 255.                          # float64
//     imsz = imsz[:, :, ::-1]                     # BGR -> RGB
//     return np.asarray(imsz, dtype=np.float32)
// as one kernel over a batch of uint8 BGR frames already on the device.
//
// The resize restates OpenCV's scalar fixed-point INTER_LINEAR for 8-bit images
// (resize.cpp: HResizeLinear / VResizeLinear with INTER_RESIZE_COEF_BITS = 11):
//   fx = (dx + 0.5) * src_w / dst_w - 0.5, sx = floor(fx), fx -= sx; clamp at the borders
//   (sx < 0 -> sx = 0, fx = 0; sx >= src_w - 1 -> sx = src_w - 1, fx = 0); coefficients
//   a0 = round((1 - fx) * 2048), a1 = round(fx * 2048) (likewise b0, b1 in y);
//   out = (b0 * (a0*S[y0][x0] + a1*S[y0][x0+1]) + b1 * (a0*S[y1][x0] + a1*S[y1][x0+1]) + 2^21) >> 22.
// cv2 is not importable here, so parity with cv2.resize is UNPINNED (its SIMD paths may
// round differently); the /255, the channel flip and the fp32 rounding are exact, and an
// identity-size resize is exact.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include "dnn_common.h"
#include "../../include/dnn_hip_ingest.h"

namespace dnnhip {

struct Axis {
  int s0, s1;  // source indices
  int a0, a1;  // fixed-point weights (sum 2048)
};

__device__ __forceinline__ Axis axis_coef(int d, int src, int dst) {
  const double scale = (double)src / (double)dst;
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  if (s < 0) {
    s = 0;
    f = 0.f;
  }
  if (s >= src - 1) {
    s = src - 1;
    f = 0.f;
  }
  Axis a;
  a.s0 = s;
  a.s1 = s + 1 < src ? s + 1 : s;
  a.a0 = (int)rintf((1.f - f) * 2048.f);
  a.a1 = (int)rintf(f * 2048.f);
  return a;
}

// one thread per output pixel (3 channels)
__global__ void preprocess_kernel(const uint8_t* __restrict__ src, int n, int h, int w, float* __restrict__ dst,
                                  int oh, int ow) {
  const long long total = (long long)n * oh * ow;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ox = (int)(i % ow);
    const long long t = i / ow;
    const int oy = (int)(t % oh);
    const int b = (int)(t / oh);
    const uint8_t* img = src + (size_t)b * h * w * 3;
    int v[3];
    if (oh == h && ow == w) {  // identity: cv2.resize copies
      const uint8_t* p = img + ((size_t)oy * w + ox) * 3;
      v[0] = p[0];
      v[1] = p[1];
      v[2] = p[2];
    } else {
      const Axis ax = axis_coef(ox, w, ow), ay = axis_coef(oy, h, oh);
      const uint8_t* r0 = img + (size_t)ay.s0 * w * 3;
      const uint8_t* r1 = img + (size_t)ay.s1 * w * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int h0 = ax.a0 * r0[ax.s0 * 3 + c] + ax.a1 * r0[ax.s1 * 3 + c];
        const int h1 = ax.a0 * r1[ax.s0 * 3 + c] + ax.a1 * r1[ax.s1 * 3 + c];
        const int o = (ay.a0 * h0 + ay.a1 * h1 + (1 << 21)) >> 22;
        v[c] = o < 0 ? 0 : (o > 255 ? 255 : o);
      }
    }
    float* q = dst + i * 3;
    // imsz / 255. in float64, BGR -> RGB, then float32
    q[0] = (float)((double)v[2] / 255.0);
    q[1] = (float)((double)v[1] / 255.0);
    q[2] = (float)((double)v[0] / 255.0);
  }
}

}  // namespace dnnhip

extern "C" int dnn_preprocess_frames(const uint8_t* d_bgr, int n, int h, int w, float* d_out, int out_h, int out_w,
                                     void* stream) {
  DNN_REQUIRE(n >= 0 && h > 0 && w > 0 && out_h > 0 && out_w > 0, "dnn_preprocess_frames: bad shape");
  if (n == 0) return 0;
  DNN_REQUIRE(d_bgr && d_out, "dnn_preprocess_frames: NULL pointer");
  const long long total = (long long)n * out_h * out_w;
  long long blocks = (total + 255) / 256;
  if (blocks > 65535) blocks = 65535;
  hipLaunchKernelGGL(dnnhip::preprocess_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     static_cast<hipStream_t>(stream), d_bgr, n, h, w, d_out, out_h, out_w);
  DNN_HIP_TRY(hipGetLastError());
  return 0;
}
