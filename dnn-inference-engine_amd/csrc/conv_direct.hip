// Direct 3x3 conv for a few input channels (YOLOv2-tiny conv0: 416x416x3 -> 16) with
// bias -> batch-norm -> leaky and the following 2x2/stride-2 max pool fused.
//
// For K = 27 and N = 16 the im2col + GEMM formulation (proj3/dnn_openblas.c:160-194) is
// pure HBM traffic: it writes and re-reads a 32-float col row per output pixel and then the
// 16-channel conv output before pooling it (≈1.5 ms at batch 64 on MI355X).  This kernel
// reads each input pixel once through an LDS patch, keeps the 4 conv outputs of a pool
// window in registers (64 fp32 FMA accumulators per thread, weights broadcast from SGPRs)
// and writes only the pooled tensor: 13 MB in + 2.8 MB out per image.
//
// Per output element the math is the reference's: conv (fp32, FMA accumulation in (kh,kw,c)
// order), then bias_add, batch_norm and leaky_relu in apply_epilogue's order and the window
// max (dnn_openblas.c:220-254) — evaluated as pool-then-epilogue (pool_then_epilogue in
// gemm_f32.h: equal values, one epilogue per pooled output), window cells past the conv output
// (odd sizes, SAME pool padding, -FLT_MAX in dnn_openblas.py:232-235) left out.
#include <hip/hip_runtime.h>
#include <cfloat>
#include "dnn_common.h"
#include "gemm_f32.h"

namespace dnnhip {

constexpr int DC_T = 16;  // pooled outputs per block edge (16 x 16 threads)

template <int CIN, int NOUT, typename OutT>
__global__ void __launch_bounds__(256)
conv3x3_pool2_direct_kernel(const float* __restrict__ in, const float* __restrict__ w, OutT* __restrict__ out,
                            DirectGeom g, EpiParams epi) {
  constexpr int PR = 2 * DC_T + 2, PC = 2 * DC_T + 2;  // input patch rows / cols
  constexpr int RS = PC * CIN + ((PC * CIN) % 2 == 0 ? 1 : 0);  // odd row stride: conflict-free reads
  __shared__ float patch[PR * RS];
  // weights staged in LDS and read as same-address (broadcast) ds_read_b128: held in SGPRs
  // instead, the 9*CIN*NOUT values overflow the SGPR file and spill through v_readlane
  __shared__ __attribute__((aligned(16))) float wl[9 * CIN * NOUT];
  for (int i = threadIdx.x; i < 9 * CIN * NOUT; i += 256) wl[i] = w[i];

  const int b = blockIdx.z, py0 = blockIdx.y * DC_T, px0 = blockIdx.x * DC_T;
  const int iy0 = 2 * py0 - g.pt, ix0 = 2 * px0 - g.pl;
  const float* inb = in + (size_t)b * g.H * g.W * CIN;
  for (int i = threadIdx.x; i < PR * PC * CIN; i += 256) {
    const int r = i / (PC * CIN), rem = i - r * (PC * CIN);
    const int col = rem / CIN, c = rem - col * CIN;
    const int iy = iy0 + r, ix = ix0 + col;
    float v = 0.f;
    if ((unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W) v = inb[((size_t)iy * g.W + ix) * CIN + c];
    patch[r * RS + rem] = v;
  }
  __syncthreads();

  const int tx = threadIdx.x & (DC_T - 1), ty = threadIdx.x / DC_T;
  const float* xp = patch + (2 * ty) * RS + (2 * tx) * CIN;  // this thread's 4x4xCIN input window

  float acc[4][NOUT];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int o = 0; o < NOUT; ++o) acc[p][o] = 0.f;
#pragma unroll 1  // bounds the live ranges: fully unrolled, hipcc parks operands in AGPRs
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int c = 0; c < CIN; ++c) {
        const float* wr = wl + ((ky * 3 + kx) * CIN + c) * NOUT;
        f32x4 wv[NOUT / 4];
#pragma unroll
        for (int o4 = 0; o4 < NOUT / 4; ++o4) wv[o4] = *reinterpret_cast<const f32x4*>(wr + 4 * o4);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const float xv = xp[((p >> 1) + ky) * RS + ((p & 1) + kx) * CIN + c];
#pragma unroll
          for (int o = 0; o < NOUT; ++o) acc[p][o] = __builtin_fmaf(xv, wv[o >> 2][o & 3], acc[p][o]);
        }
      }

  const int py = py0 + ty, px = px0 + tx;
  float pooled[NOUT];
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
    const float pb = (epi.flags & EPI_BIAS) ? epi.bias[o] : 0.f;
    const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[o] : 0.f;
    const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[o] : 1.f;
    const float pg = (epi.flags & EPI_BN) ? epi.gamma[o] : 1.f;
    // window cells past the conv output (SAME pool padding) repeat cell (0,0)
    const bool x1 = 2 * px + 1 < g.OW, y1 = 2 * py + 1 < g.OH;
    const f32x4 v = {acc[0][o], x1 ? acc[1][o] : acc[0][o], y1 ? acc[2][o] : acc[0][o],
                     x1 && y1 ? acc[3][o] : acc[0][o]};
    pooled[o] = pool_then_epilogue(v, pb, pm, ps, pg, epi.flags);
  }
  if (py < g.PH && px < g.PW) {
    OutT* dst = out + (((size_t)b * g.PH + py) * g.PW + px) * NOUT;
    if constexpr (sizeof(OutT) == 4) {
#pragma unroll
      for (int o = 0; o < NOUT; o += 4)
        *reinterpret_cast<float4*>(dst + o) = make_float4(pooled[o], pooled[o + 1], pooled[o + 2], pooled[o + 3]);
    } else {  // fp16 activations (fp16 path): 8 channels per 16-byte store
      typedef _Float16 h8 __attribute__((ext_vector_type(8)));
#pragma unroll
      for (int o = 0; o < NOUT; o += 8) {
        h8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (half_t)pooled[o + e];
        *reinterpret_cast<h8*>(dst + o) = v;
      }
    }
  }
}

bool direct_conv_pool_supported(int cin, int nout, int kh, int kw, int sh, int sw) {
  return kh == 3 && kw == 3 && sh == 1 && sw == 1 && cin >= 1 && cin <= 4 && nout == 16;
}

template <typename OutT>
static int launch_direct(const float* in, const float* w, OutT* out, const DirectGeom& g, int cin, int nout,
                         const EpiParams& epi, hipStream_t stream) {
  if (g.B == 0) return 0;
  if (nout != 16 || cin < 1 || cin > 4) {
    set_error("direct conv: unsupported cin=%d nout=%d", cin, nout);
    return -2;
  }
  dim3 grid((g.PW + DC_T - 1) / DC_T, (g.PH + DC_T - 1) / DC_T, g.B);
  switch (cin) {
    case 1:
      hipLaunchKernelGGL((conv3x3_pool2_direct_kernel<1, 16, OutT>), grid, dim3(256), 0, stream, in, w, out, g, epi);
      break;
    case 2:
      hipLaunchKernelGGL((conv3x3_pool2_direct_kernel<2, 16, OutT>), grid, dim3(256), 0, stream, in, w, out, g, epi);
      break;
    case 3:
      hipLaunchKernelGGL((conv3x3_pool2_direct_kernel<3, 16, OutT>), grid, dim3(256), 0, stream, in, w, out, g, epi);
      break;
    case 4:
      hipLaunchKernelGGL((conv3x3_pool2_direct_kernel<4, 16, OutT>), grid, dim3(256), 0, stream, in, w, out, g, epi);
      break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("launch conv3x3_pool2_direct: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int launch_conv3x3_pool2_direct(const float* in, const float* w, float* out, const DirectGeom& g, int cin, int nout,
                                const EpiParams& epi, hipStream_t stream) {
  return launch_direct<float>(in, w, out, g, cin, nout, epi, stream);
}

int launch_conv3x3_pool2_direct_f16out(const float* in, const float* w, half_t* out, const DirectGeom& g, int cin,
                                       int nout, const EpiParams& epi, hipStream_t stream) {
  return launch_direct<half_t>(in, w, out, g, cin, nout, epi, stream);
}

}  // namespace dnnhip
