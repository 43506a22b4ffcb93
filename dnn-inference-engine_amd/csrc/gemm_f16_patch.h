// fp16 3x3 conv for the long-K, wide-N layers (conv6/conv7 of YOLOv2-tiny on the fp16 path,
// BASELINE config 5): the geometry and MFMA helper shared with the kernel (gemm_f16_acc.h).
// The input sits in HBM zero-padded ([B][H+2][W+2][C], borders written once at plan finalize),
// so output pixel m's tap (dy, dx) is padded row p(m) + (dy-1)(W+2) + (dx-1): a tile of BM
// consecutive output pixels reads one contiguous run of padded rows per 64-channel chunk, staged
// once and reused by all 9 taps.  (Rounds 2-3: conv3x3_f16_patch_kernel, register-staged
// XOR-swizzled 128-B rows, 16x16x32 or 32x32x16 (DNN_HIP_P16MF); replaced in round 4, git
// history.)
#pragma once
#include <type_traits>
#include "gemm_f16.h"

namespace dnnhip {

struct Patch16Geom {
  int H, W, C;      // conv input = output spatial size (3x3, stride 1, SAME), channels
  int out_padded;   // 1: write the output into a zero-bordered [B][H+2][W+2][N] buffer
};

// v_mfma_f32_16x16x32_f16: lane l supplies A[row l&15][k 8(l>>4)..+7] and B likewise;
// D[row][col]: col = l&15, row = 4(l>>4) + reg.  (The same FLOP per cycle as 32x32x16; on
// random data the chip holds a higher clock for it, MI355X_MICROARCH DVFS item 7.)
__device__ __forceinline__ f32x4 mfma16_f16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

}  // namespace dnnhip
