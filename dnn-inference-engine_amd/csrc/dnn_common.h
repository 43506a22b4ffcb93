// Shared declarations for the MI355X (gfx950) Conv2D hot path.
// Layout conventions: activations NHWC fp32 contiguous; conv weights
// HWIO; the GEMM sees A = im2col rows [M = B*OH*OW][Kpad] with K order (kh, kw, ic) and
// B = packed weights Bt[Npad][Kpad] (K contiguous), C = NHWC output [M][ldc].
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace dnnhip {

// ---------------------------------------------------------------- errors
void set_error(const char* fmt, ...);
const char* last_error();
// true when environment variable `name` is set and starts with '0' (experiment switches)
bool getenv_flag_off(const char* name);
// compute units of the current HIP device (persistent-kernel grids)
int device_cu_count();

#define DNN_HIP_TRY(x)                                                             \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      ::dnnhip::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #x,               \
                          hipGetErrorString(e_));                                  \
      return -1;                                                                   \
    }                                                                              \
  } while (0)

#define DNN_REQUIRE(cond, ...)                                                     \
  do {                                                                             \
    if (!(cond)) {                                                                 \
      ::dnnhip::set_error(__VA_ARGS__);                                            \
      return -2;                                                                   \
    }                                                                              \
  } while (0)

// ---------------------------------------------------------------- geometry
// TF SAME/VALID output size and front pad (proj3/dnn_openblas.py:127-142).
void out_pads(int in, int k, int s, int same, int* out, int* pad_front);

struct ConvGeom {
  int B, H, W, C;        // input (unpadded) NHWC
  int OH, OW;            // output spatial
  int kh, kw, sh, sw;    // window / stride
  int pt, pl;            // front pads (zero fill)
  int K, Kpad;           // K = kh*kw*C, Kpad = multiple of the GEMM's BK
};

struct PoolGeom {
  int B, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl;  // pads filled with -FLT_MAX
  // Channels c < gt_below use `m > x ? m : x` (_mm256_max_ps, dnn_avx.c:392-405); the rest
  // use the C macro `m >= x ? m : x` (dnn_openblas.c:8,220).  They differ only on +-0/NaN.
  int gt_below;
};

// Per-output-channel epilogue of a conv: conv -> bias_add -> batch_norm -> leaky_relu,
// evaluated in exactly the reference's operation order (proj3/dnn_openblas.c:9-65,236-254).
enum EpiFlags : int {
  EPI_BIAS = 1,
  EPI_BN = 2,          // ((v - mean) / sq) * gamma, sq = sqrtf(var + eps)
  EPI_LEAKY_F64 = 4,   // v < 0 ? (float)(0.1 * (double)v) : v   (dnn_openblas.c:250)
  EPI_LEAKY_F32 = 8,   // max(v, 0.1f * v)                       (dnn_avx.c:540-542)
  EPI_BN_AB = 16,      // v * alpha - beta                       (dnn_avx.c:505-507)
  EPI_OUT_X3 = 32,     // (pool-fused fp32 implicit GEMM) store the exact 3-way bf16 split of the
                       // result into the zero-bordered split planes of an x3 conv's input
};

struct EpiParams {
  const float* bias;   // [Npad]
  const float* mean;   // [Npad] (alpha for EPI_BN_AB)
  const float* sq;     // [Npad] (beta for EPI_BN_AB)
  const float* gamma;  // [Npad]
  int flags;
};

// GEMM tile configurations (see kernels.hip). Each has its own BM/BN/BK.  The MFMA shape
// (and so the per-element summation order) depends on N only: 16x16x4 for N <= 32,
// 32x32x2 above, with the same K permutation in every config of a family.
enum GemmCfg : int {
  GEMM_256x16_K32 = 0,   // N <= 16 (conv0), register-staged, MFMA 16x16x4
  GEMM_256x32_K16 = 1,   // N <= 32 (conv1), register-staged, MFMA 16x16x4
  GEMM_128x64_K32 = 2,   // N <= 64, register-staged, MFMA 32x32x2
  GEMM_128x128_K32 = 3,  // long-K wide layers (conv6/7): LDS-DMA 2-stage ring, MFMA 32x32x2
  GEMM_64x128_K32 = 4,   // other N >= 128 layers: LDS-DMA 2-stage ring, MFMA 32x32x2
  GEMM_G64x32_K32 = 5,   // N <= 32 implicit conv: LDS-DMA 2-stage ring, 64x32 tile, MFMA 16x16x4
  GEMM_G256x64_K32 = 6,  // N <= 64 implicit conv: LDS-DMA 2-stage ring, 256x64 tile, 8 waves, MFMA 32x32x2
  GEMM_G32x128_NS4 = 7,  // N >= 128, small M (batch 1): LDS-DMA 4-stage ring, 32x128 tile, MFMA 32x32x2
  GEMM_G32x64_NS4 = 8,   // N <= 64 implicit conv, small M: LDS-DMA 4-stage ring, 32x64 tile, 2 waves
  GEMM_128x256_W8 = 9,   // split-K layers, N % 256 == 0: 128x256, 8 waves of 64x64, one workgroup per CU
  GEMM_128x512_W16 = 10, // split-K layers, N % 512 == 0 (conv5-7): 128x512, 16 waves of 64x64, 160 KB LDS
  GEMM_64x128_NS3 = 11,  // experiment: 64x128 with a 3-stage ring
  GEMM_G256x128_W8 = 12, // experiment (N % 128 == 0): 256x128, 8 waves of 64x64, 96 KB (1 per CU)
  GEMM_G192x128_W8 = 13, // unsplit long-K N % 128 == 0 layers filling one round (conv4): 192x128, 8 waves of 96x32
  GEMM_G192x64_W4 = 14,  // latency plans, M <= 192 (one frame's 169 rows in one tile), N % 64 == 0: 4 waves of 96x32
  GEMM_NUM_CFGS = 15,
};
int gemm_cfg_bm(int cfg);
int gemm_cfg_bn(int cfg);
int gemm_cfg_bk(int cfg);
int choose_gemm_cfg(long long M, int N, int K);
int choose_gemm_cfg_implicit(long long M, int N, int K);

// Implicit-GEMM conv: the A operand is read straight from the NHWC input by per-lane
// LDS-DMA addresses (no im2col buffer).  Row m of the GEMM is an output pixel; with pool=1
// rows are pool-window-major (m = 4*window + 2*dy + dx of a 2x2/stride-2 window) and the
// epilogue max-pools the 4 rows, writing [B][PH][PW][N].  Needs C == 16 or C % 32 == 0.
struct ImplicitConv {
  const float* zero;  // >= 16 B of zeros in device memory (source of padding taps)
  int H, W, C;        // input
  int OH, OW;         // conv output
  int PH, PW;         // pooled output (pool = 1)
  int kh, kw, sh, sw, pt, pl;
  int pool;
  // round-up magic numbers of OW, OH, PW, PH for the kernels' division-free row decode
  // (div_magic, gemm_f32.h); the launchers fill them (implicit_conv_magic)
  unsigned mag_ow = 0, mag_oh = 0, mag_pw = 0, mag_ph = 0;
  int sh_ow = 0, sh_oh = 0, sh_pw = 0, sh_ph = 0;
};
bool implicit_conv_supported(int C, int kh, int kw);
void implicit_conv_magic(ImplicitConv* ic);
void magic_u32(int d, unsigned* mag, int* sh);  // n / d == (umulhi(n, mag) + n) >> sh, 0 <= n < 2^31
enum GemmMode : int { GEMM_DENSE = 0, GEMM_IMPLICIT = 1, GEMM_IMPLICIT_POOL = 2 };

// ---------------------------------------------------------------- launchers
// All launchers are asynchronous on `stream` and return 0 / negative on launch error.
int launch_im2col(const float* in, float* col, const ConvGeom& g, hipStream_t stream);
// K order (ic, kh, kw), K == Kpad, one image on a padded input (the per-op im2col ABI)
int launch_im2col_ckk(const float* in, float* col, const ConvGeom& g, hipStream_t stream);
// With splits > 1 (LDS-DMA configs only) the GEMM writes `splits` raw fp32 partials
// [splits][M][N] to `slab` and NO epilogue; launch_splitk_reduce then sums them in split order
// and applies the epilogue into C.  choose_splitk depends on (N, K) only.
int choose_splitk(int N, int K, bool combine = false);
// Latency plans (dnn_plan_set_latency_mode): tile config and split count of a small-M layer so
// that its work units fill the chip (depends on M: batch-1 results are not bit-equal to a
// batch plan's rows).  In: the batch rule's (cfg, splits); kept when they fill the chip.
void choose_latency_plan(long long M, int N, int K, int* cfg, int* splits, bool pool);
bool generic_combine_cfg(int cfg);
// tile order of a GEMM launch (SplitK::nmajor): 1 = N-major
int nmajor_order(int N, int tilesN);
// Persistent implicit GEMM for unsplit short-K layers (gemm_persist.h; DNN_HIP_PERSIST=0 off):
// same arguments and bits as launch_gemm_implicit with splits = 1; -3 = not covered (fall back).
int launch_gemm_persist(int cfg, int mode, const float* in, const ImplicitConv& ic, const float* Bt, int ldb,
                        float* C, int ldc, long long M, int N, int Kpad, const EpiParams& epi, hipStream_t stream);
// With `tickets` (>= the cfg's tile count of unsigned, zero before the first launch and left
// zero by every launch) the split-K GEMM finishes itself: the last-arriving split of each tile
// sums the partials in split order and writes C with the epilogue (splitk_combine, gemm_f32.h),
// so no reduce kernel follows; `slab` must then hold splitk_fused_slab_floats() floats.
int launch_gemm(int cfg, const float* A, int lda, const float* Bt, int ldb, float* C, int ldc,
                long long M, int N, int Kpad, const EpiParams& epi, hipStream_t stream, int splits = 1,
                float* slab = nullptr, unsigned* tickets = nullptr);
// implicit conv (mode GEMM_IMPLICIT / GEMM_IMPLICIT_POOL) on the LDS-DMA configs 3..6;
// `in` is the NHWC input, M = B*OH*OW (or B*PH*PW*4 with pool; no split-K with pool)
int launch_gemm_implicit(int cfg, int mode, const float* in, const ImplicitConv& ic, const float* Bt, int ldb,
                         float* C, int ldc, long long M, int N, int Kpad, const EpiParams& epi, hipStream_t stream,
                         int splits = 1, float* slab = nullptr, unsigned* tickets = nullptr);
// slab floats and tickets a fused split-K launch of (cfg, M, N, splits) needs
long long splitk_fused_slab_floats(int cfg, long long M, int N, int splits);
long long splitk_tiles(int cfg, long long M, int N);
int launch_splitk_reduce(const float* slab, int splits, long long M, int N, float* C, int ldc,
                         const EpiParams& epi, hipStream_t stream);
int launch_maxpool(const float* in, float* out, const PoolGeom& g, hipStream_t stream);
// order 0: rows of w are (kh, kw, ic)  [HWIO flattened];  order 1: rows are (ic, kh, kw)
// [proj3 kernel_r layout, dnn_openblas.py:166-167].  Output bt[Npad][Kpad] zero padded.
int launch_pack_weights(const float* w, float* bt, int K, int N, int Kpad, int Npad, int order,
                        int kh, int kw, int C, hipStream_t stream);
// Direct 3x3/stride-1 conv (cin <= 4, 16 outputs) + epilogue + fused 2x2/stride-2 max pool
// (conv_direct.hip).  w is HWIO [9*cin][16].
struct DirectGeom {
  int B, H, W;    // input (unpadded) NHWC, channels = cin
  int OH, OW;     // conv output
  int PH, PW;     // pooled output
  int pt, pl;     // conv front pads
};
bool direct_conv_pool_supported(int cin, int nout, int kh, int kw, int sh, int sw);
int launch_conv3x3_pool2_direct(const float* in, const float* w, float* out, const DirectGeom& g, int cin,
                                int nout, const EpiParams& epi, hipStream_t stream);

// Patch conv (conv_patch.hip): 3x3 / stride 1 / SAME, C in {16, 32}, OC % 32 == 0, even
// output, + epilogue + fused 2x2/stride-2 max pool on fp32 MFMA 16x16x4.  Bt is the packed
// [Npad][Kpad] weight block with Kpad == patch_conv_kpad(C); `zero` >= 16 B of zeros.
bool patch_conv_pool_supported(int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh, int sw, int pt,
                               int pl);
int patch_conv_kpad(int C);
// out_split != nullptr: the pooled outputs as x3 split planes of a zero-bordered
// [B][PH+2][PW+2] buffer (the next layer is an x3 conv); `out` unused
int launch_conv3x3_patch_pool(const float* in, const float* Bt, int ldb, float* out, const DirectGeom& g, int C,
                              int N, const float* zero, const EpiParams& epi, hipStream_t stream,
                              unsigned short* out_split = nullptr);

// ---------------------------------------------------------------- fp16 path (kernels_f16.hip)
// fp16 activations / weights, v_mfma_f32_32x32x16_f16 with fp32 accumulate and epilogue.
typedef _Float16 half_t;
enum Gemm16Cfg : int {
  GEMM16_128x128 = 0,     // long-K wide layers with split-K (conv5-7 at batch 64)
  GEMM16_64x128 = 1,      // other N >= 128
  GEMM16_32x128_NS4 = 2,  // N >= 128, small M: 4-stage ring
  GEMM16_128x64 = 3,      // N <= 64
  GEMM16_32x64_NS4 = 4,   // N <= 64, small M
  GEMM16_128x32 = 5,      // N <= 32
  GEMM16_32x32_NS4 = 6,   // N <= 32, small M
  GEMM16_256x128_W8 = 7,  // experiment: 8 waves of 64x64 (1 workgroup per CU)
  GEMM16_128x128_W4 = 8,  // experiment: 4 waves of 64x64
  GEMM16_128x256_W8 = 9,  // experiment: 8 waves of 64x64 (1 workgroup per CU)
  GEMM16_128x512_W16 = 10, // 16 waves of 64x64, 160 KB LDS: 40 staged B per 1k flop (L2->LDS bound)
  GEMM16_NUM_CFGS = 11,
};
int choose_gemm16_cfg(long long M, int N, int K);
int choose_splitk16(int N, int K);
int gemm16_cfg_bn(int cfg);
// mode: GEMM_DENSE (A = [M][lda] fp16), GEMM_IMPLICIT / GEMM_IMPLICIT_POOL (A = NHWC fp16 input
// described by ic; C % 8 == 0).  Kpad % 64 == 0; C is fp16 [M][ldc]; split-K partials in slab.
// `tickets`: in-GEMM split-K combine as for launch_gemm (slab: splitk16_fused_slab_floats).
bool gemm16_f32out_supported(int splits, int Npad);
int launch_gemm16_f32out(const half_t* A, int lda, const half_t* Bt, int ldb, int Npad, float* C, int ldc, long long M,
                         int N, int Kpad, const EpiParams& epi, hipStream_t stream);
int launch_gemm16(int cfg, int mode, const half_t* A, int lda, const ImplicitConv& ic, const half_t* Bt, int ldb,
                  half_t* C, int ldc, long long M, int N, int Kpad, const EpiParams& epi, hipStream_t stream,
                  int splits = 1, float* slab = nullptr, unsigned* tickets = nullptr);
long long splitk16_fused_slab_floats(int cfg, long long M, int N, int splits);
long long splitk16_tiles(int cfg, long long M, int N);
int launch_splitk_reduce16(const float* slab, int splits, long long M, int N, half_t* C, int ldc,
                           const EpiParams& epi, hipStream_t stream);
int launch_f32_to_f16(const float* in, half_t* out, long long n, hipStream_t s);
int launch_f16_to_f32(const half_t* in, float* out, long long n, hipStream_t s);
int launch_maxpool16(const half_t* in, half_t* out, const PoolGeom& g, hipStream_t s, int opad = 0);
// fp16 3x3/s1/SAME conv with a zero-bordered input [B][H+2][W+2][C] (C % 64 == 0, N % 256 == 0),
// weights packed K-order (chunk, tap, c) (launch_pack_weights order 2); out_padded: write the
// output zero-bordered too (gemm_f16_acc.h)
bool conv_patch16_supported(int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh, int sw, int pt,
                            int pl);
// fp32 path "x3" conv (kernels_x3.hip, gemm_x3_patch.h): fp32 operands split exactly into three
// bf16 pieces, six bf16 MFMA products, fp32 accumulation; activations in split planes
// [B][H+2][W+2][C/32][3][32] bf16 (zero-bordered), weights packed by launch_pack_weights_x3
// which x3 kernel family runs a layer (kernels_x3.hip x3_kind): 0 wide rows, 1 / 2 2-D tiles, 3 16-channel; -1 none
int conv_x3_kind(int OC, int C);
bool conv_x3_supported(int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl);
size_t x3_act_bytes(long long nimg, int H, int W, int C);
int launch_maxpool_x3(const float* in, unsigned short* out, const PoolGeom& g, hipStream_t s);
int launch_pack_weights_x3(const float* w, unsigned short* out, int K, int N, int Npad, int C, hipStream_t s);
int x3_splits(int N, int K);  // split-K of an x3 batch-plan layer: a function of (N, K) only
int launch_conv_x3(const unsigned short* in_split, const unsigned short* Bt, float* out, unsigned short* out_split,
                   long long M, int N, int Npad, int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream,
                   int splits = 1, int pool = 0, bool lat = false);  // lat: latency-plan tile shapes allowed
bool conv_x3_pool_supported(int OC, int C, int H, int W);  // an x3 conv of this size can fuse a 2x2/s2 pool
// x3 workgroups of a layer (batch-1 latency plans take x3 only where they fill half the chip)
long long x3_tiles(long long batch, int OH, int OW, int OC, int C, int K);
// small-M x3 conv of the latency plans (gemm_x3_lat.h): raw partials [splits][M][N] of
// x3_lat_splits(N, K) K slices into `part`, summed with the epilogue by launch_x3_combine
// latency plans' 1x1 head on x3 split planes, K split inside the workgroup (gemm_x3_ktile.h)
bool conv_x3_1x1_ktile_supported(int C, int OC, int H, int W);
int launch_conv_x3_1x1_ktile(const unsigned short* in_split, const unsigned short* Bt, float* out, long long M, int N,
                             int Npad, int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream);
// latency plans' mid layers: x3 with the K split inside the workgroup (gemm_x3_ktile.h), one
// launch, no partials; deterministic, tolerance against the batch plans
bool conv_x3_ktile_supported(long long batch, int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh,
                             int sw, int pt, int pl, int pool);  // pool: 0, 1 (2x2/s2), 2 (2x2/s1 SAME)
int launch_conv_x3_ktile(const unsigned short* in_split, const unsigned short* Bt, float* out,
                         unsigned short* out_split, long long M, int N, int Npad, int K, int H, int W, int C,
                         const EpiParams& epi, hipStream_t stream, int pool);
// batch plans' small-frame x3 conv with its 2x2/s1 SAME pool fused (gemm_x3_img.h: conv5 +
// pool5), one image x 128 columns per workgroup over the whole K, split planes out
bool conv_x3_img_supported(int C, int OC, int H, int W);
int launch_conv_x3_img(const unsigned short* in_split, const unsigned short* Bt, float* out, unsigned short* out_split,
                       int n, int N, int Npad, int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream);
bool conv_x3_lat_supported(long long batch, int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh,
                           int sw, int pt, int pl);
int x3_lat_splits(int N, int K);
// 1x1 x3 conv (gemm_x3_1x1.h: conv8) on the producer's zero-bordered split planes, fp32 out [M][N]
bool conv_x3_1x1_supported(int C, int OC, int H, int W);
int launch_conv_x3_1x1(const unsigned short* in_split, const unsigned short* Bt, float* out, long long M, int N,
                       int Npad, int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream);
int launch_conv_x3_lat(const unsigned short* in_split, const unsigned short* Bt, float* part, long long M, int N,
                       int Npad, int K, int H, int W, int C, int splits, hipStream_t stream);
int launch_x3_combine(const float* part, int splits, long long slab, const EpiParams& epi, const PoolGeom& g,
                      float* out, unsigned short* out_split, hipStream_t s);
int patch16_pack_order();  // launch_pack_weights order of the patch kernel's MFMA shape (3 or 4)
// fp16 3x3/s1/SAME conv + 2x2/s2 pool on 2-D tiles (gemm_f16_tile.h: conv2-conv4 of the fp16 path),
// zero-bordered input [B][H+2][W+2][C] (C % 32 == 0, N % 64 == 0, H, W even), weights packed
// by launch_pack_weights order 5; out_padded: the pooled output zero-bordered too
bool conv_tile16_supported(int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh, int sw, int pt,
                           int pl);
// pool: 1 = 2x2/s2 (2-D tiles), 2 = 2x2/s1 SAME (whole 13 x 13 frames, conv_img16_supported)
bool conv_img16_supported(int C, int OC, int H, int W);
int launch_conv_tile16(const half_t* in_padded, const half_t* Bt, int ldb, half_t* out, int out_padded, int n, int N,
                       int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream, int pool);
int launch_conv_patch16(const half_t* in_padded, const half_t* Bt, int ldb, half_t* out, int out_padded, long long M,
                        int N, int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream);
// conv0 direct kernel with an fp16 output (fp32 input frames)
int launch_conv3x3_pool2_direct_f16out(const float* in, const float* w, half_t* out, const DirectGeom& g, int cin,
                                       int nout, const EpiParams& epi, hipStream_t stream);

// conv_small.hip: conv0 on MFMA (cin <= 3, 16 outputs, fp32 frames in, pool fused) and the
// fp16 path's conv1 patch kernel (C = 16 -> 32, pool fused)
bool conv0_mfma_supported(int cin, int nout, int kh, int kw, int sh, int sw);
int launch_conv0_mfma(const float* in, const float* w, float* out, const DirectGeom& g, int cin, const float* zero,
                      const EpiParams& epi, hipStream_t s);
int launch_conv0_mfma_f16(const float* in, const float* w, half_t* out, const DirectGeom& g, int cin,
                          const EpiParams& epi, hipStream_t s);
// clock.hip: nwg one-wave workgroups each storing {s_memtime, s_memrealtime, XCC_ID, HW_ID}
int launch_clock_stamp(hipStream_t s, unsigned long long* out, int nwg);
bool conv1_patch_f16_supported(int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh, int sw, int pt,
                               int pl);
int launch_conv1_patch_f16(const half_t* in, const half_t* Bt, int ldb, half_t* out, const DirectGeom& g,
                           const float* zero, const EpiParams& epi, hipStream_t s, int opad = 0);

// element-wise ops of the per-op ABI
int launch_bias_add(const float* in, const float* b, float* out, long long n, int C, hipStream_t s);
int launch_bn_mvg(const float* in, const float* mean, const float* sq, const float* gamma, float* out,
                  long long n, int C, hipStream_t s);
int launch_bn_ab(const float* in, const float* alpha, const float* beta, float* out, long long n,
                 int C, hipStream_t s);
int launch_leaky(const float* in, float* out, long long n, int f32_variant, hipStream_t s);

}  // namespace dnnhip
