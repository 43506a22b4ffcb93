// Hand-written gfx950 kernels for YOLOv2-tiny's Conv2D hot path.
//
//   im2col      NHWC -> col[M][Kpad], K order (kh, kw, ic) so HWIO weights are already
//               [K][N]; SAME padding by predication (no host np.pad). Reference semantics:
//               proj3/dnn_openblas.c:135-158 (there K order is (ic, kh, kw) on a pre-padded
//               input; the order is a private layout choice because weights are packed to match).
//   gemm        C[M][N] = A[M][K] * B[K][N] on fp32 MFMA (v_mfma_f32_32x32x2_f32 or
//               v_mfma_f32_16x16x4_f32), LDS double buffer, fused per-channel epilogue
//               bias -> batch-norm -> leaky in the reference's order. Replaces
//               cblas_sgemm(RowMajor,N,N,M,N,K,1,col,K,kernel_r,od,0,out,od)
//               (proj3/dnn_openblas.c:184-192) and the bias/bn/leaky passes.
//   maxpool     NHWC window max over a -FLT_MAX padded view (proj3/dnn_openblas.c:196-234,
//               padding from proj3/dnn_openblas.py:232-235).
//   element-wise bias_add / batch_norm / leaky_relu of the per-op ABI (dnn_openblas.c:9-65,
//               236-254; dnn_avx.c:483-553).
#include <hip/hip_runtime.h>
#include <cfloat>
#include "dnn_common.h"
#include "gemm_f32.h"
#include "gemm_persist.h"

namespace dnnhip {

static inline int ceil_div_i(long long a, long long b) { return (int)((a + b - 1) / b); }

static int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("launch %s: %s", what, hipGetErrorString(e));
    return -1;
  }
  return 0;
}

// ============================================================================ im2col
// 2-D grid: blockIdx.y = a chunk of <= IM2COL_KCH K columns, blockIdx.x = `rows` consecutive
// output pixels (rows of col), sized so one block moves ~16 KB.  Per-column tap offsets and
// per-row window origins are tabulated in LDS once per block, so the streaming loop does no
// integer division by layer constants.  Every thread stores float4s (coalesced row segments of
// the col matrix); when C % 4 == 0 a float4 is one vector load of 4 channels of one tap, else
// (conv0, C = 3) four scalar gathers.  Pure HBM stream: 4*(M*K) B written + the input read.
constexpr int IM2COL_THREADS = 256;
constexpr int IM2COL_KCH = 1024;      // K columns per block
constexpr int IM2COL_MAX_ROWS = 256;  // rows per block
constexpr int IM2COL_BLOCK_FLOATS = 8192;  // long-K layers (measured: 8 K floats per block beats 16 K-64 K)
constexpr int IM2COL_ILP = 4;

template <bool VEC>
__global__ void __launch_bounds__(IM2COL_THREADS)
im2col_nhwc_kernel(const float* __restrict__ in, float* __restrict__ col, ConvGeom g, long long M, int rows) {
  __shared__ int s_off[IM2COL_KCH];   // (dy*W + dx)*C + c relative to the window origin
  __shared__ int s_dydx[IM2COL_KCH];  // (dy << 16) | dx, or -1 for K padding columns
  __shared__ long long s_base[IM2COL_MAX_ROWS];
  __shared__ int s_iy[IM2COL_MAX_ROWS];
  __shared__ int s_ix[IM2COL_MAX_ROWS];

  const int k0 = blockIdx.y * IM2COL_KCH;
  const int kn = g.Kpad - k0 < IM2COL_KCH ? g.Kpad - k0 : IM2COL_KCH;  // multiple of 4
  const int kq = kn >> 2;
  const int nent = VEC ? kq : kn;  // table entries: per float4 (VEC) or per column
  for (int e = threadIdx.x; e < nent; e += IM2COL_THREADS) {
    const int k = k0 + (VEC ? 4 * e : e);
    if (k < g.K) {
      const int tap = k / g.C, c = k - tap * g.C;
      const int dy = tap / g.kw, dx = tap - dy * g.kw;
      s_off[e] = (dy * g.W + dx) * g.C + c;
      s_dydx[e] = (dy << 16) | dx;
    } else {
      s_off[e] = 0;
      s_dydx[e] = -1;
    }
  }
  const long long m0 = (long long)blockIdx.x * rows;
  for (int r = threadIdx.x; r < rows; r += IM2COL_THREADS) {
    long long m = m0 + r;
    if (m >= M) m = M - 1;
    const int ox = (int)(m % g.OW);
    const long long t = m / g.OW;
    const int oy = (int)(t % g.OH);
    const int b = (int)(t / g.OH);
    const int iy0 = oy * g.sh - g.pt, ix0 = ox * g.sw - g.pl;
    s_iy[r] = iy0;
    s_ix[r] = ix0;
    s_base[r] = (((long long)b * g.H + iy0) * g.W + ix0) * g.C;
  }
  __syncthreads();

  const int nrows = (int)((M - m0) < rows ? (M - m0) : rows);
  const int total = nrows * kq;
  // IM2COL_ILP independent gathers in flight per thread before their stores
  for (int base = threadIdx.x; base < total; base += IM2COL_ILP * IM2COL_THREADS) {
    float4 v[IM2COL_ILP];
    int dsto[IM2COL_ILP];
#pragma unroll
    for (int u = 0; u < IM2COL_ILP; ++u) {
      const int idx = base + u * IM2COL_THREADS;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      dsto[u] = -1;
      if (idx < total) {
        const int r = idx / kq;
        const int j = idx - r * kq;
        const int iy0 = s_iy[r], ix0 = s_ix[r];
        const float* src = in + s_base[r];
        dsto[u] = r * g.Kpad + 4 * j;
        if constexpr (VEC) {
          const int dd = s_dydx[j];
          const int iy = iy0 + (dd >> 16), ix = ix0 + (dd & 0xffff);
          if (dd >= 0 && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W)
            v[u] = *reinterpret_cast<const float4*>(src + s_off[j]);
        } else {
          float x[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int dd = s_dydx[4 * j + q];
            const int iy = iy0 + (dd >> 16), ix = ix0 + (dd & 0xffff);
            const bool ok = dd >= 0 && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
            x[q] = ok ? src[s_off[4 * j + q]] : 0.f;
          }
          v[u] = make_float4(x[0], x[1], x[2], x[3]);
        }
      }
    }
    float* dst = col + m0 * g.Kpad + k0;
#pragma unroll
    for (int u = 0; u < IM2COL_ILP; ++u)
      if (dsto[u] >= 0) *reinterpret_cast<float4*>(dst + dsto[u]) = v[u];
  }
}

// Row-staged im2col for C % 4 != 0 (conv0: C = 3): one block per output row (b, oy).  The kh
// input rows under it are read once, coalesced, into LDS (kh x ((OW-1)*sw + kw) x C floats,
// zeros for the padding; dynamic LDS sized to that), then the row's OW x Kpad col block is
// written as consecutive float4s (fully coalesced).  Kpad / 4 divides the 256 threads, so each
// thread keeps one float4 column j for the whole row: its 4 LDS source offsets are computed
// once, and a store costs 4 LDS reads.  Replaces four scalar HBM gathers (plus table lookups)
// per float4 (conv0: 3.0 TB/s).
__global__ void __launch_bounds__(256)
im2col_rows_kernel(const float* __restrict__ in, float* __restrict__ col, ConvGeom g) {
  extern __shared__ float s_in[];
  const int oy = blockIdx.x % g.OH, b = blockIdx.x / g.OH;
  const int npx = (g.OW - 1) * g.sw + g.kw;  // staged pixels per input row
  const int rowlen = npx * g.C;
  const int ix0 = -g.pl;
  for (int dy = 0; dy < g.kh; ++dy) {
    const int iy = oy * g.sh - g.pt + dy;
    const bool rok = (unsigned)iy < (unsigned)g.H;
    const float* src = in + (((long long)b * g.H + (rok ? iy : 0)) * g.W) * g.C;
    float* d = s_in + dy * rowlen;
    for (int px = threadIdx.x; px < npx; px += 256) {
      const int ix = ix0 + px;
      const bool ok = rok && (unsigned)ix < (unsigned)g.W;
      for (int c = 0; c < g.C; ++c) d[px * g.C + c] = ok ? src[ix * g.C + c] : 0.f;
    }
  }
  const int kq = g.Kpad >> 2;   // divides 256 (launcher)
  const int j = threadIdx.x % kq, ox0 = threadIdx.x / kq, oxs = 256 / kq;
  int t[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = 4 * j + q;
    t[q] = -1;
    if (k < g.K) {
      const int tap = k / g.C, c = k - tap * g.C;
      const int dy = tap / g.kw, dx = tap - dy * g.kw;
      t[q] = dy * rowlen + dx * g.C + c;
    }
  }
  __syncthreads();
  float* dst = col + ((long long)b * g.OH + oy) * g.OW * g.Kpad + 4 * j;
  const int xstep = g.sw * g.C;
  for (int ox = ox0; ox < g.OW; ox += oxs) {
    const int xo = ox * xstep;
    float x[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = t[q] >= 0 ? s_in[t[q] + xo] : 0.f;
    *reinterpret_cast<float4*>(dst + (size_t)ox * g.Kpad) = make_float4(x[0], x[1], x[2], x[3]);
  }
}

int launch_im2col(const float* in, float* col, const ConvGeom& g, hipStream_t stream) {
  long long M = (long long)g.B * g.OH * g.OW;
  if (M == 0) return 0;
  if (g.Kpad % 4 != 0 || g.Kpad < g.K) {
    set_error("im2col: Kpad=%d must be a multiple of 4 and >= K=%d", g.Kpad, g.K);
    return -2;
  }
  const bool vec = (g.C % 4) == 0;
  const long long row_floats = (long long)g.kh * ((g.OW - 1) * g.sw + g.kw) * g.C;
  if (!vec && g.Kpad <= 1024 && 256 % (g.Kpad / 4) == 0 && row_floats <= 16384 &&
      (long long)g.B * g.OH < 0x7fffffffLL && !getenv_flag_off("DNN_HIP_IM2COL_ROWS")) {
    hipLaunchKernelGGL(im2col_rows_kernel, dim3((unsigned)(g.B * g.OH)), dim3(256), (size_t)row_floats * 4, stream,
                       in, col, g);
    return check_launch("im2col_rows");
  }
  const int kch = g.Kpad < IM2COL_KCH ? g.Kpad : IM2COL_KCH;
  // floats moved per block: 4 K for K-chunks of <= 1024 columns' worth of short rows (conv1-3:
  // 5.4 -> 6.1 TB/s), 8 K for the long-K layers (conv4-7 lose with 4 K)
  const int blk_floats = g.Kpad < IM2COL_KCH ? 4096 : IM2COL_BLOCK_FLOATS;
  int rows = blk_floats / kch;
  rows = rows < 1 ? 1 : (rows > IM2COL_MAX_ROWS ? IM2COL_MAX_ROWS : rows);
  dim3 grid(ceil_div_i(M, rows), ceil_div_i(g.Kpad, IM2COL_KCH));
  if (vec)
    hipLaunchKernelGGL(im2col_nhwc_kernel<true>, grid, dim3(IM2COL_THREADS), 0, stream, in, col, g, M, rows);
  else
    hipLaunchKernelGGL(im2col_nhwc_kernel<false>, grid, dim3(IM2COL_THREADS), 0, stream, in, col, g, M, rows);
  return check_launch("im2col");
}

// The per-op ABI's im2col (proj3/dnn_openblas.c:135-158): K order (ic, kh, kw) on an
// already padded input, col[m][c*kh*kw + t] = in[oy*sh + t/kw][ox*sw + t%kw][c] for one image.
// Diagnostic entry point (the plan never materialises this layout): one thread per column
// element, consecutive threads write consecutive K columns of a row (coalesced stores).
__global__ void __launch_bounds__(256)
im2col_ckk_kernel(const float* __restrict__ in, float* __restrict__ col, ConvGeom g, long long total) {
  const int khw = g.kh * g.kw;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long m = e / g.K;
    const int k = (int)(e - m * g.K);
    const int c = k / khw, t = k - c * khw;
    const int dy = t / g.kw, dx = t - dy * g.kw;
    const int ox = (int)(m % g.OW), oy = (int)(m / g.OW);
    col[e] = in[((long long)(oy * g.sh + dy) * g.W + (ox * g.sw + dx)) * g.C + c];
  }
}

int launch_im2col_ckk(const float* in, float* col, const ConvGeom& g, hipStream_t stream) {
  const long long total = (long long)g.OH * g.OW * g.K;
  if (total == 0) return 0;
  const long long blocks = (total + 255) / 256;
  hipLaunchKernelGGL(im2col_ckk_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, stream, in,
                     col, g, total);
  return check_launch("im2col_ckk");
}

struct CfgInfo {
  int bm, bn, bk;
};
static const CfgInfo kCfgs[GEMM_NUM_CFGS] = {{256, 16, 32}, {256, 32, 16}, {128, 64, 32}, {128, 128, 32},
                                             {64, 128, 32},  {64, 32, 32},  {256, 64, 32}, {32, 128, 32},
                                             {32, 64, 32},   {128, 256, 32}, {128, 512, 32}, {64, 128, 32},
                                             {256, 128, 32}, {192, 128, 32}, {192, 64, 32}};

int gemm_cfg_bm(int cfg) { return kCfgs[cfg].bm; }
int gemm_cfg_bn(int cfg) { return kCfgs[cfg].bn; }
int gemm_cfg_bk(int cfg) { return kCfgs[cfg].bk; }

// Measured on MI355X at the batch-64 shapes (tools/gemm_bench.hip, tools/conv_bench.hip,
// profiles/r01_*): the LDS-DMA 128x128 two-stage ring wins the long-K layers (conv6/7:
// 110-118 TF), the 64x128 two-stage ring the other N >= 128 layers (conv3-5: 97 TF); two
// stages beat three (more workgroups per CU fit the LDS).  Every N >= 128 config
// uses 32x32x2 MFMAs with the same K permutation, so an output element's summation order does
// not depend on M: results are bit-identical across batch sizes.
int choose_gemm_cfg(long long M, int N, int K) {
  if (N <= 16) return GEMM_256x16_K32;
  if (N <= 32) return GEMM_256x32_K16;
  if (N <= 64) return GEMM_128x64_K32;
  // 128x128 tiles (2 per CU) when the long K split into choose_splitk(N, K) parts still gives
  // at least 512 work units; else 64x128 (3 per CU).  (K >= 1024: conv4 at batch 64 measured
  // 0.252 -> 0.240 ms with 128x128; conv3, K = 576, is faster on 64x128.)  Both are the 32x32x2 family with the same
  // K permutation, and the split itself depends on (N, K) only, so the summation order of an
  // output element never depends on M.
  long long t128 = ((M + 127) / 128) * ((N + 127) / 128);
  const int s = choose_splitk(N, K, false);
  if (K >= 1024 && t128 * s >= 512) {
    // split-K layers (conv5-7): one wide workgroup per CU with 16 / 8 waves of 64x64 stages
    // 80 / 96 B per MFMA instead of 128 (128x128): less LDS-DMA and L2 traffic per flop, which
    // keeps the power-limited clock up (batch 64: conv5 0.239 -> 0.216, conv6 0.855 -> 0.812,
    // conv7 1.632 -> 1.59 ms).  Same MFMA family and K order: results are unchanged bit for bit.
    if (s > 1 && N % 512 == 0) return GEMM_128x512_W16;
    if (s > 1 && N % 256 == 0) return GEMM_128x256_W8;
    // unsplit long-K layers (conv4: N = 256, K = 1152): with buffer-addressed DMA the 64x128
    // ring (3 per CU) beats 128x128 (2 per CU, 1.3 rounds at batch 64): 0.273 -> 0.224 ms
    if (s > 1) return GEMM_128x128_K32;
    // ... and 192x128 (8 waves of 96x32, 2 per CU) beats both when its tiles fill one round of
    // the 512 slots (conv4 at batch 64: 452 tiles instead of 1.76 rounds of 64x128, 26 instead
    // of 46 staged KB per MFLOP): 0.224 -> 0.215 ms.  (conv3, K = 576, measured slower on it.)
    const long long t192 = ((M + 191) / 192) * ((N + 127) / 128);
    if (N % 128 == 0 && t192 <= 512 && t192 * 5 >= 512 * 4) return GEMM_G192x128_W8;
  }
  // small M (batch 1 and the like): 64x128 would leave most CUs idle and each workgroup
  // waiting on a 2-stage ring; 32-row tiles with a 4-stage ring (same family, same K order)
  long long t64 = ((M + 63) / 64) * ((N + 127) / 128);
  if (t64 * s < 256) return GEMM_G32x128_NS4;
  return GEMM_64x128_K32;
}

// Implicit conv uses only LDS-DMA configs (the per-lane DMA source IS the im2col); same MFMA
// family per N as the dense choice above, so implicit and explicit results are bit-identical.
int choose_gemm_cfg_implicit(long long M, int N, int K) {
  if (N <= 16) return -1;
  if (N <= 32) return GEMM_G64x32_K32;
  if (N <= 64) return ((M + 255) / 256) < 256 ? GEMM_G32x64_NS4 : GEMM_G256x64_K32;
  return choose_gemm_cfg(M, N, K);
}

bool implicit_conv_supported(int C, int kh, int kw) {
  return (C == 16 || C % 32 == 0) && kh * kw <= 30;
}

// n / d == (umulhi(n, mag) + n) >> sh for 0 <= n < 2^31: the round-up method of Granlund and
// Montgomery with sh = ceil(log2 d), mag = floor(2^32 (2^sh - d) / d) + 1 (d = 1: mag 1, sh 0)
void magic_u32(int d, unsigned* mag, int* sh) {
  if (d <= 0) {
    *mag = 0;
    *sh = 0;
    return;
  }
  int l = 0;
  while ((1LL << l) < d) ++l;
  *mag = (unsigned)(((1ULL << 32) * ((1ULL << l) - (unsigned long long)d)) / (unsigned long long)d + 1);
  *sh = l;
}
void implicit_conv_magic(ImplicitConv* ic) {
  magic_u32(ic->OW, &ic->mag_ow, &ic->sh_ow);
  magic_u32(ic->OH, &ic->mag_oh, &ic->sh_oh);
  magic_u32(ic->PW, &ic->mag_pw, &ic->sh_pw);
  magic_u32(ic->PH, &ic->mag_ph, &ic->sh_ph);
}

// Split-K for the long-K wide layers: 680 128x128 tiles of conv6/7 at batch 64 fill 512
// two-per-CU slots 1.33 times; three K splits make it 3.98 (measured conv7 116 -> 127 TF
// including the reduce, tools/gemm_bench.hip, profiles/r01_gemm_bench_v2.txt); conv5's 340
// tiles become 1020 units (1.99 rounds).  Chosen from (N, K) only so every batch size sums in
// the same order.
int choose_splitk(int N, int K, bool combine) {
  if (N >= 512 && N % 4 == 0 && K >= 2048 && (K / 32) % 3 == 0) return 3;
  // (measured: splitting conv8 (N = 125, K = 1024) in two K halves with the in-GEMM combine
  // made it slower, 0.047 -> 0.050 ms at batch 64: the combine's acquire + partial round trip
  // costs more than the extra units gain.  `combine` keeps the option for shapes where it pays.)
  (void)combine;
  return 1;
}

// Latency plans.  When the batch rule's (cfg, splits) leaves the chip under 90 % occupied (256
// work units = one per CU), every candidate tile config -- the batch rule's and 32x64 for N <=
// 128 (192x64 when M <= 192 measured slower at batch 1: conv7 0.060 vs 0.051 ms) -- is tried
// with every split S <= 32 that divides its K-steps into parts of at least 6; the pick
// maximises the balance
// units / (256 * ceil(units / 256)), then prefers fewer splits (less partial traffic in the
// combine), then fewer units.  Batch 1 of YOLOv2-tiny: conv6/conv7 -> 32x128 x 16 splits (768
// units), conv5 -> x 9, conv4 -> x 4, conv3 -> x 3, conv8 -> 32x64 x 4 (tools/lat_cfg_sweep_job.sh:
// every tile/split choice of conv7 lands within 0.050-0.060 ms; the split-K combine's chain of
// memory round trips costs ~5 us per layer).
void choose_latency_plan(long long M, int N, int K, int* cfg, int* splits, bool pool) {
  if (*cfg < GEMM_128x128_K32) return;
  const long long target = 256;
  const int minsteps = 6;
  if (splitk_tiles(*cfg, M, N) * *splits * 10 >= target * 9) return;
  int cand[2] = {*cfg, N <= 128 ? GEMM_G32x64_NS4 : -1};
  double best_eff = -1.0;
  long long best_units = 0;
  int best_cfg = *cfg, best_s = *splits;
  for (int c : cand) {
    if (c < 0 || K % kCfgs[c].bk != 0) continue;
    const bool any_split = generic_combine_cfg(c);  // else only the batch combine's 2..3 splits
    const int nk = K / kCfgs[c].bk;
    const long long tiles = splitk_tiles(c, M, N);
    for (int sp = 1; sp <= 32; ++sp) {
      if (nk % sp != 0 || (sp > 1 && nk / sp < minsteps) || (!any_split && (sp > 3 || pool))) continue;
      const long long units = tiles * sp;
      const double eff = (double)units / (double)(target * ((units + target - 1) / target));
      if (eff > best_eff + 1e-9 ||
          (eff > best_eff - 1e-9 && (sp < best_s || (sp == best_s && units < best_units)))) {
        best_eff = eff;
        best_units = units;
        best_cfg = c;
        best_s = sp;
      }
    }
  }
  *cfg = best_cfg;
  *splits = best_s;
}

// LDS-DMA configs for one A mode (dense / implicit / implicit + pool); `abuf`: buffer-resource
// addressed DMA (BufDesc, gemm_f32.h), else flat 64-bit addresses
template <int MODE, bool ABUF>
static int launch_glds_t(int cfg, const float* A, int lda, const float* Bt, int ldb, float* C, int ldc, int m, int N,
                         int Kpad, const EpiParams& epi, int tilesN, const ImplicitConv& ic, const SplitK& sk,
                         const BufDesc& bd, dim3 grid, hipStream_t stream) {
  const bool gen = sk.steps > 0 && sk.tickets && (MODE == 2 || sk.splits > 3);
  if (gen) {  // latency plans: the any-split / pool-split combine (small-wave-tile configs only)
#define DNN_GLDS_GEN(BM_, BN_, WM_, WN_, MF_, NS_)                                                                   \
  hipLaunchKernelGGL((gemm_f32_glds_kernel<BM_, BN_, WM_, WN_, MF_, NS_, MODE, ABUF, true>), grid, dim3(WM_ * WN_ * 64), \
                     0, stream, A, lda, Bt, ldb, C, ldc, m, N, Kpad, epi, tilesN, ic, sk, bd)
    switch (cfg) {
      case GEMM_64x128_K32: DNN_GLDS_GEN(64, 128, 2, 2, 32, 2); break;
      case GEMM_G64x32_K32: DNN_GLDS_GEN(64, 32, 4, 1, 16, 2); break;
      case GEMM_G32x128_NS4: DNN_GLDS_GEN(32, 128, 1, 4, 32, 4); break;
      case GEMM_G32x64_NS4: DNN_GLDS_GEN(32, 64, 1, 2, 32, 4); break;
      case GEMM_64x128_NS3: DNN_GLDS_GEN(64, 128, 2, 2, 32, 3); break;
      default:
        set_error("gemm: cfg %d has no any-split combine", cfg);
        return -2;
    }
#undef DNN_GLDS_GEN
    return check_launch("gemm_glds_gen");
  }
#define DNN_GLDS(BM_, BN_, WM_, WN_, MF_, NS_)                                                                      \
  hipLaunchKernelGGL((gemm_f32_glds_kernel<BM_, BN_, WM_, WN_, MF_, NS_, MODE, ABUF>), grid, dim3(WM_ * WN_ * 64), 0, \
                     stream, A, lda, Bt, ldb, C, ldc, m, N, Kpad, epi, tilesN, ic, sk, bd)
  switch (cfg) {
    case GEMM_128x128_K32: DNN_GLDS(128, 128, 2, 2, 32, 2); break;
    case GEMM_64x128_K32: DNN_GLDS(64, 128, 2, 2, 32, 2); break;
    case GEMM_G64x32_K32: DNN_GLDS(64, 32, 4, 1, 16, 2); break;
    case GEMM_G256x64_K32: DNN_GLDS(256, 64, 4, 2, 32, 2); break;
    case GEMM_G32x128_NS4: DNN_GLDS(32, 128, 1, 4, 32, 4); break;
    case GEMM_G32x64_NS4: DNN_GLDS(32, 64, 1, 2, 32, 4); break;
    case GEMM_128x256_W8: DNN_GLDS(128, 256, 2, 4, 32, 2); break;
    case GEMM_128x512_W16: DNN_GLDS(128, 512, 2, 8, 32, 2); break;
    case GEMM_64x128_NS3: DNN_GLDS(64, 128, 2, 2, 32, 3); break;
    case GEMM_G256x128_W8: DNN_GLDS(256, 128, 4, 2, 32, 2); break;
    case GEMM_G192x128_W8: DNN_GLDS(192, 128, 2, 4, 32, 2); break;
    case GEMM_G192x64_W4: DNN_GLDS(192, 64, 2, 2, 32, 3); break;
    default:
      set_error("gemm: cfg %d is not an LDS-DMA config", cfg);
      return -2;
  }
#undef DNN_GLDS
  return check_launch("gemm_glds");
}

long long splitk_tiles(int cfg, long long M, int N) {
  return ((M + kCfgs[cfg].bm - 1) / kCfgs[cfg].bm) * ((N + kCfgs[cfg].bn - 1) / kCfgs[cfg].bn);
}
long long splitk_fused_slab_floats(int cfg, long long M, int N, int splits) {
  return splitk_tiles(cfg, M, N) * kCfgs[cfg].bm * kCfgs[cfg].bn * splits;
}

template <int MODE>
static int launch_glds(int cfg, const float* A, int lda, const float* Bt, int ldb, float* C, int ldc, int m, int N,
                       int Kpad, const EpiParams& epi, int tilesN, const ImplicitConv& ic, const SplitK& sk,
                       const BufDesc* bd, dim3 grid, hipStream_t stream) {
  if (bd)
    return launch_glds_t<MODE, true>(cfg, A, lda, Bt, ldb, C, ldc, m, N, Kpad, epi, tilesN, ic, sk, *bd, grid, stream);
  return launch_glds_t<MODE, false>(cfg, A, lda, Bt, ldb, C, ldc, m, N, Kpad, epi, tilesN, ic, sk, BufDesc{}, grid,
                                    stream);
}

// buffer descriptors fit (offsets are 32-bit, OOB_OFF = 2^31 marks padding taps)?
static bool fits_buf(long long bytes) { return bytes > 0 && bytes < 0x80000000LL; }
// DNN_HIP_GEMM_BUF=0: flat 64-bit DMA addresses (experiments and the equivalence tests)
static bool abuf_enabled() { return !getenv_flag_off("DNN_HIP_GEMM_BUF"); }

// N-major tile order (round 1 experiment, measured without gain): off
int nmajor_order(int N, int tilesN) {
  (void)N;
  (void)tilesN;
  return 0;
}

// configs whose waves hold <= 32 accumulator registers: the only ones with the any-split /
// pool-split combine compiled in (gemm_f32_glds_kernel)
bool generic_combine_cfg(int cfg) {
  return cfg == GEMM_G32x128_NS4 || cfg == GEMM_G32x64_NS4 || cfg == GEMM_64x128_K32 || cfg == GEMM_G64x32_K32 ||
         cfg == GEMM_64x128_NS3;
}

// grid and SplitK descriptor for `splits` (> 1: the kernel writes raw partials to `slab`;
// with `tickets` it also combines them itself into C)
static int split_setup(int cfg, long long M, int N, int Kpad, int splits, float* slab, unsigned* tickets, float* C,
                       int ldc, int flags, SplitK* sk, int* grid, int* tilesN) {
  const CfgInfo ci = kCfgs[cfg];
  const int tilesM = ceil_div_i(M, ci.bm);
  *tilesN = ceil_div_i(N, ci.bn);
  *grid = tilesM * *tilesN;
  *sk = SplitK{0, *grid, 0};
  if (splits > 1) {
    if (cfg < GEMM_128x128_K32 || !slab || (Kpad / 32) % splits != 0 || (!tickets && N % 4 != 0)) {
      set_error("gemm: split-K %d unsupported for cfg %d Kpad %d N %d", splits, cfg, Kpad, N);
      return -2;
    }
    *sk = SplitK{Kpad / 32 / splits, *grid, M * (long long)N};
    if (tickets && splits > 3 && !generic_combine_cfg(cfg)) {
      set_error("gemm: %d-way split combine needs a small-wave-tile config (cfg %d)", splits, cfg);
      return -2;
    }
    if (tickets) {
      if (splits > 32) {
        set_error("gemm: fused split-K combine supports 2..32 splits (got %d)", splits);
        return -2;
      }
      if (splitk_fused_slab_floats(cfg, M, N, splits) * 4 >= 0x80000000LL) {
        set_error("gemm: fused split-K slab over 2 GiB (M=%lld N=%d)", M, N);
        return -2;
      }
      sk->tickets = tickets;
      sk->out = C;
      sk->ldo = ldc;
      sk->flags = flags;
      sk->splits = splits;
    }
    *grid *= splits;
  }
  sk->nmajor = nmajor_order(N, *tilesN);
  return 0;
}

int launch_gemm(int cfg, const float* A, int lda, const float* Bt, int ldb, float* C, int ldc,
                long long M, int N, int Kpad, const EpiParams& epi, hipStream_t stream, int splits, float* slab,
                unsigned* tickets) {
  if (M == 0 || N == 0) return 0;
  if (cfg < 0 || cfg >= GEMM_NUM_CFGS) {
    set_error("gemm: bad cfg %d", cfg);
    return -2;
  }
  const CfgInfo ci = kCfgs[cfg];
  if (Kpad % ci.bk != 0 || lda % 4 != 0 || ldb % 4 != 0 || M > 0x7fffffffLL) {
    set_error("gemm: unsupported shape M=%lld Kpad=%d lda=%d ldb=%d for cfg %d", M, Kpad, lda, ldb, cfg);
    return -2;
  }
  SplitK sk;
  int g = 0, tilesN = 0;
  if (int rc = split_setup(cfg, M, N, Kpad, splits, slab, tickets, C, ldc, epi.flags, &sk, &g, &tilesN)) return rc;
  dim3 grid(g);
  const int m = (int)M;
  switch (cfg) {
    case GEMM_256x16_K32:
      hipLaunchKernelGGL((gemm_f32_mfma_kernel<256, 16, 32, 4, 1, 16>), grid, dim3(256), 0, stream, A, lda,
                         Bt, ldb, C, ldc, m, N, Kpad, epi, tilesN);
      break;
    case GEMM_256x32_K16:
      hipLaunchKernelGGL((gemm_f32_mfma_kernel<256, 32, 16, 4, 1, 16>), grid, dim3(256), 0, stream, A, lda,
                         Bt, ldb, C, ldc, m, N, Kpad, epi, tilesN);
      break;
    case GEMM_128x64_K32:
      hipLaunchKernelGGL((gemm_f32_mfma_kernel<128, 64, 32, 2, 2, 32>), grid, dim3(256), 0, stream, A, lda,
                         Bt, ldb, C, ldc, m, N, Kpad, epi, tilesN);
      break;
    default: {
      const long long a_bytes = (M * (long long)lda) * 4, b_bytes = (long long)tilesN * ci.bn * ldb * 4;
      BufDesc bd{A, (unsigned)a_bytes, (unsigned)b_bytes};
      const bool abuf = abuf_enabled() && fits_buf(a_bytes) && fits_buf(b_bytes);
      return launch_glds<GEMM_DENSE>(cfg, A, lda, Bt, ldb, sk.steps ? slab : C, sk.steps ? N : ldc, m, N, Kpad,
                                     epi, tilesN, ImplicitConv{}, sk, abuf ? &bd : nullptr, grid, stream);
    }
  }
  return check_launch("gemm");
}

int launch_gemm_implicit(int cfg, int mode, const float* in, const ImplicitConv& ic_in, const float* Bt, int ldb,
                         float* C, int ldc, long long M, int N, int Kpad, const EpiParams& epi, hipStream_t stream,
                         int splits, float* slab, unsigned* tickets) {
  if (M == 0 || N == 0) return 0;
  ImplicitConv ic = ic_in;
  implicit_conv_magic(&ic);
  if (cfg < GEMM_128x128_K32 || cfg >= GEMM_NUM_CFGS || (mode != GEMM_IMPLICIT && mode != GEMM_IMPLICIT_POOL)) {
    set_error("gemm_implicit: bad cfg %d / mode %d", cfg, mode);
    return -2;
  }
  const CfgInfo ci = kCfgs[cfg];
  if (Kpad % ci.bk != 0 || !implicit_conv_supported(ic.C, ic.kh, ic.kw) || M > 0x7fffffffLL || !ic.zero ||
      (mode == GEMM_IMPLICIT_POOL && (M % 4 != 0 || (splits > 1 && (!tickets || !generic_combine_cfg(cfg)))))) {
    set_error("gemm_implicit: unsupported shape M=%lld C=%d Kpad=%d splits=%d", M, ic.C, Kpad, splits);
    return -2;
  }
  SplitK sk;
  int g = 0, tilesN = 0;
  if (int rc = split_setup(cfg, M, N, Kpad, splits, slab, tickets, C, ldc, epi.flags, &sk, &g, &tilesN)) return rc;
  float* out = sk.steps ? slab : C;
  const int ldo = sk.steps ? N : ldc;
  // buffer-addressed DMA when each K-step is one tap (C % 32 == 0) and the descriptors fit
  const long long per_img = mode == GEMM_IMPLICIT_POOL ? 4LL * ic.PH * ic.PW : (long long)ic.OH * ic.OW;
  const long long nimg = per_img > 0 ? M / per_img : 0;
  const long long a_bytes = ((nimg * ic.H * ic.W + ic.W + 1) * (long long)ic.C) * 4;
  const long long b_bytes = (long long)tilesN * ci.bn * ldb * 4;
  BufDesc bd{in - (size_t)(ic.W + 1) * ic.C, (unsigned)a_bytes, (unsigned)b_bytes};
  const BufDesc* pbd =
      (abuf_enabled() && ic.C % 32 == 0 && fits_buf(a_bytes) && fits_buf(b_bytes)) ? &bd : nullptr;
  if (mode == GEMM_IMPLICIT)
    return launch_glds<GEMM_IMPLICIT>(cfg, in, 0, Bt, ldb, out, ldo, (int)M, N, Kpad, epi, tilesN, ic, sk, pbd,
                                      dim3(g), stream);
  return launch_glds<GEMM_IMPLICIT_POOL>(cfg, in, 0, Bt, ldb, out, ldo, (int)M, N, Kpad, epi, tilesN, ic, sk, pbd,
                                         dim3(g), stream);
}

// ---- persistent short-K implicit GEMM (gemm_persist.h)
static int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cus[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) v = 0;
    cus[dev] = v;
  }
  return cus[dev];
}

template <int BM, int BN, int WM, int WN, int MF, int NS, int MODE, int NTN>
static int launch_persist_t(const float* Bt, int ldb, float* C, int ldc, int M, int N, int Kpad,
                            const EpiParams& epi, int tilesN, int ntiles, const ImplicitConv& ic, const BufDesc& bd,
                            unsigned out_bytes, hipStream_t stream) {
  auto kern = gemm_f32_persist_kernel<BM, BN, WM, WN, MF, NS, MODE, NTN>;
  static int per_cu = -1;  // resident workgroups per CU (LDS, registers, waves)
  if (per_cu < 0) {
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, kern, WM * WN * 64, 0) != hipSuccess) v = 0;
    per_cu = v;
  }
  const int wgs = per_cu;
  long long grid = (long long)device_cus() * wgs;
  // fewer than two tiles per workgroup: the tail of the ones holding two costs more than the
  // pipelining gains (conv4 at batch 64: 452 tiles on 448 slots, 0.224 -> 0.317 ms)
  if (ntiles < 2 * grid || Kpad / 32 < NS) return -3;
  grid -= grid % 8;
  if (grid < 8) return -3;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(WM * WN * 64), 0, stream, Bt, ldb, C, ldc, M, N, Kpad, epi,
                     tilesN, ntiles, ic, bd, out_bytes);
  return check_launch("gemm_persist");
}

// DNN_HIP_PERSIST: 0 off, 1 (default) on the configs where it measured faster (256x64: conv2
// 0.236 -> 0.228 ms; on 64x128 the static tile split lost to the hardware's dynamic one, conv3
// 0.214 -> 0.224), 2 on every covered config (tests, experiments)
static int persist_level() {
  const char* e = getenv("DNN_HIP_PERSIST");
  return e ? atoi(e) : 1;
}
bool persist_enabled() { return persist_level() > 0; }

// Persistent launch of an unsplit implicit conv on the batch configs conv2-conv4 use;
// returns -3 (caller falls back to launch_gemm_implicit) when the shape or config is not one
// it covers.
int launch_gemm_persist(int cfg, int mode, const float* in, const ImplicitConv& ic_in, const float* Bt, int ldb,
                        float* C, int ldc, long long M, int N, int Kpad, const EpiParams& epi, hipStream_t stream) {
  if (M == 0 || N == 0) return 0;
  if (!persist_enabled() || (mode != GEMM_IMPLICIT && mode != GEMM_IMPLICIT_POOL) || ic_in.C % 32 != 0 ||
      M > 0x7fffffffLL || Kpad % 32 != 0 || !implicit_conv_supported(ic_in.C, ic_in.kh, ic_in.kw) ||
      (mode == GEMM_IMPLICIT_POOL && M % 4 != 0) || (epi.flags & EPI_OUT_X3))  // (split-plane output: tile kernel)
    return -3;
  ImplicitConv ic = ic_in;
  implicit_conv_magic(&ic);
  const CfgInfo ci = kCfgs[cfg];
  const int tilesM = ceil_div_i(M, ci.bm), tilesN = ceil_div_i(N, ci.bn);
  const long long ntiles = (long long)tilesM * tilesN;
  const long long per_img = mode == GEMM_IMPLICIT_POOL ? 4LL * ic.PH * ic.PW : (long long)ic.OH * ic.OW;
  const long long nimg = per_img > 0 ? M / per_img : 0;
  const long long a_bytes = ((nimg * ic.H * ic.W + ic.W + 1) * (long long)ic.C) * 4;
  const long long b_bytes = (long long)tilesN * ci.bn * ldb * 4;
  const long long o_rows = mode == GEMM_IMPLICIT_POOL ? M / 4 : M;
  const long long o_bytes = o_rows * (long long)ldc * 4;
  if (!fits_buf(a_bytes) || !fits_buf(b_bytes) || !fits_buf(o_bytes) || ntiles > 0x7fffffffLL || tilesN > 2)
    return -3;
  const BufDesc bd{in - (size_t)(ic.W + 1) * ic.C, (unsigned)a_bytes, (unsigned)b_bytes};
  const int m = (int)M, nt = (int)ntiles;
  const unsigned ob = (unsigned)o_bytes;
#define DNN_PERSIST_N(BM_, BN_, WM_, WN_, MF_, NS_, NTN_)                                                              \
  return mode == GEMM_IMPLICIT                                                                                        \
             ? launch_persist_t<BM_, BN_, WM_, WN_, MF_, NS_, 1, NTN_>(Bt, ldb, C, ldc, m, N, Kpad, epi, tilesN, nt, ic,  \
                                                                       bd, ob, stream)                                \
             : launch_persist_t<BM_, BN_, WM_, WN_, MF_, NS_, 2, NTN_>(Bt, ldb, C, ldc, m, N, Kpad, epi, tilesN, nt, ic,  \
                                                                       bd, ob, stream)
#define DNN_PERSIST(BM_, BN_, WM_, WN_, MF_, NS_)                                                                      \
  if (tilesN == 1) {                                                                                                  \
    DNN_PERSIST_N(BM_, BN_, WM_, WN_, MF_, NS_, 1);                                                                   \
  }                                                                                                                   \
  DNN_PERSIST_N(BM_, BN_, WM_, WN_, MF_, NS_, 2)
  if (cfg != GEMM_G256x64_K32 && persist_level() < 2) return -3;
  switch (cfg) {
    case GEMM_G256x64_K32: DNN_PERSIST(256, 64, 4, 2, 32, 2);
    case GEMM_64x128_K32: DNN_PERSIST(64, 128, 2, 2, 32, 2);
    case GEMM_G192x128_W8: DNN_PERSIST(192, 128, 2, 4, 32, 2);
    default: return -3;
  }
#undef DNN_PERSIST
#undef DNN_PERSIST_N
}

int launch_splitk_reduce(const float* slab, int splits, long long M, int N, float* C, int ldc,
                         const EpiParams& epi, hipStream_t stream) {
  if (M == 0 || N == 0) return 0;
  if (N % 4 != 0 || splits < 1) {
    set_error("splitk_reduce: N %d must be a multiple of 4", N);
    return -2;
  }
  if (M > 0x7fffffffLL || ldc % 4 != 0) {
    set_error("splitk_reduce: M %lld / ldc %d unsupported", M, ldc);
    return -2;
  }
  const int nq = N / 4, nqb = nq < 256 ? nq : 256, rp = 256 / nqb;
  long long blocks = (M + rp - 1) / rp;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, stream, slab, splits,
                     M * (long long)N, C, (int)M, N, ldc, epi, nqb, rp);
  return check_launch("splitk_reduce");
}

// ============================================================================ maxpool
// Window max with the reference's comparison: imax = first element; imax = imax >= x ? imax : x
// over every (di, dj), pad cells read as -FLT_MAX (np.finfo(float32).min).  The AVX ABI's
// vector channels compare with `>` instead (PoolGeom::gt_below).
template <int VEC>
__global__ void __launch_bounds__(256)
maxpool_nhwc_kernel(const float* __restrict__ in, float* __restrict__ out, PoolGeom g, long long total) {
  const int cq = g.C / VEC;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int c = (int)(i % cq) * VEC;
    long long p = i / cq;
    int ox = (int)(p % g.OW);
    long long t = p / g.OW;
    int oy = (int)(t % g.OH);
    int b = (int)(t / g.OH);
    int iy0 = oy * g.sh - g.pt, ix0 = ox * g.sw - g.pl;
    const float* base = in + (long long)b * g.H * g.W * g.C + c;
    auto fetch = [&](int iy, int ix) {
      f32x4 v;
      if ((unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W) {
        const float* s = base + ((long long)iy * g.W + ix) * g.C;
        if constexpr (VEC == 4) {
          v = *reinterpret_cast<const f32x4*>(s);
        } else {
          v[0] = *s;
        }
      } else {
        v = f32x4{-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
      }
      return v;
    };
    f32x4 m = fetch(iy0, ix0);
    for (int di = 0; di < g.kh; ++di)
      for (int dj = 0; dj < g.kw; ++dj) {
        f32x4 x = fetch(iy0 + di, ix0 + dj);
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          if (c + e < g.gt_below)
            m[e] = m[e] > x[e] ? m[e] : x[e];
          else
            m[e] = m[e] >= x[e] ? m[e] : x[e];
        }
      }
    float* d = out + p * g.C + c;
    if constexpr (VEC == 4) {
      *reinterpret_cast<f32x4*>(d) = m;
    } else {
      *d = m[0];
    }
  }
}

static dim3 stream_grid(long long total, int threads = 256) {
  long long b = (total + threads - 1) / threads;
  const long long cap = 256LL * 16;  // 256 CUs x 16 blocks, grid-stride for the rest
  return dim3((unsigned)(b < cap ? (b > 0 ? b : 1) : cap));
}

// Row form for C % 4 == 0: blockIdx.y = output row (b, oy), threads over (ox, channel quad) of
// that row: one 32-bit division per output quad instead of four 64-bit ones (pool5 of the
// plan: 0.019 -> see DESIGN.md).  Same comparisons as maxpool_nhwc_kernel.
__global__ void __launch_bounds__(256)
maxpool_rows_kernel(const float* __restrict__ in, float* __restrict__ out, PoolGeom g) {
  const int cq = g.C >> 2;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= g.OW * cq) return;
  const int row = blockIdx.y, ox = idx / cq, c = (idx - ox * cq) * 4;
  const int oy = row % g.OH, b = row / g.OH;
  const int iy0 = oy * g.sh - g.pt, ix0 = ox * g.sw - g.pl;
  const float* base = in + (size_t)b * g.H * g.W * g.C + c;
  auto fetch = [&](int iy, int ix) {
    if ((unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W)
      return *reinterpret_cast<const f32x4*>(base + ((size_t)iy * g.W + ix) * g.C);
    return f32x4{-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
  };
  f32x4 m = fetch(iy0, ix0);
  for (int di = 0; di < g.kh; ++di)
    for (int dj = 0; dj < g.kw; ++dj) {
      const f32x4 x = fetch(iy0 + di, ix0 + dj);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (c + e < g.gt_below)
          m[e] = m[e] > x[e] ? m[e] : x[e];
        else
          m[e] = m[e] >= x[e] ? m[e] : x[e];
      }
    }
  *reinterpret_cast<f32x4*>(out + ((size_t)row * g.OW + ox) * g.C + c) = m;
}

int launch_maxpool(const float* in, float* out, const PoolGeom& g, hipStream_t stream) {
  long long outs = (long long)g.B * g.OH * g.OW;
  if (outs == 0 || g.C == 0) return 0;
  const long long rows = (long long)g.B * g.OH, per_row = (long long)g.OW * (g.C / 4);
  if (g.C % 4 == 0 && rows <= 0x7fffffffLL && per_row <= 0x7fffffffLL && rows <= 65535) {
    hipLaunchKernelGGL(maxpool_rows_kernel, dim3((unsigned)((per_row + 255) / 256), (unsigned)rows), dim3(256), 0,
                       stream, in, out, g);
  } else if (g.C % 4 == 0) {
    long long total = outs * (g.C / 4);
    hipLaunchKernelGGL(maxpool_nhwc_kernel<4>, stream_grid(total), dim3(256), 0, stream, in, out, g, total);
  } else {
    long long total = outs * g.C;
    hipLaunchKernelGGL(maxpool_nhwc_kernel<1>, stream_grid(total), dim3(256), 0, stream, in, out, g, total);
  }
  return check_launch("maxpool");
}

// ============================================================================ weight packing
__global__ void pack_weights_kernel(const float* __restrict__ w, float* __restrict__ bt, int K, int N, int Kpad,
                                    int Npad, int order, int kh, int kw, int C) {
  long long total = (long long)Npad * Kpad;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int n = (int)(i / Kpad), k = (int)(i % Kpad);
    if (order == 3) {  // MFMA fragment order of the order-2 K (conv_patch16, 32x32x16): [n/32][k/16][lane][8]
      const long long e = i & 7, lane = (i >> 3) & 63, kq = (i >> 9) % (Kpad / 16), nb = (i >> 9) / (Kpad / 16);
      n = (int)(nb * 32 + (lane & 31));
      k = (int)(kq * 16 + 8 * (lane >> 5) + e);
    } else if (order == 4 || order == 5) {  // ... for 16x16x32: [n/16][k/32][lane][8]
      const long long e = i & 7, lane = (i >> 3) & 63, kq = (i >> 9) % (Kpad / 32), nb = (i >> 9) / (Kpad / 32);
      n = (int)(nb * 16 + (lane & 15));
      k = (int)(kq * 32 + 8 * (lane >> 4) + e);
    }
    float v = 0.f;
    if (n < N && k < K) {
      int src = k;
      if (order == 1) {
        int tap = k / C, c = k - tap * C;
        int dy = tap / kw, dx = tap - dy * kw;
        src = (c * kh + dy) * kw + dx;
      } else if (order >= 2) {  // k = (chunk * taps + tap) * cw + cc, c = cw * chunk + cc (conv_patch16: cw
        // 64; order 5, conv_tile16: 32-channel chunks)
        const int cw = order == 5 ? 32 : 64;
        const int taps = kh * kw, blk = k / cw, cc = k - blk * cw;
        const int chunk = blk / taps, tap = blk - chunk * taps;
        src = tap * C + cw * chunk + cc;
      }
      v = w[(long long)src * N + n];
    }
    bt[i] = v;
  }
}

int launch_pack_weights(const float* w, float* bt, int K, int N, int Kpad, int Npad, int order, int kh, int kw,
                        int C, hipStream_t stream) {
  long long total = (long long)Npad * Kpad;
  if (total == 0) return 0;
  hipLaunchKernelGGL(pack_weights_kernel, stream_grid(total), dim3(256), 0, stream, w, bt, K, N, Kpad, Npad,
                     order, kh, kw, C);
  return check_launch("pack_weights");
}

// ============================================================================ element-wise
__global__ void bias_add_kernel(const float* __restrict__ in, const float* __restrict__ b, float* __restrict__ out,
                                long long n, int C) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = in[i] + b[i % C];
}

__global__ void bn_mvg_kernel(const float* __restrict__ in, const float* __restrict__ mean,
                              const float* __restrict__ sq, const float* __restrict__ gamma,
                              float* __restrict__ out, long long n, int C) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    int d = (int)(i % C);
    out[i] = ((in[i] - mean[d]) / sq[d]) * gamma[d];
  }
}

__global__ void bn_ab_kernel(const float* __restrict__ in, const float* __restrict__ alpha,
                             const float* __restrict__ beta, float* __restrict__ out, long long n, int C) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    int d = (int)(i % C);
    float r = in[i] * alpha[d];
    out[i] = r - beta[d];
  }
}

__global__ void leaky_kernel(const float* __restrict__ in, float* __restrict__ out, long long n, int f32v) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float t = in[i];
    if (f32v) {
      float s = t * 0.1f;
      out[i] = t > s ? t : s;
    } else {
      out[i] = t < 0.f ? (float)(0.1 * (double)t) : t;
    }
  }
}

int launch_bias_add(const float* in, const float* b, float* out, long long n, int C, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(bias_add_kernel, stream_grid(n), dim3(256), 0, s, in, b, out, n, C);
  return check_launch("bias_add");
}
int launch_bn_mvg(const float* in, const float* mean, const float* sq, const float* gamma, float* out, long long n,
                  int C, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(bn_mvg_kernel, stream_grid(n), dim3(256), 0, s, in, mean, sq, gamma, out, n, C);
  return check_launch("batch_norm");
}
int launch_bn_ab(const float* in, const float* alpha, const float* beta, float* out, long long n, int C,
                 hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(bn_ab_kernel, stream_grid(n), dim3(256), 0, s, in, alpha, beta, out, n, C);
  return check_launch("batch_norm_ab");
}
int launch_leaky(const float* in, float* out, long long n, int f32_variant, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(leaky_kernel, stream_grid(n), dim3(256), 0, s, in, out, n, f32_variant);
  return check_launch("leaky_relu");
}

}  // namespace dnnhip
