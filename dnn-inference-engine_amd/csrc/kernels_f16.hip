// fp16 conv path (BASELINE config 5): launchers for the fp16 MFMA GEMM (gemm_f16.h) and the
// small fp16 kernels around it (weight / activation conversion, 2x2 max pool, split-K
// reduce).  Activations are NHWC fp16 between layers, accumulation and epilogue fp32.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cfloat>
#include "dnn_common.h"
#include "gemm_f16.h"
#include "gemm_f16_acc.h"
#include "gemm_f16_tile.h"

namespace dnnhip {

static int check16(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("launch %s: %s", what, hipGetErrorString(e));
    return -1;
  }
  return 0;
}

struct Cfg16Info {
  int bm, bn;
};
static const Cfg16Info kCfg16[GEMM16_NUM_CFGS] = {{128, 128}, {64, 128}, {32, 128}, {128, 64}, {32, 64},
                                                  {128, 32},  {32, 32},  {256, 128}, {128, 128}, {128, 256}, {128, 512}};
int gemm16_cfg_bn(int cfg) { return kCfg16[cfg].bn; }

// Same rules as the fp32 chooser (kernels.hip): every config is the 32x32x16 f16 family with
// BK = 64, and the split depends on (N, K) only, so results do not depend on M.
int choose_splitk16(int N, int K) {
  if (N >= 512 && N % 4 == 0 && K >= 2048 && (K / 64) % 3 == 0) return 3;
  return 1;
}

int choose_gemm16_cfg(long long M, int N, int K) {
  if (N <= 32) return ((M + 127) / 128) < 256 ? GEMM16_32x32_NS4 : GEMM16_128x32;
  if (N <= 64) return ((M + 127) / 128) < 256 ? GEMM16_32x64_NS4 : GEMM16_128x64;
  const int s = choose_splitk16(N, K);
  const long long t128 = ((M + 127) / 128) * ((N + 127) / 128);
  // split-K long-K layers with N % 512 == 0 (conv6/conv7): one 16-wave 128x512 workgroup per CU
  // stages 40 B per 1k flop instead of 64 (two 128x128 workgroups): the fp16 GEMM is bound by
  // the L2->LDS stream, conv7 0.252 -> 0.226 ms (batch 64).  Needs buffer-descriptor DMA; the
  // launcher falls back to 128x128 (same MFMA family and K order: same bits) when it is off.
  if (K >= 4096 && s > 1 && N % 512 == 0 && t128 * s >= 512) return GEMM16_128x512_W16;
  if (K >= 2048 && t128 * s >= 512) return GEMM16_128x128;
  const long long t64 = ((M + 63) / 64) * ((N + 127) / 128);
  if (t64 * s < 256) return GEMM16_32x128_NS4;
  return GEMM16_64x128;
}

long long splitk16_tiles(int cfg, long long M, int N) {
  return ((M + kCfg16[cfg].bm - 1) / kCfg16[cfg].bm) * ((N + kCfg16[cfg].bn - 1) / kCfg16[cfg].bn);
}
long long splitk16_fused_slab_floats(int cfg, long long M, int N, int splits) {
  return splitk16_tiles(cfg, M, N) * kCfg16[cfg].bm * kCfg16[cfg].bn * splits;
}

template <int MODE, bool ABUF>
static int launch16(int cfg, const half_t* A, int lda, const half_t* Bt, int ldb, half_t* C, float* slab, int ldc,
                    int M, int N, int Kpad, const EpiParams& epi, int tilesN, const ImplicitConv& ic,
                    const SplitK& sk, const BufDesc& bd, dim3 grid, hipStream_t st) {
  // 8 waves (two workgroups -> 4 waves per SIMD) on the 128- and 64-row tiles: the f16 GEMM
  // is LDS/L2-latency bound, and 8 waves of 32x64 / 32x32 beat 4 of 64x64 / 32x64 by 13-15%
  // on conv2-7 (MI355X, batch 64).  The wave layout does not change any summation order.
#define DNN_L16(BM_, BN_, WM_, WN_, NS_)                                                                     \
  hipLaunchKernelGGL((gemm_f16_glds_kernel<BM_, BN_, WM_, WN_, NS_, MODE, half_t, ABUF>), grid,                 \
                     dim3(WM_ * WN_ * 64), 0, st, A, lda, Bt, ldb, C, slab, ldc, M, N, Kpad, epi, tilesN, ic, sk, bd)
  switch (cfg) {
    case GEMM16_128x128: DNN_L16(128, 128, 4, 2, 2); break;
    case GEMM16_64x128: DNN_L16(64, 128, 2, 4, 2); break;
    case GEMM16_32x128_NS4: DNN_L16(32, 128, 1, 4, 4); break;
    case GEMM16_128x64: DNN_L16(128, 64, 4, 2, 2); break;
    case GEMM16_32x64_NS4: DNN_L16(32, 64, 1, 2, 4); break;
    case GEMM16_128x32: DNN_L16(128, 32, 4, 1, 2); break;
    case GEMM16_32x32_NS4: DNN_L16(32, 32, 1, 1, 4); break;
    case GEMM16_256x128_W8: DNN_L16(256, 128, 4, 2, 2); break;
    case GEMM16_128x128_W4: DNN_L16(128, 128, 2, 2, 2); break;
    case GEMM16_128x256_W8: DNN_L16(128, 256, 2, 4, 2); break;
    case GEMM16_128x512_W16:  // the ring takes all 160 KB of LDS: buffer-descriptor DMA only (no tap table)
      if constexpr (ABUF) {
        DNN_L16(128, 512, 2, 8, 2);
        break;
      } else {
        set_error("gemm16: cfg 128x512 needs buffer-descriptor DMA (shape too large or C unsupported)");
        return -2;
      }
    default:
      set_error("gemm16: bad cfg %d", cfg);
      return -2;
  }
#undef DNN_L16
  return check16("gemm_f16");
}

template <int MODE>
static int launch16_any(int cfg, const half_t* A, int lda, const half_t* Bt, int ldb, half_t* C, float* slab, int ldc,
                        int M, int N, int Kpad, const EpiParams& epi, int tilesN, const ImplicitConv& ic,
                        const SplitK& sk, const BufDesc* bd, dim3 grid, hipStream_t st) {
  if (bd)
    return launch16<MODE, true>(cfg, A, lda, Bt, ldb, C, slab, ldc, M, N, Kpad, epi, tilesN, ic, sk, *bd, grid, st);
  return launch16<MODE, false>(cfg, A, lda, Bt, ldb, C, slab, ldc, M, N, Kpad, epi, tilesN, ic, sk, BufDesc{}, grid,
                               st);
}

int launch_gemm16(int cfg, int mode, const half_t* A, int lda, const ImplicitConv& ic_in, const half_t* Bt, int ldb,
                  half_t* C, int ldc, long long M, int N, int Kpad, const EpiParams& epi, hipStream_t stream,
                  int splits, float* slab, unsigned* tickets) {
  if (M == 0 || N == 0) return 0;
  ImplicitConv ic = ic_in;
  implicit_conv_magic(&ic);
  if (cfg < 0 || cfg >= GEMM16_NUM_CFGS || mode < GEMM_DENSE || mode > GEMM_IMPLICIT_POOL) {
    set_error("gemm16: bad cfg %d / mode %d", cfg, mode);
    return -2;
  }
  // buffer-descriptor DMA (BufDesc): dense always when the descriptors fit; implicit for
  // C % 64 == 0 or C == 32.  (b_bytes is bounded with the widest tile's N padding.)
  long long a_bytes;
  const half_t* abase = A;
  if (mode == GEMM_DENSE) {
    a_bytes = M * (long long)lda * 2;
  } else {
    const long long per_img = mode == GEMM_IMPLICIT_POOL ? 4LL * ic.PH * ic.PW : (long long)ic.OH * ic.OW;
    const long long nimg = per_img > 0 ? M / per_img : 0;
    a_bytes = (nimg * ic.H * ic.W + ic.W + 1) * (long long)ic.C * 2;
    abase = A - (size_t)(ic.W + 1) * ic.C;
  }
  const long long b_bytes = (long long)((N + 511) / 512) * 512 * ldb * 2;
  const bool shape_ok = mode == GEMM_DENSE || ic.C % 64 == 0 || ic.C == 32;
  const bool abuf = !getenv_flag_off("DNN_HIP_GEMM_BUF") && shape_ok && a_bytes > 0 && a_bytes < 0x80000000LL &&
                    b_bytes > 0 && b_bytes < 0x80000000LL;
  if (cfg == GEMM16_128x512_W16 && !abuf) cfg = GEMM16_128x128;  // same MFMA family and K order
  const Cfg16Info ci = kCfg16[cfg];
  if (Kpad % 64 != 0 || ldb % 8 != 0 || M > 0x7fffffffLL || (mode == GEMM_DENSE && lda % 8 != 0) ||
      (mode != GEMM_DENSE && (ic.C % 8 != 0 || ic.kh * ic.kw > 30 || !ic.zero)) ||
      (mode == GEMM_IMPLICIT_POOL && (M % 4 != 0 || splits > 1))) {
    set_error("gemm16: unsupported shape M=%lld N=%d Kpad=%d mode=%d C=%d splits=%d", M, N, Kpad, mode, ic.C, splits);
    return -2;
  }
  const int tilesM = (int)((M + ci.bm - 1) / ci.bm), tilesN = (N + ci.bn - 1) / ci.bn;
  int grid = tilesM * tilesN;
  SplitK sk{0, grid, 0};
  if (splits > 1) {
    if (!slab || (Kpad / 64) % splits != 0 || (!tickets && N % 4 != 0) || (tickets && splits > 3)) {
      set_error("gemm16: split-K %d unsupported (Kpad %d, N %d)", splits, Kpad, N);
      return -2;
    }
    sk = SplitK{Kpad / 64 / splits, grid, M * (long long)N};
    if (tickets) {
      if (splitk16_fused_slab_floats(cfg, M, N, splits) * 4 >= 0x80000000LL) {
        set_error("gemm16: fused split-K slab over 2 GiB (M=%lld N=%d)", M, N);
        return -2;
      }
      sk.tickets = tickets;
      sk.out = reinterpret_cast<float*>(C);
      sk.ldo = ldc;
      sk.flags = epi.flags;
      sk.splits = splits;
    }
    grid *= splits;
  }
  sk.nmajor = nmajor_order(N, tilesN);
  BufDesc bd{reinterpret_cast<const float*>(abase), (unsigned)a_bytes, (unsigned)b_bytes};
  const BufDesc* pbd = abuf ? &bd : nullptr;
  switch (mode) {
    case GEMM_DENSE:
      return launch16_any<GEMM_DENSE>(cfg, A, lda, Bt, ldb, C, slab, ldc, (int)M, N, Kpad, epi, tilesN, ic, sk, pbd,
                                      dim3(grid), stream);
    case GEMM_IMPLICIT:
      return launch16_any<GEMM_IMPLICIT>(cfg, A, lda, Bt, ldb, C, slab, ldc, (int)M, N, Kpad, epi, tilesN, ic, sk,
                                         pbd, dim3(grid), stream);
    default:
      return launch16_any<GEMM_IMPLICIT_POOL>(cfg, A, lda, Bt, ldb, C, slab, ldc, (int)M, N, Kpad, epi, tilesN, ic,
                                              sk, pbd, dim3(grid), stream);
  }
}

// the fp16 plan's last layer when it is a dense GEMM without split-K (conv8): 32 x 128 tiles at
// every M (the tile shape changes no sum), the epilogue's fp32 values stored as fp32 into the
// plan's output (no fp16 rounding, no separate conversion kernel).  The tiles are 128 columns wide
// and their epilogue reads the parameters of every column of the tile, so the layer's packed
// weights and epilogue vectors must cover whole 128-column tiles (Npad % 128 == 0): a narrower head
// (OC <= 64, Npad 32 / 64) stays on the general launcher, whose tile width divides its Npad.
bool gemm16_f32out_supported(int splits, int Npad) { return splits == 1 && Npad > 0 && Npad % 128 == 0; }

int launch_gemm16_f32out(const half_t* A, int lda, const half_t* Bt, int ldb, int Npad, float* C, int ldc, long long M,
                         int N, int Kpad, const EpiParams& epi, hipStream_t stream) {
  if (M == 0 || N == 0) return 0;
  const long long a_bytes = M * (long long)lda * 2;
  const long long b_bytes = (long long)Npad * ldb * 2;  // the layer's own rows only
  if (!gemm16_f32out_supported(1, Npad) || N > Npad || Kpad % 64 != 0 || ldb % 8 != 0 || lda % 8 != 0 ||
      M > 0x7fffffffLL || a_bytes >= 0x80000000LL || b_bytes >= 0x80000000LL) {
    set_error("gemm16_f32out: unsupported shape M=%lld N=%d Kpad=%d", M, N, Kpad);
    return -2;
  }
  const int tilesM = (int)((M + 31) / 32), tilesN = (N + 127) / 128;
  SplitK sk{0, tilesM * tilesN, 0};
  sk.nmajor = nmajor_order(N, tilesN);
  const BufDesc bd{reinterpret_cast<const float*>(A), (unsigned)a_bytes, (unsigned)b_bytes};
  hipLaunchKernelGGL((gemm_f16_glds_kernel<32, 128, 1, 4, 4, GEMM_DENSE, float, true>), dim3(tilesM * tilesN),
                     dim3(256), 0, stream, A, lda, Bt, ldb, C, nullptr, ldc, (int)M, N, Kpad, epi, tilesN,
                     ImplicitConv{}, sk, bd);
  return check16("gemm16_f32out");
}

int launch_splitk_reduce16(const float* slab, int splits, long long M, int N, half_t* C, int ldc,
                           const EpiParams& epi, hipStream_t stream) {
  if (M == 0 || N == 0) return 0;
  if (N % 4 != 0 || ldc % 4 != 0 || M > 0x7fffffffLL) {
    set_error("splitk_reduce16: unsupported N %d / ldc %d", N, ldc);
    return -2;
  }
  const int nq = N / 4, nqb = nq < 256 ? nq : 256, rp = 256 / nqb;
  long long blocks = (M + rp - 1) / rp;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(splitk_reduce_kernel<half_t>, dim3((unsigned)blocks), dim3(256), 0, stream, slab, splits,
                     M * (long long)N, C, (int)M, N, ldc, epi, nqb, rp);
  return check16("splitk_reduce16");
}

// ---- element conversion
__global__ void f32_to_f16_kernel(const float* __restrict__ in, half_t* __restrict__ out, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = (half_t)in[i];
}
__global__ void f16_to_f32_kernel(const half_t* __restrict__ in, float* __restrict__ out, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = (float)in[i];
}
static long long grid_for(long long n) {
  long long b = (n + 255) / 256;
  return b < 1 ? 1 : (b > 16384 ? 16384 : b);
}
int launch_f32_to_f16(const float* in, half_t* out, long long n, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(f32_to_f16_kernel, dim3((unsigned)grid_for(n)), dim3(256), 0, s, in, out, n);
  return check16("f32_to_f16");
}
int launch_f16_to_f32(const half_t* in, float* out, long long n, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(f16_to_f32_kernel, dim3((unsigned)grid_for(n)), dim3(256), 0, s, in, out, n);
  return check16("f16_to_f32");
}

// ---- max pool on fp16 NHWC (C % 8 == 0): 8 channels per thread, the reference's window
// order and `m >= x ? m : x`, pad cells (-FLT_MAX in the reference) skipped
__global__ void maxpool16_kernel(const half_t* __restrict__ in, half_t* __restrict__ out, PoolGeom g, long long total,
                                 int opad) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  const int cq = g.C / 8;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cq) * 8;
    long long t = i / cq;
    const int ox = (int)(t % g.OW);
    t /= g.OW;
    const int oy = (int)(t % g.OH);
    const int b = (int)(t / g.OH);
    float m[8];
    bool first = true;
    for (int dy = 0; dy < g.kh; ++dy)
      for (int dx = 0; dx < g.kw; ++dx) {
        const int iy = oy * g.sh - g.pt + dy, ix = ox * g.sw - g.pl + dx;
        float v[8];
        if ((unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W) {
          const h8 x = *reinterpret_cast<const h8*>(in + (((size_t)b * g.H + iy) * g.W + ix) * g.C + c);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = -FLT_MAX;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = first ? v[e] : (m[e] >= v[e] ? m[e] : v[e]);
        first = false;
      }
    h8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (half_t)m[e];
    // opad: write into the interior of a zero-bordered [B][OH+2][OW+2][C] buffer (the input of a
    // conv3x3_f16_acc_kernel layer)
    *reinterpret_cast<h8*>(out + (((size_t)b * (g.OH + 2 * opad) + oy + opad) * (g.OW + 2 * opad) + ox + opad) * g.C +
                           c) = o;
  }
}
int launch_maxpool16(const half_t* in, half_t* out, const PoolGeom& g, hipStream_t s, int opad) {
  if (g.B == 0) return 0;
  if (g.C % 8 != 0) {
    set_error("maxpool16: C=%d must be a multiple of 8", g.C);
    return -2;
  }
  const long long total = (long long)g.B * g.OH * g.OW * (g.C / 8);
  hipLaunchKernelGGL(maxpool16_kernel, dim3((unsigned)grid_for(total)), dim3(256), 0, s, in, out, g, total, opad);
  return check16("maxpool16");
}

// ---- conv3x3_f16_acc_kernel (gemm_f16_acc.h): conv6/conv7 of the fp16 path, 176-row tiles,
// v_mfma_f32_16x16x32_f16; weights packed in order 4 ([n/16][k/32][lane][8])
constexpr int P16_NPR = 320, P16_BM = 176;
int patch16_pack_order() { return 4; }
constexpr bool P16_DEFAULT = true;  // measured: conv6 0.1415 -> 0.1286 ms, conv7 equal (batch 64)

// DNN_HIP_PATCH16=0/1 overrides the default choice of the patch kernel for eligible layers
static bool patch16_enabled() {
  const char* e = getenv("DNN_HIP_PATCH16");
  return e ? e[0] == '1' : P16_DEFAULT;
}

// rows of the padded input one bm-row tile spans (tap offsets included)
static int patch16_span(long long M, int H, int W) {
  const int Wp = W + 2;
  auto padded = [&](long long m) {
    const long long b = m / (H * W), r = m - b * H * W, oy = r / W, ox = r - oy * W;
    return (b * (H + 2) + oy + 1) * Wp + ox + 1;
  };
  long long mx = 0;
  const int bm = P16_BM;
  for (long long m0 = 0; m0 < M; m0 += bm) {
    const long long last = m0 + bm - 1 < M ? m0 + bm - 1 : M - 1;
    const long long v = padded(last) - padded(m0) + 2 * (Wp + 1) + 1;
    mx = v > mx ? v : mx;
  }
  return (int)(mx < 0x7fffffff ? mx : 0x7fffffff);
}

// the most padded rows a bm-row tile can span at any start (every alignment to the image grid;
// a batch's tiles start at multiples of bm, which reach many of them)
static int patch16_span_any(int H, int W, int bm) {
  const long long HW = (long long)H * W, Wp = W + 2;
  auto padded = [&](long long m) {
    const long long b = m / HW, r = m - b * HW, oy = r / W, ox = r - oy * W;
    return (b * (H + 2) + oy + 1) * Wp + ox + 1;
  };
  long long mx = 0;
  for (long long o = 0; o < HW; ++o) {
    const long long v = padded(o + bm - 1) - padded(o) + 2 * (Wp + 1) + 1;
    mx = v > mx ? v : mx;
  }
  return (int)(mx < 0x7fffffff ? mx : 0x7fffffff);
}

// the launcher's patch limits for any batch: the worst alignment decides it
// (patch16_span_any); the row-skewed LDS patch holds
// span * 10 + 12 * (span / Wp + 2) 16-B units (56 KiB).  A layer past them stays on the fp16 GEMM.
static bool patch16_fits(long long span, int W) {
  return span <= P16_NPR && span * 10 + 12 * (span / (W + 2) + 2) <= 7 * 8 * 64;
}

bool conv_patch16_supported(int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh, int sw, int pt,
                            int pl) {
  return kh == 3 && kw == 3 && sh == 1 && sw == 1 && pt == 1 && pl == 1 && OH == H && OW == W && C % 64 == 0 &&
         OC % 256 == 0 && patch16_enabled() && H > 0 && W > 0 &&
         patch16_fits(patch16_span_any(H, W, P16_BM), W);
}

int launch_conv_patch16(const half_t* in_padded, const half_t* Bt, int ldb, half_t* out, int out_padded, long long M,
                        int N, int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream) {
  if (M == 0 || N == 0) return 0;
  const long long nimg = M / ((long long)H * W);
  const long long in_bytes = nimg * (H + 2) * (W + 2) * (long long)C * 2;
  if (M % ((long long)H * W) != 0 || K != 9 * C || C % 64 != 0 || N % 256 != 0 || ldb < K || ldb % 8 != 0 ||
      in_bytes >= 0x80000000LL || M > 0x7fffffffLL || !patch16_fits(patch16_span(M, H, W), W)) {
    set_error("conv_patch16: unsupported shape M=%lld N=%d K=%d %dx%dx%d", M, N, K, H, W, C);
    return -2;
  }
  const int bm = P16_BM;
  const int tilesM = (int)((M + bm - 1) / bm), tilesN = N / 256;
  const Patch16Geom pg{H, W, C, out_padded};
  const long long b_bytes = (long long)N * ldb * 2;
  if (b_bytes >= 0x80000000LL) {
    set_error("conv_patch16: unsupported shape M=%lld N=%d K=%d %dx%dx%d", M, N, K, H, W, C);
    return -2;
  }
  constexpr int F16YOLO = EPI_BN_AB | EPI_LEAKY_F32;  // the fp16 path's folded epilogue, compiled in
  if (epi.flags == F16YOLO)
    hipLaunchKernelGGL((conv3x3_f16_acc_kernel<P16_BM, P16_NPR, F16YOLO>), dim3(tilesM * tilesN), dim3(512), 0, stream,
                       in_padded, Bt, ldb, out, (int)M, N, K, epi, tilesM, pg, (unsigned)in_bytes, (unsigned)b_bytes);
  else
    hipLaunchKernelGGL((conv3x3_f16_acc_kernel<P16_BM, P16_NPR, -1>), dim3(tilesM * tilesN), dim3(512), 0, stream,
                       in_padded, Bt, ldb, out, (int)M, N, K, epi, tilesM, pg, (unsigned)in_bytes, (unsigned)b_bytes);
  return check16("conv_patch16");
}

// ---- conv3x3_f16_tile_kernel (gemm_f16_tile.h): conv2-conv4 of the fp16 path, 2-D tiles with the
// 2x2/s2 pool fused; weights packed in order 5 ([n/16][k/32][lane][8], 32-channel chunks)
struct Tile16Shape {
  int th, tw, wm, tm;
};
static constexpr Tile16Shape kTile16[] = {{8, 52, 4, 7}, {4, 52, 2, 7}, {8, 26, 2, 7}};

// DNN_HIP_TILE16=0 keeps these layers on the implicit fp16 GEMM (A/B experiments)
static bool tile16_enabled() {
  const char* e = getenv("DNN_HIP_TILE16");
  return !(e && e[0] == '0');
}

// the tile shape computing the fewest rows for the frame (ties: the first, the widest workgroup)
static int tile16_shape(int H, int W) {
  int best = 0;
  long long bw = -1;
  for (int i = 0; i < 3; ++i) {
    const Tile16Shape& t = kTile16[i];
    const long long rows = (long long)((H + t.th - 1) / t.th) * ((W + t.tw - 1) / t.tw) * t.wm * t.tm * 16;
    if (bw < 0 || rows < bw) best = i, bw = rows;
  }
  return best;
}

// shape limits only (the launcher's check); the plan also applies the DNN_HIP_TILE16 switch
static bool tile16_shape_ok(int C, int OC, int H, int W) {
  return C % 32 == 0 && OC % 64 == 0 && H % 2 == 0 && W % 2 == 0 && H >= 2 && W >= 2 &&
         (long long)(H + 2) * (W + 2) * C * 2 < 0x40000000LL && (long long)OC * 9 * C * 2 < 0x80000000LL;
}

bool conv_tile16_supported(int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh, int sw, int pt,
                           int pl) {
  return kh == 3 && kw == 3 && sh == 1 && sw == 1 && pt == 1 && pl == 1 && OH == H && OW == W &&
         tile16_shape_ok(C, OC, H, W) && tile16_enabled();
}

template <int SH, int WN, int FL>
static void tile16_launch(dim3 grid, hipStream_t s, const half_t* in, const half_t* Bt, int ldb, half_t* out, int N,
                          const EpiParams& epi, int tilesX, int tilesY, int tilesN, int nsp, const Tile16Geom& g,
                          unsigned in_bytes, unsigned b_bytes) {
  constexpr Tile16Shape t = kTile16[SH];
  hipLaunchKernelGGL((conv3x3_f16_tile_kernel<t.th, t.tw, t.wm, WN, t.tm, FL>), grid, dim3(64 * t.wm * WN), 0, s, in,
                     Bt, ldb, out, N, epi, tilesX, tilesY, tilesN, nsp, g, in_bytes, b_bytes);
}

// persistent workgroups per CU (two: the kernel's registers allow two waves per SIMD);
// DNN_HIP_TILE16_WGS=n overrides it, 0 = one tile per workgroup
static int tile16_wgs_per_cu() {
  const char* e = getenv("DNN_HIP_TILE16_WGS");
  return e ? atoi(e) : 2;
}

#ifndef IMG16_BR
#define IMG16_BR 3
#endif
// whole-frame form (MODE 1) with the 2x2/s1 SAME pool fused: 13 x 13 frames (conv5 + pool5)
static bool img16_shape_ok(int C, int OC, int H, int W) {
  return H == 13 && W == 13 && C % 32 == 0 && OC % 64 == 0 && (long long)OC * 9 * C * 2 < 0x80000000LL;
}
bool conv_img16_supported(int C, int OC, int H, int W) {
  const char* e = getenv("DNN_HIP_IMG16");
  return img16_shape_ok(C, OC, H, W) && tile16_enabled() && !(e && e[0] == '0');
}

static int launch_img16(const half_t* in_padded, const half_t* Bt, int ldb, half_t* out, int out_padded, int n, int N,
                        int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream) {
  if (!img16_shape_ok(C, N, H, W) || K != 9 * C || ldb < K || ldb % 32 != 0) {
    set_error("conv_img16: unsupported shape N=%d K=%d %dx%dx%d ldb=%d", N, K, H, W, C, ldb);
    return -2;
  }
  const int tilesN = N / 64;
  const Tile16Geom g{H, W, C, H, W, out_padded};
  const long long img_in = (long long)(H + 2) * (W + 2) * C * 2;
  const long long img_out = (long long)(H + 2 * out_padded) * (W + 2 * out_padded) * N;  // halves
  const unsigned b_bytes = (unsigned)((long long)N * ldb * 2);
  constexpr int F16YOLO = EPI_BN_AB | EPI_LEAKY_F32;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int wpc = tile16_wgs_per_cu();
  const int per = (int)std::min<long long>(n, 0x7fffffffLL / img_in);
  for (int f0 = 0; f0 < n; f0 += per) {
    const int nf = std::min(per, n - f0);
    const int G = wpc > 0 ? std::max(1, std::min(nf, wpc * cus / tilesN)) : nf;
    const dim3 grid((unsigned)(G * tilesN));
    const half_t* in = in_padded + (size_t)f0 * (img_in / 2);
    half_t* o = out + (size_t)f0 * img_out;
    const unsigned ib = (unsigned)(nf * img_in);
    if (epi.flags == F16YOLO)
      hipLaunchKernelGGL((conv3x3_f16_tile_kernel<13, 13, 4, 1, 3, F16YOLO, 1, 6, 4, IMG16_BR>), grid, dim3(256), 0, stream, in,
                         Bt, ldb, o, N, epi, 1, 1, tilesN, nf, g, ib, b_bytes);
    else
      hipLaunchKernelGGL((conv3x3_f16_tile_kernel<13, 13, 4, 1, 3, -1, 1, 6, 4, IMG16_BR>), grid, dim3(256), 0, stream, in, Bt,
                         ldb, o, N, epi, 1, 1, tilesN, nf, g, ib, b_bytes);
    const int rc = check16("conv_img16");
    if (rc) return rc;
  }
  return 0;
}

int launch_conv_tile16(const half_t* in_padded, const half_t* Bt, int ldb, half_t* out, int out_padded, int n, int N,
                       int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream, int pool) {
  if (n == 0 || N == 0) return 0;
  if (pool == 2) return launch_img16(in_padded, Bt, ldb, out, out_padded, n, N, K, H, W, C, epi, stream);
  if (pool != 1 || !tile16_shape_ok(C, N, H, W) || K != 9 * C || ldb < K ||
      ldb % 32 != 0) {
    set_error("conv_tile16: unsupported shape N=%d K=%d %dx%dx%d ldb=%d", N, K, H, W, C, ldb);
    return -2;
  }
  const int sh = tile16_shape(H, W);
  const Tile16Shape& t = kTile16[sh];
  const int wn = (sh != 0 && N % 128 == 0) ? 2 : 1;
  const int tilesX = (W + t.tw - 1) / t.tw, tilesY = (H + t.th - 1) / t.th, tilesN = N / (64 * wn);
  const Tile16Geom g{H, W, C, H / 2, W / 2, out_padded};
  const long long img_in = (long long)(H + 2) * (W + 2) * C * 2;
  const long long img_out = (long long)(H / 2 + 2 * out_padded) * (W / 2 + 2 * out_padded) * N;  // halves
  const unsigned b_bytes = (unsigned)((long long)N * ldb * 2);
  constexpr int F16YOLO = EPI_BN_AB | EPI_LEAKY_F32;  // the fp16 path's folded epilogue, compiled in
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int wpc = tile16_wgs_per_cu();
  // frames per launch: the input's byte offsets stay 32-bit
  const int per = (int)std::min<long long>(n, 0x7fffffffLL / img_in);
  for (int f0 = 0; f0 < n; f0 += per) {
    const int nf = std::min(per, n - f0);
    const half_t* in = in_padded + (size_t)f0 * (img_in / 2);
    half_t* o = out + (size_t)f0 * img_out;
    const int nsp = nf * tilesY * tilesX;
    const int G = wpc > 0 ? std::max(1, std::min(nsp, wpc * cus / tilesN)) : nsp;  // workgroups per column group
    const dim3 grid((unsigned)(G * tilesN));
    const unsigned ib = (unsigned)(nf * img_in);
#define T16_GO(SH, WN, FL) \
  tile16_launch<SH, WN, FL>(grid, stream, in, Bt, ldb, o, N, epi, tilesX, tilesY, tilesN, nsp, g, ib, b_bytes)
    const bool y = epi.flags == F16YOLO;
    if (sh == 0)
      y ? T16_GO(0, 1, F16YOLO) : T16_GO(0, 1, -1);
    else if (sh == 1)
      wn == 2 ? (y ? T16_GO(1, 2, F16YOLO) : T16_GO(1, 2, -1)) : (y ? T16_GO(1, 1, F16YOLO) : T16_GO(1, 1, -1));
    else
      wn == 2 ? (y ? T16_GO(2, 2, F16YOLO) : T16_GO(2, 2, -1)) : (y ? T16_GO(2, 1, F16YOLO) : T16_GO(2, 1, -1));
#undef T16_GO
    const int rc = check16("conv_tile16");
    if (rc) return rc;
  }
  return 0;
}

}  // namespace dnnhip

#if T16DIAG
// diagnostic builds: conv3x3_f16_tile_kernel's phase stamps (gemm_f16_tile.h), class k (0: C 32,
// 1: C 64, 2: C 128, 3: other) of the last launch, n workgroups x 32 slots
extern "C" __attribute__((visibility("default"))) int dnn_t16_diag_stamps(unsigned long long* host, int k, int n) {
  if (k < 0 || k > 3 || n < 0 || n > dnnhip::T16_DIAG_WGS) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dnnhip::t16_diag_stamps), (size_t)n * 32 * sizeof(unsigned long long),
                             (size_t)k * dnnhip::T16_DIAG_WGS * 32 * sizeof(unsigned long long),
                             hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif

