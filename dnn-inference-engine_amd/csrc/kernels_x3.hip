// fp32 path, "x3" conv (gemm_x3_patch.h): exact three-way bf16 splits of fp32 operands on the
// bf16 MFMA for the 3x3 wide layers (conv6/conv7 of YOLOv2-tiny), its producers (the split
// max pool that feeds it) and its weight packing.
#include "dnn_common.h"
#include "gemm_x3_patch.h"
#include "gemm_x3_acc2.h"
#include "gemm_x3_lat.h"
#include "gemm_x3_1x1.h"
#include "gemm_x3_ktile.h"
#include "gemm_x3_img.h"

#include <cfloat>
#include <cstdlib>

namespace dnnhip {

constexpr int X3_YOLO_FL = EPI_BIAS | EPI_BN | EPI_LEAKY_F64;  // YOLO's epilogue set (compiled-in forms)

static int check_x3(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return -1;
  }
  return 0;
}

static unsigned grid_x3(long long n) {
  const long long b = (n + 255) / 256;
  return (unsigned)(b < 65535 * 8 ? (b > 0 ? b : 1) : 65535 * 8);
}

// ---- max pool (fp32 in, the reference's window order and `m >= x ? m : x`, pad cells skipped
// as in maxpool_nhwc_kernel) into the split planes of a zero-bordered x3 input; 8 channels per
// thread, one 16-B store per piece
__global__ void maxpool_x3_kernel(const float* __restrict__ in, bf16_bits* __restrict__ out, PoolGeom g,
                                  long long total) {
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
          const float* src = in + (((size_t)b * g.H + iy) * g.W + ix) * g.C + c;
          const float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 4);
          v[0] = x0.x, v[1] = x0.y, v[2] = x0.z, v[3] = x0.w, v[4] = x1.x, v[5] = x1.y, v[6] = x1.z, v[7] = x1.w;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = -FLT_MAX;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)
          m[e] = first ? v[e] : (c + e < g.gt_below ? (m[e] > v[e] ? m[e] : v[e]) : (m[e] >= v[e] ? m[e] : v[e]));
        first = false;
      }
    typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
    u16x8 s0, s1, s2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      unsigned short a, b2, c2;
      split3(m[e], a, b2, c2);
      s0[e] = a, s1[e] = b2, s2[e] = c2;
    }
    const size_t row = ((size_t)b * (g.OH + 2) + oy + 1) * (g.OW + 2) + ox + 1;
    bf16_bits* d = out + row * (3 * (size_t)g.C) + (c >> 5) * 96 + (c & 31);
    *reinterpret_cast<u16x8*>(d) = s0;
    *reinterpret_cast<u16x8*>(d + 32) = s1;
    *reinterpret_cast<u16x8*>(d + 64) = s2;
  }
}

int launch_maxpool_x3(const float* in, bf16_bits* out, const PoolGeom& g, hipStream_t s) {
  if (g.B == 0) return 0;
  if (g.C % 32 != 0) {
    set_error("maxpool_x3: C=%d must be a multiple of 32", g.C);
    return -2;
  }
  const long long total = (long long)g.B * g.OH * g.OW * (g.C / 8);
  hipLaunchKernelGGL(maxpool_x3_kernel, dim3(grid_x3(total)), dim3(256), 0, s, in, out, g, total);
  return check_x3("maxpool_x3");
}

// ---- split-K combine of the x3 conv: partials [splits][M][N] (raw fp32, `slab` floats apart)
// summed in split order ((p0 + p1) + p2 ...), the conv's fp32 epilogue, then an optional max
// pool in the reference's order (window cells in row order, `m >= x ? m : x`, pad cells
// skipped; kh = kw = 1, stride 1: no pool), into fp32 NHWC or the split planes of the next x3
// layer (out_split).  CPT channels per thread (8, or 4 for the many-slice combines of the
// latency plans: twice the threads, and every slice's load in flight at once), epilogue
// parameters loaded once per thread.
template <int KH, int KW, int S, int CPT = 8>  // KH = 0: any window (runtime loops); S = 0: any split count
__global__ void x3_combine_kernel(const float* __restrict__ part, int splits, long long slab, EpiParams epi,
                                  PoolGeom g, float* __restrict__ out, bf16_bits* __restrict__ out_split,
                                  long long total) {
  static_assert(CPT == 4 || CPT == 8, "channels per thread");
  constexpr int NV = CPT / 4;
  const int cq = g.C / CPT;
  // blocks in consecutive pixel order per XCD (xcd_tile): a window's other rows are read by
  // blocks of the same XCD, from its L2, instead of by every XCD from HBM (stride-1 pools
  // read each partial 4 times)
  const long long i = (long long)xcd_tile(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % cq) * CPT;
  long long t = i / cq;
  const int ox = (int)(t % g.OW);
  t /= g.OW;
  const int oy = (int)(t % g.OH);
  const int b = (int)(t / g.OH);
  auto ldv = [&](const float* a, float* d) {  // CPT floats, 16-B loads (c % CPT == 0)
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const float4 x = *reinterpret_cast<const float4*>(a + 4 * v);
      d[4 * v] = x.x, d[4 * v + 1] = x.y, d[4 * v + 2] = x.z, d[4 * v + 3] = x.w;
    }
  };
  // epilogue parameters of the CPT channels (the plan's arrays hold Npad >= C floats)
  float pb[CPT], pm[CPT], ps[CPT], pg[CPT];
  auto ldp = [&](const float* a, float (&d)[CPT], float dflt, bool on) {
    if (on) {
      ldv(a + c, d);
    } else {
#pragma unroll
      for (int e = 0; e < CPT; ++e) d[e] = dflt;
    }
  };
  ldp(epi.bias, pb, 0.f, (epi.flags & EPI_BIAS) != 0);
  ldp(epi.mean, pm, 0.f, (epi.flags & (EPI_BN | EPI_BN_AB)) != 0);
  ldp(epi.sq, ps, 1.f, (epi.flags & (EPI_BN | EPI_BN_AB)) != 0);
  ldp(epi.gamma, pg, 1.f, (epi.flags & EPI_BN) != 0);
  float hi[CPT], lo[CPT];
  if constexpr (KH > 0) {
    // fixed window: every load issued up front.  Window cells past the frame are clamped into
    // it: a clamped row / column is the window's first or last in-frame one, so the cell
    // repeats a window member and the max is unchanged
    float v[KH * KW][CPT];
#pragma unroll
    for (int dy = 0; dy < KH; ++dy)
#pragma unroll
      for (int dx = 0; dx < KW; ++dx) {
        int iy = oy * g.sh - g.pt + dy, ix = ox * g.sw - g.pl + dx;
        iy = iy < 0 ? 0 : iy >= g.H ? g.H - 1 : iy;
        ix = ix < 0 ? 0 : ix >= g.W ? g.W - 1 : ix;
        const float* src = part + (((size_t)b * g.H + iy) * g.W + ix) * g.C + c;
        float* w = v[dy * KW + dx];
        if constexpr (S > 0) {
          float x[S][CPT];
#pragma unroll
          for (int sp = 0; sp < S; ++sp) ldv(src + sp * slab, x[sp]);
#pragma unroll
          for (int e = 0; e < CPT; ++e) {
            w[e] = x[0][e];
#pragma unroll
            for (int sp = 1; sp < S; ++sp) w[e] += x[sp][e];  // split order ((p0 + p1) + p2 ...)
          }
        } else {  // many slices (latency plans): loads run ahead of the ordered sum
          ldv(src, w);
#pragma unroll 16
          for (int sp = 1; sp < splits; ++sp) {
            float y[CPT];
            ldv(src + sp * slab, y);
#pragma unroll
            for (int e = 0; e < CPT; ++e) w[e] += y[e];
          }
        }
      }
#pragma unroll
    for (int e = 0; e < CPT; ++e) {
      hi[e] = lo[e] = v[0][e];
#pragma unroll
      for (int q = 1; q < KH * KW; ++q) {
        hi[e] = __builtin_fmaxf(hi[e], v[q][e]);
        lo[e] = __builtin_fminf(lo[e], v[q][e]);
      }
    }
  } else {
    bool first = true;
    for (int dy = 0; dy < g.kh; ++dy)
      for (int dx = 0; dx < g.kw; ++dx) {
        const int iy = oy * g.sh - g.pt + dy, ix = ox * g.sw - g.pl + dx;
        if ((unsigned)iy >= (unsigned)g.H || (unsigned)ix >= (unsigned)g.W) continue;  // -FLT_MAX pad cell
        const float* src = part + (((size_t)b * g.H + iy) * g.W + ix) * g.C + c;
        float v[CPT];
        ldv(src, v);
        for (int sp = 1; sp < splits; ++sp) {
          float y[CPT];
          ldv(src + sp * slab, y);
#pragma unroll
          for (int e = 0; e < CPT; ++e) v[e] += y[e];
        }
#pragma unroll
        for (int e = 0; e < CPT; ++e) {
          hi[e] = first ? v[e] : __builtin_fmaxf(hi[e], v[e]);
          lo[e] = first ? v[e] : __builtin_fminf(lo[e], v[e]);
        }
        first = false;
      }
  }
  // pool before the epilogue, as the GEMMs' fused pools (pool_then_epilogue):
  // the epilogue is a chain of IEEE-monotone steps, so max f(v_i) = f(max v_i) (min for a
  // decreasing channel) -- one exact-division epilogue per output instead of one per cell
  float m[CPT];
#pragma unroll
  for (int e = 0; e < CPT; ++e) {
    const bool dec = ((epi.flags & EPI_BN) && pg[e] < 0.f) || ((epi.flags & EPI_BN_AB) && pm[e] < 0.f);
    m[e] = apply_epilogue(dec ? lo[e] : hi[e], pb[e], pm[e], ps[e], pg[e], epi.flags);
  }
  if (out_split) {
    typedef unsigned short u16v __attribute__((ext_vector_type(CPT)));
    u16v s0, s1, s2;
#pragma unroll
    for (int e = 0; e < CPT; ++e) {
      unsigned short a, b2, c2;
      split3(m[e], a, b2, c2);
      s0[e] = a, s1[e] = b2, s2[e] = c2;
    }
    const size_t row = ((size_t)b * (g.OH + 2) + oy + 1) * (g.OW + 2) + ox + 1;
    const size_t d = 2 * (row * (3 * (size_t)g.C) + (c >> 5) * 96 + (c & 31));  // (bytes)
    if constexpr (CPT == 8) {
      store16_at(out_split, d, __builtin_bit_cast(u32x4, s0));
      store16_at(out_split, d + 64, __builtin_bit_cast(u32x4, s1));
      store16_at(out_split, d + 128, __builtin_bit_cast(u32x4, s2));
    } else {
      store8_at(out_split, d, __builtin_bit_cast(u32x2, s0));
      store8_at(out_split, d + 64, __builtin_bit_cast(u32x2, s1));
      store8_at(out_split, d + 128, __builtin_bit_cast(u32x2, s2));
    }
  } else {
    const size_t d = 4 * ((((size_t)b * g.OH + oy) * g.OW + ox) * g.C + c);  // (bytes)
#pragma unroll
    for (int v = 0; v < NV; ++v)
      store16_at(out, d + 16 * v, __builtin_bit_cast(u32x4, f32x4{m[4 * v], m[4 * v + 1], m[4 * v + 2], m[4 * v + 3]}));
  }
}

int launch_x3_combine(const float* part, int splits, long long slab, const EpiParams& epi, const PoolGeom& g,
                      float* out, bf16_bits* out_split, hipStream_t s) {
  if (g.B == 0) return 0;
  if (g.C % 32 != 0 || splits < 1 || (out == nullptr) == (out_split == nullptr)) {
    set_error("x3_combine: unsupported C=%d splits=%d", g.C, splits);
    return -2;
  }
  const int win = g.kh == 2 && g.kw == 2 ? 2 : g.kh == 1 && g.kw == 1 ? 1 : 0;
  // many slices (> 2: latency plans): 4 channels per thread (8 measured slower there)
  const int cpt = splits > 2 && win > 0 ? 4 : 8;
  const long long total = (long long)g.B * g.OH * g.OW * (g.C / cpt);
  const long long out_bytes = out_split ? (long long)g.B * (g.OH + 2) * (g.OW + 2) * g.C * 6
                                        : (long long)g.B * g.OH * g.OW * g.C * 4;
  if ((total + 255) / 256 > 0x7fffffffLL || out_bytes >= 0x80000000LL) {  // (32-bit store offsets)
    set_error("x3_combine: %lld outputs", total);
    return -2;
  }
  const dim3 grid((unsigned)((total + 255) / 256));  // (64- / 128-thread blocks: same time, measured)
#define X3C(KH, KW, S, CPT) \
  hipLaunchKernelGGL((x3_combine_kernel<KH, KW, S, CPT>), grid, dim3(256), 0, s, part, splits, slab, epi, g, out, out_split, total)
  if (win == 2 && splits == 2)
    X3C(2, 2, 2, 8);
  else if (win == 2 && splits == 1)
    X3C(2, 2, 1, 8);
  else if (win == 1 && splits == 2)
    X3C(1, 1, 2, 8);
  else if (win == 1 && cpt == 4)
    X3C(1, 1, 0, 4);
  else if (win == 1)
    X3C(1, 1, 0, 8);
  else if (win == 2 && cpt == 4)
    X3C(2, 2, 0, 4);
  else if (win == 2)
    X3C(2, 2, 0, 8);
  else
    X3C(0, 0, 0, 8);
#undef X3C
  return check_x3("x3_combine");
}

// ---- weights: HWIO fp32 [K = tap * C + c][N] -> split pieces in the kernel's fragment order
// [n/16][step = chunk * 9 + tap][piece][lane][8], k inside a step = 8 (lane >> 4) + e
__global__ void pack_weights_x3_kernel(const float* __restrict__ w, bf16_bits* __restrict__ out, int K, int N, int Npad,
                                       int C, int taps) {  // taps: 9 (3x3) or 1 (1x1: step = chunk)
  const int nk = K / 32;
  const long long total = (long long)(Npad / 16) * nk * 3 * 512;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int e = (int)(i & 7), lane = (int)((i >> 3) & 63);
    const long long q = i >> 9;
    const int p = (int)(q % 3);
    const long long r = q / 3;
    const int s = (int)(r % nk), nb = (int)(r / nk);
    const int n = nb * 16 + (lane & 15);
    const int chunk = s / taps, tap = s - chunk * taps, c = chunk * 32 + 8 * (lane >> 4) + e;
    const float v = n < N ? w[((size_t)tap * C + c) * N + n] : 0.f;
    unsigned short s0, s1, s2;
    split3(v, s0, s1, s2);
    out[i] = p == 0 ? s0 : p == 1 ? s1 : s2;
  }
}

// C = 16 (conv3x3_x3_c16_kernel): [n/16][step 0..4][piece][lane][8], k = 8 (lane >> 4) + e of
// step s = tap 2 s + (k >> 4), channel k & 15 (tap 9: zero)
__global__ void pack_weights_x3c16_kernel(const float* __restrict__ w, bf16_bits* __restrict__ out, int N, int Npad) {
  const long long total = (long long)(Npad / 16) * 5 * 3 * 512;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int e = (int)(i & 7), lane = (int)((i >> 3) & 63);
    const long long q = i >> 9;
    const int p = (int)(q % 3);
    const long long r = q / 3;
    const int s = (int)(r % 5), nb = (int)(r / 5);
    const int n = nb * 16 + (lane & 15), k = 8 * (lane >> 4) + e, tap = 2 * s + (k >> 4), c = k & 15;
    const float v = n < N && tap < 9 ? w[((size_t)tap * 16 + c) * N + n] : 0.f;
    unsigned short s0, s1, s2;
    split3(v, s0, s1, s2);
    out[i] = p == 0 ? s0 : p == 1 ? s1 : s2;
  }
}

int launch_pack_weights_x3(const float* w, bf16_bits* out, int K, int N, int Npad, int C, hipStream_t s) {
  if (C == 16 && K == 144 && Npad % 32 == 0 && Npad >= N) {
    const long long total = (long long)(Npad / 16) * 5 * 3 * 512;
    hipLaunchKernelGGL(pack_weights_x3c16_kernel, dim3(grid_x3(total)), dim3(256), 0, s, w, out, N, Npad);
    return check_x3("pack_weights_x3 (c16)");
  }
  if ((K != 9 * C && K != C) || C % 32 != 0 || Npad % 64 != 0 || Npad < N) {
    set_error("pack_weights_x3: unsupported K=%d N=%d Npad=%d C=%d", K, N, Npad, C);
    return -2;
  }
  const long long total = (long long)(Npad / 16) * (K / 32) * 3 * 512;
  hipLaunchKernelGGL(pack_weights_x3_kernel, dim3(grid_x3(total)), dim3(256), 0, s, w, out, K, N, Npad, C,
                     K == C ? 1 : 9);
  return check_x3("pack_weights_x3");
}

// ---- the conv
constexpr int X3_BM = 176, X3_NPR = 320;

// DNN_HIP_X3=0 keeps these layers on the fp32 MFMA (implicit GEMM).  The DNN_HIP_* switches are
// read by the *_supported functions the plan calls when it chooses a layer's kernel; launchers
// check shape limits only, so a plan keeps running what it chose if the environment changes later.
static bool x3_enabled() {
  const char* e = getenv("DNN_HIP_X3");
  return !(e && e[0] == '0');
}

constexpr int X3_NPR_POOL = 352;  // pool-window-major tiles span more rows (26x26: 350)

// rows of the padded input one BM-row tile spans (tap offsets included); pool: window-major
static long long x3_span(long long M, int H, int W, bool pool = false) {
  const int Wp = W + 2, PH = (H + 1) / 2, PW = (W + 1) / 2;
  auto padded = [&](long long m) {
    if (pool) {
      const long long w = m >> 2, q = m & 3, b = w / (PH * PW), r = w - b * PH * PW, py = r / PW, px = r - py * PW;
      long long oy = 2 * py + (q >> 1), ox = 2 * px + (q & 1);
      if (oy >= H || ox >= W) oy = 2 * py, ox = 2 * px;
      return (b * (H + 2) + oy + 1) * Wp + ox + 1;
    }
    const long long b = m / (H * W), r = m - b * H * W, oy = r / W, ox = r - oy * W;
    return (b * (H + 2) + oy + 1) * Wp + ox + 1;
  };
  long long mx = 0;
  for (long long m0 = 0; m0 < M; m0 += X3_BM) {
    const long long last = m0 + X3_BM - 1 < M ? m0 + X3_BM - 1 : M - 1;
    const long long v = padded(last) - padded(m0) + 2 * (Wp + 1) + 1;
    mx = v > mx ? v : mx;
  }
  return mx;
}

// narrow layers: the 2-D tile kernel (conv3x3_x3_tile2_kernel), 8 x 26 (N = 64) or 4 x 26
// (N % 128 == 0) output pixels per tile: YOLOv2-tiny's 104- and 52-wide frames in whole tiles
constexpr int X3T_TM = 7;  // row blocks of 16 per wave

// which kernel runs an x3 layer: 0 the row-run kernel (N % 256 == 0), 1 tile kernel N = 64 from
// one 32-channel chunk, 2 tile kernel N % 128 == 0 (double-buffered chunks), 3 the 16-channel
// kernel (fp32 input, split while staged); -1 none (the layer stays on the fp32 MFMA).  Shape
// only: DNN_HIP_X3_C16=0 is applied by conv_x3_supported at plan time.
static int x3_kind(int N, int C) {
  if (C == 16) return N == 32 ? 3 : -1;
  if (N % 256 == 0) return 0;
  if (N == 64 && C == 32) return 1;
  if (N % 128 == 0) return 2;
  return -1;
}

int conv_x3_kind(int OC, int C) { return x3_kind(OC, C); }

bool conv_x3_supported(int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl) {
  if (!(kh == 3 && kw == 3 && sh == 1 && sw == 1 && pt == 1 && pl == 1 && OH == H && OW == W &&
        (C % 32 == 0 || C == 16) && x3_enabled()))
    return false;
  const int kind = x3_kind(OC, C);
  if (kind < 0 || ((kind == 1 || kind == 2) && getenv_flag_off("DNN_HIP_X3_TILE")) ||
      (kind == 3 && getenv_flag_off("DNN_HIP_X3_C16")))
    return false;
  // a tile must fit the patch for any batch: spans grow with M only until a tile crosses whole
  // images, so two images' worth of rows decides it (tile kernel: fixed patch)
  return kind > 0 || x3_span(2LL * H * W + X3_BM, H, W) <= X3_NPR;
}

// ... with a fused 2x2/s2 pool (pool-window-major rows; tile kernel: even frames, so windows
// never straddle tiles or the frame edge)
bool conv_x3_pool_supported(int OC, int C, int H, int W) {
  if (x3_kind(OC, C) > 0) return H % 2 == 0 && W % 2 == 0;
  const long long rows = 4LL * ((H + 1) / 2) * ((W + 1) / 2);
  return x3_span(2 * rows + X3_BM, H, W, true) <= X3_NPR_POOL;
}

long long x3_tiles(long long batch, int OH, int OW, int OC, int C, int K) {
  const int kind = x3_kind(OC, C);
  if (kind == 3) return batch * ((OH + 15) / 16) * ((OW + 25) / 26);
  if (kind > 0)
    return batch * ((OH + (kind == 1 ? 7 : 3)) / (kind == 1 ? 8 : 4)) * ((OW + 25) / 26) * (OC / (kind == 1 ? 64 : 128));
  return (batch * OH * OW + X3_BM - 1) / X3_BM * (OC / 256) * x3_splits(OC, K);
}

size_t x3_act_bytes(long long nimg, int H, int W, int C) { return (size_t)nimg * (H + 2) * (W + 2) * C * 6; }

// N = 512 (conv5): 62 x 2 = 124 tiles of 176 x 256 at batch 64, half the chip -> 2 K slices;
// wider layers fill it alone, narrower ones (N = 256: 246 tiles) too
int x3_splits(int N, int K) { return (N % 256 == 0 && N > 256 && N <= 512 && (K / 288) % 2 == 0) ? 2 : 1; }


int launch_conv_x3(const bf16_bits* in_split, const bf16_bits* Bt, float* out, bf16_bits* out_split, long long M,
                   int N, int Npad, int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream, int splits,
                   int pool, bool lat) {
  if (M == 0 || N == 0) return 0;
  // pool: M counts GEMM rows, 4 per pooled pixel
  const int PH = pool ? (H + 1) / 2 : 0, PW = pool ? (W + 1) / 2 : 0;
  const long long per_img = pool ? 4LL * PH * PW : (long long)H * W;
  const long long nimg = M / per_img;
  const long long in_bytes = (long long)x3_act_bytes(nimg, H, W, C);
  const long long b_bytes = (long long)(Npad / 16) * (K / 32) * 3072;
  const int kind = x3_kind(N, C);
  if (kind == 3) {  // fp32 NHWC input (in_split is the producer's float buffer)
    const long long in32 = nimg * H * W * 64LL, b16 = (long long)(Npad / 16) * 5 * 3072;
    if (M % per_img != 0 || K != 144 || Npad != N || splits != 1 || (pool && (H % 2 || W % 2)) ||
        in32 >= 0x80000000LL || b16 >= 0x80000000LL || (out_split == nullptr) == (out == nullptr) ||
        x3_act_bytes(nimg, pool ? PH : H, pool ? PW : W, N) >= 0x80000000ULL) {
      set_error("conv_x3 (c16): unsupported shape M=%lld N=%d K=%d %dx%dx%d", M, N, K, H, W, C);
      return -2;
    }
    const int tilesX = (W + 25) / 26, tilesY = (H + 15) / 16;
    const long long blocks = nimg * tilesX * tilesY;
    if (blocks > 0x7fffffffLL || N != 32) {
      set_error("conv_x3 (c16): N=%d (32 only) or grid too large", N);
      return -2;
    }
    const X3Geom xg{H, W, C, out_split ? 1 : 0, 1, PH, PW};
    const float* in32p = reinterpret_cast<const float*>(in_split);
    (void)b16;
    // (two accumulators per output, gemm_x3_patch.h x3_step).  DNN_HIP_X3_C16P=0 (read per
    // launch, experiments): one tile per workgroup (conv3x3_x3_c16_kernel); default: persistent
    // (conv3x3_x3_c16p_kernel, the last K step on 16x16x16; measured at batch 64: conv1 0.164 ->
    // 0.152 ms, forward -14 us), same bits up to the K = 16 step's summation
    // latency plans (one frame: 104 tiles of 16 x 26): 4 x 26 tiles, 4 waves of 2 row blocks, 416
    // tiles; tap 8 on the 32-wide MFMA (the batch plans' persistent kernel puts it on the 16-wide
    // one: not the same bits, so the batch plans never take this shape)
    const bool small = lat && blocks < 2LL * device_cu_count();
    if (small && pool) {
      const int ty4 = (H + 3) / 4;
      hipLaunchKernelGGL((conv3x3_x3_c16_kernel<4, 26, 4, 2, true>), dim3((unsigned)(nimg * tilesX * ty4)), dim3(256), 0,
                         stream, in32p, Bt, out, out_split, N, epi, tilesX, ty4, xg, (unsigned)in32);
    } else if (pool && out_split && blocks >= 4LL * device_cu_count() && !getenv_flag_off("DNN_HIP_X3_C16PP") &&
               !getenv_flag_off("DNN_HIP_X3_C16P")) {
      // batch grids (>= 4 tiles per CU): the ping-pong form, one 512-thread workgroup per CU, the
      // persistent kernel's bits (conv3x3_x3_c16pp_kernel).  DNN_HIP_X3_C16PP=0 (read per launch,
      // A/B) keeps the two-workgroup persistent kernel; DNN_HIP_X3_PP_PRIO=0 the default priority
      const int G = device_cu_count();
      const int prio = !getenv_flag_off("DNN_HIP_X3_PP_PRIO");
      if (epi.flags == X3_YOLO_FL)
        hipLaunchKernelGGL((conv3x3_x3_c16pp_kernel<X3_YOLO_FL>), dim3((unsigned)G), dim3(512), 0, stream, in32p, Bt,
                           out_split, epi, tilesX, tilesY, (int)blocks, xg, (unsigned)in32, prio);
      else
        hipLaunchKernelGGL((conv3x3_x3_c16pp_kernel<-1>), dim3((unsigned)G), dim3(512), 0, stream, in32p, Bt,
                           out_split, epi, tilesX, tilesY, (int)blocks, xg, (unsigned)in32, prio);
    } else if (getenv_flag_off("DNN_HIP_X3_C16P") || !pool) {  // (the persistent kernel: the pooled form, conv1)
      if (pool)
        hipLaunchKernelGGL((conv3x3_x3_c16_kernel<16, 26, 4, 7, true>), dim3((unsigned)blocks), dim3(256), 0, stream,
                           in32p, Bt, out, out_split, N, epi, tilesX, tilesY, xg, (unsigned)in32);
      else
        hipLaunchKernelGGL((conv3x3_x3_c16_kernel<16, 26, 4, 7, false>), dim3((unsigned)blocks), dim3(256), 0, stream,
                           in32p, Bt, out, out_split, N, epi, tilesX, tilesY, xg, (unsigned)in32);
    } else {
      const long long slots = 2LL * device_cu_count();
      const dim3 pgrid((unsigned)(blocks < slots ? blocks : slots));
#define C16P(FL_)                                                                                              \
  hipLaunchKernelGGL((conv3x3_x3_c16p_kernel<true, true, FL_>), pgrid, dim3(256), 0, stream, in32p, Bt, out,  \
                     out_split, N, epi, tilesX, tilesY, (int)blocks, xg, (unsigned)in32)
      if (epi.flags == X3_YOLO_FL)  // YOLO's epilogue set compiled in
        C16P(X3_YOLO_FL);
      else
        C16P(-1);
#undef C16P
    }
    return check_x3("conv_x3 (c16)");
  }
  if (kind > 0) {
    if (M % per_img != 0 || K != 9 * C || Npad != N || splits != 1 || (pool && (H % 2 || W % 2)) ||
        in_bytes >= 0x80000000LL || b_bytes >= 0x80000000LL || (out_split == nullptr) == (out == nullptr) ||
        x3_act_bytes(nimg, pool ? PH : H, pool ? PW : W, N) >= 0x80000000ULL) {
      set_error("conv_x3 (tile): unsupported shape M=%lld N=%d K=%d %dx%dx%d", M, N, K, H, W, C);
      return -2;
    }
    // kind 2: 4 x 26 tiles, 4 waves (1 x 4), 2 workgroups per CU (80 KB LDS each): at batch 64
    // conv3 is 1,664 tiles, 6.5 per CU, where 4 x 52 tiles of 8 waves were 3.25 rounds of one per
    // CU (measured 0.157 -> 0.131 ms).  kind 1: 8 x 26 tiles (1.35x patch rows per output row;
    // 4 x 52: 1.56x, conv2 0.142 -> 0.140 ms)
    // small batches (the single-frame latency plans: conv2 52 tiles, conv3 26 at one frame, a
    // quarter of the chip or less): 2 x 26 tiles, 2 x 2 waves of 2 row blocks x 32 columns (each
    // wave's MFMA chain 2 / 7 of the batch form's), 64 columns per workgroup.  The summation order
    // depends on (N, K) only: the same bits as the batch tiles
    const long long big = nimg * ((H + (kind == 1 ? 7 : 3)) / (kind == 1 ? 8 : 4)) * ((W + 25) / 26) *
                          (N / (kind == 1 ? 64 : 128));
    const bool small = big < 2LL * device_cu_count();
    const int TH = small ? 2 : kind == 1 ? 8 : 4, TW = 26;
    const int tilesX = (W + TW - 1) / TW, tilesY = (H + TH - 1) / TH, tilesN = N / (small || kind == 1 ? 64 : 128);
    const long long blocks = nimg * tilesX * tilesY * tilesN;
    if (blocks > 0x7fffffffLL) {
      set_error("conv_x3 (tile): grid too large");
      return -2;
    }
    const X3Geom xg{H, W, C, out_split ? 1 : 0, 1, PH, PW};
    // conv3x3_x3_tile2_kernel: 224-B LDS rows by LDS-DMA, immediate tap offsets, two accumulators
#define X3T2M(TH_, TW_, WM, WN, TM_, NBUF, POOL, FL_)                                                         \
  hipLaunchKernelGGL((conv3x3_x3_tile2_kernel<TH_, TW_, WM, WN, TM_, NBUF, POOL, FL_>), dim3((unsigned)blocks),  \
                     dim3(64 * WM * WN), 0, stream, in_split, Bt, out, out_split, N, K, epi, tilesX, tilesY, tilesN, \
                     xg, (unsigned)in_bytes, (unsigned)b_bytes)
#define X3T2(TH_, TW_, WM, WN, NBUF, POOL, FL_) X3T2M(TH_, TW_, WM, WN, X3T_TM, NBUF, POOL, FL_)
    const bool yolo = epi.flags == X3_YOLO_FL;  // YOLO's epilogue set compiled in for the pooled forms
    // N = 64 from one chunk (conv2), pooled into split planes, batch grids of >= 4 tiles per CU:
    // the ping-pong kernel, one workgroup per CU (conv3x3_x3_pp_kernel; the tile kernel's bits).
    // DNN_HIP_X3_PP=0 (read per launch, A/B) keeps the tile kernel, DNN_HIP_X3_PP_PRIO=0 its MFMA
    // steps at the default priority.  (conv3's shape -- N = 128, two chunks, 192-B skewed rows --
    // measured slower on it, 0.1199 vs 0.1133 ms: its MFMA steps are 3.6x its store steps, so the
    // two tile-kernel workgroups per CU already keep the MFMA pipes fed, and one workgroup per CU
    // serialises the CUs' 6.5 tiles.)
    if (pool && out_split && !small && blocks >= 4LL * device_cu_count() && !getenv_flag_off("DNN_HIP_X3_PP") &&
        kind == 1 && C == 32 && N == 64) {
      const int G = device_cu_count();
      const int prio = !getenv_flag_off("DNN_HIP_X3_PP_PRIO");
#define X3PP(TH_, WM_, WN_, NCH_, PU_, SK_, FL_, LEAD_)                                                             \
  hipLaunchKernelGGL((conv3x3_x3_pp_kernel<TH_, 26, WM_, WN_, X3T_TM, NCH_, PU_, SK_, FL_, LEAD_>), dim3((unsigned)G), \
                     dim3(512), 0, stream, in_split, Bt, out_split, N, epi, tilesX, tilesY, (int)blocks, xg,         \
                     (unsigned)in_bytes, (unsigned)b_bytes, prio)
      // (fragments two row blocks ahead: conv2 0.1130 -> 0.1118 ms against one, same call)
      if (yolo)
        X3PP(8, 2, 2, 1, 14, 0, X3_YOLO_FL, 2);
      else
        X3PP(8, 2, 2, 1, 14, 0, -1, 2);
#undef X3PP
      return check_x3("conv_x3 (ping-pong)");
    }
    if (small) {
      if (pool && yolo && kind == 2)
        X3T2M(2, 26, 2, 2, 2, 2, true, X3_YOLO_FL);
      else if (pool && yolo)
        X3T2M(2, 26, 2, 2, 2, 1, true, X3_YOLO_FL);
      else if (pool && kind == 2)
        X3T2M(2, 26, 2, 2, 2, 2, true, -1);
      else if (pool)
        X3T2M(2, 26, 2, 2, 2, 1, true, -1);
      else if (kind == 2)
        X3T2M(2, 26, 2, 2, 2, 2, false, -1);
      else
        X3T2M(2, 26, 2, 2, 2, 1, false, -1);
    } else if (kind == 2 && pool && yolo) {
      X3T2(4, 26, 1, 4, 2, true, X3_YOLO_FL);
    } else if (kind == 2 && pool) {
      X3T2(4, 26, 1, 4, 2, true, -1);
    } else if (kind == 2) {
      X3T2(4, 26, 1, 4, 2, false, -1);
    } else if (pool && yolo) {
      X3T2(8, 26, 2, 2, 1, true, X3_YOLO_FL);
    } else if (pool) {
      X3T2(8, 26, 2, 2, 1, true, -1);
    } else {
      X3T2(8, 26, 2, 2, 1, false, -1);
    }
#undef X3T2
#undef X3T2M
    return check_x3("conv_x3 (tile)");
  }
  if (M % per_img != 0 || K != 9 * C || C % 32 != 0 || N % 256 != 0 || Npad != N || (pool && splits != 1) ||
      in_bytes >= 0x80000000LL || b_bytes >= 0x80000000LL || M > 0x7fffffffLL ||
      x3_span(M, H, W, pool != 0) > (pool ? X3_NPR_POOL : X3_NPR) ||
      (out_split == nullptr) == (out == nullptr) || splits < 1 || (K / 288) % splits != 0 ||
      (splits > 1 && out_split != nullptr)) {
    set_error("conv_x3: unsupported shape M=%lld N=%d K=%d %dx%dx%d", M, N, K, H, W, C);
    return -2;
  }
  const int tilesM = (int)((M + X3_BM - 1) / X3_BM), tilesN = N / 256;
  // splits > 1: `out` receives the raw partials [splits][M][N] (x3_combine_kernel finishes).
  const X3Geom xg{H, W, C, splits > 1 ? 2 : out_split ? 1 : 0, splits, PH, PW};
  const dim3 grid(tilesM * tilesN * (pool ? 1 : splits));
#define X3AF(NPR_, POOL_, FL_)                                                                                    \
  hipLaunchKernelGGL((conv3x3_x3_acc2_kernel<X3_BM, NPR_, POOL_, FL_>), grid, dim3(512), 0, stream, in_split, Bt, \
                     out, out_split, (int)M, N, K, epi, tilesM, xg, (unsigned)in_bytes, (unsigned)b_bytes)
  if (epi.flags == X3_YOLO_FL && xg.out_mode != 2) {  // YOLO's set compiled in
    if (pool)
      X3AF(X3_NPR_POOL, true, X3_YOLO_FL);
    else
      X3AF(X3_NPR, false, X3_YOLO_FL);
  } else {
    if (pool)
      X3AF(X3_NPR_POOL, true, -1);
    else
      X3AF(X3_NPR, false, -1);
  }
#undef X3AF
  return check_x3("conv_x3");
}

// ---- small-M x3 conv (latency plans, gemm_x3_lat.h): 64-column tiles (NCP = 2), one or two
// chunks per workgroup, chosen so that a frame's layer is ~256 workgroups: two chunks when the
// one-chunk grid would be >= 512 (conv7: 16 N tiles x 32 chunks), else one (conv6: 16 x 16).
// DNN_HIP_X3L_CPW=1|2 forces it.  Read when a plan is built (x3_lat_splits fixes the layer's
// slice count); the launch derives the chunks per workgroup from that count.
static int x3_lat_cpw(int N, int K) {
  const char* e = getenv("DNN_HIP_X3L_CPW");
  const int force = e ? atoi(e) : 0;
  const int chunks = K / 288;
  if (force == 1 || force == 2) return chunks % force == 0 ? force : 1;
  return chunks % 2 == 0 && (long long)(N / 64) * chunks >= 512 ? 2 : 1;
}

int x3_lat_splits(int N, int K) { return (K / 288) / x3_lat_cpw(N, K); }

constexpr int X3L_NPR_SMALL = 240;  // one 13x13 frame's tile spans 225 padded rows

bool conv_x3_lat_supported(long long batch, int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh,
                           int sw, int pt, int pl) {
  if (!(kh == 3 && kw == 3 && sh == 1 && sw == 1 && pt == 1 && pl == 1 && OH == H && OW == W && C % 32 == 0 &&
        OC % 64 == 0 && x3_enabled()))
    return false;
  const long long M = batch * H * W;
  // only where one-chunk slices fill half the chip (conv6 / conv7 of a frame: 256 / 512): with
  // fewer workgroups the launch, the patch staging and the separate combine (~5-7 us each at
  // batch 1) outweigh the x3 arithmetic (measured: conv3-conv5 at 64 workgroups, with their
  // pools in the combine, no faster than the fp32 MFMA's in-GEMM split-K)
  const long long wgs = (M + X3_BM - 1) / X3_BM * (OC / 64) * (C / 32);
  const char* e = getenv("DNN_HIP_X3_LAT_MINWG");  // (experiments)
  if (wgs < (e ? atoll(e) : 128)) return false;
  return M <= 0x7fffffffLL && x3_span(M, H, W) <= X3_NPR;
}

// ---- K split inside the workgroup (latency plans' conv4 / conv5, gemm_x3_ktile.h): 32-column
// workgroups of 4 waves = 4 K groups, one wave per SIMD (two waves of a workgroup sharing a SIMD
// serialize their MFMA chains: 64-column, 8-wave workgroups measured 13.3 / 14.8 us with half
// the chip idle).  Two shapes: frames up to 26 wide with 4 chunks (conv4: 26 x 26 x 128, pooled
// or not; 2 x 14 tiles, 2 row blocks, one chunk per group) and up to 13 wide with 8 chunks
// (conv5: 13 x 13 x 256; one-row tiles, one row block, two chunks per group).
// pool: 0 none, 1 a fused 2x2/s2 pool, 2 a fused 2x2/s1 SAME pool (YOLO's pool5; 13-wide shape)
static int x3_ktile_shape(int C, int OC, int H, int W, int pool) {
  if (OC % 64 != 0) return -1;
  if (C == 128 && W > 13 && W <= 26 && (pool == 0 || (pool == 1 && H % 2 == 0 && W % 2 == 0))) return 0;
  if (C == 256 && W <= 13 && pool != 1) return 1;
  if (C == 64 && OC == 128 && W > 26 && W <= 52 && (pool == 0 || (pool == 1 && H % 2 == 0 && W % 2 == 0)))
    return 2;  // conv3
  return -1;
}

// conv3x3_x3_img_kernel (gemm_x3_img.h): whole-image tiles, instantiated for YOLOv2-tiny's 13x13
// frames.  DNN_HIP_X3_IMG=0 (plan time) keeps the wide kernel's K slices + the pool5 combine.
static bool x3_img_shape_ok(int C, int OC, int H, int W) {
  return H == 13 && W == 13 && C % 32 == 0 && OC % 128 == 0;
}
bool conv_x3_img_supported(int C, int OC, int H, int W) {
  return x3_img_shape_ok(C, OC, H, W) && x3_enabled() && !getenv_flag_off("DNN_HIP_X3_IMG");
}

int launch_conv_x3_img(const bf16_bits* in_split, const bf16_bits* Bt, float* out, bf16_bits* out_split, int n, int N,
                       int Npad, int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream) {
  if (n == 0 || N == 0) return 0;
  const long long in_bytes = (long long)x3_act_bytes(n, H, W, C);
  const long long b_bytes = (long long)(Npad / 16) * (K / 32) * 3072;
  if (!x3_img_shape_ok(C, N, H, W) || K != 9 * C || Npad != N || (out_split == nullptr) == (out == nullptr) ||
      in_bytes >= 0x80000000LL || b_bytes >= 0x80000000LL || x3_act_bytes(n, H, W, N) >= 0x80000000ULL) {
    set_error("conv_x3_img: unsupported shape n=%d N=%d K=%d %dx%dx%d", n, N, K, H, W, C);
    return -2;
  }
  const long long blocks = (long long)n * (N / 128);
  if (blocks > 0x7fffffffLL) {
    set_error("conv_x3_img: grid too large");
    return -2;
  }
  if (epi.flags == X3_YOLO_FL)
    hipLaunchKernelGGL((conv3x3_x3_img_kernel<13, 13, X3_YOLO_FL>), dim3((unsigned)blocks), dim3(512), 0, stream,
                       in_split, Bt, out, out_split, N, K, epi, C, (unsigned)in_bytes, (unsigned)b_bytes);
  else
    hipLaunchKernelGGL((conv3x3_x3_img_kernel<13, 13, -1>), dim3((unsigned)blocks), dim3(512), 0, stream, in_split, Bt,
                       out, out_split, N, K, epi, C, (unsigned)in_bytes, (unsigned)b_bytes);
  return check_x3("conv_x3_img");
}

bool conv_x3_ktile_supported(long long batch, int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh,
                             int sw, int pt, int pl, int pool) {
  if (!(kh == 3 && kw == 3 && sh == 1 && sw == 1 && pt == 1 && pl == 1 && OH == H && OW == W)) return false;
  if (!x3_enabled() || x3_ktile_shape(C, OC, H, W, pool) < 0) return false;
  return (long long)x3_act_bytes(batch, H, W, C) < 0x80000000LL &&
         (long long)(OC / 16) * (9 * C / 32) * 3072 < 0x80000000LL;
}

int launch_conv_x3_ktile(const bf16_bits* in_split, const bf16_bits* Bt, float* out, bf16_bits* out_split, long long M,
                         int N, int Npad, int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream,
                         int pool) {
  if (M == 0 || N == 0) return 0;
  const bool p2 = pool == 1;  // (pool 2, stride 1: the output frame is the input frame)
  const int PH = p2 ? (H + 1) / 2 : 0, PW = p2 ? (W + 1) / 2 : 0;
  const long long per_img = p2 ? 4LL * PH * PW : (long long)H * W;
  const long long nimg = M / per_img;
  const long long in_bytes = (long long)x3_act_bytes(nimg, H, W, C);
  const long long b_bytes = (long long)(Npad / 16) * (K / 32) * 3072;
  const int shape = x3_ktile_shape(C, N, H, W, pool);
  if (shape < 0 || M % per_img != 0 || K != 9 * C || Npad != N || in_bytes >= 0x80000000LL ||
      b_bytes >= 0x80000000LL || (out_split == nullptr) == (out == nullptr) ||
      x3_act_bytes(nimg, p2 ? PH : H, p2 ? PW : W, N) >= 0x80000000ULL) {
    set_error("conv_x3_ktile: unsupported shape M=%lld N=%d K=%d %dx%dx%d pool=%d", M, N, K, H, W, C, pool);
    return -2;
  }
  // (conv4: 2 x 14 tiles, two per 26-wide row -- 208 workgroups at one frame, not 104, each wave
  // two row blocks, not four: -2.8 us per replay, same bits; conv3 on 2 x 14 tiles measured slower)
  const int TH = shape == 1 ? 1 : 2, TW = shape == 1 ? 13 : shape == 0 ? 14 : 26;
  const int tilesX = (W + TW - 1) / TW, tilesY = (H + TH - 1) / TH, tilesN = N / 32;
  const long long blocks = nimg * tilesX * tilesY * tilesN;
  if (blocks > 0x7fffffffLL) {
    set_error("conv_x3_ktile: grid too large");
    return -2;
  }
  const X3Geom xg{H, W, C, out_split ? 1 : 0, 1, PH, PW};
  const bool yolo = epi.flags == X3_YOLO_FL;
#define X3KW(TH_, TW_, WM_, TM_, KW_, CPK_, POOL_, FL_, PL1_)                                                       \
  hipLaunchKernelGGL((conv3x3_x3_ktile_kernel<TH_, TW_, WM_, 1, TM_, KW_, CPK_, POOL_, FL_, 3, PL1_>),                \
                     dim3((unsigned)blocks), dim3(64 * WM_ * KW_), 0, stream, in_split, Bt, out, out_split, N, K, epi,  \
                     tilesX, tilesY, tilesN, xg, (unsigned)in_bytes, (unsigned)b_bytes)
#define X3K(TH_, TW_, TM_, CPK_, POOL_, FL_, PL1_) X3KW(TH_, TW_, 1, TM_, 4, CPK_, POOL_, FL_, PL1_)
  // (a 5-step weight ring measured 1 % slower than 3 in the earlier 8-wave form)
  if (shape == 2 && p2 && yolo)  // (conv3: 2 chunks = 2 K groups of 2 x 2 row blocks, 4 waves)
    X3KW(2, 26, 2, 2, 2, 1, true, X3_YOLO_FL, false);
  else if (shape == 2 && p2)
    X3KW(2, 26, 2, 2, 2, 1, true, -1, false);
  else if (shape == 2)
    X3KW(2, 26, 2, 2, 2, 1, false, -1, false);
  else if (shape == 0 && p2 && yolo)
    X3K(2, 14, 2, 1, true, X3_YOLO_FL, false);
  else if (shape == 0 && p2)
    X3K(2, 14, 2, 1, true, -1, false);
  else if (shape == 0)
    X3K(2, 14, 2, 1, false, -1, false);
  else if (pool == 2 && yolo)  // (each one-row tile computes the row below it too: 2 row blocks)
    X3K(1, 13, 2, 2, false, X3_YOLO_FL, true);
  else if (pool == 2)
    X3K(1, 13, 2, 2, false, -1, true);
  else if (yolo)
    X3K(1, 13, 1, 2, false, X3_YOLO_FL, false);
  else
    X3K(1, 13, 1, 2, false, -1, false);
#undef X3K
#undef X3KW
  return check_x3("conv_x3_ktile");
}

// 1x1 form (latency plans' conv8): 16 rows x 32 columns, K groups of one wave (4; at K = 1024: 16
// groups, 16 columns)
static bool x3_1x1_ktile_shape_ok(int C, int OC, int H, int W) {
  // the launcher's instantiations: K / 128 = 1, 2, 4 or 8 chunk quads (other widths, e.g. C = 384
  // after a kind-2 tile conv, stay on the fp32 GEMM)
  const int nq = C / 128;
  return C % 128 == 0 && (nq == 1 || nq == 2 || nq == 4 || nq == 8) && OC >= 1 && H >= 1 && W >= 1;
}
bool conv_x3_1x1_ktile_supported(int C, int OC, int H, int W) {
  return x3_1x1_ktile_shape_ok(C, OC, H, W) && x3_enabled() && !getenv_flag_off("DNN_HIP_X3_1X1");
}

int launch_conv_x3_1x1_ktile(const bf16_bits* in_split, const bf16_bits* Bt, float* out, long long M, int N, int Npad,
                             int K, int H, int W, int C, const EpiParams& epi, hipStream_t stream) {
  if (M == 0 || N == 0) return 0;
  const long long per_img = (long long)H * W, nimg = M / per_img;
  const long long in_bytes = (long long)x3_act_bytes(nimg, H, W, C);
  const long long b_bytes = (long long)(Npad / 16) * (K / 32) * 3072;
  const int cpk = K / 128;
  if (M % per_img != 0 || K != C || !x3_1x1_ktile_shape_ok(C, N, H, W) || Npad % 32 != 0 || Npad < N ||
      in_bytes >= 0x80000000LL || b_bytes >= 0x80000000LL || M > 0x7fffffffLL ||
      (cpk != 1 && cpk != 2 && cpk != 4 && cpk != 8)) {
    set_error("conv_x3_1x1_ktile: unsupported shape M=%lld N=%d K=%d %dx%dx%d", M, N, K, H, W, C);
    return -2;
  }
  // K = 1024 (conv8): 16-column workgroups (88 at one frame, not 44: -1.4 us per replay, same bits)
  const int nj = cpk == 8 ? 1 : 2;
  const int tilesM = (int)((M + 15) / 16), tilesN = Npad / (16 * nj);
  const X3Geom xg{H, W, C, 0, 1, 0, 0};
#define X3K1J(KW_, CPK_, NJ_)                                                                                         \
  hipLaunchKernelGGL((conv1x1_x3_ktile_kernel<KW_, CPK_, -1, NJ_>), dim3((unsigned)((long long)tilesM * tilesN)),      \
                     dim3(64 * KW_), 0, stream, in_split, Bt, out, (int)M, N, K, epi, tilesM, xg, (unsigned)in_bytes,    \
                     (unsigned)b_bytes)
#define X3K1W(KW_, CPK_) X3K1J(KW_, CPK_, 2)
#define X3K1(CPK_) X3K1W(4, CPK_)
  // K = 1024 (conv8): 16 groups of two chunks -- the loads of 16 waves in flight per CU, not 4
  // (graph replay -1.9 us, -1.5 us with 8 groups, same call; the groups' order changes the sums)
  if (cpk == 8)
    X3K1J(16, 2, 1);
  else if (cpk == 4)
    X3K1(4);
  else if (cpk == 2)
    X3K1(2);
  else
    X3K1(1);
#undef X3K1
#undef X3K1W
#undef X3K1J
  return check_x3("conv_x3_1x1_ktile");
}

int launch_conv_x3_lat(const bf16_bits* in_split, const bf16_bits* Bt, float* part, long long M, int N, int Npad,
                       int K, int H, int W, int C, int splits, hipStream_t stream) {
  if (M == 0 || N == 0) return 0;
  const long long per_img = (long long)H * W, nimg = M / per_img;
  const long long in_bytes = (long long)x3_act_bytes(nimg, H, W, C);
  const long long b_bytes = (long long)(Npad / 16) * (K / 32) * 3072;
  const int cpw = splits >= 1 && (K / 288) % splits == 0 ? (K / 288) / splits : 0;  // the plan's x3_lat_splits
  const long long span = M <= 0x7fffffffLL ? x3_span(M, H, W) : 1LL << 40;
  if (M % per_img != 0 || K != 9 * C || C % 32 != 0 || N % 64 != 0 || Npad != N || (cpw != 1 && cpw != 2) ||
      in_bytes >= 0x80000000LL || b_bytes >= 0x80000000LL || span > X3_NPR || part == nullptr ||
      (long long)splits * M * N * 4 >= 0x80000000LL) {  // (32-bit partial store offsets)
    set_error("conv_x3_lat: unsupported shape M=%lld N=%d K=%d %dx%dx%d splits=%d", M, N, K, H, W, C, splits);
    return -2;
  }
  const int tilesM = (int)((M + X3_BM - 1) / X3_BM), tilesN = N / 64;
  const long long blocks = (long long)tilesM * tilesN * splits;
  if (blocks > 0x7fffffffLL) {
    set_error("conv_x3_lat: grid too large");
    return -2;
  }
  const X3Geom xg{H, W, C, 2, splits, 0, 0};
#define X3L(CPW_, NPR_)                                                                                       \
  hipLaunchKernelGGL((conv3x3_x3_lat_kernel<2, CPW_, NPR_>), dim3((unsigned)blocks), dim3(512), 0, stream, in_split, \
                     Bt, part, (int)M, N, K, tilesM, xg, (unsigned)in_bytes, (unsigned)b_bytes)
  if (cpw == 2 && span <= X3L_NPR_SMALL)
    X3L(2, X3L_NPR_SMALL);
  else if (cpw == 2)
    X3L(2, X3_NPR);
  else if (span <= X3L_NPR_SMALL)
    X3L(1, X3L_NPR_SMALL);
  else
    X3L(1, X3_NPR);
#undef X3L
  return check_x3("conv_x3_lat");
}

}  // namespace dnnhip

namespace dnnhip {

// ---- 1x1 x3 conv (gemm_x3_1x1.h): YOLOv2-tiny conv8 on its producer's split planes
bool conv_x3_1x1_supported(int C, int OC, int H, int W) {
  return C % 32 == 0 && C >= 32 && OC >= 1 && H >= 1 && W >= 1 && x3_enabled() && !getenv_flag_off("DNN_HIP_X3_1X1");
}

int launch_conv_x3_1x1(const bf16_bits* in_split, const bf16_bits* Bt, float* out, long long M, int N, int Npad, int K,
                       int H, int W, int C, const EpiParams& epi, hipStream_t stream) {
  if (M == 0 || N == 0) return 0;
  const long long per_img = (long long)H * W, nimg = M / per_img;
  const long long in_bytes = (long long)x3_act_bytes(nimg, H, W, C);
  const long long b_bytes = (long long)(Npad / 16) * (K / 32) * 3072;
  if (M % per_img != 0 || K != C || C % 32 != 0 || Npad % X3_1X1_BN != 0 || Npad < N || in_bytes >= 0x80000000LL ||
      b_bytes >= 0x80000000LL || M > 0x7fffffffLL || out == nullptr) {
    set_error("conv_x3_1x1: unsupported shape M=%lld N=%d K=%d %dx%dx%d", M, N, K, H, W, C);
    return -2;
  }
  // 32-row tiles (338 workgroups at batch 64; 64-row tiles measured 0.039 vs 0.0355 ms)
  constexpr int tmw = 2;
  const long long tilesM = (M + 16 * tmw - 1) / (16 * tmw), blocks = tilesM * (Npad / X3_1X1_BN);
  if (blocks > 0x7fffffffLL) {
    set_error("conv_x3_1x1: grid too large");
    return -2;
  }
  const X3Geom xg{H, W, C, 0, 1, 0, 0};
  constexpr int BIAS = EPI_BIAS;
#define X1(FL_, TM_)                                                                                             \
  hipLaunchKernelGGL((conv1x1_x3_kernel<FL_, TM_>), dim3((unsigned)blocks), dim3(256), 0, stream, in_split, Bt, \
                     out, (int)M, N, K, epi, (int)tilesM, xg, (unsigned)in_bytes, (unsigned)b_bytes)
  if (epi.flags == BIAS)  // YOLO's detection layer: bias, linear
    X1(BIAS, 2);
  else
    X1(-1, 2);
#undef X1
  return check_x3("conv_x3_1x1");
}

}  // namespace dnnhip

#if (X3DIAG & 16) != 0
// diagnostic builds (tools/build_diag.sh, X3DIAG bit 16): the wide x3 kernel's per-workgroup
// stamps [t0, r0, t1, r1] of its last launch (s_memtime / s_memrealtime at the main loop's
// start and end) copied to host[0 .. 4n)
extern "C" __attribute__((visibility("default"))) int dnn_x3_diag_stamps(unsigned long long* host, int n) {
  if (n < 0 || n > dnnhip::X3_DIAG_WGS) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dnnhip::x3_diag_stamps), (size_t)n * 4 * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif

#if (X3DIAG & 32) != 0
// diagnostic builds (X3DIAG bit 32): conv3x3_x3_c16p_kernel's per-workgroup cycle sums of its
// last launch (C16_DIAG_SLOTS per workgroup, gemm_x3_patch.h) copied to host[0 .. slots n)
extern "C" __attribute__((visibility("default"))) int dnn_c16_diag_stamps(unsigned long long* host, int n) {
  if (n < 0 || n > dnnhip::C16_DIAG_WGS) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dnnhip::c16_diag_stamps), (size_t)n * dnnhip::C16_DIAG_SLOTS * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif

#if (X3DIAG & 256) != 0
// diagnostic builds (X3DIAG bit 256): conv3x3_x3_ktile_kernel's per-workgroup s_memrealtime
// stamps [start, patch landed, MFMAs done, end] of its last launch copied to host[0 .. 4n)
extern "C" __attribute__((visibility("default"))) int dnn_ktile_diag_stamps(unsigned long long* host, int n) {
  if (n < 0 || n > dnnhip::KT_DIAG_WGS) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dnnhip::ktile_diag_stamps), (size_t)n * 4 * sizeof(unsigned long long),
                             0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif

#if (X3DIAG & 1024) != 0
// diagnostic builds (X3DIAG bit 1024): conv3x3_x3_tile2_kernel's per-workgroup stamps of its last
// launch per layer class (T2_DIAG_SLOTS per workgroup, gemm_x3_patch.h) copied to host[0 .. slots n)
extern "C" __attribute__((visibility("default"))) int dnn_tile2_diag_stamps(unsigned long long* host, int n) {
  if (n < 0 || n > 2 * dnnhip::T2_DIAG_WGS * dnnhip::T2_DIAG_SLOTS) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dnnhip::tile2_diag_stamps), (size_t)n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif

#if (X3DIAG & 16384) != 0
// diagnostic builds (X3DIAG bit 16384): conv3x3_x3_img_kernel's per-workgroup phase stamps of its
// last launch (8 per workgroup) copied to host[0 .. 8 n)
extern "C" __attribute__((visibility("default"))) int dnn_img_diag_stamps(unsigned long long* host, int n) {
  if (n < 0 || n > dnnhip::IMG_DIAG_WGS) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dnnhip::img_diag_stamps), (size_t)n * 8 * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif

#if (X3DIAG & 8192) != 0
// diagnostic builds (X3DIAG bit 8192): conv3x3_x3_acc2_kernel's per-workgroup phase stamps of its
// last launch per layer class (N = 256 / 512 / other; 8 per workgroup) copied to host[0 .. 8 n)
extern "C" __attribute__((visibility("default"))) int dnn_acc2_diag_stamps(unsigned long long* host, int n) {
  if (n < 0 || n > 3 * dnnhip::AC_DIAG_WGS) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dnnhip::acc2_diag_stamps), (size_t)n * 8 * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif

#if (X3DIAG & 32768) != 0
// diagnostic builds (X3DIAG bit 32768): conv3x3_x3_c16pp_kernel's per-workgroup step cycle sums of its
// last launch (16 per workgroup, gemm_x3_patch.h) copied to host[0 .. 16 n)
extern "C" __attribute__((visibility("default"))) int dnn_c16pp_diag_stamps(unsigned long long* host, int n) {
  if (n < 0 || n > dnnhip::C16PP_DIAG_WGS) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dnnhip::c16pp_diag_stamps), (size_t)n * 16 * sizeof(unsigned long long),
                             0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif
#if (X3DIAG & 2048) != 0
// diagnostic builds (X3DIAG bit 2048): conv3x3_x3_pp_kernel's per-workgroup step cycle sums of its
// last launch (8 per workgroup, gemm_x3_patch.h) copied to host[0 .. 8 n)
extern "C" __attribute__((visibility("default"))) int dnn_pp_diag_stamps(unsigned long long* host, int n) {
  if (n < 0 || n > dnnhip::PP_DIAG_WGS) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dnnhip::pp_diag_stamps), (size_t)n * 8 * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif

#if (X3DIAG & 512) != 0
// diagnostic builds (X3DIAG bit 512): conv3x3_x3_lat_kernel's per-workgroup s_memrealtime stamps
// [start, patch landed, MFMAs done, end] of its last launch copied to host[0 .. 4n)
extern "C" __attribute__((visibility("default"))) int dnn_lat_diag_stamps(unsigned long long* host, int n) {
  if (n < 0 || n > dnnhip::LAT_DIAG_WGS) return -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dnnhip::lat_diag_stamps), (size_t)n * 4 * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif
