// fp32 MFMA GEMM kernels for the conv hot path (gfx950), device code only.
//
// C[M][N] = A[M][K] * Bt[N][K]^T with a fused per-output-channel epilogue.
//   A  : im2col rows (or the NHWC input itself for 1x1 convs), row-major, lda >= K
//   Bt : packed weights, row n = output channel, K contiguous (HWIO -> [N][K])
//   C  : NHWC output, row = output pixel, ldc = number of channels
// This replaces cblas_sgemm(RowMajor, N, N, M=oh*ow, N=od, K=ic*kh*kw, 1, col, K,
// kernel_r, od, 0, out, od) of proj3/dnn_openblas.c:184-192 and the bias/bn/leaky passes
// that follow it (proj3/dnn_openblas.c:9-65, 236-254).
//
// Two main loops:
//   gemm_f32_mfma_kernel   register-staged global->LDS double buffer (any BK, any tile)
//   gemm_f32_glds_kernel   LDS-DMA (global_load_lds_dwordx4) ring of NS stages with a
//                          counted vmcnt across raw s_barriers (cdna_hip_programming.md
//                          §5 "Pipelining across barriers"); LDS image XOR-swizzled on the
//                          SOURCE address so the fragment reads are conflict-free.
#pragma once
#include <hip/hip_runtime.h>
#include <cfloat>
#include <type_traits>
#include "dnn_common.h"

namespace dnnhip {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

typedef _Float16 half_t;
// store conversion of the fp32 epilogue result: identity, or round-to-nearest-even to fp16
__device__ __forceinline__ void store_out(float* p, float v) { *p = v; }
__device__ __forceinline__ void store_out(half_t* p, float v) { *p = (half_t)v; }

// x / d correctly rounded (the reference's fp32 division), as RN32(RN64(x * RN64(1/d))).
// Proof: for significands a = sig(x), b = sig(d) in [1, 2) no quotient a/b is a float
// midpoint, and its relative distance to every midpoint exceeds 2^-49 (in the [1/2, 1) binade
// a - m*b is a non-zero multiple of 2^-48 for a midpoint m = (2k+1)*2^-25, so
// |a/b - m| >= 2^-48/b > 2^-49 * a/b; in [1, 2) it is a multiple of 2^-47 with m = (2k+1)*2^-24,
// so |a/b - m| > 2^-48 > 2^-49 * a/b).  The double product is within (1+2^-53)^2 - 1 < 2^-51
// of x/d (a correctly rounded double reciprocal, one double rounding), so it lies on the same
// side of every float midpoint as x/d and rounds to RN32(x/d) — also at the overflow
// threshold, which is the midpoint between FLT_MAX and 2^128.  Zero and denormal quotients
// (where the float rounding step is coarser) take the IEEE division.  The reciprocal is per
// output channel, so the compiler hoists it out of the element loops; per element: two
// conversions and one f64 multiply.
__device__ __forceinline__ float div_rn(float x, float d) {
  const double y = 1.0 / (double)d;
  float q = (float)((double)x * y);
  // +-0, +-denormal: the IEEE division, behind a wave-uniform branch (if-converted, its ~10
  // VALU ran for every output: conv0's epilogue spent 40 of its 245 VALU per tile there)
  const bool bad = __builtin_amdgcn_classf(q, 0x0F0);
  if (__builtin_amdgcn_ballot_w64(bad)) q = bad ? x / d : q;
  return q;
}

// exact three-way bf16 split of fp32 (the x3 conv's operands, gemm_x3_patch.h)
typedef unsigned short bf16_bits;
__device__ __forceinline__ unsigned short bf16_rn(float x) { return __builtin_bit_cast(unsigned short, (__bf16)x); }
__device__ __forceinline__ float bf16_f(unsigned short h) { return __builtin_bit_cast(float, (unsigned)h << 16); }
// x = bf16_f(s0) + bf16_f(s1) + bf16_f(s2) exactly for every finite x with |x| >= 2^-100 (below
// that the pieces' exponents leave the normal range and the tail is partly lost: <= 2^-124
// absolute).  Total over finite fp32: a finite |x| above the largest bf16 (0x1.fep127, where
// round-to-nearest would give inf and x - inf a NaN) takes the TRUNCATED top piece instead, and
// the remainder (< 2^-7 |x|, 16 bits) is still split exactly by the two lower pieces, so every
// finite operand the reference's cblas_sgemm takes (dnn_openblas.c:184-192) is represented
// exactly.  +-inf and NaN keep their bf16 value in the top piece with zero lower pieces (no
// NaN from inf - inf here); their products still meet the other operand's lower pieces, which
// are 0 for any weight exact in bf16, so a non-finite operand yields NaN where fp32 would give
// +-inf: outside the finite domain the x3 path claims.
__device__ __forceinline__ void split3(float x, unsigned short& s0, unsigned short& s1, unsigned short& s2) {
  const unsigned short r = bf16_rn(x);
  const bool fin = __builtin_isfinite(x);
  const bool ovf = fin && (r & 0x7fffu) == 0x7f80u;  // finite, rounded to +-inf
  s0 = ovf ? (unsigned short)(__builtin_bit_cast(unsigned, x) >> 16) : r;
  const float r1 = fin ? x - bf16_f(s0) : 0.f;
  s1 = bf16_rn(r1);
  s2 = bf16_rn(r1 - bf16_f(s1));
}

// split3 of two values at once, packed (value a in the low half of each word): the same pieces as
// split3 for every |x| below the bf16 rounding threshold 0x1.ffp127 (x3_split_ok), where the top
// piece is finite: one v_cvt_pk_bf16_f32 per piece for both values.  Callers check x3_split_ok
// for a whole wave's values and take split3 otherwise (a wave-uniform branch).
typedef float x3_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 x3_b2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned x3_cvt_pk(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((x3_f2){a, b}, x3_b2));
}
__device__ __forceinline__ bool x3_split_ok(float x) { return __builtin_fabsf(x) < 0x1.ffp127f; }  // false for NaN
__device__ __forceinline__ void split3_pair(float a, float b, unsigned& p0, unsigned& p1, unsigned& p2) {
  p0 = x3_cvt_pk(a, b);
  const float ra = a - __builtin_bit_cast(float, p0 << 16), rb = b - __builtin_bit_cast(float, p0 & 0xffff0000u);
  p1 = x3_cvt_pk(ra, rb);
  p2 = x3_cvt_pk(ra - __builtin_bit_cast(float, p1 << 16), rb - __builtin_bit_cast(float, p1 & 0xffff0000u));
}
// the three packed piece words of values (a, b): split3_pair when `fast` (wave-uniform), else split3
__device__ __forceinline__ void split3_pack2(bool fast, float a, float b, unsigned& p0, unsigned& p1, unsigned& p2) {
  if (fast) {
    split3_pair(a, b, p0, p1, p2);
  } else {
    unsigned short a0, a1, a2, b0, b1, b2;
    split3(a, a0, a1, a2);
    split3(b, b0, b1, b2);
    p0 = (unsigned)a0 | ((unsigned)b0 << 16);
    p1 = (unsigned)a1 | ((unsigned)b1 << 16);
    p2 = (unsigned)a2 | ((unsigned)b2 << 16);
  }
}

__device__ __forceinline__ float apply_epilogue(float v, float bias, float mean, float sq, float gamma,
                                                int flags) {
  if (flags & EPI_BIAS) v = v + bias;
  if (flags & EPI_BN) v = div_rn(v - mean, sq) * gamma;
  if (flags & EPI_BN_AB) v = v * mean - sq;
  if (flags & EPI_LEAKY_F64) v = v < 0.f ? (float)(0.1 * (double)v) : v;
  if (flags & EPI_LEAKY_F32) {
    float t = v * 0.1f;
    v = v > t ? v : t;
  }
  return v;
}

template <int MF>
struct Mfma;

// v_mfma_f32_32x32x2_f32: lane l supplies A[l&31][k=l>>5], B[k=l>>5][l&31];
// D[row][col]: col = l&31, row = (reg&3) + 8*(reg>>2) + 4*(l>>5).
template <>
struct Mfma<32> {
  typedef f32x16 acc_t;
  static constexpr int KG = 8;  // k covered by one 16-byte fragment read (2 lane halves x 4 steps)
  static constexpr int PARTS = 2;
  static constexpr int REGS = 16;
  __device__ static __forceinline__ acc_t op(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ int frag_row(int lane) { return lane & 31; }
  __device__ static __forceinline__ int frag_part(int lane) { return lane >> 5; }
  __device__ static __forceinline__ int out_row(int lane, int reg) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }
  __device__ static __forceinline__ int out_col(int lane) { return lane & 31; }
};

// v_mfma_f32_16x16x4_f32: lane l supplies A[l&15][k=l>>4], B[k=l>>4][l&15];
// D[row][col]: col = l&15, row = 4*(l>>4) + reg.
template <>
struct Mfma<16> {
  typedef f32x4 acc_t;
  static constexpr int KG = 16;  // 4 lane quarters x 4 steps
  static constexpr int PARTS = 4;
  static constexpr int REGS = 4;
  __device__ static __forceinline__ acc_t op(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ int frag_row(int lane) { return lane & 15; }
  __device__ static __forceinline__ int frag_part(int lane) { return lane >> 4; }
  __device__ static __forceinline__ int out_row(int lane, int reg) { return 4 * (lane >> 4) + reg; }
  __device__ static __forceinline__ int out_col(int lane) { return lane & 15; }
};

// XCD-aware bijective block remap: the 8 XCDs each get a contiguous range of tiles, so the
// N tiles of one A row-panel run under one L2 (cdna_hip_programming.md T1).
__device__ __forceinline__ int xcd_tile(int bid, int nb) {
  const int xcd = bid & 7, q = nb >> 3, rr = nb & 7;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
}

// n / d for 0 <= n < 2^31 without a division (round-up magic numbers from the launcher,
// implicit_conv_magic).  The 32-bit sum cannot wrap: umulhi(n, mag) <= n < 2^31.
__device__ __forceinline__ int div_magic(int n, unsigned mag, int sh) {
  return (int)((__umulhi((unsigned)n, mag) + (unsigned)n) >> sh);
}

// Row m of an implicit-GEMM A operand -> image b and the input pixel (iy0, ix0) under its
// window's top-left tap; returns the bitmask of the taps inside the frame (0 for a row past M
// or past a ragged pool edge).  MODE 1: m is the output pixel (b, oy, ox); MODE 2: m = 4 *
// window + 2 * dy + dx over the pooled output's (b, py, px) windows.
template <int MODE>
__device__ __forceinline__ int implicit_row(const ImplicitConv& ic, int m, int M, int& b, int& iy0, int& ix0) {
  int oy, ox;
  bool rv = m < M;
  if constexpr (MODE == 2) {
    const int w = m >> 2, t = div_magic(w, ic.mag_pw, ic.sh_pw);
    b = div_magic(t, ic.mag_ph, ic.sh_ph);
    oy = 2 * (t - b * ic.PH) + ((m >> 1) & 1);
    ox = 2 * (w - t * ic.PW) + (m & 1);
    rv = rv && oy < ic.OH && ox < ic.OW;
  } else {
    const int t = div_magic(m, ic.mag_ow, ic.sh_ow);
    b = div_magic(t, ic.mag_oh, ic.sh_oh);
    oy = t - b * ic.OH;
    ox = m - t * ic.OW;
  }
  iy0 = oy * ic.sh - ic.pt;
  ix0 = ox * ic.sw - ic.pl;
  if (!rv) return 0;
  // in-frame taps = (window rows inside the frame) x (window columns inside the frame)
  int ym = 0, xm = 0;
  for (int d = 0; d < ic.kh; ++d) ym |= ((unsigned)(iy0 + d) < (unsigned)ic.H ? 1 : 0) << d;
  for (int d = 0; d < ic.kw; ++d) xm |= ((unsigned)(ix0 + d) < (unsigned)ic.W ? 1 : 0) << d;
  int mk = 0;
  for (int d = 0; d < ic.kh; ++d) mk |= ((ym >> d) & 1) ? xm << (d * ic.kw) : 0;
  return mk;
}

// Fused epilogue + store of one wave's accumulators (NHWC: row = pixel, col = channel).
template <int MF, int TM, int TN, int WTM, int WTN, typename OutT = float>
__device__ __forceinline__ void store_tile(const typename Mfma<MF>::acc_t (&acc)[TM][TN], OutT* __restrict__ C,
                                           int ldc, int M, int N, int m0, int n0, int wm, int wn, int lane,
                                           const EpiParams& epi) {
  typedef Mfma<MF> MM;
  const int oc = MM::out_col(lane);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WTN + j * MF + oc;
    const float pb = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
    const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
    const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
    const float pg = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;
    if (n < N) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < MM::REGS; ++r) {
          const int m = m0 + wm * WTM + i * MF + MM::out_row(lane, r);
          if (m < M) store_out(C + (size_t)m * ldc + n, apply_epilogue(acc[i][j][r], pb, pm, ps, pg, epi.flags));
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Register-staged double buffer.  K permutation: inside a KG-wide group, lane part p reads
// k = KG*g + 4p + (0..3) with one ds_read_b128 and feeds them to 4 consecutive MFMAs. A and
// B use the same mapping, so the reduction still covers every k exactly once.
template <int BM, int BN, int BK, int WM, int WN, int MF>
__global__ void __launch_bounds__(WM* WN * 64)
gemm_f32_mfma_kernel(const float* __restrict__ A, int lda, const float* __restrict__ Bt, int ldb,
                     float* __restrict__ C, int ldc, int M, int N, int K, EpiParams epi, int tilesN) {
  typedef Mfma<MF> MM;
  typedef typename MM::acc_t acc_t;
  constexpr int T = WM * WN * 64;
  constexpr int LS = BK + 4;  // LDS row stride (floats): breaks the power-of-two bank aliasing
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / MF, TN = WTN / MF;
  constexpr int KQ = BK / 4;
  constexpr int A_V4 = BM * KQ, B_V4 = BN * KQ;
  constexpr int A_LD = (A_V4 + T - 1) / T, B_LD = (B_V4 + T - 1) / T;
  static_assert(BK % MM::KG == 0, "BK must be a multiple of the fragment group");
  static_assert(WTM % MF == 0 && WTN % MF == 0, "wave tile must be a multiple of the MFMA tile");

  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LS];

  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int tm_ = tile / tilesN, tn_ = tile - tm_ * tilesN;
  const int m0 = tm_ * BM, n0 = tn_ * BN;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;

  f32x4 ra[A_LD], rb[B_LD];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      int idx = tid + i * T;
      if (A_V4 % T == 0 || idx < A_V4) {
        int row = idx / KQ, c4 = idx - (idx / KQ) * KQ;
        int gm = m0 + row;
        gm = gm < M ? gm : M - 1;
        ra[i] = *reinterpret_cast<const f32x4*>(A + (size_t)gm * lda + k0 + c4 * 4);
      }
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      int idx = tid + i * T;
      if (B_V4 % T == 0 || idx < B_V4) {
        int row = idx / KQ, c4 = idx - (idx / KQ) * KQ;
        rb[i] = *reinterpret_cast<const f32x4*>(Bt + (size_t)(n0 + row) * ldb + k0 + c4 * 4);
      }
    }
  };
  auto sstore = [&](float* As, float* Bs) {
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      int idx = tid + i * T;
      if (A_V4 % T == 0 || idx < A_V4) {
        int row = idx / KQ, c4 = idx - (idx / KQ) * KQ;
        *reinterpret_cast<f32x4*>(As + row * LS + c4 * 4) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      int idx = tid + i * T;
      if (B_V4 % T == 0 || idx < B_V4) {
        int row = idx / KQ, c4 = idx - (idx / KQ) * KQ;
        *reinterpret_cast<f32x4*>(Bs + row * LS + c4 * 4) = rb[i];
      }
    }
  };

  acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < MM::REGS; ++r) acc[i][j][r] = 0.f;

  const int fr = MM::frag_row(lane), fk = 4 * MM::frag_part(lane);
  const int a_base = (wm * WTM + fr) * LS + fk;
  const int b_base = (wn * WTN + fr) * LS + fk;

  const int nk = K / BK;
  gload(0);
  sstore(smem, smem + BM * LS);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    float* As = smem + (kt & 1) * (BM + BN) * LS;
    float* Bs = As + BM * LS;
    if (kt + 1 < nk) gload((kt + 1) * BK);
#pragma unroll
    for (int g = 0; g < BK / MM::KG; ++g) {
      f32x4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const f32x4*>(As + a_base + i * MF * LS + g * MM::KG);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bf[j] = *reinterpret_cast<const f32x4*>(Bs + b_base + j * MF * LS + g * MM::KG);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = MM::op(af[i][s], bf[j][s], acc[i][j]);
    }
    if (kt + 1 < nk) {
      float* Asn = smem + ((kt + 1) & 1) * (BM + BN) * LS;
      sstore(Asn, Asn + BM * LS);
    }
    __syncthreads();
  }
  store_tile<MF, TM, TN, WTM, WTN>(acc, C, ldc, M, N, m0, n0, wm, wn, lane, epi);
}

// ---------------------------------------------------------------------------------------
// LDS-DMA ring.  BK = 32: one tile row is 128 B = 8 slots of 16 B, one wave instruction of
// global_load_lds_dwordx4 fills one 1-KiB chunk = 8 rows (lane l -> row l/8, slot l%8).
// Slot swizzle: physical slot = logical slot ^ ((row >> 1) & 7).  It is applied to the
// per-lane SOURCE address (the DMA destination is lane-linear) and to the fragment read
// address; every 16-lane group of a ds_read_b128 then hits 16 distinct 16-B bank slots for
// both the 32x32x2 (rows l&31, parts l>>5) and 16x16x4 (rows l&15, parts l>>4) fragments.
//
// Pipeline per K-step kt (NS stages in the ring, counted waits, raw barriers):
//   s_waitcnt vmcnt(#chunks of the stages issued after kt)   -> stage kt landed (own DMAs)
//   s_barrier                                                 -> everyone's DMAs landed, and
//                                                                everyone finished reading kt-1
//   issue stage kt+NS-1 into the slot of kt-1
//   ds_read + MFMA on stage kt
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void raw_barrier() { __builtin_amdgcn_s_barrier(); }
__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
// one global_load_lds_dwordx4: 16 B per lane from `src` (per lane) into `dst` + 16*lane
// (`dst` wave-uniform)
__device__ __forceinline__ void lds_dma16(const float* src, float* dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// Stores whose instruction count per wave is fixed (persistent kernels that wait for their
// next tile's LDS-DMA with a counted vmcnt while their own stores are still in flight: the
// count is only exact if no store is ever branched around).  A buffer resource over the
// output drops a lane whose byte offset is out of range (OOB_OFF) instead of faulting, so
// the store is always issued.  Offsets are 32-bit: the launcher checks the output size.
constexpr unsigned OOB_OFF = 0x80000000u;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
}
// Cache policy of the layers' output stores (aux of the buffer stores): 16 = sc1, write-through, so a
// layer leaves no dirty L2 lines for the kernel boundary to write back (MI355X_MICROARCH: a
// dependent boundary costs + B / 6 TB/s for B dirty bytes); 0 = the default write-back policy.
#ifndef DNN_EPI_STORE_AUX
#define DNN_EPI_STORE_AUX 16
#endif
__device__ __forceinline__ void store16(__amdgpu_buffer_rsrc_t r, unsigned off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, DNN_EPI_STORE_AUX);
}
// a 16-B output store at byte offset `off` (< 2^31, checked by the launchers) from a uniform base
__device__ __forceinline__ void store16_at(const void* base, size_t off, u32x4 v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, (unsigned)off, 0, DNN_EPI_STORE_AUX);
}
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void store8_at(const void* base, size_t off, u32x2 v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b64(v, rs, (unsigned)off, 0, DNN_EPI_STORE_AUX);
}
__device__ __forceinline__ void store4_at(const void* base, size_t off, float v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rs, (unsigned)off, 0, DNN_EPI_STORE_AUX);
}
__device__ __forceinline__ void store4(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, 0);
}

// 4-B LDS-DMA (global_load_lds_dword) issued from inline asm: the compiler's wait pass does
// not see it, so it does not put a conservative vmcnt(0) before every later LDS read (it
// cannot tell a double buffer's halves apart).  The caller orders it with its own counted
// vmcnt + barrier.  `dst` must be wave-uniform; lane l writes dst + 4*l.
__device__ __forceinline__ void lds_dma4_opaque(const float* src, const float* dst) {
  const unsigned m0v =
      __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)dst);
  unsigned saved;  // M0 is a reserved register: restore it rather than clobber it
  // (s_nop 0: the wait state between the M0 write and the LDS-DMA that reads it)
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(saved)
               : "v"(src), "s"(m0v)
               : "memory");
}

// max (or min, for a channel whose epilogue is non-increasing) of a pool window's raw conv
// outputs, then the epilogue once.  The epilogue f = leaky(((v + b) - mean) / sq * gamma) is a
// chain of IEEE-rounded monotone steps (sq > 0): non-decreasing for gamma >= 0, non-increasing
// for gamma < 0 (alpha < 0 for the avx alpha/beta form).  So max_i f(v_i) == f(max_i v_i)
// (resp. f(min_i v_i)) value for value: the reference's epilogue-then-pool result
// (dnn_openblas.c:220-254) with one epilogue per pooled output instead of four.
// the epilogue with the flag set known at compile time (FL >= 0; FL < 0: the runtime `flags`)
template <int FL>
__device__ __forceinline__ float apply_epilogue_t(float v, float bias, float mean, float sq, float gamma, int flags) {
  if constexpr (FL < 0) {
    return apply_epilogue(v, bias, mean, sq, gamma, flags);
  } else {
    if constexpr ((FL & EPI_BIAS) != 0) v = v + bias;
    if constexpr ((FL & EPI_BN) != 0) v = div_rn(v - mean, sq) * gamma;
    if constexpr ((FL & EPI_BN_AB) != 0) v = v * mean - sq;
    if constexpr ((FL & EPI_LEAKY_F64) != 0) v = v < 0.f ? (float)(0.1 * (double)v) : v;
    if constexpr ((FL & EPI_LEAKY_F32) != 0) {
      const float t = v * 0.1f;
      v = v > t ? v : t;
    }
    return v;
  }
}
template <int FL>
__device__ __forceinline__ float pool_then_epilogue_t(f32x4 v, float pb, float pm, float ps, float pg, int flags) {
  const int f = FL < 0 ? flags : FL;
  const bool dec = ((f & EPI_BN) && pg < 0.f) || ((f & EPI_BN_AB) && pm < 0.f);
  const float hi = __builtin_fmaxf(__builtin_fmaxf(v[0], v[1]), __builtin_fmaxf(v[2], v[3]));
  const float lo = __builtin_fminf(__builtin_fminf(v[0], v[1]), __builtin_fminf(v[2], v[3]));
  return apply_epilogue_t<FL>(dec ? lo : hi, pb, pm, ps, pg, flags);
}

// The epilogue of NV x NC values (NC columns, their parameters per column) in place, with ONE
// wave-uniform check for all of their divisions: div_rn's fallback branch per value made every
// value's chain a basic block of its own (a conv2 tile's 14 pooled values per lane took 4.2 k
// cycles, tile2 stamps).  Same operations per value as apply_epilogue_t, so the same bits.
template <int FL, int NV, int NC>
__device__ __forceinline__ void epilogue_batch(float (&v)[NV][NC], const float (&pb)[NC], const float (&pm)[NC],
                                               const float (&ps)[NC], const float (&pg)[NC], int flags) {
  if constexpr (FL < 0 || (FL & EPI_BN) == 0) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < NV; ++i) v[i][c] = apply_epilogue_t<FL>(v[i][c], pb[c], pm[c], ps[c], pg[c], flags);
  } else {
    float x[NV][NC];
    bool bad = false;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const double y = 1.0 / (double)ps[c];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        float t = v[i][c];
        if constexpr ((FL & EPI_BIAS) != 0) t = t + pb[c];
        x[i][c] = t - pm[c];
        v[i][c] = (float)((double)x[i][c] * y);
        bad = bad || __builtin_amdgcn_classf(v[i][c], 0x0F0);
      }
    }
    if (__builtin_amdgcn_ballot_w64(bad)) {  // +-0, +-denormal quotients: the IEEE division
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int i = 0; i < NV; ++i)
          if (__builtin_amdgcn_classf(v[i][c], 0x0F0)) v[i][c] = x[i][c] / ps[c];
    }
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        float t = v[i][c] * pg[c];
        if constexpr ((FL & EPI_BN_AB) != 0) t = t * pm[c] - ps[c];
        if constexpr ((FL & EPI_LEAKY_F64) != 0) t = t < 0.f ? (float)(0.1 * (double)t) : t;
        if constexpr ((FL & EPI_LEAKY_F32) != 0) {
          const float u = t * 0.1f;
          t = t > u ? t : u;
        }
        v[i][c] = t;
      }
  }
}

// pool_then_epilogue_t over NV windows x NC columns (the window's max, or min for a decreasing
// channel, then epilogue_batch); put(i, c, value)
template <int FL, int NV, int NC, typename F>
__device__ __forceinline__ void pool_epilogue_batch(const f32x4 (&acc)[NV][NC], const float (&pb)[NC],
                                                    const float (&pm)[NC], const float (&ps)[NC],
                                                    const float (&pg)[NC], int flags, F&& put) {
  float t[NV][NC];
  const int f = FL < 0 ? flags : FL;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const bool dec = ((f & EPI_BN) && pg[c] < 0.f) || ((f & EPI_BN_AB) && pm[c] < 0.f);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const f32x4 v = acc[i][c];
      const float hi = __builtin_fmaxf(__builtin_fmaxf(v[0], v[1]), __builtin_fmaxf(v[2], v[3]));
      const float lo = __builtin_fminf(__builtin_fminf(v[0], v[1]), __builtin_fminf(v[2], v[3]));
      t[i][c] = dec ? lo : hi;
    }
  }
  epilogue_batch<FL>(t, pb, pm, ps, pg, flags);
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < NV; ++i) put(i, c, t[i][c]);
}

__device__ __forceinline__ float pool_then_epilogue(f32x4 v, float pb, float pm, float ps, float pg, int flags) {
  const bool dec = ((flags & EPI_BN) && pg < 0.f) || ((flags & EPI_BN_AB) && pm < 0.f);
  const float hi = __builtin_fmaxf(__builtin_fmaxf(v[0], v[1]), __builtin_fmaxf(v[2], v[3]));
  const float lo = __builtin_fminf(__builtin_fminf(v[0], v[1]), __builtin_fminf(v[2], v[3]));
  return apply_epilogue(dec ? lo : hi, pb, pm, ps, pg, flags);
}

// Pool-fused store (implicit mode with pool): rows are pool-window-major, 4 rows per 2x2
// window, and both MFMA layouts keep a window's 4 rows in 4 consecutive registers of one
// lane (32x32x2: regs 4q..4q+3 = rows 8q+4h+0..3; 16x16x4: regs 0..3 = rows 4(l>>4)+0..3).
// Window cells past the conv output (odd OH/OW: the SAME pool's padding, -FLT_MAX in the
// reference) are left out by repeating cell (0,0), which always exists.
template <int MF, int TM, int TN, int WTM, int WTN, typename OutT = float>
__device__ __forceinline__ void store_tile_pool(const typename Mfma<MF>::acc_t (&acc)[TM][TN],
                                                OutT* __restrict__ C, int ldc, int M, int N, int m0, int n0,
                                                int wm, int wn, int lane, const EpiParams& epi,
                                                const ImplicitConv& ic) {
  typedef Mfma<MF> MM;
  const int oc = MM::out_col(lane);
  const int nwin = M >> 2;
  const bool ragged = ((ic.OH | ic.OW) & 1) != 0;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WTN + j * MF + oc;
    const float pb = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
    const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
    const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
    const float pg = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;
    if (n >= N) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int q = 0; q < MM::REGS / 4; ++q) {
        const int win = (m0 + wm * WTM + i * MF + MM::out_row(lane, 4 * q)) >> 2;
        if (win >= nwin) continue;
        f32x4 v = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        if (ragged) {
          const int px = win % ic.PW, py = (win / ic.PW) % ic.PH;
          const bool x1 = 2 * px + 1 < ic.OW, y1 = 2 * py + 1 < ic.OH;
          if (!x1) v[1] = v[0];
          if (!y1) v[2] = v[0];
          if (!(x1 && y1)) v[3] = v[0];
        }
        const float val = pool_then_epilogue(v, pb, pm, ps, pg, epi.flags);
        if constexpr (std::is_same<OutT, float>::value) {
          if (epi.flags & EPI_OUT_X3) {  // pooled pixel -> interior row of the zero-bordered planes
            const int q1 = div_magic(win, ic.mag_pw, ic.sh_pw), px = win - q1 * ic.PW;  // no division
            const int b = div_magic(q1, ic.mag_ph, ic.sh_ph), py = q1 - b * ic.PH;
            const size_t row = ((size_t)b * (ic.PH + 2) + py + 1) * (ic.PW + 2) + px + 1;
            unsigned short s0, s1, s2;
            split3(val, s0, s1, s2);
            bf16_bits* d = reinterpret_cast<bf16_bits*>(C) + row * (3 * (size_t)N) + (n >> 5) * 96 + (n & 31);
            d[0] = s0;
            d[32] = s1;
            d[64] = s2;
            continue;
          }
        }
        store_out(C + (size_t)win * ldc + n, val);
      }
    }
  }
}

// Split-K: with sk.steps > 0 the grid is sk.splits x (tilesM x tilesN); workgroup split s
// covers K-steps [s*steps, (s+1)*steps) and stores its raw fp32 partial tile (no epilogue) to
// C + s*sk.slab; splitk_reduce_kernel then sums the partials in split order and applies the
// epilogue.  The split is chosen from (N, K) only, so summation order stays independent of M.
struct SplitK {
  int steps;         // K-steps (of 32) per split; 0 = no split
  int ntile;         // tilesM * tilesN
  long long slab;    // floats between consecutive split partials
  // fused combine (tickets != nullptr, fp32 LDS-DMA kernel): every split stores its raw tile
  // in the accumulator-native layout, the LAST split of a tile to arrive (agent-scope ticket)
  // sums all partials in split order and runs the epilogue into `out` (splitk_combine)
  unsigned* tickets = nullptr;
  float* out = nullptr;  // OutT* of the kernel (fp16 activations on the fp16 path)
  int ldo = 0;
  int flags = 0;     // epilogue of the final output
  int splits = 1;
  int nmajor = 0;    // tile -> (tm, tn) N-major: an XCD's contiguous tile range shares one N panel
};

// tile index -> (M tile, N tile): M-major (consecutive tiles walk N) or N-major (an XCD's
// contiguous range of tiles shares one weight panel, which then stays in its L2)
__device__ __forceinline__ int2 tile_coords(int tile, int tilesN, const SplitK& sk) {  // (tm, tn), by value:
  // results through references made the compiler spill them to scratch
  const int tilesM = sk.ntile / tilesN;
  const int a = sk.nmajor ? tile / tilesM : tile / tilesN;
  return sk.nmajor ? make_int2(tile - a * tilesM, a) : make_int2(a, tile - a * tilesN);
}

// Sum of the split-K partials in split order, ((p0 + p1) + p2) ..., then the fused epilogue.
// part: [splits][M][N] (slab floats apart), C: [M][ldc].  HBM-bound: (splits + 1) * M * N * 4 B.
// Thread layout (no per-element index division): a block row of nqb threads covers channel
// quads q0, q0 + nqb, ... (epilogue parameters loaded once per quad); the block's rp rows
// stride over M.
template <typename OutT>
static __global__ void __launch_bounds__(256) __attribute__((unused))
splitk_reduce_kernel(const float* __restrict__ part, int splits, long long slab, OutT* __restrict__ C, int M,
                     int N, int ldc, EpiParams epi, int nqb, int rp) {
  const int nq = N >> 2;  // N % 4 == 0 (checked by the launcher)
  const int q0 = threadIdx.x % nqb, r = threadIdx.x / nqb;
  if (r >= rp) return;
  for (int q = q0; q < nq; q += nqb) {
    const int n = 4 * q;
    f32x4 pb = {0.f, 0.f, 0.f, 0.f}, pm = {0.f, 0.f, 0.f, 0.f}, ps = {1.f, 1.f, 1.f, 1.f}, pg = {1.f, 1.f, 1.f, 1.f};
    if (epi.flags & EPI_BIAS) pb = *reinterpret_cast<const f32x4*>(epi.bias + n);
    if (epi.flags & (EPI_BN | EPI_BN_AB)) {
      pm = *reinterpret_cast<const f32x4*>(epi.mean + n);
      ps = *reinterpret_cast<const f32x4*>(epi.sq + n);
    }
    if (epi.flags & EPI_BN) pg = *reinterpret_cast<const f32x4*>(epi.gamma + n);
    for (int m = blockIdx.x * rp + r; m < M; m += gridDim.x * rp) {
      const float* p = part + (size_t)m * N + n;
      f32x4 v = *reinterpret_cast<const f32x4*>(p);
      for (int s = 1; s < splits; ++s) v = v + *reinterpret_cast<const f32x4*>(p + s * slab);
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = apply_epilogue(v[e], pb[e], pm[e], ps[e], pg[e], epi.flags);
      if constexpr (sizeof(OutT) == 4) {
        *reinterpret_cast<f32x4*>(C + (size_t)m * ldc + n) = o;
      } else {  // 4 fp16 = one 8-byte store
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<h4*>(C + (size_t)m * ldc + n) = h4{(half_t)o[0], (half_t)o[1], (half_t)o[2], (half_t)o[3]};
      }
    }
  }
}

// Fused split-K combine (Guideline 16 R1 hand-off, cdna_hip_programming.md §6): each split's
// workgroup stores its raw partial tile write-through (sc1, 16-B stores in the accumulator-native
// layout: lane-contiguous f32x4 of 4 consecutive rows, so no bounds checks and full 1-KiB wave
// stores), every wave drains (vmcnt 0), the workgroup barrier, then ONE lane adds to the tile's
// agent-scope ticket.  The workgroup whose add returns splits-1 is the last: one agent acquire
// (+ vmcnt 0 + barrier), then plain loads of the other partials, summed in split order
// ((p0 + p1) + p2 ..., the separate reduce kernel's order, so the same bits) with its own
// partial taken from registers, the epilogue, and the row-major store.  It re-arms the ticket
// (0) for the next launch.  Partial tile (split s, tile t) starts at slab + (s*ntile + t)*BM*BN.
template <int SPL, int MF, int TM, int TN, int WTM, int WTN, int NW, typename OutT = float>
__device__ __forceinline__ void splitk_combine(typename Mfma<MF>::acc_t (&acc)[TM][TN], float* __restrict__ slab,
                                               const SplitK& sk, int s, int tile, int M, int N, int m0, int n0,
                                               int wm, int wn, int wid, int lane, const EpiParams& epi0,
                                               unsigned* lds_word) {
  typedef Mfma<MF> MM;
  constexpr int Q = MM::REGS / 4;
  constexpr long long TILE_F = (long long)NW * TM * TN * Q * 256;  // = BM * BN
  const unsigned slab_bytes = (unsigned)((long long)SPL * sk.ntile * TILE_F * 4);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(slab, 0, (int)slab_bytes, 0x00020000);
  auto idx = [&](int i, int j, int q) { return ((((wid * TM + i) * TN + j) * Q + q) * 64 + lane) * 4; };
  const long long own = ((long long)s * sk.ntile + tile) * TILE_F;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const f32x4 v = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs,
                                               (unsigned)((own + idx(i, j, q)) * 4), 0, 16 /* sc1 */);
      }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(sk.tickets + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned last = t == (unsigned)(SPL - 1) ? 1u : 0u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(sk.tickets + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *lds_word = last;
  }
  __syncthreads();
  if (!*lds_word) return;

  EpiParams epi = epi0;
  epi.flags = sk.flags;
  const int oc = MM::out_col(lane);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WTN + j * MF + oc;
    const bool nok = n < N;
    const float pb = (nok && (epi.flags & EPI_BIAS)) ? epi.bias[n] : 0.f;
    const float pm = (nok && (epi.flags & (EPI_BN | EPI_BN_AB))) ? epi.mean[n] : 0.f;
    const float ps = (nok && (epi.flags & (EPI_BN | EPI_BN_AB))) ? epi.sq[n] : 1.f;
    const float pg = (nok && (epi.flags & EPI_BN)) ? epi.gamma[n] : 1.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      // all partials of this (i, j) in flight at once, then the ordered sums
      f32x4 part[SPL][Q];
#pragma unroll
      for (int ss = 0; ss < SPL; ++ss)
#pragma unroll
        for (int q = 0; q < Q; ++q)
          part[ss][q] = ss == s ? f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]}
                                : *reinterpret_cast<const f32x4*>(slab + ((long long)ss * sk.ntile + tile) * TILE_F +
                                                                  idx(i, j, q));
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        f32x4 v = part[0][q];
#pragma unroll
        for (int ss = 1; ss < SPL; ++ss) v = v + part[ss][q];
        if (!nok) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = m0 + wm * WTM + i * MF + MM::out_row(lane, 4 * q + e);
          if (m < M)
            store_out(reinterpret_cast<OutT*>(sk.out) + (size_t)m * sk.ldo + n,
                      apply_epilogue(v[e], pb, pm, ps, pg, epi.flags));
        }
      }
    }
  }
}

// Fused split-K combine for any split count (latency plans: 2..32 splits of a small-M layer)
// and for the pool-fused mode: the same hand-off as splitk_combine (write-through raw partial
// in the accumulator-native layout, drain, barrier, agent-scope ticket, acquire by the last
// split), but the last split only SUMS the partials in split order ((p0 + p1) + p2) + ... into
// its own accumulators and returns true; the caller then runs its normal store path (plain or
// pool-then-epilogue) with the real epilogue.  Returns false in every other split.
template <int MF, int TM, int TN, int NW>
__device__ __forceinline__ bool splitk_sum(typename Mfma<MF>::acc_t (&acc)[TM][TN], float* __restrict__ slab,
                                           const SplitK& sk, int s, int tile, int wid, int lane, unsigned* lds_word) {
  typedef Mfma<MF> MM;
  constexpr int Q = MM::REGS / 4;
  constexpr long long TILE_F = (long long)NW * TM * TN * Q * 256;  // = BM * BN
  const int S = sk.splits;
  const unsigned slab_bytes = (unsigned)((long long)S * sk.ntile * TILE_F * 4);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(slab, 0, (int)slab_bytes, 0x00020000);
  auto idx = [&](int i, int j, int q) { return ((((wid * TM + i) * TN + j) * Q + q) * 64 + lane) * 4; };
  const long long own = ((long long)s * sk.ntile + tile) * TILE_F;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const f32x4 v = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs,
                                               (unsigned)((own + idx(i, j, q)) * 4), 0, 16 /* sc1 */);
      }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(sk.tickets + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned last = t == (unsigned)(S - 1) ? 1u : 0u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(sk.tickets + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *lds_word = last;
  }
  __syncthreads();
  if (!*lds_word) return false;
  // partials of up to 4 splits in flight at once (uniform branches, no wait between the
  // loads), then added in split order
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      f32x4 own_v[Q], v[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q)
        own_v[q] = f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
      for (int s0 = 0; s0 < S; s0 += 4) {
        f32x4 p[4][Q];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int ss = s0 + u;
          if (ss < S && ss != s) {
            const float* src = slab + ((long long)ss * sk.ntile + tile) * TILE_F;
#pragma unroll
            for (int q = 0; q < Q; ++q) p[u][q] = *reinterpret_cast<const f32x4*>(src + idx(i, j, q));
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int ss = s0 + u;
          if (ss < S) {
#pragma unroll
            for (int q = 0; q < Q; ++q) {
              const f32x4 x = ss == s ? own_v[q] : p[u][q];
              v[q] = ss == 0 ? x : v[q] + x;
            }
          }
        }
      }
#pragma unroll
      for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][j][4 * q + e] = v[q][e];
    }
  return true;
}

// Buffer-resource addressing of the LDS-DMA sources (ABUF kernels): A and Bt are read by
// buffer_load ... lds with a per-lane 32-bit byte offset fixed for the whole tile (voffset) and
// the K-step's position as a wave-uniform soffset, so a DMA costs no 64-bit address arithmetic;
// a padding tap is a voffset past the descriptor's range (OOB_OFF), which the hardware turns
// into zeros in LDS (no zero page).  For the implicit modes the A descriptor starts (W+1)*C
// floats BEFORE the input, so every in-frame (pixel, tap) offset is non-negative.  The
// launcher picks ABUF only when both descriptors fit 2^31 bytes.
struct BufDesc {
  const float* a;   // descriptor base of A (implicit: input - (W+1)*C)
  unsigned a_bytes;
  unsigned b_bytes; // Bt: Npad * ldb * 4
};
__device__ __forceinline__ void lds_dma16_buf(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff, float* dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16, (int)voff, (int)soff,
                                           0, 0);
}

// MODE 0: dense A (col buffer or 1x1 input), MODE 1: implicit conv, MODE 2: implicit + pool.
// GEN: the any-split / pool-split combine (latency plans) compiled in; a separate
// instantiation, since its registers would cost the batch configs their occupancy
template <int BM, int BN, int WM, int WN, int MF, int NS, int MODE, bool ABUF = false, bool GEN = false>
__global__ void __launch_bounds__(WM* WN * 64)
gemm_f32_glds_kernel(const float* __restrict__ A, int lda, const float* __restrict__ Bt, int ldb,
                     float* __restrict__ C, int ldc, int M, int N, int K, EpiParams epi, int tilesN,
                     ImplicitConv ic, SplitK sk, BufDesc bd) {
  typedef Mfma<MF> MM;
  typedef typename MM::acc_t acc_t;
  constexpr int BK = 32;
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / MF, TN = WTN / MF;
  constexpr int A_CH = BM / 8, B_CH = BN / 8;
  constexpr int LPSA = A_CH / NW, LPSB = B_CH / NW, LPS = LPSA + LPSB;  // DMAs per wave per stage
  constexpr int STAGE = (BM + BN) * BK;                                  // floats per stage
  static_assert(A_CH % NW == 0 && B_CH % NW == 0, "chunks must split evenly over the waves");
  static_assert(NS >= 2 && NS <= 4, "ring depth");
  static_assert(WTM % MF == 0 && WTN % MF == 0, "wave tile must be a multiple of the MFMA tile");

  __shared__ __attribute__((aligned(1024))) float smem[NS * STAGE];

  int tile = xcd_tile(blockIdx.x, gridDim.x);
  int kbeg = 0;  // first k of this workgroup's K range
  int split = 0;
  if (sk.steps > 0) {
    split = tile / sk.ntile;
    tile -= split * sk.ntile;
    kbeg = split * sk.steps * BK;
    K = sk.steps * BK;
    if (!sk.tickets) C += split * sk.slab;
    epi.flags = 0;  // raw partial sums; the reduce kernel / the combine applies the epilogue
  }
  const int2 tc = tile_coords(tile, tilesN, sk);
  const int m0 = tc.x * BM, n0 = tc.y * BN;
  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;

  // ---- A sources.  Chunk c (8 rows) of this wave: c = wid + i*NW; lane -> row 8c + lane/8,
  // logical 16-B slot ls = (lane&7) ^ ((row>>1)&7) (the source side of the LDS swizzle).
  const float* srcA[LPSA];  // dense: row pointer + slot (advanced by k0); implicit: pixel base
  unsigned voA[LPSA];       // ABUF: byte offset of the same (dense: + slot; implicit: + slot, shifted base)
  int maskA[LPSA], lsA[LPSA];
#pragma unroll
  for (int i = 0; i < LPSA; ++i) {
    const int r = 8 * (wid + i * NW) + (lane >> 3);
    const int ls = (lane & 7) ^ ((r >> 1) & 7);
    lsA[i] = 4 * ls;
    const int m = m0 + r;
    if constexpr (MODE == 0) {
      const int gm = m < M ? m : M - 1;
      if constexpr (ABUF)
        voA[i] = (unsigned)(((size_t)gm * lda + 4 * ls) * 4);
      else
        srcA[i] = A + (size_t)gm * lda + kbeg + 4 * ls;
      maskA[i] = 0;
    } else {
      int b, iy0, ix0;
      maskA[i] = implicit_row<MODE>(ic, m, M, b, iy0, ix0);
      if constexpr (ABUF)
        voA[i] = (unsigned)(((((long long)b * ic.H + iy0) * ic.W + ix0 + ic.W + 1) * ic.C + 4 * ls) * 4);
      else
        srcA[i] = A + (((long long)b * ic.H + iy0) * ic.W + ix0) * (long long)ic.C;
    }
  }
  const float* srcB[LPSB];
  unsigned voB[LPSB];
#pragma unroll
  for (int j = 0; j < LPSB; ++j) {
    const int r = 8 * (wid + j * NW) + (lane >> 3);
    const int ls = (lane & 7) ^ ((r >> 1) & 7);
    if constexpr (ABUF)
      voB[j] = (unsigned)(((size_t)(n0 + r) * ldb + 4 * ls) * 4);
    else
      srcB[j] = Bt + (size_t)(n0 + r) * ldb + kbeg + 4 * ls;
  }
  // (built unconditionally: unused, and dropped, in the flat-address instantiation)
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)bd.a, 0, (int)bd.a_bytes, 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)bd.b_bytes, 0x00020000);

  // implicit mode: wave-uniform position of the next K-step to issue, k = tap*C + c
  int cb = 0, tapb = 0, dyb = 0, dxb = 0, dyn = 0, dxn = 1;
  if constexpr (MODE != 0) {
    tapb = kbeg / ic.C;
    cb = kbeg - tapb * ic.C;
    dyb = tapb / ic.kw;
    dxb = tapb - dyb * ic.kw;
    dyn = dxb + 1 == ic.kw ? dyb + 1 : dyb;
    dxn = dxb + 1 == ic.kw ? 0 : dxb + 1;
  }
  const long long rowstride = (long long)ic.W * ic.C;

  const bool aligned = MODE != 0 && (ic.C % BK) == 0;  // wave-uniform
  auto issue = [&](int stage, int k0) {
    float* base = smem + stage * STAGE;
    if constexpr (ABUF) {
      // MODE 0: every lane at its row's k0; implicit (C % 32 == 0 only): one tap per K-step, the
      // tap + channel offset uniform in soffset, the tap mask choosing voffset or OOB
      const unsigned koff = (unsigned)((kbeg + k0) * 4);
      const unsigned soffA =
          MODE == 0 ? koff : (unsigned)((((long long)dyb * ic.W + dxb) * ic.C + cb) * 4);
#pragma unroll
      for (int i = 0; i < LPSA; ++i) {
        const unsigned vo = (MODE == 0 || ((maskA[i] >> tapb) & 1)) ? voA[i] : OOB_OFF;
        lds_dma16_buf(rsA, vo, soffA, base + (wid + i * NW) * 256);
      }
#pragma unroll
      for (int j = 0; j < LPSB; ++j) lds_dma16_buf(rsB, voB[j], koff, base + (A_CH + wid + j * NW) * 256);
      if constexpr (MODE != 0) {  // one tap per K-step: C % 32 == 0
        cb += BK;
        if (cb >= ic.C) {
          cb = 0;
          ++tapb;
          dyb = dyn;
          dxb = dxn;
          if (dxn + 1 == ic.kw) {
            dxn = 0;
            ++dyn;
          } else {
            ++dxn;
          }
        }
      }
      return;
    }
    const long long tap_off = MODE != 0 ? (long long)dyb * rowstride + (long long)dxb * ic.C + cb : 0;
#pragma unroll
    for (int i = 0; i < LPSA; ++i) {
      const float* s;
      if constexpr (MODE == 0) {
        s = srcA[i] + k0;
      } else if (aligned) {
        // C % 32 == 0: the K-step is 32 channels of ONE tap, so the source is the lane's
        // pixel + a wave-uniform offset, gated by one bit of the lane's tap mask
        s = ((maskA[i] >> tapb) & 1) ? srcA[i] + tap_off + lsA[i] : ic.zero;
      } else {
        const int e = cb + lsA[i];
        const bool nx = e >= ic.C;
        const int c = nx ? e - ic.C : e;
        const int dy = nx ? dyn : dyb, dx = nx ? dxn : dxb;
        const int tap = tapb + (nx ? 1 : 0);
        s = ((maskA[i] >> tap) & 1) ? srcA[i] + dy * rowstride + (long long)dx * ic.C + c : ic.zero;
      }
      lds_dma16(s, base + (wid + i * NW) * 256);
    }
#pragma unroll
    for (int j = 0; j < LPSB; ++j) lds_dma16(srcB[j] + k0, base + (A_CH + wid + j * NW) * 256);
    if constexpr (MODE != 0) {  // advance the uniform tap cursor by one K-step (32 k)
      cb += BK;
      while (cb >= ic.C) {
        cb -= ic.C;
        ++tapb;
        dyb = dyn;
        dxb = dxn;
        if (dxn + 1 == ic.kw) {
          dxn = 0;
          ++dyn;
        } else {
          ++dxn;
        }
      }
    }
  };

  acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < MM::REGS; ++r) acc[i][j][r] = 0.f;

  // fragment read offsets: row base + swizzled slot for each K group
  const int fr = MM::frag_row(lane), fp = MM::frag_part(lane);
  const int sw = (fr >> 1) & 7;
  constexpr int NG = BK / MM::KG;
  int kofs[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) kofs[g] = 4 * ((g * MM::PARTS + fp) ^ sw);
  const int a_row = (wm * WTM + fr) * BK;
  const int b_row = BM * BK + (wn * WTN + fr) * BK;

  const int nk = K / BK;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s, s * BK);

  int stage = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // own DMAs of stage kt have landed once only the younger stages' remain outstanding
    const int ahead = nk - 1 - kt < NS - 2 ? nk - 1 - kt : NS - 2;
    if (ahead >= 2)
      wait_vmcnt<2 * LPS>();
    else if (ahead == 1)
      wait_vmcnt<LPS>();
    else
      wait_vmcnt<0>();
    raw_barrier();
    if (kt + NS - 1 < nk) {
      int ns = stage + NS - 1;
      ns = ns >= NS ? ns - NS : ns;
      issue(ns, (kt + NS - 1) * BK);
    }
    const float* S = smem + stage * STAGE;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      f32x4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f32x4*>(S + a_row + i * MF * BK + kofs[g]);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const f32x4*>(S + b_row + j * MF * BK + kofs[g]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = MM::op(af[i][s], bf[j][s], acc[i][j]);
    }
    // this wave's reads of `stage` are complete before it can pass the next barrier
    wait_lgkm0();
    stage = stage + 1 == NS ? 0 : stage + 1;
  }
  if constexpr (GEN) {  // the launcher picks this instantiation for > 3 splits or a pool-fused split
    static_assert(TM * TN * MM::REGS <= 32, "the any-split combine is for small wave tiles");
    if (sk.steps > 0 && sk.tickets && (MODE == 2 || sk.splits > 3)) {
      // latency plans (any split count) and pool-fused split layers: the last split sums, then
      // the normal store path below runs with the real epilogue
      if (!splitk_sum<MF, TM, TN, NW>(acc, C, sk, split, tile, wid, lane, reinterpret_cast<unsigned*>(smem))) return;
      epi.flags = sk.flags;
      C = sk.out;
      ldc = sk.ldo;
    }
  }
  if constexpr (MODE == 2) {
    store_tile_pool<MF, TM, TN, WTM, WTN>(acc, C, ldc, M, N, m0, n0, wm, wn, lane, epi, ic);
  } else {
    if (sk.steps > 0 && sk.tickets && sk.splits <= 3) {
      // batch plans: 3 splits (choose_splitk), partials loaded all at once
      if (sk.splits == 3)
        splitk_combine<3, MF, TM, TN, WTM, WTN, NW>(acc, C, sk, split, tile, M, N, m0, n0, wm, wn, wid, lane, epi,
                                                    reinterpret_cast<unsigned*>(smem));
      else
        splitk_combine<2, MF, TM, TN, WTM, WTN, NW>(acc, C, sk, split, tile, M, N, m0, n0, wm, wn, wid, lane, epi,
                                                    reinterpret_cast<unsigned*>(smem));
      return;
    }
    store_tile<MF, TM, TN, WTM, WTN>(acc, C, ldc, M, N, m0, n0, wm, wn, lane, epi);
  }
}

}  // namespace dnnhip
