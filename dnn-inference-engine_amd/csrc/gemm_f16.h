// fp16 MFMA GEMM for the fp16 conv path (BASELINE config 5), device code only.
//
// Same structure as gemm_f32_glds_kernel (gemm_f32.h): LDS-DMA ring of NS stages, 128-byte
// LDS rows XOR-swizzled on the source address, counted vmcnt + raw barriers, XCD-aware tile
// remap, dense / implicit / implicit+pool A operand, split-K into fp32 partials.  A K-step is
// BK = 64 halves (the same 128-B rows, so the same DMA and swizzle), and the math is
// v_mfma_f32_32x32x16_f16: lane l supplies A[row l&31][k 8(l>>5)..+7] and B likewise, i.e.
// exactly ONE 16-B slot per operand, so fragment slot = 2g + (l>>5) for K group g (0..3).
// Accumulation and the epilogue are fp32; the store rounds to OutT (fp16 activations, fp32
// for the last layer).  fp16 inputs: activations NHWC half, weights Bt[Npad][Kpad] half.
//
// Implicit mode: a 64-half K-step can span several taps when C < 64 (conv1: C = 16), so the
// (tap, channel) of each lane's 8-channel chunk is resolved per step from a uniform cursor
// and a per-tap offset table in LDS (tap t -> (t / kw) * W*C + (t % kw) * C).
#pragma once
#include "gemm_f32.h"

namespace dnnhip {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int wm_of(int wid, int wn) { return wid / wn; }
__device__ __forceinline__ int wn_of(int wid, int wn) { return wid - (wid / wn) * wn; }

__device__ __forceinline__ f32x16 mfma_f16(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// ABUF: buffer-descriptor LDS-DMA as in gemm_f32.h (BufDesc): per-lane 32-bit voffsets fixed per
// tile, the K-step in a uniform soffset, padding taps as OOB offsets (zero-filled).  Implicit
// mode supports it for C % 64 == 0 (one tap per 64-half K-step) and C == 32 (two taps per
// K-step: slots 4..7 of a row take the next tap, one uniform tap-to-tap delta).
template <int BM, int BN, int WM, int WN, int NS, int MODE, typename OutT, bool ABUF = false>
__global__ void __launch_bounds__(WM* WN * 64)
gemm_f16_glds_kernel(const half_t* __restrict__ A, int lda, const half_t* __restrict__ Bt, int ldb,
                     OutT* __restrict__ C, float* __restrict__ slab, int ldc, int M, int N, int K, EpiParams epi,
                     int tilesN, ImplicitConv ic, SplitK sk, BufDesc bd) {
  typedef Mfma<32> MM;
  constexpr int BK = 64;  // halves per K-step = 128 B per LDS row
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int A_CH = BM / 8, B_CH = BN / 8;
  constexpr int LPSA = A_CH / NW, LPSB = B_CH / NW, LPS = LPSA + LPSB;
  constexpr int STAGE = (BM + BN) * 32;  // floats per stage (rows of 32 floats = 64 halves)
  static_assert(A_CH % NW == 0 && B_CH % NW == 0, "chunks must split evenly over the waves");
  static_assert(NS >= 2 && NS <= 4, "ring depth");
  static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile must be a multiple of 32");

  __shared__ __attribute__((aligned(1024))) float smem[NS * STAGE];
  // implicit, flat-address DMA: tap -> element offset of (dy, dx) from the window origin
  // (the ABUF path keeps a uniform (dy, dx) cursor instead: no LDS beyond the ring)
  __shared__ int toff[ABUF ? 1 : 32];

  int tile = xcd_tile(blockIdx.x, gridDim.x);
  int kbeg = 0, split_idx = 0;
  const bool split = sk.steps > 0;
  if (split) {
    split_idx = tile / sk.ntile;
    tile -= split_idx * sk.ntile;
    kbeg = split_idx * sk.steps * BK;
    K = sk.steps * BK;
    if (!sk.tickets) slab += split_idx * sk.slab;
  }
  const int2 tc = tile_coords(tile, tilesN, sk);
  const int tm_ = tc.x, tn_ = tc.y;
  const int m0 = tm_ * BM, n0 = tn_ * BN;
  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int ntaps = ic.kh * ic.kw;

  if constexpr (MODE != 0 && !ABUF) {
    if (threadIdx.x < 32) {
      const int t = threadIdx.x, dy = t / ic.kw, dx = t - (t / ic.kw) * ic.kw;
      toff[t] = (dy * ic.W + dx) * ic.C;
    }
    __syncthreads();
  }

  // ---- A sources (chunk c = wid + i*NW holds rows 8c..8c+7; lane -> row 8c + lane/8 and
  // logical 16-B slot ls = (lane&7) ^ ((row>>1)&7))
  const half_t* srcA[LPSA];
  unsigned voA[LPSA];  // ABUF byte offsets (implicit: shifted base, + slot channel)
  int maskA[LPSA], lsA[LPSA], secA[LPSA];
  const bool two_taps = MODE != 0 && ic.C == 32;  // ABUF implicit with C == 32
#pragma unroll
  for (int i = 0; i < LPSA; ++i) {
    const int r = 8 * (wid + i * NW) + (lane >> 3);
    const int ls = (lane & 7) ^ ((r >> 1) & 7);
    lsA[i] = 8 * ls;  // halves
    secA[i] = two_taps && ls >= 4 ? 1 : 0;
    const int m = m0 + r;
    if constexpr (MODE == 0) {
      const int gm = m < M ? m : M - 1;
      if constexpr (ABUF)
        voA[i] = (unsigned)(((size_t)gm * lda + 8 * ls) * 2);
      else
        srcA[i] = A + (size_t)gm * lda + kbeg + 8 * ls;
      maskA[i] = 0;
    } else {
      int b, iy0, ix0;
      maskA[i] = implicit_row<MODE>(ic, m, M, b, iy0, ix0);
      if constexpr (ABUF)
        voA[i] = (unsigned)(((((long long)b * ic.H + iy0) * ic.W + ix0 + ic.W + 1) * ic.C + 8 * (two_taps ? (ls & 3) : ls)) * 2);
      else
        srcA[i] = A + (((long long)b * ic.H + iy0) * ic.W + ix0) * (long long)ic.C;
    }
  }
  const half_t* srcB[LPSB];
  unsigned voB[LPSB];
#pragma unroll
  for (int j = 0; j < LPSB; ++j) {
    const int r = 8 * (wid + j * NW) + (lane >> 3);
    const int ls = (lane & 7) ^ ((r >> 1) & 7);
    if constexpr (ABUF)
      voB[j] = (unsigned)(((size_t)(n0 + r) * ldb + 8 * ls) * 2);
    else
      srcB[j] = Bt + (size_t)(n0 + r) * ldb + kbeg + 8 * ls;
  }
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)bd.a, 0, (int)bd.a_bytes, 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)bd.b_bytes, 0x00020000);

  // implicit: uniform cursor (tap, channel) of the next K-step's first element
  int tapb = 0, cb = 0;
  int dyb = 0, dxb = 0;  // ABUF: (dy, dx) of tap tapb
  if constexpr (MODE != 0) {
    tapb = kbeg / ic.C;
    cb = kbeg - tapb * ic.C;
    dyb = tapb / ic.kw;
    dxb = tapb - dyb * ic.kw;
  }
  const float* zero = ic.zero;

  auto issue = [&](int stage, int k0) {
    float* base = smem + stage * STAGE;
    if constexpr (ABUF) {
      const unsigned koff = (unsigned)((kbeg + k0) * 2);
      unsigned soffA = koff, dsec = 0;
      if constexpr (MODE != 0) {
        soffA = (unsigned)((((long long)dyb * ic.W + dxb) * ic.C + cb) * 2);
        // next tap: (dy, dx+1), or (dy+1, 0) past the row
        dsec = (unsigned)((dxb + 1 == ic.kw ? (ic.W - (ic.kw - 1)) : 1) * ic.C * 2);
      }
#pragma unroll
      for (int i = 0; i < LPSA; ++i) {
        unsigned vo = voA[i];
        if constexpr (MODE != 0) vo = ((maskA[i] >> (tapb + secA[i])) & 1) ? vo + (secA[i] ? dsec : 0u) : OOB_OFF;
        lds_dma16_buf(rsA, vo, soffA, base + (wid + i * NW) * 256);
      }
#pragma unroll
      for (int j = 0; j < LPSB; ++j) lds_dma16_buf(rsB, voB[j], koff, base + (A_CH + wid + j * NW) * 256);
      if constexpr (MODE != 0) {
        cb += BK;
        while (cb >= ic.C) {
          cb -= ic.C;
          ++tapb;
          if (++dxb == ic.kw) {
            dxb = 0;
            ++dyb;
          }
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < LPSA; ++i) {
      const void* s;
      if constexpr (MODE == 0) {
        s = srcA[i] + k0;
      } else {
        int e = cb + lsA[i], t = tapb;
        while (e >= ic.C) {
          e -= ic.C;
          ++t;
        }
        s = (t < ntaps && ((maskA[i] >> t) & 1)) ? (const void*)(srcA[i] + toff[t] + e) : (const void*)zero;
      }
      lds_dma16(reinterpret_cast<const float*>(s), base + (wid + i * NW) * 256);
    }
#pragma unroll
    for (int j = 0; j < LPSB; ++j)
      lds_dma16(reinterpret_cast<const float*>(srcB[j] + k0), base + (A_CH + wid + j * NW) * 256);
    if constexpr (MODE != 0) {
      cb += BK;
      while (cb >= ic.C) {
        cb -= ic.C;
        ++tapb;
      }
    }
  };

  MM::acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int fr = lane & 31, fp = lane >> 5;
  const int sw = (fr >> 1) & 7;
  int kofs[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) kofs[g] = 4 * ((2 * g + fp) ^ sw);  // float offset of the 16-B slot
  const int a_row = (wm_of(wid, WN) * WTM + fr) * 32;
  const int b_row = BM * 32 + (wn_of(wid, WN) * WTN + fr) * 32;

  const int nk = K / BK;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s, s * BK);

  int stage = 0;
  for (int kt = 0; kt < nk; ++kt) {
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
    for (int g = 0; g < 4; ++g) {
      f16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f16x8*>(S + a_row + i * 32 * 32 + kofs[g]);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const f16x8*>(S + b_row + j * 32 * 32 + kofs[g]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_f16(af[i], bf[j], acc[i][j]);
    }
    wait_lgkm0();
    stage = stage + 1 == NS ? 0 : stage + 1;
  }
  const int wm = wm_of(wid, WN), wn = wn_of(wid, WN);
  if (split && sk.tickets) {  // in-GEMM combine (gemm_f32.h splitk_combine), output OutT
    if (sk.splits == 3)
      splitk_combine<3, 32, TM, TN, WTM, WTN, NW, OutT>(acc, slab, sk, split_idx, tile, M, N, m0, n0, wm, wn, wid, lane,
                                                        epi, reinterpret_cast<unsigned*>(smem));
    else
      splitk_combine<2, 32, TM, TN, WTM, WTN, NW, OutT>(acc, slab, sk, split_idx, tile, M, N, m0, n0, wm, wn, wid, lane,
                                                        epi, reinterpret_cast<unsigned*>(smem));
    return;
  }
  if (split) {
    EpiParams raw = epi;
    raw.flags = 0;  // raw partial sums; the reduce kernel applies the epilogue
    store_tile<32, TM, TN, WTM, WTN, float>(acc, slab, N, M, N, m0, n0, wm, wn, lane, raw);
  } else if constexpr (MODE == 2) {
    store_tile_pool<32, TM, TN, WTM, WTN, OutT>(acc, C, ldc, M, N, m0, n0, wm, wn, lane, epi, ic);
  } else {
    store_tile<32, TM, TN, WTM, WTN, OutT>(acc, C, ldc, M, N, m0, n0, wm, wn, lane, epi);
  }
}

}  // namespace dnnhip
