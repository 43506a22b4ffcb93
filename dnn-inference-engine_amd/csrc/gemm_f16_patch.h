// fp16 3x3 conv for the long-K, wide-N layers (conv6/conv7 of YOLOv2-tiny on the fp16 path,
// BASELINE config 5), device code only.
//
// Why a second fp16 GEMM: gemm_f16_glds_kernel stages A and B through LDS for every 64-half
// K-step.  On 128x512 tiles that is 80 KB per 8.4 MFLOP, 40 B/clk/CU at the fp16 MFMA rate,
// while L2-served LDS-DMA delivers ~30 B/clk and Infinity-Cache-served ~14 (MI355X_MICROARCH
// "Indexed rows"): conv7 ran at 36 % of peak, bound by that stream.  Here
//   * A (the activations) is staged ONCE per 64-channel chunk and reused by all 9 taps: the
//     input sits in HBM zero-padded ([B][H+2][W+2][C], borders written once at plan
//     finalize), so output pixel m's tap (dy, dx) is padded row p(m) + (dy-1)(W+2) + (dx-1).
//     A tile of BM consecutive output pixels reads one contiguous run of padded rows
//     [p(m0) - (W+3), p(m_last) + (W+3)] (<= NPR rows): no masks, one pass per chunk,
//     register-staged (loaded at tap 0, written to the other LDS buffer at tap 4), so chunk
//     j+1 lands during chunk j's 9 taps and every wait is the compiler's own (no LDS-DMA for
//     its wait insertion to fence the other buffer's reads with);
//   * B (the weights, packed K-order (chunk, tap, c)) goes straight from L2 to registers in
//     MFMA fragment order, two K-steps ahead: no LDS, no barrier per K-step;
//   * each of the 8 waves owns BM x 32 outputs (TM = BM/32 accumulators), so no wave
//     duplicates another's B and the workgroup needs one barrier per chunk.
// Per K-step and workgroup: 32 KB of B + ~4.5 KB of A per 12.6 MFLOP (BM = 192) instead of
// 80 KB per 8.4 MFLOP.  Summation order per output: chunk-major, tap, channel, fixed by (N, K):
// batch-invariant like the other fp16 kernels (not the fp32 path's order; the fp16 path holds
// a tolerance).
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

// BM rows (multiple of MF) x 256 columns per workgroup, 8 waves of BM x 32, NPR patch rows;
// MF = 32: v_mfma_f32_32x32x16_f16 (TM = BM/32 accumulators of 16), MF = 16:
// v_mfma_f32_16x16x32_f16 (TM = BM/16 x 2 accumulators of 4: 16-row granularity, so BM = 176
// gives 62 x 4 = 248 tiles for conv6/conv7 instead of 57 x 4 = 228 with BM = 192).
template <int BM, int NPR, typename OutT, int MF = 32>
__global__ void __launch_bounds__(512, 1)
conv3x3_f16_patch_kernel(const half_t* __restrict__ in, const half_t* __restrict__ Bt, int ldb, OutT* __restrict__ out,
                         int M, int N, int K, EpiParams epi, int tilesM, Patch16Geom g, unsigned in_bytes) {
  constexpr int BN = 256, TM = BM / MF, TN = 32 / MF;  // 8 waves of BM x 32
  constexpr int KG = MF == 32 ? 4 : 2;                  // MFMA k-groups per 64-half K-step
  constexpr int PPT = (NPR * 8 + 511) / 512;  // 16-B patch pieces per thread
  typedef typename std::conditional<MF == 32, f32x16, f32x4>::type acc_t;
  constexpr int NR = MF == 32 ? 16 : 4;
  static_assert(BM % MF == 0 && NPR % 8 == 0 && (MF == 32 || MF == 16), "shape");
  __shared__ __attribute__((aligned(1024))) float smem[2 * NPR * 32];  // 2 patches of NPR rows x 128 B

  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  // tiles N-major inside each XCD's contiguous range: the XCD's CUs share one weight panel
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int tn = tile / tilesM, tm = tile - tn * tilesM;
  const int m0 = tm * BM, n0 = tn * BN + wid * 32;  // this wave's 32 columns
  const int Wp = g.W + 2, HWo = g.H * g.W;
  auto padded = [&](int m) {
    const int b = m / HWo, r = m - b * HWo, oy = r / g.W, ox = r - oy * g.W;
    return (b * (g.H + 2) + oy + 1) * Wp + ox + 1;
  };
  const int P0 = padded(m0) - (Wp + 1);  // first patch row (>= 0: p(0) = Wp + 1)

  // A fragment rows: lane's output row r = MF i + fr -> patch row of tap (1, 1)
  const int fr = lane & (MF - 1), fp = MF == 32 ? lane >> 5 : lane >> 4;
  int prow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int m = m0 + MF * i + fr;
    m = m < M ? m : M - 1;
    prow[i] = padded(m) - P0;
  }

  // patch staging: 16-B piece q = tid + 512 u of the NPR x 8 pieces -> patch row
  // tid/8 + 64 u, logical slot tid % 8, stored at physical slot (tid % 8) ^ ((row >> 1) & 7)
  // (the same for every u: 64 u rows keep (row >> 1) & 7); piece u is one uniform step apart
  static_assert(NPR == 64 * PPT, "NPR must be a multiple of 64 (every piece in range)");
  const int prow0 = threadIdx.x >> 3, pls = threadIdx.x & 7;
  const unsigned pvo = (unsigned)(((size_t)(P0 + prow0) * g.C + 8 * pls) * 2);
  const int pdst = prow0 * 32 + 4 * (pls ^ ((prow0 >> 1) & 7));
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  // piece u of patch j+1 is loaded at tap u of chunk j and written to LDS at tap u + 2 (its
  // in-order vmcnt slack is the B ring's two K-steps anyway), so few staging registers live
  u32x4 pst[PPT];
  auto load_piece = [&](int chunk, int u) {
    pst[u] = __builtin_amdgcn_raw_buffer_load_b128(rsA, pvo, chunk * 128 + u * 64 * g.C * 2, 0);
  };
  auto store_piece = [&](int buf, int u) {
    *reinterpret_cast<u32x4*>(smem + buf * NPR * 32 + pdst + u * 64 * 32) = pst[u];
  };

  // B fragments straight to registers: the weights are packed in MFMA fragment order
  // ([n/MF][k/(1024/MF)][lane][8 halves], launch_pack_weights order 3 / 4), so one fragment
  // is one contiguous 1-KiB load (per-lane offset fixed, the K position uniform)
  const unsigned bvo = (unsigned)((size_t)(n0 / MF) * ldb * 2 * MF + lane * 16);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)((size_t)(n0 - wid * 32 + 256) * ldb * 2),
                                                     0x00020000);
  const int nk = K / 64, nch = nk / 9;
  f16x8 bq[3][4];  // B of K-steps s .. s+2 (two ahead): slot s % 3 == tap % 3, as 9 % 3 == 0
  // (MF = 32: [group q]; MF = 16: [2 group + n-block j])
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[a][q] = f16x8{};
  auto load_b = [&](int s, f16x8 (&dst)[4]) {
    // unconditional (past the end: another panel's weights or the descriptor's zeros, never
    // used): a conditional load leaves the wait insertion to assume it was not issued, so every
    // later wait for an older fragment would drain this one too (and the staging registers
    // would be spilled across the branch)
    {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        dst[q] = __builtin_bit_cast(
            f16x8, __builtin_amdgcn_raw_buffer_load_b128(
                       rsB, bvo + (MF == 32 ? 0u : (unsigned)((q & 1) * ldb * 32)),
                       MF == 32 ? (4 * s + q) * 1024 : (2 * s + (q >> 1)) * 1024, 0));
    }
  };

  acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[i][j][r] = 0.f;

#pragma unroll
  for (int u = 0; u < PPT; ++u) load_piece(0, u);
  load_b(0, bq[0]);
  load_b(1, bq[1]);
#pragma unroll
  for (int u = 0; u < PPT; ++u) store_piece(0, u);
  wait_lgkm0();
  __syncthreads();

  constexpr int LAG = MF == 32 ? 2 : 1;  // taps between a piece's load and its LDS store
  static_assert(PPT + LAG <= 9, "patch pieces must be written within the chunk");
  // A fragment address of row `row`, group q: row*32 + 4*((SQ q + fp) ^ ((row >> 1) & 7))
  //   = (row*32 + 4*y) ^ (4 SQ q) with y = ((row >> 1) & 7) ^ fp (SQ = 2 for MF 32, 4 for MF 16)
  constexpr int QX = MF == 32 ? 8 : 16;
  auto tap_base = [&](int t, int (&ab)[TM]) {
    const int toff = (t / 3 - 1) * Wp + (t % 3 - 1);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      int pr = prow[i];
      asm volatile("" : "+v"(pr));  // keep the 9 taps' addresses from being hoisted (54 VGPRs)
      const int row = pr + toff;
      ab[i] = row * 32 + 4 * (((row >> 1) & 7) ^ fp);
    }
  };
  // MF = 16 walks the fragment addresses from tap to tap (row = ab >> 5 recovers the patch
  // row), so the 11 prow registers are dead after the first tap
  auto step_base = [&](int delta, int (&ab)[TM]) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = (ab[i] >> 5) + delta;
      ab[i] = row * 32 + 4 * (((row >> 1) & 7) ^ fp);
    }
  };
  int ab[TM];
  if constexpr (MF == 16) tap_base(0, ab);
  for (int j = 0; j < nch; ++j) {
    const bool next = j + 1 < nch;
    const float* P = smem + (j & 1) * NPR * 32;
    // groups g = 4 t + q of this chunk; the fragments of group g + 1 are read while group g's
    // MFMAs run (two fragment sets in flight)
    if constexpr (MF == 32) tap_base(0, ab);
    f16x8 af[2][TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[0][i] = *reinterpret_cast<const f16x8*>(P + ab[i]);
    static_assert(KG == 4 || KG == 2, "k-groups");
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int s = 9 * j + t;
      // (chunk nch is loaded and stored too, into the idle buffer, for the reason load_b gives:
      // past the channels of the last row the descriptor returns zeros)
      // Taps are scheduling regions: the scheduler otherwise sinks a piece's load down to its
      // LDS store and waits vmcnt(0) for it
      __builtin_amdgcn_sched_barrier(0);
      if (t < PPT) load_piece(j + 1, t);
      load_b(s + 2, bq[(t + 2) % 3]);
      if (t >= LAG && t < PPT + LAG) store_piece((j + 1) & 1, t - LAG);
#pragma unroll
      for (int q = 0; q < KG; ++q) {
        const int cur = q & 1, nxt = cur ^ 1;
        if (q < KG - 1) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
            af[nxt][i] = *reinterpret_cast<const f16x8*>(P + (ab[i] ^ (QX * (q + 1))));
        } else if (t < 8) {
          if constexpr (MF == 16)
            step_base(t % 3 == 2 ? Wp - 2 : 1, ab);
          else
            tap_base(t + 1, ab);
#pragma unroll
          for (int i = 0; i < TM; ++i) af[nxt][i] = *reinterpret_cast<const f16x8*>(P + ab[i]);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if constexpr (MF == 32)
              acc[i][j] = mfma_f16(af[cur][i], bq[t % 3][q], acc[i][j]);
            else
              acc[i][j] = mfma16_f16(af[cur][i], bq[t % 3][2 * q + j], acc[i][j]);
          }
      }
    }
    if constexpr (MF == 16) step_base(-(2 * Wp + 2), ab);  // tap 8 -> tap 0
    if (next) {  // patch j+1 written by every wave; every wave done reading patch j
      wait_lgkm0();
      raw_barrier();
    }
  }

  // epilogue: bias/BN/leaky, output fp16 (plain [M][N] or zero-bordered padded rows); the
  // tile's output row indices are tabulated once in LDS (no per-element divisions)
  int* orow = reinterpret_cast<int*>(smem);
  __syncthreads();  // every wave is done with the patches
  if (threadIdx.x < BM) {
    const int m = m0 + threadIdx.x;
    orow[threadIdx.x] = m >= M ? -1 : (g.out_padded ? padded(m) : m);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + MF * j + fr;
    const float pb = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
    const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
    const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
    const float pg = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;
    if (n >= N) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int o = orow[MF * i + Mfma<MF>::out_row(lane, r)];
        if (o >= 0) store_out(out + (size_t)o * N + n, apply_epilogue(acc[i][j][r], pb, pm, ps, pg, epi.flags));
      }
  }
}

}  // namespace dnnhip
