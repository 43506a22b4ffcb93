// fp32 3x3 conv on the bf16 MFMA with exact three-way operand splits ("x3"), for the long-K,
// wide-N layers of the fp32 path (conv6/conv7 of YOLOv2-tiny), device code only.
//
// Why: the fp32 MFMA (v_mfma_f32_32x32x2f32) peaks at 157 TFLOP/s, the bf16 one at 2.5 PF.
// Every finite fp32 x with |x| >= 2^-100 is EXACTLY x0 + x1 + x2 with x0 = bf16(x), x1 =
// bf16(x - x0), x2 = bf16(x - x0 - x1) (round-to-nearest: 8 + 8 + 8 significand bits cover
// 24, and every difference is exact).  A product a*b is then the sum of the nine a_i*b_j; the
// six with i + j <= 2 are formed (each exact in the fp32 accumulator's input), the three
// dropped ones are <= 2^-24 |a b| together with rounding.  tools/bf16x6_probe.hip measured the
// result against float64 at K = 288 / 2304 / 9216: max |err| / sum|a b| 1.7e-7 - 3.4e-7,
// the fp32 MFMA (which reproduces a sequential fp32 FMA chain) 2.1e-7 - 3.0e-7: the same
// accuracy class as fp32, 6 bf16 MFMAs per fp32 product instead of 1/16 of the rate.
//
// Layout (written by the producers: maxpool_x3_kernel, this kernel's own epilogue):
// activations zero-bordered [B][H+2][W+2] rows, each row C/32 chunks of [3 pieces][32 ch]
// bf16 (192 B per chunk).  Weights (pack_weights_x3_kernel): [n/16][step][piece][lane][8]
// with step = chunk * 9 + tap over 32-channel chunks, i.e. MFMA fragment order of
// v_mfma_f32_16x16x32_bf16 (n = 16 nb + (lane & 15), k = 8 (lane >> 4) + e).
// Per output and 32-channel step: the corrections a2b0 + a1b1 + a0b2 + a1b0 + a0b1 and the main
// product a0b0 (x3_step: two accumulators, or the round-2 form: corrections summed from zero and
// added per step); steps chunk-major, tap-minor.  The order depends on (N, K) only, so batch rows
// are bit-identical to batch-1 runs; it is not the fp32 MFMA path's order (DNN_HIP_X3=0 selects
// that path).
//
// This file: the layout, the step, the pooled split-plane store and the narrow-layer kernels
// (2-D output tiles: conv2/conv3; 16 channels: conv1).  The wide-N layers' kernel (conv4-conv7)
// is conv3x3_x3_acc2_kernel (gemm_x3_acc2.h).
#pragma once
#include "gemm_f16.h"

// X3DIAG (diagnostic builds only, tools/build_diag.sh; see also gemm_x3_acc2.h): bit 32 records
// conv3x3_x3_c16p_kernel's per-workgroup phase cycles (results unchanged), bit 64 drops its pool /
// epilogue math, bit 128 replaces its input split by a 2-instruction truncation (wrong results),
// bit 1024 records conv3x3_x3_tile2_kernel's per-workgroup phase stamps (results unchanged)
#ifndef X3DIAG
#define X3DIAG 0
#endif
namespace dnnhip {

#if (X3DIAG & 32) != 0  // conv3x3_x3_c16p_kernel phase cycles (gemm_x3_patch.h)
constexpr int C16_DIAG_WGS = 1024;
constexpr int C16_DIAG_SLOTS = 10;
// [workgroup][slot]: wave 0's s_memtime sums over its tiles -- 0 the loop-top drain, 1 split + row
// table + next loads, 2 barrier, 3 MFMAs, 4 barrier, 5 epilogue math + stage, 6 split-plane
// stores, 7 barrier; 8 tiles
__device__ unsigned long long c16_diag_stamps[C16_DIAG_WGS * C16_DIAG_SLOTS];
#endif

#if (X3DIAG & 1024) != 0  // conv3x3_x3_tile2_kernel phase stamps
constexpr int T2_DIAG_WGS = 4096;
constexpr int T2_DIAG_SLOTS = 16;
// [layer (0: N = 64, 1: wider)][workgroup][slot], wave 0 unless noted: 0 s_memrealtime at start,
// 1-4 s_memtime at start, patch landed, MFMAs done, end; 5 s_memrealtime at end; 6 HW_ID; 7
// XCC_ID; 8-11 s_memtime when wave 0-3 finished its MFMAs; 12 after the epilogue's first barrier,
// 13 after the row-table barrier, 14 after the pooled values are staged
__device__ unsigned long long tile2_diag_stamps[2 * T2_DIAG_WGS * T2_DIAG_SLOTS];
#define T2_STAMP(k, v)                                                                               \
  if (threadIdx.x == 0 && blockIdx.x < T2_DIAG_WGS)                                                  \
    tile2_diag_stamps[((N == 64 ? 0 : 1) * T2_DIAG_WGS + blockIdx.x) * T2_DIAG_SLOTS + (k)] = (v);
#define T2_STAMPW(k, v)                                                                              \
  if ((threadIdx.x & 63) == 0 && threadIdx.x < 256 && blockIdx.x < T2_DIAG_WGS)                      \
    tile2_diag_stamps[((N == 64 ? 0 : 1) * T2_DIAG_WGS + blockIdx.x) * T2_DIAG_SLOTS + (k) + (threadIdx.x >> 6)] = (v);
#else
#define T2_STAMP(k, v)
#define T2_STAMPW(k, v)
#endif

#if (X3DIAG & 2048) != 0  // conv3x3_x3_pp_kernel step cycles
constexpr int PP_DIAG_WGS = 512;
// [workgroup][slot]: s_memtime sums of wave 0 (team A) in 0-2 and wave 4 (team B) in 3-5: MFMA
// step work, store step work, barrier waits; 6 total cycles of wave 0
__device__ unsigned long long pp_diag_stamps[PP_DIAG_WGS * 8];
#endif

#if (X3DIAG & 32768) != 0  // conv3x3_x3_c16pp_kernel step cycles
constexpr int C16PP_DIAG_WGS = 512;
// [workgroup][slot]: s_memtime sums of wave 0 (team A) in 0-3 and wave 4 (team B) in 4-7: MFMA steps,
// store steps' wait + split + next loads, their fold + epilogue + stores, barrier waits; 8 total
// cycles of wave 0; 9 tiles of team A
__device__ unsigned long long c16pp_diag_stamps[C16PP_DIAG_WGS * 16];
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct X3Geom {
  int H, W, C;     // conv input = output spatial size (3x3, stride 1, SAME), channels
  int out_mode;    // 0: fp32 [M][N] after the epilogue; 1: split planes into a zero-bordered
                   // [B][H+2][W+2] buffer (next x3 layer); 2: raw fp32 partial of split-K slice
                   // s at out + s*M*N (no epilogue; x3_combine_kernel finishes)
  int splits;      // K split into this many contiguous chunk ranges (grid = tiles x splits)
  int PH, PW;      // POOL kernels: the 2x2/s2 pooled output (rows are pool-window-major)
};

__device__ __forceinline__ f32x4 mfma16_bf16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// One 32-channel step of one 16 x 16 block, column block jb of the weight set b[piece][jb].
// A2 (gemm_x3_acc2.h): corrections a2b0, a1b1, a0b2, a1b0, a0b1 back to back onto accc, the main
// product a0b0 onto acc; else the round-2 form: corrections from zero, acc = (acc + a0b0) + c.
template <bool A2, int NB>
__device__ __forceinline__ void x3_step(f32x4& acc, f32x4& accc, const bf16x8 (&a)[3], const bf16x8 (&b)[3][NB],
                                        int jb) {
  if constexpr (A2) {
    f32x4 c = accc;
    c = mfma16_bf16(a[2], b[0][jb], c);
    c = mfma16_bf16(a[1], b[1][jb], c);
    c = mfma16_bf16(a[0], b[2][jb], c);
    c = mfma16_bf16(a[1], b[0][jb], c);
    c = mfma16_bf16(a[0], b[1][jb], c);
    accc = c;
    acc = mfma16_bf16(a[0], b[0][jb], acc);
  } else {
    f32x4 c = mfma16_bf16(a[2], b[0][jb], f32x4{0.f, 0.f, 0.f, 0.f});
    c = mfma16_bf16(a[1], b[1][jb], c);
    c = mfma16_bf16(a[0], b[2][jb], c);
    c = mfma16_bf16(a[1], b[0][jb], c);
    c = mfma16_bf16(a[0], b[1][jb], c);
    const f32x4 m = mfma16_bf16(a[0], b[0][jb], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = m[r] + c[r];
  }
}
template <int TM, int NB>
__device__ __forceinline__ void x3_fold(f32x4 (&acc)[TM][NB], const f32x4 (&accc)[TM][NB]) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = acc[i][j][r] + accc[i][j][r];
}

// One output column's epilogue parameters (bias, mean, sqrt(var + eps), gamma; absent terms the
// identity).  The single-frame kernels load them with their first operands, not at the epilogue:
// at one frame a load issued there is a whole memory round trip (~1.5 us) on the critical path.
struct X3EpiCol {
  float pb, pm, ps, pg;
};
__device__ __forceinline__ X3EpiCol x3_epi_col(const EpiParams& epi, int eflags, int n) {
  X3EpiCol c;
  c.pb = (eflags & EPI_BIAS) ? epi.bias[n] : 0.f;
  c.pm = (eflags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
  c.ps = (eflags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
  c.pg = (eflags & EPI_BN) ? epi.gamma[n] : 1.f;
  return c;
}

// Pooled split-plane store through LDS (the narrow x3 kernels' epilogue): a wave's pooled values
// of TM row blocks (4 windows x 32 columns each) are written to a wave-private stage in the MFMA
// layout (lane (fr, fq) of block i: window 4 i + fq, column 16 jb + fr; 48-float rows, so the
// two lane halves of a ds_write_b32 fall on disjoint banks), then each lane takes (window, 8
// columns) tasks: two 16-B stage reads, the exact split of the 8 values and one 16-B store per
// piece into the window's 192-B record (3 x 32 bf16 at out_split + o n3 + col0).  The values and
// splits are those of one scalar store per piece and output.
constexpr int X3_STG_ROW = 48;
// (orow_of(w): the output record of the tile's window w < no, or -1)
template <int TM, typename OF>
__device__ __forceinline__ void x3_pool_split_store_f(const float* stg, OF&& orow_of, int no, int wbase,
                                                      bf16_bits* __restrict__ out_split, size_t n3, int col0,
                                                      int lane) {
  wait_lgkm0();  // the stage is wave-private
  for (int task = lane; task < 16 * TM; task += 64) {
    const int wl = task >> 2, c8 = 8 * (task & 3), w = wbase + wl;
    const int o = w < no ? orow_of(w) : -1;
    if (o < 0) continue;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(stg + wl * X3_STG_ROW + c8);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(stg + wl * X3_STG_ROW + c8 + 4);
    bool ok = true;
#pragma unroll
    for (int e = 0; e < 4; ++e) ok = ok && x3_split_ok(lo[e]) && x3_split_ok(hi[e]);
    const bool fast = __builtin_amdgcn_ballot_w64(!ok) == 0;  // (pairs of one v_cvt_pk per piece)
    u32x4 q[3];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      unsigned w0, w1, w2;
      split3_pack2(fast, e < 2 ? lo[2 * e] : hi[2 * e - 4], e < 2 ? lo[2 * e + 1] : hi[2 * e - 3], w0, w1, w2);
      q[0][e] = w0;
      q[1][e] = w1;
      q[2][e] = w2;
    }
    const size_t d = (size_t)o * n3 + col0 + c8;  // (halves)
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) store16_at(out_split, 2 * (d + 32 * pc), q[pc]);
  }
}
template <int TM>
__device__ __forceinline__ void x3_pool_split_store(const float* stg, const int* orow, int no, int wbase,
                                                    bf16_bits* __restrict__ out_split, size_t n3, int col0,
                                                    int lane) {
  x3_pool_split_store_f<TM>(stg, [&](int w) { return orow[w]; }, no, wbase, out_split, n3, col0, lane);
}

// POOL (all x3 conv kernels): a fused 2x2/s2 max pool -- GEMM rows pool-window-major (row 4 w +
// 2 dy + dx = cell (dy, dx) of pooled pixel w; cells past an odd edge repeat cell (0, 0)), so a
// lane's 4 accumulator registers (rows 4 q .. 4 q + 3 of its 16 x 16 block) are one window:
// pooled before the epilogue (pool_then_epilogue, as the fp32 GEMMs' fused pools).

// 16-channel layers (YOLOv2-tiny conv1, 208x208x16 -> 32): the input is the producer's plain
// fp32 NHWC (no split planes), split into the three bf16 pieces while the patch is staged
// (frame padding = the descriptor's zeros).  K = 144 runs as 5 steps of 32: step s feeds k
// 0-15 from tap 2s and k 16-31 from tap 2s + 1 (lane group fq >> 1 picks the tap; tap 9 has zero
// weights), so a lane's A fragment is 8 channels of one tap, 16 B at patch pixel (row + tap
// offset) * 96 + 32 piece + 16 (fq & 1) (conflict-free for 16 consecutive or window-major rows
// at the 96-B pitch).  The 30 KB of weights of the 32 columns (all of K) are copied into LDS
// once per workgroup and read per step (6 fragments per 7 row blocks), instead of every wave
// streaming them from L2 (73 B per MFMA at 2 waves per tile).  One chunk: no double buffer;
// two workgroups per CU overlap each other's staging.  Same product order per step as the
// kernels above; 32 columns (WN = 1), WM waves of TM 16-row blocks.
template <int TH, int TW, int WM, int TM, bool POOL, bool A2 = true>  // A2: as the tile kernel
__global__ void __launch_bounds__(64 * WM, 2)  // (waves per SIMD) two: <= 256 registers
conv3x3_x3_c16_kernel(const float* __restrict__ in, const bf16_bits* __restrict__ Bt, float* __restrict__ out,
                      bf16_bits* __restrict__ out_split, int N, EpiParams epi, int tilesX, int tilesY, X3Geom g,
                      unsigned in_bytes) {
  constexpr int NT = 64 * WM, PB = 96, PW2 = TW + 2, PR = (TH + 2) * PW2, T = TH * TW, NS = 5;
  constexpr int ITEMS = PR * 4, PPT = (ITEMS + NT - 1) / NT;  // item = (patch pixel, channel quad)
  constexpr int BB = 2 * NS * 3 * 1024, BPT = (BB / 16 + NT - 1) / NT;  // weight bytes, 16-B loads/thread
  static_assert(TH % 2 == 0 && TW % 2 == 0 && WM * TM * 16 >= T && (WM * TM - 3) * 16 < T, "shape");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[BB + PR * PB];
  unsigned char* const patch = smem + BB;

  const int lane = threadIdx.x & 63;
  const int wm = wave_uniform(threadIdx.x >> 6);
  int t = xcd_tile(blockIdx.x, gridDim.x);
  const int tx = t % tilesX;
  t /= tilesX;
  const int ty = t % tilesY;
  const int b = t / tilesY;
  const int y0 = ty * TH, x0 = tx * TW;

  // weights: the packed [n/16][step][piece][lane][8] block of columns 0-31 is contiguous
  {
    u32x4 w[BPT];
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      int e = threadIdx.x + u * NT;
      e = e < BB / 16 ? e : BB / 16 - 1;
      w[u] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned char*>(Bt) + 16 * e);
    }
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      int e = threadIdx.x + u * NT;
      e = e < BB / 16 ? e : BB / 16 - 1;
      *reinterpret_cast<u32x4*>(smem + 16 * e) = w[u];
    }
  }
  {  // patch: 16-B fp32 channel quad -> three 8-B bf16 quads (pieces at 32 p + 8 q of the pixel)
    const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
    constexpr int SB = 4;  // items in flight per thread
#pragma unroll
    for (int u0 = 0; u0 < PPT; u0 += SB) {
      f32x4 v[SB];
      int dst[SB];
#pragma unroll
      for (int d = 0; d < SB; ++d) {
        int e = threadIdx.x + (u0 + d) * NT;
        e = e < ITEMS ? e : ITEMS - 1;
        const int pr = e >> 2, q = e & 3, py = pr / PW2, px = pr - py * PW2;
        const int iy = y0 - 1 + py, ix = x0 - 1 + px;
        const bool ok = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
        const unsigned vo = ok ? (unsigned)((((b * g.H + iy) * g.W + ix) * 16 + 4 * q) * 4) : OOB_OFF;
        v[d] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, vo, 0, 0));
        dst[d] = pr * PB + 8 * q;
      }
      bool ok = true;
#pragma unroll
      for (int d = 0; d < SB; ++d)
#pragma unroll
        for (int c = 0; c < 4; ++c) ok = ok && x3_split_ok(v[d][c]);
      const bool fast = __builtin_amdgcn_ballot_w64(!ok) == 0;  // (pairs of one v_cvt_pk per piece)
#pragma unroll
      for (int d = 0; d < SB; ++d) {
        uint2 w[3];
        split3_pack2(fast, v[d][0], v[d][1], w[0].x, w[1].x, w[2].x);
        split3_pack2(fast, v[d][2], v[d][3], w[0].y, w[1].y, w[2].y);
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(patch + dst[d] + 32 * p) = w[p];
      }
    }
  }

  const int fr = lane & 15, fq = lane >> 4, th = fq >> 1;  // th: this lane's tap within a step pair
  int prow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int r = (wm * TM + i) * 16 + fr;
    r = r < T ? r : T - 1;
    int ly, lx;
    if constexpr (POOL) {
      const int w = r >> 2, q = r & 3;
      ly = 2 * (w / (TW / 2)) + (q >> 1);
      lx = 2 * (w % (TW / 2)) + (q & 1);
    } else {
      ly = r / TW;
      lx = r % TW;
    }
    prow[i] = ((ly + 1) * PW2 + lx + 1) * PB + 16 * (fq & 1);
  }

  f32x4 acc[TM][2], accc[TM][2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = accc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  auto toff = [&](int s) {  // this lane's tap offset (bytes) in step s
    const int ta = 2 * s, tb = 2 * s + 1 < 9 ? 2 * s + 1 : 8;  // (tap 9: zero weights)
    const int oa = ((ta / 3 - 1) * PW2 + (ta % 3 - 1)) * PB, ob = ((tb / 3 - 1) * PW2 + (tb % 3 - 1)) * PB;
    return th ? ob : oa;
  };
  auto frag = [&](int i, int off, bf16x8 (&a)[3]) {
    int pr = prow[i];
    asm volatile("" : "+v"(pr));
    const unsigned char* q = patch + pr + off;
#pragma unroll
    for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(q + 32 * p);
  };
  auto bfrag = [&](int s, bf16x8 (&bb)[3][2]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bb[p][j] = *reinterpret_cast<const bf16x8*>(smem + (j * NS * 3 + s * 3 + p) * 1024 + lane * 16);
  };
  bf16x8 af[2][3], bq[2][3][2];
  frag(0, toff(0), af[0]);
  bfrag(0, bq[0]);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int off = toff(s), off_next = toff(s + 1 < NS ? s + 1 : s);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int cur = (s * TM + i) & 1, nxt = cur ^ 1;
      if (i + 1 < TM)
        frag(i + 1, off, af[nxt]);
      else if (s + 1 < NS)
        frag(0, off_next, af[nxt]);
      if (i == 0 && s + 1 < NS) bfrag(s + 1, bq[(s + 1) & 1]);  // next step's weights
      const bf16x8(&bb)[3][2] = bq[s & 1];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) x3_step<A2>(acc[i][jb], accc[i][jb], af[cur], bb, jb);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  if constexpr (A2) x3_fold(acc, accc);
  // epilogue (as conv3x3_x3_tile_kernel)
  int* orow = reinterpret_cast<int*>(smem);
  __syncthreads();
  constexpr int NO = POOL ? T / 4 : T;
  const int Wp = g.W + 2;
  for (int r = threadIdx.x; r < NO; r += NT) {
    int o;
    if constexpr (POOL) {
      const int py = (y0 >> 1) + r / (TW / 2), px = (x0 >> 1) + r % (TW / 2);
      o = (py >= g.PH || px >= g.PW) ? -1
          : g.out_mode == 1         ? (b * (g.PH + 2) + py + 1) * (g.PW + 2) + px + 1
                                    : (b * g.PH + py) * g.PW + px;
    } else {
      const int oy = y0 + r / TW, ox = x0 + r % TW;
      o = (oy >= g.H || ox >= g.W) ? -1 : g.out_mode == 1 ? (b * (g.H + 2) + oy + 1) * Wp + ox + 1 : (b * g.H + oy) * g.W + ox;
    }
    orow[r] = o;
  }
  __syncthreads();
  if constexpr (POOL) {
    if (g.out_mode == 1) {  // staged 16-B split-plane stores (x3_pool_split_store)
      static_assert(1024 + WM * TM * 4 * X3_STG_ROW * 4 <= BB + PR * PB && NO * 4 <= 1024, "stage");
      float* stg = reinterpret_cast<float*>(smem + 1024) + wm * (TM * 4 * X3_STG_ROW);
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        const int n = 16 * jb + fr;
        const float pb = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
        const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
        const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
        const float pg = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
          stg[(4 * i + fq) * X3_STG_ROW + 16 * jb + fr] = pool_then_epilogue(acc[i][jb], pb, pm, ps, pg, epi.flags);
      }
      x3_pool_split_store<TM>(stg, orow, NO, 4 * wm * TM, out_split, 96, 0, lane);
      return;
    }
  }
#pragma unroll
  for (int jb = 0; jb < 2; ++jb) {
    const int n = 16 * jb + fr;
    const float pb = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
    const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
    const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
    const float pg = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;
    auto put = [&](int o, float v) {
      if (g.out_mode == 1) {
        unsigned short s0, s1, s2;
        split3(v, s0, s1, s2);
        bf16_bits* d = out_split + (size_t)o * 96 + n;
        d[0] = s0;
        d[32] = s1;
        d[64] = s2;
      } else {
        out[(size_t)o * N + n] = v;
      }
    };
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rb = 16 * (wm * TM + i);
      if constexpr (POOL) {
        const int w = rb / 4 + fq;
        const int o = w < NO ? orow[w] : -1;
        if (o >= 0) put(o, pool_then_epilogue(acc[i][jb], pb, pm, ps, pg, epi.flags));
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb + 4 * fq + r;
          const int o = row < NO ? orow[row] : -1;
          if (o >= 0) put(o, apply_epilogue(acc[i][jb][r], pb, pm, ps, pg, epi.flags));
        }
      }
    }
  }
}


// 16-channel layers, persistent (conv1): the 16-channel kernel's tile (TH x TW = 16 x 26 output
// pixels, 4 waves of 7 row blocks, 32 columns, pool-window-major rows) and fragments, but each
// workgroup (two per CU) loops over tiles t, t + G, ...: the 30 KB of weights are copied into LDS
// once per workgroup instead of once per tile, and the next tile's fp32 patch (8 x 16 B per
// thread) is loaded into registers right after this tile's split is written, so its latency runs
// under this tile's MFMAs; the other workgroup on the CU computes while this one splits and
// stores.  Per tile: split -> barrier -> MFMAs -> barrier -> epilogue (its stage in the patch
// area) -> barrier.  HALF: the last K step (tap 8 alone: k 128-143) on v_mfma_f32_16x16x16_bf16
// instead of a 16x16x32 step whose upper half is a zero tap -- 27 instead of 30 16x16x32-sized
// MFMAs per block and column block, if the K = 16 form issues in half the cycles.  Summation
// order: as the 16-channel kernel (two accumulators; steps 0-4), the order depending on (N, K)
// only.  LDS: 30 KB weights + 48 KB split patch + 1.7 KB row table = 79 KB (two per CU).
template <bool POOL, bool HALF, int FL = -1>
__global__ void __launch_bounds__(256, 2)
conv3x3_x3_c16p_kernel(const float* __restrict__ in, const bf16_bits* __restrict__ Bt, float* __restrict__ out,
                       bf16_bits* __restrict__ out_split, int N, EpiParams epi, int tilesX, int tilesY, int ntiles,
                       X3Geom g, unsigned in_bytes) {
  constexpr int TH = 16, TW = 26, WM = 4, TM = 7;
  constexpr int NT = 64 * WM, PB = 96, PW2 = TW + 2, PR = (TH + 2) * PW2, T = TH * TW, NS = 5;
  constexpr int ITEMS = PR * 4, PPT = (ITEMS + NT - 1) / NT;  // item = (patch pixel, channel quad)
  constexpr int BB = 2 * NS * 3 * 1024, BPT = (BB / 16 + NT - 1) / NT;
  constexpr int NO = POOL ? T / 4 : T;
  constexpr int PATCH = PR * PB;
  static_assert(WM * TM * 16 >= T && (WM * TM - 3) * 16 < T && PPT == 8, "shape");
  static_assert(WM * TM * 4 * X3_STG_ROW * 4 <= PATCH, "epilogue stage inside the patch area");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[BB + PATCH + NO * 4];
  unsigned char* const patch = smem + BB;
  int* const orow = reinterpret_cast<int*>(smem + BB + PATCH);

  const int lane = threadIdx.x & 63;
  const int eflags = FL < 0 ? epi.flags : FL;  // FL: the epilogue flag set compiled in (-1: runtime)
  const int wm = wave_uniform(threadIdx.x >> 6);
  const int fr = lane & 15, fq = lane >> 4, th = fq >> 1;
  const int Wp = g.W + 2;
  // the 32 columns' epilogue parameters, into LDS once per workgroup (registers would spill;
  // a load at each tile's epilogue is a memory round trip there)
  __shared__ f32x4 epl[32];
  if (threadIdx.x < 32) {
    const X3EpiCol c = x3_epi_col(epi, eflags, threadIdx.x);
    epl[threadIdx.x] = f32x4{c.pb, c.pm, c.ps, c.pg};
  }

  // weights once: the packed [n/16][step][piece][lane][8] block of columns 0-31 is contiguous
  {
    u32x4 w[BPT];
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      int e = threadIdx.x + u * NT;
      e = e < BB / 16 ? e : BB / 16 - 1;
      w[u] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned char*>(Bt) + 16 * e);
    }
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      int e = threadIdx.x + u * NT;
      e = e < BB / 16 ? e : BB / 16 - 1;
      *reinterpret_cast<u32x4*>(smem + 16 * e) = w[u];
    }
  }

  // per-lane patch items (fixed per thread): pixel pr, channel quad q; dst in the split patch
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  auto tile_xy = [&](int t, int& b, int& y0, int& x0) {
    const int tx = t % tilesX, tt = t / tilesX, ty = tt % tilesY;
    b = tt / tilesY;
    y0 = ty * TH;
    x0 = tx * TW;
  };
  f32x4 stg[PPT];
  auto load_tile = [&](int t) {
    int b, y0, x0;
    tile_xy(t, b, y0, x0);
#pragma unroll
    for (int d = 0; d < PPT; ++d) {
      int e = threadIdx.x + d * NT;
      e = e < ITEMS ? e : ITEMS - 1;
      const int pr = e >> 2, q = e & 3, py = pr / PW2, px = pr - py * PW2;
      const int iy = y0 - 1 + py, ix = x0 - 1 + px;
      const bool ok = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      const unsigned vo = ok ? (unsigned)((((b * g.H + iy) * g.W + ix) * 16 + 4 * q) * 4) : OOB_OFF;
      stg[d] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, vo, 0, 0));
    }
  };
  auto split_tile = [&]() {  // 16-B fp32 channel quad -> three 8-B bf16 quads (pieces at 32 p + 8 q)
    bool ok = true;
#pragma unroll
    for (int d = 0; d < PPT; ++d)
#pragma unroll
      for (int c = 0; c < 4; ++c) ok = ok && x3_split_ok(stg[d][c]);
    const bool fast = __builtin_amdgcn_ballot_w64(!ok) == 0;  // (pairs of one v_cvt_pk per piece)
#pragma unroll
    for (int d = 0; d < PPT; ++d) {
      int e = threadIdx.x + d * NT;
      e = e < ITEMS ? e : ITEMS - 1;
      const int dst = (e >> 2) * PB + 8 * (e & 3);
      uint2 w[3];
      if constexpr ((X3DIAG & 128) != 0) {  // (diagnostic: truncating 2-piece "split", 2 v_perm per pair)
        const unsigned a0 = __builtin_bit_cast(unsigned, stg[d][0]), a1 = __builtin_bit_cast(unsigned, stg[d][1]);
        const unsigned a2 = __builtin_bit_cast(unsigned, stg[d][2]), a3 = __builtin_bit_cast(unsigned, stg[d][3]);
        w[0] = uint2{__builtin_amdgcn_perm(a1, a0, 0x07060302u), __builtin_amdgcn_perm(a3, a2, 0x07060302u)};
        w[1] = uint2{__builtin_amdgcn_perm(a1, a0, 0x05040100u), __builtin_amdgcn_perm(a3, a2, 0x05040100u)};
        w[2] = uint2{0u, 0u};
        (void)fast;
      } else {
        split3_pack2(fast, stg[d][0], stg[d][1], w[0].x, w[1].x, w[2].x);
        split3_pack2(fast, stg[d][2], stg[d][3], w[0].y, w[1].y, w[2].y);
      }
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(patch + dst + 32 * p) = w[p];
    }
  };

  // fragment rows (fixed per lane): the pixel of tap (1, 1) of row (wm TM + i) 16 + fr
  // (packed two per register: byte offsets < PR PB < 2^16; the other offsets are uniform or per lane)
  constexpr int NPP = (TM + 1) / 2;
  static_assert(PR * PB < 65536, "16-bit patch offsets");
  unsigned prow2[NPP];
#pragma unroll
  for (int k = 0; k < NPP; ++k) prow2[k] = 0;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int r = (wm * TM + i) * 16 + fr;
    r = r < T ? r : T - 1;
    int ly, lx;
    if constexpr (POOL) {
      const int w = r >> 2, q = r & 3;
      ly = 2 * (w / (TW / 2)) + (q >> 1);
      lx = 2 * (w % (TW / 2)) + (q & 1);
    } else {
      ly = r / TW;
      lx = r % TW;
    }
    prow2[i / 2] |= (unsigned)(((ly + 1) * PW2 + lx + 1) * PB) << (16 * (i % 2));
  }
  auto prow = [&](int i) {
    unsigned w = prow2[i / 2];
    asm volatile("" : "+v"(w));
    return (int)((w >> (16 * (i % 2))) & 0xffffu);
  };
  const int fqo = 16 * (fq & 1);
  auto toff = [&](int s) {  // this lane's tap offset (bytes) in full step s
    const int ta = 2 * s, tb = 2 * s + 1 < 9 ? 2 * s + 1 : 8;
    const int oa = ((ta / 3 - 1) * PW2 + (ta % 3 - 1)) * PB, ob = ((tb / 3 - 1) * PW2 + (tb % 3 - 1)) * PB;
    return th ? ob : oa;
  };
  auto frag = [&](int i, int off, bf16x8 (&a)[3]) {
    const unsigned char* q = patch + prow(i) + fqo + off;
#pragma unroll
    for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(q + 32 * p);
  };
  auto bfrag = [&](int s, bf16x8 (&bb)[3][2]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bb[p][j] = *reinterpret_cast<const bf16x8*>(smem + (j * NS * 3 + s * 3 + p) * 1024 + lane * 16);
  };
  // HALF: the K = 16 step (tap 8, channels 4 fq .. 4 fq + 3): A 8 B at the lane's pixel + tap 8,
  // B 8 B of the packed step 4 (lane fr + 16 (fq >> 1), element 4 (fq & 1))
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  const int hoff = (PW2 + 1) * PB + 8 * fq;  // tap (2, 2) relative to (1, 1), 8 fq in the pixel
  const int hb = (fr + 16 * (fq >> 1)) * 16 + 8 * (fq & 1);

  const int G = gridDim.x;
  int t = blockIdx.x;
#if (X3DIAG & 32) != 0  // per-phase s_memtime sums (c16_diag_stamps)
  unsigned long long dg[C16_DIAG_SLOTS] = {}, dg_t1 = 0;
#define C16_STAMP(k)                                             \
  {                                                              \
    const unsigned long long now = __builtin_amdgcn_s_memtime(); \
    dg[k] += now - dg_t1;                                        \
    dg_t1 = now;                                                 \
  }
#else
#define C16_STAMP(k)
#endif
  if (t < ntiles) load_tile(t);
  while (t < ntiles) {
#if (X3DIAG & 32) != 0
    dg_t1 = __builtin_amdgcn_s_memtime();
    ++dg[8];
#endif
    int b, y0, x0;
    tile_xy(t, b, y0, x0);
    // all of this wave's memory operations retired: the staged loads, and the previous tile's
    // stores (X3DIAG 32: ~80 cycles, they are done by now).  (Round 4, measured: leaving those
    // stores in flight -- a fixed store count per wave, so that the wait could leave them
    // outstanding -- made the next tile's patch loads, issued behind them, ~10k cycles slower
    // per tile: conv1 0.152 -> 0.19 ms.)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    C16_STAMP(0)
    split_tile();
    for (int r = threadIdx.x; r < NO; r += NT) {
      int o;
      if constexpr (POOL) {
        const int py = (y0 >> 1) + r / (TW / 2), px = (x0 >> 1) + r % (TW / 2);
        o = (py >= g.PH || px >= g.PW) ? -1
            : g.out_mode == 1         ? (b * (g.PH + 2) + py + 1) * (g.PW + 2) + px + 1
                                      : (b * g.PH + py) * g.PW + px;
      } else {
        const int oy = y0 + r / TW, ox = x0 + r % TW;
        o = (oy >= g.H || ox >= g.W) ? -1 : g.out_mode == 1 ? (b * (g.H + 2) + oy + 1) * Wp + ox + 1 : (b * g.H + oy) * g.W + ox;
      }
      orow[r] = o;
    }
    const int tn = t + G;
    if (tn < ntiles) load_tile(tn);  // in flight during this tile's MFMAs
    C16_STAMP(1)
    __syncthreads();                 // the patch, the row table (and, first time, the weights) written
    C16_STAMP(2)

    f32x4 acc[TM][2], accc[TM][2];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = accc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int NSF = HALF ? NS - 1 : NS;  // full 16x16x32 steps
    // B fragments single-buffered (read at each step's start; the other workgroup's waves cover
    // the latency): the staging registers of the next tile take the second buffer's room
    bf16x8 af[2][3], bq[3][2];
    frag(0, toff(0), af[0]);
#pragma unroll
    for (int s = 0; s < NSF; ++s) {
      const int off = toff(s), off_next = toff(s + 1 < NSF ? s + 1 : s);
      bfrag(s, bq);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int cur = (s * TM + i) & 1, nxt = cur ^ 1;
        if (i + 1 < TM)
          frag(i + 1, off, af[nxt]);
        else if (s + 1 < NSF)
          frag(0, off_next, af[nxt]);
        const bf16x8(&bb)[3][2] = bq;
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) x3_step<true>(acc[i][jb], accc[i][jb], af[cur], bb, jb);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (HALF) {
      s16x4 hbq[3][2];
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          hbq[p][j] = *reinterpret_cast<const s16x4*>(smem + (j * NS * 3 + 4 * 3 + p) * 1024 + hb);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int pr = prow(i);
        s16x4 a[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const s16x4*>(patch + pr + hoff + 32 * p);
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
          f32x4 c = accc[i][jb];
          c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[2], hbq[0][jb], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[1], hbq[1][jb], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[0], hbq[2][jb], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[1], hbq[0][jb], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[0], hbq[1][jb], c, 0, 0, 0);
          accc[i][jb] = c;
          acc[i][jb] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[0], hbq[0][jb], acc[i][jb], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    x3_fold(acc, accc);
    C16_STAMP(3)
    __syncthreads();  // every wave is done with the patch: the epilogue stages reuse it
    C16_STAMP(4)

    if constexpr (POOL) {
      if (g.out_mode == 1) {  // staged 16-B split-plane stores (x3_pool_split_store)
        float* stgp = reinterpret_cast<float*>(patch) + wm * (TM * 4 * X3_STG_ROW);
        float epb[2], epm[2], eps[2], epg[2];
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
          const f32x4 e = epl[16 * jb + fr];
          epb[jb] = e[0], epm[jb] = e[1], eps[jb] = e[2], epg[jb] = e[3];
        }
        if constexpr ((X3DIAG & 64) != 0) {  // (diagnostic: no pool / epilogue math)
#pragma unroll
          for (int jb = 0; jb < 2; ++jb)
#pragma unroll
            for (int i = 0; i < TM; ++i) stgp[(4 * i + fq) * X3_STG_ROW + 16 * jb + fr] = acc[i][jb][0] + epb[jb];
        } else {
          pool_epilogue_batch<FL>(acc, epb, epm, eps, epg, epi.flags,
                                  [&](int i, int jb, float v) { stgp[(4 * i + fq) * X3_STG_ROW + 16 * jb + fr] = v; });
        }
        C16_STAMP(5)
        x3_pool_split_store<TM>(stgp, orow, NO, 4 * wm * TM, out_split, 96, 0, lane);
        C16_STAMP(6)
        __syncthreads();  // stages read before the next tile's split overwrites the patch area
        C16_STAMP(7)
        t = tn;
        continue;
      }
    }
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
      const int n = 16 * jb + fr;
      const float pb = (eflags & EPI_BIAS) ? epi.bias[n] : 0.f;
      const float pm = (eflags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
      const float ps = (eflags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
      const float pg = (eflags & EPI_BN) ? epi.gamma[n] : 1.f;
      auto put = [&](int o, float v) {
        if (g.out_mode == 1) {
          unsigned short s0, s1, s2;
          split3(v, s0, s1, s2);
          bf16_bits* d = out_split + (size_t)o * 96 + n;
          d[0] = s0;
          d[32] = s1;
          d[64] = s2;
        } else {
          out[(size_t)o * N + n] = v;
        }
      };
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int rb = 16 * (wm * TM + i);
        if constexpr (POOL) {
          const int w = rb / 4 + fq;
          const int o = w < NO ? orow[w] : -1;
          if (o >= 0) put(o, pool_then_epilogue_t<FL>(acc[i][jb], pb, pm, ps, pg, epi.flags));
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = rb + 4 * fq + r;
            const int o = row < NO ? orow[row] : -1;
            if (o >= 0) put(o, apply_epilogue_t<FL>(acc[i][jb][r], pb, pm, ps, pg, epi.flags));
          }
        }
      }
    }
    __syncthreads();  // the row table is rewritten by the next tile
    t = tn;
  }
#if (X3DIAG & 32) != 0
  if (threadIdx.x == 0 && blockIdx.x < C16_DIAG_WGS) {  // (vector stores from lane 0)
    unsigned long long* d = c16_diag_stamps + C16_DIAG_SLOTS * blockIdx.x;
#pragma unroll
    for (int k = 0; k < C16_DIAG_SLOTS; ++k) d[k] = dg[k];
  }
#endif
#undef C16_STAMP
}


// Ping-pong form of the persistent 16-channel kernel (round 6: conv1 at batch grids).  The c16p
// stamps (round 4): per tile the split of the staged fp32 patch (~4.7 k cycles), the MFMAs (~9.6 k,
// ~6 k of them the wave's own) and the pool / epilogue / split-plane stores (~6 k) run one after
// the other in each workgroup, and two independent workgroups per CU line them up at random (MFMA
// pipes ~57 % busy).  Here ONE workgroup per CU runs two teams of 4 waves (one wave of each team
// per SIMD) over a contiguous range of the CU's tiles (team A the even ones, team B the odd ones)
// in lock step, as conv3x3_x3_pp_kernel: every step ends at a workgroup barrier; in each step one
// team runs its MFMAs (at issue priority 1) while the other runs its store step -- issue the loads
// of its next tile's fp32 patch into registers, fold, pool + epilogue through the stage and store
// the pooled split planes of the tile it just computed, then split the next patch into the team's
// patch area (the loads' latency under the epilogue; no staging registers live in the MFMA step,
// which reads the next K step's B fragments during the current one instead).  LDS: the 30 KB of weights once (both
// teams), one split patch per team (48 KB each), one stage area (the store steps never overlap),
// 150 KB in all.  Products, order and epilogue per output are conv3x3_x3_c16p_kernel<true, true>'s:
// the same bits (tested).
template <int FL = -1>
__global__ void __launch_bounds__(512, 1)
conv3x3_x3_c16pp_kernel(const float* __restrict__ in, const bf16_bits* __restrict__ Bt,
                        bf16_bits* __restrict__ out_split, EpiParams epi, int tilesX, int tilesY, int ntiles,
                        X3Geom g, unsigned in_bytes, int ppprio) {
  constexpr int TH = 16, TW = 26, WM = 4, TM = 7;
  constexpr int NT = 64 * WM, PB = 96, PW2 = TW + 2, PR = (TH + 2) * PW2, T = TH * TW, NS = 5;
  constexpr int ITEMS = PR * 4, PPT = (ITEMS + NT - 1) / NT;  // item = (patch pixel, channel quad), per team
  constexpr int BB = 2 * NS * 3 * 1024, BPT = (BB / 16 + 2 * NT - 1) / (2 * NT);
  constexpr int NO = T / 4, PATCH = PR * PB, STGW = TM * 4 * X3_STG_ROW;  // stage floats per wave
  static_assert(WM * TM * 16 >= T && (WM * TM - 3) * 16 < T && PPT == 8, "shape");
  static_assert(BB + 2 * PATCH + WM * STGW * 4 + 32 * 16 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[BB + 2 * PATCH + WM * STGW * 4];
  __shared__ f32x4 epl[32];

  const int lane = threadIdx.x & 63;
  const int eflags = FL < 0 ? epi.flags : FL;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int team = wid >> 2, wm = wid & 3, tt = threadIdx.x & (NT - 1);
  const int fr = lane & 15, fq = lane >> 4, th = fq >> 1;
  unsigned char* const patch = smem + BB + team * PATCH;
  float* const stgp = reinterpret_cast<float*>(smem + BB + 2 * PATCH) + wm * STGW;
  // this workgroup's tiles [lo, hi) (balanced, XCD-local order); the team's k-th is lo + team + 2 k
  const int wg = xcd_tile(blockIdx.x, gridDim.x);
  const int lo = (int)((long long)ntiles * wg / gridDim.x), hi = (int)((long long)ntiles * (wg + 1) / gridDim.x);
  const int nmine = (hi - lo - team + 1) / 2;

  if (threadIdx.x < 32) {
    const X3EpiCol c = x3_epi_col(epi, eflags, threadIdx.x);
    epl[threadIdx.x] = f32x4{c.pb, c.pm, c.ps, c.pg};
  }
  {  // weights once (both teams): the packed [n/16][step][piece][lane][8] block of columns 0-31
    u32x4 w[BPT];
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      int e = threadIdx.x + u * 2 * NT;
      e = e < BB / 16 ? e : BB / 16 - 1;
      w[u] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned char*>(Bt) + 16 * e);
    }
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      int e = threadIdx.x + u * 2 * NT;
      e = e < BB / 16 ? e : BB / 16 - 1;
      *reinterpret_cast<u32x4*>(smem + 16 * e) = w[u];
    }
  }

  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  auto tile_of = [&](int k, int& b, int& y0, int& x0) {
    const int t = lo + team + 2 * k;
    const int tx = t % tilesX, t2 = t / tilesX, ty = t2 % tilesY;
    b = t2 / tilesY;
    y0 = ty * TH;
    x0 = tx * TW;
  };
  f32x4 stg[PPT];
  auto load_tile = [&](int k) {
    int b, y0, x0;
    tile_of(k, b, y0, x0);
#pragma unroll
    for (int d = 0; d < PPT; ++d) {
      int e = tt + d * NT;
      e = e < ITEMS ? e : ITEMS - 1;
      const int pr = e >> 2, q = e & 3, py = pr / PW2, px = pr - py * PW2;
      const int iy = y0 - 1 + py, ix = x0 - 1 + px;
      const bool ok = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      const unsigned vo = ok ? (unsigned)((((b * g.H + iy) * g.W + ix) * 16 + 4 * q) * 4) : OOB_OFF;
      stg[d] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, vo, 0, 0));
    }
  };
  auto split_tile = [&]() {  // 16-B fp32 channel quad -> three 8-B bf16 quads (pieces at 32 p + 8 q)
    bool ok = true;
#pragma unroll
    for (int d = 0; d < PPT; ++d)
#pragma unroll
      for (int c = 0; c < 4; ++c) ok = ok && x3_split_ok(stg[d][c]);
    const bool fast = __builtin_amdgcn_ballot_w64(!ok) == 0;
#pragma unroll
    for (int d = 0; d < PPT; ++d) {
      int e = tt + d * NT;
      e = e < ITEMS ? e : ITEMS - 1;
      const int dst = (e >> 2) * PB + 8 * (e & 3);
      uint2 w[3];
      split3_pack2(fast, stg[d][0], stg[d][1], w[0].x, w[1].x, w[2].x);
      split3_pack2(fast, stg[d][2], stg[d][3], w[0].y, w[1].y, w[2].y);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(patch + dst + 32 * p) = w[p];
    }
  };

  // fragment rows as conv3x3_x3_c16p_kernel (pool-window-major rows)
  constexpr int NPP = (TM + 1) / 2;
  static_assert(PR * PB < 65536, "16-bit patch offsets");
  unsigned prow2[NPP];
#pragma unroll
  for (int k = 0; k < NPP; ++k) prow2[k] = 0;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int r = (wm * TM + i) * 16 + fr;
    r = r < T ? r : T - 1;
    const int w = r >> 2, q = r & 3;
    const int ly = 2 * (w / (TW / 2)) + (q >> 1), lx = 2 * (w % (TW / 2)) + (q & 1);
    prow2[i / 2] |= (unsigned)(((ly + 1) * PW2 + lx + 1) * PB) << (16 * (i % 2));
  }
  auto prow = [&](int i) {
    unsigned w = prow2[i / 2];
    asm volatile("" : "+v"(w));
    return (int)((w >> (16 * (i % 2))) & 0xffffu);
  };
  const int fqo = 16 * (fq & 1);
  auto toff = [&](int s) {
    const int ta = 2 * s, tb = 2 * s + 1 < 9 ? 2 * s + 1 : 8;
    const int oa = ((ta / 3 - 1) * PW2 + (ta % 3 - 1)) * PB, ob = ((tb / 3 - 1) * PW2 + (tb % 3 - 1)) * PB;
    return th ? ob : oa;
  };
  auto frag = [&](int i, int off, bf16x8 (&a)[3]) {
    const unsigned char* q = patch + prow(i) + fqo + off;
#pragma unroll
    for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(q + 32 * p);
  };
  auto bfrag = [&](int s, bf16x8 (&bb)[3][2]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bb[p][j] = *reinterpret_cast<const bf16x8*>(smem + (j * NS * 3 + s * 3 + p) * 1024 + lane * 16);
  };
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  const int hoff = (PW2 + 1) * PB + 8 * fq;
  const int hb = (fr + 16 * (fq >> 1)) * 16 + 8 * (fq & 1);

  // prologue: each team's first patch split into its area
  if (nmine > 0) {
    load_tile(0);
    split_tile();
  }
  __syncthreads();  // weights, epl, both teams' first patches

  const int nA = (hi - lo + 1) / 2, nB = (hi - lo) / 2;
  const int nsteps = 2 * nA > 2 * nB + 1 ? 2 * nA : 2 * nB + 1;
#if (X3DIAG & 32768) != 0
  unsigned long long dg[4] = {0, 0, 0, 0}, t_in = __builtin_amdgcn_s_memtime(), t_start = t_in;
#define C16PP_MARK(slot)                                           \
  {                                                                \
    const unsigned long long t_now = __builtin_amdgcn_s_memtime(); \
    dg[slot] += t_now - t_in;                                      \
    t_in = t_now;                                                  \
  }
#else
#define C16PP_MARK(slot)
#endif
  if (team == 1) {
    C16PP_MARK(2)
    __syncthreads();
    C16PP_MARK(3)
  }
  for (int k = 0; k < nmine; ++k) {
    f32x4 acc[TM][2], accc[TM][2];
    {  // MFMA step of tile k (conv3x3_x3_c16p_kernel's loop)
      if (ppprio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = accc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      // (unlike the two-workgroup kernel, no other MFMA wave shares the SIMD to cover a stall, so the
      // next step's B fragments are read during this step -- two sets -- and the K = 16 step's A
      // fragments one block ahead)
      constexpr int NSF = NS - 1;  // full 16x16x32 steps; tap 8 alone on 16x16x16 below
      bf16x8 af[2][3], bq[2][3][2];
      s16x4 hbq[3][2];
      frag(0, toff(0), af[0]);
      bfrag(0, bq[0]);
#pragma unroll
      for (int s = 0; s < NSF; ++s) {
        const int off = toff(s), off_next = toff(s + 1 < NSF ? s + 1 : s);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int cur = (s * TM + i) & 1, nxt = cur ^ 1;
          if (i == 0 && s + 1 < NSF) bfrag(s + 1, bq[(s + 1) & 1]);
          if (i == 0 && s + 1 == NSF) {
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
              for (int j = 0; j < 2; ++j)
                hbq[p][j] = *reinterpret_cast<const s16x4*>(smem + (j * NS * 3 + 4 * 3 + p) * 1024 + hb);
          }
          if (i + 1 < TM)
            frag(i + 1, off, af[nxt]);
          else if (s + 1 < NSF)
            frag(0, off_next, af[nxt]);
#pragma unroll
          for (int jb = 0; jb < 2; ++jb) x3_step<true>(acc[i][jb], accc[i][jb], af[cur], bq[s & 1], jb);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      s16x4 ha[2][3];
      auto hfrag = [&](int i, s16x4 (&a)[3]) {
        const int pr = prow(i);
#pragma unroll
        for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const s16x4*>(patch + pr + hoff + 32 * p);
      };
      hfrag(0, ha[0]);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (i + 1 < TM) hfrag(i + 1, ha[(i + 1) & 1]);
        const s16x4(&a)[3] = ha[i & 1];
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
          f32x4 c = accc[i][jb];
          c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[2], hbq[0][jb], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[1], hbq[1][jb], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[0], hbq[2][jb], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[1], hbq[0][jb], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[0], hbq[1][jb], c, 0, 0, 0);
          accc[i][jb] = c;
          acc[i][jb] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[0], hbq[0][jb], acc[i][jb], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      wait_lgkm0();
      if (ppprio) __builtin_amdgcn_s_setprio(0);
    }
    C16PP_MARK(0)
    __syncthreads();  // the team's patch is read by all its waves (and the other team's store step is done)
    C16PP_MARK(3)
    {  // store step: tile k + 1's fp32 patch loaded, tile k's pooled split planes out, tile k + 1 split
      // into the team's patch area (the loads in flight under the epilogue and stores; the
      // compiler's wait before the split counts the stores issued after them)
      if (k + 1 < nmine) load_tile(k + 1);
      x3_fold(acc, accc);
      int b, y0, x0;
      tile_of(k, b, y0, x0);
      float epb[2], epm[2], eps[2], epg[2];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        const f32x4 e = epl[16 * jb + fr];
        epb[jb] = e[0], epm[jb] = e[1], eps[jb] = e[2], epg[jb] = e[3];
      }
      pool_epilogue_batch<FL>(acc, epb, epm, eps, epg, epi.flags,
                              [&](int i, int jb, float v) { stgp[(4 * i + fq) * X3_STG_ROW + 16 * jb + fr] = v; });
      auto orow_of = [&](int w) {
        const int py = (y0 >> 1) + w / (TW / 2), px = (x0 >> 1) + w % (TW / 2);
        return (py >= g.PH || px >= g.PW) ? -1 : (b * (g.PH + 2) + py + 1) * (g.PW + 2) + px + 1;
      };
      x3_pool_split_store_f<TM>(stgp, orow_of, NO, 4 * wm * TM, out_split, 96, 0, lane);
      C16PP_MARK(2)
      if (k + 1 < nmine) split_tile();
      wait_lgkm0();  // the split patch written, the stage read
      C16PP_MARK(1)
    }
    __syncthreads();
    C16PP_MARK(3)
  }
  for (int st = team + 2 * nmine; st < nsteps; ++st) __syncthreads();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if (X3DIAG & 32768) != 0
  if ((threadIdx.x & 255) == 0 && blockIdx.x < C16PP_DIAG_WGS) {  // (vector stores from lane 0)
    unsigned long long* d = c16pp_diag_stamps + 16 * blockIdx.x + 4 * team;
    d[0] = dg[0], d[1] = dg[1], d[2] = dg[2], d[3] = dg[3];
    if (team == 0) {
      c16pp_diag_stamps[16 * blockIdx.x + 8] = __builtin_amdgcn_s_memtime() - t_start;
      c16pp_diag_stamps[16 * blockIdx.x + 9] = (unsigned long long)nmine;
    }
  }
#endif
#undef C16PP_MARK
}


// Narrow layers (N = 64 / 128: YOLOv2-tiny conv2 / conv3, 104x104 and 52x52 frames).  A run of
// consecutive rows spans whole image rows plus a two-row halo, so on wide frames the wide kernel
// (gemm_x3_acc2.h) would stage 2.2-5x its tile's pixels (x3_span); here a workgroup owns a 2-D
// tile of TH x TW output pixels and 32 WN columns, and stages its (TH + 2) x (TW + 2) patch.  WM x
// WN waves of TM 16-row blocks x 32 columns; tile rows raster, or pool-window-major (POOL: TH, TW
// even, so a 2x2 window never leaves its tile).  Rows past the tile (WM TM 16 > TH TW) and pixels
// past the frame compute on clamped rows and are not stored.  Weights straight from L2 to
// registers two steps ahead (a 3-step ring).  Round 4 layout, the wide kernel's: 224-B LDS pixel rows (the 192 data
// bytes of a 32-channel chunk + 32 never-read bytes; tools: 2.86 extra conflict cycles per
// fragment read at these tiles, the same as the 192-B rows' XOR swizzle, with plain offsets)
// filled by LDS-DMA (1 KiB pieces, per-lane source = its pixel row's chunk + 16 u, no staging
// registers), so a fragment address is a per-block register + a tap offset that is an
// instruction immediate (no per-fragment multiply, XOR or shift: the old loop spent ~6 VALU per
// fragment, one a quarter-rate v_mul_lo).  Chunk j + 1 is DMA'd into the other buffer when chunk
// j starts (NBUF = 2) or after it (NBUF = 1, one buffer).  Two accumulators per output (A2) for
// every configuration.  (Rounds 2-3: register-staged 192-B rows with an XOR swizzle, per-step adds
// for N = 128: conv3 0.127 -> 0.114 ms, conv2 0.129 -> 0.126 ms with this form; git history.)
template <int TH, int TW, int WM, int WN, int TM, int NBUF, bool POOL, int FL = -1>
__global__ void __launch_bounds__(64 * WM * WN, 512 / (64 * WM * WN))
conv3x3_x3_tile2_kernel(const bf16_bits* __restrict__ in, const bf16_bits* __restrict__ Bt, float* __restrict__ out,
                        bf16_bits* __restrict__ out_split, int N, int K, EpiParams epi, int tilesX, int tilesY,
                        int tilesN, X3Geom g, unsigned in_bytes, unsigned b_bytes) {
  constexpr int NW = WM * WN, NT = 64 * NW, LP = 224, PU = LP / 16, PW2 = TW + 2, PR = (TH + 2) * PW2, T = TH * TW;
  constexpr int NPC = (PR * PU + 63) / 64, NPW = (NPC + NW - 1) / NW;  // 1-KiB DMA pieces per chunk / per wave
  constexpr int BUFB = NPW * NW * 1024;
  static_assert(TH % 2 == 0 && TW % 2 == 0 && WM * TM * 16 >= T && (WM * TM - 2) * 16 < T && (NBUF == 1 || NBUF == 2) &&
                    NPW <= 24,
                "shape");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NBUF * BUFB];
  // batch tiles: the workgroup's 32 WN columns' epilogue parameters, loaded into LDS at the start
  // (a load issued at the epilogue is a memory round trip of ~2 k cycles there, tile2 stamps), in
  // the last buffer's unused tail: the DMA pieces past the patch (NPC) are not issued, and the
  // LDS stays at two workgroups per CU (conv3's pair fills the 160 KiB exactly)
  static_assert(TM <= 2 || (NPW * NW - NPC) * 1024 >= 32 * WN * 16, "epilogue parameters in the buffer tail");
  f32x4* const epl = reinterpret_cast<f32x4*>(smem + NBUF * BUFB - 32 * WN * 16);

  const int lane = threadIdx.x & 63;
  const int eflags = FL < 0 ? epi.flags : FL;  // FL: the epilogue flag set compiled in (-1: runtime)
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int wn = wid % WN, wm = wid / WN;
  int t = xcd_tile(blockIdx.x, gridDim.x);
  const int tn = t % tilesN;
  t /= tilesN;
  const int tx = t % tilesX;
  t /= tilesX;
  const int ty = t % tilesY;
  const int b = t / tilesY;
  const int y0 = ty * TH, x0 = tx * TW;
  const int n0 = tn * (32 * WN) + wn * 32;
  const int Wp = g.W + 2;
  const int fr = lane & 15, fq = lane >> 4;
  T2_STAMP(0, __builtin_amdgcn_s_memrealtime())
  T2_STAMP(1, __builtin_amdgcn_s_memtime())
  T2_STAMP(6, (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)))
  T2_STAMP(7, (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11)))

  // fragment rows: byte offset of the lane's tap-(0, 0) pixel row of block i (+ 16 fq)
  int rowoff[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int r = (wm * TM + i) * 16 + fr;
    r = r < T ? r : T - 1;
    int ly, lx;
    if constexpr (POOL) {
      const int w = r >> 2, q = r & 3;
      ly = 2 * (w / (TW / 2)) + (q >> 1);
      lx = 2 * (w % (TW / 2)) + (q & 1);
    } else {
      ly = r / TW;
      lx = r % TW;
    }
    rowoff[i] = (ly * PW2 + lx) * LP + 16 * fq;
  }

  // patch DMA: piece k of this wave covers LDS units U = 64 (wid + NW k) + lane = pixel row r =
  // U / PU (rows past the patch repeat the last), unit u = U % PU; source = the padded pixel
  // (y0 + r / PW2, x0 + r % PW2) of image b, chunk c, + 16 u (units 12, 13: the next 32 bytes)
  const int nk = K / 32, nch = nk / 9;
  const unsigned rowB = 6u * (unsigned)g.C;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  const unsigned pbase = (unsigned)((b * (g.H + 2) + y0) * Wp + x0);  // padded pixel of patch (0, 0)
  auto issue_chunk = [&](int c, int buf) {
#pragma unroll
    for (int k = 0; k < NPW; ++k) {
      if (wid + NW * k >= NPC) break;  // (wave-uniform: pieces past the patch hold no read row)
      const unsigned U = 64u * (unsigned)(wid + NW * k) + (unsigned)lane;
      unsigned r = U / PU;
      const unsigned u = U - r * PU;
      r = r < (unsigned)PR ? r : (unsigned)PR - 1;
      const unsigned py = r / PW2, px = r - py * PW2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsA, (__attribute__((address_space(3))) void*)(smem + buf * BUFB + 1024 * (wid + NW * k)), 16,
          (int)((pbase + py * (unsigned)Wp + px) * rowB + 16u * u), (int)(c * 192), 0, 0);
    }
  };

  const unsigned bvo = (unsigned)((n0 / 16) * nk * 3072 + lane * 16);
  const int bjs = nk * 3072;
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)b_bytes, 0x00020000);
  bf16x8 bq[3][3][2];
  auto load_b = [&](int s, bf16x8 (&dst)[3][2]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        dst[p][j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, bvo, s * 3072 + p * 1024 + j * bjs, 0));
  };

  f32x4 acc[TM][2], accc[TM][2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = accc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_chunk(0, 0);
  load_b(0, bq[0]);
  load_b(1, bq[1]);
  // small tiles (the single-frame plans): the epilogue parameters with the first operands
  constexpr bool PREP = TM <= 2;
  X3EpiCol ecp[2] = {};
  if constexpr (!PREP) {
    if (threadIdx.x < 32 * WN) {
      const X3EpiCol c = x3_epi_col(epi, eflags, tn * (32 * WN) + threadIdx.x);
      epl[threadIdx.x] = f32x4{c.pb, c.pm, c.ps, c.pg};
    }
  }
  if constexpr (PREP) {
    ecp[0] = x3_epi_col(epi, eflags, n0 + fr);
    ecp[1] = x3_epi_col(epi, eflags, n0 + 16 + fr);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  T2_STAMP(2, __builtin_amdgcn_s_memtime())

  auto frag = [&](const unsigned char* P, int i, int tap, bf16x8 (&a)[3]) {
    const int toff = ((tap / 3) * PW2 + (tap % 3)) * LP;
    const unsigned char* q = P + rowoff[i] + toff;
#pragma unroll
    for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(q + 64 * p);
  };
  for (int j = 0; j < nch; ++j) {
    const unsigned char* P = smem + (NBUF == 2 ? (j & 1) : 0) * BUFB;
    if (NBUF == 2 && j + 1 < nch) issue_chunk(j + 1, (j + 1) & 1);  // the other buffer: read in chunk j - 1
    bf16x8 af[2][3];
    frag(P, 0, 0, af[0]);
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int s = 9 * j + tp;
      __builtin_amdgcn_sched_barrier(0);
      load_b(s + 2, bq[(tp + 2) % 3]);  // (past the last step: unused, in-range or zero-filled)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int cur = i & 1, nxt = cur ^ 1;
        if (i + 1 < TM)
          frag(P, i + 1, tp, af[nxt]);
        else if (tp < 8)
          frag(P, 0, tp + 1, af[nxt]);
        const bf16x8(&bb)[3][2] = bq[tp % 3];
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) x3_step<true>(acc[i][jb], accc[i][jb], af[cur], bb, jb);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (TM & 1) {
        if (tp < 8) {
#pragma unroll
          for (int p = 0; p < 3; ++p) af[0][p] = af[1][p];
        }
      }
    }
    // the ring holds steps s + 1, s + 2 in slots (tp + 1) % 3 = 0 and 1 for the next chunk (9 % 3 == 0)
    if (j + 1 < nch) {
      if constexpr (NBUF == 1) {
        wait_lgkm0();
        __syncthreads();  // every wave done with the patch
        issue_chunk(j + 1, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      wait_lgkm0();
      __syncthreads();  // chunk j + 1 landed (every wave's pieces); chunk j read by every wave
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  T2_STAMP(3, __builtin_amdgcn_s_memtime())
  T2_STAMPW(8, __builtin_amdgcn_s_memtime())

  x3_fold(acc, accc);
  int* orow = reinterpret_cast<int*>(smem);
  __syncthreads();
  T2_STAMP(12, __builtin_amdgcn_s_memtime())
  constexpr int NO = POOL ? T / 4 : T;
  for (int r = threadIdx.x; r < NO; r += NT) {
    int o;
    if constexpr (POOL) {
      const int py = (y0 >> 1) + r / (TW / 2), px = (x0 >> 1) + r % (TW / 2);
      o = (py >= g.PH || px >= g.PW) ? -1
          : g.out_mode == 1         ? (b * (g.PH + 2) + py + 1) * (g.PW + 2) + px + 1
                                    : (b * g.PH + py) * g.PW + px;
    } else {
      const int oy = y0 + r / TW, ox = x0 + r % TW;
      o = (oy >= g.H || ox >= g.W) ? -1 : g.out_mode == 1 ? (b * (g.H + 2) + oy + 1) * Wp + ox + 1 : (b * g.H + oy) * g.W + ox;
    }
    orow[r] = o;
  }
  __syncthreads();
  T2_STAMP(13, __builtin_amdgcn_s_memtime())
  if constexpr (POOL) {
    if (g.out_mode == 1) {  // staged 16-B split-plane stores (x3_pool_split_store)
      static_assert(1024 + NW * TM * 4 * X3_STG_ROW * 4 <= NBUF * BUFB && NO * 4 <= 1024, "stage");
      float* stg = reinterpret_cast<float*>(smem + 1024) + wid * (TM * 4 * X3_STG_ROW);
      float pb[2], pm[2], ps[2], pg[2];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        X3EpiCol ec = ecp[jb];
        if constexpr (!PREP) {
          const f32x4 e = epl[wn * 32 + 16 * jb + fr];
          ec = X3EpiCol{e[0], e[1], e[2], e[3]};
        }
        pb[jb] = ec.pb, pm[jb] = ec.pm, ps[jb] = ec.ps, pg[jb] = ec.pg;
      }
      pool_epilogue_batch<FL>(acc, pb, pm, ps, pg, epi.flags,
                              [&](int i, int jb, float v) { stg[(4 * i + fq) * X3_STG_ROW + 16 * jb + fr] = v; });
      T2_STAMP(14, __builtin_amdgcn_s_memtime())
      x3_pool_split_store<TM>(stg, orow, NO, 4 * wm * TM, out_split, 3 * (size_t)N, (n0 >> 5) * 96, lane);
      T2_STAMP(4, __builtin_amdgcn_s_memtime())
      T2_STAMP(5, __builtin_amdgcn_s_memrealtime())
      return;
    }
  }
#pragma unroll
  for (int jb = 0; jb < 2; ++jb) {
    const int n = n0 + 16 * jb + fr;  // < N: N % (32 WN) == 0 (launcher)
    X3EpiCol ec = ecp[jb];
    if constexpr (!PREP) {
      const f32x4 e = epl[wn * 32 + 16 * jb + fr];
      ec = X3EpiCol{e[0], e[1], e[2], e[3]};
    }
    const float pb = ec.pb, pm = ec.pm, ps = ec.ps, pg = ec.pg;
    const int cofs = (n >> 5) * 96 + (n & 31);
    auto put = [&](int o, float v) {
      if (g.out_mode == 1) {
        unsigned short s0, s1, s2;
        split3(v, s0, s1, s2);
        bf16_bits* d = out_split + (size_t)o * (3 * N) + cofs;
        d[0] = s0;
        d[32] = s1;
        d[64] = s2;
      } else {
        out[(size_t)o * N + n] = v;
      }
    };
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rb = 16 * (wm * TM + i);
      if constexpr (POOL) {
        const int w = rb / 4 + fq;
        const int o = w < NO ? orow[w] : -1;
        if (o >= 0) put(o, pool_then_epilogue_t<FL>(acc[i][jb], pb, pm, ps, pg, epi.flags));
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb + 4 * fq + r;
          const int o = row < NO ? orow[row] : -1;
          if (o >= 0) put(o, apply_epilogue_t<FL>(acc[i][jb][r], pb, pm, ps, pg, epi.flags));
        }
      }
    }
  }
  T2_STAMP(4, __builtin_amdgcn_s_memtime())
  T2_STAMP(5, __builtin_amdgcn_s_memrealtime())
}
#undef T2_STAMP
#undef T2_STAMPW

// Ping-pong form of the narrow tile kernel for batch grids (round 5): conv2 of YOLOv2-tiny at batch
// 64 (N = 64, one 32-channel chunk, 8 x 26 tiles; the NCH / PU / SK parameters also took conv3's
// shape, bit-exact but slower than the tile kernel: kernels_x3.hip).
// tile2 stamps (tools/tile2_diag.py): a tile's workgroup spends ~5 k cycles waiting for its patch
// and ~6.6 k in the epilogue beside its MFMA loop; two independent workgroups per CU line those
// phases up at random.  Here ONE workgroup per CU runs two teams of WM x WN = 4 waves (one wave of
// each team per SIMD) over a contiguous range of the CU's tiles (team A the even ones, team B the
// odd ones) in lock step: every step ends at a workgroup barrier, and in each step one team runs
// its MFMA loop over the tile's chunks while the other stores its previous tile (fold, pool +
// epilogue through its waves' LDS stages, split-plane stores) and loads every chunk of its next
// patch and its first weights.  Per team the same loop as conv3x3_x3_tile2_kernel (same
// products and order, same epilogue): the same bits.  LDS per team: NCH patch buffers of PU-unit
// pixel rows, the image row skewed by SK units (conv2: 224-B rows; conv3: 192-B rows + 2, so
// that four buffers fit: 0.92 modelled extra cycles per fragment read either way); one stage area
// (the teams' store steps never overlap) and the epilogue parameters.  The row table is computed
// per window (no team-wide barrier inside a step).
template <int TH, int TW, int WM, int WN, int TM, int NCH, int PU, int SK, int FL = -1, int PPLEAD = 1>
__global__ void __launch_bounds__(512, 1)
conv3x3_x3_pp_kernel(const bf16_bits* __restrict__ in, const bf16_bits* __restrict__ Bt,
                     bf16_bits* __restrict__ out_split, int N, EpiParams epi, int tilesX, int tilesY, int ntiles,
                     X3Geom g, unsigned in_bytes, unsigned b_bytes, int ppprio) {
  constexpr int NW = WM * WN, PW2 = TW + 2, T = TH * TW, RU = PW2 * PU + SK;  // units per patch row
  constexpr int NPC = ((TH + 2) * RU + 63) / 64, NPW = (NPC + NW - 1) / NW;
  constexpr int BUFB = NPW * NW * 1024, STGB = NW * TM * 4 * X3_STG_ROW * 4, NO = T / 4, NK = 9 * NCH;
  static_assert(NW == 4 && PU >= 12 && TH % 2 == 0 && TW % 2 == 0 && WM * TM * 16 >= T && (WM * TM - 2) * 16 < T &&
                    NPW <= 24 && 2 * NCH * BUFB + STGB + 32 * WN * 16 <= 160 * 1024,
                "shape");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * NCH * BUFB + STGB];
  __shared__ f32x4 epl[32 * WN];

  const int lane = threadIdx.x & 63;
  const int eflags = FL < 0 ? epi.flags : FL;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int team = wid >> 2, wt = wid & 3;
  const int wn = wt % WN, wm = wt / WN;
  const int n0 = wn * 32;  // N = 32 WN (launcher)
  const int Wp = g.W + 2;
  const int fr = lane & 15, fq = lane >> 4;
  // this workgroup's tiles [lo, hi) (balanced, XCD-local order); the team's k-th is lo + team + 2 k
  const int wg = xcd_tile(blockIdx.x, gridDim.x);
  const int lo = (int)((long long)ntiles * wg / gridDim.x), hi = (int)((long long)ntiles * (wg + 1) / gridDim.x);
  const int nmine = (hi - lo - team + 1) / 2;
  unsigned char* const P = smem + team * NCH * BUFB;
  float* const stg = reinterpret_cast<float*>(smem + 2 * NCH * BUFB) + wt * (TM * 4 * X3_STG_ROW);

  int rowoff[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int r = (wm * TM + i) * 16 + fr;
    r = r < T ? r : T - 1;
    const int w = r >> 2, q = r & 3;
    const int ly = 2 * (w / (TW / 2)) + (q >> 1), lx = 2 * (w % (TW / 2)) + (q & 1);
    rowoff[i] = (ly * RU + lx * PU) * 16 + 16 * fq;
  }
  auto tile_of = [&](int k, int& b, int& y0, int& x0) {
    const int t = lo + team + 2 * k;
    const int tx = t % tilesX, tt = t / tilesX, ty = tt % tilesY;
    b = tt / tilesY;
    y0 = ty * TH;
    x0 = tx * TW;
  };

  // patch DMA: LDS unit U of a chunk's buffer = patch row U / RU, pixel (U % RU) / PU, unit
  // (U % RU) % PU; units past 12 of a pixel and the SK skew units read neighbouring bytes (never read)
  const unsigned rowB = 6u * (unsigned)g.C;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  auto issue_patch = [&](int k) {  // every chunk of the team's k-th tile into its buffers
    int b, y0, x0;
    tile_of(k, b, y0, x0);
    const unsigned pbase = (unsigned)((b * (g.H + 2) + y0) * Wp + x0);
    // (an opaque copy of the lane index: the per-piece row / unit arithmetic is recomputed per
    // tile instead of hoisted out of the tile loop into ~40 registers live across the MFMAs)
    unsigned ln = (unsigned)lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int kk = 0; kk < NPW; ++kk) {
      if (wt + NW * kk >= NPC) break;  // (wave-uniform)
      const unsigned U = 64u * (unsigned)(wt + NW * kk) + ln;
      unsigned jr = U / RU;
      const unsigned rem = U - jr * RU;
      unsigned px = rem / PU, u = rem - px * PU;
      if (px >= (unsigned)PW2) px = PW2 - 1, u = PU - 1;
      jr = jr < (unsigned)(TH + 2) ? jr : TH + 1;
      const int vo = (int)((pbase + jr * (unsigned)Wp + px) * rowB + 16u * u);
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsA, (__attribute__((address_space(3))) void*)(P + c * BUFB + 1024 * (wt + NW * kk)), 16, vo, c * 192, 0, 0);
    }
  };

  const unsigned bvo = (unsigned)((n0 / 16) * NK * 3072 + lane * 16);
  const int bjs = NK * 3072;
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)b_bytes, 0x00020000);
  bf16x8 bq[3][3][2];
  auto load_b = [&](int s, bf16x8 (&dst)[3][2]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        dst[p][j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, bvo, s * 3072 + p * 1024 + j * bjs, 0));
  };

  if (threadIdx.x < 32 * WN) {
    const X3EpiCol c = x3_epi_col(epi, eflags, threadIdx.x);
    epl[threadIdx.x] = f32x4{c.pb, c.pm, c.ps, c.pg};
  }
  if (nmine > 0) issue_patch(0);
  load_b(0, bq[0]);
  load_b(1, bq[1]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x4 acc[TM][2], accc[TM][2];
  auto frag = [&](const unsigned char* Pc, int i, int tap, bf16x8 (&a)[3]) {
    const int toff = ((tap / 3) * RU + (tap % 3) * PU) * 16;
    const unsigned char* q = Pc + rowoff[i] + toff;
#pragma unroll
    for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(q + 64 * p);
  };
  // team A: steps 0, 1 = MFMAs of tile 0, store of tile 0 (+ load of tile 1), ...; team B one step
  // later.  Each team's loop is MFMA step, barrier, store step, barrier (accumulators live within
  // an iteration only); the leading / trailing barriers pad both teams to the same step count
  const int nA = (hi - lo + 1) / 2, nB = (hi - lo) / 2;
  const int nsteps = 2 * nA > 2 * nB + 1 ? 2 * nA : 2 * nB + 1;
#if (X3DIAG & 2048) != 0
  unsigned long long dg[4] = {0, 0, 0, 0}, t_in = __builtin_amdgcn_s_memtime(), t_start = t_in;
  const bool dwave = (threadIdx.x & 255) == 0;
#define PP_MARK(slot)                                              \
  {                                                                \
    const unsigned long long t_now = __builtin_amdgcn_s_memtime(); \
    dg[slot] += t_now - t_in;                                      \
    t_in = t_now;                                                  \
  }
#else
#define PP_MARK(slot)
#endif
  if (team == 1) {
    PP_MARK(1)
    __syncthreads();
    PP_MARK(2)
  }
  for (int k = 0; k < nmine; ++k) {
    // MFMA step of tile k, at a higher issue priority than the other team's store step on the same
    // SIMDs (MI355X_MICROARCH: VALU issue between two waves goes by priority, then age)
    {
      if (ppprio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = accc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const unsigned char* Pc = P + c * BUFB;
        // fragments PPLEAD row blocks ahead through a ring of PPLEAD + 1 sets (9 TM a multiple of
        // the ring: every chunk starts at slot 0)
        constexpr int RING = PPLEAD + 1, NBC = 9 * TM;
        static_assert(NCH == 1 || NBC % RING == 0, "fragment ring phase per chunk");
        bf16x8 af[RING][3];
#pragma unroll
        for (int l = 0; l < PPLEAD; ++l) frag(Pc, l % TM, l / TM, af[l]);
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const int s = 9 * c + tp;
          __builtin_amdgcn_sched_barrier(0);
          // (X3DIAG 4096, diagnostic: step 0's weights for every step -- no weight loads in the loop)
          if (s + 2 < NK && (X3DIAG & 4096) == 0) load_b(s + 2, bq[(s + 2) % 3]);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const int bi = TM * tp + i;
            if (bi + PPLEAD < NBC) frag(Pc, (bi + PPLEAD) % TM, (bi + PPLEAD) / TM, af[(bi + PPLEAD) % RING]);
            const bf16x8(&bb)[3][2] = bq[(X3DIAG & 4096) != 0 ? 0 : s % 3];
#pragma unroll
            for (int jb = 0; jb < 2; ++jb) x3_step<true>(acc[i][jb], accc[i][jb], af[bi % RING], bb, jb);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      wait_lgkm0();
      if (ppprio) __builtin_amdgcn_s_setprio(0);
    }
    PP_MARK(0)
    __syncthreads();
    PP_MARK(2)
    // store step: tile k out, tile k + 1's patch and first weights in
    {
      if (k + 1 < nmine) issue_patch(k + 1);
      x3_fold(acc, accc);
      int b, y0, x0;
      tile_of(k, b, y0, x0);
      float pb[2], pm[2], ps[2], pg[2];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        const f32x4 e = epl[n0 + 16 * jb + fr];
        pb[jb] = e[0], pm[jb] = e[1], ps[jb] = e[2], pg[jb] = e[3];
      }
      pool_epilogue_batch<FL>(acc, pb, pm, ps, pg, epi.flags,
                              [&](int i, int jb, float v) { stg[(4 * i + fq) * X3_STG_ROW + 16 * jb + fr] = v; });
      auto orow_of = [&](int w) {
        const int py = (y0 >> 1) + w / (TW / 2), px = (x0 >> 1) + w % (TW / 2);
        return (py >= g.PH || px >= g.PW) ? -1 : (b * (g.PH + 2) + py + 1) * (g.PW + 2) + px + 1;
      };
      x3_pool_split_store_f<TM>(stg, orow_of, NO, 4 * wm * TM, out_split, 3 * (size_t)N, (n0 >> 5) * 96, lane);
      if (k + 1 < nmine) {
        load_b(0, bq[0]);  // (after the epilogue: registers)
        load_b(1, bq[1]);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's patch pieces and weights
      wait_lgkm0();
    }
    PP_MARK(1)
    __syncthreads();
    PP_MARK(2)
  }
  for (int st = team + 2 * nmine; st < nsteps; ++st) __syncthreads();
#if (X3DIAG & 2048) != 0
  if (dwave && blockIdx.x < PP_DIAG_WGS) {
    unsigned long long* d = pp_diag_stamps + 8 * blockIdx.x + 3 * team;
    d[0] = dg[0], d[1] = dg[1], d[2] = dg[2];
    if (team == 0) pp_diag_stamps[8 * blockIdx.x + 6] = __builtin_amdgcn_s_memtime() - t_start;
  }
#endif
#undef PP_MARK
}

}  // namespace dnnhip
