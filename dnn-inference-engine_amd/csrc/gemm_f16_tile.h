// fp16 3x3 conv + 2x2/s2 max-pool for the narrow layers of the fp16 path (conv2-conv4 of
// YOLOv2-tiny, BASELINE config 5), device code only.  Round 5: these layers ran on the implicit
// fp16 GEMM (gemm_f16.h: every tap's A tile gathered from HBM / L2 per K-step) at 43-62 us each
// where the fp16 MFMA floor of each is ~10 us.
//
// A workgroup owns a TH x TW tile of output pixels of one frame (pool-window-major rows: rows
// 4w .. 4w + 3 are the 2x2 window w, so the pool is a max over one MFMA result's four registers)
// and WN groups of 64 columns; WM x WN waves, each TM 16-row blocks x 64 columns (4 column
// blocks, acc 16 TM registers).  Operand traffic per 32-channel K-step and wave: TM KiB of A
// fragments from LDS, 4 KiB of weights from L1 / L2; at TM = 7 and two waves per SIMD that is
// half the LDS and half the L1 bandwidth the MFMAs need (the conv6/conv7 kernel's 32-column waves
// are LDS-bound: 2 reads per 4 MFMAs).
//   * the zero-bordered input's (TH + 2) x (TW + 2) patch of one 32-channel chunk is LDS-DMA'd
//     (buffer_load ... lds, 1-KiB pieces) as 64-B pixel rows, each image row skewed by SK = 2
//     units (tools: 0.31 extra conflict cycles per fragment read at 8 x 52 and 4 x 52 tiles,
//     0.92 at 8 x 26; plain 64-B rows 4.0-5.9);
//   * persistent workgroups (two per CU): a workgroup's (tile, chunk) pairs run as one stream,
//     the next pair's patch DMA'd into the other buffer while the current one computes, so a
//     tile's input load hides behind the previous tile's MFMAs;
//   * weights (order 5: [n/16][k/32][lane][8], k = (chunk 9 + tap) 32 + c) straight from L2 to
//     registers two K-steps ahead (a ring of three); A fragments two blocks ahead (a ring of
//     three), a fragment address = a per-block register + a tap immediate;
//   * epilogue: pool (max, or min where the epilogue decreases), the fp16 path's epilogue, fp16
//     into a wave-private LDS stage, then 16-B stores of 8 halves into the (optionally
//     zero-bordered) pooled output.
// Per output the products run chunk by chunk, tap by tap, one v_mfma_f32_16x16x32_f16 per
// 32-channel group: the order depends on (C, N) only (batch-invariant).
#pragma once
#include "gemm_f16.h"
#include "gemm_f16_acc.h"

namespace dnnhip {

#ifndef T16DIAG
#define T16DIAG 0
#endif
#if T16DIAG
// diagnostic builds (-DT16DIAG=1, tools/build_diag.sh): per-workgroup phase stamps of the last
// launch per input width class (C 32 / 64 / 128 / other), wave 0: [0] realtime start, [1] memtime
// start, [2] prologue done, per pair q < 8: [3 + 3q] MFMA end, [4 + 3q] barrier passed, [5 + 3q]
// epilogue done; [27] memtime end, [28] realtime end, [29] HW_ID, [30] XCC_ID, [31] tiles
constexpr int T16_DIAG_WGS = 1024;
__device__ unsigned long long t16_diag_stamps[4 * T16_DIAG_WGS * 32];
#define T16_STAMP(k, v)                                                                              \
  {                                                                                                  \
    if (threadIdx.x == 0 && blockIdx.x < T16_DIAG_WGS)                                               \
      t16_diag_stamps[((g.C == 32 ? 0 : g.C == 64 ? 1 : g.C == 128 ? 2 : 3) * T16_DIAG_WGS + blockIdx.x) * 32 + (k)] = (v); \
  }
#else
#define T16_STAMP(k, v) {}
#endif

struct Tile16Geom {
  int H, W, C;     // conv input = output size (3x3, stride 1, SAME), channels
  int PH, PW;      // pooled output size (H / 2, W / 2)
  int out_padded;  // 1: pooled output into a zero-bordered [B][PH+2][PW+2][N] buffer
};

// MODE 0: 2-D tiles, pool-window-major rows, 2x2/s2 pool (above).  MODE 1 (conv5 + pool5): the
// whole TH x TW frame per tile in raster rows, the epilogue's fp16 values staged for the whole
// frame and the 2x2/s1 SAME pool taken from the stage (pool of the rounded values == rounding of
// the pooled value: rounding is monotone); PU-unit pixel rows (13 x 13 frames: 96-B rows skewed by
// 4 units per image row, 1.45 extra conflict cycles per fragment read; 64-B rows 4.7).
template <int TH, int TW, int WM, int WN, int TM, int FL = -1, int MODE = 0, int PU = 4, int SK = 2, int BR = 3>
__global__ void __launch_bounds__(64 * WM * WN, 2)
conv3x3_f16_tile_kernel(const half_t* __restrict__ in, const half_t* __restrict__ Bt, int ldb, half_t* __restrict__ out,
                        int N, EpiParams epi, int tilesX, int tilesY, int tilesN, int nspatial, Tile16Geom g,
                        unsigned in_bytes, unsigned b_bytes) {
  constexpr int NW = WM * WN, PW2 = TW + 2, RU = PU * PW2 + SK, T = TH * TW, NJ = 4;
  constexpr int NU = (TH + 2) * RU, NP = (NU + 63) / 64, NPW = (NP + NW - 1) / NW;  // units / pieces per chunk
  constexpr int BUFB = NP * 1024;
  constexpr int SROW = 72;  // stage row pitch (halves): 64 columns + 8 (144-B rows)
  constexpr int STGB = TM * 4 * SROW * 2;  // per wave
  static_assert(WM * TM * 16 >= T && (WM - 1) * TM * 16 < T && NPW <= 16 && PU >= 4 && (MODE == 0 || MODE == 1) &&
                    (MODE == 0 ? TH % 2 == 0 && TW % 2 == 0 && NW * STGB <= BUFB : T * 64 * WN * 2 <= BUFB),
                "shape");
  // LDS regions (round 6 audit, DESIGN.md §2 "fp16 tile-kernel race"): two patch buffers of BUFB
  // bytes, then the epilogue parameters (epl, WN x 64 f32x4).  Every access is bounded here:
  //  * the DMA writes pieces 0 .. NP - 1 of a buffer, 1 KiB each: NP * 1024 == BUFB;
  //  * the farthest fragment read (row T - 1 at tap (2, 2), lane quarter 3, 16 B) ends inside the
  //    patch's NU units: (RU (TH + 1) + PU (TW + 1)) 16 + 64 <= 16 NU <= BUFB;
  //  * the MODE 0 stage (NW waves x STGB) and the MODE 1 stage (T rows x 64 WN halves) fit one
  //    buffer, so the stage never reaches the other buffer (the next pair's patch) or epl;
  //  * epl reads are epl[wn 64 + 16 jb + fr] < 64 WN;
  //  * two workgroups per CU (__launch_bounds__) fit the 160 KiB of LDS.
  static_assert(NP * 1024 == BUFB && NP * 64 >= NU, "patch pieces");
  static_assert((RU * (TH + 1) + PU * (TW + 1)) * 16 + 64 <= NU * 16, "fragment reads inside the patch");
  static_assert(MODE == 0 ? (NW * STGB <= BUFB && 4 * TM * SROW * 2 == STGB) : (T * 64 * WN * 2 <= BUFB), "stage");
  static_assert(WN * 64 == 16 * NJ * WN, "epl covers the workgroup's columns");
  static_assert(2 * (2 * BUFB + WN * 64 * 16) <= 160 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUFB + WN * 64 * 16];
  f32x4* const epl = reinterpret_cast<f32x4*>(smem + 2 * BUFB);

  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int wn = wid % WN, wm = wid / WN;
  // persistent: workgroup w keeps column group tn = w % tilesN and takes the spatial tiles
  // w / tilesN + G k (G = grid / tilesN); its (tile, chunk) pairs run as one stream q, the patch
  // of pair q + 1 DMA'd into the other buffer while pair q computes (also across tiles)
  const int tn = blockIdx.x % tilesN, G = gridDim.x / tilesN, sp0 = blockIdx.x / tilesN;
  const int ntl = (nspatial - sp0 + G - 1) / G;
  const int n0 = tn * (64 * WN) + wn * 64;
  const int Wp = g.W + 2;
  const int fr = lane & 15, fq = lane >> 4;
  T16_STAMP(0, __builtin_amdgcn_s_memrealtime())
  T16_STAMP(1, __builtin_amdgcn_s_memtime())
  T16_STAMP(29, (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)))
  T16_STAMP(30, (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11)))
  T16_STAMP(31, ntl)
  auto tile_xyb = [&](int k, int& b, int& y0, int& x0) {
    int t = sp0 + G * k;
    const int tx = t % tilesX;
    t /= tilesX;
    const int ty = t % tilesY;
    b = t / tilesY;
    y0 = ty * TH;
    x0 = tx * TW;
  };

  // fragment rows: LDS byte offset of the lane's tap-(0, 0) pixel (+ 16 fq)
  int rowoff[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int r = (wm * TM + i) * 16 + fr;
    r = r < T ? r : T - 1;
    int ly, lx;
    if constexpr (MODE == 0) {
      const int w = r >> 2, q = r & 3;
      ly = 2 * (w / (TW / 2)) + (q >> 1);
      lx = 2 * (w % (TW / 2)) + (q & 1);
    } else {
      ly = r / TW;
      lx = r % TW;
    }
    rowoff[i] = (RU * ly + PU * lx) * 16 + 16 * fq;
  }
  auto rowoff_of = [&](int i) {
    int v = rowoff[i];
    asm volatile("" : "+v"(v));
    return v;
  };

  // patch DMA: unit U = 64 piece + lane -> patch row py = U / RU, column px, 16-B unit u (the SK
  // spare units of a row load its last unit; never read); source: padded pixel (y0 + py, x0 + px)
  // of frame b, chunk c.  Reads past the frame (edge tiles) feed rows that are not stored; past
  // the buffer they return zero.  The per-piece offsets within a patch are the same for every tile.
  const int nch = g.C / 32;
  const unsigned rowB = 2u * (unsigned)g.C;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  unsigned pofs[NPW];
#pragma unroll
  for (int k = 0; k < NPW; ++k) {
    const unsigned U = 64u * (unsigned)(wid + NW * k) + (unsigned)lane;
    unsigned py = U / RU;
    const unsigned rem = U - py * RU;
    unsigned px = rem / PU, u = rem % PU;
    if (px >= (unsigned)PW2) px = PW2 - 1, u = PU - 1;
    py = py < (unsigned)(TH + 2) ? py : (unsigned)(TH + 1);
    pofs[k] = (py * (unsigned)Wp + px) * rowB + 16u * u;
  }
  auto issue = [&](int q, int buf) {
    int b, y0, x0;
    tile_xyb(q / nch, b, y0, x0);
    const unsigned base = (unsigned)((b * (g.H + 2) + y0) * Wp + x0) * rowB;
    const int c = q % nch;
#pragma unroll
    for (int k = 0; k < NPW; ++k) {
      if (wid + NW * k >= NP) break;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsA, (__attribute__((address_space(3))) void*)(smem + buf * BUFB + 1024 * (wid + NW * k)), 16,
          (int)(base + pofs[k]), c * 64, 0, 0);
    }
  };

  // weights (order 5): 16-column block nb at nb ldb 32 bytes, K-step s at s KiB
  const unsigned bvo = (unsigned)((n0 / 16) * ldb * 32 + lane * 16);
  const int bjs = ldb * 32;
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)b_bytes, 0x00020000);
  // weight ring of BR K-steps, loads BR - 1 steps ahead (9 % BR == 0: the same slots every pair).
  // A vector-memory load waits for every older one, the next pair's patch DMA included: the
  // DMA has BR - 1 steps to land before the loop stalls on a weight issued after it.
  static_assert(9 % BR == 0 && BR >= 3, "weight ring");
  f16x8 bq[BR][NJ];
  auto load_b = [&](int s, f16x8 (&dst)[NJ]) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      dst[j] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, bvo, s * 1024 + j * bjs, 0));
  };
  const int S = 9 * nch;  // K-steps per tile (the weight stream wraps at each tile)

  f32x4 acc[TM][NJ];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int eflags = FL < 0 ? epi.flags : FL;
  issue(0, 0);
#pragma unroll
  for (int l = 0; l < BR - 1; ++l) load_b(l, bq[l]);
  if (threadIdx.x < 64 * WN) {  // the workgroup's epilogue parameters
    const int n = tn * (64 * WN) + threadIdx.x;
    epl[threadIdx.x] = f32x4{(eflags & EPI_BIAS) ? epi.bias[n] : 0.f,
                             (eflags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f,
                             (eflags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f, (eflags & EPI_BN) ? epi.gamma[n] : 1.f};
  }
  vm_wait<0>();
  __syncthreads();
  T16_STAMP(2, __builtin_amdgcn_s_memtime())

  constexpr int LEAD = 2, RING = 3;
  static_assert((9 * TM) % RING == 0, "fragment ring phase per chunk");
  f16x8 af[RING];
  auto blk = [&](const unsigned char* Pb, int bi) {
    const int tp = bi / TM;
    return Pb + rowoff_of(bi % TM) + (RU * (tp / 3) + PU * (tp % 3)) * 16;
  };
#pragma unroll
  for (int l = 0; l < LEAD; ++l) af[l] = *reinterpret_cast<const f16x8*>(blk(smem, l));
  typedef half_t h8v __attribute__((ext_vector_type(8)));
  const int nq = ntl * nch;
  for (int q = 0; q < nq; ++q) {
    const int c = q % nch;
    const unsigned char* P = smem + (q & 1) * BUFB;
    if (q + 1 < nq) issue(q + 1, (q + 1) & 1);  // the other buffer: read in pair q - 1
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int s = 9 * c + tp;
      __builtin_amdgcn_sched_barrier(0);
      {
        int s2 = s + BR - 1;  // (past the tile's last step: the next tile's first steps; BR - 1 < 9 <= S)
        s2 = s2 < S ? s2 : s2 - S;
        load_b(s2, bq[(tp + BR - 1) % BR]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int bi = TM * tp + i;
        const f16x8 a = af[bi % RING];
        if (bi + LEAD < 9 * TM) af[(bi + LEAD) % RING] = *reinterpret_cast<const f16x8*>(blk(P, bi + LEAD));
#pragma unroll
        for (int jb = 0; jb < NJ; ++jb) acc[i][jb] = mfma16_f16(a, bq[tp % BR][jb], acc[i][jb]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // the ring holds the next pair's first BR - 1 steps in slots 0 .. BR - 2 (9 % BR == 0)
    if (q < 8) T16_STAMP(3 + 3 * q, __builtin_amdgcn_s_memtime())
    vm_wait<0>();  // this wave's DMA pieces of pair q + 1 landed
    wait_lgkm0();
    __syncthreads();  // every wave's pieces landed; pair q's buffer read by every wave
    if (q < 8) T16_STAMP(4 + 3 * q, __builtin_amdgcn_s_memtime())
    if (MODE == 1 && c == nch - 1) {
      // epilogue of frame q / nch: fp16 values of every pixel x the workgroup's 64 WN columns
      // into the just-read buffer, then the 2x2/s1 SAME pool from it, 8 columns per thread
      int b, y0, x0;
      tile_xyb(q / nch, b, y0, x0);
      half_t* const st = reinterpret_cast<half_t*>(smem + (q & 1) * BUFB);
      constexpr int SW = 64 * WN;
#pragma unroll
      for (int jb = 0; jb < NJ; ++jb) {
        const f32x4 e = epl[wn * 64 + 16 * jb + fr];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = (wm * TM + i) * 16 + 4 * fq + r;
            if (row < T)
              st[row * SW + wn * 64 + 16 * jb + fr] =
                  (half_t)apply_epilogue_t<FL>(acc[i][jb][r], e[0], e[1], e[2], e[3], epi.flags);
          }
          acc[i][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      wait_lgkm0();
      __syncthreads();
      const int ncol0 = tn * (64 * WN);
      for (int idx = threadIdx.x; idx < T * (SW / 8); idx += 64 * NW) {
        const int p = idx / (SW / 8), gq = idx - p * (SW / 8);
        const int y = p / TW, x = p - y * TW;
        const h8v* sp = reinterpret_cast<const h8v*>(st + p * SW + 8 * gq);
        h8v v = sp[0];
        if (x + 1 < TW) v = __builtin_elementwise_max(v, sp[SW / 8]);
        if (y + 1 < TH) {
          v = __builtin_elementwise_max(v, sp[TW * (SW / 8)]);
          if (x + 1 < TW) v = __builtin_elementwise_max(v, sp[(TW + 1) * (SW / 8)]);
        }
        const size_t o = g.out_padded ? (size_t)(b * (TH + 2) + y + 1) * (TW + 2) + x + 1 : (size_t)(b * TH + y) * TW + x;
        store16_at(out, 2 * (o * N + ncol0 + 8 * gq), __builtin_bit_cast(u32x4, v));
      }
      wait_lgkm0();
      __syncthreads();  // the stage read before pair q + 2's DMA reuses the buffer
    }
    if (MODE == 0 && c == nch - 1) {
      // epilogue of tile q / nch through the just-read buffer: window (block i, fq) of column
      // 16 jb + fr -> the wave's stage row 4 i + fq, then 16-B stores of 8 halves
      int b, y0, x0;
      tile_xyb(q / nch, b, y0, x0);
      half_t* const st = reinterpret_cast<half_t*>(smem + (q & 1) * BUFB + wid * STGB);
#pragma unroll
      for (int jb = 0; jb < NJ; ++jb) {
        const f32x4 e = epl[wn * 64 + 16 * jb + fr];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          st[(4 * i + fq) * SROW + 16 * jb + fr] =
              (half_t)pool_then_epilogue_t<FL>(acc[i][jb], e[0], e[1], e[2], e[3], epi.flags);
          acc[i][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      wait_lgkm0();
      constexpr int NWIN = TM * 4, NO = T / 4;
#pragma unroll
      for (int ps = 0; ps < (NWIN * 8 + 63) / 64; ++ps) {
        const int idx = 64 * ps + lane, wl = idx >> 3, gq = idx & 7;
        const int w = wm * NWIN + wl;
        if (wl < NWIN && w < NO) {
          const int py = (y0 >> 1) + w / (TW / 2), px = (x0 >> 1) + w % (TW / 2);
          if (py < g.PH && px < g.PW) {
            const size_t o = g.out_padded ? (size_t)(b * (g.PH + 2) + py + 1) * (g.PW + 2) + px + 1
                                          : (size_t)(b * g.PH + py) * g.PW + px;
            store16_at(out, 2 * (o * N + n0 + 8 * gq), *reinterpret_cast<const u32x4*>(st + wl * SROW + 8 * gq));
          }
        }
      }
      wait_lgkm0();
      __syncthreads();  // the stage read before pair q + 2's DMA reuses the buffer
      if (q < 8) T16_STAMP(5 + 3 * q, __builtin_amdgcn_s_memtime())
    }
    if (q + 1 < nq) {
#pragma unroll
      for (int l = 0; l < LEAD; ++l) af[l] = *reinterpret_cast<const f16x8*>(blk(smem + ((q + 1) & 1) * BUFB, l));
    }
  }
  T16_STAMP(27, __builtin_amdgcn_s_memtime())
  T16_STAMP(28, __builtin_amdgcn_s_memrealtime())
}

}  // namespace dnnhip
