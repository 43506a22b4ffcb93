// MFMA kernels for the two small-channel layers of YOLOv2-tiny.
//
// conv0_mfma_pool_kernel<F16>: 3x3 / stride 1 / SAME conv of fp32 NHWC frames with <= 3
//   input channels and 16 outputs + epilogue + 2x2/s2 max pool (conv0: 416x416x3 -> 16,
//   pooled 208x208).  The input halo patch sits in LDS as 4-channel pixels, so each MFMA
//   operand is a single LDS read at a compile-time tap offset (no im2col anywhere):
//   F16 = false: 9 x v_mfma_f32_16x16x4_f32 per 16-pixel tile (lane part = channel, exact
//   fp32 products); F16 = true: 3 x v_mfma_f32_16x16x16_f16 (lane part = tap; fp16 path).
//   Weights (HWIO [K][16]) live in registers.  Rows are pool-window-major (row = 4*window +
//   2*dy + dx), so a lane's 4 accumulator registers are one pool window: pool, then the
//   epilogue once (pool_then_epilogue, gemm_f32.h).  Replaces conv3x3_pool2_direct_kernel's
//   fp32 FMA loop (VALU-bound at ~50 TF, SQ counters) for cin <= 3.
//
// conv1_patch_f16_kernel: the fp16 path's conv1 (208x208x16 -> 32, pooled): the fp32 patch
//   kernel's structure (conv_patch.hip) in fp16 — one LDS-DMA pass stages the 18x18x16 half
//   patch per 16x16 tile, each lane holds its weight fragments in registers, and every K-step
//   of v_mfma_f32_16x16x32_f16 covers two taps (lane part p: tap 2s + p/2, channels
//   8(p&1)..+7), tap 9 being zero.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cfloat>
#include <type_traits>
#include "dnn_common.h"
#include "gemm_f32.h"

namespace dnnhip {

typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int SC_T = 16;        // conv outputs per tile edge (8 x 8 pool windows)
constexpr int SC_P = SC_T + 2;  // patch edge

// ------------------------------------------------------------------------------ conv0
// LDS patch: 18 x 18 pixels x 4 channels (cin <= 3 zero-padded to 4; fp32 for the fp32
// path, fp16 for the fp16 path), so every MFMA operand is one LDS read at a compile-time tap
// offset from the lane's pixel:
//   fp32: 9 x v_mfma_f32_16x16x4_f32 per 16-pixel tile, lane part p = channel p, one tap each
//   fp16: 3 x v_mfma_f32_16x16x16_f16, lane part p = tap 4g + p (taps 9..11 zero), one
//         ds_read_b64 = the pixel's 4 channels
typedef _Float16 h4_t __attribute__((ext_vector_type(4)));

template <int CIN, bool F16, typename OutT>
__global__ void __launch_bounds__(256)
conv0_mfma_pool_kernel(const float* __restrict__ in, const float* __restrict__ w, OutT* __restrict__ out,
                       DirectGeom g, int tilesX, int tilesY, int ntiles, EpiParams epi) {
  static_assert(CIN >= 1 && CIN <= 3, "patch pixels hold 4 channels");
  typedef typename std::conditional<F16, half_t, float>::type PT;
  constexpr int NPX = SC_P * SC_P;          // 324 patch pixels
  constexpr int PPT = (NPX + 255) / 256;    // pixels per thread
  __shared__ __attribute__((aligned(16))) PT patch[NPX * 4];
  __shared__ __attribute__((aligned(16))) float stage[4][2][8][16];  // per wave: 2 window rows x 8 windows x 16 ch

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int fr = lane & 15, fp = lane >> 4, n = lane & 15;

  // B fragments (HWIO [tap*CIN + c][16]), once per workgroup
  float wv[9];
  h4_t bw[3];
  if constexpr (F16) {
#pragma unroll
    for (int gq = 0; gq < 3; ++gq) {
      const int t = 4 * gq + fp;
#pragma unroll
      for (int c = 0; c < 4; ++c) bw[gq][c] = (half_t)((t < 9 && c < CIN) ? w[(t * CIN + c) * 16 + n] : 0.f);
    }
  } else {
#pragma unroll
    for (int t = 0; t < 9; ++t) wv[t] = fp < CIN ? w[(t * CIN + fp) * 16 + n] : 0.f;
  }
  const float pb_ = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
  const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
  const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
  const float pg = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;

  // this lane's pixel (patch index of its window origin) in each of its 4 M-tiles
  int pix[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int wi = fr >> 2, pos = fr & 3;
    const int y = 4 * wid + 2 * (i >> 1) + (pos >> 1);
    const int x = 2 * (4 * (i & 1) + wi) + (pos & 1);
    pix[i] = y * SC_P + x;
  }

  // prefetch of a tile's halo patch into registers: CIN floats per pixel, zero outside the frame
  auto fetch = [&](int t, float (&v)[PPT][CIN]) {
    const int tx = t % tilesX, tt = t / tilesX, ty = tt % tilesY, b = tt / tilesY;
    const float* inb = in + (size_t)b * g.H * g.W * CIN;
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      const int q = threadIdx.x + 256 * u;
      const int r = q / SC_P, c = q - (q / SC_P) * SC_P;
      const int iy = ty * SC_T - g.pt + r, ix = tx * SC_T - g.pl + c;
      const bool ok = q < NPX && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      const float* src = inb + ((size_t)iy * g.W + ix) * CIN;
#pragma unroll
      for (int e = 0; e < CIN; ++e) v[u][e] = ok ? src[e] : 0.f;
    }
  };

  float pre[PPT][CIN];
  int t = blockIdx.x;
  if (t < ntiles) fetch(t, pre);
  for (; t < ntiles; t += gridDim.x) {
    const int tx = t % tilesX, tt = t / tilesX, ty = tt % tilesY, b = tt / tilesY;
    const int y0 = ty * SC_T, x0 = tx * SC_T;
    // raw barriers with LDS-only waits (__syncthreads would also drain the global stores)
    wait_lgkm0();
    raw_barrier();
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      const int q = threadIdx.x + 256 * u;
      if (q < NPX) {
        if constexpr (F16) {
          h4_t h;
#pragma unroll
          for (int c = 0; c < 4; ++c) h[c] = (half_t)(c < CIN ? pre[u][c] : 0.f);
          *reinterpret_cast<h4_t*>(patch + 4 * q) = h;
        } else {
          f32x4 f;
#pragma unroll
          for (int c = 0; c < 4; ++c) f[c] = c < CIN ? pre[u][c] : 0.f;
          *reinterpret_cast<f32x4*>(patch + 4 * q) = f;
        }
      }
    }
    wait_lgkm0();
    raw_barrier();
    if (t + (int)gridDim.x < ntiles) fetch(t + gridDim.x, pre);  // in flight during the MFMAs

    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (F16) {
#pragma unroll
      for (int gq = 0; gq < 3; ++gq) {
        const int tap = 4 * gq + fp;  // lane part fp
        const int toff = tap < 9 ? (tap / 3) * SC_P + tap % 3 : 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          h4_t a = *reinterpret_cast<const h4_t*>(patch + 4 * (pix[i] + toff));
          if (tap >= 9) a = h4_t{0, 0, 0, 0};
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(a, bw[gq], acc[i], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int toff = (tap / 3) * SC_P + tap % 3;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(patch[4 * (pix[i] + toff) + fp], wv[tap], acc[i], 0, 0, 0);
      }
    }

    // pool + epilogue into the wave's LDS stage, then 16-B coalesced stores
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int wy = (y0 >> 1) + 2 * wid + (i >> 1), wx = (x0 >> 1) + 4 * (i & 1) + fp;
      // window cells past the conv output (odd sizes: SAME pool padding) repeat cell (0,0)
      const bool x1 = 2 * wx + 1 < g.OW, y1 = 2 * wy + 1 < g.OH;
      const f32x4 v = {acc[i][0], x1 ? acc[i][1] : acc[i][0], y1 ? acc[i][2] : acc[i][0],
                       x1 && y1 ? acc[i][3] : acc[i][0]};
      stage[wid][i >> 1][4 * (i & 1) + fp][n] = pool_then_epilogue(v, pb_, pm, ps, pg, epi.flags);
    }
    wait_lgkm0();  // this wave's stage writes have landed (the stage is wave-private)
    constexpr int VEC = F16 ? 8 : 4;
    for (int c = lane; c < 2 * 128 / VEC; c += 64) {
      const int lr = c / (128 / VEC), f = (c % (128 / VEC)) * VEC;  // f: float index in the row's run
      const int wy = (y0 >> 1) + 2 * wid + lr, wxs = (x0 >> 1) + f / 16;
      if (wy >= g.PH || wxs >= g.PW) continue;
      const float* src = &stage[wid][lr][0][0] + f;
      OutT* dst = out + (((size_t)b * g.PH + wy) * g.PW + (x0 >> 1)) * 16 + f;
      if constexpr (F16) {
        h8_t o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (half_t)src[e];
        *reinterpret_cast<h8_t*>(dst) = o;
      } else {
        *reinterpret_cast<f32x4*>(dst) = *reinterpret_cast<const f32x4*>(src);
      }
    }
    wait_lgkm0();  // stage reads done before the next tile overwrites it
  }
}

// conv0_packed_pool_kernel<CIN>: the fp32 conv0 with K = 9*CIN packed densely into
// ceil(K/4) v_mfma_f32_16x16x4_f32 steps (CIN = 3: 7 MFMAs per 16-pixel tile instead of the 9
// one-tap-per-MFMA steps above, k = 27 multiplying a zero weight).  K order is the
// reference's im2col order (tap-major, channel-minor, dnn_openblas.c:135-158), so every
// accumulator is the same fmaf chain over k = 0..26 as the explicit im2col + GEMM path: same
// bits.  The halo patch is DMA'd straight from the NHWC frame rows (one 4-B LDS-DMA lane per
// float of the 18 x CIN floats of a patch row: no register staging, no channel padding) into
// a double buffer, the next tile's rows in flight during this tile's MFMAs; lane part p of
// step s reads k = 4s + p at a per-lane LDS offset koff[s] (dy*RS + dx*CIN + c) from its
// pixel, the M-tile offset being an immediate.  (RS = 56: every ds_read_b32 is exactly
// 2-way; no row stride makes the two pixel rows of an M-tile conflict-free.)
// C0DIAG (diagnostic builds only, wrong results): bit 1 drops the loop's patch DMA, 2 the pool and
// epilogue arithmetic, 4 the MFMAs (a VALU multiply-add on the same LDS reads instead)
#ifndef C0DIAG
#define C0DIAG 0
#endif
constexpr int C0_RS = 56;  // patch row stride (floats) >= 18 * CIN
constexpr int C0_ROWS_PER_WAVE = 5;  // 20 row DMAs per tile over 4 waves (rows 18, 19 dummies)

// Round 4 diagnostics (same box): without the loop's patch DMA 0.124 -> 0.104 ms, without the
// pool/epilogue arithmetic 0.110, without the MFMAs (a VALU FMA on the same LDS reads) 0.083.
// An x3 conv0 (K = 9 taps x (3 channels + 0) on 3 steps of v_mfma_f32_16x16x16_bf16 from a split
// patch [piece][pixel][4], 144 instead of 224 MFMA cycles per 16 pixels, register-staged frame
// loads split on the way into LDS) measured 0.149 vs 0.138 ms in one process: the split staging,
// the 2.6x LDS read bytes and 5 instead of 7 waves per SIMD cost more than the MFMA cycles saved
// (git history).
// FL: the epilogue flag set at compile time (-1: runtime `epi.flags`); EVEN: OH and OW even, so
// no pool window is ragged (YOLO's 416 x 416: the per-window edge selects drop out).  (Round 3's
// SPL form stored conv1's split planes here: conv1 -15 us, conv0 +23 us; removed, git history.)
// D16 (round 6; CIN = 3, W % 4 == 0): the patch rows by 16-B LDS-DMA, three rows per
// instruction.  A patch row is the aligned run of 22 pixels from x0 - 4 (17 units of 16 B, 68
// floats: the 18 patch pixels start at float 9); with W % 4 == 0 and x0 % 16 == 0 a 16-B unit never
// straddles the frame edge, so out-of-frame units take the out-of-range offset as whole units.  Two
// DMA instructions per wave and tile (rows 3 j .. 3 j + 2 for j = wid, wid + 4; waves 2 and 3's
// second repeats triplet 4 / 5) instead of five 4-B row DMAs.
template <int CIN, int FL = -1, bool EVEN = false, bool D16 = false, int NB = 3>
#ifndef C0_D16_OCC
#define C0_D16_OCC 8
#endif
__global__ void __launch_bounds__(256, D16 ? C0_D16_OCC : 7)  // 7-8 waves per SIMD (<= 64-72 registers): latency-bound, occupancy pays
conv0_packed_pool_kernel(const float* __restrict__ in, const float* __restrict__ w, float* __restrict__ out,
                         DirectGeom g, int tilesX, int tilesY, int ntiles, const float* __restrict__ zero,
                         EpiParams epi, uint4 mags) {  // mags: magic numbers of tilesX, tilesY (div_magic)
  constexpr int K = 9 * CIN, KS = (K + 3) / 4, RW = SC_P * CIN, RS = D16 ? 68 : C0_RS;
  constexpr int NDMA = D16 ? 2 : C0_ROWS_PER_WAVE;  // DMA instructions per wave and tile
  constexpr int PROWS = D16 ? 18 : 4 * C0_ROWS_PER_WAVE;  // LDS rows per buffer
  constexpr int X0F = D16 ? 3 * CIN : 0;  // float offset of patch pixel 0 in an LDS row
  static_assert(RW <= RS && RW <= 64 && (!D16 || CIN == 3), "patch row");
  static_assert(NB >= 3 && NB <= 5, "patch ring");
  __shared__ __attribute__((aligned(16))) float patch[NB][PROWS * RS];  // ring of NB buffers
  __shared__ __attribute__((aligned(16))) float stage[4][2][8][16];  // per wave: 2 window rows x 8 windows x 16 ch

  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int fr = lane & 15, fp = lane >> 4, n = lane & 15;

  // B fragments (HWIO [k = tap*CIN + c][16]) and the A offsets of k = 4s + fp
  float wv[KS];
  int koff[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 4 * s + fp;
    const int tap = k / CIN, c = k - (k / CIN) * CIN, dy = tap / 3, dx = tap - (tap / 3) * 3;
    wv[s] = k < K ? w[k * 16 + n] : 0.f;
    koff[s] = k < K ? dy * RS + dx * CIN + c : 0;
  }
  const float pb_ = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
  const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
  const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
  const float pg = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;

  // the lane's pixel in M-tile 0 (rows pool-window-major: row = 4*window + 2*dy + dx); M-tile
  // i adds the constant 2*(i>>1) rows and 8*(i&1) pixels
  const int pix0 = (4 * wid + ((fr & 3) >> 1)) * RS + (2 * (fr >> 2) + (fr & 1)) * CIN + X0F;

  // tile coordinates: one set of divisions per tile, shared by its DMA issue and its stores
  struct Tile {
    int b, ty, tx;
  };
  auto coords = [&](int t) {  // two multiply-high divisions (scalar), not two integer divisions
    const int tt = div_magic(t, mags.x, (int)mags.y), b = div_magic(tt, mags.z, (int)mags.w);
    return Tile{b, tt - b * tilesY, t - tt * tilesX};
  };
  // lane l of a patch row DMA copies float l of the row's 18 * CIN (the row is contiguous in
  // the NHWC frame), through a buffer descriptor with 32-bit offsets: lanes past the frame's
  // edges take an offset past its range, which reads zero.  Every wave issues exactly
  // C0_ROWS_PER_WAVE DMAs per tile (rows 18, 19 and the tiles past the end are dummies), so
  // the counted waits below are exact.
  const auto rsIn = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)((size_t)g.B * g.H * g.W * CIN * 4), 0x00020000);
  (void)zero;
  auto issue = [&](const Tile& c, bool valid, int buf) {
    if constexpr (D16) {
      // lane l < 51 of instruction j: patch row 3 j + l / 17, unit l % 17 of the run from pixel
      // xa = 16 tx - 4 (patch pixel 0 = xa + 3: pl == 1, launcher)
      const int xa = c.tx * SC_T - 4, y0 = c.ty * SC_T - g.pt;
      const int r3 = lane / 17, u = lane - 17 * r3;
      const int xu = xa + (4 * u) / 3;  // first pixel the unit touches (units never straddle the edge)
      const bool xok = valid && lane < 51 && xu >= 0 && xu < g.W;
      const unsigned rstride = (unsigned)(g.W * CIN * 4);
      const unsigned lo = (unsigned)(((c.b * g.H + y0) * g.W + xa) * CIN * 4 + 16 * u);
#pragma unroll
      for (int q = 0; q < NDMA; ++q) {
        // (waves 2 and 3's second instruction repeats triplet 4 / 5 of waves 0 and 1: the same bytes
        // into the same LDS rows, so no spare rows; a fixed DMA count per wave)
        const int j = wid + 4 * q < 6 ? wid + 4 * q : wid + 2, r = 3 * j + r3;
        const bool ok = xok && r < SC_P && (unsigned)(y0 + r) < (unsigned)g.H;
        if (lane < 51)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsIn, (__attribute__((address_space(3))) void*)&patch[buf][3 * j * RS],
                                                   16, (int)(ok ? lo + (unsigned)r * rstride : OOB_OFF), 0, 0, 0);
      }
      return;
    }
    const int x0 = c.tx * SC_T - g.pl, y0 = c.ty * SC_T - g.pt;
    const int px = x0 + lane / CIN;
    const bool xok = valid && (unsigned)px < (unsigned)g.W;
    const int row0 = (c.b * g.H + y0) * g.W * CIN;  // float index of the tile's patch row 0 (may be < 0)
    const unsigned lo = (unsigned)((row0 + x0 * CIN + lane) * 4);
    const unsigned rstride = (unsigned)(g.W * CIN * 4);
#pragma unroll
    for (int u = 0; u < C0_ROWS_PER_WAVE; ++u) {
      const int r = wid + 4 * u;
      const bool ok = xok && r < SC_P && (unsigned)(y0 + r) < (unsigned)g.H;
      if (lane < RW)  // (lanes past the row would land in the next row's LDS)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsIn, (__attribute__((address_space(3))) void*)&patch[buf][r * RS],
                                                 4, (int)(ok ? lo + (unsigned)r * rstride : OOB_OFF), 0, 0, 0);
    }
  };

  // NB - 1 tiles in flight: tile t's rows were issued NB - 1 iterations ago.  Per wave and tile the
  // VMEM stream is NDMA DMAs then ST stores, so when tile t is consumed the ops issued after its
  // DMAs are: stores(t - NB + 1), then DMAs(t + i) and stores(t - NB + 1 + i) for i = 1 .. NB - 2
  // -- (NB - 2) NDMA + (NB - 1) ST -- and in the first iterations j < NB - 1 the prologue's later
  // DMAs and the j stores since: (NB - 2) NDMA + j ST.  (NB = 3: stores(t-2), DMAs(t+1), stores(t-1).)
  constexpr int ST = 1;
  const auto orsrc = out_rsrc(out, (unsigned)((size_t)g.B * g.PH * g.PW * 16 * sizeof(float)));
  const int G = gridDim.x;
  int t = blockIdx.x;
  Tile q[NB - 1];  // tiles t, t + G, ..., t + (NB - 2) G
#pragma unroll
  for (int j = 0; j < NB - 1; ++j) q[j] = coords(t + j * G < ntiles ? t + j * G : 0);
  if (t < ntiles) {
#pragma unroll
    for (int j = 0; j < NB - 1; ++j) issue(q[j], t + j * G < ntiles, j);
  }
  int buf = 0;
  for (int it = 0; t < ntiles; t += G, ++it) {
    if (it == 0)
      wait_vmcnt<(NB - 2) * NDMA>();
    else if (it == 1)
      wait_vmcnt<(NB - 2) * NDMA + ST>();
    else if (NB > 3 && it == 2)
      wait_vmcnt<(NB - 2) * NDMA + 2 * ST>();
    else if (NB > 4 && it == 3)
      wait_vmcnt<(NB - 2) * NDMA + 3 * ST>();
    else
      wait_vmcnt<(NB - 2) * NDMA + (NB - 1) * ST>();
    raw_barrier();  // every wave's rows of `buf` landed; every wave finished reading tile t-1's buffer
    // tile t + (NB - 1) G into the buffer tile t - 1 used (dummy past the end: the count stays fixed)
    const int t2 = t + (NB - 1) * G;
    const Tile nn = coords(t2 < ntiles ? t2 : 0);
    if (!(C0DIAG & 1)) issue(nn, t2 < ntiles, buf == 0 ? NB - 1 : buf - 1);
    const float* P = patch[buf];

    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float* a = P + pix0 + koff[s];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr ((C0DIAG & 4) != 0)
          acc[i][s & 3] += a[2 * (i >> 1) * RS + 8 * (i & 1) * CIN] * wv[s];
        else
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2 * (i >> 1) * RS + 8 * (i & 1) * CIN], wv[s], acc[i], 0, 0, 0);
      }
    }

    const Tile cur = q[0];
    const int b = cur.b, y0 = cur.ty * SC_T, x0 = cur.tx * SC_T;
#pragma unroll
    for (int j = 0; j + 1 < NB - 1; ++j) q[j] = q[j + 1];
    q[NB - 2] = nn;
    // pool + epilogue into the wave's LDS stage (the four windows' divisions behind one
    // wave-uniform check: pool_epilogue_batch), then 16-B coalesced stores
    f32x4 pv[4][1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x4 v = acc[i];
      if constexpr (!EVEN) {
        const int wy = (y0 >> 1) + 2 * wid + (i >> 1), wx = (x0 >> 1) + 4 * (i & 1) + fp;
        const bool x1 = 2 * wx + 1 < g.OW, y1 = 2 * wy + 1 < g.OH;
        v = f32x4{acc[i][0], x1 ? acc[i][1] : acc[i][0], y1 ? acc[i][2] : acc[i][0], x1 && y1 ? acc[i][3] : acc[i][0]};
      }
      pv[i][0] = v;
    }
    if constexpr ((C0DIAG & 2) != 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) stage[wid][i >> 1][4 * (i & 1) + fp][n] = pv[i][0][0] + pv[i][0][1] + pv[i][0][2] + pv[i][0][3];
    } else {
      const float cb[1] = {pb_}, cm[1] = {pm}, cs[1] = {ps}, cg[1] = {pg};
      pool_epilogue_batch<FL>(pv, cb, cm, cs, cg, epi.flags,
                              [&](int i, int, float e) { stage[wid][i >> 1][4 * (i & 1) + fp][n] = e; });
    }
    wait_lgkm0();  // the stage is wave-private
    {  // one 16-B store per lane (2 window rows x 8 windows x 16 channels per wave)
      const int lr = lane >> 5, f = (lane & 31) * 4;
      const int wy = (y0 >> 1) + 2 * wid + lr, wxs = (x0 >> 1) + f / 16;
      const unsigned off = (wy < g.PH && wxs < g.PW)
                               ? (unsigned)(((((size_t)b * g.PH + wy) * g.PW + (x0 >> 1)) * 16 + f) * sizeof(float))
                               : OOB_OFF;
      store16(orsrc, off, *reinterpret_cast<const f32x4*>(&stage[wid][lr][0][0] + f));
    }
    wait_lgkm0();
    buf = buf == NB - 1 ? 0 : buf + 1;
  }
  wait_vmcnt<0>();  // no LDS-DMA may land after the workgroup exits
}

bool conv0_mfma_supported(int cin, int nout, int kh, int kw, int sh, int sw) {
  return kh == 3 && kw == 3 && sh == 1 && sw == 1 && cin >= 1 && cin <= 3 && nout == 16;
}

template <bool F16, typename OutT>
static int launch_conv0(const float* in, const float* w, OutT* out, const DirectGeom& g, int cin,
                        const EpiParams& epi, hipStream_t s) {
  if (g.B == 0) return 0;
  const int tilesX = (g.OW + SC_T - 1) / SC_T, tilesY = (g.OH + SC_T - 1) / SC_T;
  const long long blocks = (long long)g.B * tilesX * tilesY;
  if (blocks > 0x7fffffffLL || cin < 1 || cin > 3 || g.PH != (g.OH + 1) / 2 || g.PW != (g.OW + 1) / 2) {
    set_error("conv0_mfma: unsupported shape (cin=%d)", cin);
    return -2;
  }
  // persistent: 8 workgroups per CU loop over the tiles (weights loaded once per workgroup,
  // the next tile's patch prefetched into registers during the current tile's MFMAs)
  const int nt = (int)blocks;
  const char* eg = getenv("DNN_HIP_C0_GRID");  // (tuning experiments: workgroups of the launch)
  // (fp16 conv0 at batch 64: 2048 89.4 us, 4096 85.1, 8192 87.2; the fp32 form of this kernel is only
  // the fallback of launch_conv0_mfma -- YOLO's fp32 conv0 runs conv0_packed_pool_kernel -- and
  // keeps its round-4 cap of 2048)
  const int gmax = eg && atoi(eg) > 0 ? atoi(eg) : F16 ? 4096 : 2048;
  const dim3 grid((unsigned)(nt < gmax ? nt : gmax));
  switch (cin) {
    case 1: hipLaunchKernelGGL((conv0_mfma_pool_kernel<1, F16, OutT>), grid, dim3(256), 0, s, in, w, out, g, tilesX, tilesY, nt, epi); break;
    case 2: hipLaunchKernelGGL((conv0_mfma_pool_kernel<2, F16, OutT>), grid, dim3(256), 0, s, in, w, out, g, tilesX, tilesY, nt, epi); break;
    default: hipLaunchKernelGGL((conv0_mfma_pool_kernel<3, F16, OutT>), grid, dim3(256), 0, s, in, w, out, g, tilesX, tilesY, nt, epi); break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("launch conv0_mfma: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int launch_conv0_mfma(const float* in, const float* w, float* out, const DirectGeom& g, int cin, const float* zero,
                      const EpiParams& epi, hipStream_t s) {
  if (cin != 3 || !zero)
    return launch_conv0<false, float>(in, w, out, g, cin, epi, s);
  if (g.B == 0) return 0;
  const int tilesX = (g.OW + SC_T - 1) / SC_T, tilesY = (g.OH + SC_T - 1) / SC_T;
  const long long blocks = (long long)g.B * tilesX * tilesY;
  if ((size_t)g.B * g.PH * g.PW * 16 * sizeof(float) >= OOB_OFF ||
      (size_t)g.B * g.H * g.W * cin * sizeof(float) >= OOB_OFF)  // 32-bit load / store offsets
    return launch_conv0<false, float>(in, w, out, g, cin, epi, s);
  if (blocks > 0x7fffffffLL || g.PH != (g.OH + 1) / 2 || g.PW != (g.OW + 1) / 2) {
    set_error("conv0_packed: unsupported shape");
    return -2;
  }
  unsigned mx, my;
  int sx, sy;
  magic_u32(tilesX, &mx, &sx);
  magic_u32(tilesY, &my, &sy);
  // YOLO's flag set (bias, BatchNorm, the reference's double-rounded leaky) and even frames
  // compiled in; anything else takes the runtime-flag instantiation
  constexpr int YOLO = EPI_BIAS | EPI_BN | EPI_LEAKY_F64;
  const bool even = g.OH % 2 == 0 && g.OW % 2 == 0;
  const uint4 mags = make_uint4(mx, (unsigned)sx, my, (unsigned)sy);
  // persistent workgroups loop over the tiles: 4 rounds of the occupancy the compiled kernel
  // allows (7 per CU at 72 registers: 28 per CU, ~6 tiles each), so the dispatcher refills CUs
  // that finish early.  Measured at batch 64 (workgroups per CU: ms): one resident round 7:
  // 0.185, 8 (the 8th as a lone second round): 0.168, 14: 0.153, 28: 0.1485, 56: 0.153, one tile
  // per workgroup (169): 0.184.
  // (cached per instantiation and device: the occupancy query runs on a device's first launch)
  auto slots_of = [](const void* kern, long long (&cache)[64]) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (cache[dev] > 0) return cache[dev];
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, kern, 256, 0) != hipSuccess || v < 1) v = 1;
    v = 4 * (v < 8 ? v : 8);
    return cache[dev] = (long long)v * device_cu_count();
  };
#define C0PN(FL_, EV_, D16_, NB_)                                                                               \
  do {                                                                                                           \
    static long long cache[64] = {};                                                                             \
    const long long slots =                                                                                      \
        slots_of(reinterpret_cast<const void*>(conv0_packed_pool_kernel<3, FL_, EV_, D16_, NB_>), cache);        \
    const unsigned grid = (unsigned)(blocks < slots ? blocks : slots);                                           \
    hipLaunchKernelGGL((conv0_packed_pool_kernel<3, FL_, EV_, D16_, NB_>), dim3(grid), dim3(256), 0, s, in, w,    \
                       out, g, tilesX, tilesY, (int)blocks, zero, epi, mags);                                    \
  } while (0)
  // (patch ring depth: 4 and 5 buffers measured slower at batch 64 -- 0.1242 / 0.1353 / 0.1424 ms for
  // 3 / 4 / 5, same process: the LDS they take costs a workgroup per CU each, and occupancy hides
  // more of the DMA latency than the deeper ring)
#define C0P(FL_, EV_, D16_) C0PN(FL_, EV_, D16_, 3)
  // 16-B patch-row DMAs (D16) where units cannot straddle the frame edge: W % 4 == 0, one pixel of
  // left padding (SAME 3x3).  DNN_HIP_C0_D16=0 (read per launch, A/B): the 4-B row DMAs; same bits
  const bool d16 = g.W % 4 == 0 && g.pl == 1 && !getenv_flag_off("DNN_HIP_C0_D16");
  if (epi.flags == YOLO && even) {
    if (d16)
      C0P(YOLO, true, true);
    else
      C0P(YOLO, true, false);
  } else if (even) {
    if (d16)
      C0P(-1, true, true);
    else
      C0P(-1, true, false);
  } else {
    if (d16)
      C0P(-1, false, true);
    else
      C0P(-1, false, false);
  }
#undef C0P
#undef C0PN
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("launch conv0_packed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}
int launch_conv0_mfma_f16(const float* in, const float* w, half_t* out, const DirectGeom& g, int cin,
                          const EpiParams& epi, hipStream_t s) {
  return launch_conv0<true, half_t>(in, w, out, g, cin, epi, s);
}

// ------------------------------------------------------------------------------ conv1 fp16
#ifndef C1F16_STAGE
#define C1F16_STAGE 1
#endif
// in: fp16 NHWC [B][H][W][16]; Bt: packed fp16 weights [32][ldb] (k = tap*16 + c, ldb >= 144);
// out: fp16 pooled [B][PH][PW][32] (opad: the interior of a zero-bordered [B][PH+2][PW+2][32]
// buffer, the tile kernel's input).  SAME 3x3 stride 1, even OH/OW.
// Round 5: persistent workgroups (conv1 is memory-bound: 16 x 16 tiles of 40 MFMAs per wave, so
// a one-tile workgroup spent most of its life waiting for its patch and loading its weights):
// weights loaded once per workgroup, tile t + 1's patch DMA'd into the other buffer while tile t
// computes.  Same products, same order: same bits as the one-tile form (DNN_HIP_C1F16_WGS=0).
__global__ void __launch_bounds__(256)
conv1_patch_f16_kernel(const half_t* __restrict__ in, const half_t* __restrict__ Bt, int ldb,
                       half_t* __restrict__ out, DirectGeom g, int tilesX, int tilesY, const float* __restrict__ zero,
                       EpiParams epi, int opad, int ntiles) {
  constexpr int C = 16;
  constexpr int PATCH = SC_P * SC_P * C;      // halves
  constexpr int PATCH_CH = (PATCH * 2 + 1023) / 1024;  // 1-KiB DMA chunks
  constexpr int SP = 40;  // output stage row pitch (halves): 32 columns + 8
  __shared__ __attribute__((aligned(1024))) float smem[2 * PATCH_CH * 256 + 4 * 16 * SP / 2];
  half_t* const stg = reinterpret_cast<half_t*>(smem + 2 * PATCH_CH * 256);

  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  auto issue = [&](int t, int buf) {  // tile t's patch: 16-B chunks = 8 channels; pixel pp = chunk / 2
    const int tx = t % tilesX, ty = (t / tilesX) % tilesY, b = t / (tilesX * tilesY);
    const int y0 = ty * SC_T, x0 = tx * SC_T;
    const half_t* inb = in + (size_t)b * g.H * g.W * C;
    for (int c = wid; c < PATCH_CH; c += 4) {
      const int q = c * 64 + lane;  // 16-B chunk index
      const int pp = q >> 1, half8 = (q & 1) * 8;
      const int py = pp / SC_P, px = pp - py * SC_P;
      const int iy = y0 - 1 + py, ix = x0 - 1 + px;
      const bool ok = pp < SC_P * SC_P && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      lds_dma16(ok ? reinterpret_cast<const float*>(inb + ((size_t)iy * g.W + ix) * C + half8) : zero,
                smem + buf * (PATCH_CH * 256) + c * 256);
    }
  };

  // B fragments in registers: K-step s (0..4) covers taps 2s, 2s+1; lane part p -> tap 2s + p/2,
  // channels 8(p&1)..+7; N-tile j -> output channel 16j + (lane&15)
  const int fr = lane & 15, fp = lane >> 4;
  h8_t bw[5][2];
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const int tap = 2 * s + (fp >> 1);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (tap < 9)
        bw[s][j] = *reinterpret_cast<const h8_t*>(Bt + (size_t)(16 * j + fr) * ldb + tap * C + 8 * (fp & 1));
      else
        bw[s][j] = h8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  float pb[2], pm[2], ps[2], pg[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = 16 * j + fr;
    pb[j] = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
    pm[j] = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
    ps[j] = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
    pg[j] = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;
  }

  int t = blockIdx.x;
  if (t < ntiles) issue(t, 0);
  for (int k = 0; t < ntiles; ++k, t += gridDim.x) {
    wait_vmcnt<0>();  // this wave's pieces of tile t (and its previous tile's stores)
    raw_barrier();    // every wave's pieces landed; the other buffer's tile read by every wave
    if (t + (int)gridDim.x < ntiles) issue(t + gridDim.x, (k + 1) & 1);
    const half_t* P = reinterpret_cast<const half_t*>(smem + (k & 1) * (PATCH_CH * 256));
    const int tx = t % tilesX, ty = (t / tilesX) % tilesY, b = t / (tilesX * tilesY);
    const int y0 = ty * SC_T, x0 = tx * SC_T;

    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int wi = fr >> 2, pos = fr & 3;
      const int y = 4 * wid + 2 * (i >> 1) + (pos >> 1);
      const int x = 2 * (4 * (i & 1) + wi) + (pos & 1);
      const int base = (y * SC_P + x) * C + 8 * (fp & 1);
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        const int tap = 2 * s + (fp >> 1);
        h8_t a = h8_t{0, 0, 0, 0, 0, 0, 0, 0};
        if (tap < 9) a = *reinterpret_cast<const h8_t*>(P + base + ((tap / 3) * SC_P + tap % 3) * C);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bw[s][j], acc[i][j], 0, 0, 0);
      }
    }

#if C1F16_STAGE
    // the wave's 2 x 8 windows x 32 columns through its LDS stage: one 16-B store per lane
    half_t* const st = stg + wid * (16 * SP);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        st[((i >> 1) * 8 + 4 * (i & 1) + fp) * SP + 16 * j + fr] =
            (half_t)pool_then_epilogue(acc[i][j], pb[j], pm[j], ps[j], pg[j], epi.flags);
    wait_lgkm0();
    {
      typedef half_t h8v __attribute__((ext_vector_type(8)));
      const int wl = lane >> 2, cg = lane & 3;
      const int wy = (y0 >> 1) + 2 * wid + (wl >> 3), wx = (x0 >> 1) + (wl & 7);
      const h8v v = *reinterpret_cast<const h8v*>(st + wl * SP + 8 * cg);
      if (wy < g.PH && wx < g.PW)
        store16_at(out, 2 * ((((size_t)b * (g.PH + 2 * opad) + wy + opad) * (g.PW + 2 * opad) + wx + opad) * 32 + 8 * cg),
                   __builtin_bit_cast(u32x4, v));
    }
#else
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = 16 * j + fr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int wy = (y0 >> 1) + 2 * wid + (i >> 1), wx = (x0 >> 1) + 4 * (i & 1) + fp;
        if (wy < g.PH && wx < g.PW)
          store_out(out + (((size_t)b * (g.PH + 2 * opad) + wy + opad) * (g.PW + 2 * opad) + wx + opad) * 32 + n,
                    pool_then_epilogue(acc[i][j], pb[j], pm[j], ps[j], pg[j], epi.flags));
      }
    }
#endif
    wait_lgkm0();  // (this tile's patch and stage reads done before the barrier that frees its buffer)
  }
}

bool conv1_patch_f16_supported(int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh, int sw, int pt,
                               int pl) {
  return C == 16 && OC == 32 && kh == 3 && kw == 3 && sh == 1 && sw == 1 && pt == 1 && pl == 1 && OH == H &&
         OW == W && OH % 2 == 0 && OW % 2 == 0;
}

int launch_conv1_patch_f16(const half_t* in, const half_t* Bt, int ldb, half_t* out, const DirectGeom& g,
                           const float* zero, const EpiParams& epi, hipStream_t s, int opad) {
  if (g.B == 0) return 0;
  if (ldb < 144 || ldb % 8 || g.OH % 2 || g.OW % 2 || g.PH != g.OH / 2 || g.PW != g.OW / 2 || g.pt != 1 ||
      g.pl != 1 || !zero) {
    set_error("conv1_patch_f16: unsupported shape");
    return -2;
  }
  const int tilesX = (g.OW + SC_T - 1) / SC_T, tilesY = (g.OH + SC_T - 1) / SC_T;
  const long long tiles = (long long)g.B * tilesX * tilesY;
  if (tiles > 0x7fffffffLL) {
    set_error("conv1_patch_f16: too many tiles");
    return -2;
  }
  // persistent workgroups per CU (DNN_HIP_C1F16_WGS; 0: one tile per workgroup)
  const char* ev = getenv("DNN_HIP_C1F16_WGS");
  const int wpc = ev ? atoi(ev) : 8;  // (batch 64: one-tile 73.9 us, 4 per CU 59.9, 8 per CU 56.0)
  int dev = 0, cus = 256;
  if (wpc > 0 && hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const long long blocks = wpc > 0 ? std::min<long long>(tiles, (long long)wpc * cus) : tiles;
  hipLaunchKernelGGL(conv1_patch_f16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, Bt, ldb, out, g, tilesX,
                     tilesY, zero, epi, opad, (int)tiles);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("launch conv1_patch_f16: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

}  // namespace dnnhip
