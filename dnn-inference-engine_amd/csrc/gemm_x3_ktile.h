// x3 3x3 conv for the single-frame latency plans' mid layers (YOLOv2-tiny conv4: 26x26x128 ->
// 256 + 2x2 pool, conv5: 13x13x256 -> 512), device code only.
//
// At one frame these layers are 13-26 output rows of 26 or 13 pixels: the batch kernel's
// 176 x 256 tiles are 4 per layer, and the fp32 MFMA's split-K GEMM (its K slices combined by the
// last-arriving workgroup) took 14.4 / 17.5 us, most of it serial MFMA chains (a 32 x 32 wave
// tile over 256-288 of K on the 64-cycle 32x32x2 fp32 MFMA) and the combine's memory round trip.
// Here a workgroup owns a TH x TW tile (one or two image rows) and 32 WN columns, and splits K INSIDE the
// workgroup: KW groups of WM x WN waves, group k taking chunks k CPK .. k CPK + CPK - 1; every
// chunk of the tile's patch is staged by LDS-DMA at once, so no wave waits on another until the
// end, where groups 1 .. KW - 1 hand their folded sums to group 0 through LDS and group 0 adds
// them in group order, then runs the epilogue (fused 2x2 pool, split-plane or fp32 stores) as
// the tile kernel does.  Per output: each group's x3 steps (two accumulators, gemm_x3_patch.h
// x3_step, chunk-major tap-minor), folded, then the groups summed 0, 1, ..., KW - 1: the order
// depends on (N, K, KW) only, deterministic, not the batch kernels' (latency plans are held to
// the fp32 tolerance, as their fp32 split-K GEMMs).
#pragma once
#include "gemm_x3_patch.h"

namespace dnnhip {

#if (X3DIAG & 256) != 0  // diagnostic builds: per workgroup s_memrealtime at start, patch landed, MFMAs done,
                         // end; 14/26-wide tiles at workgroups 0-511, 13-wide at 512-1023
constexpr int KT_DIAG_WGS = 1024;
__device__ unsigned long long ktile_diag_stamps[KT_DIAG_WGS * 4];
#define KT_STAMP(k)                                                       \
  if (threadIdx.x == 0 && blockIdx.x < KT_DIAG_WGS / 2)                   \
    ktile_diag_stamps[4 * (blockIdx.x + (TW > 13 ? 0 : KT_DIAG_WGS / 2)) + (k)] = __builtin_amdgcn_s_memrealtime();
#else
#define KT_STAMP(k)
#endif

template <int TH, int TW, int WM, int WN, int TM, int KW, int CPK, bool POOL, int FL = -1, int NB = 3, bool PL1 = false>
__global__ void __launch_bounds__(64 * WM * WN * KW, 1)
conv3x3_x3_ktile_kernel(const bf16_bits* __restrict__ in, const bf16_bits* __restrict__ Bt, float* __restrict__ out,
                        bf16_bits* __restrict__ out_split, int N, int K, EpiParams epi, int tilesX, int tilesY,
                        int tilesN, X3Geom g, unsigned in_bytes, unsigned b_bytes) {
  constexpr int NG = WM * WN, NW = NG * KW, NT = 64 * NW, LP = 224, PU = LP / 16, PW2 = TW + 2;
  // PL1: a 2x2 stride-1 SAME pool fused (YOLO's pool5): the tile also computes the row below it
  constexpr int TR = PL1 ? (TH + 1) * TW : TH * TW;
  constexpr int PR = (TH + 2 + (PL1 ? 1 : 0)) * PW2, T = TH * TW, NCH = KW * CPK;
  constexpr int NPC = (PR * PU + 63) / 64;           // 1-KiB DMA pieces per chunk
  constexpr int BUFB = NPC * 1024;                   // one chunk's patch
  constexpr int NPW = (NCH * NPC + NW - 1) / NW;     // pieces per wave, all chunks
  constexpr int RED = (KW - 1) * NG * TM * 2 * 1024;  // groups 1 .. KW - 1: f32x4 per lane, block, column block
  constexpr int NO = POOL ? T / 4 : T;
  constexpr int PATCH = NCH * BUFB;
  constexpr int SM = (PATCH > RED ? PATCH : RED);
  static_assert((!POOL || (TH % 2 == 0 && TW % 2 == 0)) && WM * TM * 16 >= TR && (WM * TM - 2) * 16 < TR && NW <= 16,
                "shape");
  static_assert(!PL1 || (!POOL && NG == 1 && 4 * T <= 64 && RED + TR * 36 * 4 <= SM), "stride-1 pool");
  static_assert(SM + NO * 4 <= 160 * 1024 && RED % 1024 == 0 && RED + NG * TM * 4 * X3_STG_ROW * 4 <= SM, "LDS");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SM + NO * 4];
  int* const orow = reinterpret_cast<int*>(smem + SM);

  KT_STAMP(0)
  const int lane = threadIdx.x & 63;
  const int eflags = FL < 0 ? epi.flags : FL;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int kg = wid / NG, wg = wid - kg * NG, wn = wg % WN, wm = wg / WN;
  // column-group-major inside each XCD's contiguous range: the workgroups of one 64-column group
  // (the same weights) share an L2
  const int ntile = (int)gridDim.x / tilesN;
  int t = xcd_tile(blockIdx.x, gridDim.x);
  const int tn = t / ntile;
  t -= tn * ntile;
  const int tx = t % tilesX;
  t /= tilesX;
  const int ty = t % tilesY;
  const int b = t / tilesY;
  const int y0 = ty * TH, x0 = tx * TW;
  const int n0 = tn * (32 * WN) + wn * 32;
  const int Wp = g.W + 2;
  const int fr = lane & 15, fq = lane >> 4;

  int rowoff[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int r = (wm * TM + i) * 16 + fr;
    r = r < TR ? r : TR - 1;
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

  // the whole patch, every chunk: piece q = wid + NW k of the NCH NPC pieces (past the last:
  // the last again) -> chunk q / NPC, LDS units U = 64 (q % NPC) + lane of that chunk's buffer
  const int nk = K / 32;
  const unsigned rowB = 6u * (unsigned)g.C;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  const unsigned pbase = (unsigned)((b * (g.H + 2) + y0) * Wp + x0);
#pragma unroll
  for (int k = 0; k < NPW; ++k) {
    int q = wid + NW * k;
    q = q < NCH * NPC ? q : NCH * NPC - 1;
    const int c = q / NPC, pq = q - c * NPC;
    const unsigned U = 64u * (unsigned)pq + (unsigned)lane;
    unsigned r = U / PU;
    const unsigned u = U - r * PU;
    r = r < (unsigned)PR ? r : (unsigned)PR - 1;
    const unsigned py = r / PW2, px = r - py * PW2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(smem + c * BUFB + 1024 * pq),
                                             16, (int)((pbase + py * (unsigned)Wp + px) * rowB + 16u * u),
                                             (int)(c * 192), 0, 0);
  }

  // weights: this wave's 32 columns, steps 9 (kg CPK) .. 9 (kg CPK + CPK) - 1, NB - 1 ahead in an
  // NB-step register ring (steps past the group's last read the next group's, or zeros past K)
  const unsigned bvo = (unsigned)((n0 / 16) * nk * 3072 + lane * 16);
  const int bjs = nk * 3072;
  const int s0 = 9 * kg * CPK;
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)b_bytes, 0x00020000);
  bf16x8 bq[NB][3][2];
  auto load_b = [&](int s, bf16x8 (&dst)[3][2]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        dst[p][j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, bvo, (s0 + s) * 3072 + p * 1024 + j * bjs, 0));
  };
#pragma unroll
  for (int k = 0; k + 1 < NB; ++k) load_b(k, bq[k]);
  const X3EpiCol ecp[2] = {x3_epi_col(epi, eflags, n0 + fr), x3_epi_col(epi, eflags, n0 + 16 + fr)};  // (prefetched)
  // PL1: this lane's pooled task (pixel lane / 4 of the tile row, channels n0 + 8 (lane % 4) ..
  // + 7) and its 8 channels' epilogue parameters
  f32x4 p1[4][2];
  if constexpr (PL1) {
    const int c = n0 + 8 * (lane & 3);
    const float* src[4] = {epi.bias, epi.mean, epi.sq, epi.gamma};
    const bool use[4] = {(eflags & EPI_BIAS) != 0, (eflags & (EPI_BN | EPI_BN_AB)) != 0,
                         (eflags & (EPI_BN | EPI_BN_AB)) != 0, (eflags & EPI_BN) != 0};
    const float dflt[4] = {0.f, 0.f, 1.f, 1.f};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        p1[q][h] = use[q] ? *reinterpret_cast<const f32x4*>(src[q] + c + 4 * h) : f32x4{dflt[q], dflt[q], dflt[q], dflt[q]};
  }

  f32x4 acc[TM][2], accc[TM][2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = accc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every chunk of the patch landed
  KT_STAMP(1)

  auto frag = [&](const unsigned char* P, int i, int tap, bf16x8 (&a)[3]) {
    const int toff = ((tap / 3) * PW2 + (tap % 3)) * LP;
    const unsigned char* q = P + rowoff[i] + toff;
#pragma unroll
    for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(q + 64 * p);
  };
#pragma unroll
  for (int cc = 0; cc < CPK; ++cc) {
    const unsigned char* P = smem + (kg * CPK + cc) * BUFB;
    bf16x8 af[2][3];
    frag(P, 0, 0, af[0]);
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int s = 9 * cc + tp;
      __builtin_amdgcn_sched_barrier(0);
      load_b(s + NB - 1, bq[(s + NB - 1) % NB]);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int cur = i & 1, nxt = cur ^ 1;
        if (i + 1 < TM)
          frag(P, i + 1, tp, af[nxt]);
        else if (tp < 8)
          frag(P, 0, tp + 1, af[nxt]);
        const bf16x8(&bb)[3][2] = bq[s % NB];
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
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  x3_fold(acc, accc);
  KT_STAMP(2)

  // groups 1 .. KW - 1 hand their sums to group 0 (the patch area is free once every wave is past
  // its last fragment read); group 0 adds them in group order
  wait_lgkm0();
  __syncthreads();
  f32x4* const red = reinterpret_cast<f32x4*>(smem);
  if (kg > 0) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) red[((((kg - 1) * NG + wg) * TM + i) * 2 + jb) * 64 + lane] = acc[i][jb];
  }
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
  if (kg > 0) return;
#pragma unroll
  for (int k = 1; k < KW; ++k)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) acc[i][jb] = acc[i][jb] + red[((((k - 1) * NG + wg) * TM + i) * 2 + jb) * 64 + lane];

  if constexpr (PL1) {
    // raw sums of the TH + 1 computed rows into a wave-private stage (rows of 36 floats, past
    // `red`), then per lane one task: pixel x of the tile's row, 8 channels; window (y, x), (y,
    // x + 1), (y + 1, x), (y + 1, x + 1) with x + 1 / y + 1 clamped into the frame (SAME: the
    // pad never wins a max), pooled before the epilogue (pool_then_epilogue, as the 2x2/s2 pools)
    float* stg = reinterpret_cast<float*>(smem + RED);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * i + 4 * fq + r;
          if (row < TR) stg[row * 36 + 16 * jb + fr] = acc[i][jb][r];
        }
    wait_lgkm0();
    const int x = lane >> 2, c8 = 8 * (lane & 3);
    if (lane < 4 * T) {
      const int y = y0 + x / TW, xx = x0 + x % TW;  // (TH = 1: x / TW = 0)
      if (y < g.H && xx < g.W) {
        const int lx = x % TW, ly = x / TW;
        const int lx1 = xx + 1 < g.W ? lx + 1 : lx, ly1 = y + 1 < g.H ? ly + 1 : ly;
        const int ra = ly * TW + lx, rb = ly * TW + lx1, rc = ly1 * TW + lx, rd = ly1 * TW + lx1;
        float o[8];
        f32x4 win[1][8];
        float cb[8], cm[8], cs[8], cg[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 va = *reinterpret_cast<const f32x4*>(stg + ra * 36 + c8 + 4 * h);
          const f32x4 vb = *reinterpret_cast<const f32x4*>(stg + rb * 36 + c8 + 4 * h);
          const f32x4 vc = *reinterpret_cast<const f32x4*>(stg + rc * 36 + c8 + 4 * h);
          const f32x4 vd = *reinterpret_cast<const f32x4*>(stg + rd * 36 + c8 + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            win[0][4 * h + e] = f32x4{va[e], vb[e], vc[e], vd[e]};
            cb[4 * h + e] = p1[0][h][e], cm[4 * h + e] = p1[1][h][e], cs[4 * h + e] = p1[2][h][e], cg[4 * h + e] = p1[3][h][e];
          }
        }
        pool_epilogue_batch<FL>(win, cb, cm, cs, cg, epi.flags, [&](int, int c, float e) { o[c] = e; });
        if (g.out_mode == 1) {
          const size_t op = ((size_t)b * (g.H + 2) + y + 1) * (size_t)Wp + xx + 1;
          u32x4 q[3];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            unsigned w0, w1, w2;
            split3_pack2(false, o[2 * e], o[2 * e + 1], w0, w1, w2);
            q[0][e] = w0;
            q[1][e] = w1;
            q[2][e] = w2;
          }
          const size_t d = op * (3 * (size_t)N) + (n0 >> 5) * 96 + c8;
#pragma unroll
          for (int pc = 0; pc < 3; ++pc) store16_at(out_split, 2 * (d + 32 * pc), q[pc]);
        } else {
          const size_t d = (((size_t)b * g.H + y) * g.W + xx) * N + n0 + c8;
          store16_at(out, 4 * d, __builtin_bit_cast(u32x4, f32x4{o[0], o[1], o[2], o[3]}));
          store16_at(out, 4 * d + 16, __builtin_bit_cast(u32x4, f32x4{o[4], o[5], o[6], o[7]}));
        }
      }
    }
    KT_STAMP(3)
    return;
  }

  if constexpr (POOL) {
    if (g.out_mode == 1) {  // staged 16-B split-plane stores (x3_pool_split_store), group 0's waves
      float* stg = reinterpret_cast<float*>(smem + RED) + wg * (TM * 4 * X3_STG_ROW);  // (past `red`)
      const float cb[2] = {ecp[0].pb, ecp[1].pb}, cm[2] = {ecp[0].pm, ecp[1].pm}, cs[2] = {ecp[0].ps, ecp[1].ps},
                  cg[2] = {ecp[0].pg, ecp[1].pg};
      pool_epilogue_batch<FL>(acc, cb, cm, cs, cg, epi.flags,
                              [&](int i, int jb, float v) { stg[(4 * i + fq) * X3_STG_ROW + 16 * jb + fr] = v; });
      x3_pool_split_store<TM>(stg, orow, NO, 4 * wm * TM, out_split, 3 * (size_t)N, (n0 >> 5) * 96, lane);
      KT_STAMP(3)
      return;
    }
  }
#pragma unroll
  for (int jb = 0; jb < 2; ++jb) {
    const int n = n0 + 16 * jb + fr;
    const float pb = ecp[jb].pb, pm = ecp[jb].pm, ps = ecp[jb].ps, pg = ecp[jb].pg;
    const int cofs = (n >> 5) * 96 + (n & 31);
    auto put = [&](int o, float v) {
      if (g.out_mode == 1) {
        unsigned short s0_, s1_, s2_;
        split3(v, s0_, s1_, s2_);
        bf16_bits* d = out_split + (size_t)o * (3 * N) + cofs;
        d[0] = s0_;
        d[32] = s1_;
        d[64] = s2_;
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
  KT_STAMP(3)
}
#undef KT_STAMP

// The 1x1 form (latency plans' conv8: 13x13x1024 -> 125 on conv7's split planes): 16 pixel rows
// x 32 columns per workgroup, KW groups of one wave, group k taking chunks k CPK .. k CPK + CPK -
// 1; every chunk's 16 rows staged by LDS-DMA at once, the groups' folded sums added in group
// order by group 0, fp32 epilogue into out [M][N] (columns past N, the packing's padding, not
// stored).  At one frame: 11 x 4 = 44 workgroups with an 8-step chain each, where the batch
// kernel's 32 x 128 tiles over all of K were 6 (21 us) and the fp32 split-K GEMM 11.5 us.
template <int KW, int CPK, int FL = -1, int NJ = 2>  // NJ: 16-column blocks per workgroup (1 or 2)
__global__ void __launch_bounds__(64 * KW, 1)
conv1x1_x3_ktile_kernel(const bf16_bits* __restrict__ in, const bf16_bits* __restrict__ Bt, float* __restrict__ out,
                        int M, int N, int K, EpiParams epi, int tilesM, X3Geom g, unsigned in_bytes,
                        unsigned b_bytes) {
  constexpr int NW = KW, LP = 224, PU = LP / 16, BM = 16, NCH = KW * CPK;
  constexpr int NPC = (BM * PU + 63) / 64;        // 1-KiB DMA pieces per chunk (16 rows: 4)
  constexpr int BUFB = NPC * 1024;
  constexpr int NPW = (NCH * NPC + NW - 1) / NW;  // pieces per wave, all chunks
  constexpr int RED = (KW - 1) * 2 * 1024;
  constexpr int SM = NCH * BUFB > RED ? NCH * BUFB : RED;
  static_assert(SM <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SM];

  const int lane = threadIdx.x & 63;
  const int eflags = FL < 0 ? epi.flags : FL;
  const int kg = wave_uniform(threadIdx.x >> 6);
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int tn = tile / tilesM, tm = tile - tn * tilesM;
  const int m0 = tm * BM, n0 = tn * 16 * NJ;
  const int fr = lane & 15, fq = lane >> 4;
  const int nk = K / 32, Wp = g.W + 2, HWo = g.H * g.W;
  auto padded = [&](int m) {
    m = m < M ? m : M - 1;
    const int b = m / HWo, r = m - b * HWo, oy = r / g.W, ox = r - oy * g.W;
    return (b * (g.H + 2) + oy + 1) * Wp + ox + 1;
  };

  const unsigned rowB = 6u * (unsigned)g.C;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
#pragma unroll
  for (int k = 0; k < NPW; ++k) {
    int q = kg + NW * k;
    q = q < NCH * NPC ? q : NCH * NPC - 1;
    const int c = q / NPC, pq = q - c * NPC;
    const unsigned U = 64u * (unsigned)pq + (unsigned)lane;
    unsigned r = U / PU;
    const unsigned u = U - r * PU;
    r = r < (unsigned)BM ? r : (unsigned)BM - 1;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(smem + c * BUFB + 1024 * pq),
                                             16, (int)((unsigned)padded(m0 + (int)r) * rowB + 16u * u),
                                             (int)(c * 192), 0, 0);
  }
  const unsigned bvo = (unsigned)((n0 / 16) * nk * 3072 + lane * 16);
  const int bjs = nk * 3072, s0 = kg * CPK;
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)b_bytes, 0x00020000);
  bf16x8 bq[CPK][3][2];  // every step of the group's chunks in flight at once (CPK <= 8)
#pragma unroll
  for (int c = 0; c < CPK; ++c)
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bq[c][p][j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, bvo, (s0 + c) * 3072 + p * 1024 + j * bjs, 0));
  const X3EpiCol ecp[2] = {x3_epi_col(epi, eflags, n0 + fr < N ? n0 + fr : N - 1),
                           x3_epi_col(epi, eflags, n0 + 16 + fr < N ? n0 + 16 + fr : N - 1)};
  f32x4 acc[2], accc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) acc[j] = accc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int c = 0; c < CPK; ++c) {
    const unsigned char* P = smem + (s0 + c) * BUFB + fr * LP + 16 * fq;
    bf16x8 af[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) af[p] = *reinterpret_cast<const bf16x8*>(P + 64 * p);
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb) x3_step<true>(acc[jb], accc[jb], af, bq[c], jb);
  }
#pragma unroll
  for (int jb = 0; jb < NJ; ++jb) acc[jb] = acc[jb] + accc[jb];  // (x3_fold)
  wait_lgkm0();
  __syncthreads();
  f32x4* const red = reinterpret_cast<f32x4*>(smem);
  if (kg > 0) {
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb) red[((kg - 1) * 2 + jb) * 64 + lane] = acc[jb];
  }
  __syncthreads();
  if (kg > 0) return;
#pragma unroll
  for (int k = 1; k < KW; ++k)
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb) acc[jb] = acc[jb] + red[((k - 1) * 2 + jb) * 64 + lane];
#pragma unroll
  for (int jb = 0; jb < NJ; ++jb) {
    const int n = n0 + 16 * jb + fr;
    if (n >= N) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + 4 * fq + r;
      if (m < M)
        out[(size_t)m * N + n] = apply_epilogue_t<FL>(acc[jb][r], ecp[jb].pb, ecp[jb].pm, ecp[jb].ps, ecp[jb].pg, epi.flags);
    }
  }
}

}  // namespace dnnhip
