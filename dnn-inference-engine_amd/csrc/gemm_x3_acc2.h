// fp32 3x3 conv on the bf16 MFMA with exact three-way operand splits ("x3", gemm_x3_patch.h),
// two accumulators per output and no per-step adds: the default kernel of the wide-N layers of
// the fp32 path (YOLOv2-tiny conv4-conv7), device code only.
//
// Round 2's kernel summed each 32-channel step's five correction products from zero and added
// them into the accumulator: 4 v_add per 6 MFMAs, with two waves per SIMD sharing the vector
// issue of v_mfma_f32_16x16x32_bf16's 16-cycle slot.  Here every output keeps TWO accumulators over the whole K range: `accm` takes the main
// product a0*b0 of every step, `accc` the five corrections a2b0 + a1b1 + a0b2 + a1b0 + a0b1;
// the output is accm + accc, one add per output at the end.  The main accumulator still sees
// one MFMA rounding per step and no longer the per-step add; the corrections (<= 2^-7 of the
// main product each) are rounded at their own, 2^-8 smaller, magnitude
// (tests/test_gpu_parity.py::test_x3_conv_vs_oracle holds the error to <= 1.25x the fp32
// MFMA path's).  Summation order: per output, accm over the steps (chunk-major, tap-minor) of
// a0 b0; accc over the same steps of (a2b0, a1b1, a1b0, a0b2, a0b1) in that order; then
// accm + accc.  It depends on (N, K) only (batch rows are
// bit-identical to batch-1 runs).
#pragma once
#include "gemm_x3_patch.h"

// X3DIAG (diagnostic builds only, tools/build_diag.sh; wrong results unless noted): bit 1 drops
// the loop's patch DMA (the patch keeps chunk 0), 2 its weight loads (tap 0's weights
// throughout), 4 the epilogue of fp32-output layers, 8 the chunk barrier; bit 16 (results
// unchanged) records per workgroup s_memtime / s_memrealtime at the main loop's start and end in
// x3_diag_stamps (read by dnn_x3_diag_stamps): the in-kernel clock (MI355X_MICROARCH, DVFS item
// 6).  Operand data stays random: zero operands clock higher and would flatter the variant.
#ifndef X3DIAG
#define X3DIAG 0
#endif
namespace dnnhip {

#if (X3DIAG & 16) != 0
constexpr int X3_DIAG_WGS = 8192;
__device__ unsigned long long x3_diag_stamps[X3_DIAG_WGS * 4];  // [workgroup][t0, r0, t1, r1]
#endif
#if (X3DIAG & 8192) != 0  // per-layer phase stamps (results unchanged), wave 0:
// [layer: N = 256 / 512 / other][workgroup][0 s_memrealtime start, 1 s_memtime start, 2 prologue
// done, 3 loop done, 4 end, 5 s_memrealtime end, 6 HW_ID, 7 XCC_ID]
constexpr int AC_DIAG_WGS = 512;
__device__ unsigned long long acc2_diag_stamps[3 * AC_DIAG_WGS * 8];
#define AC_STAMP(k, v)                                                                                      \
  if (threadIdx.x == 0 && blockIdx.x < AC_DIAG_WGS)                                                         \
    acc2_diag_stamps[((N == 256 ? 0 : N == 512 ? 1 : 2) * AC_DIAG_WGS + blockIdx.x) * 8 + (k)] = (v);
#else
#define AC_STAMP(k, v)
#endif

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Structure: BM x 256 tiles, 8 waves of BM x 32 (two per SIMD, 256 registers each: the two
// accumulator sets take 176), the weights of the next tap loaded while this one runs (48), the
// patch of one 32-channel chunk staged by LDS-DMA into a double buffer (no staging registers),
// one barrier per chunk.  Why two waves per SIMD: a one-wave-per-SIMD form (4 waves of 176 x 64
// with 512 registers, round 3, git history) lost its MFMA pipe to the issue cost of every
// vector-memory instruction (~60 cycles each: the weight loads alone 12 % of the kernel,
// measured with diagnostic builds that dropped them), which only a partner wave can cover.
// LDS rows of LP = 224 bytes (the 192 data bytes; the padding bytes are whatever follows the
// chunk in global memory, never read): 192-B rows cost 7 bank-conflict cycles per fragment read
// at 13-wide frames, 224 about 4 (tools/lds_conflict_model.py: the two 8-lane halves of each
// ds_read_b128 lane group fall on even / odd bank quads for any 8 rows distinct mod 8; the
// image-row wraps inside a 16-row fragment leave the rest) with plain row-offset addresses.
// (Measured and removed in round 4, in git history: 192-B rows, an XOR swizzle (~5 VALU per
// fragment), a row-skewed layout without the wrap conflicts (+64 -> 142 VALU per tap: conv7
// +3.7 %), a stagger of waves 4-7's loads (+1.6-2.6 %).)
// The next row block's A fragments are read inside this block's MFMAs, each piece as soon as
// this block's last MFMA on that piece has issued (correction order a2b0, a1b1, a1b0, a0b2, a0b1
// -- a2 and a1 retire early), so their LDS latency is covered by the wave's own MFMAs; the patch
// rows are packed three per register to make room (conv7 -2 %, conv6 -1.5 %).
// FL: the epilogue flag set at compile time (-1: runtime `epi.flags`; the launcher compiles in
// YOLO's bias + BatchNorm + double-rounded leaky set), same arithmetic either way.
template <int BM, int NPR, bool POOL, int FL = -1>
__global__ void __launch_bounds__(512, 2)
conv3x3_x3_acc2_kernel(const bf16_bits* __restrict__ in, const bf16_bits* __restrict__ Bt, float* __restrict__ out,
                       bf16_bits* __restrict__ out_split, int M, int N, int K, EpiParams epi, int tilesM, X3Geom g,
                       unsigned in_bytes, unsigned b_bytes) {
  constexpr int BN = 256, TM = BM / 16, RB = 192, NJ = 2, NW = 8, LP = 224;
  constexpr int NQW = (NPR * LP + NW * 1024 - 1) / (NW * 1024);  // 1-KiB DMA pieces per wave per patch
  constexpr int BUFB = NQW * NW * 1024;                            // one patch buffer (>= NPR LP)
  static_assert(BM % 16 == 0 && NQW <= 18 && NPR <= 1023, "shape");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUFB];

  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  AC_STAMP(0, __builtin_amdgcn_s_memrealtime())
  AC_STAMP(1, __builtin_amdgcn_s_memtime())
  AC_STAMP(6, (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)))
  AC_STAMP(7, (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11)))
  const int tile_s = xcd_tile(blockIdx.x, gridDim.x), ntiles = gridDim.x / g.splits;
  const int split = tile_s / ntiles, tile = tile_s - split * ntiles;
  // tiles N-major inside each XCD's contiguous range (~31 M tiles of one N panel per XCD).
  // (Round 4: 2 panels x ~16 M tiles per XCD, so each patch is fetched from beyond L2 by 2 XCDs
  // instead of 4, measured within 0.5 % on conv4-conv7: the patch DMA's beyond-L2 bytes are not
  // what costs -- tools/x3_ab.py, git history)
  const int tn = tile / tilesM, tm = tile - tn * tilesM;
  const int m0 = tm * BM, n0 = tn * BN + wid * 32;  // this wave's 32 columns
  const int Wp = g.W + 2, HWo = g.H * g.W;
  auto padded = [&](int m) {
    const int b = m / HWo, r = m - b * HWo, oy = r / g.W, ox = r - oy * g.W;
    return (b * (g.H + 2) + oy + 1) * Wp + ox + 1;
  };
  auto pixrow = [&](int m) {
    if constexpr (!POOL) {
      return padded(m);
    } else {
      const int w = m >> 2, q = m & 3, PHW = g.PH * g.PW;
      const int b = w / PHW, r = w - b * PHW, py = r / g.PW, px = r - py * g.PW;
      int oy = 2 * py + (q >> 1), ox = 2 * px + (q & 1);
      if (oy >= g.H || ox >= g.W) oy = 2 * py, ox = 2 * px;
      return (b * (g.H + 2) + oy + 1) * Wp + ox + 1;
    }
  };
  const int P0 = pixrow(m0) - (Wp + 1);  // first patch row

  // A fragment of row-block i: patch row of the lane's tap (0, 0) (rows past M repeat row M - 1),
  // packed three per register (10-bit fields: a patch row < NPR <= 1023); unpacked per use
  const int fr = lane & 15, fq = lane >> 4;
  constexpr int NPK = (TM + 2) / 3;
  unsigned prk[NPK];
#pragma unroll
  for (int k = 0; k < NPK; ++k) prk[k] = 0;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int m = m0 + 16 * i + fr;
    m = m < M ? m : M - 1;
    prk[i / 3] |= (unsigned)(pixrow(m) - P0 - (Wp + 1)) << (10 * (i % 3));
  }
  auto rowoff = [&](int i) {  // byte offset of block i's tap-(0, 0) fragment
    unsigned w = prk[i / 3];
    asm volatile("" : "+v"(w));  // unpacked per use: hoisted out of the tap loop it is 11 registers again
    const unsigned pr = (w >> (10 * (i % 3))) & 1023u;
    return (int)__umul24(pr, (unsigned)LP) + 16 * fq;
  };

  // patch DMA: this wave's piece k lands at LDS byte 1024 (wid + 8 k) + 16 lane = patch row r
  // (LP bytes each: the 192 data bytes of the chunk and the next LP - 192 bytes of global memory
  // as never-read padding), unit u; one 16-B unit from (P0 + r) rowB + chunk 192 + 16 u
  const int nk = K / 32, nch = nk / 9 / g.splits, cb = split * nch;
  const int rowB = 6 * g.C;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  const unsigned dsoff = (unsigned)(P0 * rowB + cb * RB);
  auto issue_patch = [&](int chunk, int k, int buf) {
    const unsigned b = 1024u * (unsigned)(wid + NW * k) + 16u * (unsigned)lane;
    const unsigned r = b / LP, u = (b - r * LP) >> 4;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rsA, (__attribute__((address_space(3))) void*)(smem + buf * BUFB + 1024 * (wid + NW * k)), 16,
        (int)(__umul24(r, (unsigned)rowB) + 16 * u), (int)(dsoff + chunk * RB), 0, 0);
  };

  // weights [n/16][step][piece][lane][8]: the wave's two 16-column blocks, one tap ahead
  const unsigned bvo = (unsigned)((n0 / 16) * nk * 3072 + lane * 16 + cb * 9 * 3072);
  const int bjs = nk * 3072;
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)b_bytes, 0x00020000);
  bf16x8 bq[2][3][NJ];
  auto load_b1 = [&](int s, int p, int j, bf16x8& dst) {
    dst = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, bvo, s * 3072 + p * 1024 + j * bjs, 0));
  };
  auto load_b = [&](int s, bf16x8 (&dst)[3][NJ]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < NJ; ++j) load_b1(s, p, j, dst[p][j]);
  };

  f32x4 accm[TM][NJ], accc[TM][NJ];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      accm[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      accc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

#pragma unroll
  for (int k = 0; k < NQW; ++k) issue_patch(0, k, 0);
  load_b(0, bq[0]);
  vm_wait<0>();
  __syncthreads();
  AC_STAMP(2, __builtin_amdgcn_s_memtime())
#if (X3DIAG & 16) != 0
  const unsigned long long st0 = __builtin_amdgcn_s_memtime(), sr0 = __builtin_amdgcn_s_memrealtime();
#endif

  // Per tap: TM row blocks of 12 MFMAs (per column block the five corrections back to back,
  // then the main product), the first ones also issuing the next tap's weights and DMA pieces
  // t (and t + 9 when NQW > 9) of chunk j + 1; the chunk's barrier after tap 8 waits for this
  // wave's DMA pieces and everyone's reads.
  const int nsteps = 9 * nch;
  const unsigned char* P = smem;
  int t = 0, j = 0;
  bf16x8 af[3];  // the current block's fragments, read during the previous block
  auto read_frag = [&](const unsigned char* q, int p) { af[p] = *reinterpret_cast<const bf16x8*>(q + 64 * p); };
#pragma unroll
  for (int p = 0; p < 3; ++p) read_frag(P + rowoff(0), p);
  for (int s = 0; s < nsteps; ++s) {
    const int toff = (t / 3) * Wp + (t % 3);  // tap (dy, dx) relative to (0, 0)
    const int toffn = t < 8 ? ((t + 1) / 3) * Wp + ((t + 1) % 3) : 0;  // the next tap's
    const int toffB = toff * LP, toffnB = toffn * LP;                  // ... in LDS bytes
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      // the tap's vector-memory instructions spread over its first row blocks (one each: a
      // lone wave stalls ~60 cycles per issue, and waves in step after the chunk barrier would
      // otherwise all stall at once): the next tap's 6 weight fragments, then the DMA pieces
      static_assert(TM >= 3 * NJ + 2, "row blocks to spread the tap's loads over");
      static_for<0, 3 * NJ + 2>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        if (i != q) return;
        if constexpr (q < 3 * NJ) {
          if constexpr ((X3DIAG & 2) != 0)
            bq[1][q / NJ][q % NJ] = bq[0][q / NJ][q % NJ];  // (the same random weights every tap)
          else
            load_b1(s + 1, q / NJ, q % NJ, bq[1][q / NJ][q % NJ]);
        }
        if constexpr (q == 3 * NJ && !(X3DIAG & 1)) issue_patch(j + 1, t < NQW ? t : NQW - 1, (j + 1) & 1);  // (uniform count per tap)
        if constexpr (NQW > 9 && q == 3 * NJ + 1 && !(X3DIAG & 1))  // pieces past NQW rewrite piece NQW - 1
          issue_patch(j + 1, t + 9 < NQW ? t + 9 : NQW - 1, (j + 1) & 1);
      });
      // next block: block i + 1 of this tap, or block 0 of the next tap (after tap 8 the read
      // goes to this chunk's buffer and is repeated from the next one after the barrier)
      const unsigned char* qn = i + 1 < TM ? P + rowoff(i + 1 < TM ? i + 1 : 0) + toffB : P + rowoff(0) + toffnB;
      bf16x8 a[3] = {af[0], af[1], af[2]};
#pragma unroll
      for (int jb = 0; jb < NJ; ++jb) {
        const bool lastjb = jb == NJ - 1;
        f32x4 c = accc[i][jb];
        c = mfma16_bf16(a[2], bq[0][0][jb], c);
        if (lastjb) read_frag(qn, 2);
        c = mfma16_bf16(a[1], bq[0][1][jb], c);
        c = mfma16_bf16(a[1], bq[0][0][jb], c);
        if (lastjb) read_frag(qn, 1);
        c = mfma16_bf16(a[0], bq[0][2][jb], c);
        c = mfma16_bf16(a[0], bq[0][1][jb], c);
        accc[i][jb] = c;
        accm[i][jb] = mfma16_bf16(a[0], bq[0][0][jb], accm[i][jb]);
        if (lastjb) read_frag(qn, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int jb = 0; jb < NJ; ++jb) bq[0][p][jb] = bq[1][p][jb];
    if (++t == 9) {
      t = 0;
      ++j;
      vm_wait<0>();  // this wave's DMA pieces landed (issued mid-tap: ~5 row blocks ago)
      wait_lgkm0();
      if (!(X3DIAG & 8)) raw_barrier();
      P = smem + (j & 1) * BUFB;
#pragma unroll
      for (int p = 0; p < 3; ++p) read_frag(P + rowoff(0), p);
    }
  }
  vm_wait<0>();
  AC_STAMP(3, __builtin_amdgcn_s_memtime())
#if (X3DIAG & 16) != 0
  {
    const unsigned long long st1 = __builtin_amdgcn_s_memtime(), sr1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x < X3_DIAG_WGS) {  // (vector stores from lane 0)
      unsigned long long* d = x3_diag_stamps + 4 * blockIdx.x;
      d[0] = st0;
      d[1] = sr0;
      d[2] = st1;
      d[3] = sr1;
    }
  }
#endif

  // epilogue: the reference's fp32 epilogue on accm + accc, then fp32 [M][N], the split planes of
  // the next x3 layer's zero-bordered input, or the raw partial of split-K slice `split`
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r) accm[i][jb][r] = accm[i][jb][r] + accc[i][jb][r];
  int* orow = reinterpret_cast<int*>(smem);
  if ((X3DIAG & 4) != 0 && g.out_mode == 0) {  // keep the sums live without storing them (fp32-out
    // layers only: a skipped producer would hand its consumer zeros, which clock higher)
    float z = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int jb = 0; jb < NJ; ++jb) z += accm[i][jb][0] + accm[i][jb][1] + accm[i][jb][2] + accm[i][jb][3];
    if (z == 1.2345f) out[0] = z;
    return;
  }
  __syncthreads();
  if constexpr (POOL) {
    if (threadIdx.x < BM / 4) {
      const int w = (m0 >> 2) + threadIdx.x, PHW = g.PH * g.PW;
      const int b = w / PHW, r = w - b * PHW, py = r / g.PW, px = r - py * g.PW;
      orow[threadIdx.x] = 4 * w >= M ? -1 : g.out_mode == 1 ? (b * (g.PH + 2) + py + 1) * (g.PW + 2) + px + 1 : w;
    }
    __syncthreads();
    if (g.out_mode == 1) {  // staged 16-B split-plane stores (x3_pool_split_store)
      static_assert(1024 + NW * TM * 4 * X3_STG_ROW * 4 <= 2 * BUFB && BM <= 1024, "stage");
      float* stg = reinterpret_cast<float*>(smem + 1024) + wid * (TM * 4 * X3_STG_ROW);
      float pb[NJ], pm[NJ], ps[NJ], pg[NJ];
#pragma unroll
      for (int jb = 0; jb < NJ; ++jb) {
        const X3EpiCol ec = x3_epi_col(epi, FL < 0 ? epi.flags : FL, n0 + 16 * jb + fr);
        pb[jb] = ec.pb, pm[jb] = ec.pm, ps[jb] = ec.ps, pg[jb] = ec.pg;
      }
      pool_epilogue_batch<FL>(accm, pb, pm, ps, pg, epi.flags,
                              [&](int i, int jb, float v) { stg[(4 * i + fq) * X3_STG_ROW + 16 * jb + fr] = v; });
      x3_pool_split_store<TM>(stg, orow, BM / 4, 0, out_split, 3 * (size_t)N, (n0 >> 5) * 96, lane);
      AC_STAMP(4, __builtin_amdgcn_s_memtime())
      AC_STAMP(5, __builtin_amdgcn_s_memrealtime())
      return;
    }
    static_for<0, NJ>([&](auto jbc) {
      constexpr int jb = decltype(jbc)::value;
      const int n = n0 + 16 * jb + fr;
      const float pb = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
      const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
      const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
      const float pg = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;
      const int cofs = (n >> 5) * 96 + (n & 31);
      static_for<0, TM>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const int o = orow[4 * i + fq];
        if (o < 0) return;
        const float e = pool_then_epilogue_t<FL>(accm[i][jb], pb, pm, ps, pg, epi.flags);
        if (g.out_mode == 1) {
          unsigned short s0, s1, s2;
          split3(e, s0, s1, s2);
          bf16_bits* d = out_split + (size_t)o * (3 * N) + cofs;
          d[0] = s0;
          d[32] = s1;
          d[64] = s2;
        } else {
          out[(size_t)o * N + n] = e;
        }
      });
    });
    return;
  }
  if (threadIdx.x < BM) {
    const int m = m0 + threadIdx.x;
    orow[threadIdx.x] = m >= M ? -1 : (g.out_mode == 1 ? padded(m) : m);
  }
  __syncthreads();
  // Each row block's 16 x 32 outputs of the wave pass through a wave-private LDS stage (fp32 rows
  // of 36: the MFMA-layout writes are conflict-free) and leave as 16-B stores: lane l takes row
  // l / 4, columns 8 (l % 4) .. + 7 -- 2 stores of fp32, or 3 of split planes (one per piece), per
  // row block where the MFMA layout stored one scalar per output (3 per output as split planes).
  // Same epilogue arithmetic and split per value as before.
  static_assert(BM * 4 <= 1024, "row table below the stages");
  float* const stg = reinterpret_cast<float*>(smem + 1024) + wid * (16 * 36);
  float pb[NJ], pm[NJ], ps[NJ], pg[NJ];
#pragma unroll
  for (int jb = 0; jb < NJ; ++jb) {
    const int f = FL < 0 ? epi.flags : FL;
    const int n = n0 + 16 * jb + fr;
    pb[jb] = (f & EPI_BIAS) ? epi.bias[n] : 0.f;
    pm[jb] = (f & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
    ps[jb] = (f & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
    pg[jb] = (f & EPI_BN) ? epi.gamma[n] : 1.f;
  }
  const int rr = lane >> 2, c8 = 8 * (lane & 3);
  static_for<0, TM>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    float v[4][NJ];
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r][jb] = accm[i][jb][r];
    if (g.out_mode != 2) epilogue_batch<FL>(v, pb, pm, ps, pg, epi.flags);
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r) stg[(4 * fq + r) * 36 + 16 * jb + fr] = v[r][jb];
    wait_lgkm0();
    const f32x4 lo = *reinterpret_cast<const f32x4*>(stg + rr * 36 + c8);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(stg + rr * 36 + c8 + 4);
    const int o = orow[16 * i + rr];
    wait_lgkm0();  // (the stage is rewritten by the next row block)
    if (o >= 0) {
      if (g.out_mode == 1) {
        bool ok = true;
#pragma unroll
        for (int e = 0; e < 4; ++e) ok = ok && x3_split_ok(lo[e]) && x3_split_ok(hi[e]);
        const bool fast = __builtin_amdgcn_ballot_w64(!ok) == 0;  // (over the active lanes: uniform among them)
        u32x4 q[3];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          unsigned w0, w1, w2;
          split3_pack2(fast, e < 2 ? lo[2 * e] : hi[2 * e - 4], e < 2 ? lo[2 * e + 1] : hi[2 * e - 3], w0, w1, w2);
          q[0][e] = w0;
          q[1][e] = w1;
          q[2][e] = w2;
        }
        const size_t d = (size_t)o * (3 * N) + (n0 >> 5) * 96 + c8;  // (halves)
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) store16_at(out_split, 2 * (d + 32 * pc), q[pc]);
      } else {
        const size_t d = ((size_t)(g.out_mode == 2 ? split * M : 0) + o) * N + n0 + c8;  // (floats)
        store16_at(out, 4 * d, __builtin_bit_cast(u32x4, lo));
        store16_at(out, 4 * d + 16, __builtin_bit_cast(u32x4, hi));
      }
    }
  });
  AC_STAMP(4, __builtin_amdgcn_s_memtime())
  AC_STAMP(5, __builtin_amdgcn_s_memrealtime())
}
#undef AC_STAMP

}  // namespace dnnhip
