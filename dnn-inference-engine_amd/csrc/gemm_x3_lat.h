// fp32 3x3 conv on the bf16 MFMA with exact three-way operand splits ("x3", gemm_x3_patch.h) for
// SMALL M: the latency plans (config 2, one frame: conv6 / conv7 of YOLOv2-tiny at M = 169),
// device code only.
//
// At batch 1 the batch kernel's 176 x 256 tiles are 4 per layer: the chip is filled only by
// splitting K, and one 176 x 256 x 288 slice is a long serial chain for its 8 waves (measured
// round 2: conv6 / conv7 as 16 / 32 such slices 0.053 / 0.056 ms with their combines, against
// 0.034 / 0.051 on the fp32 MFMA).  Here a workgroup covers all 176 rows of ONE 32-channel
// chunk (CPW = 1) or two (CPW = 2) for BN = 32 NCP columns, and its 8 waves split that work
// three ways -- NCP column pairs x CPW chunks x RG row groups -- so a wave holds only TMW =
// ceil(11 / RG) row blocks of one chunk: conv7 (32 chunks, N = 1024) as 16 N tiles x 16 slices of
// two chunks, conv6 (16 chunks) as 16 x 16 slices of one chunk, 256 workgroups each, two waves
// per SIMD.  Every workgroup stages its whole patch (all 9 taps of its chunks) by LDS-DMA once,
// then runs 9 taps (unrolled) with the next NB - 1 taps' weights in flight; no barrier inside.
//
// Arithmetic per output as gemm_x3_acc2.h (accm: a0 b0; accc: a2b0, a1b1, a0b2, a1b0, a0b1 over
// the chunk's 9 taps; then accm + accc); CPW = 2 adds the second chunk's sum (through LDS),
// and the slices' raw partials [splits][M][N] are summed in slice order by x3_combine_kernel
// with the epilogue.  The order depends on (N, K) and the launch rule only: a latency plan is
// deterministic but not bit-equal to the batch plan (tolerance, as the fp32 latency plans).
#pragma once
#include "gemm_x3_acc2.h"

namespace dnnhip {

#if (X3DIAG & 512) != 0  // diagnostic builds: per workgroup s_memrealtime at start, patch landed, MFMAs done, end
constexpr int LAT_DIAG_WGS = 1024;
__device__ unsigned long long lat_diag_stamps[LAT_DIAG_WGS * 4];
#define LAT_STAMP(k) \
  if (threadIdx.x == 0 && blockIdx.x < LAT_DIAG_WGS) lat_diag_stamps[4 * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime();
#else
#define LAT_STAMP(k)
#endif

template <int NCP, int CPW, int NPR, int NB = 3, int LP = 224>
__global__ void __launch_bounds__(512, 1)
conv3x3_x3_lat_kernel(const bf16_bits* __restrict__ in, const bf16_bits* __restrict__ Bt, float* __restrict__ part,
                      int M, int N, int K, int tilesM, X3Geom g, unsigned in_bytes, unsigned b_bytes) {
  constexpr int BM = 176, TM = BM / 16, NW = 8, NJ = 2, RB = 192;
  constexpr int RG = NW / (NCP * CPW), TMW = (TM + RG - 1) / RG;
  constexpr int NQ = (NPR * LP + 1023) / 1024;           // 1-KiB DMA pieces per patch
  constexpr int NQW = (CPW * NQ + NW - 1) / NW;          // ... per wave (all patches)
  constexpr int BUFB = NQ * 1024;
  constexpr int RED = CPW > 1 ? NCP * RG * TMW * NJ * 1024 : 0;  // second-chunk sums (f32x4 per lane)
  constexpr int SMEM = CPW * BUFB > RED ? CPW * BUFB : RED;
  static_assert(NCP * CPW * RG == NW && (CPW == 1 || CPW == 2) && LP % 16 == 0 && LP >= RB, "shape");
  static_assert(SMEM <= 160 * 1024, "LDS");
  constexpr int LPB = (3 * NJ + TMW - 1) / TMW;  // next-tap weight loads issued per row block
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];
  LAT_STAMP(0)

  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int cp = wid % NCP, ch = (wid / NCP) % CPW, rg = wid / (NCP * CPW);
  // slice-major inside each XCD's contiguous range: the N tiles of one slice read one patch
  const int tile_s = xcd_tile(blockIdx.x, gridDim.x), ntiles = gridDim.x / g.splits;
  const int split = tile_s / ntiles, tile = tile_s - split * ntiles;
  const int tn = tile / tilesM, tm = tile - tn * tilesM;
  const int m0 = tm * BM, n0 = tn * (32 * NCP) + cp * 32;  // this wave's 32 columns
  const int Wp = g.W + 2, HWo = g.H * g.W;
  auto padded = [&](int m) {
    const int b = m / HWo, r = m - b * HWo, oy = r / g.W, ox = r - oy * g.W;
    return (b * (g.H + 2) + oy + 1) * Wp + ox + 1;
  };
  const int P0 = padded(m0) - (Wp + 1);  // first patch row
  const int mlast = (m0 + BM < M ? m0 + BM : M) - 1;

  // A fragment of this wave's row block i (tile block rg TMW + i): LDS byte offset of the lane's
  // tap (0, 0) row + 16 fq in its chunk's patch
  const int fr = lane & 15, fq = lane >> 4;
  int prow[TMW];
#pragma unroll
  for (int i = 0; i < TMW; ++i) {
    int m = m0 + 16 * (rg * TMW + i) + fr;
    m = m < mlast ? m : mlast;
    prow[i] = ch * BUFB + (padded(m) - P0 - (Wp + 1)) * LP + 16 * fq;
  }

  const int nk = K / 32, chunk0 = split * CPW;
  const int rowB = 6 * g.C;
  // weights [n/16][step][piece][lane][8]: this wave's chunk, two 16-column blocks
  const unsigned bvo = (unsigned)((n0 / 16) * nk * 3072 + (chunk0 + ch) * 9 * 3072 + lane * 16);
  const int bjs = nk * 3072;
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)b_bytes, 0x00020000);
  // a ring of NB taps' weights (each weight is read by this workgroup only, from HBM)
  bf16x8 bq[NB][3][NJ];
  auto load_b1 = [&](int s, int p, int j, bf16x8& dst) {
    dst = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, bvo, s * 3072 + p * 1024 + j * bjs, 0));
  };
#pragma unroll
  for (int s = 0; s < NB - 1; ++s)
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < NJ; ++j) load_b1(s, p, j, bq[s][p][j]);

  // patches: piece q of chunk c lands at LDS byte c BUFB + 1024 q + 16 lane = patch row r, unit u
  // (LP-byte rows: the chunk's 192 data bytes, then never-read padding); all pieces of all the
  // workgroup's chunks spread over the 8 waves, the surplus re-issuing the last piece
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
#pragma unroll
  for (int k = 0; k < NQW; ++k) {
    int q = wid + NW * k;
    q = q < CPW * NQ ? q : CPW * NQ - 1;
    const int c = q / NQ, qq = q - c * NQ;
    const unsigned b = 1024u * (unsigned)qq + 16u * (unsigned)lane;
    const unsigned r = b / LP, u = (b - r * LP) >> 4;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rsA, (__attribute__((address_space(3))) void*)(smem + c * BUFB + 1024 * qq), 16,
        (int)(__umul24(r, (unsigned)rowB) + 16 * u), (int)(P0 * rowB + (chunk0 + c) * RB), 0, 0);
  }

  f32x4 accm[TMW][NJ], accc[TMW][NJ];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      accm[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      accc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  vm_wait<0>();
  __syncthreads();
  LAT_STAMP(1)

  // the last row group's surplus block (RG TMW > 11) is skipped (a uniform branch)
  const bool tail = TMW * RG > TM && rg == RG - 1;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int toff = (t / 3) * Wp + (t % 3);
    bf16x8 (&bc)[3][NJ] = bq[t % NB];
    bf16x8 (&bn)[3][NJ] = bq[(t + NB - 1) % NB];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TMW; ++i) {
      if (t + NB - 1 < 9) {
#pragma unroll
        for (int l = i * LPB; l < (i + 1) * LPB && l < 3 * NJ; ++l) load_b1(t + NB - 1, l / NJ, l % NJ, bn[l / NJ][l % NJ]);
      }
      if (i == TMW - 1 && tail) continue;
      bf16x8 a[3];
      const unsigned char* q = smem + prow[i] + toff * LP;
#pragma unroll
      for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(q + 64 * p);
#pragma unroll
      for (int jb = 0; jb < NJ; ++jb) {
        f32x4 c = accc[i][jb];
        c = mfma16_bf16(a[2], bc[0][jb], c);
        c = mfma16_bf16(a[1], bc[1][jb], c);
        c = mfma16_bf16(a[0], bc[2][jb], c);
        c = mfma16_bf16(a[1], bc[0][jb], c);
        c = mfma16_bf16(a[0], bc[1][jb], c);
        accc[i][jb] = c;
        accm[i][jb] = mfma16_bf16(a[0], bc[0][jb], accm[i][jb]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  vm_wait<0>();
  LAT_STAMP(2)

#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r) accm[i][jb][r] = accm[i][jb][r] + accc[i][jb][r];

  if constexpr (CPW == 2) {  // chunk 0's sum + chunk 1's, through LDS (the patches are dead)
    f32x4* red = reinterpret_cast<f32x4*>(smem);
    auto idx = [&](int i, int jb) { return (((cp * RG + rg) * TMW + i) * NJ + jb) * 64 + lane; };
    __syncthreads();
    if (ch == 1) {
#pragma unroll
      for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int jb = 0; jb < NJ; ++jb) red[idx(i, jb)] = accm[i][jb];
    }
    __syncthreads();
    if (ch == 1) return;
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
      for (int jb = 0; jb < NJ; ++jb) {
        const f32x4 o = red[idx(i, jb)];
#pragma unroll
        for (int r = 0; r < 4; ++r) accm[i][jb][r] = accm[i][jb][r] + o[r];
      }
  }

  // raw partial of slice `split`: part[split][m][n] (x3_combine_kernel sums and runs the epilogue).
  // (Round 4, X3DIAG 512 at one frame, conv7: patch 4.4 us, MFMA loop 8.5-9.3 us for wave 0, the
  // rest of the waves' loops + these stores 4.7 us -- two waves per SIMD make a SIMD's MFMA work
  // ~10 us, and a frame's x3 conv7 is ~9 us of MFMA on all 1,024 SIMDs at 2 GHz; staging these
  // stores through LDS as whole 16-B row pieces measured the same.)
  const size_t dst = (size_t)split * M * N;  // (floats)
#pragma unroll
  for (int i = 0; i < TMW; ++i) {
    if (i == TMW - 1 && tail) continue;
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb) {
      const int n = n0 + 16 * jb + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 16 * (rg * TMW + i) + 4 * fq + r;
        if (m <= mlast) store4_at(part, 4 * (dst + (size_t)m * N + n), accm[i][jb][r]);
      }
    }
  }
  LAT_STAMP(3)
}
#undef LAT_STAMP

}  // namespace dnnhip
