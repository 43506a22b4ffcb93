// fp16 3x3 conv for the long-K, wide-N layers on the fp16 path (conv6/conv7 of YOLOv2-tiny,
// BASELINE config 5), round 3: the x3 kernel's structure (gemm_x3_acc2.h) for one product per
// MFMA, device code only.
//
// Why a successor to conv3x3_f16_patch_kernel (gemm_f16_patch.h): there every wave owns 176 x 32
// outputs, so each 16-row A fragment (one ds_read_b128) feeds 2 MFMAs.  Per CU and 64-channel
// chunk that is 8 waves x 9 taps x 11 blocks x 2 groups = 1,584 fragment reads at 4 + ~3.9 LDS
// cycles each (tools/lds_conflict_model.py's lane-group model for 13-wide frames: XOR-swizzled
// 128-B rows 3.9 extra) = 12.5k LDS cycles against 12.7k cycles of MFMA issue per SIMD pair --
// the LDS array, not the MFMA, sets its pace (it ran at 43-46 % of the fp16 peak).  Here:
//   * each wave owns 96 x 64 outputs (NJ = 4 column blocks: 4 MFMAs per fragment, half the
//     reads); the 8 waves are 4 column groups x 2 row groups of 6 / 5 row blocks, and the two
//     waves of a column group share a SIMD (workgroup wave w and w + 4), so every SIMD runs 11
//     blocks.  The price: both row groups load the same weights (L2 hits for the second);
//   * the patch of a 64-channel chunk is LDS-DMA'd (`buffer_load ... lds`) into the other half of
//     a double buffer during the current chunk, rows padded to LP = 160 B (3.7 extra cycles per
//     read, VALU-free; 128-B rows: 12), one barrier per chunk, no staging registers;
//   * the next tap's 8 weight fragments go straight to registers, spread over the tap's first
//     row blocks.
// Summation order per output: chunk, tap, then the two 32-channel groups of the tap, each one
// v_mfma_f32_16x16x32_f16 -- the same as conv3x3_f16_patch_kernel<176, ..., 16> (same bits).
#pragma once
#include "gemm_f16_patch.h"
#include "gemm_x3_acc2.h"

namespace dnnhip {

template <int NPR, int LP = 160>
__global__ void __launch_bounds__(512, 1)
conv3x3_f16_lds_kernel(const half_t* __restrict__ in, const half_t* __restrict__ Bt, int ldb, half_t* __restrict__ out,
                       int M, int N, int K, EpiParams epi, int tilesM, Patch16Geom g, unsigned in_bytes,
                       unsigned b_bytes) {
  constexpr int BM = 176, TM = BM / 16, BN = 256, NJ = 4, NW = 8, RB = 128, RG = 2, TMW = (TM + RG - 1) / RG;
  constexpr int NQW = (NPR * LP + NW * 1024 - 1) / (NW * 1024);  // 1-KiB DMA pieces per wave per patch
  constexpr int BUFB = NQW * NW * 1024;
  static_assert(LP % 16 == 0 && LP >= RB && NQW <= 9, "shape");
  constexpr int LPB = (2 * NJ + TMW - 1) / TMW;  // next-tap weight loads per row block
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUFB];

  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int cg = wid & 3, rg = wid >> 2;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int tn = tile / tilesM, tm = tile - tn * tilesM;
  const int m0 = tm * BM, n0 = tn * BN + cg * 64;  // this wave's 64 columns
  const int Wp = g.W + 2, HWo = g.H * g.W;
  auto padded = [&](int m) {
    const int b = m / HWo, r = m - b * HWo, oy = r / g.W, ox = r - oy * g.W;
    return (b * (g.H + 2) + oy + 1) * Wp + ox + 1;
  };
  const int P0 = padded(m0) - (Wp + 1);
  const int mlast = (m0 + BM < M ? m0 + BM : M) - 1;

  const int fr = lane & 15, fq = lane >> 4;
  int prow[TMW];
#pragma unroll
  for (int i = 0; i < TMW; ++i) {
    int m = m0 + 16 * (rg * TMW + i) + fr;
    m = m < mlast ? m : mlast;
    prow[i] = (padded(m) - P0 - (Wp + 1)) * LP + 16 * fq;
  }

  const int nch = K / 64 / 9;
  const int rowB = 2 * g.C;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  const unsigned dsoff = (unsigned)(P0 * rowB);
  auto issue_patch = [&](int chunk, int k, int buf) {
    const unsigned b = 1024u * (unsigned)(wid + NW * k) + 16u * (unsigned)lane;
    const unsigned r = b / LP, u = (b - r * LP) >> 4;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rsA, (__attribute__((address_space(3))) void*)(smem + buf * BUFB + 1024 * (wid + NW * k)), 16,
        (int)(__umul24(r, (unsigned)rowB) + 16 * u), (int)(dsoff + chunk * RB), 0, 0);
  };

  // weights [n/16][k/32][lane][8] (launch_pack_weights order 4, K order (chunk, tap, channel)):
  // column block jb at + jb * ldb * 32 bytes, group kq = 2 (9 chunk + tap) + q at + kq * 1 KiB
  const unsigned bvo = (unsigned)((n0 / 16) * ldb * 32 + lane * 16);
  const int bjs = ldb * 32;
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)b_bytes, 0x00020000);
  f16x8 bq[2][2][NJ];
  auto load_b1 = [&](int s, int q, int jb, f16x8& dst) {
    dst = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, bvo, (2 * s + q) * 1024 + jb * bjs, 0));
  };

  f32x4 acc[TMW][NJ];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb) load_b1(0, q, jb, bq[0][q][jb]);
#pragma unroll
  for (int k = 0; k < NQW; ++k) issue_patch(0, k, 0);
  vm_wait<0>();
  __syncthreads();

  const bool tail = TMW * RG > TM && rg == RG - 1;  // the last row group's surplus block
  const int nsteps = 9 * nch;
  const unsigned char* P = smem;
  int t = 0, j = 0;
  for (int s = 0; s < nsteps; ++s) {
    const int toff = (t / 3) * Wp + (t % 3);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TMW; ++i) {
#pragma unroll
      for (int l = i * LPB; l < (i + 1) * LPB && l < 2 * NJ; ++l) load_b1(s + 1, l / NJ, l % NJ, bq[1][l / NJ][l % NJ]);
      if (i == TMW - 2) issue_patch(j + 1, t < NQW ? t : NQW - 1, (j + 1) & 1);  // (uniform count per tap)
      if (i == TMW - 1 && tail) continue;
      const unsigned char* qa = P + prow[i] + toff * LP;
      const f16x8 a0 = *reinterpret_cast<const f16x8*>(qa);
      const f16x8 a1 = *reinterpret_cast<const f16x8*>(qa + 64);
#pragma unroll
      for (int jb = 0; jb < NJ; ++jb) acc[i][jb] = mfma16_f16(a0, bq[0][0][jb], acc[i][jb]);
#pragma unroll
      for (int jb = 0; jb < NJ; ++jb) acc[i][jb] = mfma16_f16(a1, bq[0][1][jb], acc[i][jb]);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int jb = 0; jb < NJ; ++jb) bq[0][q][jb] = bq[1][q][jb];
    if (++t == 9) {
      t = 0;
      ++j;
      vm_wait<0>();
      wait_lgkm0();
      raw_barrier();
      P = smem + (j & 1) * BUFB;
    }
  }
  vm_wait<0>();

  // epilogue: bias/BN/leaky, fp16 out (plain [M][N] or zero-bordered padded rows)
  int* orow = reinterpret_cast<int*>(smem);
  __syncthreads();
  if (threadIdx.x < BM) {
    const int m = m0 + threadIdx.x;
    orow[threadIdx.x] = m >= M ? -1 : (g.out_padded ? padded(m) : m);
  }
  __syncthreads();
  static_for<0, NJ>([&](auto jbc) {
    constexpr int jb = decltype(jbc)::value;
    const int n = n0 + 16 * jb + fr;
    const float pb = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
    const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
    const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
    const float pg = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;
    static_for<0, TMW>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if (i == TMW - 1 && tail) return;
      static_for<0, 4>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        const int o = orow[16 * (rg * TMW + i) + 4 * fq + r];
        if (o >= 0) store_out(out + (size_t)o * N + n, apply_epilogue(acc[i][jb][r], pb, pm, ps, pg, epi.flags));
      });
    });
  });
}

}  // namespace dnnhip
