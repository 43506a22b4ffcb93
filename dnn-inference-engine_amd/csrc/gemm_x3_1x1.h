// fp32 1x1 conv on the bf16 MFMA with exact three-way operand splits (the x3 arithmetic of
// gemm_x3_patch.h / gemm_x3_acc2.h): YOLOv2-tiny conv8 (13x13x1024 -> 125), the reference's
// im2col-free sgemm of a 1x1 kernel (dnn_openblas.c:184-192 with K = C).  Device code only.
//
// A is the producer's zero-bordered split planes (conv7's epilogue, row padded(m) of
// [B][H+2][W+2], 32-channel chunk c at bytes 192 c: 32 bf16 of each piece), B the packed weights
// [n/16][step = chunk][piece][lane][8] (pack_weights_x3_kernel with one tap).  A workgroup owns 16
// TMW rows x 128 columns; its 4 waves take 32 columns each (TMW x 2 blocks of 16 x 16).  Per 32-channel
// step: the tile's 32 A rows (224-B LDS rows, as the wide kernel: the two 8-lane halves of each
// ds_read_b128 lane group fall on even / odd bank quads) arrive by LDS-DMA into a ring of NS
// slots, issued NS - 1 steps ahead; each wave's 6 B fragments come from L2 two steps ahead into a
// register ring of 3; one barrier per step.  Two accumulators per output over all of K (accm:
// a0 b0; accc: a2b0, a1b1, a1b0, a0b2, a0b1 -- gemm_x3_acc2.h's PF order), then accm + accc and
// the fp32 epilogue into out [M][N].  The summation order depends on K only (batch rows are
// bit-identical to batch-1 runs).
#pragma once
#include "gemm_x3_patch.h"
#include "gemm_x3_acc2.h"  // static_for

namespace dnnhip {

constexpr int X3_1X1_BN = 128, X3_1X1_LP = 224, X3_1X1_NS = 6;

// TMW: 16-row blocks per wave (the tile has 16 TMW rows)
template <int FL, int TMW>
__global__ void __launch_bounds__(256, 2)
conv1x1_x3_kernel(const bf16_bits* __restrict__ in, const bf16_bits* __restrict__ Bt, float* __restrict__ out, int M,
                  int N, int K, EpiParams epi, int tilesM, X3Geom g, unsigned in_bytes, unsigned b_bytes) {
  constexpr int BM = 16 * TMW, LP = X3_1X1_LP, NS = X3_1X1_NS, RB = 192;
  constexpr int NPC = (BM * LP + 1023) / 1024;  // one-KiB DMA pieces per step (7 for 32 rows)
  constexpr int SLOT = NPC * 1024;              // a step's LDS slot: whole pieces (>= BM LP)
  constexpr int PPW = (NPC + 3) / 4;          // pieces per wave per step
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NS * SLOT];

  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int tn = tile / tilesM, tm = tile - tn * tilesM;
  const int m0 = tm * BM, n0 = tn * X3_1X1_BN + wid * 32;
  const int nk = K / 32;
  const int Wp = g.W + 2, HWo = g.H * g.W;
  auto padded = [&](int m) {
    m = m < M ? m : M - 1;
    const int b = m / HWo, r = m - b * HWo, oy = r / g.W, ox = r - oy * g.W;
    return (b * (g.H + 2) + oy + 1) * Wp + ox + 1;
  };

  // A pieces: wave w issues pieces w, w + 4, ... (pieces past NPC repeat piece w: same bytes to
  // the same LDS address), so every wave issues exactly PPW DMAs per step and the counted waits hold.
  // Piece k, lane l: LDS byte 1024 k + 16 l of the slot = row r, unit u; units past the 12 data
  // units of a row read the next global bytes (the descriptor returns zeros past the buffer):
  // padding that is never read back
  const int rowB = 6 * g.C;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  unsigned avo[PPW];
  int apc[PPW];
#pragma unroll
  for (int h = 0; h < PPW; ++h) {
    const int k = wid + 4 * h < NPC ? wid + 4 * h : wid;
    apc[h] = k;
    const unsigned b = 1024u * (unsigned)k + 16u * (unsigned)lane;
    const unsigned r = b / LP, u = (b - r * LP) >> 4;
    avo[h] = (unsigned)padded(m0 + (int)(r < (unsigned)BM ? r : BM - 1)) * (unsigned)rowB + 16u * u;
  }
  auto issue_a = [&](int step, int sl) {  // sl = step % NS
    const int st = step < nk ? step : nk - 1;  // (past the end: a valid chunk into a slot never read)
    unsigned char* slot = smem + sl * SLOT;
#pragma unroll
    for (int h = 0; h < PPW; ++h)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(slot + 1024 * apc[h]),
                                               16, (int)avo[h], st * RB, 0, 0);
  };

  // B fragments: the wave's two 16-column blocks, steps ahead in a register ring of 3
  const unsigned bvo = (unsigned)((n0 / 16) * nk * 3072 + lane * 16);
  const int bjs = nk * 3072;
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)b_bytes, 0x00020000);
  bf16x8 bq[3][3][2];
  auto load_b = [&](int step, bf16x8 (&dst)[3][2]) {
    const int st = step < nk ? step : nk - 1;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        dst[p][j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, bvo, st * 3072 + p * 1024 + j * bjs, 0));
  };

  f32x4 accm[TMW][2], accc[TMW][2];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) accm[i][j] = accc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue in the steady state's issue order: A(0..2), B(0), A(3), B(1), A(4); step s then
  // waits for B(s) and everything older (A(s) included): the ops issued after B(s) are A(s + 3)
  // (PPW) and step s - 1's B(s + 1) (6) and A(s + 4) (PPW)
  static_assert(NS == 6, "vmcnt accounting below");
  issue_a(0, 0);
  issue_a(1, 1);
  issue_a(2, 2);
  load_b(0, bq[0]);
  issue_a(3, 3);
  load_b(1, bq[1]);
  issue_a(4, 4);
  const int fr = lane & 15, fq = lane >> 4;
  // six steps per iteration, so that the register ring and the LDS slot of a step are static
  for (int s0 = 0; s0 < nk; s0 += NS) {
    static_for<0, NS>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      const int s = s0 + u;
      if (s >= nk) return;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 + 2 * PPW) : "memory");
      __builtin_amdgcn_s_barrier();  // every wave's pieces of A(s) landed; step s - 1's reads done
      load_b(s + 2, bq[(u + 2) % 3]);
      issue_a(s + 5, (u + 5) % NS);  // into the slot step s - 1 read
      const unsigned char* P = smem + u * SLOT;
      bf16x8 a[TMW][3];
#pragma unroll
      for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          a[i][p] = *reinterpret_cast<const bf16x8*>(P + (16 * i + fr) * LP + 64 * p + 16 * fq);
      const bf16x8(&b)[3][2] = bq[u % 3];
#pragma unroll
      for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
          f32x4 c = accc[i][jb];
          c = mfma16_bf16(a[i][2], b[0][jb], c);
          c = mfma16_bf16(a[i][1], b[1][jb], c);
          c = mfma16_bf16(a[i][1], b[0][jb], c);
          c = mfma16_bf16(a[i][0], b[2][jb], c);
          c = mfma16_bf16(a[i][0], b[1][jb], c);
          accc[i][jb] = c;
          accm[i][jb] = mfma16_bf16(a[i][0], b[0][jb], accm[i][jb]);
        }
    });
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup exits

#pragma unroll
  for (int jb = 0; jb < 2; ++jb) {
    const int f = FL < 0 ? epi.flags : FL;
    const int n = n0 + 16 * jb + fr;
    if (n >= N) continue;
    const float pb = (f & EPI_BIAS) ? epi.bias[n] : 0.f;
    const float pm = (f & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
    const float ps = (f & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
    const float pg = (f & EPI_BN) ? epi.gamma[n] : 1.f;
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 16 * i + 4 * fq + r;
        if (m < M)
          out[(size_t)m * N + n] = apply_epilogue_t<FL>(accm[i][jb][r] + accc[i][jb][r], pb, pm, ps, pg, epi.flags);
      }
  }
}

}  // namespace dnnhip
