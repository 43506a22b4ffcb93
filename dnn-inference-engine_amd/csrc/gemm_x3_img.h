// fp32 3x3 conv on the x3 arithmetic (gemm_x3_patch.h) for small frames, one whole image per
// workgroup, with the 2x2 / stride-1 SAME max pool that follows it fused (YOLOv2-tiny conv5 +
// pool5 in batch plans), device code only.  Round 5.
//
// Why: the wide kernel (gemm_x3_acc2.h) runs conv5 (13x13x256 -> 512, K = 2304) as 62 x 2 tiles
// of 176 x 256 in 2 K slices to fill the chip; each slice writes 180 KB of raw fp32 partials per
// workgroup (phase stamps, X3DIAG 8192: ~26 k cycles of its ~206 k) and pool5 then reads both
// slices back to sum, pool and split them (~23 us).  Here a workgroup owns one image (H W <= 176
// rows: 11 16-row blocks) and 128 output columns over the whole K: B x N / 128 = 256 workgroups at
// batch 64, no partials, and pool5 runs on the image's raw sums from LDS before the epilogue.
//
// Layout: the image's zero-bordered (H + 2) x (W + 2) pixel rows of a 32-channel chunk (224-B LDS
// rows, 12 data units + 2 never read) LDS-DMA'd into the other half of a double buffer while the
// current chunk runs; a tap is an immediate offset.  8 waves: 4 column groups of 32 x 2 row
// halves (blocks 0-5 and 6-10), so each SIMD runs 11 blocks per step (its two waves: one of each
// half).  Per output the chunk-major, tap-minor x3 steps of the other x3 kernels (x3_step, two
// accumulators folded once) over the whole K; the order depends on (N, K) only, so batch rows are
// bit-identical to one-frame runs of the same plan kind.
// Epilogue: the folded sums into an LDS stage [H W][128 + 4], then per (pixel, 8 columns): the
// window max (min for a decreasing channel, pool_then_epilogue), the epilogue with one
// wave-uniform division check, the exact split and three 16-B stores of the next layer's planes
// (or two fp32 16-B stores when the layer is the plan's last).
#pragma once
#include "gemm_x3_acc2.h"

namespace dnnhip {

template <int H, int W, int FL = -1>
__global__ void __launch_bounds__(512, 1)
conv3x3_x3_img_kernel(const bf16_bits* __restrict__ in, const bf16_bits* __restrict__ Bt, float* __restrict__ out,
                      bf16_bits* __restrict__ out_split, int N, int K, EpiParams epi, int C, unsigned in_bytes,
                      unsigned b_bytes) {
  constexpr int NW = 8, LP = 224, PU = LP / 16, WP = W + 2, PR = (H + 2) * WP, HW = H * W, TM = 6, SR = 132;
  constexpr int NPC = (PR * PU + 63) / 64, NPW = (NPC + NW - 1) / NW, BUFB = NPW * NW * 1024;
  static_assert(HW <= 176 && HW > 80 && 2 * BUFB >= HW * SR * 4 && 2 * BUFB <= 150 * 1024, "shape");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUFB];
  __shared__ f32x4 epl[128];

  const int lane = threadIdx.x & 63;
  const int eflags = FL < 0 ? epi.flags : FL;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int cg = wid & 3, rh = wid >> 2;
  const int nbw = rh == 0 ? TM : (HW - 96 + 15) / 16;  // this wave's row blocks (6, then the rest)
  const int nblk = N / 128;
  const int t = xcd_tile(blockIdx.x, gridDim.x);
  const int b = t / nblk, nb = t - b * nblk;
  const int n0 = nb * 128 + cg * 32;
  const int fr = lane & 15, fq = lane >> 4;

  int rowoff[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int r = rh * 96 + 16 * i + fr;
    r = r < HW ? r : HW - 1;
    rowoff[i] = ((r / W) * WP + r % W) * LP + 16 * fq;
  }

  const int nk = K / 32, nch = nk / 9;
  const unsigned rowB = 6u * (unsigned)C;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  const unsigned pbase = (unsigned)(b * PR);  // padded pixel (0, 0) of the image
  auto issue_chunk = [&](int c, int buf) {
#pragma unroll
    for (int k = 0; k < NPW; ++k) {
      if (wid + NW * k >= NPC) break;  // (wave-uniform)
      const unsigned U = 64u * (unsigned)(wid + NW * k) + (unsigned)lane;
      unsigned r = U / PU;
      const unsigned u = U - r * PU;
      r = r < (unsigned)PR ? r : (unsigned)PR - 1;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsA, (__attribute__((address_space(3))) void*)(smem + buf * BUFB + 1024 * (wid + NW * k)), 16,
          (int)((pbase + r) * rowB + 16u * u), (int)(c * 192), 0, 0);
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

  if (threadIdx.x < 128) {
    const X3EpiCol c = x3_epi_col(epi, eflags, nb * 128 + threadIdx.x);
    epl[threadIdx.x] = f32x4{c.pb, c.pm, c.ps, c.pg};
  }
  f32x4 acc[TM][2], accc[TM][2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = accc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_chunk(0, 0);
  load_b(0, bq[0]);
  load_b(1, bq[1]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  auto frag = [&](const unsigned char* P, int i, int tap, bf16x8 (&a)[3]) {
    const int toff = ((tap / 3) * WP + (tap % 3)) * LP;
    const unsigned char* q = P + rowoff[i] + toff;
#pragma unroll
    for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(q + 64 * p);
  };
  for (int j = 0; j < nch; ++j) {
    const unsigned char* P = smem + (j & 1) * BUFB;
    if (j + 1 < nch) issue_chunk(j + 1, (j + 1) & 1);  // the other buffer: read in chunk j - 1
    bf16x8 af[2][3];
    frag(P, 0, 0, af[0]);
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int s = 9 * j + tp;
      __builtin_amdgcn_sched_barrier(0);
      load_b(s + 2, bq[(tp + 2) % 3]);  // (past the last step: unused, in-range or zero-filled)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (i < nbw) {  // (wave-uniform: the second half has one block fewer)
          const int cur = i & 1, nxt = cur ^ 1;
          if (i + 1 < nbw)
            frag(P, i + 1, tp, af[nxt]);
          else if (tp < 8)
            frag(P, 0, tp + 1, af[nxt]);
          const bf16x8(&bb)[3][2] = bq[tp % 3];
#pragma unroll
          for (int jb = 0; jb < 2; ++jb) x3_step<true>(acc[i][jb], accc[i][jb], af[cur], bb, jb);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (tp < 8 && (nbw & 1)) {  // (an odd block count read the next tap's first block into slot 1)
#pragma unroll
        for (int p = 0; p < 3; ++p) af[0][p] = af[1][p];
      }
    }
    // the ring holds steps s + 1, s + 2 in slots (tp + 1) % 3 = 0 and 1 for the next chunk (9 % 3 == 0)
    if (j + 1 < nch) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      wait_lgkm0();
      __syncthreads();  // chunk j + 1 landed (every wave's pieces); chunk j read by every wave
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  x3_fold(acc, accc);
  wait_lgkm0();
  __syncthreads();  // every wave is done with the patch buffers: the stage reuses them

  // the image's raw sums, [pixel][128 columns (+ 4)]
  float* const stg = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    if (i < nbw) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rh * 96 + 16 * i + 4 * fq + r;
        if (row < HW) {
#pragma unroll
          for (int jb = 0; jb < 2; ++jb) stg[row * SR + cg * 32 + 16 * jb + fr] = acc[i][jb][r];
        }
      }
    }
  }
  __syncthreads();

  // pool (2x2 / s1 SAME: cells past the frame's right or bottom edge repeat the pixel) + epilogue
  // + split, one (pixel, 8 columns) task per thread and pass: three 16-B piece stores
  for (int task = threadIdx.x; task < HW * 16; task += NW * 64) {
    const int pix = task >> 4, c8 = 8 * (task & 15);
    const int y = pix / W, x = pix - y * W;
    const int px1 = x + 1 < W ? pix + 1 : pix, py1 = y + 1 < H ? pix + W : pix, pxy = y + 1 < H ? px1 + W : px1;
    f32x4 win[1][8];
    float cb[8], cm[8], cs[8], cgm[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 va = *reinterpret_cast<const f32x4*>(stg + pix * SR + c8 + 4 * h);
      const f32x4 vb = *reinterpret_cast<const f32x4*>(stg + px1 * SR + c8 + 4 * h);
      const f32x4 vc = *reinterpret_cast<const f32x4*>(stg + py1 * SR + c8 + 4 * h);
      const f32x4 vd = *reinterpret_cast<const f32x4*>(stg + pxy * SR + c8 + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        win[0][4 * h + e] = f32x4{va[e], vb[e], vc[e], vd[e]};
        const f32x4 ep = epl[c8 + 4 * h + e];
        cb[4 * h + e] = ep[0], cm[4 * h + e] = ep[1], cs[4 * h + e] = ep[2], cgm[4 * h + e] = ep[3];
      }
    }
    float o[8];
    pool_epilogue_batch<FL>(win, cb, cm, cs, cgm, epi.flags, [&](int, int c, float e) { o[c] = e; });
    const int n = nb * 128 + c8;
    if (out_split == nullptr) {  // fp32 [B][H][W][N] (the plan's last layer)
      float* d = out + ((size_t)b * HW + pix) * N + n;
      *reinterpret_cast<f32x4*>(d) = f32x4{o[0], o[1], o[2], o[3]};
      *reinterpret_cast<f32x4*>(d + 4) = f32x4{o[4], o[5], o[6], o[7]};
      continue;
    }
    bool ok = true;
#pragma unroll
    for (int e = 0; e < 8; ++e) ok = ok && x3_split_ok(o[e]);
    const bool fast = __builtin_amdgcn_ballot_w64(!ok) == 0;
    u32x4 q[3];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      unsigned w0, w1, w2;
      split3_pack2(fast, o[2 * e], o[2 * e + 1], w0, w1, w2);
      q[0][e] = w0;
      q[1][e] = w1;
      q[2][e] = w2;
    }
    bf16_bits* d = out_split + ((size_t)b * PR + (y + 1) * WP + x + 1) * (3 * (size_t)N) + (n >> 5) * 96 + (n & 31);
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) *reinterpret_cast<u32x4*>(d + 32 * pc) = q[pc];
  }
}

}  // namespace dnnhip
