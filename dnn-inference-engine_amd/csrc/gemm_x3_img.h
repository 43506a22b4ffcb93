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
// rows, 12 data units + 2 never read; image rows skewed by 4 units) LDS-DMA'd into the other half of a double buffer while the
// current chunk runs; a tap is an immediate offset.  8 waves of all 11 row blocks x 16 columns
// (each weight fragment serves the whole image: 3 weight loads per 66 MFMAs, the wide kernel's
// density; 4 column groups x 2 row halves of 32 columns measured 78 % MFMA-busy in the loop with
// twice the loads, and the 5-block half waited for the 6-block one).  Per output the chunk-major,
// tap-minor x3 steps of the other x3 kernels (x3_step, two
// accumulators folded once) over the whole K; the order depends on (N, K) only, so batch rows are
// bit-identical to one-frame runs of the same plan kind.
// Epilogue: the folded sums into an LDS stage [H W][128 + 4], then per (pixel, 8 columns): the
// window max (min for a decreasing channel, pool_then_epilogue), the epilogue with one
// wave-uniform division check, the exact split and three 16-B stores of the next layer's planes
// (or two fp32 16-B stores when the layer is the plan's last).
#pragma once
#include "gemm_x3_acc2.h"

namespace dnnhip {

#if (X3DIAG & 16384) != 0  // phase stamps (results unchanged), wave 0 and wave 7:
// [workgroup][0 s_memrealtime start, 1 s_memtime start, 2 prologue done, 3 loop done (wave 0),
// 4 loop done (wave 7), 5 raw sums staged, 6 end, 7 s_memrealtime end]
constexpr int IMG_DIAG_WGS = 512;
__device__ unsigned long long img_diag_stamps[IMG_DIAG_WGS * 8];
#define IMG_STAMP(k, v) \
  if (threadIdx.x == 0 && blockIdx.x < IMG_DIAG_WGS) img_diag_stamps[blockIdx.x * 8 + (k)] = (v);
#else
#define IMG_STAMP(k, v)
#endif

template <int H, int W, int FL = -1>
__global__ void __launch_bounds__(512, 1)
conv3x3_x3_img_kernel(const bf16_bits* __restrict__ in, const bf16_bits* __restrict__ Bt, float* __restrict__ out,
                      bf16_bits* __restrict__ out_split, int N, int K, EpiParams epi, int C, unsigned in_bytes,
                      unsigned b_bytes) {
  constexpr int NW = 8, LP = 224, PU = LP / 16, WP = W + 2, PR = (H + 2) * WP, HW = H * W, TM = (HW + 15) / 16, SR = 132;
  // LDS: padded image row y at unit RU y, pixel x of it at + PU x (the SK units after an image
  // row's pixels are never read): tools/lds_conflict_model.py, 13-wide images, 16 consecutive
  // output pixels per fragment: 5.09 extra cycles per ds_read_b128 without the skew, 1.45 with
  // SK = 4 -- at 16 columns per wave (one A fragment per 6 MFMAs) the unskewed reads held the
  // loop LDS-bound (80 % MFMA-busy)
  constexpr int SK = 4, RU = PU * WP + SK;
  constexpr int NPC = ((H + 2) * RU + 63) / 64, NPW = (NPC + NW - 1) / NW, BUFB = NPW * NW * 1024;
  static_assert(HW <= 176 && HW > 80 && 2 * BUFB >= HW * SR * 4 && 2 * BUFB <= 150 * 1024, "shape");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUFB];
  __shared__ f32x4 epl[128];

  const int lane = threadIdx.x & 63;
  const int eflags = FL < 0 ? epi.flags : FL;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int nblk = N / 128;
  const int t = xcd_tile(blockIdx.x, gridDim.x);
  const int b = t / nblk, nb = t - b * nblk;
  const int n0 = nb * 128 + wid * 16;  // this wave's 16 columns
  const int fr = lane & 15, fq = lane >> 4;
  IMG_STAMP(0, __builtin_amdgcn_s_memrealtime())
  IMG_STAMP(1, __builtin_amdgcn_s_memtime())

  int rowoff[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int r = 16 * i + fr;
    r = r < HW ? r : HW - 1;
    rowoff[i] = ((r / W) * RU + (r % W) * PU) * 16 + 16 * fq;
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
      unsigned y = U / RU;
      const unsigned rem = U - y * RU;
      unsigned x = rem / PU, u = rem - x * PU;
      if (x >= (unsigned)WP) x = WP - 1, u = PU - 1;  // (skew units: a harmless in-image source)
      y = y < (unsigned)(H + 2) ? y : H + 1;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsA, (__attribute__((address_space(3))) void*)(smem + buf * BUFB + 1024 * (wid + NW * k)), 16,
          (int)((pbase + y * WP + x) * rowB + 16u * u), (int)(c * 192), 0, 0);
    }
  };

  const unsigned bvo = (unsigned)((n0 / 16) * nk * 3072 + lane * 16);
  const int bjs = nk * 3072;
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)b_bytes, 0x00020000);
  (void)bjs;
  bf16x8 bq[3][3][1];
  auto load_b = [&](int s, bf16x8 (&dst)[3][1]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
      dst[p][0] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, bvo, s * 3072 + p * 1024, 0));
  };

  if (threadIdx.x < 128) {
    const X3EpiCol c = x3_epi_col(epi, eflags, nb * 128 + threadIdx.x);
    epl[threadIdx.x] = f32x4{c.pb, c.pm, c.ps, c.pg};
  }
  f32x4 acc[TM][1], accc[TM][1];
#pragma unroll
  for (int i = 0; i < TM; ++i) acc[i][0] = accc[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_chunk(0, 0);
  load_b(0, bq[0]);
  load_b(1, bq[1]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  IMG_STAMP(2, __builtin_amdgcn_s_memtime())

  auto frag = [&](const unsigned char* P, int i, int tap, bf16x8 (&a)[3]) {
    const int toff = ((tap / 3) * RU + (tap % 3) * PU) * 16;
    const unsigned char* q = P + rowoff[i] + toff;
#pragma unroll
    for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(q + 64 * p);
  };
  // fragments read LEAD = 2 row blocks ahead through a ring of 3 sets (one block is 6 MFMAs, 96
  // cycles: a one-block lead left the LDS latency exposed); 9 TM % 3 == 0, so every chunk starts
  // at slot 0
  constexpr int LEAD = 2, RING = 3, NBC = 9 * TM;
  static_assert(NBC % RING == 0, "fragment ring phase per chunk");
  auto blk = [&](const unsigned char* P, int bi, bf16x8 (&a)[3]) { frag(P, bi % TM, bi / TM, a); };
  for (int j = 0; j < nch; ++j) {
    const unsigned char* P = smem + (j & 1) * BUFB;
    if (j + 1 < nch) issue_chunk(j + 1, (j + 1) & 1);  // the other buffer: read in chunk j - 1
    bf16x8 af[RING][3];
#pragma unroll
    for (int l = 0; l < LEAD; ++l) blk(P, l, af[l]);
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int s = 9 * j + tp;
      __builtin_amdgcn_sched_barrier(0);
      load_b(s + 2, bq[(tp + 2) % 3]);  // (past the last step: unused, in-range or zero-filled)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int bi = TM * tp + i;
        if (bi + LEAD < NBC) blk(P, bi + LEAD, af[(bi + LEAD) % RING]);
        x3_step<true>(acc[i][0], accc[i][0], af[bi % RING], bq[tp % 3], 0);
        __builtin_amdgcn_sched_barrier(0);
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
  IMG_STAMP(3, __builtin_amdgcn_s_memtime())
#if (X3DIAG & 16384) != 0
  if (threadIdx.x == 448 && blockIdx.x < IMG_DIAG_WGS) img_diag_stamps[blockIdx.x * 8 + 4] = __builtin_amdgcn_s_memtime();
#endif
  x3_fold(acc, accc);
  wait_lgkm0();
  __syncthreads();  // every wave is done with the patch buffers: the stage reuses them

  // the image's raw sums, [pixel][128 columns (+ 4)]
  float* const stg = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * i + 4 * fq + r;
      if (row < HW) stg[row * SR + wid * 16 + fr] = acc[i][0][r];
    }
  }
  __syncthreads();
  IMG_STAMP(5, __builtin_amdgcn_s_memtime())

  // pool (2x2 / s1 SAME: cells past the frame's right or bottom edge repeat the pixel) + epilogue
  // + split, one (pixel, 8 columns) task per thread and pass: three 16-B piece stores
  // (a thread's 8 columns are the same in every pass: task steps by a multiple of 16)
  const int c8 = 8 * (threadIdx.x & 15);
  float cb[8], cm[8], cs[8], cgm[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const f32x4 ep = epl[c8 + e];
    cb[e] = ep[0], cm[e] = ep[1], cs[e] = ep[2], cgm[e] = ep[3];
  }
#pragma unroll 2
  for (int task = threadIdx.x; task < HW * 16; task += NW * 64) {
    const int pix = task >> 4;
    const int y = pix / W, x = pix - y * W;
    const int px1 = x + 1 < W ? pix + 1 : pix, py1 = y + 1 < H ? pix + W : pix, pxy = y + 1 < H ? px1 + W : px1;
    f32x4 win[1][8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 va = *reinterpret_cast<const f32x4*>(stg + pix * SR + c8 + 4 * h);
      const f32x4 vb = *reinterpret_cast<const f32x4*>(stg + px1 * SR + c8 + 4 * h);
      const f32x4 vc = *reinterpret_cast<const f32x4*>(stg + py1 * SR + c8 + 4 * h);
      const f32x4 vd = *reinterpret_cast<const f32x4*>(stg + pxy * SR + c8 + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) win[0][4 * h + e] = f32x4{va[e], vb[e], vc[e], vd[e]};
    }
    float o[8];
    pool_epilogue_batch<FL>(win, cb, cm, cs, cgm, epi.flags, [&](int, int c, float e) { o[c] = e; });
    const int n = nb * 128 + c8;
    if (out_split == nullptr) {  // fp32 [B][H][W][N] (the plan's last layer)
      const size_t d = ((size_t)b * HW + pix) * N + n;  // (floats)
      store16_at(out, 4 * d, __builtin_bit_cast(u32x4, f32x4{o[0], o[1], o[2], o[3]}));
      store16_at(out, 4 * d + 16, __builtin_bit_cast(u32x4, f32x4{o[4], o[5], o[6], o[7]}));
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
    const size_t d = ((size_t)b * PR + (y + 1) * WP + x + 1) * (3 * (size_t)N) + (n >> 5) * 96 + (n & 31);
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) store16_at(out_split, 2 * (d + 32 * pc), q[pc]);
  }
  IMG_STAMP(6, __builtin_amdgcn_s_memtime())
  IMG_STAMP(7, __builtin_amdgcn_s_memrealtime())
}
#undef IMG_STAMP

}  // namespace dnnhip
