// fp16 3x3 conv for the long-K, wide-N layers of the fp16 path (conv6/conv7 of YOLOv2-tiny,
// BASELINE config 5) on the fp32 path's wide x3 kernel structure (gemm_x3_acc2.h), device code
// only.  Round 4: replaces conv3x3_f16_patch_kernel (register-staged 128-B rows with an XOR
// swizzle, weights two taps ahead, one scalar fp16 store per output), which held the fp16 MFMA
// at 45 % of its peak where the x3 kernel holds the same v_mfma 16x16x32 issue at 62-65 %:
//   * the patch of one 64-channel chunk (<= NPR zero-bordered input rows) is LDS-DMA'd
//     (buffer_load ... lds, 1-KiB pieces) into the other half of a double buffer while the
//     current chunk runs: no staging registers, one barrier per chunk;
//   * LDS rows of LP = 160 bytes (the 128 data bytes + 32 never-read ones), skewed by 12 units per
//     image row (below): 0.36 extra conflict cycles per fragment read (plain 160-B rows: 3.95,
//     the old kernel's swizzle ~4) -- at 2 reads per 4 MFMAs the fp16 loop is LDS-bound
//     (~2 x 7.7 LDS cycles per 16 at full MFMA rate with the conflicts);
//   * the tap's vector-memory instructions (4 weight fragments, 1 DMA piece) spread one per row
//     block over its first blocks; the A fragments read two row blocks ahead (a ring of three);
//   * the epilogue staged through a wave-private LDS tile: one 16-B fp16 store per lane and row
//     block instead of one 2-B store per output.
// Same products in the same order as the round-3 kernel (per output: chunk, tap, 32-channel group;
// v_mfma_f32_16x16x32_f16), same weight packing (order 4: [n/16][k/32][lane][8]), same epilogue
// arithmetic: same bits (checked against it on the GPU before it was removed).  Measured at batch
// 64 (same process, interleaved): conv7 0.175 -> 0.151 ms, conv6 0.098 -> 0.083 ms; the skew
// alone -0.4 %, the two-block fragment lead -9 % (one block: conv7 0.166).
//
// The input sits in HBM zero-padded ([B][H+2][W+2][C], borders written once at plan finalize), so
// output pixel m's tap (dy, dx) is padded row p(m) + (dy-1)(W+2) + (dx-1): a tile of BM consecutive
// output pixels reads one contiguous run of padded rows per 64-channel chunk, staged once and
// reused by all 9 taps.
#pragma once
#include <type_traits>
#include "gemm_f16.h"
#include "gemm_x3_acc2.h"

namespace dnnhip {

struct Patch16Geom {
  int H, W, C;      // conv input = output spatial size (3x3, stride 1, SAME), channels
  int out_padded;   // 1: write the output into a zero-bordered [B][H+2][W+2][N] buffer
};

// v_mfma_f32_16x16x32_f16: lane l supplies A[row l&15][k 8(l>>4)..+7] and B likewise;
// D[row][col]: col = l&15, row = 4(l>>4) + reg.  (The same FLOP per cycle as 32x32x16; on
// random data the chip holds a higher clock for it, MI355X_MICROARCH DVFS item 7.)
__device__ __forceinline__ f32x4 mfma16_f16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

template <int BM, int NPR, int FL = -1>
__global__ void __launch_bounds__(512, 2)
conv3x3_f16_acc_kernel(const half_t* __restrict__ in, const half_t* __restrict__ Bt, int ldb, half_t* __restrict__ out,
                       int M, int N, int K, EpiParams epi, int tilesM, Patch16Geom g, unsigned in_bytes,
                       unsigned b_bytes) {
  constexpr int BN = 256, TM = BM / 16, RB = 128, NJ = 2, NW = 8, LP = 160;
  constexpr int NQW = (NPR * LP + NW * 1024 - 1) / (NW * 1024);  // 1-KiB DMA pieces per wave per patch
  constexpr int BUFB = NQW * NW * 1024;
  static_assert(BM % 16 == 0 && NQW <= 9 && NPR <= 1023 && TM >= 2 * NJ + 1, "shape");
  // (the skewed rows need NPR PU + SK (NPR / Wp + 2) units: the launcher checks it against BUFB)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUFB];

  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int tn = tile / tilesM, tm = tile - tn * tilesM;
  const int m0 = tm * BM, n0 = tn * BN + wid * 32;  // this wave's 32 columns
  const int Wp = g.W + 2, HWo = g.H * g.W;
  auto padded = [&](int m) {
    const int b = m / HWo, r = m - b * HWo, oy = r / g.W, ox = r - oy * g.W;
    return (b * (g.H + 2) + oy + 1) * Wp + ox + 1;
  };
  const int P0 = padded(m0) - (Wp + 1);  // first patch row

  // Row-skewed LDS layout (tools/lds_conflict_model.py: 3.72 -> 0.36 extra conflict cycles per
  // fragment read at 13-wide frames): patch row P (relative to the tile's first, P0) sits at LDS
  // unit U(P) = PU P + SK y(P), y(P) = (q0 + P) / Wp its image row (q0 = P0 % Wp), so the
  // 3-position jump of an image-row wrap inside a 16-row fragment lands like a 1-position step.
  // A tap (dy, dx) adds the uniform (PU (dy Wp + dx) + SK dy) units (a tap-(0, 0) row's column
  // is < W, so dx never crosses a row).  The fragment bases are per-block registers (the fp16
  // kernel has the room the x3 kernel lacked).
  constexpr int PU = LP / 16, SK = 12;
  const int fr = lane & 15, fq = lane >> 4;
  const int q0 = P0 % Wp;
  int rowoff[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int m = m0 + 16 * i + fr;
    m = m < M ? m : M - 1;
    const int pr = padded(m) - P0 - (Wp + 1);
    rowoff[i] = (PU * pr + SK * ((q0 + pr) / Wp)) * 16 + 16 * fq;
  }
  auto rowoff_of = [&](int i) {
    int v = rowoff[i];
    asm volatile("" : "+v"(v));
    return v;
  };
  auto tap_bytes = [&](int t) { return (PU * ((t / 3) * Wp + (t % 3)) + SK * (t / 3)) * 16; };

  // patch DMA: piece k of this wave = LDS bytes 1024 (wid + 8 k) + 16 lane = unit U; with V = U +
  // PU q0 = RU j + PU x + u (RU = PU Wp + SK units per image row): patch row P = Wp j + x - q0,
  // unit u (units 8, 9 of a row: the next 32 bytes of global memory; x >= Wp: the SK spare units,
  // given row P's last unit) -- never read
  const int nk = K / 64, nch = nk / 9;
  const int rowB = 2 * g.C;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  const unsigned dsoff = (unsigned)(P0 * rowB);
  const unsigned RU = (unsigned)(PU * Wp + SK);
  auto issue_patch = [&](int chunk, int k, int buf) {
    const unsigned V = 64u * (unsigned)(wid + NW * k) + (unsigned)lane + (unsigned)(PU * q0);
    const unsigned jr = V / RU, rem = V - jr * RU;
    unsigned x = rem / PU, u = rem - x * PU;
    if (x >= (unsigned)Wp) x = Wp - 1, u = PU - 1;
    const unsigned r = (unsigned)Wp * jr + x - (unsigned)q0;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rsA, (__attribute__((address_space(3))) void*)(smem + buf * BUFB + 1024 * (wid + NW * k)), 16,
        (int)(__umul24(r, (unsigned)rowB) + 16 * u), (int)(dsoff + chunk * RB), 0, 0);
  };

  // weights (order 4): 16-column block nb at nb ldb 32 bytes, K-step s group q at (2 s + q) KiB
  const unsigned bvo = (unsigned)((n0 / 16) * ldb * 32 + lane * 16);
  const int bjs = ldb * 32;
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)b_bytes, 0x00020000);
  f16x8 bq[2][2][NJ];
  auto load_b1 = [&](int s, int q, int j, f16x8& dst) {
    dst = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, bvo, (2 * s + q) * 1024 + j * bjs, 0));
  };

  f32x4 acc[TM][NJ];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int k = 0; k < NQW; ++k) issue_patch(0, k, 0);
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int j = 0; j < NJ; ++j) load_b1(0, q, j, bq[0][q][j]);
  vm_wait<0>();
  __syncthreads();

  // Per chunk: 9 taps x TM row blocks (b = TM t + i, all static), 4 MFMAs each (2 32-channel
  // groups x 2 column blocks).  The A fragments of block b + 2 are read during block b (a ring of
  // three fragment sets: 9 TM % 3 == 0, so every chunk starts at slot 0): at 4 MFMAs per block a
  // one-block lead left the LDS latency exposed.  Weights of tap t + 1 and DMA piece t of chunk
  // j + 1 are issued one per row block over the tap's first blocks.
  constexpr int LEAD = 2, RING = 3;  // (a 3-block lead with a ring of 9 measured equal)
  static_assert((9 * TM) % RING == 0 && LEAD < RING && LEAD >= 1, "fragment ring phase per chunk");
  const unsigned char* P = smem;
  f16x8 af[RING][2];
  auto rd = [&](int slot, const unsigned char* q) {
    af[slot][0] = *reinterpret_cast<const f16x8*>(q);
    af[slot][1] = *reinterpret_cast<const f16x8*>(q + 64);
  };
  auto blk = [&](const unsigned char* Pb, int bi) { return Pb + rowoff_of(bi % TM) + tap_bytes(bi / TM); };
#pragma unroll
  for (int l = 0; l < LEAD; ++l) rd(l, blk(P, l));
  for (int j = 0; j < nch; ++j) {
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int bi = TM * t + i;
        static_for<0, 2 * NJ + 1>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          if (i != q) return;
          if constexpr (q < 2 * NJ)
            load_b1(9 * j + t + 1, q / NJ, q % NJ, bq[(t + 1) & 1][q / NJ][q % NJ]);
          else
            issue_patch(j + 1, t < NQW ? t : NQW - 1, (j + 1) & 1);
        });
        const f16x8(&a)[2] = af[bi % RING];
        const f16x8(&bb)[2][NJ] = bq[t & 1];
#pragma unroll
        for (int jb = 0; jb < NJ; ++jb) acc[i][jb] = mfma16_f16(a[0], bb[0][jb], acc[i][jb]);
        if (bi + LEAD < 9 * TM) rd((bi + LEAD) % RING, blk(P, bi + LEAD));  // (the next chunk's first: after its barrier)
#pragma unroll
        for (int jb = 0; jb < NJ; ++jb) acc[i][jb] = mfma16_f16(a[1], bb[1][jb], acc[i][jb]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // the next chunk's tap 0 weights went to bq[9 & 1]
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int jb = 0; jb < NJ; ++jb) bq[0][q][jb] = bq[1][q][jb];
    vm_wait<0>();  // this wave's DMA pieces landed
    wait_lgkm0();
    raw_barrier();
    P = smem + ((j + 1) & 1) * BUFB;
#pragma unroll
    for (int l = 0; l < LEAD; ++l) rd(l, blk(P, l));
  }
  vm_wait<0>();
  wait_lgkm0();

  // epilogue: per row block, the wave's 16 x 32 outputs through a wave-private LDS stage (fp32
  // rows of 36), the reference's fp16-path epilogue, then one 16-B store of 8 halves per lane
  int* orow = reinterpret_cast<int*>(smem);
  __syncthreads();
  if (threadIdx.x < BM) {
    const int m = m0 + threadIdx.x;
    orow[threadIdx.x] = m >= M ? -1 : (g.out_padded ? padded(m) : m);
  }
  __syncthreads();
  static_assert(BM * 4 <= 1024 && 1024 + NW * 16 * 36 * 4 <= 2 * BUFB, "stage");
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
  typedef half_t h8v __attribute__((ext_vector_type(8)));
  static_for<0, TM>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        stg[(4 * fq + r) * 36 + 16 * jb + fr] = apply_epilogue_t<FL>(acc[i][jb][r], pb[jb], pm[jb], ps[jb], pg[jb], epi.flags);
    wait_lgkm0();
    const f32x4 lo = *reinterpret_cast<const f32x4*>(stg + rr * 36 + c8);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(stg + rr * 36 + c8 + 4);
    const int o = orow[16 * i + rr];
    wait_lgkm0();  // (the stage is rewritten by the next row block)
    if (o >= 0) {
      h8v v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = (half_t)lo[e];
        v[e + 4] = (half_t)hi[e];
      }
      store16_at(out, 2 * ((size_t)o * N + n0 + c8), __builtin_bit_cast(u32x4, v));
    }
  });
}

}  // namespace dnnhip
