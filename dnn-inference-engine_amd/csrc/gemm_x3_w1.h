// x3 3x3 conv (exact three-way bf16 splits of the fp32 operands, gemm_x3_patch.h), one wave
// per SIMD: the wide-N layers of the fp32 path (YOLOv2-tiny conv4-conv7), device code only.
//
// Why a second form.  The two-wave kernel (conv3x3_x3_patch_kernel) spends, per 16 x 16 block
// and 32-channel step, 6 MFMAs plus 4 v_add (the correction chain summed from zero, then one add
// into the accumulator) and re-reads the A fragment for every 32 columns: 1.4 VALU per
// v_mfma_f32_16x16x32_bf16, whose 16-cycle slot leaves 8 cycles of vector issue (MI355X_MICROARCH
// cycle constants), so two waves per SIMD ran issue-bound at 72 % MFMA busy.  Here each output
// keeps TWO accumulators over the whole K range: `accm` takes the main product a0*b0 of every
// step, `accc` the five corrections a2b0 + a1b1 + a0b2 + a1b0 + a0b1; the output is accm + accc,
// one add per output at the end.  The main accumulator still sees one MFMA rounding per step
// (as in the two-wave kernel) and no longer the per-step add; the corrections (<= 2^-7 of the
// main product each) are rounded at their own, 2^-8 smaller, magnitude.  The loop issues no
// adds at all.  The doubled accumulators need 352 registers for a 176 x 64 wave tile, so the
// workgroup is 4 waves, one per SIMD, 512 registers each (VGPR + AGPR).
//
// Per wave: BM x 64 (4 column blocks of 16), in NH passes of JH = 4 / NH column blocks per tap
// (the weight fragments of one pass live in registers, the next pass's are loaded while it
// runs).  Patch: the tile's <= NPR padded input rows of one 32-channel chunk (192 B per row:
// 3 pieces x 32 channels bf16, slots swizzled as in the two-wave kernel) staged into a double
// buffer by LDS-DMA (buffer_load ... lds, 1 KiB per wave instruction, source-side swizzle),
// chunk j + 1 in flight during chunk j's first 8 taps; one barrier per chunk.
//
// Summation order: per output, accm over the steps (chunk-major, tap-minor) of a0 b0, accc over
// the same steps of (a2b0, a1b1, a0b2, a1b0, a0b1) in that order, then accm + accc.  It depends
// on (N, K) only (batch rows are bit-identical to batch-1 runs) and is not the two-wave
// kernel's order (DNN_HIP_X3V selects that one).
#pragma once
#include "gemm_x3_patch.h"

namespace dnnhip {

// The loop is written against fixed register files: the compiler selects ONE MFMA form per
// function (accumulators in AGPRs), and 352 accumulators do not fit 256 AGPRs, so it shuttled
// them through VGPRs and scratch (1,250 v_accvgpr copies + 290 spills per chunk).  Here the
// corrections `accc` and the weight fragments live in AGPRs (224), the main accumulators `accm`,
// the A fragments and addresses in VGPRs (~230): MFMAs, weight loads and the patch DMA are
// inline asm, and every vector-memory wait in the loop is counted by hand (the compiler sees no
// vector-memory instruction there).
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4_t x3_rsrc(const void* base, unsigned bytes) {
  const unsigned long long p = (unsigned long long)base;
  return u32x4_t{(unsigned)p, (unsigned)(p >> 32) & 0xffffu, bytes, 0x00020000u};
}
// acc (AGPR) += a (VGPR) * b (AGPR)
__device__ __forceinline__ void mfma_x3_a(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "a"(b));
}
// acc (VGPR) += a (VGPR) * b (AGPR)
__device__ __forceinline__ void mfma_x3_v(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
}
// One 32-channel step of one 16 x 16 block: the five corrections back to back on c (AGPR),
// a2b0, a1b1, a0b2, a1b0, a0b1, then the main product a0b0 on m (VGPR).  One asm statement:
// a dependent MFMA right behind its producer takes the srcC forwarding path (full rate on one
// accumulator), and the compiler, which cannot see that these are MFMAs, would otherwise put
// an s_nop between every two of them.
__device__ __forceinline__ void mfma_x3_chain(f32x4& c, f32x4& m, const bf16x8 (&a)[3], const bf16x8& b0,
                                              const bf16x8& b1, const bf16x8& b2) {
  asm volatile(
      "v_mfma_f32_16x16x32_bf16 %0, %2, %5, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %3, %6, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %4, %7, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %3, %5, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %4, %6, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %4, %5, %1"
      : "+a"(c), "+v"(m)
      : "v"(a[2]), "v"(a[1]), "v"(a[0]), "v"(b0), "v"(b1), "v"(b2));
}
// ... with the main accumulator in AGPRs too (the last row block: VGPR headroom)
__device__ __forceinline__ void mfma_x3_chain_aa(f32x4& c, f32x4& m, const bf16x8 (&a)[3], const bf16x8& b0,
                                                 const bf16x8& b1, const bf16x8& b2) {
  asm volatile(
      "v_mfma_f32_16x16x32_bf16 %0, %2, %5, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %3, %6, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %4, %7, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %3, %5, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %4, %6, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %4, %5, %1"
      : "+a"(c), "+a"(m)
      : "v"(a[2]), "v"(a[1]), "v"(a[0]), "v"(b0), "v"(b1), "v"(b2));
}
// 16 B per lane from rsrc + voff + soff + IMM into an AGPR quad (counted by the caller's vmcnt)
template <int IMM>
__device__ __forceinline__ void load_b128_agpr(bf16x8& d, u32x4_t rsrc, unsigned voff, unsigned soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4" : "=a"(d) : "v"(voff), "s"(rsrc), "s"(soff), "n"(IMM));
}
// LDS-DMA: 16 B per lane from rsrc + voff + soff into LDS (m0v) + 16 lane (m0v wave-uniform);
// M0 is reserved by the compiler, so it is restored
__device__ __forceinline__ void lds_dma16_asm(u32x4_t rsrc, unsigned voff, unsigned soff, unsigned m0v) {
  unsigned saved;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(saved)
      : "v"(voff), "s"(rsrc), "s"(m0v), "s"(soff)
      : "memory");
}
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

// SWZ: the patch rows' 16-B slots XOR-swizzled by row bit 2 as in the two-wave kernel (each
// fragment address then needs the row's bit: a dependent chain of ~6 VALU per fragment, which
// a lone wave per SIMD cannot hide behind a partner's MFMAs); false: plain 192-B rows, the
// fragment address one v_add of a per-block base and the tap's uniform offset.
template <int BM, int NPR, bool POOL, bool SWZ = false>
__global__ void __launch_bounds__(256, 1)
conv3x3_x3_w1_kernel(const bf16_bits* __restrict__ in, const bf16_bits* __restrict__ Bt, float* __restrict__ out,
                     bf16_bits* __restrict__ out_split, int M, int N, int K, EpiParams epi, int tilesM, X3Geom g,
                     unsigned in_bytes, unsigned b_bytes) {
  constexpr int BN = 256, TM = BM / 16, RB = 192, NJ = 4, NH = 2, JH = NJ / NH;
  // register files: AGPRs hold only MFMA-written accumulators (accc, and the main accumulators
  // of the last MA row blocks: 176 + 16 MA), so the allocator never moves a value there; VGPRs
  // hold the other main accumulators, the fragments, the weights and the addresses
  constexpr int MA = 3;
  constexpr int NQW = NPR * RB / 1024 / 4;  // 1-KiB DMA pieces per wave per patch
  static_assert(BM % 16 == 0 && NPR % 64 == 0 && NPR <= 1024, "shape");
  static_assert(NQW % 3 == 0, "DMA source pattern repeats every 3 pieces (12 KiB = 64 rows)");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * NPR * RB];

  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int tile_s = xcd_tile(blockIdx.x, gridDim.x), ntiles = gridDim.x / g.splits;
  const int split = tile_s / ntiles, tile = tile_s - split * ntiles;
  const int tn = tile / tilesM, tm = tile - tn * tilesM;
  const int m0 = tm * BM, n0 = tn * BN + wid * 64;  // this wave's 64 columns
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

  // A fragment of row-block i: lane's output row 16 i + fr -> patch row prow[i] (tap (1, 1));
  // its k slot fq of piece p at row * 192 + 64 p + 16 (fq ^ ((row >> 1) & 2)) (gemm_x3_patch.h)
  const int fr = lane & 15, fq = lane >> 4;
  int prow[TM];  // SWZ: patch row (tap (1, 1)); else: byte offset of the tap (0, 0) row + 16 fq
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int m = m0 + 16 * i + fr;
    m = m < M ? m : M - 1;
    prow[i] = SWZ ? pixrow(m) - P0 : (pixrow(m) - P0 - (Wp + 1)) * RB + 16 * fq;
  }

  // patch DMA: this wave's piece k lands at LDS byte 1024 (wid + 4 k) + 16 lane = patch row r,
  // physical unit u (piece u / 4, slot u % 4); the lane fetches the logical slot that belongs
  // there.  The pattern repeats every 3 pieces (64 rows): 3 per-lane offsets + a uniform one.
  const int nk = K / 32, nch = nk / 9 / g.splits, cb = split * nch;
  const int rowB = 6 * g.C;  // bytes per padded row (all chunks)
  unsigned dvo[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int b = 1024 * (wid + 4 * k) + 16 * lane;
    const int r = b / RB, u = (b - r * RB) >> 4, ls = SWZ ? (u & 3) ^ ((r >> 1) & 2) : (u & 3);
    dvo[k] = (unsigned)((P0 + r) * rowB + cb * RB + 64 * (u >> 2) + 16 * ls);
  }
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  auto issue_patch = [&](int chunk, int k, int buf) {
    const unsigned soff = (unsigned)(chunk * RB + (k / 3) * 64 * rowB);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(smem + buf * NPR * RB + 1024 * (wid + 4 * k)),
                                             16, (int)dvo[k % 3], (int)soff, 0, 0);
  };

  // weight fragments: [n/16][step][piece][lane][8]; half-step hs = NH s + h holds column blocks
  // JH h .. JH h + JH - 1 of step s; a ring of two half-steps, in AGPRs
  const unsigned bvo = (unsigned)((n0 / 16) * nk * 3072 + lane * 16 + cb * 9 * 3072);
  const int bjs = nk * 3072;  // next 16-column block
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)b_bytes, 0x00020000);
  bf16x8 bq[2][3][JH];
  // unconditional (past the last step: the descriptor's zeros or another panel, never used)
  auto load_b = [&](int hs, bf16x8 (&dst)[3][JH]) {
    const int s = hs / NH, h = hs - (hs / NH) * NH;
#pragma unroll
    for (int j = 0; j < JH; ++j) {
      const unsigned so = (unsigned)(s * 3072 + (h * JH + j) * bjs);
#pragma unroll
      for (int p = 0; p < 3; ++p)
        dst[p][j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, bvo, so + p * 1024, 0));
    }
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

  auto frag = [&](const unsigned char* P, int i, int toff, bf16x8 (&a)[3]) {
    const unsigned char* q;
    if constexpr (SWZ) {
      int pr = prow[i];
      asm volatile("" : "+v"(pr));  // keep the taps' addresses from being hoisted
      const int row = pr + toff;
      q = P + row * RB + 16 * (fq ^ ((row >> 1) & 2));
    } else {
      q = P + prow[i] + (toff + Wp + 1) * RB;
    }
#pragma unroll
    for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(q + 64 * p);
  };

  // The loop runs over taps (9 per 32-channel chunk): a body of 2 half-step slots x TM row
  // blocks x 6 JH MFMAs, small enough for the register allocator to keep every accumulator
  // and weight in place (an unrolled 9-tap body made it shuttle accumulators through VGPRs
  // around the loop-carried weights, which is unsafe next to MFMAs it cannot see in asm).
  // Per slot q = 2 t + h: one DMA piece of chunk j + 1 (piece q mod NQW: every slot issues
  // exactly one, so the compiler's vmcnt for the weights is the same on every path; the
  // re-issued pieces rewrite the same bytes), then the next slot's weights, then the row
  // blocks, each reading the next block's fragments (the next tap's first block at the end;
  // after the last tap a harmless re-read that the chunk switch overwrites) while its MFMAs
  // run.  The chunk's barrier waits for everything but the last slot's weight loads.
  static_assert(NQW <= 9 * NH, "one DMA piece per slot");
  const int nsteps = 9 * nch;
  const unsigned char* P = smem;
  bf16x8 af[2][3];
  frag(P, 0, -(Wp + 1), af[0]);
  int t = 0, j = 0;
  for (int s = 0; s < nsteps; ++s) {
    const int toff = (t / 3 - 1) * Wp + (t % 3 - 1);
    const int toff_next = ((t + 1) / 3 - 1) * Wp + ((t + 1) % 3 - 1);
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int q = NH * t + h;  // this slot
      __builtin_amdgcn_sched_barrier(0);
      issue_patch(j + 1, q < NQW ? q : q - NQW, (j + 1) & 1);
      load_b(s * NH + h + 1, bq[(h + 1) & 1]);
      const bf16x8(&b)[3][JH] = bq[h];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int c = h * TM + i, cur = c & 1, nxt = cur ^ 1;
        if (i + 1 < TM)
          frag(P, i + 1, toff, af[nxt]);
        else if (h + 1 < NH)
          frag(P, 0, toff, af[nxt]);
        else  // (unconditional: a branch here made the compiler merge the fragment values)
          frag(P, 0, t < 8 ? toff_next : toff, af[nxt]);
        const bf16x8(&a)[3] = af[cur];
#pragma unroll
        for (int j2 = 0; j2 < JH; ++j2) {
          if (i < TM - MA)
            mfma_x3_chain(accc[i][h * JH + j2], accm[i][h * JH + j2], a, b[0][j2], b[1][j2], b[2][j2]);
          else  // the last MA row blocks' main accumulators in AGPRs (VGPR headroom)
            mfma_x3_chain_aa(accc[i][h * JH + j2], accm[i][h * JH + j2], a, b[0][j2], b[1][j2], b[2][j2]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    static_assert((NH * TM) % 2 == 0, "the next tap's first fragments land in af[0]");
    if (++t == 9) {  // chunk done: every wave's reads of patch j are complete, chunk j + 1 landed
      t = 0;
      ++j;
      // own DMA pieces landed (only the next slot's weight loads, 3 JH, are younger; the
      // compiler cannot see that other waves read them after the barrier), own reads done
      vm_wait<3 * JH>();
      wait_lgkm0();
      raw_barrier();
      P = smem + (j & 1) * NPR * RB;
      frag(P, 0, -(Wp + 1), af[0]);
    }
  }
  // the weight loads of the slot past the end are still in flight into AGPRs the epilogue may
  // reuse; the MFMA results need their write-back wait states before VALU / accvgpr reads
  vm_wait<0>();
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");

  // epilogue: the reference's fp32 epilogue on accm + accc, then fp32 [M][N], the split planes
  // of the next x3 layer's zero-bordered input, or the raw partial of split-K slice `split`
  // (sum first, so the AGPRs of accc are free for the epilogue's temporaries; one row block at a
  // time, so the compiler does not hoist every element's table read and parameters at once)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r) accm[i][jb][r] = accm[i][jb][r] + accc[i][jb][r];
  int* orow = reinterpret_cast<int*>(smem);
  __syncthreads();
  if constexpr (POOL) {
    if (threadIdx.x < BM / 4) {
      const int w = (m0 >> 2) + threadIdx.x, PHW = g.PH * g.PW;
      const int b = w / PHW, r = w - b * PHW, py = r / g.PW, px = r - py * g.PW;
      orow[threadIdx.x] = 4 * w >= M ? -1 : g.out_mode == 1 ? (b * (g.PH + 2) + py + 1) * (g.PW + 2) + px + 1 : w;
    }
    __syncthreads();
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb) {
      const int n = n0 + 16 * jb + fr;
      const float pb = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
      const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
      const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
      const float pg = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;
      const int cofs = (n >> 5) * 96 + (n & 31);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        __builtin_amdgcn_sched_barrier(0);
        const int o = orow[4 * i + fq];
        if (o < 0) continue;
        const float e = pool_then_epilogue(accm[i][jb], pb, pm, ps, pg, epi.flags);
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
      }
    }
    return;
  }
  if (threadIdx.x < BM) {
    const int m = m0 + threadIdx.x;
    orow[threadIdx.x] = m >= M ? -1 : (g.out_mode == 1 ? padded(m) : m);
  }
  __syncthreads();
  // (compile-time indices: with #pragma unroll the compiler left this 176-element body rolled
  // and kept accm in scratch for it)
  static_for<0, NJ>([&](auto jbc) {
    constexpr int jb = decltype(jbc)::value;
    const int n = n0 + 16 * jb + fr;  // < N: N % 256 == 0 (launcher)
    const float pb = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
    const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
    const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
    const float pg = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;
    const int cofs = (n >> 5) * 96 + (n & 31);
    static_for<0, TM>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      static_for<0, 4>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        __builtin_amdgcn_sched_barrier(0);
        const int o = orow[16 * i + 4 * fq + r];
        if (o < 0) return;
        const float v = accm[i][jb][r];
        if (g.out_mode == 2) {
          out[((size_t)split * M + o) * N + n] = v;
          return;
        }
        const float e = apply_epilogue(v, pb, pm, ps, pg, epi.flags);
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
  });
}

}  // namespace dnnhip
