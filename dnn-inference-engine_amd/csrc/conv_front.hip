// The front end of the fp32 path in one kernel: conv0 (3 -> 16 channels, 3x3 SAME, BiasAdd /
// BatchNorm / LeakyReLU, 2x2/s2 max pool) straight into conv1 (16 -> 32, the same chain and
// pool), YOLOv2-tiny's first two conv layers (proj3/yolov2tiny.py:30-40; each layer is the
// reference's im2col + cblas_sgemm + bias/bn/leaky/pool, dnn_openblas.c:135-254).
//
// Why: apart, conv0 writes its pooled 16-channel output (177 MB at batch 64) and conv1 reads it
// back and splits it into bf16 pieces; both kernels spend most of their time outside the MFMA
// (conv0: patch DMA, epilogue; conv1: the split and its epilogue).  Here conv0's
// pooled output never leaves the CU: it is computed for conv1's tile plus a one-pixel halo,
// split into the three bf16 pieces in its epilogue, and written straight into conv1's LDS patch.
//
// One workgroup per CU, persistent over 16 x 16 conv1 output tiles (8 x 8 pooled), 8 waves in
// two roles on every SIMD (a workgroup's waves go to SIMDs cyclically, so each SIMD holds one
// of each):
//   producers (waves 0-3): DMA the tile's 38 x 40-pixel frame patch (fp32, 3 channels) into one
//     of two LDS frame buffers a tile ahead; conv0 on v_mfma_f32_16x16x4_f32 for the 18 x 18
//     pooled pixels conv1's 3x3 taps read (81 blocks of 4 pool windows), exactly as
//     conv0_packed_pool_kernel: K = 27 packed into 7 steps in the reference's im2col order, rows
//     pool-window-major, pool then epilogue; pooled pixels outside the frame become conv1's zero
//     padding; each value split (split3) into conv1's patch buffer P[tile & 1];
//   consumers (waves 4-7): conv1 on P[tile & 1] exactly as conv3x3_x3_c16p_kernel (two taps per
//     16x16x32 K step, tap 8 alone on 16x16x16, two accumulators), each wave 4 row blocks of 16
//     pool-window-major rows x 32 columns, its weights (all 144 K x 32 columns, 3 pieces) held in
//     registers for the kernel's lifetime; pool, epilogue, then the staged split-plane store of
//     the x3 kernels (x3_pool_split_store) into conv2's zero-bordered input.
// The roles hand off through LDS counters (no s_barrier after the start: the two roles run
// different instruction streams): a producer fills P[k & 1] once the consumers have released
// it (tile k - 2 read), the consumers start a tile once all four producers have filled it; the
// producers meet once per tile to rotate their frame buffers.  Every MFMA sequence per output
// is the one of the two separate kernels, so the result is bit-identical to conv0_packed ->
// conv3x3_x3_c16p (tested), whatever the tile order.
//
// LDS: P 2 x 18 x 18 x 96 B (62,208) + frame 2 x 38 x 480 B (36,480) + stages 4 x 3 KiB (12,288)
// + counters and row tables: 111 KB, one workgroup per CU.
#include <hip/hip_runtime.h>
#include "dnn_common.h"
#include "gemm_x3_patch.h"
#include "gemm_x3_acc2.h"  // static_for

// FRONTDIAG (diagnostic builds only, tools/build_diag.sh with FILE=conv_front.hip; results
// unchanged): per wave s_memtime sums over the last launch -- front_diag[workgroup][wave][slot]:
// 0 kernel total, 1 waits on the other role (producers: FREE; consumers: FULL), 2 producers' conv0
// work, 3 consumers' conv1 work, 4 producers' frame-buffer meeting (vmcnt + PSYNC), 5 tiles
#ifndef FRONTDIAG
#define FRONTDIAG 0
#endif

namespace dnnhip {

#if FRONTDIAG
constexpr int FRONT_DIAG_WGS = 256, FRONT_DIAG_SLOTS = 6;
__device__ unsigned long long front_diag[FRONT_DIAG_WGS * 16 * FRONT_DIAG_SLOTS];
#endif

namespace front {
constexpr int TT = 16;             // conv1 output tile edge (pre-pool)
constexpr int PE = TT + 2;         // conv1 patch edge = pooled conv0 pixels per tile edge (18)
constexpr int NPIX = PE * PE;      // 324 pooled conv0 pixels = pool windows of conv0
constexpr int NBLK0 = NPIX / 4;    // 81 conv0 MFMA blocks (4 windows x 4 cells)
constexpr int PB = 96;             // conv1 patch pixel: 3 pieces x 16 channels x 2 B
constexpr int PBYTES = NPIX * PB;  // 31,104
constexpr int FR = 2 * TT + 6;     // frame patch rows (38)
constexpr int FPX = 2 * TT + 8;    // frame patch pixels per row (40: one alignment pixel each side)
constexpr int RS = 3 * FPX;        // frame patch row stride in floats (120 = 30 16-B DMA lanes)
constexpr int NRP = FR / 2;        // DMA instructions per frame patch (two rows each)
constexpr int NS = 5;              // conv1 K steps of 32 (taps 2s, 2s + 1; tap 9 zero)
static_assert(NPIX % 4 == 0 && FR % 2 == 0 && NBLK0 == 81, "tile");
}  // namespace front

struct FrontGeom {
  int B, H, W;         // frames (3 channels)
  int PH0, PW0;        // conv0 pooled = conv1 in/out (pre-pool) size
  int PH1, PW1;        // conv1 pooled
  int tilesX, tilesY;  // conv1 16 x 16 tiles per frame
};

// 16-B LDS-DMA (buffer_load_dwordx4 ... lds) from inline asm: the compiler's wait pass does not
// see it, so it puts no vmcnt(0) before every later LDS read (it cannot tell the frame buffers
// apart, and would wait for the next tile's DMA before this tile's first read).  The caller
// orders it with its own vmcnt wait + hand-off.  lane l writes dst + 16 l; `dst` wave-uniform.
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lds_dma16_opaque(u32x4v rsrc, unsigned voff, const void* dst) {
  const unsigned m0v =
      __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)dst);
  unsigned saved;  // M0 is a reserved register: restore it rather than clobber it
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(saved)
      : "v"(voff), "s"(rsrc), "s"(m0v)
      : "memory");
}

// tile of the workgroup's k-th iteration: each round of G tiles is handed to the G workgroups so
// that the workgroups of one XCD take consecutive tiles (their frame halos meet in one L2)
__device__ __forceinline__ int front_tile(int k, int G) { return k * G + xcd_tile(blockIdx.x, G); }

// div_rn (gemm_f32.h) with the reciprocal precomputed: the same quotient bit for bit
__device__ __forceinline__ float div_rn_r(float x, float d, double y) {
  float q = (float)((double)x * y);
  const bool bad = __builtin_amdgcn_classf(q, 0x0F0);
  if (__builtin_amdgcn_ballot_w64(bad)) q = bad ? x / d : q;
  return q;
}

// one "slot" schedule: NM MFMA items and NV VALU stages interleaved in program order, each MFMA
// item followed by its share of the stages, fenced by sched_barrier so the compiler keeps the
// interleave (a wave issues in order; an MFMA leaves most of its cycles to the wave's other
// instructions)
template <int NM, int NV, class FM, class FV>
__device__ __forceinline__ void front_interleave(FM&& fm, FV&& fv) {
  constexpr int NS = NM > 0 ? NM : 1;
  static_for<0, NS>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if constexpr (NM > 0) fm(std::integral_constant<int, i>{});
    static_for<(i * NV) / NS, ((i + 1) * NV) / NS>([&](auto vc) { fv(std::integral_constant<int, decltype(vc)::value>{}); });
    __builtin_amdgcn_sched_barrier(0);
  });
}

// LDS hand-off counters between the roles (monotonic over the kernel)
enum FrontCnt { FC_PSYNC = 0, FC_FULL0 = 1, FC_FULL1 = 2, FC_FREE0 = 3, FC_FREE1 = 4, FC_N = 8 };
typedef __attribute__((address_space(3))) unsigned lds_u32;
__device__ __forceinline__ void front_signal(unsigned* c) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes have landed
  if ((threadIdx.x & 63) == 0) __atomic_fetch_add((lds_u32*)c, 1u, __ATOMIC_RELAXED);  // one count per wave
}
// spin (with sleeps) until *c >= target; bounded so a broken hand-off cannot hang the GPU
__device__ __forceinline__ void front_wait(unsigned* c, unsigned target) {
  volatile lds_u32* v = (volatile lds_u32*)c;
  for (int guard = 0; *v < target && guard < (1 << 22); ++guard) __builtin_amdgcn_s_sleep(1);
  asm volatile("" ::: "memory");
}

constexpr int FRONT_NP = 8, FRONT_NC = 8;  // producer / consumer waves (two of each per SIMD)

template <int FL>
__global__ void __launch_bounds__(1024, 1)
conv01_front_kernel(const float* __restrict__ in, const float* __restrict__ w0, EpiParams epi0,
                    const bf16_bits* __restrict__ Bt1, EpiParams epi1, bf16_bits* __restrict__ out_split, FrontGeom g,
                    int ntiles, unsigned in_bytes, unsigned out_bytes) {
  using namespace front;
  constexpr int YOLO = EPI_BIAS | EPI_BN | EPI_LEAKY_F64;
  constexpr int STG1 = 2 * 4 * X3_STG_ROW;  // conv1 stage floats per consumer wave: 2 blocks x 4 windows
  __shared__ __attribute__((aligned(1024))) unsigned char patch[2 * PBYTES];
  __shared__ __attribute__((aligned(1024))) float frame[2][FR * RS];
  __shared__ __attribute__((aligned(1024))) unsigned char wlds[2 * NS * 3 * 1024];  // conv1 weights
  __shared__ __attribute__((aligned(16))) float stage[FRONT_NC][STG1];
  __shared__ unsigned cnt[FC_N];

  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int G = gridDim.x;
  const int nk = (ntiles - xcd_tile(blockIdx.x, G) + G - 1) / G;  // tiles of this workgroup
  const int tpi = g.tilesX * g.tilesY;
  auto decode = [&](int t, int& b, int& ty, int& tx) {
    b = t / tpi;
    const int r = t - b * tpi;
    ty = r / g.tilesX;
    tx = r - ty * g.tilesX;
  };
  {  // conv1 weights into LDS once: the packed [n/16][step][piece][lane][8] block of columns 0-31
    constexpr int BB = 2 * NS * 3 * 1024, BPT = (BB / 16 + 1023) / 1024;
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int e = threadIdx.x + u * 1024;
      if (e < BB / 16)
        *reinterpret_cast<u32x4*>(wlds + 16 * e) =
            *reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned char*>(Bt1) + 16 * e);
    }
  }
  if (threadIdx.x < FC_N) cnt[threadIdx.x] = 0;
  __syncthreads();
#if FRONTDIAG
  unsigned long long fd_[FRONT_DIAG_SLOTS] = {}, fd_t = __builtin_amdgcn_s_memtime(), fd_start = fd_t;
#define FRONT_ST(k_)                                               \
  {                                                                \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    fd_[k_] += now_ - fd_t;                                        \
    fd_t = now_;                                                   \
  }
#else
#define FRONT_ST(k_)
#endif

  if (wid < FRONT_NP) {
    // ====================================================================== producers: conv0
    // lane (n = fr, fq) of the output; B fragments of the 7 packed K steps (HWIO [k = tap * 3 +
    // c][16]) and the A offsets of k = 4 s + fq (the reference's im2col order, as
    // conv0_packed_pool_kernel: the same bits)
    const int pw = wid, n0c = fr;
    float wv[7];
    int koff[7];
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const int k = 4 * s + fq;
      const int tap = k / 3, c = k - (k / 3) * 3, dy = tap / 3, dx = tap - (tap / 3) * 3;
      wv[s] = k < 27 ? w0[k * 16 + n0c] : 0.f;
      koff[s] = k < 27 ? dy * RS + dx * 3 + c : 0;
    }
    const int ef0 = FL < 0 ? epi0.flags : FL;
    const float pb0 = (ef0 & EPI_BIAS) ? epi0.bias[n0c] : 0.f;
    const float pm0 = (ef0 & (EPI_BN | EPI_BN_AB)) ? epi0.mean[n0c] : 0.f;
    const float ps0 = (ef0 & (EPI_BN | EPI_BN_AB)) ? epi0.sq[n0c] : 1.f;
    const float pg0 = (ef0 & EPI_BN) ? epi0.gamma[n0c] : 1.f;
    const bool dec0 = ((ef0 & EPI_BN) && pg0 < 0.f) || ((ef0 & EPI_BN_AB) && pm0 < 0.f);  // pool takes the min
    const double rsq0 = 1.0 / (double)ps0;
    // this wave's blocks blk_j = pw + 8 j: two groups of 5 (j 0-4, 5-9) and, for wave 0, the 81st
    // block (j = 10).  The frame offset of the lane's A row's tap-(0, 0) pixel: window 4 blk +
    // (fr >> 2), cell ((fr & 3) >> 1, fr & 1)
    auto aoff_of = [&](int j) {
      const int wa = 4 * (pw + 8 * j) + (fr >> 2);
      const int pya = (wa * 3641) >> 16, pxa = wa - PE * pya;  // wa / 18 for wa < 324
      return (2 * pya + ((fr & 3) >> 1)) * RS + (2 * pxa + (fr & 1) + 1) * 3;
    };

    // frame patch DMA: instruction j of this wave covers rows 2 rp, 2 rp + 1 (rp = pw + 8 j), lane
    // l < 60 one 16-B chunk q = l % 30 of row 2 rp + l / 30.  The patch starts one pixel left of
    // the tap halo so that 4-pixel groups (3 chunks) align with the frame's edges (W % 4 == 0):
    // a chunk is wholly inside or wholly outside the frame, and outside ones read zero.
    const unsigned long long ia = (unsigned long long)(uintptr_t)in;
    const u32x4v rsIn = {(unsigned)ia, (unsigned)(ia >> 32) & 0xffffu, in_bytes, 0x00020000u};  // as make_buffer_rsrc
    const int drow = lane >= 30 ? 1 : 0, dq = lane - 30 * drow, dgrp = dq / 3;
    auto issue = [&](int t, int buf) {
      int b, ty, tx;
      decode(t, b, ty, tx);
      const int fy0 = 2 * TT * ty - 3, fx0 = 2 * TT * tx - 4;
      const bool xok = (unsigned)(fx0 + 4 * dgrp) < (unsigned)g.W;
      const int rowf = (b * g.H + fy0) * g.W + fx0;  // pixel index of patch (0, 0) (may be < 0)
#pragma unroll
      for (int j = 0; j < (NRP + FRONT_NP - 1) / FRONT_NP; ++j) {
        const int rp = pw + FRONT_NP * j;
        if (rp < NRP && lane < 60) {
          const int r = 2 * rp + drow;
          const bool ok = xok && (unsigned)(fy0 + r) < (unsigned)g.H;
          const unsigned off = ok ? (unsigned)(((rowf + r * g.W) * 3 + 4 * dq) * 4) : OOB_OFF;
          lds_dma16_opaque(rsIn, off, &frame[buf][rp * 2 * RS]);
        }
      }
    };

    f32x4 c0[2][5];   // the two groups' accumulators
    float a0n[2][5];  // A values one step ahead
    int aoff[5];
    float ev[5], er[5];
    auto m0_pre = [&](const float* F, int gi) {
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        aoff[q] = aoff_of(5 * gi + q);
        a0n[0][q] = F[aoff[q] + koff[0]];
      }
    };
    // MFMA item i of group gi: step st = i / 5 of chain q = i % 5
    auto m0_item = [&](const float* F, int gi, auto ic) {
      constexpr int i = decltype(ic)::value, st = i / 5, q = i % 5;
      if constexpr (st == 0) c0[gi][q] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (st + 1 < 7) a0n[(st + 1) & 1][q] = F[aoff[q] + koff[st + 1]];
      if constexpr ((FRONTDIAG & 4) != 0)  // (diagnostic: a VALU multiply-add instead of the MFMA)
        c0[gi][q][st & 3] += a0n[st & 1][q] * wv[st];
      else
        c0[gi][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0n[st & 1][q], wv[st], c0[gi][q], 0, 0, 0);
    };
    // epilogue stage v of group gi (7 stages x 5 blocks, stage-major): pool, the exact epilogue,
    // conv1's zero padding outside the frame, the three pieces into conv1's patch (split3)
    auto e0_stage = [&](unsigned char* P, int qy0, int qx0, int gi, auto vc) {
      constexpr int v = decltype(vc)::value, st = v / 5, q = v % 5;
      const f32x4& c = c0[gi][q];
      const int wo = 4 * (pw + 8 * (5 * gi + q)) + fq;
      unsigned short* d = reinterpret_cast<unsigned short*>(P + wo * PB) + n0c;
      if constexpr ((FRONTDIAG & 8) != 0) {  // (diagnostic: no epilogue, the raw value's top half)
        if constexpr (st == 0) d[0] = (unsigned short)(__builtin_bit_cast(unsigned, c[0] + c[1] + c[2] + c[3]) >> 16);
      } else if constexpr (st == 0) {
        const float hi = __builtin_fmaxf(__builtin_fmaxf(c[0], c[1]), __builtin_fmaxf(c[2], c[3]));
        const float lo = __builtin_fminf(__builtin_fminf(c[0], c[1]), __builtin_fminf(c[2], c[3]));
        ev[q] = dec0 ? lo : hi;
      } else if constexpr (st == 1) {
        if constexpr (FL == YOLO)
          ev[q] = div_rn_r((ev[q] + pb0) - pm0, ps0, rsq0) * pg0;
        else
          ev[q] = apply_epilogue_t<FL>(ev[q], pb0, pm0, ps0, pg0, epi0.flags);
      } else if constexpr (st == 2) {
        if constexpr (FL == YOLO) ev[q] = ev[q] < 0.f ? (float)(0.1 * (double)ev[q]) : ev[q];
      } else if constexpr (st == 3) {
        const int pyo = (wo * 3641) >> 16, pxo = wo - PE * pyo;
        const bool inside = (unsigned)(qy0 + pyo) < (unsigned)g.PH0 && (unsigned)(qx0 + pxo) < (unsigned)g.PW0;
        ev[q] = inside ? ev[q] : 0.f;
      } else if constexpr (st == 4) {  // split3 (gemm_f32.h), first piece
        const float x = ev[q];
        const unsigned short r = bf16_rn(x);
        const bool fin = __builtin_isfinite(x);
        const bool ovf = fin && (r & 0x7fffu) == 0x7f80u;
        const unsigned short s0 = ovf ? (unsigned short)(__builtin_bit_cast(unsigned, x) >> 16) : r;
        er[q] = fin ? x - bf16_f(s0) : 0.f;
        d[0] = s0;
      } else if constexpr (st == 5) {
        const unsigned short s1 = bf16_rn(er[q]);
        d[16] = s1;
        er[q] = er[q] - bf16_f(s1);
      } else {
        d[32] = bf16_rn(er[q]);
      }
    };
    auto block81 = [&](const float* F, unsigned char* P, int qy0, int qx0) {  // wave 0's 81st block
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 7; ++st) c = __builtin_amdgcn_mfma_f32_16x16x4f32(F[aoff_of(10) + koff[st]], wv[st], c, 0, 0, 0);
      const int wo = 4 * 80 + fq;
      const int pyo = (wo * 3641) >> 16, pxo = wo - PE * pyo;
      const bool inside = (unsigned)(qy0 + pyo) < (unsigned)g.PH0 && (unsigned)(qx0 + pxo) < (unsigned)g.PW0;
      const float e = pool_then_epilogue_t<FL>(c, pb0, pm0, ps0, pg0, epi0.flags);
      unsigned short s0, s1, s2;
      split3(inside ? e : 0.f, s0, s1, s2);
      unsigned short* d = reinterpret_cast<unsigned short*>(P + wo * PB) + n0c;
      d[0] = s0;
      d[16] = s1;
      d[32] = s2;
    };

    // tile k: frame k landed (own wait + the producers' meeting), the DMA of tile k + 1 issued;
    // [group 0 MFMAs | group 1 epilogue of tile k - 1], then tile k - 1 handed over;
    // [group 1 MFMAs | group 0 epilogue of tile k] once the consumers have released P[k & 1]
    auto tile = [&](auto hpc, int k) {
      constexpr bool HP = decltype(hpc)::value;  // tile k - 1's group 1 epilogue pending
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's rows of frame[k & 1] landed
      front_signal(&cnt[FC_PSYNC]);
      front_wait(&cnt[FC_PSYNC], FRONT_NP * (unsigned)(k + 1));  // all landed; everyone done with tile k - 1's frame
      FRONT_ST(4)
      if (k + 1 < nk) issue(front_tile(k + 1, G), (k + 1) & 1);
      int b, ty, tx, bp = 0, typ = 0, txp = 0;
      decode(front_tile(k, G), b, ty, tx);
      if (HP) decode(front_tile(k - 1, G), bp, typ, txp);
      const int qy0 = TT * ty - 1, qx0 = TT * tx - 1, qy0p = TT * typ - 1, qx0p = TT * txp - 1;
      const float* F = frame[k & 1];
      unsigned char* P = patch + (k & 1) * PBYTES;
      unsigned char* Pp = patch + ((k + 1) & 1) * PBYTES;  // tile k - 1's buffer
      m0_pre(F, 0);
      front_interleave<35, HP ? 35 : 0>([&](auto ic) { m0_item(F, 0, ic); },
                                       [&](auto vc) { e0_stage(Pp, qy0p, qx0p, 1, vc); });
      if constexpr (HP) front_signal(&cnt[FC_FULL0 + ((k + 1) & 1)]);  // tile k - 1 complete in P[(k - 1) & 1]
      FRONT_ST(2)
      if (k >= 2) front_wait(&cnt[FC_FREE0 + (k & 1)], FRONT_NC * (unsigned)(k / 2));  // tile k - 2 read
      FRONT_ST(1)
      m0_pre(F, 1);
      front_interleave<35, 35>([&](auto ic) { m0_item(F, 1, ic); }, [&](auto vc) { e0_stage(P, qy0, qx0, 0, vc); });
      if (pw == 0) block81(F, P, qy0, qx0);  // (before the next meeting: the frame buffer is then refilled)
      FRONT_ST(2)
    };
    if (nk > 0) {
      issue(front_tile(0, G), 0);
      tile(std::false_type{}, 0);
      for (int k = 1; k < nk; ++k) tile(std::true_type{}, k);
      // the last tile's group 1 epilogue and hand-over
      const int k = nk - 1;
      int b, ty, tx;
      decode(front_tile(k, G), b, ty, tx);
      unsigned char* P = patch + (k & 1) * PBYTES;
      static_for<0, 35>([&](auto vc) { e0_stage(P, TT * ty - 1, TT * tx - 1, 1, vc); });
      front_signal(&cnt[FC_FULL0 + (k & 1)]);
      FRONT_ST(2)
    }
  } else {
    // ====================================================================== consumers: conv1
    // blocks 2 cw, 2 cw + 1 of the tile's 16 (pool-window-major rows), 32 columns, the x3 steps of
    // conv3x3_x3_c16p_kernel (two taps per 16x16x32 step, tap 8 on 16x16x16, two accumulators),
    // weights from LDS; epilogue through a wave-private stage into 16-B split-plane stores
    const int cw = wid - FRONT_NP;
    const int ef1 = FL < 0 ? epi1.flags : FL;
    X3EpiCol ec[2];
    ec[0] = x3_epi_col(epi1, ef1, fr);
    ec[1] = x3_epi_col(epi1, ef1, 16 + fr);
    int prow[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (2 * cw + i) * 16 + fr, w = r >> 2, q = r & 3;
      const int ly = 2 * (w >> 3) + (q >> 1), lx = 2 * (w & 7) + (q & 1);
      prow[i] = ((ly + 1) * PE + lx + 1) * PB;
    }
    const int th = fq >> 1, fqo = 16 * (fq & 1);
    auto toff = [&](int s) {  // this lane's tap offset (bytes) in full step s
      const int ta = 2 * s, tb = 2 * s + 1 < 9 ? 2 * s + 1 : 8;
      const int oa = ((ta / 3 - 1) * PE + (ta % 3 - 1)) * PB, ob = ((tb / 3 - 1) * PE + (tb % 3 - 1)) * PB;
      return th ? ob : oa;
    };
    const int hoff = (PE + 1) * PB + 8 * fq;                   // tap (2, 2) relative to (1, 1), channels 4 fq..
    const int hb = (fr + 16 * (fq >> 1)) * 16 + 8 * (fq & 1);  // the K = 16 step's B: 8 B of packed step 4
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    const auto rsOut = __builtin_amdgcn_make_buffer_rsrc((void*)out_split, 0, (int)out_bytes, 0x00020000);
    float* stg = stage[cw];
    for (int k = 0; k < nk; ++k) {
      int b, ty, tx;
      decode(front_tile(k, G), b, ty, tx);
      front_wait(&cnt[FC_FULL0 + (k & 1)], FRONT_NP * (unsigned)(k / 2 + 1));  // the producers filled P[k & 1]
      FRONT_ST(1)
      const unsigned char* P = patch + (k & 1) * PBYTES;
      f32x4 acc[2][2], accc[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = accc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      bf16x8 af[2][3], bq[3][2];
      auto frag = [&](int i, int off, bf16x8 (&a)[3]) {
        const unsigned char* q = P + prow[i] + fqo + off;
#pragma unroll
        for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(q + 32 * p);
      };
      frag(0, toff(0), af[0]);
#pragma unroll
      for (int s = 0; s < NS - 1; ++s) {
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            bq[p][j] = *reinterpret_cast<const bf16x8*>(wlds + (j * NS * 3 + s * 3 + p) * 1024 + lane * 16);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int cur = i, nxt = i ^ 1;
          if (i == 0)
            frag(1, toff(s), af[nxt]);
          else if (s + 1 < NS - 1)
            frag(0, toff(s + 1), af[nxt]);
          if constexpr ((FRONTDIAG & 2) == 0) {
#pragma unroll
            for (int jb = 0; jb < 2; ++jb) x3_step<true>(acc[i][jb], accc[i][jb], af[cur], bq, jb);
          } else {  // (diagnostic: no conv1 MFMAs in the full steps)
            acc[i][0][0] += __builtin_bit_cast(float, (unsigned)__builtin_bit_cast(unsigned short, af[cur][0][0]) << 16) +
                            __builtin_bit_cast(float, (unsigned)__builtin_bit_cast(unsigned short, bq[0][0][0]) << 16);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      {  // the K = 16 step (tap 8 alone)
        s16x4 ha[2][3], hq[2][3];
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            ha[j][p] = *reinterpret_cast<const s16x4*>(P + prow[j] + hoff + 32 * p);
            hq[j][p] = *reinterpret_cast<const s16x4*>(wlds + (j * NS * 3 + 4 * 3 + p) * 1024 + hb);
          }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int jb = 0; jb < 2; ++jb) {
            f32x4 c = accc[i][jb];
            c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ha[i][2], hq[jb][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ha[i][1], hq[jb][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ha[i][0], hq[jb][2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ha[i][1], hq[jb][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ha[i][0], hq[jb][1], c, 0, 0, 0);
            accc[i][jb] = c;
            acc[i][jb] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ha[i][0], hq[jb][0], acc[i][jb], 0, 0, 0);
          }
      }
      front_signal(&cnt[FC_FREE0 + (k & 1)]);  // P[k & 1] read: the producers may fill it with tile k + 2
      x3_fold(acc, accc);
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          stg[(4 * i + fq) * X3_STG_ROW + 16 * jb + fr] =
              pool_then_epilogue_t<FL>(acc[i][jb], ec[jb].pb, ec[jb].pm, ec[jb].ps, ec[jb].pg, epi1.flags);
      wait_lgkm0();  // the stage is wave-private
      {  // x3_pool_split_store's task layout, 32 tasks (lanes 0-31: window lane / 4, 8 columns)
        const int wl = (lane & 31) >> 2, c8 = 8 * (lane & 3);
        const f32x4 lo = *reinterpret_cast<const f32x4*>(stg + wl * X3_STG_ROW + c8);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(stg + wl * X3_STG_ROW + c8 + 4);
        bool ok = true;
#pragma unroll
        for (int e = 0; e < 4; ++e) ok = ok && x3_split_ok(lo[e]) && x3_split_ok(hi[e]);
        const bool fast = __builtin_amdgcn_ballot_w64(!ok) == 0;
        u32x4 qv[3];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          unsigned w0_, w1_, w2_;
          split3_pack2(fast, e < 2 ? lo[2 * e] : hi[2 * e - 4], e < 2 ? lo[2 * e + 1] : hi[2 * e - 3], w0_, w1_, w2_);
          qv[0][e] = w0_;
          qv[1][e] = w1_;
          qv[2][e] = w2_;
        }
        const int w = 8 * cw + wl, py = w >> 3, px = w & 7;
        const int o = (b * (g.PH1 + 2) + 8 * ty + py + 1) * (g.PW1 + 2) + 8 * tx + px + 1;
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) {
          const unsigned off = lane < 32 ? (unsigned)((o * 96 + 32 * pc + c8) * 2) : OOB_OFF;
          __builtin_amdgcn_raw_buffer_store_b128(qv[pc], rsOut, off, 0, 0);
        }
      }
      FRONT_ST(3)
    }
  }
#if FRONTDIAG
  fd_[0] = __builtin_amdgcn_s_memtime() - fd_start;
  if (lane == 0 && blockIdx.x < FRONT_DIAG_WGS)
    for (int q_ = 0; q_ < FRONT_DIAG_SLOTS; ++q_)
      front_diag[(blockIdx.x * 16 + wid) * FRONT_DIAG_SLOTS + q_] = q_ == 5 ? (unsigned long long)nk : fd_[q_];
#endif
#undef FRONT_ST
}

// opt-in (DNN_HIP_FRONT=1): measured slower than the two kernels it replaces
static bool front_enabled() {
  const char* e = getenv("DNN_HIP_FRONT");
  return e && e[0] == '1';
}

bool conv01_front_supported(int B, int H, int W) {
  return front_enabled() && B > 0 && H % 32 == 0 && W % 32 == 0 &&
         (size_t)B * H * W * 12 < OOB_OFF && (size_t)B * (H / 4 + 2) * (W / 4 + 2) * 192 < OOB_OFF;
}

int launch_conv01_front(const float* in, const float* w0, const EpiParams& epi0, const bf16_bits* Bt1,
                        const EpiParams& epi1, bf16_bits* out_split, int B, int H, int W, hipStream_t s) {
  if (B == 0) return 0;
  if (!conv01_front_supported(B, H, W)) {
    set_error("conv01_front: unsupported shape %dx%dx%d", B, H, W);
    return -2;
  }
  FrontGeom g{B, H, W, H / 2, W / 2, H / 4, W / 4, W / 32, H / 32};
  const int ntiles = B * g.tilesX * g.tilesY;
  const int cus = device_cu_count();
  const int G = ntiles < cus ? ntiles : cus;
  const unsigned in_bytes = (unsigned)((size_t)B * H * W * 12);
  const unsigned out_bytes = (unsigned)((size_t)B * (H / 4 + 2) * (W / 4 + 2) * 192);
  constexpr int YOLO = EPI_BIAS | EPI_BN | EPI_LEAKY_F64;
  if (epi0.flags == YOLO && epi1.flags == YOLO)
    hipLaunchKernelGGL((conv01_front_kernel<YOLO>), dim3(G), dim3(1024), 0, s, in, w0, epi0, Bt1, epi1, out_split, g,
                       ntiles, in_bytes, out_bytes);
  else
    hipLaunchKernelGGL((conv01_front_kernel<-1>), dim3(G), dim3(1024), 0, s, in, w0, epi0, Bt1, epi1, out_split, g,
                       ntiles, in_bytes, out_bytes);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("launch conv01_front: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

}  // namespace dnnhip

#if FRONTDIAG
extern "C" __attribute__((visibility("default"))) int dnn_front_diag_stamps(unsigned long long* host, int n) {
  if (n > dnnhip::FRONT_DIAG_WGS * 16 * dnnhip::FRONT_DIAG_SLOTS) n = dnnhip::FRONT_DIAG_WGS * 16 * dnnhip::FRONT_DIAG_SLOTS;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dnnhip::front_diag), (size_t)n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? n : -1;
}
#endif
