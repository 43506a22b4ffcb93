// Patch conv: 3x3 / stride 1 / SAME conv with 16 or 32 input channels (YOLOv2-tiny conv1:
// 208x208x16 -> 32) + bias/BN/leaky epilogue + the following 2x2/stride-2 max pool, on
// fp32 MFMA 16x16x4.
//
// With K = 144 the implicit GEMM (gemm_f32_glds_kernel MODE 2) spends more vector issue on
// per-row setup, per-tap DMA address arithmetic and the 4 epilogues of every pooled output
// than the MFMAs take (≈1,100 VALU instructions per wave against 80 MFMAs, SQ counters in
// profiles/).  Here a workgroup owns a 16x16-pixel output tile and 32 output channels:
//   * one LDS-DMA pass stages the (16+2)x(16+2)xC input patch (halo and SAME padding from
//     the zero page) and the 32 x Kpad weight block; nothing else is loaded;
//   * every tap (dy, dx) is then a constant LDS offset from a per-lane base, so the main
//     loop is ds_read_b128 + MFMA only;
//   * A rows are pool-window-major (row = 4*window + 2*dy + dx), so the 16x16x4 result keeps
//     a window's 4 conv outputs in one lane's 4 registers; the lane pools first and runs the
//     epilogue once per pooled output (see pool_then_epilogue).
// K order: tap-major, channels in groups of 16 with the K permutation of gemm_f32.h (lane part
// p reads channels 4p..4p+3 and feeds them to 4 consecutive MFMAs), i.e. the exact MFMA
// sequence per accumulator of the implicit-GEMM path with the 16x16x4 family, so both give
// the same bits (tests/test_gpu_parity.py).
#include <hip/hip_runtime.h>
#include <cfloat>
#include "dnn_common.h"
#include "gemm_f32.h"

namespace dnnhip {

constexpr int PT_EDGE = 16;           // conv-output pixels per tile edge (8 x 8 pool windows)
constexpr int PT_PATCH = PT_EDGE + 2;  // patch edge: 1-pixel halo on each side
constexpr int PT_NB = 32;             // output channels per workgroup

__host__ __device__ constexpr int patch_kpad(int C) { return (9 * C + 31) / 32 * 32; }

template <int C>
__global__ void __launch_bounds__(256)
conv3x3_patch_pool_kernel(const float* __restrict__ in, const float* __restrict__ Bt, float* __restrict__ out,
                          DirectGeom g, int N, int tilesX, int tilesY, int nblkN, const float* __restrict__ zero,
                          EpiParams epi, bf16_bits* __restrict__ out_split) {
  typedef Mfma<16> MM;
  constexpr int KP = patch_kpad(C);
  constexpr int PATCH = PT_PATCH * PT_PATCH * C;  // floats
  constexpr int PATCH_CH = (PATCH + 255) / 256;    // 1-KiB DMA chunks (64 lanes x 16 B)
  constexpr int W_CH = PT_NB * KP / 256;
  static_assert(C % 16 == 0 && (PT_NB * KP) % 256 == 0, "patch conv shape");
  __shared__ __attribute__((aligned(1024))) float smem[(PATCH_CH + W_CH) * 256];

  // tile order: output-channel block fastest, then x, y, image (neighbours share halo rows)
  int t = xcd_tile(blockIdx.x, gridDim.x);
  const int nb = t % nblkN;
  t /= nblkN;
  const int tx = t % tilesX;
  t /= tilesX;
  const int ty = t % tilesY;
  const int b = t / tilesY;
  const int y0 = ty * PT_EDGE, x0 = tx * PT_EDGE;
  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);

  // ---- stage the input patch and the weight block (LDS-DMA, lane-linear destinations)
  const float* inb = in + (size_t)b * g.H * g.W * C;
  for (int c = wid; c < PATCH_CH; c += 4) {
    const int f = c * 256 + 4 * lane;
    const int pp = f / C, ch = f - pp * C;
    const int py = pp / PT_PATCH, px = pp - py * PT_PATCH;
    const int iy = y0 - 1 + py, ix = x0 - 1 + px;
    const bool ok = pp < PT_PATCH * PT_PATCH && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
    lds_dma16(ok ? inb + ((size_t)iy * g.W + ix) * C + ch : zero, smem + c * 256);
  }
  const float* wsrc = Bt + (size_t)nb * PT_NB * KP + 4 * lane;
  for (int c = wid; c < W_CH; c += 4) lds_dma16(wsrc + c * 256, smem + (PATCH_CH + c) * 256);
  wait_vmcnt<0>();
  raw_barrier();

  // ---- fragments.  Wave w owns conv rows 4w..4w+3 x 16 columns = 4 M-tiles of 16 rows;
  // M-tile i covers window row (i>>1) and window columns 4(i&1)..4(i&1)+3; its row r is
  // window r>>2, position r&3 = (dy, dx) = (pos>>1, pos&1).
  const int fr = lane & 15, fp = lane >> 4;
  int abase[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int wi = fr >> 2, pos = fr & 3;
    const int y = 4 * wid + 2 * (i >> 1) + (pos >> 1);
    const int x = 2 * (4 * (i & 1) + wi) + (pos & 1);
    abase[i] = (y * PT_PATCH + x) * C + 4 * fp;
  }
  const float* Ws = smem + PATCH_CH * 256;
  const int bbase = fr * KP + 4 * fp;

  MM::acc_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
    for (int cc = 0; cc < C / 16; ++cc) {
      const int aoff = ((tap / 3) * PT_PATCH + (tap % 3)) * C + 16 * cc;
      const int boff = tap * C + 16 * cc;
      f32x4 af[4], bf[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const f32x4*>(smem + abase[i] + aoff);
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = *reinterpret_cast<const f32x4*>(Ws + bbase + 16 * j * KP + boff);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = MM::op(af[i][s], bf[j][s], acc[i][j]);
    }
  }

  // ---- pool + epilogue + store: lane holds window fp of M-tile i, channel 16j + fr
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = nb * PT_NB + 16 * j + fr;
    const float pb = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
    const float pm = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
    const float ps = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
    const float pg = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int wy = (y0 >> 1) + 2 * wid + (i >> 1), wx = (x0 >> 1) + 4 * (i & 1) + fp;
      const float v = pool_then_epilogue(acc[i][j], pb, pm, ps, pg, epi.flags);
      if (!(wy < g.PH && wx < g.PW && n < N)) continue;
      if (out_split) {  // x3 split planes of the zero-bordered next-layer input
        unsigned short s0, s1, s2;
        split3(v, s0, s1, s2);
        bf16_bits* d = out_split + (((size_t)b * (g.PH + 2) + wy + 1) * (g.PW + 2) + wx + 1) * (3 * (size_t)N) +
                       (n >> 5) * 96 + (n & 31);
        d[0] = s0;
        d[32] = s1;
        d[64] = s2;
      } else {
        out[(((size_t)b * g.PH + wy) * g.PW + wx) * N + n] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Persistent form for C = 16 (YOLOv2-tiny conv1), same MFMA sequence per accumulator as the
// kernel above (so the same bits):
//   * each lane keeps its weight fragments for all 9 taps and both 16-channel N-tiles in
//     registers (18 x f32x4), loaded once per workgroup: no weight staging per tile, no B reads
//     from LDS (those were 4-way bank conflicts at the 640-B weight row pitch);
//   * the input patch is double-buffered in LDS: tile k+1's patch is DMA'd while tile k's MFMAs
//     run, so the load latency is hidden inside the workgroup, not only by other workgroups;
//   * the 4 16-B channel quads of a patch pixel are stored XOR-swizzled by the patch row's
//     parity (quad q at q ^ 2(y&1)), which makes every ds_read_b128 of the A fragments
//     conflict-free for all 9 taps (the plain layout is 2-way: two pixels of a 16-lane group
//     share each 64-B bank quarter); the DMA applies the swizzle on the source side.
constexpr int PP_C = 16;
constexpr int PP_PIX = PT_PATCH * PT_PATCH;             // 324 patch pixels
constexpr int PP_CH = (PP_PIX * PP_C + 255) / 256;      // 1-KiB DMA chunks per patch (21)
constexpr int PP_WG_PER_CU = 3;                         // 2 x 21 KiB of LDS per workgroup

// X3OUT: store the pooled outputs as x3 split planes (3 bf16 pieces, 2-B buffer stores) into a
// zero-bordered [B][PH+2][PW+2][3][32] buffer at `out` (the next layer is an x3 conv)
template <bool X3OUT>
__global__ void __launch_bounds__(256, PP_WG_PER_CU)  // 3 waves per SIMD: <= 168 registers
conv3x3_patch_pool_c16_persistent(const float* __restrict__ in, const float* __restrict__ Bt, int ldb,
                                  float* __restrict__ out, DirectGeom g, int tilesX, int tilesY, int ntiles,
                                  const float* __restrict__ zero, EpiParams epi) {
  constexpr int NST = X3OUT ? 24 : 8;  // stores per tile and lane (always issued)
  typedef Mfma<16> MM;
  constexpr int C = PP_C;
  __shared__ __attribute__((aligned(1024))) float smem[2 * PP_CH * 256];
  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int fr = lane & 15, fp = lane >> 4;

  // weight fragments: tap, N-tile j -> Bt[16j + fr][tap*16 + 4fp .. +3]
  f32x4 bw[9][2];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bw[tap][j] = *reinterpret_cast<const f32x4*>(Bt + (size_t)(16 * j + fr) * ldb + tap * C + 4 * fp);
  float pb[2], pm[2], ps[2], pg[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = 16 * j + fr;
    pb[j] = (epi.flags & EPI_BIAS) ? epi.bias[n] : 0.f;
    pm[j] = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.mean[n] : 0.f;
    ps[j] = (epi.flags & (EPI_BN | EPI_BN_AB)) ? epi.sq[n] : 1.f;
    pg[j] = (epi.flags & EPI_BN) ? epi.gamma[n] : 1.f;
  }

  // A fragment bases (floats) for even / odd tap rows dy: the lane's pixel in M-tile i, its
  // channel quad fp swizzled by the parity of the patch row it lands on
  int abase[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int wi = fr >> 2, pos = fr & 3;
    const int y = 4 * wid + 2 * (i >> 1) + (pos >> 1);
    const int x = 2 * (4 * (i & 1) + wi) + (pos & 1);
#pragma unroll
    for (int d = 0; d < 2; ++d) abase[i][d] = (y * PT_PATCH + x) * C + 4 * (fp ^ (2 * ((y + d) & 1)));
  }

  // DMA of tile t's patch into buffer `buf`: physical quad ps of pixel pp holds channel quad
  // ps ^ 2(py & 1)
  auto issue_patch = [&](int t, int buf) {
    const int tx = t % tilesX, tt = t / tilesX, ty = tt % tilesY, b = tt / tilesY;
    const float* inb = in + (size_t)b * g.H * g.W * C;
    for (int c = wid; c < PP_CH; c += 4) {
      const int f = c * 256 + 4 * lane;
      const int pp = f / C, q = (f - pp * C) >> 2;
      const int py = pp / PT_PATCH, px = pp - py * PT_PATCH;
      const int iy = ty * PT_EDGE - 1 + py, ix = tx * PT_EDGE - 1 + px;
      const bool ok = pp < PP_PIX && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
      lds_dma16(ok ? inb + ((size_t)iy * g.W + ix) * C + 4 * (q ^ (2 * (py & 1))) : zero,
                smem + (buf * PP_CH + c) * 256);
    }
  };

  const auto orsrc = out_rsrc(out, X3OUT ? (unsigned)((size_t)g.B * (g.PH + 2) * (g.PW + 2) * 32 * 6)
                                       : (unsigned)((size_t)g.B * g.PH * g.PW * 32 * sizeof(float)));
  int t = blockIdx.x, buf = 0;
  if (t < ntiles) issue_patch(t, 0);
  for (; t < ntiles; t += gridDim.x) {
    // this wave's DMAs of `buf` landed: all but the previous tile's NST stores (issued after
    // them, never branched around: buffer stores) have completed
    if (buf == 0 && t == (int)blockIdx.x)
      wait_vmcnt<0>();
    else
      wait_vmcnt<NST>();
    raw_barrier();    // everyone's landed; everyone finished reading buf ^ 1
    if (t + (int)gridDim.x < ntiles) issue_patch(t + gridDim.x, buf ^ 1);
    const float* P = smem + buf * PP_CH * 256;

    MM::acc_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, aoff = (dy * PT_PATCH + tap % 3) * C;
      f32x4 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const f32x4*>(P + abase[i][dy & 1] + aoff);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = MM::op(af[i][s], bw[tap][j][s], acc[i][j]);
    }

    const int tx = t % tilesX, tt = t / tilesX, ty = tt % tilesY, b = tt / tilesY;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = 16 * j + fr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int wy = ty * (PT_EDGE / 2) + 2 * wid + (i >> 1), wx = tx * (PT_EDGE / 2) + 4 * (i & 1) + fp;
        const float v = pool_then_epilogue(acc[i][j], pb[j], pm[j], ps[j], pg[j], epi.flags);
        const bool in_frame = wy < g.PH && wx < g.PW;
        if constexpr (X3OUT) {
          unsigned short s0, s1, s2;
          split3(v, s0, s1, s2);
          const unsigned o = in_frame ? (unsigned)(((((size_t)b * (g.PH + 2) + wy + 1) * (g.PW + 2) + wx + 1) * 96 + n) * 2)
                                      : OOB_OFF;
          __builtin_amdgcn_raw_buffer_store_b16(s0, orsrc, o, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b16(s1, orsrc, o + (in_frame ? 64u : 0u), 0, 0);
          __builtin_amdgcn_raw_buffer_store_b16(s2, orsrc, o + (in_frame ? 128u : 0u), 0, 0);
        } else {
          store4(orsrc, in_frame ? (unsigned)(((((size_t)b * g.PH + wy) * g.PW + wx) * 32 + n) * 4) : OOB_OFF, v);
        }
      }
    }
    buf ^= 1;
  }
}

// OC == 32 only: the implicit/explicit GEMMs use the 16x16x4 family for N <= 32 and 32x32x2
// above, and the plan keeps one MFMA family per layer shape so every path of a layer gives the
// same bits (the kernel itself handles any OC % 32 == 0).
bool patch_conv_pool_supported(int C, int OC, int H, int W, int OH, int OW, int kh, int kw, int sh, int sw, int pt,
                               int pl) {
  return kh == 3 && kw == 3 && sh == 1 && sw == 1 && pt == 1 && pl == 1 && OH == H && OW == W &&
         (C == 16 || C == 32) && OC == PT_NB && OH % 2 == 0 && OW % 2 == 0;
}

int patch_conv_kpad(int C) { return patch_kpad(C); }

int launch_conv3x3_patch_pool(const float* in, const float* Bt, int ldb, float* out, const DirectGeom& g, int C,
                              int N, const float* zero, const EpiParams& epi, hipStream_t stream,
                              unsigned short* out_split) {
  if (g.B == 0) return 0;
  if (!(C == 16 || C == 32) || N % PT_NB != 0 || ldb != patch_kpad(C) || g.OH % 2 || g.OW % 2 ||
      g.PH != g.OH / 2 || g.PW != g.OW / 2 || g.OH != g.H || g.OW != g.W || g.pt != 1 || g.pl != 1) {
    set_error("patch conv: unsupported shape C=%d N=%d ldb=%d %dx%d", C, N, ldb, g.OH, g.OW);
    return -2;
  }
  const int tilesX = (g.OW + PT_EDGE - 1) / PT_EDGE, tilesY = (g.OH + PT_EDGE - 1) / PT_EDGE;
  const int nblkN = N / PT_NB;
  const long long blocks = (long long)g.B * tilesY * tilesX * nblkN;
  if (blocks > 0x7fffffffLL) {
    set_error("patch conv: grid too large");
    return -2;
  }
  const size_t out_bytes = out_split ? (size_t)g.B * (g.PH + 2) * (g.PW + 2) * N * 6 : (size_t)g.B * g.PH * g.PW * N * 4;
  if (C == 16 && N == 32 && out_bytes < OOB_OFF) {
    // persistent: as many workgroups as fit resident (3 per CU by LDS), each looping over tiles
    const long long slots = (long long)device_cu_count() * PP_WG_PER_CU;
    const unsigned grid = (unsigned)(blocks < slots ? blocks : slots);
    if (out_split)
      hipLaunchKernelGGL(conv3x3_patch_pool_c16_persistent<true>, dim3(grid), dim3(256), 0, stream, in, Bt, ldb,
                         reinterpret_cast<float*>(out_split), g, tilesX, tilesY, (int)blocks, zero, epi);
    else
      hipLaunchKernelGGL(conv3x3_patch_pool_c16_persistent<false>, dim3(grid), dim3(256), 0, stream, in, Bt, ldb, out,
                         g, tilesX, tilesY, (int)blocks, zero, epi);
  } else if (C == 16)
    hipLaunchKernelGGL((conv3x3_patch_pool_kernel<16>), dim3((unsigned)blocks), dim3(256), 0, stream, in, Bt, out, g,
                       N, tilesX, tilesY, nblkN, zero, epi, reinterpret_cast<bf16_bits*>(out_split));
  else
    hipLaunchKernelGGL((conv3x3_patch_pool_kernel<32>), dim3((unsigned)blocks), dim3(256), 0, stream, in, Bt, out, g,
                       N, tilesX, tilesY, nblkN, zero, epi, reinterpret_cast<bf16_bits*>(out_split));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("launch conv3x3_patch_pool: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

}  // namespace dnnhip
