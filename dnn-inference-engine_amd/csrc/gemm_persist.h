// Persistent implicit-GEMM for the short-K fp32 conv layers (used for conv2 of YOLOv2-tiny at
// batch 64, 9 K-steps per tile: 0.236 -> 0.228 ms; on conv3's 64x128 tiles the static tile
// split lost to the hardware's dynamic one, 0.214 -> 0.224), device code only.
//
// gemm_f32_glds_kernel runs one tile per workgroup: every tile pays its row decode, the
// first stages' DMA latency and its epilogue with nothing of its own in flight, and the
// tiles of a round start together (~2.8 K-steps of fixed cost per tile, 23 %
// of conv2's).  Here each workgroup walks a list of tiles and the LDS-DMA ring runs straight
// across tile boundaries: the next tile's first stages are issued during the current tile's
// last K-steps and land while its epilogue (pool, bias/BN/leaky, stores) runs.
//
// Same MFMA family, K order, fragment reads and epilogue as gemm_f32_glds_kernel (buffer-
// descriptor DMA, one tap per K-step, C % 32 == 0), so every output bit is the same.
//
// Counted waits across tile boundaries: the epilogue issues exactly E buffer stores per wave
// (out-of-range rows go to OOB_OFF, which the hardware drops), so when the stage being waited
// for was issued before the last epilogue, E more operations may still be outstanding:
// vmcnt(later stages * LPS + E).  Epilogue parameters of every N tile live in registers
// (loaded once), so the epilogue issues no loads.
//
// Tile order: the 8 XCDs each own a contiguous range of tiles (as xcd_tile), walked by the
// workgroups on that XCD with stride = their count, so concurrent workgroups of an XCD work on
// neighbouring tiles (shared A rows and weight panels in its L2).
#pragma once
#include "gemm_f32.h"

namespace dnnhip {

template <int LPS, int E, int NS>
__device__ __forceinline__ void persist_wait(int later, bool stores_after) {
  static_assert(NS <= 4, "ring depth");
  if (stores_after) {
    if (NS >= 4 && later >= 2)
      wait_vmcnt<(NS >= 4 ? 2 * LPS + E : 0)>();
    else if (NS >= 3 && later >= 1)
      wait_vmcnt<(NS >= 3 ? LPS + E : 0)>();
    else
      wait_vmcnt<E>();
  } else {
    if (NS >= 4 && later >= 2)
      wait_vmcnt<(NS >= 4 ? 2 * LPS : 0)>();
    else if (NS >= 3 && later >= 1)
      wait_vmcnt<(NS >= 3 ? LPS : 0)>();
    else
      wait_vmcnt<0>();
  }
}

// MODE 1: implicit conv; MODE 2: implicit conv + 2x2/s2 pool (rows pool-window-major).
// NTN: N tiles whose epilogue parameters a lane holds (tilesN <= NTN).
template <int BM, int BN, int WM, int WN, int MF, int NS, int MODE, int NTN>
__global__ void __launch_bounds__(WM* WN * 64)
gemm_f32_persist_kernel(const float* __restrict__ Bt, int ldb, float* __restrict__ C, int ldc, int M, int N, int K,
                        EpiParams epi, int tilesN, int ntiles, ImplicitConv ic, BufDesc bd, unsigned out_bytes) {
  typedef Mfma<MF> MM;
  typedef typename MM::acc_t acc_t;
  constexpr int BK = 32;
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / MF, TN = WTN / MF;
  constexpr int A_CH = BM / 8, B_CH = BN / 8;
  constexpr int LPSA = A_CH / NW, LPSB = B_CH / NW, LPS = LPSA + LPSB;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int Q = MM::REGS / 4;
  constexpr int E = MODE == 2 ? TM * TN * Q : TM * TN * MM::REGS;  // stores per wave per tile
  static_assert(A_CH % NW == 0 && B_CH % NW == 0, "chunks must split evenly over the waves");
  static_assert(NS >= 2 && NS <= 4, "ring depth");
  static_assert((NS - 2) * LPS + E <= 63, "vmcnt range");
  static_assert(MODE == 1 || MODE == 2, "implicit modes only");

  __shared__ __attribute__((aligned(1024))) float smem[NS * STAGE];

  const int lane = threadIdx.x & 63;
  const int wid = wave_uniform(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;

  // this workgroup's tiles: tstart + slot + ord * nslot, ord < nmine
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
  const int q8 = ntiles >> 3, r8 = ntiles & 7;
  const int tstart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int tlen = q8 + (xcd < r8 ? 1 : 0);
  const int nmine = slot < tlen ? (tlen - slot + nslot - 1) / nslot : 0;
  if (nmine == 0) return;
  const int nk = K / BK;
  const int total = nmine * nk;

  // epilogue parameters of every N tile (epi arrays are Npad = tilesN * BN long)
  const int oc = MM::out_col(lane);
  float pb[NTN][TN], pm[NTN][TN], ps[NTN][TN], pg[NTN][TN];
#pragma unroll
  for (int t = 0; t < NTN; ++t)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = t * BN + wn * WTN + j * MF + oc;
      const bool ok = t < tilesN;
      pb[t][j] = (ok && (epi.flags & EPI_BIAS)) ? epi.bias[n] : 0.f;
      pm[t][j] = (ok && (epi.flags & (EPI_BN | EPI_BN_AB))) ? epi.mean[n] : 0.f;
      ps[t][j] = (ok && (epi.flags & (EPI_BN | EPI_BN_AB))) ? epi.sq[n] : 1.f;
      pg[t][j] = (ok && (epi.flags & EPI_BN)) ? epi.gamma[n] : 1.f;
    }
  __builtin_amdgcn_s_waitcnt(0);  // parameters in registers before any DMA is counted

  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)bd.a, 0, (int)bd.a_bytes, 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, (int)bd.b_bytes, 0x00020000);
  const auto rsC = out_rsrc(C, out_bytes);

  // ---- issue side: per-lane DMA sources of the tile being issued + the uniform tap cursor
  int it = 0, ik = 0;
  unsigned voA[LPSA], voB[LPSB];
  int maskA[LPSA];
  int cb = 0, tapb = 0, dyb = 0, dxb = 0, dyn = 0, dxn = 0;
  auto setup_issue = [&](int ord) {
    const int tile = tstart + slot + ord * nslot;
    const int tm_ = tile / tilesN, tn_ = tile - (tile / tilesN) * tilesN;
    const int m0 = tm_ * BM, n0 = tn_ * BN;
#pragma unroll
    for (int i = 0; i < LPSA; ++i) {
      const int r = 8 * (wid + i * NW) + (lane >> 3);
      const int ls = (lane & 7) ^ ((r >> 1) & 7);
      int b, iy0, ix0;
      maskA[i] = implicit_row<MODE>(ic, m0 + r, M, b, iy0, ix0);
      voA[i] = (unsigned)(((((long long)b * ic.H + iy0) * ic.W + ix0 + ic.W + 1) * ic.C + 4 * ls) * 4);
    }
#pragma unroll
    for (int j = 0; j < LPSB; ++j) {
      const int r = 8 * (wid + j * NW) + (lane >> 3);
      const int ls = (lane & 7) ^ ((r >> 1) & 7);
      voB[j] = (unsigned)(((size_t)(n0 + r) * ldb + 4 * ls) * 4);
    }
    cb = 0;
    tapb = 0;
    dyb = 0;
    dxb = 0;
    dyn = ic.kw == 1 ? 1 : 0;
    dxn = ic.kw == 1 ? 0 : 1;
  };
  auto issue = [&](int stage) {
    float* base = smem + stage * STAGE;
    const unsigned koff = (unsigned)(ik * BK * 4);
    const unsigned soffA = (unsigned)((((long long)dyb * ic.W + dxb) * ic.C + cb) * 4);
#pragma unroll
    for (int i = 0; i < LPSA; ++i)
      lds_dma16_buf(rsA, ((maskA[i] >> tapb) & 1) ? voA[i] : OOB_OFF, soffA, base + (wid + i * NW) * 256);
#pragma unroll
    for (int j = 0; j < LPSB; ++j) lds_dma16_buf(rsB, voB[j], koff, base + (A_CH + wid + j * NW) * 256);
    cb += BK;  // one tap per K-step (C % 32 == 0)
    if (cb >= ic.C) {
      cb = 0;
      ++tapb;
      dyb = dyn;
      dxb = dxn;
      if (dxn + 1 == ic.kw) {
        dxn = 0;
        ++dyn;
      } else {
        ++dxn;
      }
    }
    if (++ik == nk) {
      ik = 0;
      if (++it < nmine) setup_issue(it);
    }
  };

  acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < MM::REGS; ++r) acc[i][j][r] = 0.f;

  const int fr = MM::frag_row(lane), fp = MM::frag_part(lane);
  const int sw = (fr >> 1) & 7;
  constexpr int NG = BK / MM::KG;
  int kofs[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) kofs[g] = 4 * ((g * MM::PARTS + fp) ^ sw);
  const int a_row = (wm * WTM + fr) * BK;
  const int b_row = BM * BK + (wn * WTN + fr) * BK;

  setup_issue(0);
  int issued = 0;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (issued < total) {
      issue(s);
      ++issued;
    }

  const int nwin = M >> 2;
  const bool ragged = ((ic.OH | ic.OW) & 1) != 0;
  int ct = 0, ck = 0, stage = 0;
  int epi_mark = 0;  // stages g < epi_mark were issued before the last epilogue's stores
  for (int g = 0; g < total; ++g) {
    const int ahead = issued - g - 1;
    persist_wait<LPS, E, NS>(ahead < NS - 2 ? ahead : NS - 2, g < epi_mark);
    raw_barrier();
    if (issued < total) {
      int ns = stage + NS - 1;
      ns = ns >= NS ? ns - NS : ns;
      issue(ns);
      ++issued;
    }
    const float* S = smem + stage * STAGE;
#pragma unroll
    for (int gg = 0; gg < NG; ++gg) {
      f32x4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f32x4*>(S + a_row + i * MF * BK + kofs[gg]);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const f32x4*>(S + b_row + j * MF * BK + kofs[gg]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = MM::op(af[i][s], bf[j][s], acc[i][j]);
    }
    wait_lgkm0();
    stage = stage + 1 == NS ? 0 : stage + 1;
    if (++ck < nk) continue;

    // ---- epilogue of tile ct: exactly E buffer stores per wave
    const int tile = tstart + slot + ct * nslot;
    const int tm_ = tile / tilesN, tn_ = tile - (tile / tilesN) * tilesN;
    const int m0 = tm_ * BM, n0 = tn_ * BN;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float qb = pb[0][j], qm = pm[0][j], qs = ps[0][j], qg = pg[0][j];
#pragma unroll
      for (int t = 1; t < NTN; ++t)
        if (tn_ == t) {
          qb = pb[t][j];
          qm = pm[t][j];
          qs = ps[t][j];
          qg = pg[t][j];
        }
      const int n = n0 + wn * WTN + j * MF + oc;
      const bool nok = n < N;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if constexpr (MODE == 2) {
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            const int win = (m0 + wm * WTM + i * MF + MM::out_row(lane, 4 * q)) >> 2;
            f32x4 v = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
            if (ragged) {
              const int t1 = div_magic(win, ic.mag_pw, ic.sh_pw);
              const int px = win - t1 * ic.PW, py = t1 - div_magic(t1, ic.mag_ph, ic.sh_ph) * ic.PH;
              const bool x1 = 2 * px + 1 < ic.OW, y1 = 2 * py + 1 < ic.OH;
              if (!x1) v[1] = v[0];
              if (!y1) v[2] = v[0];
              if (!(x1 && y1)) v[3] = v[0];
            }
            const unsigned off = (nok && win < nwin) ? (unsigned)(((size_t)win * ldc + n) * 4) : OOB_OFF;
            store4(rsC, off, pool_then_epilogue(v, qb, qm, qs, qg, epi.flags));
          }
        } else {
#pragma unroll
          for (int r = 0; r < MM::REGS; ++r) {
            const int m = m0 + wm * WTM + i * MF + MM::out_row(lane, r);
            const unsigned off = (nok && m < M) ? (unsigned)(((size_t)m * ldc + n) * 4) : OOB_OFF;
            store4(rsC, off, apply_epilogue(acc[i][j][r], qb, qm, qs, qg, epi.flags));
          }
        }
      }
    }
    epi_mark = issued;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < MM::REGS; ++r) acc[i][j][r] = 0.f;
    ck = 0;
    ++ct;
  }
  // every issued DMA was waited for (g = total - 1 waited with no later stage); the last
  // epilogue's stores drain before the wave ends
}

}  // namespace dnnhip
