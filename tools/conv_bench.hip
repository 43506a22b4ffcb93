// Conv-layer microbenchmark: implicit-GEMM (+ fused 2x2 pool) variants against the explicit
// im2col + GEMM + maxpool path of the library (bit-exact reference: same MFMA family and K
// permutation), on the YOLOv2-tiny batch-64 layer shapes.
//   make -C dnn-inference-engine_amd/csrc && hipcc -O3 -std=c++17 --offload-arch=gfx950 -c \
//     -ffp-contract=off tools/conv_bench.hip dnn-inference-engine_amd/csrc/build/{kernels,conv_direct,plan,legacy}.o \
//     -o tools/conv_bench
//   ./tools/conv_bench [iters] [layer filter]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>
#include "../dnn-inference-engine_amd/csrc/gemm_f32.h"

using namespace dnnhip;

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e = (x);                                                                       \
    if (e != hipSuccess) {                                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));        \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)
#define RC(x)                                                                                 \
  do {                                                                                        \
    if ((x) != 0) {                                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, last_error());                \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)

__global__ void fill_kernel(float* p, size_t n, unsigned seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 16;
    x *= 0x7feb352d;
    x ^= x >> 15;
    x *= 0x846ca68b;
    x ^= x >> 16;
    p[i] = (((x >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f) * scale;
  }
}

struct Layer {
  const char* name;
  int B, H, W, C, N;
  bool pool;
};

typedef std::function<void(const float* in, const ImplicitConv& ic, const float* Bt, int Kpad, float* out, int M,
                           int N, const EpiParams& epi, hipStream_t s)>
    ImplFn;

struct Variant {
  std::string name;
  int bm, bn;
  ImplFn fn;
};

template <int BM, int BN, int WM, int WN, int MF, int NS>
Variant impl(const char* nm) {
  return {nm, BM, BN,
          [](const float* in, const ImplicitConv& ic, const float* Bt, int Kpad, float* out, int M, int N,
             const EpiParams& epi, hipStream_t s) {
            const int tilesN = (N + BN - 1) / BN;
            const int grid = ((M + BM - 1) / BM) * tilesN;
            if (ic.pool)
              hipLaunchKernelGGL((gemm_f32_glds_kernel<BM, BN, WM, WN, MF, NS, GEMM_IMPLICIT_POOL>), dim3(grid),
                                 dim3(WM * WN * 64), 0, s, in, 0, Bt, Kpad, out, N, M, N, Kpad, epi, tilesN, ic,
                                 SplitK{0, 0, 0}, BufDesc{});
            else
              hipLaunchKernelGGL((gemm_f32_glds_kernel<BM, BN, WM, WN, MF, NS, GEMM_IMPLICIT>), dim3(grid),
                                 dim3(WM * WN * 64), 0, s, in, 0, Bt, Kpad, out, N, M, N, Kpad, epi, tilesN, ic,
                                 SplitK{0, 0, 0}, BufDesc{});
          }};
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 10;
  const char* filt = argc > 2 ? argv[2] : "";
  std::vector<Layer> layers = {{"conv1", 64, 208, 208, 16, 32, true},   {"conv2", 64, 104, 104, 32, 64, true},
                               {"conv3", 64, 52, 52, 64, 128, true},    {"conv4", 64, 26, 26, 128, 256, true},
                               {"conv5", 64, 13, 13, 256, 512, false},  {"conv6", 64, 13, 13, 512, 1024, false},
                               {"conv7", 64, 13, 13, 1024, 1024, false}};
  // variants grouped by MFMA family (N <= 32: 16x16x4, else 32x32x2)
  std::vector<Variant> small = {
      impl<128, 32, 4, 1, 16, 3>("i128x32 w4 ns3"), impl<128, 32, 4, 1, 16, 2>("i128x32 w4 ns2"),
      impl<256, 32, 4, 1, 16, 2>("i256x32 w4 ns2"),
      impl<64, 32, 4, 1, 16, 2>("i64x32 w4 ns2")};
  std::vector<Variant> mid = {
      impl<128, 64, 2, 2, 32, 3>("i128x64 ns3"), impl<128, 64, 2, 2, 32, 2>("i128x64 ns2"),
      impl<256, 64, 4, 2, 32, 2>("i256x64 w8 ns2"), impl<64, 64, 2, 2, 32, 2>("i64x64 ns2"),
      impl<128, 64, 4, 1, 32, 2>("i128x64 w4x1 ns2")};
  std::vector<Variant> wide = {impl<64, 128, 2, 2, 32, 3>("i64x128 ns3"), impl<64, 128, 2, 2, 32, 2>("i64x128 ns2"),
                               impl<128, 128, 2, 2, 32, 2>("i128x128 ns2"),
                               impl<128, 128, 2, 2, 32, 3>("i128x128 ns3"),
                               impl<128, 64, 2, 2, 32, 3>("i128x64 ns3")};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  for (const Layer& L : layers) {
    if (filt[0] && !strstr(L.name, filt)) continue;
    const int K = 9 * L.C;
    const int OH = L.H, OW = L.W, PH = L.pool ? (L.H + 1) / 2 : OH, PW = L.pool ? (L.W + 1) / 2 : OW;
    const long long Mexp = (long long)L.B * OH * OW;
    const int Mimp = L.pool ? 4 * L.B * PH * PW : (int)Mexp;
    const int N = L.N;
    // reference config (explicit path) and Kpad/Npad common to both
    const int cfg = choose_gemm_cfg(Mexp, N, K);
    const int Kpad = (K + 31) / 32 * 32, Npad = (N + 127) / 128 * 128;
    float *in, *w, *bt, *col, *conv, *ref, *out, *epi_buf, *zero;
    const size_t n_in = (size_t)L.B * L.H * L.W * L.C, n_out = (size_t)L.B * PH * PW * N;
    CK(hipMalloc(&in, n_in * 4));
    CK(hipMalloc(&w, (size_t)K * N * 4));
    CK(hipMalloc(&bt, (size_t)Npad * Kpad * 4));
    CK(hipMalloc(&col, (size_t)Mexp * Kpad * 4));
    CK(hipMalloc(&conv, (size_t)Mexp * N * 4));
    CK(hipMalloc(&ref, n_out * 4));
    CK(hipMalloc(&out, n_out * 4));
    CK(hipMalloc(&epi_buf, 4 * Npad * 4));
    CK(hipMalloc(&zero, 256));
    CK(hipMemset(zero, 0, 256));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, in, n_in, 1u, 1.0f);
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, w, (size_t)K * N, 2u, sqrtf(6.0f / K));
    hipLaunchKernelGGL(fill_kernel, dim3(64), dim3(256), 0, st, epi_buf, (size_t)Npad, 3u, 0.1f);  // bias
    std::vector<float> ones(3 * Npad, 1.0f);
    for (int i = 0; i < Npad; ++i) ones[i] = 0.02f * (i % 7);  // mean
    CK(hipMemcpy(epi_buf + Npad, ones.data(), 3 * Npad * 4, hipMemcpyHostToDevice));
    RC(launch_pack_weights(w, bt, K, N, Kpad, Npad, 0, 3, 3, L.C, st));
    EpiParams epi{epi_buf, epi_buf + Npad, epi_buf + 2 * Npad, epi_buf + 3 * Npad, EPI_BIAS | EPI_BN | EPI_LEAKY_F64};
    // explicit reference
    ConvGeom g{L.B, L.H, L.W, L.C, OH, OW, 3, 3, 1, 1, 1, 1, K, Kpad};
    auto explicit_path = [&]() {
      RC(launch_im2col(in, col, g, st));
      RC(launch_gemm(cfg, col, Kpad, bt, Kpad, L.pool ? conv : ref, N, Mexp, N, Kpad, epi, st));
      if (L.pool) {
        PoolGeom pg{L.B, OH, OW, N, PH, PW, 2, 2, 2, 2, 0, 0, 0};
        RC(launch_maxpool(conv, ref, pg, st));
      }
    };
    explicit_path();
    CK(hipStreamSynchronize(st));
    std::vector<float> href(n_out), hout(n_out);
    CK(hipMemcpy(href.data(), ref, n_out * 4, hipMemcpyDeviceToHost));
    ImplicitConv ic{zero, L.H, L.W, L.C, OH, OW, PH, PW, 3, 3, 1, 1, 1, 1, L.pool ? 1 : 0};
    std::vector<Variant>& vars = N <= 32 ? small : (N <= 64 ? mid : wide);
    const double flops = 2.0 * Mexp * N * K;
    // explicit timing
    std::vector<float> t_exp;
    std::vector<std::vector<float>> t(vars.size());
    for (size_t v = 0; v < vars.size(); ++v) {
      CK(hipMemset(out, 0, n_out * 4));
      vars[v].fn(in, ic, bt, Kpad, out, Mimp, N, epi, st);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(st));
      CK(hipMemcpy(hout.data(), out, n_out * 4, hipMemcpyDeviceToHost));
      size_t diff = 0;
      for (size_t i = 0; i < n_out; ++i) diff += memcmp(&hout[i], &href[i], 4) != 0;
      printf("  %-6s %-20s bit-exact vs explicit: %s (%zu diffs)\n", L.name, vars[v].name.c_str(),
             diff ? "NO" : "yes", diff);
    }
    for (int r = 0; r < iters; ++r) {
      CK(hipEventRecord(e0, st));
      explicit_path();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t_exp.push_back(ms);
      for (size_t v = 0; v < vars.size(); ++v) {
        vars[v].fn(in, ic, bt, Kpad, out, Mimp, N, epi, st);
        CK(hipEventRecord(e0, st));
        vars[v].fn(in, ic, bt, Kpad, out, Mimp, N, epi, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[v].push_back(ms);
      }
    }
    auto med = [](std::vector<float> x) {
      std::sort(x.begin(), x.end());
      return x[x.size() / 2];
    };
    printf("%-6s %-20s %8.3f ms %7.1f TF/s  (im2col+gemm%s)\n", L.name, "explicit", med(t_exp),
           flops / med(t_exp) / 1e9, L.pool ? "+pool" : "");
    for (size_t v = 0; v < vars.size(); ++v)
      printf("%-6s %-20s %8.3f ms %7.1f TF/s  %5.1f%% of 157.3\n", L.name, vars[v].name.c_str(), med(t[v]),
             flops / med(t[v]) / 1e9, 100.0 * flops / med(t[v]) / 1e9 / 157.3);
    fflush(stdout);
    CK(hipFree(in));
    CK(hipFree(w));
    CK(hipFree(bt));
    CK(hipFree(col));
    CK(hipFree(conv));
    CK(hipFree(ref));
    CK(hipFree(out));
    CK(hipFree(epi_buf));
    CK(hipFree(zero));
  }
  return 0;
}
