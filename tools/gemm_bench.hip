// Standalone microbenchmark of the conv GEMM variants on the YOLOv2-tiny batch-64 shapes.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off tools/gemm_bench.hip -o tools/gemm_bench
//   ./tools/gemm_bench [iters] [shape filter]
// Times every variant with HIP events (same process, interleaved rounds, median) and checks
// 2048 sampled outputs against a float64 host dot product.
#include <hip/hip_runtime.h>
#include <algorithm>
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

__global__ void fill_kernel(float* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 16;
    x *= 0x7feb352d;
    x ^= x >> 15;
    x *= 0x846ca68b;
    x ^= x >> 16;
    p[i] = ((x >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
  }
}

struct Variant {
  std::string name;
  int bm, bn;
  std::function<void(const float*, int, const float*, int, float*, int, int, int, int, EpiParams, int, hipStream_t)>
      launch;
};

template <int BM, int BN, int BK, int WM, int WN, int MF>
Variant reg_variant(const char* nm) {
  return {nm, BM, BN,
          [](const float* A, int lda, const float* B, int ldb, float* C, int ldc, int M, int N, int K, EpiParams e,
             int grid, hipStream_t s) {
            int tilesN = (N + BN - 1) / BN;
            hipLaunchKernelGGL((gemm_f32_mfma_kernel<BM, BN, BK, WM, WN, MF>), dim3(grid), dim3(WM * WN * 64), 0, s,
                               A, lda, B, ldb, C, ldc, M, N, K, e, tilesN);
          }};
}

static float* g_slab = nullptr;  // split-K partials (allocated in main)

template <int BM, int BN, int WM, int WN, int MF, int NS, int SPLIT = 1>
Variant glds_variant(const char* nm) {
  return {nm, BM, BN,
          [](const float* A, int lda, const float* B, int ldb, float* C, int ldc, int M, int N, int K, EpiParams e,
             int grid, hipStream_t s) {
            int tilesN = (N + BN - 1) / BN;
            if (SPLIT == 1) {
              hipLaunchKernelGGL((gemm_f32_glds_kernel<BM, BN, WM, WN, MF, NS, 0>), dim3(grid), dim3(WM * WN * 64), 0,
                                 s, A, lda, B, ldb, C, ldc, M, N, K, e, tilesN, ImplicitConv{}, SplitK{0, 0, 0},
                                 BufDesc{});
            } else {
              SplitK sk{K / 32 / SPLIT, grid, (long long)M * N};
              hipLaunchKernelGGL((gemm_f32_glds_kernel<BM, BN, WM, WN, MF, NS, 0>), dim3(grid * SPLIT),
                                 dim3(WM * WN * 64), 0, s, A, lda, B, ldb, g_slab, N, M, N, K, e, tilesN,
                                 ImplicitConv{}, sk, BufDesc{});
              const int nqb = N / 4 < 256 ? N / 4 : 256, rp = 256 / nqb;
              hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(2048), dim3(256), 0, s, g_slab, SPLIT, sk.slab, C, M,
                                 N, ldc, e, nqb, rp);
            }
          }};
}

struct Shape {
  const char* name;
  int M, N, K;
};

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 10;
  const char* filt = argc > 2 ? argv[2] : "";
  std::vector<Shape> shapes = {{"conv7", 10816, 1024, 9216}, {"conv6", 10816, 1024, 4608},
                               {"conv7big", 65536, 1024, 9216}, {"conv5", 10816, 512, 2304},
                               {"conv4", 43264, 256, 1152},  {"conv3", 173056, 128, 576}};
  std::vector<Variant> vars = {
      glds_variant<128, 128, 2, 2, 32, 2>("glds 128x128 ns2"),
      glds_variant<128, 128, 2, 2, 32, 2, 2>("glds 128x128 ns2 sk2"),
      glds_variant<128, 128, 2, 2, 32, 2, 3>("glds 128x128 ns2 sk3"),
      glds_variant<128, 128, 2, 2, 32, 2, 4>("glds 128x128 ns2 sk4"),
      glds_variant<256, 128, 4, 2, 32, 2>("glds 256x128 w8 ns2"),
      glds_variant<256, 128, 4, 2, 32, 2, 3>("glds 256x128 w8 sk3"),
      glds_variant<256, 128, 4, 2, 32, 2, 4>("glds 256x128 w8 sk4"),
      glds_variant<256, 128, 4, 2, 32, 2, 8>("glds 256x128 w8 sk8"),
      glds_variant<64, 128, 2, 2, 32, 2>("glds 64x128 ns2"),
      glds_variant<64, 128, 2, 2, 32, 2, 3>("glds 64x128 ns2 sk3"),
  };
  hipStream_t st;
  CK(hipStreamCreate(&st));
  CK(hipMalloc(&g_slab, (size_t)8 * 65536 * 1024 * 4));  // up to 8 partials of the largest C
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int dev;
  hipDeviceProp_t prop;
  CK(hipGetDevice(&dev));
  CK(hipGetDeviceProperties(&prop, dev));
  printf("device %s, %d CUs, clock %d MHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate / 1000);

  for (const Shape& sh : shapes) {
    if (filt[0] && !strstr(sh.name, filt)) continue;
    const int M = sh.M, N = sh.N, K = sh.K;
    float *A, *B, *C;
    CK(hipMalloc(&A, (size_t)M * K * 4));
    CK(hipMalloc(&B, (size_t)N * K * 4));
    CK(hipMalloc(&C, (size_t)M * N * 4));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, A, (size_t)M * K, 1u);
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, B, (size_t)N * K, 2u);
    CK(hipStreamSynchronize(st));
    std::vector<float> hA((size_t)M * K), hB((size_t)N * K), hC((size_t)M * N);
    CK(hipMemcpy(hA.data(), A, hA.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hB.data(), B, hB.size() * 4, hipMemcpyDeviceToHost));
    const double flops = 2.0 * M * N * (double)K;
    EpiParams epi{nullptr, nullptr, nullptr, nullptr, 0};
    std::vector<std::vector<float>> times(vars.size());
    // correctness first
    for (size_t v = 0; v < vars.size(); ++v) {
      Variant& V = vars[v];
      int grid = ((M + V.bm - 1) / V.bm) * ((N + V.bn - 1) / V.bn);
      CK(hipMemset(C, 0, (size_t)M * N * 4));
      V.launch(A, K, B, K, C, N, M, N, K, epi, grid, st);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(st));
      CK(hipMemcpy(hC.data(), C, hC.size() * 4, hipMemcpyDeviceToHost));
      double maxerr = 0, maxref = 0;
      unsigned s = 12345;
      for (int t = 0; t < 2048; ++t) {
        s = s * 1103515245u + 12345u;
        int m = (s >> 8) % M;
        s = s * 1103515245u + 12345u;
        int n = (s >> 8) % N;
        double ref = 0;
        for (int k = 0; k < K; ++k) ref += (double)hA[(size_t)m * K + k] * hB[(size_t)n * K + k];
        maxerr = std::max(maxerr, std::fabs(ref - hC[(size_t)m * N + n]));
        maxref = std::max(maxref, std::fabs(ref));
      }
      printf("  %-22s %-6s check maxerr/maxref = %.2e %s\n", V.name.c_str(), sh.name, maxerr / maxref,
             maxerr / maxref < 1e-5 ? "ok" : "FAIL");
    }
    // interleaved timing rounds
    for (int round = 0; round < iters; ++round) {
      for (size_t v = 0; v < vars.size(); ++v) {
        Variant& V = vars[v];
        int grid = ((M + V.bm - 1) / V.bm) * ((N + V.bn - 1) / V.bn);
        V.launch(A, K, B, K, C, N, M, N, K, epi, grid, st);
        CK(hipEventRecord(e0, st));
        V.launch(A, K, B, K, C, N, M, N, K, epi, grid, st);
        V.launch(A, K, B, K, C, N, M, N, K, epi, grid, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        times[v].push_back(ms / 2);
      }
    }
    for (size_t v = 0; v < vars.size(); ++v) {
      auto t = times[v];
      std::sort(t.begin(), t.end());
      float med = t[t.size() / 2], mn = t[0];
      printf("%-6s %-22s median %8.3f ms  min %8.3f ms  %7.1f TF/s  %5.1f%% of 157.3\n", sh.name, vars[v].name.c_str(),
             med, mn, flops / med / 1e9, 100.0 * flops / med / 1e9 / 157.3);
    }
    fflush(stdout);
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
  }
  return 0;
}
