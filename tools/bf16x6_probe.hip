// Probe: accuracy of an fp32 GEMM formed from three-way bf16 splits on the bf16 MFMA
// (x = x0 + x1 + x2 exactly; the six products with i + j <= 2) against the fp32 MFMA and a
// float64 reference, at the K of YOLOv2-tiny's layers.  Standalone: hipcc -O3
// --offload-arch=gfx950 tools/bf16x6_probe.hip -o /tmp/bf16x6_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ inline void split3(const float* x, bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 a = (__bf16)x[e];
    const float r = x[e] - (float)a;
    const __bf16 b = (__bf16)r;
    const float r2 = r - (float)b;
    h[e] = a;
    m[e] = b;
    l[e] = (__bf16)r2;
  }
}

// one wave per 32x32 tile; A [M][K], B [N][K] row-major; variant 0: one accumulator, large
// terms first; 1: one accumulator, small terms first; 2: correction terms in a second
// accumulator added at the end
__global__ void emu_kernel(const float* A, const float* B, float* C, int M, int N, int K, int variant) {
  const int lane = threadIdx.x, tm = blockIdx.x, tn = blockIdx.y;
  const int r = lane & 31, kh = lane >> 5;
  const float* a = A + (size_t)(tm * 32 + r) * K;
  const float* b = B + (size_t)(tn * 32 + r) * K;
  f32x16 acc = {}, acc2 = {};
  for (int k = 0; k < K; k += 16) {
    float xa[8], xb[8];
    for (int e = 0; e < 8; ++e) {
      xa[e] = a[k + 8 * kh + e];
      xb[e] = b[k + 8 * kh + e];
    }
    bf16x8 a0, a1, a2, b0, b1, b2;
    split3(xa, a0, a1, a2);
    split3(xb, b0, b1, b2);
    if (variant == 0) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc, 0, 0, 0);
    } else if (variant == 1) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc, 0, 0, 0);
    } else {
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc2, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc, 0, 0, 0);
    }
  }
  for (int q = 0; q < 16; ++q) {
    const int row = (q & 3) + 8 * (q >> 2) + 4 * kh;
    C[(size_t)(tm * 32 + row) * N + tn * 32 + r] = variant == 2 ? acc[q] + acc2[q] : acc[q];
  }
}

__global__ void f32_kernel(const float* A, const float* B, float* C, int M, int N, int K) {
  const int lane = threadIdx.x, tm = blockIdx.x, tn = blockIdx.y;
  const int r = lane & 31, kh = lane >> 5;
  const float* a = A + (size_t)(tm * 32 + r) * K;
  const float* b = B + (size_t)(tn * 32 + r) * K;
  f32x16 acc = {};
  for (int k = 0; k < K; k += 2) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k + kh], b[k + kh], acc, 0, 0, 0);
  for (int q = 0; q < 16; ++q) {
    const int row = (q & 3) + 8 * (q >> 2) + 4 * kh;
    C[(size_t)(tm * 32 + row) * N + tn * 32 + r] = acc[q];
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e_)); exit(1); } } while (0)

int main() {
  const int Ks[] = {288, 2304, 9216};
  const int M = 128, N = 128;
  std::mt19937 rng(7);
  for (int K : Ks) {
    for (int dist = 0; dist < 2; ++dist) {  // 0: normal activations/weights; 1: post-leaky (>= -0.1x) acts
      std::normal_distribution<float> nd(0.f, 1.f);
      std::vector<float> A((size_t)M * K), B((size_t)N * K);
      for (auto& v : A) { v = nd(rng); if (dist == 1 && v < 0) v *= 0.1f; }
      for (auto& v : B) v = nd(rng) * 0.05f;
      std::vector<double> ref((size_t)M * N), mag((size_t)M * N);
      std::vector<float> seq((size_t)M * N);
      for (int m = 0; m < M; ++m)
        for (int n = 0; n < N; ++n) {
          double s = 0, g = 0;
          float f = 0.f;
          for (int k = 0; k < K; ++k) {
            const double p = (double)A[(size_t)m * K + k] * B[(size_t)n * K + k];
            s += p;
            g += fabs(p);
            f = fmaf(A[(size_t)m * K + k], B[(size_t)n * K + k], f);
          }
          ref[(size_t)m * N + n] = s;
          mag[(size_t)m * N + n] = g;
          seq[(size_t)m * N + n] = f;
        }
      float *dA, *dB, *dC;
      CK(hipMalloc(&dA, A.size() * 4));
      CK(hipMalloc(&dB, B.size() * 4));
      CK(hipMalloc(&dC, (size_t)M * N * 4));
      CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
      std::vector<float> C((size_t)M * N);
      auto report = [&](const char* name, const std::vector<float>& c) {
        double mx = 0, mr = 0, rms = 0;
        for (size_t i = 0; i < c.size(); ++i) {
          const double e = fabs((double)c[i] - ref[i]);
          mx = fmax(mx, e / mag[i]);
          mr = fmax(mr, e / fmax(fabs(ref[i]), 1e-30));
          rms += (e / mag[i]) * (e / mag[i]);
        }
        printf("K=%5d dist=%d %-14s max|e|/sum|ab| %.3e  rms %.3e  max rel %.3e\n", K, dist, name, mx,
               sqrt(rms / c.size()), mr);
      };
      report("cpu fp32 fma", seq);
      hipLaunchKernelGGL(f32_kernel, dim3(M / 32, N / 32), dim3(64), 0, 0, dA, dB, dC, M, N, K);
      CK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
      report("mfma f32", C);
      const char* vn[] = {"bf16x6 big1st", "bf16x6 sml1st", "bf16x6 2acc"};
      for (int v = 0; v < 3; ++v) {
        hipLaunchKernelGGL(emu_kernel, dim3(M / 32, N / 32), dim3(64), 0, 0, dA, dB, dC, M, N, K, v);
        CK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
        report(vn[v], C);
      }
      CK(hipFree(dA));
      CK(hipFree(dB));
      CK(hipFree(dC));
    }
  }
  return 0;
}
