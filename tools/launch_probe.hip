// Dependent-launch floor on MI355X: the time per kernel of a chain of N back-to-back kernels
// on one stream, eager and as one HIP graph, for kernels that do (almost) nothing -- what a
// single-frame latency plan (BASELINE config 2) pays per layer before any work.
//   hipcc -O3 --offload-arch=gfx950 tools/launch_probe.hip -o tools/launch_probe && tools/launch_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <algorithm>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

__global__ void k_empty() {}

// each workgroup writes `per_wg` floats (vector stores), so the kernel leaves dirty L2 lines
__global__ void k_write(float* p, int per_wg) {
  float* q = p + (size_t)blockIdx.x * per_wg;
  for (int i = threadIdx.x; i < per_wg; i += blockDim.x) q[i] = (float)i;
}

// reads what the previous kernel wrote (a dependent chain through memory)
__global__ void k_rw(const float* a, float* b, int per_wg) {
  const float* p = a + (size_t)blockIdx.x * per_wg;
  float* q = b + (size_t)blockIdx.x * per_wg;
  for (int i = threadIdx.x; i < per_wg; i += blockDim.x) q[i] = p[i] + 1.f;
}

struct Case {
  const char* name;
  int kind, grid, block, per_wg;
};

int main() {
  const int N = 48, REPS = 20;
  float *a = nullptr, *b = nullptr;
  CK(hipMalloc(&a, 64 << 20));
  CK(hipMalloc(&b, 64 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const Case cases[] = {
      {"empty 1 WG", 0, 1, 64, 0},
      {"empty 256 WG x 256", 0, 256, 256, 0},
      {"empty 2048 WG x 256", 0, 2048, 256, 0},
      {"write 256 WG, 4 KB each (1 MB)", 1, 256, 256, 1024},
      {"write 256 WG, 32 KB each (8 MB)", 1, 256, 256, 8192},
      {"read+write 256 WG, 4 KB each (1 MB)", 2, 256, 256, 1024},
      {"read+write 1024 WG, 4 KB each (4 MB)", 2, 1024, 256, 1024},
  };
  auto launch = [&](const Case& c, int i) {
    if (c.kind == 0)
      hipLaunchKernelGGL(k_empty, dim3(c.grid), dim3(c.block), 0, s);
    else if (c.kind == 1)
      hipLaunchKernelGGL(k_write, dim3(c.grid), dim3(c.block), 0, s, (i & 1) ? a : b, c.per_wg);
    else
      hipLaunchKernelGGL(k_rw, dim3(c.grid), dim3(c.block), 0, s, (i & 1) ? a : b, (i & 1) ? b : a, c.per_wg);
  };
  printf("%-40s %12s %12s\n", "case (chain of 48 kernels)", "eager us/k", "graph us/k");
  for (const Case& c : cases) {
    for (int i = 0; i < N; ++i) launch(c, i);
    CK(hipStreamSynchronize(s));
    std::vector<float> te, tg;
    for (int r = 0; r < REPS; ++r) {
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < N; ++i) launch(c, i);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      te.push_back(ms * 1e3f / N);
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < N; ++i) launch(c, i);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < REPS; ++r) {
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      tg.push_back(ms * 1e3f / N);
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    std::sort(te.begin(), te.end());
    std::sort(tg.begin(), tg.end());
    printf("%-40s %12.2f %12.2f\n", c.name, te[REPS / 2], tg[REPS / 2]);
  }
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
