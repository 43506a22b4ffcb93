// Cycle probe for v_mfma_f32_16x16x32_bf16 issue patterns on gfx950 (one wave per SIMD,
// 4 waves per workgroup, one workgroup per CU).  Each pattern is one asm block of 12 MFMAs,
// looped; s_memtime around the loop gives cycles per MFMA.  Operands are random bf16.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o tools/mfma_probe && tools/mfma_probe
// Patterns:
//   0  12 independent accumulators, AGPR C/D
//   1  12 independent accumulators, VGPR C/D
//   2  [5 dependent on c0 (AGPR), m0 (VGPR)] [5 dependent on c1, m1]   (x3 w1 kernel order)
//   3  [5 dep c0][5 dep c1] then m0 m1 (VGPR)
//   4  [5 dep c0, m0][5 dep c1, m1], all AGPR
//   5  12 independent, alternating AGPR / VGPR C/D
//   6  [5 dep c0][5 dep c1] interleaved c0 c1 c0 c1 ... (dependent at distance 2), then m0 m1, all AGPR
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define M(D, A, B) "v_mfma_f32_16x16x32_bf16 " D ", " A ", " B ", " D "\n\t"

template <int P, int U = 1>
__global__ void __launch_bounds__(256, 1) probe(const bf16x8* in, float* out, long long* cyc, int iters) {
  const int l = threadIdx.x;
  bf16x8 a0 = in[l], a1 = in[l + 256], a2 = in[l + 512], b0 = in[l + 768], b1 = in[l + 1024], b2 = in[l + 1280];
  f32x4 acc[12];
  for (int i = 0; i < 12; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
   for (int u = 0; u < U; ++u) {
    if constexpr (P == 0) {
      asm volatile(M("%0", "%12", "%15") M("%1", "%13", "%16") M("%2", "%14", "%17") M("%3", "%12", "%16")
                       M("%4", "%13", "%17") M("%5", "%14", "%15") M("%6", "%12", "%17") M("%7", "%13", "%15")
                           M("%8", "%14", "%16") M("%9", "%12", "%15") M("%10", "%13", "%16") M("%11", "%14", "%17")
                   : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3]), "+a"(acc[4]), "+a"(acc[5]),
                     "+a"(acc[6]), "+a"(acc[7]), "+a"(acc[8]), "+a"(acc[9]), "+a"(acc[10]), "+a"(acc[11])
                   : "v"(a0), "v"(a1), "v"(a2), "v"(b0), "v"(b1), "v"(b2));
    } else if constexpr (P == 1) {
      asm volatile(M("%0", "%12", "%15") M("%1", "%13", "%16") M("%2", "%14", "%17") M("%3", "%12", "%16")
                       M("%4", "%13", "%17") M("%5", "%14", "%15") M("%6", "%12", "%17") M("%7", "%13", "%15")
                           M("%8", "%14", "%16") M("%9", "%12", "%15") M("%10", "%13", "%16") M("%11", "%14", "%17")
                   : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
                     "+v"(acc[6]), "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11])
                   : "v"(a0), "v"(a1), "v"(a2), "v"(b0), "v"(b1), "v"(b2));
    } else if constexpr (P == 2 || P == 3 || P == 4) {
      // %0 c0, %1 m0, %2 c1, %3 m1; %4.. a2 a1 a0, %7.. b0 b1 b2
#define CH(C) M(C, "%4", "%7") M(C, "%5", "%8") M(C, "%6", "%9") M(C, "%5", "%7") M(C, "%6", "%8")
      if constexpr (P == 2)
        asm volatile(CH("%0") M("%1", "%6", "%7") CH("%2") M("%3", "%6", "%7")
                     : "+a"(acc[0]), "+v"(acc[1]), "+a"(acc[2]), "+v"(acc[3])
                     : "v"(a2), "v"(a1), "v"(a0), "v"(b0), "v"(b1), "v"(b2));
      else if constexpr (P == 3)
        asm volatile(CH("%0") CH("%2") M("%1", "%6", "%7") M("%3", "%6", "%7")
                     : "+a"(acc[0]), "+v"(acc[1]), "+a"(acc[2]), "+v"(acc[3])
                     : "v"(a2), "v"(a1), "v"(a0), "v"(b0), "v"(b1), "v"(b2));
      else
        asm volatile(CH("%0") M("%1", "%6", "%7") CH("%2") M("%3", "%6", "%7")
                     : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3])
                     : "v"(a2), "v"(a1), "v"(a0), "v"(b0), "v"(b1), "v"(b2));
#undef CH
    } else if constexpr (P == 5) {
      asm volatile(M("%0", "%12", "%15") M("%1", "%13", "%16") M("%2", "%14", "%17") M("%3", "%12", "%16")
                       M("%4", "%13", "%17") M("%5", "%14", "%15") M("%6", "%12", "%17") M("%7", "%13", "%15")
                           M("%8", "%14", "%16") M("%9", "%12", "%15") M("%10", "%13", "%16") M("%11", "%14", "%17")
                   : "+a"(acc[0]), "+v"(acc[1]), "+a"(acc[2]), "+v"(acc[3]), "+a"(acc[4]), "+v"(acc[5]),
                     "+a"(acc[6]), "+v"(acc[7]), "+a"(acc[8]), "+v"(acc[9]), "+a"(acc[10]), "+v"(acc[11])
                   : "v"(a0), "v"(a1), "v"(a2), "v"(b0), "v"(b1), "v"(b2));
    } else {
      asm volatile(M("%0", "%4", "%7") M("%2", "%4", "%7") M("%0", "%5", "%8") M("%2", "%5", "%8")
                       M("%0", "%6", "%9") M("%2", "%6", "%9") M("%0", "%5", "%7") M("%2", "%5", "%7")
                           M("%0", "%6", "%8") M("%2", "%6", "%8") M("%1", "%6", "%7") M("%3", "%6", "%7")
                   : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3])
                   : "v"(a2), "v"(a1), "v"(a0), "v"(b0), "v"(b1), "v"(b2));
    }
   }
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int i = 0; i < 12; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + l] = s;
  if (l % 64 == 0) cyc[blockIdx.x * 4 + l / 64] = t1 - t0, cyc[gridDim.x * 4 + blockIdx.x * 4 + l / 64] = r1 - r0;
}

template <int P, int U = 1>
double run(const bf16x8* in, float* out, long long* cyc, int blocks, int iters) {
  iters /= U;
  hipLaunchKernelGGL((probe<P, U>), dim3(blocks), dim3(256), 0, 0, in, out, cyc, iters);
  hipDeviceSynchronize();
  hipLaunchKernelGGL((probe<P, U>), dim3(blocks), dim3(256), 0, 0, in, out, cyc, iters);
  hipDeviceSynchronize();
  std::vector<long long> h(blocks * 8);
  hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  printf("   [clock %.3f GHz] ", (double)h[0] / h[blocks * 4] * 0.1);
  h.resize(blocks * 4);
  std::sort(h.begin(), h.end());
  return (double)h[h.size() / 2] / iters / U / 12;
}

int main() {
  const int blocks = 256, iters = 20000;
  std::vector<unsigned short> hin(1536 * 8);
  srand(1);
  for (auto& v : hin) v = (unsigned short)(0x3c00 + (rand() & 0x3ff) + ((rand() & 1) << 15));
  bf16x8* in;
  float* out;
  long long* cyc;
  hipMalloc(&in, hin.size() * 2);
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&cyc, blocks * 8 * 8);
  hipMemcpy(in, hin.data(), hin.size() * 2, hipMemcpyHostToDevice);
  // s_memtime counts at the shader clock (MI355X_MICROARCH: tick = shader cycle)
  printf("pattern cycles_per_mfma\n");
  printf("0 indep AGPR            %.2f\n", run<0>(in, out, cyc, blocks, iters));
  printf("1 indep VGPR            %.2f\n", run<1>(in, out, cyc, blocks, iters));
  printf("2 chain5A+V x2 (w1)     %.2f\n", run<2>(in, out, cyc, blocks, iters));
  printf("3 chain5A x2 then 2V    %.2f\n", run<3>(in, out, cyc, blocks, iters));
  printf("4 chain5A+A x2          %.2f\n", run<4>(in, out, cyc, blocks, iters));
  printf("5 indep alt A/V         %.2f\n", run<5>(in, out, cyc, blocks, iters));
  printf("6 chains interleaved A  %.2f\n", run<6>(in, out, cyc, blocks, iters));
  printf("0 indep AGPR x8 unroll  %.2f\n", run<0, 8>(in, out, cyc, blocks, iters));
  printf("2 w1 order x8 unroll    %.2f\n", run<2, 8>(in, out, cyc, blocks, iters));
  // s_memtime vs s_memrealtime (100 MHz): the clock the loop ran at
  printf("(clock check follows)\n");
  hipFree(in);
  hipFree(out);
  hipFree(cyc);
  return 0;
}
