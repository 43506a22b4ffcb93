// Shader-clock stamps (measurement, SURVEY.md §8(d) "re-derive the peak from the measured sclk"):
// a launch of `nwg` one-wave workgroups in which each workgroup records its 64-bit shader-clock
// counter (s_memtime), the constant 100 MHz counter (s_memrealtime), its XCD (XCC_ID) and its
// HW_ID.  Two launches on a stream bracket a region; per XCD, delta(memtime) / delta(memrealtime)
// x 100 MHz is the mean shader clock over it.  The plan can bracket one kernel of every forward
// with them (dnn_plan_clock_begin), which gives the dominant kernel's own clock.
#include <hip/hip_runtime.h>
#include "dnn_common.h"

namespace dnnhip {

__global__ void __launch_bounds__(64) clock_stamp_kernel(unsigned long long* __restrict__ out) {
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned long long r = __builtin_amdgcn_s_memrealtime();
  const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xfu;
  const unsigned hw = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
  const unsigned lane = threadIdx.x;
  if (lane < 4) {  // lanes 0-3 store the four values (vector stores)
    const unsigned long long v = lane == 0 ? t : lane == 1 ? r : lane == 2 ? (unsigned long long)xcc : hw;
    out[4 * (size_t)blockIdx.x + lane] = v;
  }
}

int launch_clock_stamp(hipStream_t s, unsigned long long* out, int nwg) {
  if (!out || nwg <= 0 || nwg > 65536) {
    set_error("clock_stamp: bad arguments (out %p, nwg %d)", (void*)out, nwg);
    return -2;
  }
  hipLaunchKernelGGL(clock_stamp_kernel, dim3(nwg), dim3(64), 0, s, out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("launch clock_stamp: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

}  // namespace dnnhip

extern "C" __attribute__((visibility("default"))) int dnn_clock_stamp(void* stream, unsigned long long* dev_out,
                                                                      int nwg) {
  return dnnhip::launch_clock_stamp(reinterpret_cast<hipStream_t>(stream), dev_out, nwg);
}
