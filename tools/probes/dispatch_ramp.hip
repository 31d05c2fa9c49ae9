// How fast are a grid's workgroups started?  Thread 0 of every block stamps
// the 100 MHz wall clock at entry; the block then idles `spin` x ~64 cycles
// (so residency limits show) and stamps again at exit.  Launch shapes and
// dynamic LDS are the caller's (tools/dispatch_ramp_probe.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void k_ramp(unsigned long long* st, int spin) {
  extern __shared__ float lds[];
  if (threadIdx.x == 0) st[2 * blockIdx.x] = wall_clock64();
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0) lds[0] = 1.f;
  __syncthreads();
  if (threadIdx.x == 0) st[2 * blockIdx.x + 1] = wall_clock64() + (lds[0] > 2.f);
}

extern "C" int ramp_launch(unsigned long long* st, int blocks, int threads, int lds, int spin, hipStream_t s) {
  hipLaunchKernelGGL(k_ramp, dim3(blocks), dim3(threads), lds, s, st, spin);
  return (int)hipGetLastError();
}
