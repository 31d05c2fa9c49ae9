// Timing probe (tools/bwd_phases_probe.py): the shipped k_bwd_all with its
// PTO_STAMP phase marks compiled in.  Thread 0 of every block writes the
// 100 MHz wall clock (s_memrealtime, chip-wide) at each mark into
// g_stamps[block][slot]: slot 0 = entry, 7 = exit, 1..5 = the role's phases
// (mnist_kernels.hip).  Timing only; its own .so.
#include <hip/hip_runtime.h>
#define PTO_STAMP_SLOTS 8
#define PTO_MAX_BLOCKS 4096
__device__ unsigned long long g_stamps[PTO_MAX_BLOCKS * PTO_STAMP_SLOTS];
__device__ __forceinline__ void pto_stamp(int k) {
  if (threadIdx.x == 0 && blockIdx.x < PTO_MAX_BLOCKS) g_stamps[blockIdx.x * PTO_STAMP_SLOTS + k] = wall_clock64();
}
struct PtoEndStamp {
  __device__ PtoEndStamp() { pto_stamp(0); }
  __device__ ~PtoEndStamp() { pto_stamp(7); }
};
#define PTO_STAMP(k) pto_stamp(k)
#define PTO_STAMP_SCOPE() PtoEndStamp pto_end_stamp_
#include "bwd_roles.hip"

extern "C" __attribute__((visibility("default"))) int probe_read_stamps(unsigned long long* out, int n) {
  if (n > PTO_MAX_BLOCKS * PTO_STAMP_SLOTS) return -1;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), (size_t)n * sizeof(unsigned long long));
}
