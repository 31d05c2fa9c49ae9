// Timing probe (tools/exchange_phases_probe.py): the shipped MNIST kernels
// with their PTO_STAMP marks compiled in, so the overlapped multi-GPU
// step's F12 launch (conv role + fc role + conv blocks) reports per-block
// phase times.  Thread 0 of every block writes the 100 MHz wall clock at
// each mark into g_stamps[block][slot]: 0 entry, 7 exit; conv role 1 =
// barrier 0 passed, 2 = SGD stores issued, 3 = published, 4 = barrier 1
// passed; conv blocks 5 = conv-role wait over, 1 = weights staged, 2 =
// conv1 done, 3 = conv2 done.  Timing only; its own .so.
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
#include "../../pytorch_operator_1_amd/csrc/kernels/mnist_kernels.hip"

extern "C" long long pto_ar_timeout_ticks() { return 500LL * 100000LL; }

extern "C" __attribute__((visibility("default"))) int probe_read_stamps(unsigned long long* out, int n) {
  if (n > PTO_MAX_BLOCKS * PTO_STAMP_SLOTS) return -1;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), (size_t)n * sizeof(unsigned long long));
}
