// Generic fp32 kernels shared by the fused trainer and the nn.Module path:
//   * multi-tensor fused SGD (momentum, weight decay, nesterov, grad scale,
//     grad zeroing) — one launch for every parameter tensor (K8+K10 of
//     SURVEY §2.9, incl. the DDP 1/world scale of K9),
//   * row-wise log_softmax forward/backward and fused cross-entropy
//     (log_softmax + NLL, forward and dlogits in one pass) (K7).
#include "mfma_f32.h"
#include "sgd_f32.h"

struct SgdTensor {
  float* p;
  float* g;
  float* m;
  long long n;
};

namespace {

constexpr int SGD_CHUNK = 256 * 4;  // elements per block (one float4 per thread: max parallelism)

__global__ __launch_bounds__(256) void k_sgd_multi(const SgdTensor* __restrict__ ts,
                                                   const int* __restrict__ block_start, int ntensors,
                                                   const float* __restrict__ lr_ptr, float lr, float mom, float wd,
                                                   float gscale, int nesterov, int zero_grad,
                                                   long long* __restrict__ bidx, long long nbatches) {
  // The optimizer is the last launch of a training step: it also advances
  // the device-side batch cursor read by the next step's kernels.
  if (bidx && blockIdx.x == 0 && threadIdx.x == 0) *bidx = (*bidx + 1) % nbatches;
  // locate the tensor of this block (ntensors is small; binary search)
  int lo = 0, hi = ntensors - 1;
  const int bid = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (block_start[mid] <= bid) lo = mid; else hi = mid - 1;
  }
  const SgdTensor t = ts[lo];
  if (lr_ptr) lr = *lr_ptr;
  const long long base = (long long)(bid - block_start[lo]) * SGD_CHUNK;
  const bool vec = ((((uintptr_t)t.p) | ((uintptr_t)t.g) | ((uintptr_t)t.m)) & 15) == 0;
  {
    const long long i = base + (long long)threadIdx.x * 4;
    if (i >= t.n) return;
    if (vec && i + 3 < t.n) {
      float4 p = *reinterpret_cast<float4*>(t.p + i);
      float4 g = *reinterpret_cast<float4*>(t.g + i);
      float4 m = t.m ? *reinterpret_cast<float4*>(t.m + i) : float4{0.f, 0.f, 0.f, 0.f};
      sgd_elem(p.x, g.x, m.x, lr, mom, wd, gscale, nesterov);
      sgd_elem(p.y, g.y, m.y, lr, mom, wd, gscale, nesterov);
      sgd_elem(p.z, g.z, m.z, lr, mom, wd, gscale, nesterov);
      sgd_elem(p.w, g.w, m.w, lr, mom, wd, gscale, nesterov);
      *reinterpret_cast<float4*>(t.p + i) = p;
      if (t.m) *reinterpret_cast<float4*>(t.m + i) = m;
      if (zero_grad) *reinterpret_cast<float4*>(t.g + i) = float4{0.f, 0.f, 0.f, 0.f};
    } else {
      for (long long e = i; e < i + 4 && e < t.n; ++e) {
        float m = t.m ? t.m[e] : 0.f;
        float p = t.p[e], g = t.g[e];
        sgd_elem(p, g, m, lr, mom, wd, gscale, nesterov);
        t.p[e] = p;
        if (t.m) t.m[e] = m;
        if (zero_grad) t.g[e] = 0.f;
      }
    }
  }
}

// One wave per row of x[R, C].  mode 0: log_softmax -> y.  mode 1: fused
// cross-entropy: loss_rows[r] = lse - x[r, t[r]], dx = (softmax - onehot) *
// gscale (so backward is a single scale of the saved dx).
__global__ __launch_bounds__(256) void k_rowwise_softmax(const float* __restrict__ x, float* __restrict__ y,
                                                         const int64_t* __restrict__ target,
                                                         float* __restrict__ loss_rows, float* __restrict__ dx,
                                                         int R, int C, float gscale, int mode) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= R) return;
  const float* xr = x + (size_t)row * C;
  float mx = -INFINITY;
  for (int c = lane; c < C; c += 64) mx = fmaxf(mx, xr[c]);
  mx = wave_max(mx);
  float se = 0.f;
  for (int c = lane; c < C; c += 64) se += __expf(xr[c] - mx);
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  if (mode == 0) {
    for (int c = lane; c < C; c += 64) y[(size_t)row * C + c] = xr[c] - lse;
    return;
  }
  const int t = (int)target[row];
  if (lane == 0) loss_rows[row] = lse - xr[t];
  if (dx)
    for (int c = lane; c < C; c += 64)
      dx[(size_t)row * C + c] = (__expf(xr[c] - lse) - (c == t ? 1.f : 0.f)) * gscale;
}

// log_softmax backward: dx = dy - exp(y) * sum(dy)
__global__ __launch_bounds__(256) void k_log_softmax_bwd(const float* __restrict__ dy, const float* __restrict__ y,
                                                         float* __restrict__ dx, int R, int C) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= R) return;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += dy[(size_t)row * C + c];
  s = wave_sum(s);
  for (int c = lane; c < C; c += 64) {
    const size_t i = (size_t)row * C + c;
    dx[i] = dy[i] - __expf(y[i]) * s;
  }
}

__global__ __launch_bounds__(256) void k_scale(float* __restrict__ x, const float* __restrict__ s, float c,
                                               long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] *= (s ? *s : 1.f) * c;
}

// sum of n floats into out[0] (block partials + atomics; out pre-zeroed)
__global__ __launch_bounds__(256) void k_sum(const float* __restrict__ x, float* __restrict__ out, long long n,
                                             float scale) {
  float s = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) s += x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, s * scale);
}

// Empty kernel: measures the cost of one more launch boundary inside a
// replayed graph (tools/kernel_floor_probe.py, tools/graph_launch_probe.py).
__global__ void k_noop(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0) *p = 0;
}

// Launch-floor probes (tools/kernel_floor_probe.py): an otherwise empty
// block of NT threads with `lds_rounds` LDS exchange + barrier rounds and an
// optional coalesced store of `nstore` floats.
template <int NT>
__global__ __launch_bounds__(NT) void k_probe(float* out, int nstore, int lds_rounds) {
  __shared__ float x[NT];
  float v = (float)threadIdx.x;
  for (int r = 0; r < lds_rounds; ++r) {
    x[threadIdx.x] = v;
    __syncthreads();
    v += x[(threadIdx.x + 1) % NT];
    __syncthreads();
  }
  const int i = blockIdx.x * NT + threadIdx.x;
  if (out && i < nstore) out[i] = v;
}

// `rounds` grid-wide barriers (all blocks must be co-resident: the caller
// keeps blocks <= #CUs).  One thread per block: agent release, counter add,
// spin until every block of this round arrived, agent acquire.  The spin is
// bounded by `max_spin` polls per round (a lost arrival ends the kernel
// instead of hanging it) and records the failure in ctr[1].
__global__ __launch_bounds__(1024) void k_gridbar(unsigned* ctr, int rounds, int max_spin) {
  for (int r = 0; r < rounds; ++r) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      atomicAdd(ctr, 1u);
      const unsigned target = (unsigned)(r + 1) * gridDim.x;
      int n = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && n < max_spin) {
        __builtin_amdgcn_s_sleep(1);
        ++n;
      }
      if (n >= max_spin) atomicOr(ctr + 1, 1u);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
}

// Where each workgroup ran (utils/cu_partition.py): thread 0 records the
// XCD (HW_REG_XCC_ID) and the HW_ID word (CU / SH / SE / queue fields) of its
// wave, then the whole group idles `spin` x ~64 cycles so a large grid is
// spread over every CU the queue may use instead of being drained by the
// first few.  out[2 * blockIdx.x + {0, 1}] = {xcc id, hw id}.
__global__ __launch_bounds__(64) void k_cu_id(unsigned* __restrict__ out, int spin) {
  if (threadIdx.x == 0) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(1);
}

// Self-test of the cross-lane helpers of mfma_f32.h (DPP / permlane swaps):
// one wave, inputs a[64], b[64] -> out[11][64] (tests/test_kernels_gpu.py).
__global__ __launch_bounds__(64) void k_lane_ops_selftest(const float* __restrict__ a, const float* __restrict__ b,
                                                          float* __restrict__ out) {
  const int l = threadIdx.x;
  const float x = a[l], y = b[l];
  out[0 * 64 + l] = lane_xor1(x);
  out[1 * 64 + l] = lane_xor2(x);
  out[2 * 64 + l] = lane_mirror8(x);
  out[3 * 64 + l] = lane_xor8(x);
  out[4 * 64 + l] = lane_sum32(x);
  out[5 * 64 + l] = halve32(x, y);
  out[6 * 64 + l] = halve16(x, y);
  out[7 * 64 + l] = row16_sum(x);
  out[8 * 64 + l] = row16_max(x);
  out[9 * 64 + l] = wave_sum(x);
  out[10 * 64 + l] = wave_max(x);
}

// Synthetic MNIST-shaped data (models/mnist.py synthetic_mnist): a
// counter-based splitmix64 hash of (seed, image, pixel) -- the same formula
// the host implements in numpy, so both produce identical values.  Label =
// hash(seed, image, 784) % 10; pixel = clamp(u * 0.3 + 0.7 * [inside the
// label's 6x6 blob], 0, 1), normalised like Normalize((0.1307,), (0.3081,)).
// Every float operation is rounded separately (no contraction) to match the
// host.  One thread per pixel; 785 counters per image.
__device__ __forceinline__ unsigned long long smix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void k_synth_mnist(float* __restrict__ x, int64_t* __restrict__ y, long long n,
                                                     unsigned long long key) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * 784) return;
  const long long i = t / 784;
  const int p = (int)(t - i * 784);
  const int lab = (int)(smix64((unsigned long long)(i * 785 + 784) * 0x9E3779B97F4A7C15ULL + key) % 10ULL);
  const unsigned long long u64 = smix64((unsigned long long)(i * 785 + p) * 0x9E3779B97F4A7C15ULL + key);
  const float u = (float)(u64 >> 40) * (1.0f / 16777216.0f);
  const int r = p / 28, c = p - r * 28;
  const int y0 = lab < 3 ? 2 : (lab < 6 ? 11 : (lab < 9 ? 20 : 11));
  const int x0 = lab == 9 ? 8 : 2 + 9 * (lab % 3);
  float v = __fmul_rn(u, 0.3f);
  if (r >= y0 && r < y0 + 6 && c >= x0 && c < x0 + 6) v = __fadd_rn(v, 0.7f);
  v = fminf(fmaxf(v, 0.f), 1.f);
  x[t] = __fdiv_rn(__fsub_rn(v, 0.1307f), 0.3081f);
  if (p == 0) y[i] = lab;
}

}  // namespace

#define PTO_API extern "C" __attribute__((visibility("default")))

// key = splitmix64(seed) (the host computes it the same way)
PTO_API int pto_synth_mnist(float* x, int64_t* y, long long n, unsigned long long key, hipStream_t s) {
  if (n < 0 || !x || !y) return -1;
  if (n == 0) return 0;
  const long long tot = n * 784;
  hipLaunchKernelGGL(k_synth_mnist, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, x, y, n, key);
  return (int)hipGetLastError();
}

PTO_API int pto_lane_ops_selftest(const float* a, const float* b, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_lane_ops_selftest, dim3(1), dim3(64), 0, s, a, b, out);
  return (int)hipGetLastError();
}

PTO_API int pto_probe_kernel(int blocks, int threads, float* out, int nstore, int lds_rounds, hipStream_t s) {
  if (threads == 64)
    hipLaunchKernelGGL(k_probe<64>, dim3(blocks), dim3(64), 0, s, out, nstore, lds_rounds);
  else if (threads == 256)
    hipLaunchKernelGGL(k_probe<256>, dim3(blocks), dim3(256), 0, s, out, nstore, lds_rounds);
  else if (threads == 1024)
    hipLaunchKernelGGL(k_probe<1024>, dim3(blocks), dim3(1024), 0, s, out, nstore, lds_rounds);
  else
    return -1;
  return (int)hipGetLastError();
}

PTO_API int pto_gridbar_probe(int blocks, int threads, unsigned* ctr, int rounds, int max_spin, hipStream_t s) {
  if (blocks < 1 || blocks > 256 || threads < 64 || threads > 1024 || (threads & 63)) return -1;
  hipLaunchKernelGGL(k_gridbar, dim3(blocks), dim3(threads), 0, s, ctr, rounds, max_spin);
  return (int)hipGetLastError();
}

PTO_API int pto_cu_id_probe(int blocks, unsigned* out, int spin, hipStream_t s) {
  if (blocks < 1 || blocks > 65536 || !out || spin < 0) return -1;
  hipLaunchKernelGGL(k_cu_id, dim3(blocks), dim3(64), 0, s, out, spin);
  return (int)hipGetLastError();
}

// A stream whose hardware queue may only use the CUs set in mask[0..words)
// (bit i of word w = CU 32 w + i), for ranks that share one GPU
// (utils/cu_partition.py).  Destroy with pto_stream_destroy.
PTO_API int pto_stream_create_cu_mask(unsigned words, const unsigned* mask, hipStream_t* out) {
  if (!words || !mask || !out) return -1;
  return (int)hipExtStreamCreateWithCUMask(out, words, mask);
}

PTO_API int pto_stream_get_cu_mask(hipStream_t s, unsigned words, unsigned* mask) {
  if (!words || !mask) return -1;
  return (int)hipExtStreamGetCUMask(s, words, mask);
}

PTO_API int pto_stream_destroy(hipStream_t s) { return (int)hipStreamDestroy(s); }

PTO_API int pto_sgd_block_count(long long n) { return (int)((n + SGD_CHUNK - 1) / SGD_CHUNK); }

// ts / block_start live in device memory (prepared once by the caller and
// reused every step, so the launch is graph-capturable).
PTO_API int pto_sgd_multi(const SgdTensor* ts, const int* block_start, int ntensors, int nblocks,
                          const float* lr_ptr, float lr, float mom, float wd, float gscale, int nesterov,
                          int zero_grad, long long* bidx, long long nbatches, hipStream_t s) {
  if (nblocks <= 0) return 0;
  hipLaunchKernelGGL(k_sgd_multi, dim3(nblocks), dim3(256), 0, s, ts, block_start, ntensors, lr_ptr, lr, mom, wd,
                     gscale, nesterov, zero_grad, bidx, nbatches);
  return (int)hipGetLastError();
}

PTO_API int pto_log_softmax_fwd(const float* x, float* y, int R, int C, hipStream_t s) {
  hipLaunchKernelGGL(k_rowwise_softmax, dim3((R + 3) / 4), dim3(256), 0, s, x, y, nullptr, nullptr, nullptr, R, C,
                     1.f, 0);
  return (int)hipGetLastError();
}

PTO_API int pto_log_softmax_bwd(const float* dy, const float* y, float* dx, int R, int C, hipStream_t s) {
  hipLaunchKernelGGL(k_log_softmax_bwd, dim3((R + 3) / 4), dim3(256), 0, s, dy, y, dx, R, C);
  return (int)hipGetLastError();
}

PTO_API int pto_cross_entropy_fwd(const float* x, const int64_t* target, float* loss_rows, float* dx, int R, int C,
                                  float gscale, hipStream_t s) {
  hipLaunchKernelGGL(k_rowwise_softmax, dim3((R + 3) / 4), dim3(256), 0, s, x, nullptr, target, loss_rows, dx, R, C,
                     gscale, 1);
  return (int)hipGetLastError();
}

PTO_API int pto_scale(float* x, const float* sptr, float c, long long n, hipStream_t s) {
  hipLaunchKernelGGL(k_scale, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, sptr, c, n);
  return (int)hipGetLastError();
}

PTO_API int pto_sum(const float* x, float* out, long long n, float scale, hipStream_t s) {
  int blocks = (int)((n + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(k_sum, dim3(blocks), dim3(256), 0, s, x, out, n, scale);
  return (int)hipGetLastError();
}

PTO_API int pto_noop(int blocks, hipStream_t s) {
  hipLaunchKernelGGL(k_noop, dim3(blocks), dim3(64), 0, s, nullptr);
  return (int)hipGetLastError();
}

// Upload an instantiated graph's launch resources ahead of its first timed
// replay (the handle from torch.cuda.CUDAGraph.raw_cuda_graph_exec()).
PTO_API int pto_graph_upload(void* exec, hipStream_t s) {
  return (int)hipGraphUpload(reinterpret_cast<hipGraphExec_t>(exec), s);
}
