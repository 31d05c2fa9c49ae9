// Multi-tensor AdamW for the large-model configs (ResNet-50 / Llama-3-8B
// DDP, BASELINE configs 3-4), one launch for every parameter tensor.
//
// Mixed precision layout (sized for 288 GB HBM per MI355X): model params
// and grads in bf16 (what the forward/backward and the RCCL bucket
// all-reduce touch: 2 + 2 bytes/param), fp32 master weights + fp32 Adam
// moments held only by the optimizer (12 bytes/param).  Llama-3-8B:
// 8.03e9 x 16 B = 128 GB per GPU before activations.
//
// The op is HBM-bound (per param: read 2+4+4+4, write 2+4+4+4 bytes), so
// every lane moves 8 elements per step: 16-byte bf16 loads/stores and
// 2 x 16-byte fp32 accesses per state tensor (Guideline 13).
#include <hip/hip_runtime.h>
#include <stdint.h>

struct AdamTensor {
  void* p;         // param: bf16 (mixed) or fp32
  void* g;         // grad: bf16 (mixed) or fp32
  float* master;   // fp32 master weights (mixed only; nullptr for fp32 params)
  float* m;
  float* v;
  long long n;
};

namespace {

constexpr int ADAM_CHUNK = 256 * 8;  // elements per block (8 per thread)

__device__ __forceinline__ float bf2f(uint16_t x) { return __uint_as_float(((uint32_t)x) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // round-to-nearest-even
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)(u >> 16) | ((u & 0xffff) ? 0x40 : 0);  // inf/nan
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

struct AdamHyper {
  float lr, beta1, beta2, eps, wd, bc1, bc2, gscale;
};

__device__ __forceinline__ void adam_elem(float& w, float g, float& m, float& v, const AdamHyper& h) {
  g *= h.gscale;
  m = h.beta1 * m + (1.f - h.beta1) * g;
  v = h.beta2 * v + (1.f - h.beta2) * g * g;
  const float mhat = m / h.bc1, vhat = v / h.bc2;
  w = w * (1.f - h.lr * h.wd) - h.lr * mhat / (sqrtf(vhat) + h.eps);  // decoupled decay (AdamW)
}

template <bool MIXED>
__global__ __launch_bounds__(256) void k_adamw_multi(const AdamTensor* __restrict__ ts,
                                                     const int* __restrict__ block_start, int ntensors,
                                                     const float* __restrict__ lr_ptr, AdamHyper h,
                                                     int zero_grad) {
  int lo = 0, hi = ntensors - 1;
  const int bid = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (block_start[mid] <= bid) lo = mid; else hi = mid - 1;
  }
  const AdamTensor t = ts[lo];
  if (lr_ptr) h.lr = *lr_ptr;
  const long long i0 = (long long)(bid - block_start[lo]) * ADAM_CHUNK + (long long)threadIdx.x * 8;
  if (i0 >= t.n) return;
  const bool full = i0 + 8 <= t.n;
  if (MIXED) {
    uint16_t* pb = reinterpret_cast<uint16_t*>(t.p);
    uint16_t* gb = reinterpret_cast<uint16_t*>(t.g);
    const bool vec = full && ((((uintptr_t)(pb + i0)) | ((uintptr_t)(gb + i0)) | ((uintptr_t)(t.master + i0)) |
                               ((uintptr_t)(t.m + i0)) | ((uintptr_t)(t.v + i0))) & 15) == 0;
    if (vec) {
      const uint4 gv = *reinterpret_cast<const uint4*>(gb + i0);
      float4 w0 = reinterpret_cast<float4*>(t.master + i0)[0], w1 = reinterpret_cast<float4*>(t.master + i0)[1];
      float4 m0 = reinterpret_cast<float4*>(t.m + i0)[0], m1 = reinterpret_cast<float4*>(t.m + i0)[1];
      float4 v0 = reinterpret_cast<float4*>(t.v + i0)[0], v1 = reinterpret_cast<float4*>(t.v + i0)[1];
      const uint16_t* gs = reinterpret_cast<const uint16_t*>(&gv);
      float w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      float m[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
      float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      uint16_t out[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        adam_elem(w[j], bf2f(gs[j]), m[j], v[j], h);
        out[j] = f2bf(w[j]);
      }
      reinterpret_cast<float4*>(t.master + i0)[0] = float4{w[0], w[1], w[2], w[3]};
      reinterpret_cast<float4*>(t.master + i0)[1] = float4{w[4], w[5], w[6], w[7]};
      reinterpret_cast<float4*>(t.m + i0)[0] = float4{m[0], m[1], m[2], m[3]};
      reinterpret_cast<float4*>(t.m + i0)[1] = float4{m[4], m[5], m[6], m[7]};
      reinterpret_cast<float4*>(t.v + i0)[0] = float4{v[0], v[1], v[2], v[3]};
      reinterpret_cast<float4*>(t.v + i0)[1] = float4{v[4], v[5], v[6], v[7]};
      *reinterpret_cast<uint4*>(pb + i0) = *reinterpret_cast<const uint4*>(out);
      if (zero_grad) *reinterpret_cast<uint4*>(gb + i0) = uint4{0, 0, 0, 0};
    } else {
      for (long long e = i0; e < i0 + 8 && e < t.n; ++e) {
        float w = t.master[e], m = t.m[e], v = t.v[e];
        adam_elem(w, bf2f(gb[e]), m, v, h);
        t.master[e] = w; t.m[e] = m; t.v[e] = v;
        pb[e] = f2bf(w);
        if (zero_grad) gb[e] = 0;
      }
    }
  } else {
    float* p = reinterpret_cast<float*>(t.p);
    float* g = reinterpret_cast<float*>(t.g);
    for (long long e = i0; e < i0 + 8 && e < t.n; ++e) {
      float w = p[e], m = t.m[e], v = t.v[e];
      adam_elem(w, g[e], m, v, h);
      p[e] = w; t.m[e] = m; t.v[e] = v;
      if (zero_grad) g[e] = 0.f;
    }
  }
}

// bf16 <-> fp32 flat casts (master-weight init, checkpoint export)
__global__ __launch_bounds__(256) void k_bf16_to_f32(const uint16_t* __restrict__ x, float* __restrict__ y, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = bf2f(x[i]);
}

}  // namespace

#define PTO_API extern "C" __attribute__((visibility("default")))

PTO_API int pto_adamw_block_count(long long n) { return (int)((n + ADAM_CHUNK - 1) / ADAM_CHUNK); }

// step = 1-based optimizer step (bias corrections computed here).
PTO_API int pto_adamw_multi(const AdamTensor* ts, const int* block_start, int ntensors, int nblocks, int mixed,
                            const float* lr_ptr, float lr, float beta1, float beta2, float eps, float wd, int step,
                            float gscale, int zero_grad, hipStream_t s) {
  if (nblocks <= 0) return 0;
  AdamHyper h{lr, beta1, beta2, eps, wd, 1.f - powf(beta1, (float)step), 1.f - powf(beta2, (float)step), gscale};
  if (mixed)
    hipLaunchKernelGGL(k_adamw_multi<true>, dim3(nblocks), dim3(256), 0, s, ts, block_start, ntensors, lr_ptr, h,
                       zero_grad);
  else
    hipLaunchKernelGGL(k_adamw_multi<false>, dim3(nblocks), dim3(256), 0, s, ts, block_start, ntensors, lr_ptr, h,
                       zero_grad);
  return (int)hipGetLastError();
}

PTO_API int pto_bf16_to_f32(const void* x, float* y, long long n, hipStream_t s) {
  hipLaunchKernelGGL(k_bf16_to_f32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<const uint16_t*>(x), y, n);
  return (int)hipGetLastError();
}
