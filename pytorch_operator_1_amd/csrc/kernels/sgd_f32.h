// SGD-momentum element update shared by the multi-tensor SGD launch
// (common_kernels.hip) and the MNIST kernels that run the optimizer inside
// backward/forward launches (mnist_kernels.hip, "fused optimizer" schedule).
//
// buf = momentum*buf + (gscale*g + wd*p);  p -= lr * (nesterov ? d + momentum*buf : buf)
// = torch.optim.SGD with dampening = 0 (torch's first step sets buf = d,
// identical to momentum*0 + d with a zero-initialised buffer).
#pragma once
#include <hip/hip_runtime.h>

__device__ __forceinline__ void sgd_elem(float& p, float g, float& m, float lr, float mom, float wd, float gs,
                                         int nesterov) {
  float d = g * gs;
  if (wd != 0.f) d = fmaf(wd, p, d);
  if (mom != 0.f) {
    m = fmaf(mom, m, d);
    d = nesterov ? fmaf(mom, m, d) : m;
  }
  p = fmaf(-lr, d, p);
}

// Optimizer hyper-parameters as the fused kernels receive them (lr from
// device memory so LR schedules survive graph replay).
struct SgdArgs {
  const float* lr;
  float mom, wd, gscale;
  int nesterov;
  int variant;  // kernel-variant selector for launches that carry SgdArgs (0 = default)
};

// One float4 group (4 elements at i, 16-byte aligned, i + 3 < n) of a flat
// (p, g, m) range: update p, m in place and zero g (unless the producer of g
// overwrites it every step: zero_g = false saves the store).
__device__ __forceinline__ void sgd_flat4(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                          long long i, float lr, const SgdArgs& a, bool zero_g = true) {
  float4 pv = *reinterpret_cast<float4*>(p + i);
  const float4 gv = *reinterpret_cast<const float4*>(g + i);
  float4 mv = *reinterpret_cast<float4*>(m + i);
  sgd_elem(pv.x, gv.x, mv.x, lr, a.mom, a.wd, a.gscale, a.nesterov);
  sgd_elem(pv.y, gv.y, mv.y, lr, a.mom, a.wd, a.gscale, a.nesterov);
  sgd_elem(pv.z, gv.z, mv.z, lr, a.mom, a.wd, a.gscale, a.nesterov);
  sgd_elem(pv.w, gv.w, mv.w, lr, a.mom, a.wd, a.gscale, a.nesterov);
  *reinterpret_cast<float4*>(p + i) = pv;
  *reinterpret_cast<float4*>(m + i) = mv;
  if (zero_g) *reinterpret_cast<float4*>(g + i) = float4{0.f, 0.f, 0.f, 0.f};
}
