// LDS access-pattern probe (tools/lds_patterns_probe.py): each kernel is
// one access pattern of the MNIST step's conv2 wgrad role, repeated, so a
// rocprofv3 --pmc pass gives its SQ_LDS_BANK_CONFLICT per instruction.
// Built into its own .so; nothing here ships.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PROBE extern "C" __global__ __launch_bounds__(256)
constexpr int REP = 64;

// 4 consecutive lanes write the 4 bytes of one dword (the wgrad code staging)
PROBE void p_b8_same_dword(uint32_t* out, int salt) {
  __shared__ uint8_t s[4096];
  const int t = threadIdx.x;
  for (int i = 0; i < REP; ++i) {
    s[(t + 256 * (i & 3)) ^ (salt & 3)] = (uint8_t)(t + i);
    __builtin_amdgcn_s_barrier();
  }
  __syncthreads();
  out[t] = s[t * 4] + s[t * 4 + 1];
}

// control: lane l writes byte 0 of dword l
PROBE void p_b8_own_dword(uint32_t* out, int salt) {
  __shared__ uint8_t s[4096 * 4];
  const int t = threadIdx.x;
  for (int i = 0; i < REP; ++i) {
    s[4 * ((t + 256 * (i & 3)) ^ (salt & 3))] = (uint8_t)(t + i);
    __builtin_amdgcn_s_barrier();
  }
  __syncthreads();
  out[t] = s[t * 4] + s[t * 16];
}

// the wgrad grad staging: scalar stores, transposed + swizzled
PROBE void p_gs_store(uint32_t* out, int salt) {
  __shared__ float gs[6 * 800];
  const int tid = threadIdx.x;
  for (int i = 0; i < REP; ++i) {
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int e = tid + 256 * q;
      if (e < 6 * 200) {
        const int smp = e / 200, r = e - smp * 200, oc_ = r >> 2, G = r & 3;
        const int sw = (oc_ >> 2) & 3;
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) gs[smp * 800 + oc_ * 16 + 4 * (gg ^ sw) + G] = (float)(i + gg + salt);
      }
    }
    __builtin_amdgcn_s_barrier();
  }
  __syncthreads();
  out[tid] = __float_as_uint(gs[tid * 3]);
}

// the wgrad MFMA loop's patch reads for column tile nt (koff per lane), one
// sample: 4 G x (ap[0], ap[1], ap[12], ap[13])
PROBE void p_patch_reads(uint32_t* out, int nt) {
  __shared__ float as[6 * 288];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  for (int i = tid; i < 6 * 288; i += 256) as[i] = (float)i;
  __syncthreads();
  const int col0 = nt * 16, ic0 = col0 / 25;
  const int kk = col0 + (lane & 15);
  const bool kvalid = kk < 500;
  const int ic = kvalid ? kk / 25 : ic0, r25 = kvalid ? kk - ic * 25 : 0;
  const int kh = r25 / 5, kw = r25 - kh * 5;
  const int koff = (ic - ic0) * 144 + kh * 12 + kw;
  float acc = 0.f;
  for (int i = 0; i < REP; ++i) {
    const int smp = i % 6;
#pragma unroll
    for (int G = 0; G < 4; ++G) {
      const float* ap = as + smp * 288 + koff + 24 * G + 2 * g;
      acc += ap[0] * ap[1] + ap[12] * ap[13];
    }
  }
  out[tid] = __float_as_uint(acc);
}

// the wgrad loop's grad (b128) + code (b32) reads
PROBE void p_gc_reads(uint32_t* out, int salt) {
  __shared__ __attribute__((aligned(16))) float gs[6 * 800];
  __shared__ uint32_t cs[6 * 200];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane >> 4;
  for (int i = tid; i < 6 * 800; i += 256) gs[i] = (float)i;
  for (int i = tid; i < 6 * 200; i += 256) cs[i] = i;
  __syncthreads();
  const int oc = wv * 16 + (lane & 15);
  const int goff = oc * 16 + 4 * (g ^ ((oc >> 2) & 3));
  float acc = 0.f;
  uint32_t ac = 0;
  for (int i = 0; i < REP; ++i) {
    const int smp = (i + salt) % 6;
    const float4 g4 = *reinterpret_cast<const float4*>(gs + smp * 800 + goff);
    ac += cs[(smp * 800 + goff) >> 2];
    acc += g4.x + g4.y * g4.z - g4.w;
  }
  out[tid] = __float_as_uint(acc) + ac;
}

extern "C" int probe_lds_patterns(uint32_t* out, hipStream_t s) {
  for (int k = 0; k < 4; ++k) {
    hipLaunchKernelGGL(p_b8_same_dword, dim3(1), dim3(256), 0, s, out, k);
    hipLaunchKernelGGL(p_b8_own_dword, dim3(1), dim3(256), 0, s, out, k);
    hipLaunchKernelGGL(p_gs_store, dim3(1), dim3(256), 0, s, out, k);
    hipLaunchKernelGGL(p_gc_reads, dim3(1), dim3(256), 0, s, out, k);
  }
  for (int nt = 0; nt < 32; ++nt) hipLaunchKernelGGL(p_patch_reads, dim3(1), dim3(256), 0, s, out, nt);
  return (int)hipGetLastError();
}

// LDS broadcast / conflict rules: one address function x instruction kind
// per dispatch (order: kind-major, see tools/lds_patterns_probe.py)
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ int rule_addr(int mode, int lane) {
  const int c = lane & 15, g = lane >> 4;
  const int kh = c / 5, kw = c - kh * 5;
  switch (mode) {
    case 0: return lane;                       // 64 distinct, consecutive
    case 1: return 0;                          // one address
    case 2: return c;                          // 16 addresses, lanes l, l+16, l+32, l+48 share
    case 3: return lane >> 2;                  // 16 addresses, 4 consecutive lanes share
    case 4: return kh * 12 + kw + 2 * g;       // the wgrad patch read (tile 0)
    case 5: return kh * 12 + kw;               // same without the 2g group offset
    case 6: return 2 * lane;                   // stride 2
    default: return lane * 64;                 // one bank: 64-way
  }
}

PROBE void p_rule(uint32_t* out, int mode, int kind) {
  __shared__ __attribute__((aligned(16))) float s[8192];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 8192; i += 256) s[i] = (float)i;
  __syncthreads();
  const int a = rule_addr(mode, lane) & 4095;
  const uint32_t base = (uint32_t)(uintptr_t)(s) + 4u * (uint32_t)a;
  float acc = 0.f;
  for (int i = 0; i < REP; ++i) {
    if (kind == 0) {
      float x;
      asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(base) : "memory");
      acc += x;
    } else if (kind == 1) {
      f2v x;
      asm volatile("ds_read2_b32 %0, %1 offset1:1\n s_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(base) : "memory");
      acc += x.x + x.y;
    } else {
      f2v x;  // 8-byte aligned pair at 2a
      asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(base + 4u * (uint32_t)a) : "memory");
      acc += x.x + x.y;
    }
  }
  out[tid] = __float_as_uint(acc);
}

extern "C" int probe_lds_rules(uint32_t* out, hipStream_t s) {
  for (int kind = 0; kind < 3; ++kind)
    for (int mode = 0; mode < 8; ++mode) hipLaunchKernelGGL(p_rule, dim3(1), dim3(256), 0, s, out, mode, kind);
  return (int)hipGetLastError();
}
