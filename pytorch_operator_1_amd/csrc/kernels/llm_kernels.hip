// Memory-bound kernels of the Llama-3 / ResNet DDP configs (BASELINE
// configs 3-4), bf16 activations with fp32 math.  GEMMs go to hipBLASLt;
// everything between the GEMMs is fused here so each activation tensor
// crosses HBM once per direction:
//
//   add_rmsnorm_fwd   h = x + r (optional), y = h * rstd(h) * w      1 read x,r  1 write h,y
//   rmsnorm_bwd       dx = rstd*(dy*w) - h*rstd^3/D*<dy*w,h> + dres  (dres = grad flowing
//                     into h from the residual stream -> add fused), dw partials
//   swiglu_fwd/bwd    gu = [gate | up] from one fused W13 GEMM
//   rope_fwd/bwd      in place on the q,k heads of the fused QKV GEMM output
//   ce_fwd/bwd        vocab-wide cross entropy on bf16 logits (128256 columns),
//                     gradient written in place into the logits buffer
//
// Rows are processed by one 256-thread block (4 waves); each thread moves
// 8 bf16 (16 bytes) per access (Guideline 13).  bf16 is raw uint16_t.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ float bf2f(uint16_t x) { return __uint_as_float(((uint32_t)x) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)(u >> 16) | ((u & 0xffff) ? 0x40 : 0);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

struct V8 {
  float v[8];
};
__device__ __forceinline__ V8 ld8(const uint16_t* p) {
  const uint4 q = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
  V8 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r.v[2 * i] = __uint_as_float(w[i] << 16);
    r.v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
  return r;
}
__device__ __forceinline__ V8 unpack8(const uint4 q) {  // bf16x8 -> 8 floats
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
  V8 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r.v[2 * i] = __uint_as_float(w[i] << 16);
    r.v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
  return r;
}
__device__ __forceinline__ void st8(uint16_t* p, const V8& r) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(r.v[2 * i]) | ((uint32_t)f2bf(r.v[2 * i + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = uint4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// 256-thread block reduction (4 waves); red must hold 4 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

constexpr int NT = 256;
constexpr int RMS_MAXV = 4;  // up to 4 x 8 x 256 = 8192 columns held in registers

// ---------------------------------------------------------------- RMSNorm
template <bool RES>
__global__ __launch_bounds__(NT) void k_add_rmsnorm_fwd(const uint16_t* __restrict__ x, const uint16_t* __restrict__ r,
                                                         const uint16_t* __restrict__ w, uint16_t* __restrict__ h,
                                                         uint16_t* __restrict__ y, float* __restrict__ rstd, int D,
                                                         float eps) {
  __shared__ float red[4];
  const long long row = blockIdx.x;
  const uint16_t* xr = x + row * D;
  V8 hv[RMS_MAXV];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < RMS_MAXV; ++j) {
    const int c = (j * NT + threadIdx.x) * 8;
    if (c < D) {
      hv[j] = ld8(xr + c);
      if (RES) {
        const V8 rv = ld8(r + row * D + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) hv[j].v[e] += rv.v[e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) ss += hv[j].v[e] * hv[j].v[e];
      }
    }
  }
  // Residual sum is rounded to bf16 (it is the stored residual stream);
  // normalise the rounded value so forward and backward agree.
  if (RES) {
    ss = 0.f;
#pragma unroll
    for (int j = 0; j < RMS_MAXV; ++j) {
      const int c = (j * NT + threadIdx.x) * 8;
      if (c < D) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          hv[j].v[e] = bf2f(f2bf(hv[j].v[e]));
          ss += hv[j].v[e] * hv[j].v[e];
        }
        st8(h + row * D + c, hv[j]);
      }
    }
  }
  const float rs = rsqrtf(block_sum(ss, red) / (float)D + eps);
  if (threadIdx.x == 0) rstd[row] = rs;
#pragma unroll
  for (int j = 0; j < RMS_MAXV; ++j) {
    const int c = (j * NT + threadIdx.x) * 8;
    if (c < D) {
      const V8 wv = ld8(w + c);
      V8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o.v[e] = bf2f(f2bf(hv[j].v[e] * rs)) * wv.v[e];  // HF: w * (x*rstd).to(bf16)
      st8(y + row * D + c, o);
    }
  }
}

// One block per group of rows; dw partial sums in registers -> part[G][D].
// V = 8-column vectors per thread (D <= V * 2048): the register arrays are
// sized for the real width.  Every load of row i+1 (h, dy, the residual
// gradient, rstd) is issued before row i's block reduction, so the row loop
// is not one memory round trip per row behind the reduction (Llama-3-8B:
// 157 us per call at 3.5 TB/s before).
template <int V>
__global__ __launch_bounds__(NT) void k_rmsnorm_bwd(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ h,
                                                    const uint16_t* __restrict__ w, const float* __restrict__ rstd,
                                                    const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx,
                                                    float* __restrict__ part, int M, int D) {
  __shared__ float red[4];
  // the weight row and the prefetched rows stay packed bf16 (4 registers per
  // 8 columns, unpacked where used): V = 2 fits 128 registers, so all four
  // 4-wave workgroups of a CU are resident (162 registers and a 768 + 256
  // block tail before)
  uint4 wq[V];
  V8 dwacc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c = (j * NT + threadIdx.x) * 8;
    wq[j] = c < D ? *reinterpret_cast<const uint4*>(w + c) : uint4{0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 8; ++e) dwacc[j].v[e] = 0.f;
  }
  uint4 hn[V], gn[V], rn[V];
  float rsn = 0.f;
  auto load = [&](long long row) {
    if (row >= M) return;
    rsn = rstd[row];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = (j * NT + threadIdx.x) * 8;
      if (c < D) {
        hn[j] = *reinterpret_cast<const uint4*>(h + row * D + c);
        gn[j] = *reinterpret_cast<const uint4*>(dy + row * D + c);
        if (dres) rn[j] = *reinterpret_cast<const uint4*>(dres + row * D + c);
      }
    }
  };
  load(blockIdx.x);
  for (long long row = blockIdx.x; row < M; row += gridDim.x) {
    const float rs = rsn;
    uint4 hc[V], gc[V], rc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      hc[j] = hn[j];
      gc[j] = gn[j];
      rc[j] = rn[j];
    }
    load(row + gridDim.x);  // in flight during this row's math and reduction
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = (j * NT + threadIdx.x) * 8;
      if (c < D) {
        const V8 hv = unpack8(hc[j]), gv = unpack8(gc[j]), wv = unpack8(wq[j]);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float n = bf2f(f2bf(hv.v[e] * rs));
          dwacc[j].v[e] += gv.v[e] * n;
          dot += gv.v[e] * wv.v[e] * hv.v[e];  // g = dy * w
        }
      }
    }
    const float k = block_sum(dot, red) * rs * rs * rs / (float)D;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = (j * NT + threadIdx.x) * 8;
      if (c < D) {
        const V8 hv = unpack8(hc[j]), gv = unpack8(gc[j]), wv = unpack8(wq[j]);
        V8 rv;
        if (dres) rv = unpack8(rc[j]);
        V8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          o.v[e] = (dres ? rv.v[e] : 0.f) + (rs * (gv.v[e] * wv.v[e]) - k * hv.v[e]);
        st8(dx + row * D + c, o);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c = (j * NT + threadIdx.x) * 8;
    if (c < D) {
      float4* pp = reinterpret_cast<float4*>(part + (long long)blockIdx.x * D + c);
      pp[0] = float4{dwacc[j].v[0], dwacc[j].v[1], dwacc[j].v[2], dwacc[j].v[3]};
      pp[1] = float4{dwacc[j].v[4], dwacc[j].v[5], dwacc[j].v[6], dwacc[j].v[7]};
    }
  }
}

// dw[c] = bf16(sum_g part[g][c]): 64 columns per block as 16 float4 column
// quads x 16 row slices, 8 independent 16-byte loads in flight per thread
// (the first version summed with one dependent load per iteration: 64 us per
// call for 1024 x 4096 partials, 65 calls per Llama-3-8B step); the 16
// slices are combined in a fixed order (deterministic).
__global__ __launch_bounds__(NT) void k_colsum_bf16(const float* __restrict__ part, uint16_t* __restrict__ dw, int G,
                                                    int D) {
  __shared__ float4 s[16][16];
  const int q = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + 4 * q;
  float4 a = {0.f, 0.f, 0.f, 0.f};
  if (c < D) {
    int g = sl;
    for (; g + 16 * 7 < G; g += 16 * 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(part + (long long)(g + 16 * u) * D + c);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
      }
    }
    for (; g < G; g += 16) {
      const float4 v = *reinterpret_cast<const float4*>(part + (long long)g * D + c);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  s[sl][q] = a;
  __syncthreads();
  if (sl == 0 && c < D) {
    float4 t = s[0][q];
#pragma unroll
    for (int r = 1; r < 16; ++r) {
      t.x += s[r][q].x; t.y += s[r][q].y; t.z += s[r][q].z; t.w += s[r][q].w;
    }
    dw[c] = f2bf(t.x); dw[c + 1] = f2bf(t.y); dw[c + 2] = f2bf(t.z); dw[c + 3] = f2bf(t.w);
  }
}

// ---------------------------------------------------------------- SwiGLU
__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + __expf(-x)); }

// gu [M][2F] (gate | up) -> out [M][F];  8 columns per thread.
__global__ __launch_bounds__(NT) void k_swiglu_fwd(const uint16_t* __restrict__ gu, uint16_t* __restrict__ out,
                                                   long long M, int F) {
  const int F8 = F >> 3;
  const long long total = M * F8;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const long long m = i / F8;
    const int c = (int)(i - m * F8) * 8;
    const V8 g = ld8(gu + m * 2 * F + c), u = ld8(gu + m * 2 * F + F + c);
    V8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o.v[e] = bf2f(f2bf(g.v[e] * sigmoidf(g.v[e]))) * u.v[e];
    st8(out + m * F + c, o);
  }
}

__global__ __launch_bounds__(NT) void k_swiglu_bwd(const uint16_t* __restrict__ gu, const uint16_t* __restrict__ dout,
                                                   uint16_t* __restrict__ dgu, long long M, int F) {
  const int F8 = F >> 3;
  const long long total = M * F8;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const long long m = i / F8;
    const int c = (int)(i - m * F8) * 8;
    const V8 g = ld8(gu + m * 2 * F + c), u = ld8(gu + m * 2 * F + F + c), d = ld8(dout + m * F + c);
    V8 dg, du;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float s = sigmoidf(g.v[e]);
      const float silu = g.v[e] * s;
      du.v[e] = d.v[e] * silu;
      dg.v[e] = d.v[e] * u.v[e] * s * (1.f + g.v[e] * (1.f - s));
    }
    st8(dgu + m * 2 * F + c, dg);
    st8(dgu + m * 2 * F + F + c, du);
  }
}

// SwiGLU backward that ALSO writes the gradient transposed, dgu_t [2F][M]:
// what the gate|up projection's K-contiguous weight gradient consumes
// (ops/llm.py _LinearTW, dW = dgu^T X from K(token)-contiguous operands), so
// the step no longer transposes the largest activation gradient of the MLP
// ([16384 x 28672] per layer on Llama-3-8B) in a pass of its own.  Block =
// 128 tokens x 64 features: each thread computes 4 tokens x 8 features of dg
// and du, stores them row-major as k_swiglu_bwd, and drops them into two LDS
// tiles [feature][token] (row pitch 130 halves: the paired-token 32-bit
// writes of a wave spread over the banks); the transposed rows then leave as
// 16-byte stores, 256 contiguous bytes per feature row and tile (64-token
// tiles, 128-byte rows, measured 4.2 TB/s).
constexpr int SWT = 64;        // features per block
constexpr int SWT_M = 128;     // tokens per block
constexpr int SWT_LD = 130;    // LDS row pitch (halves)
__global__ __launch_bounds__(NT) void k_swiglu_bwd_t(const uint16_t* __restrict__ gu, const uint16_t* __restrict__ dout,
                                                     uint16_t* __restrict__ dgu, uint16_t* __restrict__ dgu_t,
                                                     long long M, int F) {
  __shared__ __attribute__((aligned(16))) uint16_t tg[SWT * SWT_LD], tu[SWT * SWT_LD];
  const int ntf = F / SWT;
  const long long m0 = (long long)(blockIdx.x / ntf) * SWT_M;
  const int f0 = (blockIdx.x % ntf) * SWT;
  const int t = threadIdx.x, fg = t & 7, tq = t >> 3;  // 8 features at 8*fg, tokens 2tq, 2tq+1, 64+2tq, 65+2tq
  const int c = f0 + 8 * fg;
  // all 12 loads of the thread's 4 tokens in flight before the first use
  V8 gl[4], ul[4], dl[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long long m = m0 + 64 * (i >> 1) + 2 * tq + (i & 1);
    const long long mm = m < M ? m : m0;
    gl[i] = ld8(gu + mm * 2 * F + c);
    ul[i] = ld8(gu + mm * 2 * F + F + c);
    dl[i] = ld8(dout + mm * F + c);
  }
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    V8 dg[2], du[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const long long m = m0 + 64 * half + 2 * tq + k;
      const bool ok = m < M;
      const V8& g = gl[2 * half + k];
      const V8& u = ul[2 * half + k];
      const V8& d = dl[2 * half + k];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sg = sigmoidf(g.v[e]);  // the same expressions as k_swiglu_bwd
        const float silu = g.v[e] * sg;
        du[k].v[e] = d.v[e] * silu;
        dg[k].v[e] = d.v[e] * u.v[e] * sg * (1.f + g.v[e] * (1.f - sg));
      }
      if (ok) {
        st8(dgu + m * 2 * F + c, dg[k]);
        st8(dgu + m * 2 * F + F + c, du[k]);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {  // the token pair as one 32-bit word per feature
      const int row = (8 * fg + e) * SWT_LD + 64 * half + 2 * tq;
      *reinterpret_cast<uint32_t*>(tg + row) = (uint32_t)f2bf(dg[0].v[e]) | ((uint32_t)f2bf(dg[1].v[e]) << 16);
      *reinterpret_cast<uint32_t*>(tu + row) = (uint32_t)f2bf(du[0].v[e]) | ((uint32_t)f2bf(du[1].v[e]) << 16);
    }
  }
  __syncthreads();
  // 2 x 64 feature rows x 16 chunks of 8 tokens = 2048 16-byte stores, 8 per thread
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int idx = t + NT * q, half = idx >> 10, r = (idx >> 4) & 63, ch = idx & 15;
    const uint16_t* src = (half ? tu : tg) + r * SWT_LD + 8 * ch;
    const long long m = m0 + 8 * ch;
    if (m >= M) continue;
    const long long orow = (long long)(half ? F : 0) + f0 + r;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = *reinterpret_cast<const uint32_t*>(src + 2 * j);
    if (m + 8 <= M) {
      *reinterpret_cast<uint4*>(dgu_t + orow * M + m) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      for (int j = 0; j < 8 && m + j < M; ++j) dgu_t[orow * M + m + j] = src[j];
    }
  }
}

// ---------------------------------------------------------------- RoPE
// qkv row m = (b*S + s) has nh heads of D at stride row_stride; rotate the
// first nrot heads (q and k).  rotate_half convention: pairs (i, i + D/2).
// cs = [S][D/2] cos, sn = [S][D/2] sin (fp32).  sign = +1 fwd, -1 bwd.
// src == dst: in place over the nrot heads only (nh == nrot).  src != dst:
// all nh heads are written, heads >= nrot copied unchanged (backward: the
// incoming gradient is never modified).
__global__ __launch_bounds__(NT) void k_rope(const uint16_t* src, uint16_t* dst, const float* __restrict__ cs,
                                             const float* __restrict__ sn, long long M, int S, int nrot, int nh, int D,
                                             long long row_stride, float sign) {
  const int H2 = D >> 1, Q = H2 >> 2;  // 4 pairs per thread
  const long long total = M * nh * Q;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int q = (int)(i % Q);
    const long long t = i / Q;
    const int hd = (int)(t % nh);
    const long long m = t / nh;
    const int s = (int)(m % S);
    const long long off = m * row_stride + (long long)hd * D + q * 4;
    const uint2 lo = *reinterpret_cast<const uint2*>(src + off), hi = *reinterpret_cast<const uint2*>(src + off + H2);
    uint16_t* base = dst + off;
    if (hd >= nrot) {
      *reinterpret_cast<uint2*>(base) = lo;
      *reinterpret_cast<uint2*>(base + H2) = hi;
      continue;
    }
    const float4 c = *reinterpret_cast<const float4*>(cs + (long long)s * H2 + q * 4);
    const float4 n = *reinterpret_cast<const float4*>(sn + (long long)s * H2 + q * 4);
    const float x1[4] = {__uint_as_float(lo.x << 16), __uint_as_float(lo.x & 0xffff0000u), __uint_as_float(lo.y << 16),
                         __uint_as_float(lo.y & 0xffff0000u)};
    const float x2[4] = {__uint_as_float(hi.x << 16), __uint_as_float(hi.x & 0xffff0000u), __uint_as_float(hi.y << 16),
                         __uint_as_float(hi.y & 0xffff0000u)};
    const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sign * n.x, sign * n.y, sign * n.z, sign * n.w};
    uint16_t o1[4], o2[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o1[e] = f2bf(x1[e] * cc[e] - x2[e] * ss[e]);
      o2[e] = f2bf(x2[e] * cc[e] + x1[e] * ss[e]);
    }
    *reinterpret_cast<uint2*>(base) = uint2{(uint32_t)o1[0] | ((uint32_t)o1[1] << 16), (uint32_t)o1[2] | ((uint32_t)o1[3] << 16)};
    *reinterpret_cast<uint2*>(base + H2) =
        uint2{(uint32_t)o2[0] | ((uint32_t)o2[1] << 16), (uint32_t)o2[2] | ((uint32_t)o2[3] << 16)};
  }
}

// ---------------------------------------------------------------- cross entropy
// One block per row of V logits (bf16).  fwd: lse[m], loss[m] (0 for ignored).
__global__ __launch_bounds__(NT) void k_ce_fwd(const uint16_t* __restrict__ logits, const long long* __restrict__ labels,
                                               float* __restrict__ lse, float* __restrict__ loss, int V,
                                               long long ignore_index) {
  __shared__ float red[4];
  const long long row = blockIdx.x;
  const uint16_t* z = logits + row * V;
  float mx = -INFINITY, sum = 0.f;
  const int V8n = V >> 3;
  for (int i = threadIdx.x; i < V8n; i += NT) {  // online max/sum, 8 logits at a time
    const V8 a = ld8(z + i * 8);
    float lm = a.v[0];
#pragma unroll
    for (int e = 1; e < 8; ++e) lm = fmaxf(lm, a.v[e]);
    if (lm > mx) {
      sum *= __expf(mx - lm);
      mx = lm;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) sum += __expf(a.v[e] - mx);
  }
  for (int c = V8n * 8 + threadIdx.x; c < V; c += NT) {
    const float a = bf2f(z[c]);
    if (a > mx) {
      sum *= __expf(mx - a);
      mx = a;
    }
    sum += __expf(a - mx);
  }
  const float gmx = block_max(mx, red);
  sum = (mx == -INFINITY) ? 0.f : sum * __expf(mx - gmx);
  const float l = gmx + __logf(block_sum(sum, red));
  if (threadIdx.x == 0) {
    const long long y = labels[row];
    lse[row] = l;
    loss[row] = (y == ignore_index) ? 0.f : l - bf2f(z[y]);
  }
}

// dz = (softmax(z) - onehot(y)) * scale[0], in place on z.
__global__ __launch_bounds__(NT) void k_ce_bwd(uint16_t* __restrict__ logits, const long long* __restrict__ labels,
                                               const float* __restrict__ lse, const float* __restrict__ scale, int V,
                                               long long ignore_index) {
  const long long row = blockIdx.x;
  uint16_t* z = logits + row * V;
  const long long y = labels[row];
  const float sc = (y == ignore_index) ? 0.f : scale[0];
  const float l = lse[row];
  const int V8n = V >> 3;
  for (int i = threadIdx.x; i < V8n; i += NT) {
    V8 a = ld8(z + i * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = i * 8 + e;
      a.v[e] = (__expf(a.v[e] - l) - (c == y ? 1.f : 0.f)) * sc;
    }
    st8(z + i * 8, a);
  }
  for (int c = V8n * 8 + threadIdx.x; c < V; c += NT) z[c] = f2bf((__expf(bf2f(z[c]) - l) - (c == y ? 1.f : 0.f)) * sc);
}

inline unsigned grid_for(long long work, int per_block = NT) {
  long long g = (work + per_block - 1) / per_block;
  if (g > 256 * 64) g = 256 * 64;  // grid-stride beyond 64 blocks per CU
  if (g < 1) g = 1;
  return (unsigned)g;
}

// ---------------------------------------------------------------- transpose
// out[c][r] = in[r][c] for a [rows x cols] bf16 matrix (row strides ld_in /
// ld_out).  Keeps the transposed weight copies W^T of the Llama linears
// that make every dgrad GEMM K-contiguous (dX = dY (W^T)^T, the forward's
// operand layout) and the transposed activations of the K-contiguous dW.
// Register transpose, no LDS: each lane owns an 8x8 sub-tile -- eight 16-B
// row loads in flight, 32 v_perm_b32, eight 16-B column stores.  Output
// dword m of transposed row k is (R[2m][k], R[2m+1][k]): one byte permute of
// input dwords R[2m].d[k/2] and R[2m+1].d[k/2] (low or high halves).  Lane
// (g, ch) = (lane >> 3, lane & 7) takes rows 8g.., cols 8ch.. of its wave's
// 64x64 tile, so each load instruction reads eight full 128-B row segments
// and each store instruction writes eight full 128-B output-row segments.
// A block is 4 waves side by side: a 64 x 256 input tile.
__global__ __launch_bounds__(256) void k_transpose_bf16(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                                        long long rows, long long cols, long long ld_in,
                                                        long long ld_out, int vec) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long r = (long long)blockIdx.y * 64 + 8 * (lane >> 3);
  const long long c = ((long long)blockIdx.x * 4 + w) * 64 + 8 * (lane & 7);
  if (r >= rows || c >= cols) return;
  const bool full = vec && r + 8 <= rows && c + 8 <= cols;
  uint32_t a[8][4];
  if (full) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint4 v = *reinterpret_cast<const uint4*>(in + (r + i) * ld_in + c);
      a[i][0] = v.x; a[i][1] = v.y; a[i][2] = v.z; a[i][3] = v.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t lo = (r + i < rows && c + 2 * d < cols) ? in[(r + i) * ld_in + c + 2 * d] : 0u;
        const uint32_t hi = (r + i < rows && c + 2 * d + 1 < cols) ? in[(r + i) * ld_in + c + 2 * d + 1] : 0u;
        a[i][d] = lo | (hi << 16);
      }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t sel = (k & 1) ? 0x07060302u : 0x05040100u;  // high / low halves of both dwords
    uint32_t o[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) o[m] = __builtin_amdgcn_perm(a[2 * m + 1][k >> 1], a[2 * m][k >> 1], sel);
    if (full) {
      *reinterpret_cast<uint4*>(out + (c + k) * ld_out + r) = make_uint4(o[0], o[1], o[2], o[3]);
    } else if (c + k < cols) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (r + e < rows) out[(c + k) * ld_out + r + e] = (uint16_t)((e & 1) ? (o[e >> 1] >> 16) : (o[e >> 1] & 0xffffu));
    }
  }
}

// out[c][r] = in[r][c] for a [rows x cols] bf16 matrix (row strides ld_in /
// ld_out).  Keeps the transposed weight copies W^T of the Llama linears
// that make every dgrad GEMM K-contiguous (dX = dY (W^T)^T, the forward's
// operand layout).  64x64 tile per 256-thread block through LDS.  Global
// loads AND stores are 8 lanes per 128-byte row (16 B each).  LDS image:
// 128-B rows, 16-B chunk c of row r stored at chunk c ^ ((r >> 3) & 7), so
// the column reads (8 consecutive rows 8k..8k+7 of one column per lane,
// k = lane & 7) of a wave fall on 32 distinct banks.
}  // namespace

#define PTO_API extern "C" __attribute__((visibility("default")))

// Errors: -1 = unsupported shape (D % 8 != 0 or D > 8192).
PTO_API int pto_add_rmsnorm_fwd(const void* x, const void* r, const void* w, void* h, void* y, float* rstd, long long M,
                                int D, float eps, hipStream_t s) {
  if (D % 8 || D > RMS_MAXV * NT * 8) return -1;
  if (M <= 0) return 0;
  if (r)
    hipLaunchKernelGGL(k_add_rmsnorm_fwd<true>, dim3((unsigned)M), dim3(NT), 0, s, (const uint16_t*)x,
                       (const uint16_t*)r, (const uint16_t*)w, (uint16_t*)h, (uint16_t*)y, rstd, D, eps);
  else
    hipLaunchKernelGGL(k_add_rmsnorm_fwd<false>, dim3((unsigned)M), dim3(NT), 0, s, (const uint16_t*)x, nullptr,
                       (const uint16_t*)w, nullptr, (uint16_t*)y, rstd, D, eps);
  return (int)hipGetLastError();
}

// part must hold G*D floats with G = pto_rmsnorm_bwd_groups(M).
PTO_API int pto_rmsnorm_bwd_groups(long long M) { return (int)(M < 1024 ? (M < 1 ? 1 : M) : 1024); }

PTO_API int pto_rmsnorm_bwd(const void* dy, const void* h, const void* w, const float* rstd, const void* dres, void* dx,
                            void* dw, float* part, long long M, int D, hipStream_t s) {
  if (D % 8 || D > RMS_MAXV * NT * 8) return -1;
  if (M <= 0) return 0;
  const int G = pto_rmsnorm_bwd_groups(M);
  const int V = (D + 8 * NT - 1) / (8 * NT);
  auto* kb = V <= 1 ? k_rmsnorm_bwd<1> : V == 2 ? k_rmsnorm_bwd<2> : V == 3 ? k_rmsnorm_bwd<3> : k_rmsnorm_bwd<4>;
  hipLaunchKernelGGL(kb, dim3(G), dim3(NT), 0, s, (const uint16_t*)dy, (const uint16_t*)h, (const uint16_t*)w, rstd,
                     (const uint16_t*)dres, (uint16_t*)dx, part, (int)M, D);
  hipLaunchKernelGGL(k_colsum_bf16, dim3((D + 63) / 64), dim3(NT), 0, s, part, (uint16_t*)dw, G, D);
  return (int)hipGetLastError();
}

PTO_API int pto_swiglu_fwd(const void* gu, void* out, long long M, int F, hipStream_t s) {
  if (F % 8) return -1;
  hipLaunchKernelGGL(k_swiglu_fwd, dim3(grid_for(M * (F / 8))), dim3(NT), 0, s, (const uint16_t*)gu, (uint16_t*)out,
                     M, F);
  return (int)hipGetLastError();
}

PTO_API int pto_swiglu_bwd(const void* gu, const void* dout, void* dgu, long long M, int F, hipStream_t s) {
  if (F % 8) return -1;
  hipLaunchKernelGGL(k_swiglu_bwd, dim3(grid_for(M * (F / 8))), dim3(NT), 0, s, (const uint16_t*)gu,
                     (const uint16_t*)dout, (uint16_t*)dgu, M, F);
  return (int)hipGetLastError();
}

// dgu_t: [2F][M] (row stride M, M % 8 == 0 for the vector stores' alignment).
PTO_API int pto_swiglu_bwd_t(const void* gu, const void* dout, void* dgu, void* dgu_t, long long M, int F,
                             hipStream_t s) {
  if (F % SWT || M < 1 || M % 8 || (((uintptr_t)dgu_t) & 15)) return -1;
  const long long blocks = ((M + SWT_M - 1) / SWT_M) * (F / SWT);
  if (blocks > 0x7fffffff) return -1;
  hipLaunchKernelGGL(k_swiglu_bwd_t, dim3((unsigned)blocks), dim3(NT), 0, s, (const uint16_t*)gu,
                     (const uint16_t*)dout, (uint16_t*)dgu, (uint16_t*)dgu_t, M, F);
  return (int)hipGetLastError();
}

// out == nullptr: in place on the first nrot heads.  Otherwise out receives
// every one of the nh heads (rotated or copied).
PTO_API int pto_rope(const void* qkv, void* out, const float* cs, const float* sn, long long M, int S, int nrot,
                     int nh, int D, long long row_stride, int backward, hipStream_t s) {
  if (D % 8) return -1;
  const int heads = out ? nh : nrot;
  hipLaunchKernelGGL(k_rope, dim3(grid_for(M * heads * (D / 8))), dim3(NT), 0, s, (const uint16_t*)qkv,
                     out ? (uint16_t*)out : (uint16_t*)qkv, cs, sn, M, S, nrot, heads, D, row_stride,
                     backward ? -1.f : 1.f);
  return (int)hipGetLastError();
}

PTO_API int pto_ce_fwd(const void* logits, const long long* labels, float* lse, float* loss, long long M, int V,
                       long long ignore_index, hipStream_t s) {
  if (V % 8) return -1;
  if (M <= 0) return 0;
  hipLaunchKernelGGL(k_ce_fwd, dim3((unsigned)M), dim3(NT), 0, s, (const uint16_t*)logits, labels, lse, loss, V,
                     ignore_index);
  return (int)hipGetLastError();
}

PTO_API int pto_ce_bwd(void* logits, const long long* labels, const float* lse, const float* scale, long long M, int V,
                       long long ignore_index, hipStream_t s) {
  if (V % 8) return -1;
  if (M <= 0) return 0;
  hipLaunchKernelGGL(k_ce_bwd, dim3((unsigned)M), dim3(NT), 0, s, (uint16_t*)logits, labels, lse, scale, V,
                     ignore_index);
  return (int)hipGetLastError();
}

// out = in^T (bf16, [rows x cols] -> [cols x rows]); 16-byte vector path
// when both pointers are 16-B aligned and both row strides are multiples of
// 8 elements, element-wise edges.
PTO_API int pto_transpose_bf16(const void* in, void* out, long long rows, long long cols, long long ld_in,
                               long long ld_out, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return 0;
  if (ld_in < cols || ld_out < rows || (cols + 255) / 256 > 0x7fffffff || (rows + 63) / 64 > 65535) return -1;
  const int vec = !(((((uintptr_t)in) | ((uintptr_t)out)) & 15) || (ld_in & 7) || (ld_out & 7));
  dim3 grid((unsigned)((cols + 255) / 256), (unsigned)((rows + 63) / 64));
  hipLaunchKernelGGL(k_transpose_bf16, grid, dim3(256), 0, s, reinterpret_cast<const uint16_t*>(in),
                     reinterpret_cast<uint16_t*>(out), rows, cols, ld_in, ld_out, vec);
  return (int)hipGetLastError();
}
