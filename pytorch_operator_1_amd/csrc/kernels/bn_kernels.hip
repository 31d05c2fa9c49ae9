// Fused training-mode BatchNorm (+ residual add) (+ ReLU) for channels-last
// bf16 activations, fp32 statistics / affine parameters (ResNet-50, BASELINE
// config 3).
//
// Why: in the ResNet-50 bf16 step MIOpen's NHWC batch-norm kernels plus the
// separate ReLU / residual-add / ReLU-backward elementwise passes were 60 %
// of the kernel time (profiles/resnet50_window_r1.md: BN 15.7 ms + 6.6 ms
// elementwise of 40 ms).  Here every BN layer is
//   forward : stats (1 read) -> finalize (per channel) -> apply (1 read,
//             + residual read, 1 write; ReLU and the add in the same pass)
//   backward: reduce (reads dy, x [, y]; for the residual variant also writes
//             g = dy * relu-mask, which IS the identity branch's gradient)
//             -> finalize -> apply (dx = k1*g + k2*x + k3)
// with the ReLU mask recomputed from x (no saved mask, no extra pass).
//
// Layout: x is [M = N*H*W][C] (channels_last memory), C = 8 * 2^k <= 2048,
// so a row is C/8 threads of 16-byte bf16x8 loads and a 256-thread block
// covers 2048/C rows per iteration: every access is a coalesced 16-byte
// vector.  Per-block partial sums (fp32, <= a few hundred rows per thread)
// are combined per channel in fp64 by the finalize kernels, so E[x^2] -
// E[x]^2 keeps full precision.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace {

constexpr int BN_T = 256;
constexpr int BN_U = 8;     // loads in flight per thread in the reduction kernels
constexpr int BN_FT = 1024;  // finalize block: 32 channels x 32 partial groups

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // round to nearest even
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

struct V8 {
  float v[8];
};
__device__ __forceinline__ V8 load8(const uint16_t* p) {
  const uint4 r = *reinterpret_cast<const uint4*>(p);
  V8 o;
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o.v[2 * j] = __uint_as_float(w[j] << 16);
    o.v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
  return o;
}
__device__ __forceinline__ uint4 store8(uint16_t* p, const V8& a) {
  uint4 r;
  r.x = (uint32_t)f2bf(a.v[0]) | ((uint32_t)f2bf(a.v[1]) << 16);
  r.y = (uint32_t)f2bf(a.v[2]) | ((uint32_t)f2bf(a.v[3]) << 16);
  r.z = (uint32_t)f2bf(a.v[4]) | ((uint32_t)f2bf(a.v[5]) << 16);
  r.w = (uint32_t)f2bf(a.v[6]) | ((uint32_t)f2bf(a.v[7]) << 16);
  *reinterpret_cast<uint4*>(p) = r;
  return r;
}
__device__ __forceinline__ V8 loadf8(const float* p) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  return V8{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
}

// Block-level combine of per-thread 8-channel partials (s, q) over the
// row groups of the block; thread layout: tid = rsub * tpr + col.
__device__ __forceinline__ void block_combine(const float (&s)[8], const float (&q)[8], int C, float* red,
                                              float* __restrict__ out_s, float* __restrict__ out_q) {
  const int tpr = C >> 3, rpi = BN_T / tpr, tid = threadIdx.x, rsub = tid / tpr, c8 = (tid - rsub * tpr) * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[rsub * C + c8 + j] = s[j];
    red[2048 + rsub * C + c8 + j] = q[j];
  }
  __syncthreads();
  for (int c = tid; c < C; c += BN_T) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rpi; ++r) {
      a += red[r * C + c];
      b += red[2048 + r * C + c];
    }
    out_s[c] = a;
    out_q[c] = b;
  }
}

// Per-block sums of x and x^2 per channel -> part[blk][2][C].
__global__ __launch_bounds__(BN_T) void k_bn_stats(const uint16_t* __restrict__ x, long long M, int C, int iters,
                                                   float* __restrict__ part) {
  __shared__ float red[4096];
  const int tpr = C >> 3, rpi = BN_T / tpr, tid = threadIdx.x, rsub = tid / tpr, c8 = (tid - rsub * tpr) * 8;
  float s[8] = {}, q[8] = {};
  const long long r0 = (long long)blockIdx.x * iters * rpi + rsub;
  for (int it = 0; it < iters; it += BN_U) {  // BN_U independent 16-byte loads in flight
    V8 a[BN_U];
    bool ok[BN_U];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {  // unconditional loads (row 0 when out of range), masked below
      const long long row = r0 + (long long)(it + u) * rpi;
      ok[u] = it + u < iters && row < M;
      a[u] = load8(x + (ok[u] ? row : 0) * C + c8);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = ok[u] ? a[u].v[j] : 0.f;
        s[j] += v;
        q[j] = fmaf(v, v, q[j]);
      }
  }
  block_combine(s, q, C, red, part + (long long)blockIdx.x * 2 * C, part + (long long)blockIdx.x * 2 * C + C);
}

// Sum of the per-block partials of 32 channels (both the s and the q
// column) in fp64: thread = (column 0..63, group 0..15) sums every 16th
// block, then the 16 groups are combined in LDS.  Returns, for threads
// 0..31 of the block, (S, Q) of channel blockIdx.x * 32 + tid.
__device__ __forceinline__ void combine_partials(const float* __restrict__ part, int nblk, int C, double* red,
                                                 double& S, double& Q) {
  const int t = threadIdx.x, col = t & 63, grp = t >> 6;
  const int c = blockIdx.x * 32 + (col & 31);
  double acc = 0.0;
  if (c < C) {
    const float* p = part + (col >> 5) * C + c;
    // up to 2048 partial rows: 32 loads in flight per thread, then the adds
    int b = grp;
    for (; b + 31 * (BN_FT / 64) < nblk; b += 32 * (BN_FT / 64)) {
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = p[(long long)(b + u * (BN_FT / 64)) * 2 * C];
#pragma unroll
      for (int u = 0; u < 32; ++u) acc += (double)v[u];
    }
    for (; b < nblk; b += BN_FT / 64) acc += (double)p[(long long)b * 2 * C];
  }
  red[grp * 64 + col] = acc;
  __syncthreads();
  S = Q = 0.0;
  if (t < 32) {
    for (int g = 0; g < BN_FT / 64; ++g) {
      S += red[g * 64 + t];
      Q += red[g * 64 + 32 + t];
    }
  }
}

// Per channel: mean / rstd from the partials (fp64), the affine folded into
// scale/shift, running statistics (unbiased variance) and the batch counter.
__global__ __launch_bounds__(BN_FT) void k_bn_finalize(const float* __restrict__ part, int nblk, long long M, int C,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps, float momentum,
                                                       float* __restrict__ run_mean, float* __restrict__ run_var,
                                                       long long* __restrict__ nbt, float* __restrict__ stat) {
  __shared__ double red[BN_FT];
  double s, q;
  combine_partials(part, nblk, C, red, s, q);
  const int c = blockIdx.x * 32 + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
  if (threadIdx.x >= 32 || c >= C) return;
  const double mean = s / (double)M;
  double var = q / (double)M - mean * mean;
  var = var > 0.0 ? var : 0.0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * rstd;
  stat[c] = (float)mean;
  stat[C + c] = rstd;
  stat[2 * C + c] = sc;
  stat[3 * C + c] = beta[c] - (float)mean * sc;
  if (run_mean) {
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unb;
  }
}

// y = [relu](x * scale + shift [+ res]); EW_U vectors per thread iteration,
// all loads issued before the first use (RES/RELU are template parameters,
// out-of-range slots load vector 0 and are not stored).  mask (optional):
// one byte per 8-channel vector, bit j = (stored y_j > 0) -- the backward of
// relu(bn(x) + res) reads it instead of y (1/16 of the bytes).
constexpr int EW_U = 4;
template <bool RES, bool RELU>
__global__ __launch_bounds__(BN_T) void k_bn_apply(const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
                                                   uint16_t* __restrict__ y, long long n8, int C,
                                                   const float* __restrict__ stat, uint8_t* __restrict__ mask) {
  const long long stride = (long long)gridDim.x * BN_T;
  // the grid stride (gridDim.x * 2048 elements) is a multiple of C (a power
  // of two <= 2048): a thread's 8 channels never change, so its affine
  // coefficients are loaded once, not per vector
  const int c0 = (int)((((long long)blockIdx.x * BN_T + threadIdx.x) * 8) & (C - 1));
  const V8 sc = loadf8(stat + 2 * C + c0), sh = loadf8(stat + 3 * C + c0);
  for (long long i0 = (long long)blockIdx.x * BN_T + threadIdx.x; i0 < n8; i0 += EW_U * stride) {
    V8 a[EW_U], r[EW_U];
    long long ii[EW_U];
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      ii[u] = i0 + u * stride;
      const long long k = ii[u] < n8 ? ii[u] : 0;
      a[u] = load8(x + k * 8);
      if (RES) r[u] = load8(res + k * 8);
    }
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      if (ii[u] >= n8) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = fmaf(a[u].v[j], sc.v[j], sh.v[j]);
        if (RES) v += r[u].v[j];
        a[u].v[j] = RELU ? fmaxf(v, 0.f) : v;
      }
      const uint4 w = store8(y + ii[u] * 8, a[u]);
      if (mask) {
        const uint32_t h[4] = {w.x, w.y, w.z, w.w};
        uint32_t b = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          b |= (bf2f((uint16_t)(h[j] & 0xffffu)) > 0.f ? 1u : 0u) << (2 * j) |
               (bf2f((uint16_t)(h[j] >> 16)) > 0.f ? 1u : 0u) << (2 * j + 1);
        mask[ii[u]] = (uint8_t)b;
      }
    }
  }
}

// Backward reduction: g = dy * mask; per channel sums of g and g * xhat.
// mode 0: no ReLU; 1: ReLU, mask recomputed from x (x*scale+shift > 0);
// 2: ReLU after a residual add, mask = (y > 0) from the forward's bitmask,
// and g is stored (it is also the gradient of the residual input).
// MODE is a template parameter so every load of an unrolled group is
// issued before the first use (a runtime mode branch between them split the
// group); the row bound is clamped instead of predicated for the same reason.
template <int MODE>
__global__ __launch_bounds__(BN_T) void k_bn_bwd_reduce(const uint16_t* __restrict__ dy,
                                                        const uint16_t* __restrict__ x,
                                                        const uint8_t* __restrict__ ymask, long long M, int C,
                                                        int iters, const float* __restrict__ stat,
                                                        uint16_t* __restrict__ g_out, float* __restrict__ part) {
  __shared__ float red[4096];
  const int tpr = C >> 3, rpi = BN_T / tpr, tid = threadIdx.x, rsub = tid / tpr, c8 = (tid - rsub * tpr) * 8;
  const V8 mean = loadf8(stat + c8), rstd = loadf8(stat + C + c8);
  const V8 sc = loadf8(stat + 2 * C + c8), sh = loadf8(stat + 3 * C + c8);
  float s[8] = {}, q[8] = {};
  const long long r0 = (long long)blockIdx.x * iters * rpi + rsub;
  constexpr int U = BN_U;  // 16-byte loads in flight: 2 streams x U rows (+ U mask bytes in mode 2)
  for (int it = 0; it < iters; it += U) {
    V8 g[U], a[U];
    uint32_t mk[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = r0 + (long long)(it + u) * rpi;
      ok[u] = it + u < iters && row < M;
      const long long o = (ok[u] ? row : 0) * C + c8;  // row 0 when out of range: in bounds, masked below
      g[u] = load8(dy + o);
      a[u] = load8(x + o);
      if (MODE == 2) mk[u] = ymask[o >> 3];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) {
#pragma unroll
        for (int j = 0; j < 8; ++j) g[u].v[j] = 0.f, a[u].v[j] = 0.f;
      }
      if (MODE == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (!(fmaf(a[u].v[j], sc.v[j], sh.v[j]) > 0.f)) g[u].v[j] = 0.f;
      } else if (MODE == 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (!((mk[u] >> j) & 1u)) g[u].v[j] = 0.f;
        const long long row = r0 + (long long)(it + u) * rpi;
        if (ok[u]) store8(g_out + row * C + c8, g[u]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += g[u].v[j];
        q[j] = fmaf(g[u].v[j], (a[u].v[j] - mean.v[j]) * rstd.v[j], q[j]);
      }
    }
  }
  block_combine(s, q, C, red, part + (long long)blockIdx.x * 2 * C, part + (long long)blockIdx.x * 2 * C + C);
}

// dbeta = sum g, dgamma = sum g*xhat; dx = k1*g + k2*x + k3 coefficients.
__global__ __launch_bounds__(BN_FT) void k_bn_bwd_finalize(const float* __restrict__ part, int nblk, long long M,
                                                           int C, const float* __restrict__ gamma,
                                                           const float* __restrict__ stat,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                           float* __restrict__ coef) {
  __shared__ double red[BN_FT];
  double s, q;
  combine_partials(part, nblk, C, red, s, q);
  const int c = blockIdx.x * 32 + threadIdx.x;
  if (threadIdx.x >= 32 || c >= C) return;
  const float mean = stat[c], rstd = stat[C + c];
  dbeta[c] = (float)s;
  dgamma[c] = (float)q;
  const double k1 = (double)gamma[c] * rstd;
  const double k2 = -k1 * rstd * q / (double)M;
  const double k3 = -k1 * s / (double)M - k2 * mean;
  coef[c] = (float)k1;
  coef[C + c] = (float)k2;
  coef[2 * C + c] = (float)k3;
}

// dx = k1 * g + k2 * x + k3 with g = dy (mode 0), dy * relu-mask recomputed
// from x (mode 1) or the stored g (mode 2, passed as gsrc); EW_U vectors per
// thread iteration, loads first.
template <int MODE>
__global__ __launch_bounds__(BN_T) void k_bn_bwd_apply(const uint16_t* __restrict__ gsrc,
                                                       const uint16_t* __restrict__ x, uint16_t* __restrict__ dx,
                                                       long long n8, int C, const float* __restrict__ stat,
                                                       const float* __restrict__ coef) {
  const long long stride = (long long)gridDim.x * BN_T;
  // fixed channels per thread (see k_bn_apply): coefficients loaded once
  const int c0 = (int)((((long long)blockIdx.x * BN_T + threadIdx.x) * 8) & (C - 1));
  const V8 k1 = loadf8(coef + c0), k2 = loadf8(coef + C + c0), k3 = loadf8(coef + 2 * C + c0);
  V8 sc{}, sh{};
  if (MODE == 1) sc = loadf8(stat + 2 * C + c0), sh = loadf8(stat + 3 * C + c0);
  for (long long i0 = (long long)blockIdx.x * BN_T + threadIdx.x; i0 < n8; i0 += EW_U * stride) {
    V8 g[EW_U], a[EW_U];
    long long ii[EW_U];
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      ii[u] = i0 + u * stride;
      const long long k = ii[u] < n8 ? ii[u] : 0;
      g[u] = load8(gsrc + k * 8);
      a[u] = load8(x + k * 8);
    }
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      if (ii[u] >= n8) continue;
      if (MODE == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (!(fmaf(a[u].v[j], sc.v[j], sh.v[j]) > 0.f)) g[u].v[j] = 0.f;
      }
      V8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o.v[j] = fmaf(k1.v[j], g[u].v[j], fmaf(k2.v[j], a[u].v[j], k3.v[j]));
      store8(dx + ii[u] * 8, o);
    }
  }
}

bool bn_shape_ok(long long M, int C) {
  if (M < 1 || C < 8 || C > 2048 || (C & 7)) return false;
  const int tpr = C >> 3;
  return (tpr & (tpr - 1)) == 0;  // power of two <= 256
}

// Reduction grid.  These passes stream HBM, so what matters is bytes in
// flight: BN_U 16-byte loads per thread x resident threads.  Each block
// streams one contiguous slab of rows; interleaving the blocks' rows (one
// 4 KB chunk per block per iteration, a grid-wide contiguous window)
// measured slower in round 4: stats 3.94 -> 3.78 TB/s and the ReLU backward
// reduce 4.83 -> 3.99 TB/s at 411 MB (profiles/bn_r4.md).  Round 1 capped
// the grid at 512 blocks (256 at C = 2048: one 4-wave block per CU) and ran
// at ~40 % of HBM bandwidth; the default now allows 1024 blocks (4 per CU)
// with >= 8 row iterations each, partials bounded to 4 M floats (16 MB).
void bn_grid(long long M, int C, int* nblk, int* iters) {
  constexpr int maxblk = 1024, minit = 8;
  const int rpi = BN_T / (C >> 3);
  const long long rows_iters = (M + rpi - 1) / rpi;
  long long nb = (rows_iters + minit - 1) / minit;
  const long long cap = 4194304 / C < maxblk ? 4194304 / C : maxblk;
  if (nb > cap) nb = cap;
  if (nb < 1) nb = 1;
  *nblk = (int)nb;
  *iters = (int)((rows_iters + nb - 1) / nb);
}

int elementwise_blocks(long long n8) {
  long long b = (n8 + BN_T * EW_U - 1) / (BN_T * EW_U);  // ~EW_U vectors per thread
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}


// ------------------------------------------------------------ max pool ----
// The ResNet stem's 3x3 / stride-2 / pad-1 max pool over channels-last bf16
// (relu(bn1(conv1)) -> layer1), forward and backward, 8 channels (16 B) per
// thread.  Forward writes the pooled map and one argmax code per output
// element (tap index kh*K+kw, uint8); backward is a GATHER: every input
// element sums dy over the (<= 4 at stride 2) windows whose code points at
// it, so there are no atomics and no zero-fill of dx (PyTorch's NHWC kernels
// took 0.62 + 0.25 ms/step for this, profiles/resnet50_window_r4.md).
// Semantics of torch.nn.functional.max_pool2d: padding never wins, the first
// maximum in (kh, kw) order wins a tie, NaN propagates.
struct PoolShape {
  int N, H, W, C, OH, OW, K, S, P;
};

__global__ __launch_bounds__(BN_T) void k_maxpool_fwd(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                      uint8_t* __restrict__ code, PoolShape sh) {
  // 32-bit index math (the launcher checks the element count fits): the
  // 64-bit divisions of the first version were most of the kernel's time
  const uint32_t c8n = (uint32_t)sh.C >> 3;
  const uint32_t t = blockIdx.x * BN_T + threadIdx.x;
  if (t >= (uint32_t)sh.N * sh.OH * sh.OW * c8n) return;
  const int c8 = (int)(t % c8n);
  uint32_t pix = t / c8n;
  const int ow = (int)(pix % (uint32_t)sh.OW);
  pix /= (uint32_t)sh.OW;
  const int oh = (int)(pix % (uint32_t)sh.OH);
  const int n = (int)(pix / (uint32_t)sh.OH);
  // torch's loop: maxval = -inf, index = the first in-bounds tap, then
  // "if (val > maxval || isnan(val))" in (kh, kw) order
  const int h0 = oh * sh.S - sh.P, w0 = ow * sh.S - sh.P;
  const int kh0 = max(0, -h0), kw0 = max(0, -w0);
  float m[8];
  int k[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[j] = -__builtin_inff();
    k[j] = kh0 * sh.K + kw0;
  }
  for (int kh = kh0; kh < sh.K && h0 + kh < sh.H; ++kh)
    for (int kw = kw0; kw < sh.K && w0 + kw < sh.W; ++kw) {
      const V8 v = load8(x + (((long long)n * sh.H + h0 + kh) * sh.W + w0 + kw) * sh.C + c8 * 8);
      const int tap = kh * sh.K + kw;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (v.v[j] > m[j] || __builtin_isnan(v.v[j])) {
          m[j] = v.v[j];
          k[j] = tap;
        }
    }
  const long long o = (((long long)n * sh.OH + oh) * sh.OW + ow) * sh.C + c8 * 8;
  V8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r.v[j] = m[j];
  store8(y + o, r);
  uint2 cd;
  cd.x = (uint32_t)k[0] | ((uint32_t)k[1] << 8) | ((uint32_t)k[2] << 16) | ((uint32_t)k[3] << 24);
  cd.y = (uint32_t)k[4] | ((uint32_t)k[5] << 8) | ((uint32_t)k[6] << 16) | ((uint32_t)k[7] << 24);
  *reinterpret_cast<uint2*>(code + o) = cd;
}

__global__ __launch_bounds__(BN_T) void k_maxpool_bwd(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ code,
                                                      uint16_t* __restrict__ dx, PoolShape sh) {
  const uint32_t c8n = (uint32_t)sh.C >> 3;
  const uint32_t t = blockIdx.x * BN_T + threadIdx.x;
  if (t >= (uint32_t)sh.N * sh.H * sh.W * c8n) return;
  const int c8 = (int)(t % c8n);
  uint32_t pix = t / c8n;
  const int iw = (int)(pix % (uint32_t)sh.W);
  pix /= (uint32_t)sh.W;
  const int ih = (int)(pix % (uint32_t)sh.H);
  const int n = (int)(pix / (uint32_t)sh.H);
  // windows oh with oh*S - P <= ih <= oh*S - P + K - 1
  const int hp = ih + sh.P, wp = iw + sh.P;
  const int oh0 = hp >= sh.K ? (hp - sh.K) / sh.S + 1 : 0, oh1 = min(sh.OH - 1, hp / sh.S);
  const int ow0 = wp >= sh.K ? (wp - sh.K) / sh.S + 1 : 0, ow1 = min(sh.OW - 1, wp / sh.S);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int oh = oh0; oh <= oh1; ++oh)
    for (int ow = ow0; ow <= ow1; ++ow) {
      const int tap = (hp - oh * sh.S) * sh.K + (wp - ow * sh.S);
      const long long o = (((long long)n * sh.OH + oh) * sh.OW + ow) * sh.C + c8 * 8;
      const uint2 cd = *reinterpret_cast<const uint2*>(code + o);
      const V8 g = load8(dy + o);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t cj = ((j < 4 ? cd.x : cd.y) >> (8 * (j & 3))) & 0xffu;
        if ((int)cj == tap) acc[j] += g.v[j];
      }
    }
  V8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r.v[j] = acc[j];
  store8(dx + (((long long)n * sh.H + ih) * sh.W + iw) * sh.C + c8 * 8, r);
}


// ------------------------------------------------------------ the stem ----
// ResNet-50's first convolution (7x7, stride 2, pad 3, 3 -> 64 channels,
// 224 -> 112) over channels-last bf16, as an implicit GEMM on MFMA.  MIOpen
// ran it as an asm implicit GEMM after zero-filling the 411 MB output
// (0.36 + 0.09 ms/step, profiles/resnet50_r5.md).
//   GEMM: M = output pixels of one output row (112, padded to 4 x 32), N =
//   64 channels (2 x 32), K = 7 filter rows x 24: per filter row the 21 (kw,
//   c) taps at t = 1 + 3 kw + c, zero weights at t = 0, 22, 23, plus 8 zero
//   k at the end (176 = 11 MFMA k-steps of 16).
//   LDS: the 7 input rows of an output row, row element (iw + 3)*3 + c + 1,
//   so tap t of output pixel ow sits at element 6 ow + t: every A fragment
//   (8 consecutive k) is 4 dword reads, and a source row (224 x 3 bf16 =
//   336 dwords) lands 5 dwords in, dword-aligned on both sides.
//   Block = 4 waves, STEM_ROWS output rows; wave w owns output pixels
//   32w..32w+31 and both channel halves (2 accumulators); the weight
//   fragments (prepared once per step by k_stem_wprep) stay in registers
//   for all the block's rows; the next row's input is loaded into registers
//   while the current one computes; outputs leave through LDS as 16-byte
//   row stores.
typedef __bf16 stem_bf16x8 __attribute__((ext_vector_type(8)));
typedef float stem_f32x16 __attribute__((ext_vector_type(16)));
constexpr int STEM_KP = 176, STEM_RW = 696, STEM_ROWS = 8, STEM_OPITCH = 72;
constexpr int STEM_LOADS = (7 * 336 + 255) / 256;  // input dwords per thread per output row

// wp[co][k] (bf16) from the OIHW-indexed weight with arbitrary strides
__global__ __launch_bounds__(256) void k_stem_wprep(const float* __restrict__ w, long long s0, long long s1,
                                                    long long s2, long long s3, uint16_t* __restrict__ wp) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 64 * STEM_KP) return;
  const int co = i / STEM_KP, k = i - co * STEM_KP, kh = k / 24, t = k - kh * 24;
  float v = 0.f;
  if (kh < 7 && t >= 1 && t <= 21) {
    const int kw = (t - 1) / 3, c = (t - 1) - 3 * kw;
    v = w[co * s0 + c * s1 + kh * s2 + kw * s3];
  }
  wp[i] = f2bf(v);
}

__device__ __forceinline__ void stem_load_row(const uint32_t* __restrict__ x, int N, int r, uint32_t (&v)[STEM_LOADS]) {
  // the 7 input rows of output row r (= n*112 + oh), as dwords; 0 outside
  const int tid = threadIdx.x;
  const bool live = r < N * 112;
  const int n = live ? r / 112 : 0, oh = live ? r - n * 112 : 0;
#pragma unroll
  for (int q = 0; q < STEM_LOADS; ++q) {
    const int d = tid + 256 * q, kh = d / 336, j = d - kh * 336;
    const int ih = 2 * oh - 3 + kh;
    v[q] = (live && d < 7 * 336 && ih >= 0 && ih < 224) ? x[((long long)n * 224 + ih) * 336 + j] : 0u;
  }
}

__global__ __launch_bounds__(256) void k_stem_fwd(const uint16_t* __restrict__ x, const uint16_t* __restrict__ wp,
                                                  uint16_t* __restrict__ y, int N) {
  __shared__ __attribute__((aligned(16))) uint32_t in_s[(7 * STEM_RW + 96) / 2];
  __shared__ __attribute__((aligned(16))) uint16_t out_s[128 * STEM_OPITCH];
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  // zero the never-written dwords of every row once (pad and iw < 0 / >= 224)
  for (int i = tid; i < (7 * STEM_RW + 96) / 2; i += 256) in_s[i] = 0u;
  // weight fragments: B[k = 8(l>>5)+j][col = l&31], both channel halves
  stem_bf16x8 bf[2][11];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int s = 0; s < 11; ++s)
      bf[h][s] = *reinterpret_cast<const stem_bf16x8*>(wp + (32 * h + (lane & 31)) * STEM_KP + 16 * s + 8 * (lane >> 5));
  const int rows = N * 112;
  const int r0 = blockIdx.x * STEM_ROWS;
  const uint32_t* x32 = reinterpret_cast<const uint32_t*>(x);
  uint32_t nxt[STEM_LOADS];
  stem_load_row(x32, N, r0, nxt);
  const int ow = 32 * wv + (lane & 31);  // this lane's A row (output pixel)
  for (int rr = 0; rr < STEM_ROWS; ++rr) {
    const int r = r0 + rr;
    if (r >= rows) break;
    __syncthreads();  // the previous row's LDS reads / out_s reads are done
#pragma unroll
    for (int q = 0; q < STEM_LOADS; ++q) {
      const int d = tid + 256 * q, kh = d / 336, j = d - kh * 336;
      if (d < 7 * 336) in_s[kh * (STEM_RW / 2) + 5 + j] = nxt[q];
    }
    __syncthreads();
    if (rr + 1 < STEM_ROWS) stem_load_row(x32, N, r + 1, nxt);  // in flight while this row computes
    stem_f32x16 acc0 = {}, acc1 = {};
#pragma unroll
    for (int s = 0; s < 11; ++s) {
      const int k0 = 16 * s + 8 * (lane >> 5);
      const int kh = min(k0 / 24, 6), t0 = k0 - (k0 / 24) * 24;  // k >= 168: zero weights, any finite A
      const uint32_t* a = in_s + (kh * STEM_RW + 6 * ow + t0) / 2;
      const uint32_t av[4] = {a[0], a[1], a[2], a[3]};
      const stem_bf16x8 A = __builtin_bit_cast(stem_bf16x8, av);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, bf[0][s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, bf[1][s], acc1, 0, 0, 0);
    }
    // C: col = l&31 (channel), row = (i&3) + 8(i>>2) + 4(l>>5) (pixel in the wave's 32)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int px = 32 * wv + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      out_s[px * STEM_OPITCH + (lane & 31)] = f2bf(acc0[i]);
      out_s[px * STEM_OPITCH + 32 + (lane & 31)] = f2bf(acc1[i]);
    }
    __syncthreads();
    uint16_t* yr = y + (long long)r * 112 * 64;
    for (int c = tid; c < 112 * 8; c += 256) {  // 112 pixels x 8 chunks of 8 channels
      const int px = c >> 3, ch = c & 7;
      *reinterpret_cast<uint4*>(yr + px * 64 + 8 * ch) = *reinterpret_cast<const uint4*>(out_s + px * STEM_OPITCH + 8 * ch);
    }
  }
}

}  // namespace

#define PTO_API extern "C" __attribute__((visibility("default")))

// Scratch floats the launchers need for (M, C): partials.
PTO_API int pto_bn_scratch_floats(long long M, int C) {
  if (!bn_shape_ok(M, C)) return -1;
  int nblk, iters;
  bn_grid(M, C, &nblk, &iters);
  return nblk * 2 * C;  // <= 8 M floats (bn_grid caps nblk * C at 4 M)
}

// Forward: stat = [mean | rstd | scale | shift] (4*C floats, saved for the
// backward); res / run_mean / run_var / nbt may be null.
PTO_API int pto_bn_fwd(const void* x, const void* res, void* y, long long M, int C, const float* gamma,
                       const float* beta, float eps, float momentum, float* run_mean, float* run_var, long long* nbt,
                       float* stat, float* scratch, int relu, void* mask, hipStream_t s) {
  if (!bn_shape_ok(M, C)) return -1;
  if ((((uintptr_t)x) | ((uintptr_t)y) | ((uintptr_t)res)) & 15) return -1;
  int nblk, iters;
  bn_grid(M, C, &nblk, &iters);
  hipLaunchKernelGGL(k_bn_stats, dim3(nblk), dim3(BN_T), 0, s, reinterpret_cast<const uint16_t*>(x), M, C, iters,
                     scratch);
  hipLaunchKernelGGL(k_bn_finalize, dim3((C + 31) / 32), dim3(BN_FT), 0, s, scratch, nblk, M, C, gamma, beta,
                     eps, momentum, run_mean, run_var, nbt, stat);
  const long long n8 = M * C / 8;
  auto* ka = res ? (relu ? k_bn_apply<true, true> : k_bn_apply<true, false>)
                 : (relu ? k_bn_apply<false, true> : k_bn_apply<false, false>);
  hipLaunchKernelGGL(ka, dim3(elementwise_blocks(n8)), dim3(BN_T), 0, s, reinterpret_cast<const uint16_t*>(x),
                     reinterpret_cast<const uint16_t*>(res), reinterpret_cast<uint16_t*>(y), n8, C, stat,
                     reinterpret_cast<uint8_t*>(mask));
  return (int)hipGetLastError();
}

// Forward whose statistics pass already happened elsewhere: part holds
// nblk rows of [2][C] partial sums / sums of squares of x (the 3x3 conv's
// epilogue, conv3x3.hip), so only finalize + apply run.
PTO_API int pto_bn_fwd_part(const float* part, int nblk, const void* x, const void* res, void* y, long long M, int C,
                            const float* gamma, const float* beta, float eps, float momentum, float* run_mean,
                            float* run_var, long long* nbt, float* stat, int relu, void* mask, hipStream_t s) {
  if (!bn_shape_ok(M, C) || !part || nblk < 1) return -1;
  if ((((uintptr_t)x) | ((uintptr_t)y) | ((uintptr_t)res)) & 15) return -1;
  hipLaunchKernelGGL(k_bn_finalize, dim3((C + 31) / 32), dim3(BN_FT), 0, s, part, nblk, M, C, gamma, beta, eps,
                     momentum, run_mean, run_var, nbt, stat);
  const long long n8 = M * C / 8;
  auto* ka = res ? (relu ? k_bn_apply<true, true> : k_bn_apply<true, false>)
                 : (relu ? k_bn_apply<false, true> : k_bn_apply<false, false>);
  hipLaunchKernelGGL(ka, dim3(elementwise_blocks(n8)), dim3(BN_T), 0, s, reinterpret_cast<const uint16_t*>(x),
                     reinterpret_cast<const uint16_t*>(res), reinterpret_cast<uint16_t*>(y), n8, C, stat,
                     reinterpret_cast<uint8_t*>(mask));
  return (int)hipGetLastError();
}

// Backward.  mode 0/1/2 as k_bn_bwd_reduce; ymask (the forward's ReLU
// bitmask, M*C/8 bytes) needed for mode 2, where g_out (= d residual) is
// also written.  coef: 3*C floats scratch.
PTO_API int pto_bn_bwd(const void* dy, const void* x, const void* ymask, void* dx, void* g_out, long long M, int C,
                       const float* gamma, const float* stat, float* dgamma, float* dbeta, float* coef,
                       float* scratch, int mode, hipStream_t s) {
  if (!bn_shape_ok(M, C) || mode < 0 || mode > 2 || (mode == 2 && (!ymask || !g_out))) return -1;
  if ((((uintptr_t)dy) | ((uintptr_t)x) | ((uintptr_t)dx) | ((uintptr_t)g_out)) & 15) return -1;
  int nblk, iters;
  bn_grid(M, C, &nblk, &iters);
  auto* kr = mode == 0 ? k_bn_bwd_reduce<0> : (mode == 1 ? k_bn_bwd_reduce<1> : k_bn_bwd_reduce<2>);
  hipLaunchKernelGGL(kr, dim3(nblk), dim3(BN_T), 0, s, reinterpret_cast<const uint16_t*>(dy),
                     reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const uint8_t*>(ymask), M, C, iters, stat,
                     reinterpret_cast<uint16_t*>(g_out), scratch);
  hipLaunchKernelGGL(k_bn_bwd_finalize, dim3((C + 31) / 32), dim3(BN_FT), 0, s, scratch, nblk, M, C, gamma,
                     stat, dgamma, dbeta, coef);
  const long long n8 = M * C / 8;
  const void* gsrc = mode == 2 ? g_out : dy;
  auto* kb = mode == 1 ? k_bn_bwd_apply<1> : k_bn_bwd_apply<0>;  // mode 2 applies like 0 (g stored)
  hipLaunchKernelGGL(kb, dim3(elementwise_blocks(n8)), dim3(BN_T), 0, s, reinterpret_cast<const uint16_t*>(gsrc),
                     reinterpret_cast<const uint16_t*>(x), reinterpret_cast<uint16_t*>(dx), n8, C, stat, coef);
  return (int)hipGetLastError();
}

// Max pool (channels-last bf16, C % 8 == 0, K*K <= 255): y [N, OH, OW, C],
// code [N, OH, OW, C] uint8; backward dx [N, H, W, C] fully written.
static bool pool_ok(const PoolShape& sh, const void* a, const void* b) {
  return sh.N > 0 && sh.H > 0 && sh.W > 0 && sh.C > 0 && sh.C % 8 == 0 && sh.K > 0 && sh.K * sh.K <= 255 &&
         sh.S > 0 && sh.P >= 0 && 2 * sh.P <= sh.K && sh.OH == (sh.H + 2 * sh.P - sh.K) / sh.S + 1 &&
         sh.OW == (sh.W + 2 * sh.P - sh.K) / sh.S + 1 && sh.OH > 0 && sh.OW > 0 &&
         (long long)sh.N * sh.H * sh.W * sh.C < (1ll << 31) &&  // 32-bit element indices in the kernels
         !((((uintptr_t)a) | ((uintptr_t)b)) & 15);
}

PTO_API int pto_maxpool_fwd(const void* x, void* y, void* code, int N, int H, int W, int C, int OH, int OW, int K,
                            int S, int P, hipStream_t s) {
  const PoolShape sh{N, H, W, C, OH, OW, K, S, P};
  if (!pool_ok(sh, x, y) || (((uintptr_t)code) & 7)) return -1;
  const long long total = (long long)N * OH * OW * (C / 8);
  hipLaunchKernelGGL(k_maxpool_fwd, dim3((unsigned)((total + BN_T - 1) / BN_T)), dim3(BN_T), 0, s,
                     reinterpret_cast<const uint16_t*>(x), reinterpret_cast<uint16_t*>(y),
                     reinterpret_cast<uint8_t*>(code), sh);
  return (int)hipGetLastError();
}

PTO_API int pto_maxpool_bwd(const void* dy, const void* code, void* dx, int N, int H, int W, int C, int OH, int OW,
                            int K, int S, int P, hipStream_t s) {
  const PoolShape sh{N, H, W, C, OH, OW, K, S, P};
  if (!pool_ok(sh, dy, dx) || (((uintptr_t)code) & 7)) return -1;
  const long long total = (long long)N * H * W * (C / 8);
  hipLaunchKernelGGL(k_maxpool_bwd, dim3((unsigned)((total + BN_T - 1) / BN_T)), dim3(BN_T), 0, s,
                     reinterpret_cast<const uint16_t*>(dy), reinterpret_cast<const uint8_t*>(code),
                     reinterpret_cast<uint16_t*>(dx), sh);
  return (int)hipGetLastError();
}

// The ResNet stem conv (7x7 / 2 / pad 3, 3 -> 64, 224 -> 112) over
// channels-last bf16.  w: fp32 [64][3][7][7] indexed with element strides
// s0..s3; wp: 64*176 bf16 scratch (rebuilt every call: the weights change
// every step).
PTO_API int pto_stem_fwd(const void* x, const float* w, long long s0, long long s1, long long s2, long long s3,
                         void* wp, void* y, int N, hipStream_t s) {
  if (N < 1 || ((((uintptr_t)x) | ((uintptr_t)wp) | ((uintptr_t)y)) & 15)) return -1;
  hipLaunchKernelGGL(k_stem_wprep, dim3((64 * STEM_KP + 255) / 256), dim3(256), 0, s, w, s0, s1, s2, s3,
                     reinterpret_cast<uint16_t*>(wp));
  const int blocks = (N * 112 + STEM_ROWS - 1) / STEM_ROWS;
  hipLaunchKernelGGL(k_stem_fwd, dim3(blocks), dim3(256), 0, s, reinterpret_cast<const uint16_t*>(x),
                     reinterpret_cast<const uint16_t*>(wp), reinterpret_cast<uint16_t*>(y), N);
  return (int)hipGetLastError();
}
