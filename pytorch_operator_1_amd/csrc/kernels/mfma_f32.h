// fp32 MFMA tile machinery for gfx950 (CDNA4).
//
// All training math in this package is exact fp32 (the reference trains in
// fp32, examples/mnist/mnist.py), so GEMM-shaped work runs on
// v_mfma_f32_16x16x4_f32: 16x16 output tile per wave, K=4 per instruction,
// 32-cycle issue / 40-cycle dependent latency -> every wave keeps two
// independent accumulator chains so the matrix pipe never waits on itself.
//
// Operand lane maps (cdna_hip_programming.md §3):
//   A: lane l holds A[i = l&15][k = l>>4]
//   B: lane l holds B[k = l>>4][j = l&15]
//   C/D: lane l, reg r -> row (l>>4)*4 + r, col l&15
//
// The K order inside a group of four MFMAs is free (a sum is a sum), so a
// lane streams FOUR CONSECUTIVE k of its own row/col per group:
//   MFMA j of a group uses k = k0 + 4*(l>>4) + j
// which turns K-contiguous operands into one 16-byte load per lane per
// group instead of four strided 4-byte loads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define PTO_DEV __device__ __forceinline__

PTO_DEV f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

PTO_DEV f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// Operand layouts.  For A ("rows" = M): MK = a[m*ld + k] (K contiguous),
// KM = a[k*ld + m].  For B ("rows" = N): NK = b[n*ld + k], KN = b[k*ld + n].
enum { LAY_ROWK = 0, LAY_KROW = 1 };

// Load the 4 consecutive-k operand values for one lane.  `row` is the
// M index (A) or N index (B) this lane owns; rows >= R and k >= K read 0.
// VEC (ROWK only): the caller guarantees ld % 4 == 0, K % 4 == 0 and a
// 16-byte aligned base, so every group is one float4 load with no per-lane
// alignment branch (a divergent branch there serialises the prefetch).
template <int LAY, bool VEC = false>
PTO_DEV void load4(const float* __restrict__ p, int ld, int row, int R, int k0, int K, float v[4]) {
  if (LAY == LAY_ROWK && VEC) {
    const bool ok = row < R && k0 < K;
    const float4 t = *reinterpret_cast<const float4*>(p + (ok ? (size_t)row * ld + k0 : 0));
    v[0] = ok ? t.x : 0.f; v[1] = ok ? t.y : 0.f; v[2] = ok ? t.z : 0.f; v[3] = ok ? t.w : 0.f;
    return;
  }
  if (row >= R) {
    v[0] = v[1] = v[2] = v[3] = 0.f;
    return;
  }
  if (LAY == LAY_ROWK) {
    const float* q = p + (size_t)row * ld + k0;
    if (k0 + 3 < K && ((ld & 3) == 0) && ((((uintptr_t)q) & 15) == 0)) {
      const float4 t = *reinterpret_cast<const float4*>(q);
      v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (k0 + j < K) ? q[j] : 0.f;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (k0 + j < K) ? p[(size_t)(k0 + j) * ld + row] : 0.f;
  }
}

// One wave: 16x16 tile at (m0, n0) of C = A * B over k in [kb, ke).
// kb must be a multiple of 4 (it is always a multiple of 16 here).
//
// These GEMMs are tiny and their operands were just written by the
// previous kernel (often on another XCD), so every load is a ~1 us trip to
// the Infinity Cache.  The loop therefore issues the operands of NG
// 16-deep k-groups (NG*8 loads per lane) before the first MFMA: one memory
// round trip per 16*NG of K instead of one per 16.
template <int AL, int BL, int NG = 8, bool AV = false, bool BV = false>
PTO_DEV f32x4 wave_tile_16x16(const float* __restrict__ A, int lda, const float* __restrict__ B, int ldb,
                              int M, int N, int K, int m0, int n0, int kb, int ke) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  f32x4 acc0 = zero4(), acc1 = zero4();
  const int kend = ke < K ? ke : K;
  for (int k = kb; k < kend; k += 16 * NG) {
    float a[NG][4], b[NG][4];
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      load4<AL, AV>(A, lda, m0 + r, M, k + 16 * q + 4 * g, kend, a[q]);
      load4<BL, BV>(B, ldb, n0 + r, N, k + 16 * q + 4 * g, kend, b[q]);
    }
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      acc0 = mfma16x16x4(a[q][0], b[q][0], acc0);
      acc1 = mfma16x16x4(a[q][1], b[q][1], acc1);
      acc0 = mfma16x16x4(a[q][2], b[q][2], acc0);
      acc1 = mfma16x16x4(a[q][3], b[q][3], acc1);
    }
  }
  return acc0 + acc1;
}

// Block of 4 waves, each wave an independent 16x16 tile over the full K.
// `vbid` is the virtual block id inside a multi-part launch.
template <int AL, int BL, class Epi, int NG = 8>
PTO_DEV void block_gemm_4tiles(const float* A, int lda, const float* B, int ldb, int M, int N, int K, int vbid,
                               Epi epi) {
  const int mtiles = (M + 15) >> 4, ntiles = (N + 15) >> 4;
  const int tile = vbid * 4 + (threadIdx.x >> 6);
  if (tile >= mtiles * ntiles) return;
  const int mt = tile % mtiles, nt = tile / mtiles;
  f32x4 acc = wave_tile_16x16<AL, BL, NG>(A, lda, B, ldb, M, N, K, mt * 16, nt * 16, 0, K);
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int m = mt * 16 + (lane >> 4) * 4 + rr, n = nt * 16 + (lane & 15);
    if (m < M && n < N) epi(m, n, acc[rr]);
  }
}

// Block of KS waves (blockDim = 64*KS) cooperating on ONE 16x16 tile: K
// split KS ways, partial tiles reduced through LDS, epilogue by the first
// 256 threads (one output element each).  `red` >= KS*256 floats.
template <int AL, int BL, class Epi, int KS = 4, bool AV = false, bool BV = false>
PTO_DEV void block_gemm_splitk(const float* A, int lda, const float* B, int ldb, int M, int N, int K, int vbid,
                               float* red, Epi epi) {
  const int mtiles = (M + 15) >> 4;
  const int mt = vbid % mtiles, nt = vbid / mtiles;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kc = (((K + KS - 1) / KS) + 15) & ~15;
  f32x4 acc = wave_tile_16x16<AL, BL, 8, AV, BV>(A, lda, B, ldb, M, N, K, mt * 16, nt * 16, w * kc, (w + 1) * kc);
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) red[w * 256 + ((lane >> 4) * 4 + rr) * 16 + (lane & 15)] = acc[rr];
  __syncthreads();
  const int t = threadIdx.x;
  if (t < 256) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < KS; ++q) v += red[q * 256 + t];
    const int m = mt * 16 + (t >> 4), n = nt * 16 + (t & 15);
    if (m < M && n < N) epi(m, n, v);
  }
}

template <int AL, int BL, class Epi>
PTO_DEV void block_gemm_splitk4(const float* A, int lda, const float* B, int ldb, int M, int N, int K, int vbid,
                                float* red, Epi epi) {
  block_gemm_splitk<AL, BL, Epi, 4>(A, lda, B, ldb, M, N, K, vbid, red, epi);
}

// Column sums out[n] = sum_m x[m*ld + n] for 64 consecutive columns per
// block of 256 threads: 4 row-groups x 64 columns, loads issued 16 rows at
// a time, LDS combine.  `red` >= 256 floats.
PTO_DEV void block_colsum64(const float* __restrict__ x, int ld, int M, int N, int col0, float* red,
                            float* __restrict__ out, float scale = 1.f) {
  const int t = threadIdx.x, c = col0 + (t & 63), rg = t >> 6;
  float s = 0.f;
  if (c < N) {
    for (int m0 = rg; m0 < M; m0 += 64) {
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + 4 * q;
        v[q] = m < M ? x[(size_t)m * ld + c] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) s += v[q];
    }
  }
  red[t] = s;
  __syncthreads();
  if (t < 64 && c < N) out[c] = (red[t] + red[t + 64] + red[t + 128] + red[t + 192]) * scale;
}

// Same column sums, handed to epi(0, column, sum) instead of stored.
template <class Epi>
PTO_DEV void block_colsum64_epi(const float* __restrict__ x, int ld, int M, int N, int col0, float* red, Epi epi) {
  const int t = threadIdx.x, c = col0 + (t & 63), rg = t >> 6;
  float s = 0.f;
  if (c < N) {
    for (int m0 = rg; m0 < M; m0 += 64) {
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + 4 * q;
        v[q] = m < M ? x[(size_t)m * ld + c] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) s += v[q];
    }
  }
  red[t] = s;
  __syncthreads();
  if (t < 64 && c < N) epi(0, c, red[t] + red[t + 64] + red[t + 128] + red[t + 192]);
}

// Cross-lane exchanges on the VALU (DPP) and the gfx950 permlane swaps,
// instead of __shfl_xor's ds_bpermute (an LDS-crossbar round trip per step:
// a dependent reduction of 6 steps waits ~6 of them).
//   lane_xor1 / lane_xor2: quad_perm;  lane_xor8: row_ror:8 (= xor 8 in a
//   16-lane row);  lane_mirror8: row_half_mirror (lane i <- i ^ 7 in a group
//   of 8) -- a valid partner for a reduction step on bit 2, since i ^ 7
//   differs from i in that bit and the sets being merged stay disjoint.
#define PTO_DPP(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), (ctrl), 0xF, 0xF, false))
PTO_DEV float lane_xor1(float v) { return PTO_DPP(v, 0xB1); }     // quad_perm [1,0,3,2]
PTO_DEV float lane_xor2(float v) { return PTO_DPP(v, 0x4E); }     // quad_perm [2,3,0,1]
PTO_DEV float lane_mirror8(float v) { return PTO_DPP(v, 0x141); } // row_half_mirror
PTO_DEV float lane_xor8(float v) { return PTO_DPP(v, 0x128); }    // row_ror:8
// x + (x of lane ^ 32), in every lane (v_permlane32_swap)
PTO_DEV float lane_sum32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// One halving step across lane bit 5 (or, with permlane16, bit 4): lanes
// with the bit clear keep slot a, the others slot b, and each adds its
// partner's copy of the slot it keeps: x keeps a's, y b's
// (v_permlane32_swap / v_permlane16_swap exchange exactly those halves).
PTO_DEV float halve32(float a, float b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
PTO_DEV float halve16(float a, float b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// all-reduce (sum / max) over the 16-lane rows
PTO_DEV float row16_sum(float v) {
  v += lane_xor8(v);
  v += lane_mirror8(v);
  v += lane_xor2(v);
  return v + lane_xor1(v);
}
PTO_DEV float row16_max(float v) {
  v = fmaxf(v, lane_xor8(v));
  v = fmaxf(v, lane_mirror8(v));
  v = fmaxf(v, lane_xor2(v));
  return fmaxf(v, lane_xor1(v));
}

PTO_DEV float wave_sum(float v) {
  v = lane_sum32(v);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return row16_sum(__uint_as_float(r[0]) + __uint_as_float(r[1]));
}

PTO_DEV float wave_max(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return row16_max(fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1])));
}
