// Causal GQA flash attention for gfx950 (bf16 in/out, fp32 accumulate),
// head_dim 128: forward, and backward as dK/dV + dQ kernels.  Replaces the
// ROCm SDPA path in the Llama-3 config (profiles/llama8b_step_rocprof.md:
// attention fwd+bwd was 4.3 ms/layer, 26 % of the step).
//
// Layout: Q/K/V are read in place from the fused QKV projection output
// ([tokens][(H + 2 Hkv) * 128], any row stride), O is written as
// [tokens][H * 128] (what the output projection consumes, no transpose),
// gradients dQ/dK/dV are written into a dQKV buffer of the QKV layout.
//
// MFMA: v_mfma_f32_32x32x16_bf16.  Lane maps (cdna_hip_programming.md §3):
// A[row l&31][k 8(l>>5)+j], B[k 8(l>>5)+j][col l&31], C col = l&31,
// row = (i&3) + 8(i>>2) + 4(l>>5).
//
// Forward / dQ structure ("swapped" products, every softmax quantity
// lane-local): a wave owns 32 query rows of one head; the block's 4 waves
// are the 4 query heads sharing one KV head (GQA group), so one K/V tile in
// LDS serves all of them.  S^T = K Q^T puts the query on the lane: row max /
// sum are 32 in-lane ops + one cross-half exchange.  O^T = V^T P^T keeps the
// query on the lane too, so the online-softmax rescale is a per-lane scalar.
// P^T's B operand is built in registers with v_cvt_pk_bf16_f32 +
// v_permlane32_swap; V^T's A operand comes from ds_read_b64_tr_b16
// transposed reads of the row-major V tile.  K/V tiles (64 keys) are
// register-staged from global memory one tile ahead into a 2-deep LDS ring
// with an XOR-swizzled image (conflict-free for b128 row reads and the
// transposed reads).
//
// dK/dV structure: a wave owns 32 keys (K and V fragments in registers,
// dK^T / dV^T accumulated in registers over every query row of the 4 heads
// of the group); S and dP are computed with the key on the lane, so their
// accumulators feed the dV^T / dK^T products through the same cvt+swap;
// the row constants -LSE and -delta are the accumulators' initial values.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int HD = 128;            // head dim
constexpr int QT = 32;             // query rows per wave
constexpr int KT = 64;             // keys per tile
constexpr int NW = 4;              // waves per block
constexpr int NT = NW * 64;
constexpr int TILE_B = KT * HD * 2;  // 16 KiB per K or V tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr float ATTN_DEFER = 8.f;  // forward: running-max slack (log2 units) before O is rescaled

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// XOR-swizzled [rows][256 B] image (cdna_hip_programming.md T10 image (b)):
// byte offset of 16-byte chunk ch (0..15) of row r.
__device__ __forceinline__ int swz(int r, int ch) { return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))); }

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ unsigned pack2(float a, float b) {
  bf16x2 t = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, t);
}

// Accumulator regs [8s .. 8s+7] of a 32x32 C tile whose row index runs
// over the MFMA k dimension of the next product -> that product's operand
// fragment for k-slot s (16 rows): lanes 0-31 need rows 16s+0..7, lanes
// 32-63 rows 16s+8..15; each half holds 4 of them, the partner the rest.
__device__ __forceinline__ bf16x8 acc_to_operand(const float* r) {
  unsigned x0 = pack2(r[0], r[1]), x1 = pack2(r[2], r[3]);
  unsigned y0 = pack2(r[4], r[5]), y1 = pack2(r[6], r[7]);
  auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
  auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
  u32x4 o = {s0[0], s1[0], s0[1], s1[1]};
  return __builtin_bit_cast(bf16x8, o);
}

// A (or B) operand with k running along the ROWS of a row-major LDS tile
// (keys for V^T, queries for dO^T / Q^T): two transposed reads.  Operand
// row index (d) = col0 + (lane & 31); k = krow0 + 8*(lane>>5) + j.
__device__ __forceinline__ bf16x8 tr_operand(const char* tile, int krow0, int col0) {
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int row = krow0 + 8 * (g >> 1) + (li >> 2);
  const int ch = ((col0 + 16 * (g & 1)) >> 3) + ((li & 3) >> 1);
  const char* p0 = tile + swz(row, ch) + 8 * (li & 1);
  const char* p1 = tile + swz(row + 4, ch) + 8 * (li & 1);
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p1);
  u32x2 ua = __builtin_bit_cast(u32x2, a), ub = __builtin_bit_cast(u32x2, b);
  u32x4 o = {ua[0], ua[1], ub[0], ub[1]};
  return __builtin_bit_cast(bf16x8, o);
}

// Row operand (k along the columns = head dim): 16 bytes of row
// r0 + (lane&31), chunk 2*ks + (lane>>5).
__device__ __forceinline__ bf16x8 row_operand(const char* tile, int r0, int ks) {
  const int lane = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8*>(tile + swz(r0 + (lane & 31), 2 * ks + (lane >> 5)));
}

// Cooperative tile copy global -> registers -> LDS (64 rows x 256 B):
// four 16-byte pieces per thread.  Kept as named scalars and loaded
// unconditionally (the last iteration re-reads its own tile): a
// conditionally-filled struct/array is demoted to scratch by hipcc and
// every load then waits vmcnt(0) before its scratch store.
template <int NTH = NT>
__device__ __forceinline__ uint4 tile_piece_load(const __bf16* base, long long rs, int p) {
  const int c = threadIdx.x + NTH * p, r = c >> 4, ch = c & 15;
  return *reinterpret_cast<const uint4*>(base + (long long)r * rs + ch * 8);
}
template <int NTH = NT>
__device__ __forceinline__ void tile_piece_store(char* tile, int p, uint4 v) {
  const int c = threadIdx.x + NTH * p, r = c >> 4, ch = c & 15;
  *reinterpret_cast<uint4*>(tile + swz(r, ch)) = v;
}
#define TILE_LOAD(R, base, rs)              \
  R##0 = tile_piece_load(base, rs, 0);      \
  R##1 = tile_piece_load(base, rs, 1);      \
  R##2 = tile_piece_load(base, rs, 2);      \
  R##3 = tile_piece_load(base, rs, 3)
#define TILE_STORE(R, tile)             \
  tile_piece_store(tile, 0, R##0);      \
  tile_piece_store(tile, 1, R##1);      \
  tile_piece_store(tile, 2, R##2);      \
  tile_piece_store(tile, 3, R##3)
// Same for a block of NTH threads (constexpr in scope): 1024 / NTH pieces.
#define TILE_LOAD_W(R, base, rs)                                  \
  R##0 = tile_piece_load<NTH>(base, rs, 0);                       \
  R##1 = tile_piece_load<NTH>(base, rs, 1);                       \
  if constexpr (NTH == 256) {                                     \
    R##2 = tile_piece_load<NTH>(base, rs, 2);                     \
    R##3 = tile_piece_load<NTH>(base, rs, 3);                     \
  }
#define TILE_STORE_W(R, tile)                                     \
  tile_piece_store<NTH>(tile, 0, R##0);                           \
  tile_piece_store<NTH>(tile, 1, R##1);                           \
  if constexpr (NTH == 256) {                                     \
    tile_piece_store<NTH>(tile, 2, R##2);                         \
    tile_piece_store<NTH>(tile, 3, R##3);                         \
  }

struct AttnShape {
  int B, S, H, Hkv;
  long long q_rs, k_rs, v_rs;  // row strides (elements) of the Q/K/V sources
  long long o_rs;              // row stride of O / dO
  float scale;                 // softmax scale (1/sqrt(128))
};

// Block -> (batch, kv head, block-of-4-units); unit u = qt*G + g.
// XCD-aware: consecutive linear indices (same batch/kv head, i.e. the same
// K/V working set) land on one XCD; heaviest causal tiles first.
struct BlockMap {
  int b, kvh, bi;
};
__device__ __forceinline__ BlockMap map_block(const AttnShape& sh, int per_pair) {
  const int nblk = gridDim.x, bid = blockIdx.x;
  int lin = bid;
  if ((nblk & 7) == 0) lin = (bid & 7) * (nblk >> 3) + (bid >> 3);
  const int pair = lin / per_pair;
  BlockMap m;
  m.b = pair / sh.Hkv;
  m.kvh = pair % sh.Hkv;
  m.bi = per_pair - 1 - (lin % per_pair);
  return m;
}

// ------------------------------------------------------------------ forward
template <int NWV>
__global__ __launch_bounds__(NWV * 64, 2) void k_attn_fwd(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                    const __bf16* __restrict__ v, __bf16* __restrict__ o,
                                                    float* __restrict__ lse, AttnShape sh) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [2 stages][K | V]
  const int G = sh.H / sh.Hkv;
  constexpr int NTH = NWV * 64;
  const int per_pair = (sh.S / QT) * G / NWV;
  const BlockMap bm = map_block(sh, per_pair);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, hi = lane >> 5, ql = lane & 31;
  const int u = bm.bi * NWV + w, qt = u / G, h = bm.kvh * G + (u % G);
  const int q0 = qt * QT;
  const int qt_max = (bm.bi * NWV + NWV - 1) / G;
  const int ntiles = (qt_max * QT + QT + KT - 1) / KT;
  const long long tok0 = (long long)bm.b * sh.S;

  const __bf16* kb = k + tok0 * sh.k_rs + (long long)bm.kvh * HD;
  const __bf16* vb = v + tok0 * sh.v_rs + (long long)bm.kvh * HD;

  // Q fragments (B operand of S^T = K Q^T): row q0+ql, d = 16ks + 8hi .. +7
  bf16x8 qf[8];
  {
    const __bf16* qr = q + (tok0 + q0 + ql) * sh.q_rs + (long long)h * HD + 8 * hi;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qr + 16 * ks);
  }
  f32x16 acc_o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) acc_o[db] = (f32x16){};
  float m_run = -INFINITY, l_run = 0.f;
  const float sl = sh.scale * LOG2E;
  const int qrow = q0 + ql;

  uint4 tk0, tk1, tk2, tk3, tv0, tv1, tv2, tv3;
  TILE_LOAD_W(tk, kb, sh.k_rs);
  TILE_LOAD_W(tv, vb, sh.v_rs);
  TILE_STORE_W(tk, smem);
  TILE_STORE_W(tv, smem + TILE_B);
  {  // tile 1 in flight across the first barrier (tile 0 again when there is none)
    const int kn = ntiles > 1 ? KT : 0;
    TILE_LOAD_W(tk, kb + (long long)kn * sh.k_rs, sh.k_rs);
    TILE_LOAD_W(tv, vb + (long long)kn * sh.v_rs, sh.v_rs);
  }
  __syncthreads();

  // unrolled x2 so the LDS ring slot is a compile-time constant: the
  // lane-dependent LDS addresses stay loop-invariant (immediate offsets).
  // Staging is split across the barrier: tile t+1 (loaded during step t-1)
  // is written to the other slot at the top of step t, then tile t+2's loads
  // are issued, so they land under step t's math AND the barrier after it.
  auto step_fn = [&](const int t, auto bufc) {
    constexpr int SLOT = decltype(bufc)::value;
    const int k0 = t * KT;
    const char* ktile = smem + SLOT * 2 * TILE_B;
    const char* vtile = ktile + TILE_B;
    if (t + 1 < ntiles) {
      char* nt = smem + (SLOT ^ 1) * 2 * TILE_B;
      TILE_STORE_W(tk, nt);
      TILE_STORE_W(tv, nt + TILE_B);
    }
    {  // tile t+2 (the last iterations re-read their own)
      const int kn = (t + 2 < ntiles) ? k0 + 2 * KT : k0;
      TILE_LOAD_W(tk, kb + (long long)kn * sh.k_rs, sh.k_rs);
      TILE_LOAD_W(tv, vb + (long long)kn * sh.v_rs, sh.v_rs);
    }
    if (k0 <= q0 + QT - 1) {  // wave-uniform: this tile has unmasked keys for this wave
      // S^T (keys on registers, query on the lane)
      f32x16 st[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        st[kt] = (f32x16){};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) st[kt] = mfma(row_operand(ktile, 32 * kt, ks), qf[ks], st[kt]);
      }
      // causal mask only on the diagonal tile (wave-uniform branch: the
      // other tiles run no compare/select)
      if (k0 + KT - 1 > q0) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = k0 + 32 * kt + (i & 3) + 8 * (i >> 2) + 4 * hi;
            if (key > qrow) st[kt][i] = -INFINITY;
          }
      }
      // raw-score max (the softmax scale is positive), then one fma per
      // score: p = exp2(s * c - m)
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, st[kt][i]);
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      // deferred max: the running max (log2 units) moves only when some row
      // of the wave grew by more than ATTN_DEFER, so O is rescaled on a few
      // tiles instead of on most of them (P is then bounded by 2^ATTN_DEFER
      // instead of 1: the same relative bf16 rounding, l and lse unchanged
      // in value).  The decision comes before this tile's P exists and after
      // the previous tile's P.V: nothing at the old scale is pending.
      float alpha = 1.f;
      if (__any(mx * sl > m_run + ATTN_DEFER)) {
        const float m_new = fmaxf(m_run, mx * sl);
        alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
#pragma unroll
        for (int db = 0; db < 4; ++db) acc_o[db] *= alpha;
      }
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = __builtin_amdgcn_exp2f(fmaf(st[kt][i], sl, -m_run));
          st[kt][i] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 32);
      l_run = l_run * alpha + rs;
      bf16x8 pf[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        float tmp[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) tmp[j] = st[ks >> 1][8 * (ks & 1) + j];
        pf[ks] = acc_to_operand(tmp);
      }
      // O^T += V^T P^T
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc_o[db] = mfma(tr_operand(vtile, 16 * ks, 32 * db), pf[ks], acc_o[db]);
    }
    __syncthreads();
    };
  for (int t0 = 0; t0 < ntiles; t0 += 2) {
    step_fn(t0, std::integral_constant<int, 0>{});
    if (t0 + 1 < ntiles) step_fn(t0 + 1, std::integral_constant<int, 1>{});
  }
  // epilogue: O[q][d] = O^T[d][q] / l ; lane holds d = 32db + 8g + 4hi + (0..3)
  const float inv = 1.f / l_run;
  __bf16* orow = o + (tok0 + qrow) * sh.o_rs + (long long)h * HD + 4 * hi;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u32x2 pk = {pack2(acc_o[db][4 * g] * inv, acc_o[db][4 * g + 1] * inv),
                  pack2(acc_o[db][4 * g + 2] * inv, acc_o[db][4 * g + 3] * inv)};
      *reinterpret_cast<u32x2*>(orow + 32 * db + 8 * g) = pk;
    }
  if (hi == 0) lse[((long long)bm.b * sh.H + h) * sh.S + qrow] = m_run + __log2f(l_run);
}

// ------------------------------------------------------------ backward prep
// delta[b][h][s] = sum_d dO * O (fp32): 16 lanes per (token, head) row, one
// 16-byte load of O and of dO per lane (32 lanes of 8-byte loads before:
// 66 us per call at 4 TB/s on the Llama-3-8B shape).
__global__ __launch_bounds__(256) void k_attn_bwd_delta(const __bf16* __restrict__ o, const __bf16* __restrict__ dout,
                                                        float* __restrict__ delta, AttnShape sh) {
  const long long row = (long long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const long long nrows = (long long)sh.B * sh.S * sh.H;
  if (row >= nrows) return;
  const long long tok = row / sh.H;
  const int h = (int)(row % sh.H);
  const int l = threadIdx.x & 15;
  const __bf16* a = o + tok * sh.o_rs + (long long)h * HD + 8 * l;
  const __bf16* b = dout + tok * sh.o_rs + (long long)h * HD + 8 * l;
  const u32x4 ua = *reinterpret_cast<const u32x4*>(a), ub = *reinterpret_cast<const u32x4*>(b);
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    s += __uint_as_float(ua[e] << 16) * __uint_as_float(ub[e] << 16);
    s += __uint_as_float(ua[e] & 0xffff0000u) * __uint_as_float(ub[e] & 0xffff0000u);
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) s += __shfl_xor(s, off, 16);
  if (l == 0) {
    const int b_ = (int)(tok / sh.S), s_ = (int)(tok % sh.S);
    delta[((long long)b_ * sh.H + h) * sh.S + s_] = s;
  }
}

// --------------------------------------------------------------- dQ kernel
// Same decomposition as the forward.  Per key tile: S^T = K Q^T,
// dP^T = V dO^T (V rows from LDS, dO fragments in registers),
// P = exp2(S^T*c - lse2), dS = P (dP^T - delta), dQ^T += K^T dS^T.
template <int NWV>
__global__ __launch_bounds__(NWV * 64, 2) void k_attn_bwd_dq(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                       const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                       const float* __restrict__ lse, const float* __restrict__ delta,
                                                       __bf16* __restrict__ dq, long long dq_rs, AttnShape sh) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int G = sh.H / sh.Hkv;
  constexpr int NTH = NWV * 64;
  const int per_pair = (sh.S / QT) * G / NWV;
  const BlockMap bm = map_block(sh, per_pair);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, hi = lane >> 5, ql = lane & 31;
  const int u = bm.bi * NWV + w, qt = u / G, h = bm.kvh * G + (u % G);
  const int q0 = qt * QT;
  const int qt_max = (bm.bi * NWV + NWV - 1) / G;
  const int ntiles = (qt_max * QT + QT + KT - 1) / KT;
  const long long tok0 = (long long)bm.b * sh.S;
  const __bf16* kb = k + tok0 * sh.k_rs + (long long)bm.kvh * HD;
  const __bf16* vb = v + tok0 * sh.v_rs + (long long)bm.kvh * HD;
  const int qrow = q0 + ql;

  bf16x8 qf[8], df[8];
  {
    const __bf16* qr = q + (tok0 + qrow) * sh.q_rs + (long long)h * HD + 8 * hi;
    const __bf16* dr = dout + (tok0 + qrow) * sh.o_rs + (long long)h * HD + 8 * hi;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      qf[ks] = *reinterpret_cast<const bf16x8*>(qr + 16 * ks);
      df[ks] = *reinterpret_cast<const bf16x8*>(dr + 16 * ks);
    }
  }
  const long long li = ((long long)bm.b * sh.H + h) * sh.S + qrow;
  const float lse2 = lse[li], dlt = delta[li];
  const float sl = sh.scale * LOG2E;
  f32x16 acc[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) acc[db] = (f32x16){};

  uint4 tk0, tk1, tk2, tk3, tv0, tv1, tv2, tv3;
  TILE_LOAD_W(tk, kb, sh.k_rs);
  TILE_LOAD_W(tv, vb, sh.v_rs);
  TILE_STORE_W(tk, smem);
  TILE_STORE_W(tv, smem + TILE_B);
  {
    const int kn = ntiles > 1 ? KT : 0;
    TILE_LOAD_W(tk, kb + (long long)kn * sh.k_rs, sh.k_rs);
    TILE_LOAD_W(tv, vb + (long long)kn * sh.v_rs, sh.v_rs);
  }
  __syncthreads();
  // unrolled x2 (compile-time LDS slot); staging split across the barrier
  // as in the forward
  auto step_fn = [&](const int t, auto bufc) {
    constexpr int SLOT = decltype(bufc)::value;
    const int k0 = t * KT;
    const char* ktile = smem + SLOT * 2 * TILE_B;
    const char* vtile = ktile + TILE_B;
    if (t + 1 < ntiles) {
      char* nt = smem + (SLOT ^ 1) * 2 * TILE_B;
      TILE_STORE_W(tk, nt);
      TILE_STORE_W(tv, nt + TILE_B);
    }
    {
      const int kn = (t + 2 < ntiles) ? k0 + 2 * KT : k0;
      TILE_LOAD_W(tk, kb + (long long)kn * sh.k_rs, sh.k_rs);
      TILE_LOAD_W(tv, vb + (long long)kn * sh.v_rs, sh.v_rs);
    }
    if (k0 <= q0 + QT - 1) {
      const bool diag = k0 + KT - 1 > q0;
      // one 32-key half at a time: S^T/dP^T accumulators for 32 keys only
      // (keeps the kernel inside 256 VGPRs, no scratch)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        f32x16 st = (f32x16){}, dp = (f32x16){};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          st = mfma(row_operand(ktile, 32 * kt, ks), qf[ks], st);
          dp = mfma(row_operand(vtile, 32 * kt, ks), df[ks], dp);
        }
        if (diag) {  // wave-uniform: causal mask on the diagonal tile only
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = k0 + 32 * kt + (i & 3) + 8 * (i >> 2) + 4 * hi;
            if (key > qrow) st[i] = -INFINITY;
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = __builtin_amdgcn_exp2f(fmaf(st[i], sl, -lse2));
          st[i] = p * (dp[i] - dlt);  // dS (softmax scale applied at the end)
        }
        bf16x8 sf[2];
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) {
          float tmp[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) tmp[j] = st[8 * hs + j];
          sf[hs] = acc_to_operand(tmp);
        }
#pragma unroll
        for (int db = 0; db < 4; ++db)
#pragma unroll
          for (int hs = 0; hs < 2; ++hs)
            acc[db] = mfma(tr_operand(ktile, 32 * kt + 16 * hs, 32 * db), sf[hs], acc[db]);
      }
    }
    __syncthreads();
    };
  for (int t0 = 0; t0 < ntiles; t0 += 2) {
    step_fn(t0, std::integral_constant<int, 0>{});
    if (t0 + 1 < ntiles) step_fn(t0 + 1, std::integral_constant<int, 1>{});
  }
  __bf16* drow = dq + (tok0 + qrow) * dq_rs + (long long)h * HD + 4 * hi;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float c = sh.scale;
      u32x2 pk = {pack2(acc[db][4 * g] * c, acc[db][4 * g + 1] * c), pack2(acc[db][4 * g + 2] * c, acc[db][4 * g + 3] * c)};
      *reinterpret_cast<u32x2*>(drow + 32 * db + 8 * g) = pk;
    }
}

// ------------------------------------------------------------ dK/dV kernel
// Block = (batch, kv head, 128 keys); wave w owns keys kb0 + 32w .. +31.
// Loops over the G query heads x 32-row query tiles from the diagonal on;
// Q and dO tiles (32 x 128) + LSE/delta rows are staged in LDS per step
// (shared by the 4 waves).  Per step and wave: S = Q K^T and dP = dO V^T
// (key on the lane, K/V fragments in registers, accumulators initialised
// with -lse2/c and -delta), P = exp2(c S), dS = P dP;
// dV^T += dO^T P, dK^T += Q^T dS (transposed LDS reads of dO / Q).
constexpr int KB = NW * 32;           // keys per block
constexpr int QSTG = 64;               // query rows staged per step (two 32-row MFMA tiles)
constexpr int QTB = QSTG * 256;        // one staged 64 x 128 bf16 tile in bytes
__global__ __launch_bounds__(NT, 1) void k_attn_bwd_dkdv(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                         const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                         const float* __restrict__ lse, const float* __restrict__ delta,
                                                         __bf16* __restrict__ dk, __bf16* __restrict__ dv,
                                                         long long dkv_rs, AttnShape sh) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [2][Q | dO] + [2][lse | delta]
  float* rowc = reinterpret_cast<float*>(smem + 4 * QTB);       // [2][lse 64 | delta 64]
  const int G = sh.H / sh.Hkv;
  const int nkb = sh.S / KB;
  // block -> (b, kvh, key block), heaviest (earliest keys) first, XCD-grouped
  const int nblk = gridDim.x, bid = blockIdx.x;
  int lin = bid;
  if ((nblk & 7) == 0) lin = (bid & 7) * (nblk >> 3) + (bid >> 3);
  const int pair = lin / nkb, kbi = lin % nkb;
  const int b = pair / sh.Hkv, kvh = pair % sh.Hkv;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, hi = lane >> 5, kl = lane & 31;
  const int kb0 = kbi * KB, key = kb0 + 32 * w + kl;
  const long long tok0 = (long long)b * sh.S;

  // K, V fragments (B operands of S = Q K^T and dP = dO V^T)
  bf16x8 kf[8], vf[8];
  {
    const __bf16* kr = k + (tok0 + key) * sh.k_rs + (long long)kvh * HD + 8 * hi;
    const __bf16* vr = v + (tok0 + key) * sh.v_rs + (long long)kvh * HD + 8 * hi;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      kf[ks] = *reinterpret_cast<const bf16x8*>(kr + 16 * ks);
      vf[ks] = *reinterpret_cast<const bf16x8*>(vr + 16 * ks);
    }
  }
  f32x16 dka[4], dva[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    dka[db] = (f32x16){};
    dva[db] = (f32x16){};
  }
  const float sl = sh.scale * LOG2E;
  const float inv_sl = 1.f / sl;
  const int nqt = (sh.S - kb0) / QSTG;  // staged query tiles from the block's first key on
  const int nsteps = G * nqt;

  // step s -> (head g, staged query tile qt): Q/dO tiles of 64 rows x 256 B
  // = 1024 chunks of 16 B each, 4 per thread (named scalars, see TILE_LOAD)
  uint4 rq0, rq1, rq2, rq3, rd0, rd1, rd2, rd3;
  float rc = 0.f;
  auto stage = [&](int s) {
    const int g = s / nqt, qt = s % nqt, h = kvh * G + g;
    const long long tok = tok0 + kb0 + (long long)qt * QSTG;
    const __bf16* qh = q + tok * sh.q_rs + (long long)h * HD;
    const __bf16* dh = dout + tok * sh.o_rs + (long long)h * HD;
    TILE_LOAD(rq, qh, sh.q_rs);
    TILE_LOAD(rd, dh, sh.o_rs);
    const long long li = ((long long)b * sh.H + h) * sh.S + kb0 + (long long)qt * QSTG;
    rc = threadIdx.x < 64 ? lse[li + threadIdx.x] : (threadIdx.x < 128 ? delta[li + threadIdx.x - 64] : 0.f);
  };
  auto commit = [&](int buf) {
    char* qtile = smem + buf * 2 * QTB;
    TILE_STORE(rq, qtile);
    TILE_STORE(rd, qtile + QTB);
    if (threadIdx.x < 128) rowc[buf * 128 + threadIdx.x] = rc;
  };

  stage(0);
  commit(0);
  __syncthreads();
  // unrolled x2 so the LDS ring slot is a compile-time constant: the
  // lane-dependent LDS addresses stay loop-invariant (immediate offsets)
  auto step_fn = [&](const int s, auto bufc) {
    constexpr int SLOT = decltype(bufc)::value;
    const int buf = SLOT;
    stage(s + 1 < nsteps ? s + 1 : s);
    const int qt = s % nqt;
#pragma unroll
    for (int sub = 0; sub < QSTG / QT; ++sub) {
    const int q0 = kb0 + qt * QSTG + sub * QT;  // first query row of this 32-row tile
    if (q0 + QT - 1 >= kb0 + 32 * w) {  // wave-uniform: some query >= some key of this wave
      const char* qtile = smem + buf * 2 * QTB + sub * QT * 256;
      const char* dtile = qtile + QTB;
      const float* lrow = rowc + buf * 128 + sub * QT;
      // accumulator init with the row constants: row q = (i&3)+8(i>>2)+4hi
      f32x16 sa, pa;
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const float4 l4 = *reinterpret_cast<const float4*>(lrow + 8 * gg + 4 * hi);
        const float4 d4 = *reinterpret_cast<const float4*>(lrow + QSTG + 8 * gg + 4 * hi);
        sa[4 * gg] = -l4.x * inv_sl; sa[4 * gg + 1] = -l4.y * inv_sl;
        sa[4 * gg + 2] = -l4.z * inv_sl; sa[4 * gg + 3] = -l4.w * inv_sl;
        pa[4 * gg] = -d4.x; pa[4 * gg + 1] = -d4.y; pa[4 * gg + 2] = -d4.z; pa[4 * gg + 3] = -d4.w;
      }
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        sa = mfma(row_operand(qtile, 0, ks), kf[ks], sa);
        pa = mfma(row_operand(dtile, 0, ks), vf[ks], pa);
      }
      if (q0 < kb0 + 32 * w + 31) {  // wave-uniform: causal mask on diagonal tiles only
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qr = q0 + (i & 3) + 8 * (i >> 2) + 4 * hi;
          if (key > qr) sa[i] = -INFINITY;
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(sa[i] * sl);
        sa[i] = p;
        pa[i] = p * pa[i];  // dS
      }
      bf16x8 pf[2], sf[2];
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        float t0[8], t1[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          t0[j] = sa[8 * qs + j];
          t1[j] = pa[8 * qs + j];
        }
        pf[qs] = acc_to_operand(t0);
        sf[qs] = acc_to_operand(t1);
      }
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int qs = 0; qs < 2; ++qs) {
          dva[db] = mfma(tr_operand(dtile, 16 * qs, 32 * db), pf[qs], dva[db]);
          dka[db] = mfma(tr_operand(qtile, 16 * qs, 32 * db), sf[qs], dka[db]);
        }
    }
    }  // sub-tile
    if (s + 1 < nsteps) commit(buf ^ 1);
    __syncthreads();
    };
  for (int s0 = 0; s0 < nsteps; s0 += 2) {
    step_fn(s0, std::integral_constant<int, 0>{});
    if (s0 + 1 < nsteps) step_fn(s0 + 1, std::integral_constant<int, 1>{});
  }
  // dK^T / dV^T: lane = key, registers = d (32db + 8g + 4hi + 0..3)
  __bf16* dkr = dk + (tok0 + key) * dkv_rs + (long long)kvh * HD + 4 * hi;
  __bf16* dvr = dv + (tok0 + key) * dkv_rs + (long long)kvh * HD + 4 * hi;
  const float c = sh.scale;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u32x2 pk = {pack2(dka[db][4 * g] * c, dka[db][4 * g + 1] * c), pack2(dka[db][4 * g + 2] * c, dka[db][4 * g + 3] * c)};
      *reinterpret_cast<u32x2*>(dkr + 32 * db + 8 * g) = pk;
      u32x2 pv = {pack2(dva[db][4 * g], dva[db][4 * g + 1]), pack2(dva[db][4 * g + 2], dva[db][4 * g + 3])};
      *reinterpret_cast<u32x2*>(dvr + 32 * db + 8 * g) = pv;
    }
}


// ------------------------------------- dK/dV kernel, producer / consumer
// Same block (batch, kv head, 128 keys) and query sweep, 8 waves in two
// roles on the same 4 x 32 keys (wave w and w + 4 share a SIMD):
//   producers (waves 0-3): S = Q K^T and dP = dO V^T (accumulators
//     initialised with the row constants), P = exp2(c S'), dS = P dP', and
//     the bf16 B operands of the dV^T / dK^T products -> LDS;
//   consumers (waves 4-7): dV^T += dO^T P, dK^T += Q^T dS from those
//     operands, one step behind.
// 16 MFMAs per 32-row query slice on each side and no recomputation; the
// producers' softmax VALU issues beside the consumers' MFMAs on the same
// SIMD.  Each wave holds either K/V fragments + S/dP or the two
// accumulators, so the kernel fits 256 registers (two waves per SIMD).
// One 32-row slice per step; Q/dO tiles in a 3-slot ring (staged for t+1,
// read by the producers for t and by the consumers for t-1), operands in a
// 2-slot ring; one barrier per step.
constexpr int PC_TB = QT * 256;  // one 32 x 128 bf16 tile (bytes)
constexpr int PC_OPB = NW * 4 * 64 * 16;  // operands of one step: 4 waves x 4 frags x 64 lanes x 16 B
constexpr int PC_LDS = 3 * 2 * PC_TB + 3 * 2 * QT * 4 + 2 * PC_OPB;

// KVW: complete the producers' K/V fragment loads before the loop (an
// explicit vmcnt(0) the waitcnt pass sees).  Without it hipcc's loop-header
// merge still counts those 16 loads as pending inside the loop and emits
// vmcnt(7) .. vmcnt(0) between the S/dP MFMAs -- in steady state that waits
// for the NEXT slice's Q/dO/row-constant loads issued at the top of the same
// step, i.e. one global-load latency on the producers' chain every step.
template <bool KVW>
__global__ __launch_bounds__(2 * NT) void k_attn_bwd_dkdv_pc(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                             const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                             const float* __restrict__ lse, const float* __restrict__ delta,
                                                             __bf16* __restrict__ dk, __bf16* __restrict__ dv,
                                                             long long dkv_rs, AttnShape sh) {
  constexpr int NTH = 2 * NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // [3 slots][Q tile | dO tile], [3 slots][lse 32 | delta 32], [2 slots][operands]
  float* rowc = reinterpret_cast<float*>(smem + 3 * 2 * PC_TB);
  char* opnd = smem + 3 * 2 * PC_TB + 3 * 2 * QT * 4;
  const int G = sh.H / sh.Hkv;
  const int nkb = sh.S / KB;
  const int nblk = gridDim.x, bid = blockIdx.x;
  int lin = bid;
  if ((nblk & 7) == 0) lin = (bid & 7) * (nblk >> 3) + (bid >> 3);
  const int pair = lin / nkb, kbi = lin % nkb;
  const int b = pair / sh.Hkv, kvh = pair % sh.Hkv;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, hi = lane >> 5, kl = lane & 31;
  const bool producer = w < NW;  // wave-uniform
  const int kw = w & (NW - 1);
  const int kb0 = kbi * KB, key = kb0 + 32 * kw + kl;
  const long long tok0 = (long long)b * sh.S;
  const float sl = sh.scale * LOG2E;
  const float inv_sl = 1.f / sl;
  const int nqt = (sh.S - kb0) / QT;
  const int nsteps = G * nqt;

  uint4 rq, rd;
  float rc = 0.f;
  // slices are walked with incremental (head, query tile) counters: no
  // integer division per step (it was ~20 SALU instructions per use)
  auto stage = [&](int g, int qt) {
    const int h = kvh * G + g;
    const long long tok = tok0 + kb0 + (long long)qt * QT;
    rq = tile_piece_load<NTH>(q + tok * sh.q_rs + (long long)h * HD, sh.q_rs, 0);
    rd = tile_piece_load<NTH>(dout + tok * sh.o_rs + (long long)h * HD, sh.o_rs, 0);
    const long long li = ((long long)b * sh.H + h) * sh.S + kb0 + (long long)qt * QT;
    rc = threadIdx.x < QT ? lse[li + threadIdx.x] : (threadIdx.x < 2 * QT ? delta[li + threadIdx.x - QT] : 0.f);
  };
  auto commit = [&](int slot) {
    char* qtile = smem + slot * 2 * PC_TB;
    tile_piece_store<NTH>(qtile, 0, rq);
    tile_piece_store<NTH>(qtile + PC_TB, 0, rd);
    if (threadIdx.x < 2 * QT) rowc[slot * 2 * QT + threadIdx.x] = rc;
  };
  // wave-uniform activity / diagonal of query slice `qt` for this wave's keys
  auto active = [&](int qt) { return kb0 + qt * QT + QT - 1 >= kb0 + 32 * kw; };
  auto diagonal = [&](int qt) { return kb0 + qt * QT < kb0 + 32 * kw + 31; };

  auto produce = [&](int qt, int tslot, int oslot, const bf16x8* kf, const bf16x8* vf) {
    if (!active(qt)) return;
    const char* qtile = smem + tslot * 2 * PC_TB;
    const char* dtile = qtile + PC_TB;
    const float* lrow = rowc + tslot * 2 * QT;
    f32x16 sa, pa;
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const float4 l4 = *reinterpret_cast<const float4*>(lrow + 8 * gg + 4 * hi);
      const float4 d4 = *reinterpret_cast<const float4*>(lrow + QT + 8 * gg + 4 * hi);
      sa[4 * gg] = -l4.x * inv_sl; sa[4 * gg + 1] = -l4.y * inv_sl;
      sa[4 * gg + 2] = -l4.z * inv_sl; sa[4 * gg + 3] = -l4.w * inv_sl;
      pa[4 * gg] = -d4.x; pa[4 * gg + 1] = -d4.y; pa[4 * gg + 2] = -d4.z; pa[4 * gg + 3] = -d4.w;
    }
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      sa = mfma(row_operand(qtile, 0, ks), kf[ks], sa);
      pa = mfma(row_operand(dtile, 0, ks), vf[ks], pa);
    }
    if (diagonal(qt)) {
      const int q0 = kb0 + qt * QT;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qr = q0 + (i & 3) + 8 * (i >> 2) + 4 * hi;
        if (key > qr) sa[i] = -INFINITY;
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = __builtin_amdgcn_exp2f(sa[i] * sl);
      sa[i] = p;
      pa[i] = p * pa[i];  // dS
    }
    bf16x8* o = reinterpret_cast<bf16x8*>(opnd + oslot * PC_OPB + kw * (4 * 64 * 16)) + lane;
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      float t0[8], t1[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        t0[j] = sa[8 * qs + j];
        t1[j] = pa[8 * qs + j];
      }
      o[64 * qs] = acc_to_operand(t0);        // P fragments 0, 1
      o[64 * (2 + qs)] = acc_to_operand(t1);  // dS fragments 2, 3
    }
  };
  auto consume = [&](int qt, int tslot, int oslot, f32x16* dka, f32x16* dva) {
    if (!active(qt)) return;
    const char* qtile = smem + tslot * 2 * PC_TB;
    const char* dtile = qtile + PC_TB;
    const bf16x8* o = reinterpret_cast<const bf16x8*>(opnd + oslot * PC_OPB + kw * (4 * 64 * 16)) + lane;
    bf16x8 pf[2], sf[2];
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      pf[qs] = o[64 * qs];
      sf[qs] = o[64 * (2 + qs)];
    }
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        dva[db] = mfma(tr_operand(dtile, 16 * qs, 32 * db), pf[qs], dva[db]);
        dka[db] = mfma(tr_operand(qtile, 16 * qs, 32 * db), sf[qs], dka[db]);
      }
  };

  auto next = [&](int& g, int& qt) {
    if (++qt == nqt) {
      qt = 0;
      ++g;
    }
  };
  stage(0, 0);
  commit(0);
  __syncthreads();
  int ng = 0, nq = 0;  // (head, query tile) of slice t + 1
  next(ng, nq);
  // iteration t: stage step t+1, producers step t, consumers step t-1.  The
  // two roles run separate loops with the same barrier count (nsteps + 1),
  // so the K/V fragments (producers) and the dK/dV accumulators (consumers)
  // are never live together.
  if (producer) {
    bf16x8 kf[8], vf[8];
    {
      const __bf16* kr = k + (tok0 + key) * sh.k_rs + (long long)kvh * HD + 8 * hi;
      const __bf16* vr = v + (tok0 + key) * sh.v_rs + (long long)kvh * HD + 8 * hi;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        kf[ks] = *reinterpret_cast<const bf16x8*>(kr + 16 * ks);
        vf[ks] = *reinterpret_cast<const bf16x8*>(vr + 16 * ks);
      }
    }
    if constexpr (KVW) {  // a use of every fragment register: hipcc waits for the loads here
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) asm volatile("" ::"v"(kf[ks]), "v"(vf[ks]));
    }
    int ts = 0;  // tile slot of step t (t mod 3)
    int tq = 0;  // query tile of step t (t mod nqt)
    for (int t = 0; t <= nsteps; ++t) {
      const int tn = ts == 2 ? 0 : ts + 1;
      if (t + 1 < nsteps) stage(ng, nq);
      if (t < nsteps) produce(tq, ts, t & 1, kf, vf);
      if (t + 1 < nsteps) commit(tn);
      __syncthreads();
      ts = tn;
      tq = tq + 1 == nqt ? 0 : tq + 1;
      next(ng, nq);
    }
    return;
  }
  f32x16 dka[4], dva[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    dka[db] = (f32x16){};
    dva[db] = (f32x16){};
  }
  int ts = 0;
  int cq = 0;  // query tile of step t - 1
  for (int t = 0; t <= nsteps; ++t) {
    const int tn = ts == 2 ? 0 : ts + 1;
    const int tp = ts == 0 ? 2 : ts - 1;
    if (t + 1 < nsteps) stage(ng, nq);
    if (t >= 1) {
      consume(cq, tp, (t - 1) & 1, dka, dva);
      cq = cq + 1 == nqt ? 0 : cq + 1;
    }
    if (t + 1 < nsteps) commit(tn);
    __syncthreads();
    ts = tn;
    next(ng, nq);
  }
  // consumers: dK^T / dV^T, lane = key, registers = d (32db + 8g + 4hi + 0..3)
  __bf16* dkr = dk + (tok0 + key) * dkv_rs + (long long)kvh * HD + 4 * hi;
  __bf16* dvr = dv + (tok0 + key) * dkv_rs + (long long)kvh * HD + 4 * hi;
  const float c = sh.scale;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u32x2 pk = {pack2(dka[db][4 * g] * c, dka[db][4 * g + 1] * c), pack2(dka[db][4 * g + 2] * c, dka[db][4 * g + 3] * c)};
      *reinterpret_cast<u32x2*>(dkr + 32 * db + 8 * g) = pk;
      u32x2 pv = {pack2(dva[db][4 * g], dva[db][4 * g + 1]), pack2(dva[db][4 * g + 2], dva[db][4 * g + 3])};
      *reinterpret_cast<u32x2*>(dvr + 32 * db + 8 * g) = pv;
    }
}

// ------------------------------- dK/dV kernel, two producers per consumer
// Same block (batch, kv head, 128 keys), query sweep and products as
// k_attn_bwd_dkdv_pc, but 12 waves: per SIMD (waves w, w + 4, w + 8 share
// one, keys kb0 + 32 (w & 3) ..) two producers and one consumer.  A
// producer's slice is split over two barrier intervals:
//   interval s     S = Q K^T, dP = dO V^T (16 MFMAs, accumulators kept),
//   interval s + 1 mask, P = exp2(c S'), dS = P dP', bf16 operands -> LDS,
// and the two producers are half a slice apart (A takes even slices, B odd),
// so in every interval one producer's softmax VALU issues beside the other
// producer's and the consumer's MFMAs (consumer: slice s in interval s + 2).
// In the one-producer kernel the softmax sat between the S/dP MFMAs and the
// barrier with only the consumer's MFMAs to cover it.  Producers also stage
// the Q / dO tiles and row constants two slices ahead (one 16-byte chunk
// of each tile per producer thread).  LDS: 4 tile slots (slice s mod 4: read
// by the producer in s, kept for the consumer in s + 2, refilled at the end
// of s + 3), 2 operand slots, 4 row-constant slots: 97 KB, one block per CU.
constexpr int P3_NSLOT = 4;
constexpr int P3_ROWC = 2 * QT;  // floats per slot: -lse / sl (32), -delta (32)
constexpr int P3_LDS = P3_NSLOT * 2 * PC_TB + P3_NSLOT * P3_ROWC * 4 + 2 * PC_OPB;

__global__ __launch_bounds__(3 * NT) void k_attn_bwd_dkdv_p3(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                             const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                             const float* __restrict__ lse, const float* __restrict__ delta,
                                                             __bf16* __restrict__ dk, __bf16* __restrict__ dv,
                                                             long long dkv_rs, AttnShape sh) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* rowc = reinterpret_cast<float*>(smem + P3_NSLOT * 2 * PC_TB);
  char* opnd = smem + P3_NSLOT * 2 * PC_TB + P3_NSLOT * P3_ROWC * 4;
  const int G = sh.H / sh.Hkv;
  const int nkb = sh.S / KB;
  const int nblk = gridDim.x, bid = blockIdx.x;
  int lin = bid;
  if ((nblk & 7) == 0) lin = (bid & 7) * (nblk >> 3) + (bid >> 3);
  const int pair = lin / nkb, kbi = lin % nkb;
  const int b = pair / sh.Hkv, kvh = pair % sh.Hkv;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, hi = lane >> 5, kl = lane & 31;
  const int role = w >> 2;  // 0 producer A (even slices), 1 producer B (odd slices), 2 consumer
  const int kw = w & (NW - 1);
  const int kb0 = kbi * KB, key = kb0 + 32 * kw + kl;
  const long long tok0 = (long long)b * sh.S;
  const float sl = sh.scale * LOG2E;
  const float inv_sl = 1.f / sl;
  const int nqt = (sh.S - kb0) / QT;
  const int nsteps = G * nqt;
  const int tp = threadIdx.x & (2 * NT - 1);  // producer thread 0..511 (staging)

  // staging (producers): slice s -> one Q and one dO chunk per thread, and
  // the transformed row constant for threads < 64; two register sets
  uint4 q0r, d0r, q1r, d1r;
  float c0r = 0.f, c1r = 0.f;
  auto ld = [&](int s, uint4& qr, uint4& dr, float& cr) {
    const int g = s / nqt, qt = s - g * nqt, h = kvh * G + g;
    const long long tok = tok0 + kb0 + (long long)qt * QT;
    qr = tile_piece_load<2 * NT>(q + tok * sh.q_rs + (long long)h * HD, sh.q_rs, 0);
    dr = tile_piece_load<2 * NT>(dout + tok * sh.o_rs + (long long)h * HD, sh.o_rs, 0);
    const long long li = ((long long)b * sh.H + h) * sh.S + kb0 + (long long)qt * QT;
    // every thread issues exactly three loads (threads >= 64 re-read a delta
    // entry): no branch around a load, so hipcc's vmcnt before a register
    // set's LDS write counts only the younger set's three loads
    const float x = (tp < QT ? lse : delta)[li + (tp & (QT - 1))];
    cr = tp < QT ? -x * inv_sl : -x;
  };
  auto st = [&](int s, const uint4& qr, const uint4& dr, float cr) {
    const int slot = s & (P3_NSLOT - 1);
    char* qtile = smem + slot * 2 * PC_TB;
    tile_piece_store<2 * NT>(qtile, 0, qr);
    tile_piece_store<2 * NT>(qtile + PC_TB, 0, dr);
    if (tp < 2 * QT) rowc[slot * P3_ROWC + tp] = cr;
  };
  auto active = [&](int s) { return s % nqt >= kw; };    // some query >= some key of this wave
  auto diagonal = [&](int s) { return s % nqt == kw; };  // causal mask needed

  if (role < 2) {
    const int p = role;
    bf16x8 kf[8], vf[8];
    {
      const __bf16* kr = k + (tok0 + key) * sh.k_rs + (long long)kvh * HD + 8 * hi;
      const __bf16* vr = v + (tok0 + key) * sh.v_rs + (long long)kvh * HD + 8 * hi;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        kf[ks] = *reinterpret_cast<const bf16x8*>(kr + 16 * ks);
        vf[ks] = *reinterpret_cast<const bf16x8*>(vr + 16 * ks);
      }
    }
    ld(0, q0r, d0r, c0r);
    ld(nsteps > 1 ? 1 : 0, q1r, d1r, c1r);
    st(0, q0r, d0r, c0r);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) asm volatile("" ::"v"(kf[ks]), "v"(vf[ks]));  // see KVW above
    __syncthreads();
    f32x16 sa, pa;  // S' and dP' of this producer's current slice, live across one barrier
    auto mfma_phase = [&](int s) {
      if (!active(s)) return;
      const int slot = s & (P3_NSLOT - 1);
      const char* qtile = smem + slot * 2 * PC_TB;
      const char* dtile = qtile + PC_TB;
      const float* lrow = rowc + slot * P3_ROWC;
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const float4 l4 = *reinterpret_cast<const float4*>(lrow + 8 * gg + 4 * hi);
        const float4 d4 = *reinterpret_cast<const float4*>(lrow + QT + 8 * gg + 4 * hi);
        sa[4 * gg] = l4.x; sa[4 * gg + 1] = l4.y; sa[4 * gg + 2] = l4.z; sa[4 * gg + 3] = l4.w;
        pa[4 * gg] = d4.x; pa[4 * gg + 1] = d4.y; pa[4 * gg + 2] = d4.z; pa[4 * gg + 3] = d4.w;
      }
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        sa = mfma(row_operand(qtile, 0, ks), kf[ks], sa);
        pa = mfma(row_operand(dtile, 0, ks), vf[ks], pa);
      }
    };
    auto valu_phase = [&](int s) {
      if (!active(s)) return;
      if (diagonal(s)) {
        const int q0 = kb0 + (s % nqt) * QT;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qr = q0 + (i & 3) + 8 * (i >> 2) + 4 * hi;
          if (key > qr) sa[i] = -INFINITY;
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pv = __builtin_amdgcn_exp2f(sa[i] * sl);
        sa[i] = pv;
        pa[i] = pv * pa[i];  // dS
      }
      bf16x8* o = reinterpret_cast<bf16x8*>(opnd + (s & 1) * PC_OPB + kw * (4 * 64 * 16)) + lane;
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        float t0[8], t1[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          t0[j] = sa[8 * qs + j];
          t1[j] = pa[8 * qs + j];
        }
        o[64 * qs] = acc_to_operand(t0);        // P fragments 0, 1
        o[64 * (2 + qs)] = acc_to_operand(t1);  // dS fragments 2, 3
      }
    };
    // interval t: stage slice t+2 (register set t&1), S/dP of slice t
    // (producer t&1) or softmax of slice t-1 (the other producer), write
    // slice t+1 (set (t+1)&1) into its slot, barrier.  Unrolled x2 so the
    // register set and this producer's phase are compile-time.
    auto interval = [&](int t, auto par) {
      constexpr int PAR = decltype(par)::value;
      {  // unconditional (past the end: re-read the last slice, never stored)
        const int sn = t + 2 < nsteps ? t + 2 : nsteps - 1;
        if constexpr (PAR == 0) ld(sn, q0r, d0r, c0r);
        else ld(sn, q1r, d1r, c1r);
      }
      if (p == PAR) {
        if (t < nsteps) mfma_phase(t);
      } else {
        if (t >= 1 && t - 1 < nsteps) valu_phase(t - 1);
      }
      if (t + 1 < nsteps) {
        if constexpr (PAR == 0) st(t + 1, q1r, d1r, c1r);
        else st(t + 1, q0r, d0r, c0r);
      }
      __syncthreads();
    };
    for (int t = 0; t < nsteps + 2; t += 2) {
      interval(t, std::integral_constant<int, 0>{});
      if (t + 1 < nsteps + 2) interval(t + 1, std::integral_constant<int, 1>{});
    }
    return;
  }
  // consumer: slice s in interval s + 2 (same barrier count: prologue + nsteps + 2)
  __syncthreads();
  f32x16 dka[4], dva[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    dka[db] = (f32x16){};
    dva[db] = (f32x16){};
  }
  for (int t = 0; t < nsteps + 2; ++t) {
    const int s = t - 2;
    if (s >= 0 && active(s)) {
      const int slot = s & (P3_NSLOT - 1);
      const char* qtile = smem + slot * 2 * PC_TB;
      const char* dtile = qtile + PC_TB;
      const bf16x8* o = reinterpret_cast<const bf16x8*>(opnd + (s & 1) * PC_OPB + kw * (4 * 64 * 16)) + lane;
      bf16x8 pf[2], sf[2];
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        pf[qs] = o[64 * qs];
        sf[qs] = o[64 * (2 + qs)];
      }
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int qs = 0; qs < 2; ++qs) {
          dva[db] = mfma(tr_operand(dtile, 16 * qs, 32 * db), pf[qs], dva[db]);
          dka[db] = mfma(tr_operand(qtile, 16 * qs, 32 * db), sf[qs], dka[db]);
        }
    }
    __syncthreads();
  }
  __bf16* dkr = dk + (tok0 + key) * dkv_rs + (long long)kvh * HD + 4 * hi;
  __bf16* dvr = dv + (tok0 + key) * dkv_rs + (long long)kvh * HD + 4 * hi;
  const float c = sh.scale;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u32x2 pk = {pack2(dka[db][4 * g] * c, dka[db][4 * g + 1] * c), pack2(dka[db][4 * g + 2] * c, dka[db][4 * g + 3] * c)};
      *reinterpret_cast<u32x2*>(dkr + 32 * db + 8 * g) = pk;
      u32x2 pv = {pack2(dva[db][4 * g], dva[db][4 * g + 1]), pack2(dva[db][4 * g + 2], dva[db][4 * g + 3])};
      *reinterpret_cast<u32x2*>(dvr + 32 * db + 8 * g) = pv;
    }
}

}  // namespace

#define PTO_API extern "C" __attribute__((visibility("default")))

static bool attn_shape_ok(const AttnShape& sh) {
  if (sh.H % sh.Hkv) return false;
  const int G = sh.H / sh.Hkv;
  return sh.S % KB == 0 && sh.S % KT == 0 && ((sh.S / QT) * G) % NW == 0 && sh.B > 0;
}

static AttnShape make_shape(int B, int S, int H, int Hkv, long long q_rs, long long k_rs, long long v_rs,
                            long long o_rs, float scale) {
  AttnShape sh{B, S, H, Hkv, q_rs, k_rs, v_rs, o_rs, scale};
  return sh;
}

// Returns -1 for unsupported shapes (S % 128, H % Hkv, head_dim != 128 is the
// caller's contract).
// Waves per forward / dQ block: 8 (two 32-row query tiles x the 4 heads of
// a GQA group share each K/V tile: 4 waves per SIMD at the same 64 KB of
// LDS) unless the shape does not split into 8.
static int attn_waves(const AttnShape& sh) {
  const int G = sh.H / sh.Hkv;
  return (((sh.S / QT) * G) % 8 == 0) ? 8 : 4;
}

template <int NWV>
static void launch_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const AttnShape& sh,
                            hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_attn_fwd<NWV>, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * TILE_B);
    attr = true;
  }
  const int G = sh.H / sh.Hkv;
  const int nblk = sh.B * sh.Hkv * ((sh.S / QT) * G / NWV);
  hipLaunchKernelGGL(k_attn_fwd<NWV>, dim3(nblk), dim3(NWV * 64), 4 * TILE_B, s, (const __bf16*)q,
                     (const __bf16*)k, (const __bf16*)v, (__bf16*)o, lse, sh);
}

template <int NWV>
static void launch_attn_dq(const void* q, const void* k, const void* v, const void* dout, const float* lse,
                           const float* delta, void* dq, long long dqkv_rs, const AttnShape& sh, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_attn_bwd_dq<NWV>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              4 * TILE_B);
    attr = true;
  }
  const int G = sh.H / sh.Hkv;
  hipLaunchKernelGGL(k_attn_bwd_dq<NWV>, dim3(sh.B * sh.Hkv * ((sh.S / QT) * G / NWV)), dim3(NWV * 64), 4 * TILE_B,
                     s, (const __bf16*)q, (const __bf16*)k, (const __bf16*)v, (const __bf16*)dout, lse, delta,
                     (__bf16*)dq, dqkv_rs, sh);
}

// dK/dV kernel: PTO_ATTN_DKDV_PC=2 -> k_attn_bwd_dkdv_p3 (12 waves, two
// producers + one consumer per SIMD), 1 -> k_attn_bwd_dkdv_pc (8 waves,
// producer / consumer), 0 -> k_attn_bwd_dkdv (4 waves, one wave per SIMD).
static int attn_dkdv_pc() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PTO_ATTN_DKDV_PC");
    v = e ? atoi(e) : 1;
  }
  return v;
}

// PTO_ATTN_PC_KVWAIT=0 restores the producer loop without the explicit
// K/V-fragment wait (for A/B runs); default on.
static bool attn_pc_kvwait() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PTO_ATTN_PC_KVWAIT");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

template <bool KVW>
static void launch_attn_dkdv_pc(const void* q, const void* k, const void* v, const void* dout, const float* lse,
                                const float* delta, void* dk, void* dv, long long dqkv_rs, const AttnShape& sh,
                                hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_attn_bwd_dkdv_pc<KVW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              PC_LDS);
    attr = true;
  }
  hipLaunchKernelGGL(k_attn_bwd_dkdv_pc<KVW>, dim3(sh.B * sh.Hkv * (sh.S / KB)), dim3(2 * NT), PC_LDS, s,
                     (const __bf16*)q, (const __bf16*)k, (const __bf16*)v, (const __bf16*)dout, lse, delta,
                     (__bf16*)dk, (__bf16*)dv, dqkv_rs, sh);
}

PTO_API int pto_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int H,
                         int Hkv, long long q_rs, long long k_rs, long long v_rs, long long o_rs, float scale,
                         hipStream_t s) {
  const AttnShape sh = make_shape(B, S, H, Hkv, q_rs, k_rs, v_rs, o_rs, scale);
  if (!attn_shape_ok(sh)) return -1;
  if (attn_waves(sh) == 8)
    launch_attn_fwd<8>(q, k, v, o, lse, sh, s);
  else
    launch_attn_fwd<4>(q, k, v, o, lse, sh, s);
  return (int)hipGetLastError();
}

// delta = rowsum(dO * O); dq/dk/dv written at row stride dqkv_rs (the dQKV
// buffer; dk/dv point at the K / V column blocks).
PTO_API int pto_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                         const float* lse, float* delta, void* dq, void* dk, void* dv, long long dqkv_rs, int B,
                         int S, int H, int Hkv, long long q_rs, long long k_rs, long long v_rs, long long o_rs,
                         float scale, hipStream_t s) {
  const AttnShape sh = make_shape(B, S, H, Hkv, q_rs, k_rs, v_rs, o_rs, scale);
  if (!attn_shape_ok(sh)) return -1;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_attn_bwd_dkdv, hipFuncAttributeMaxDynamicSharedMemorySize,
                        4 * QTB + 2 * 128 * 4);
    attr = true;
  }
  const long long rows = (long long)B * S * H;
  hipLaunchKernelGGL(k_attn_bwd_delta, dim3((unsigned)((rows + 15) / 16)), dim3(256), 0, s, (const __bf16*)o,
                     (const __bf16*)dout, delta, sh);
  if (attn_dkdv_pc() == 2) {
    static bool attr3 = false;
    if (!attr3) {
      (void)hipFuncSetAttribute((const void*)k_attn_bwd_dkdv_p3, hipFuncAttributeMaxDynamicSharedMemorySize, P3_LDS);
      attr3 = true;
    }
    hipLaunchKernelGGL(k_attn_bwd_dkdv_p3, dim3(B * Hkv * (S / KB)), dim3(3 * NT), P3_LDS, s, (const __bf16*)q,
                       (const __bf16*)k, (const __bf16*)v, (const __bf16*)dout, lse, delta, (__bf16*)dk,
                       (__bf16*)dv, dqkv_rs, sh);
  } else if (attn_dkdv_pc()) {
    if (attn_pc_kvwait())
      launch_attn_dkdv_pc<true>(q, k, v, dout, lse, delta, dk, dv, dqkv_rs, sh, s);
    else
      launch_attn_dkdv_pc<false>(q, k, v, dout, lse, delta, dk, dv, dqkv_rs, sh, s);
  } else {
    hipLaunchKernelGGL(k_attn_bwd_dkdv, dim3(B * Hkv * (S / KB)), dim3(NT), 4 * QTB + 2 * 128 * 4, s,
                       (const __bf16*)q, (const __bf16*)k, (const __bf16*)v, (const __bf16*)dout, lse, delta,
                       (__bf16*)dk, (__bf16*)dv, dqkv_rs, sh);
  }
  if (attn_waves(sh) == 8)
    launch_attn_dq<8>(q, k, v, dout, lse, delta, dq, dqkv_rs, sh, s);
  else
    launch_attn_dq<4>(q, k, v, dout, lse, delta, dq, dqkv_rs, sh, s);
  return (int)hipGetLastError();
}
