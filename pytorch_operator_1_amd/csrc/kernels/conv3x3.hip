// ResNet-50's 3x3 convolutions (pad 1, stride 1 or 2) as an MFMA implicit
// GEMM over channels-last bf16, with the next BatchNorm's batch statistics
// reduced in the epilogue (BASELINE config 3).
//
// GEMM view: out[m][k] = sum_{tap, c} x[pixel(m) + tap][c] * w[k][tap][c],
// m = (n, oh, ow) output pixel, k = output channel, tap = (r, s) of the 3x3
// window, c = input channel.  Both operands are K-contiguous 128-byte rows
// per (row, tap, 64-channel slice): the A row is the input pixel's channel
// vector (or zeros in the padding), the B row the filter's -- so one K step
// is BK = 64 channels of ONE tap, and a block walks 9 * C / 64 such steps.
//
// Block: 256 threads = 4 waves laid out WM x WN (WM * WN = 4), each wave a
// 64 x 64 sub-tile = 2 x 2 v_mfma_f32_32x32x16_bf16 accumulators, so the
// block tile is (64 WM) x (64 WN): 256 x 64 for the 64-channel layer,
// 128 x 128 above.  Operands are staged global -> registers -> LDS, double
// buffered (the loads of step t+1 are in flight while step t's MFMAs run;
// one barrier per step), rows XOR-swizzled by 16-byte chunk (chunk q of row
// r at q ^ (r & 7)), so every fragment read (ds_read_b128: 32 rows x 16 B per
// half-wave) and every staging write hits 8 distinct 16-byte bank groups.
//
// Epilogue: the fp32 accumulators are rounded to bf16 once, written through
// LDS as 16-byte rows (coalesced NHWC stores), and -- optional -- the
// per-channel sum and sum of squares of the ROUNDED outputs over the
// block's rows land in part[mtile][2][K]: exactly what the BatchNorm
// statistics pass (bn_kernels.hip k_bn_stats) would have computed from the
// stored tensor, so the fused BN forward skips that full read of it.
//
// The input gradient of a stride-1 3x3 conv is the same convolution of dY
// with the filter flipped and transposed (w'[c][2-r][2-s][k] = w[k][r][s][c],
// k_conv3x3_wflip): the data-gradient path reuses this kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __bf16 c3_bf16x8 __attribute__((ext_vector_type(8)));
typedef float c3_f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned c3_u32x4 __attribute__((ext_vector_type(4)));  // 16-byte moves (HIP's uint4 struct copies
                                                                // compile to private-memory memcpys here)

constexpr int C3_T = 256;  // threads per block
constexpr int C3_BK = 64;  // channels per K step (one 128-byte row per operand row)

__device__ __forceinline__ uint16_t c3_f2bf(float f) {  // round to nearest even (finite inputs)
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float c3_bf2f(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }

// Staged operand rows: RB = 2 * BK bytes (BK channels of one tap), CPR =
// BK / 8 16-byte chunks.  Chunk q of row r sits at chunk q ^ key(r), key =
// (r / (256 / RB)) % CPR: the rows sharing one 256-byte bank row occupy its
// segments, and the key walks the chunk within the segment, so any 16
// consecutive rows read at one chunk index cover all 64 banks once (the
// MFMA fragment reads: 32 rows x one chunk per half-wave).
template <int RB>
__device__ __forceinline__ int c3_swz(int r, int q) {
  constexpr int RPB = 256 / RB, CPR = RB / 16;
  return r * RB + ((q ^ ((r / RPB) % CPR)) << 4);
}

// XCD-aware block order (cdna_hip_programming.md T1, the bijective form):
// hardware block b runs on XCD b % 8; logical ids are dealt so that each XCD
// gets a contiguous range -- the channel tiles of one pixel tile (adjacent
// logical ids) then share that XCD's L2 for their A rows.
__device__ __forceinline__ int c3_xcd_remap(int b, int nwg) {
  const int xcd = b & 7, local = b >> 3, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

// R: filter size, 3 (pad 1) or 1 (pad 0: the 1x1 convolutions are the same
// GEMM with one tap, so they share the kernel and its statistics epilogue).
// NB: LDS staging buffers.  2 (the 3x3 convs: 9 C / 64 K steps, the next
// step's tile staged while this one multiplies); 1 for the 1x1 convs (1-8
// K steps: half the LDS, so twice the workgroups per CU keep loads in
// flight, at the price of a second barrier per step).
// PERSIST: a grid of resident workgroups walks the tiles (tile = block +
// i * grid); otherwise one tile per workgroup (XCD-remapped).  A 1x1 conv's
// grid is 3k-12k short workgroups, whose dispatch alone (~3.5 ns each,
// profiles/mnist_step_pmc_r6.md) is a large share of its time.
template <int WM, int WN, int S, int BK, int PF, int R = 3, int NB = 2, bool PERSIST = false>
__global__ __launch_bounds__(C3_T) __attribute__((amdgpu_waves_per_eu(1, NB == 1 ? 4 : 2))) void k_conv3x3_fwd(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                      uint16_t* __restrict__ y, float* __restrict__ part, int N, int H,
                                                      int W, int C, int OH, int OW, int K) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  constexpr int RB = BK * 2, CPR = BK / 8;                 // bytes and 16-byte chunks per staged row
  constexpr int RPI = C3_T / CPR;                          // rows staged per pass of the block
  constexpr int AQ = BM / RPI, BQ = BN / RPI;              // 16-byte chunks per thread per step
  static_assert(AQ >= 1 && BQ >= 1 && BM % RPI == 0 && BN % RPI == 0, "tile / thread mismatch");
  extern __shared__ __attribute__((aligned(16))) unsigned char c3_smem[];
  // buffer b: A rows at c3_smem + b * BM * RB, B rows at Bs0 + b * BN * RB
  unsigned char* const Bs0 = c3_smem + NB * BM * RB;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv / WN, wn = wv % WN;
  const int M = N * OH * OW;
  // logical block -> (m tile, n tile), n fastest: the channel tiles of one
  // pixel tile are adjacent logical ids, i.e. on one XCD (c3_xcd_remap)
  const int ntn = K / BN;
  const int ntiles = ((M + BM - 1) / BM) * ntn;
  for (int lb = PERSIST ? (int)blockIdx.x : c3_xcd_remap(blockIdx.x, gridDim.x); lb < ntiles;
       lb = PERSIST ? lb + (int)gridDim.x : ntiles) {
  if (PERSIST) __syncthreads();  // the previous tile's epilogue reads of the LDS image are done
  const int mt = lb / ntn, nt = lb - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;

  // Operands through buffer loads (32-bit offsets, hardware range check):
  // a tap that falls in the padding gets an out-of-range offset and reads
  // zeros -- no per-element select, no 64-bit address math per load.
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(x), 0, N * H * W * C * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(w), 0, K * R * R * C * 2, 0x00020000);
  constexpr int C3_OOB = 0x7ffffff0;
  constexpr int P = R / 2;  // padding
  // per staged A chunk: byte offset of its row's window origin (pixel
  // (oh S - P, ow S - P), possibly in the padding) and the R*R-bit mask of
  // the taps that land inside the image
  const int q = tid % CPR, rsub = tid / CPR;
  int a_off[AQ], a_ok[AQ];
#pragma unroll
  for (int i = 0; i < AQ; ++i) {
    const int m = m0 + rsub + i * RPI;
    a_off[i] = 0;
    a_ok[i] = 0;
    if (m < M) {
      const int n = m / (OH * OW), rem = m - n * (OH * OW);
      const int oh = rem / OW, ow = rem - oh * OW;
      const int ih = oh * S - P, iw = ow * S - P;
      a_off[i] = (((n * H + ih) * W + iw) * C + q * 8) * 2;
#pragma unroll
      for (int tp = 0; tp < R * R; ++tp)
        if ((unsigned)(ih + tp / R) < (unsigned)H && (unsigned)(iw + tp % R) < (unsigned)W) a_ok[i] |= 1 << tp;
    }
  }
  int b_off[BQ];
#pragma unroll
  for (int i = 0; i < BQ; ++i) b_off[i] = ((n0 + rsub + i * RPI) * R * R * C + q * 8) * 2;
  const int csteps = C / BK, T = R * R * csteps;

  // Two register sets (P0, P1): with PF = 2 the loads of step t+2 are
  // issued while step t computes, so each tile has two steps' MFMA time to
  // arrive (one step was latency-bound: ~1.5 us per K step against 0.43 us
  // of MFMA work per SIMD, profiles/resnet50_r6.md); PF = 1 uses P0 only.
  c3_u32x4 ra0[AQ], rb0[BQ], ra1[AQ], rb1[BQ];
#define C3_LOAD(t_, RA, RBV)                                                                            \
  {                                                                                                     \
    const int tap_ = (t_) / csteps, c0_ = ((t_) - tap_ * csteps) * BK;                                 \
    const int r_ = tap_ / R, s_ = tap_ - r_ * R;                                                        \
    const int toff_ = ((r_ * W + s_) * C + c0_) * 2;                                                    \
    _Pragma("unroll") for (int i = 0; i < AQ; ++i) RA[i] = __builtin_bit_cast(                          \
        c3_u32x4, __builtin_amdgcn_raw_buffer_load_b128(                                                \
                      xr, ((a_ok[i] >> tap_) & 1) ? a_off[i] + toff_ : C3_OOB, 0, 0));                  \
    _Pragma("unroll") for (int i = 0; i < BQ; ++i) RBV[i] = __builtin_bit_cast(                         \
        c3_u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, b_off[i], (tap_ * C + c0_) * 2, 0));        \
  }
#define C3_STAGE(buf_, RA, RBV)                                                                         \
  {                                                                                                     \
    _Pragma("unroll") for (int i = 0; i < AQ; ++i) *reinterpret_cast<c3_u32x4*>(                        \
        c3_smem + (buf_) * (BM * RB) + c3_swz<RB>(rsub + i * RPI, q)) = RA[i];                          \
    _Pragma("unroll") for (int i = 0; i < BQ; ++i) *reinterpret_cast<c3_u32x4*>(                        \
        Bs0 + (buf_) * (BN * RB) + c3_swz<RB>(rsub + i * RPI, q)) = RBV[i];                             \
  }

  c3_f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = c3_f32x16{};
  const int fr = lane & 31, fh = lane >> 5;
// One K step from LDS buffer buf_: every fragment read of the step is
// issued first (16 ds_read_b128, 64 VGPRs), then the 16 MFMAs, each waiting
// only for its own operands (counted lgkmcnt) -- with fragment registers
// reused per 16-deep slice the reads of slice kk+1 waited for slice kk's
// MFMAs and every slice exposed the LDS latency.
#define C3_MATH(buf_)                                                                                   \
  {                                                                                                     \
    const unsigned char* A = c3_smem + (buf_) * (BM * RB);                                              \
    const unsigned char* B = Bs0 + (buf_) * (BN * RB);                                                  \
    c3_bf16x8 af[BK / 16][2], bf[BK / 16][2];                                                           \
    _Pragma("unroll") for (int kk = 0; kk < BK / 16; ++kk) _Pragma("unroll") for (int i = 0; i < 2; ++i) { \
      af[kk][i] = *reinterpret_cast<const c3_bf16x8*>(A + c3_swz<RB>(wm * 64 + i * 32 + fr, 2 * kk + fh)); \
      bf[kk][i] = *reinterpret_cast<const c3_bf16x8*>(B + c3_swz<RB>(wn * 64 + i * 32 + fr, 2 * kk + fh)); \
    }                                                                                                   \
    __builtin_amdgcn_sched_barrier(0); /* the scheduler would re-serialise them onto 16 VGPRs */          \
    _Pragma("unroll") for (int kk = 0; kk < BK / 16; ++kk) _Pragma("unroll") for (int i = 0; i < 2; ++i) \
        _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                   \
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kk][i], bf[kk][j], acc[i][j], 0, 0, 0); \
  }

  if (NB == 1) {
    C3_LOAD(0, ra0, rb0)
    C3_STAGE(0, ra0, rb0)
    __syncthreads();
    for (int t = 0; t < T; ++t) {
      if (t + 1 < T) C3_LOAD(t + 1, ra0, rb0)  // in flight under this step's MFMAs
      C3_MATH(0)
      if (t + 1 < T) {
        __syncthreads();  // every wave's fragment reads of the one buffer are done
        C3_STAGE(0, ra0, rb0)
      }
      __syncthreads();
    }
  } else if (PF == 1) {
    C3_LOAD(0, ra0, rb0)
    C3_STAGE(0, ra0, rb0)
    __syncthreads();
    for (int t = 0; t < T; ++t) {
      const int buf = t & 1;
      if (t + 1 < T) C3_LOAD(t + 1, ra0, rb0)  // in flight under this step's MFMAs
      C3_MATH(buf)
      if (t + 1 < T) C3_STAGE(buf ^ 1, ra0, rb0)  // the other buffer: last read one step ago
      __syncthreads();
    }
  } else {
    // P0 holds even tiles, P1 odd ones; LDS buffer = tile parity
    C3_LOAD(0, ra0, rb0)
    if (T > 1) C3_LOAD(1, ra1, rb1)
    C3_STAGE(0, ra0, rb0)
    __syncthreads();
    for (int t = 0; t < T; t += 2) {
      if (t + 2 < T) C3_LOAD(t + 2, ra0, rb0)
      C3_MATH(0)
      if (t + 1 < T) C3_STAGE(1, ra1, rb1)  // tile t+1: its loads were issued a step ago
      __syncthreads();
      if (t + 1 >= T) break;
      if (t + 3 < T) C3_LOAD(t + 3, ra1, rb1)
      C3_MATH(1)
      if (t + 2 < T) C3_STAGE(0, ra0, rb0)
      __syncthreads();
    }
  }
#undef C3_MATH
#undef C3_LOAD
#undef C3_STAGE

  // ---- epilogue: round once, statistics of the rounded values, rows
  // through LDS as 16-byte vectors.  Output tile image: [BM][BN] bf16 at
  // row stride BN*2 + 16 bytes (pad: the column writes below hit distinct
  // banks), then the [WM][2][BN] statistics partials, in the staging
  // buffers (free after the last barrier; the launcher sizes LDS for both).
  constexpr int OLD = BN * 2 + 16;
  unsigned char* O = c3_smem;
  float ssum[2] = {0.f, 0.f}, ssq[2] = {0.f, 0.f};  // per lane's column j (= wn*64 + j*32 + fr)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
        const int col = wn * 64 + j * 32 + fr;
        const bool valid = m0 + row < M;
        const uint16_t b = c3_f2bf(acc[i][j][e]);
        *reinterpret_cast<uint16_t*>(O + row * OLD + col * 2) = b;
        const float v = valid ? c3_bf2f(b) : 0.f;
        ssum[j] += v;
        ssq[j] = fmaf(v, v, ssq[j]);
      }
  float* red = reinterpret_cast<float*>(c3_smem + BM * OLD);  // [WM][2][BN]
  if (part) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // lanes l and l + 32 hold the same column
      ssum[j] += __shfl_xor(ssum[j], 32);
      ssq[j] += __shfl_xor(ssq[j], 32);
    }
    if (fh == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        red[(wm * 2 + 0) * BN + wn * 64 + j * 32 + fr] = ssum[j];
        red[(wm * 2 + 1) * BN + wn * 64 + j * 32 + fr] = ssq[j];
      }
    }
  }
  __syncthreads();
  if (part) {
    for (int c = tid; c < 2 * BN; c += C3_T) {
      const int which = c / BN, col = c - which * BN;
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < WM; ++g) v += red[(g * 2 + which) * BN + col];
      part[(long long)mt * 2 * K + which * K + n0 + col] = v;
    }
  }
  constexpr int RC = BN / 8;  // 16-byte chunks per output row
#pragma unroll
  for (int i = 0; i < BM * RC / C3_T; ++i) {
    const int e = tid + i * C3_T, row = e / RC, ch = e - row * RC;
    if (m0 + row < M)
      *reinterpret_cast<c3_u32x4*>(y + (long long)(m0 + row) * K + n0 + ch * 8) =
          *reinterpret_cast<const c3_u32x4*>(O + row * OLD + ch * 16);
  }
  }  // tile loop
}

// ---------------------------------------------------------------------------
// The same convolution with LDS-DMA staging (buffer_load ... lds): operand
// tiles go straight from memory into a 4-stage LDS ring, BK = 32 channels
// per K step (64-byte rows, 16 KB per stage at 128 x 128), three steps in
// flight ahead of the one being multiplied, each step retired by a counted
// vmcnt + a raw barrier (cdna_hip_programming.md §5 "Pipelining across
// barriers"; every VMEM op in the loop is an LDS-DMA, so the counts are
// exact).  Register staging (above) keeps one step in flight and paid the
// load latency on every step.  The DMA writes lane-linear LDS (wave base +
// 16 * lane), so the XOR swizzle is applied to the SOURCE chunk; padding
// taps read an out-of-range offset, which the DMA lands as zeros.

typedef __attribute__((address_space(3))) void* c3_lds_ptr;

// One 16-byte-per-lane LDS-DMA (wrapped: the target builtin used directly in
// the kernel body made host-side compilation drop the kernel's launch stub)
__device__ __forceinline__ void c3_dma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (c3_lds_ptr)lds, 16, voff, soff, 0, 0);
}

template <int N>
__device__ __forceinline__ void c3_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int WM, int WN, int S, int NBUF, int AHEAD>
__global__ __launch_bounds__(C3_T) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_conv3x3_fwd_dma(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y, float* __restrict__ part,
    int N, int H, int W, int C, int OH, int OW, int K) {
  constexpr int BM = 64 * WM, BN = 64 * WN, BK = 32, RB = 64, CPR = 4;
  constexpr int ROWS_PER_OP = 64 / CPR;              // rows one wave instruction lands (1 KB)
  constexpr int AOPS = BM / (4 * ROWS_PER_OP);       // DMA instructions per wave for A per step
  constexpr int BOPS = BN / (4 * ROWS_PER_OP);
  constexpr int LPS = AOPS + BOPS;                   // VMEM ops per thread per step
  constexpr int STAGE = (BM + BN) * RB;
  static_assert(AOPS >= 1 && BOPS >= 1 && NBUF * STAGE <= 163840 && AHEAD < NBUF && AHEAD >= 1, "ring");
  extern __shared__ __attribute__((aligned(16))) unsigned char c3_smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WN, wn = wv % WN;
  const int M = N * OH * OW;
  const int ntn = K / BN;
  const int lb = c3_xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lb / ntn, nt = lb - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(x), 0, N * H * W * C * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(w), 0, K * 9 * C * 2, 0x00020000);
  constexpr int C3_OOB = 0x7ffffff0;

  // the lane's row within each of its DMA ops, and the source chunk that
  // lands at its (linear) LDS slot: slot (lane & 3) of row r holds logical
  // chunk (lane & 3) ^ key(r)
  const int lrow = lane / CPR, lslot = lane % CPR;
  int a_off[AOPS], a_ok[AOPS];
#pragma unroll
  for (int i = 0; i < AOPS; ++i) {
    const int r = (i * 4 + wv) * ROWS_PER_OP + lrow;  // tile row
    const int ch = lslot ^ ((r >> 2) & 3);
    const int m = m0 + r;
    a_off[i] = 0;
    a_ok[i] = 0;
    if (m < M) {
      const int n = m / (OH * OW), rem = m - n * (OH * OW);
      const int oh = rem / OW, ow = rem - oh * OW;
      const int ih = oh * S - 1, iw = ow * S - 1;
      a_off[i] = (((n * H + ih) * W + iw) * C + ch * 8) * 2;
#pragma unroll
      for (int tp = 0; tp < 9; ++tp)
        if ((unsigned)(ih + tp / 3) < (unsigned)H && (unsigned)(iw + tp % 3) < (unsigned)W) a_ok[i] |= 1 << tp;
    }
  }
  int b_off[BOPS];
#pragma unroll
  for (int i = 0; i < BOPS; ++i) {
    const int r = (i * 4 + wv) * ROWS_PER_OP + lrow;
    b_off[i] = ((n0 + r) * 9 * C + (lslot ^ ((r >> 2) & 3)) * 8) * 2;
  }
  const int csteps = C / BK, T = 9 * csteps;

  // issue step t's DMA into ring stage t % NBUF (a macro, not a lambda: a
  // lambda holding these builtins lost the kernel's host-side launch stub)
#define C3D_ISSUE(t_)                                                                                    \
  {                                                                                                      \
    const int st_ = (t_) % NBUF;                                                                     \
    const int tap_ = (t_) / csteps, c0_ = ((t_) - tap_ * csteps) * BK;                                  \
    const int r_ = tap_ / 3, s_ = tap_ - r_ * 3;                                                         \
    const int toff_ = ((r_ * W + s_) * C + c0_) * 2;                                                     \
    unsigned char* base_ = c3_smem + st_ * STAGE;                                                        \
    _Pragma("unroll") for (int i = 0; i < AOPS; ++i)                                                     \
        c3_dma16(xr, base_ + (i * 4 + wv) * ROWS_PER_OP * RB,                                            \
                 ((a_ok[i] >> tap_) & 1) ? a_off[i] + toff_ : C3_OOB, 0);                                \
    _Pragma("unroll") for (int i = 0; i < BOPS; ++i)                                                     \
        c3_dma16(wr, base_ + BM * RB + (i * 4 + wv) * ROWS_PER_OP * RB, b_off[i], (tap_ * C + c0_) * 2);  \
  }

  c3_f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = c3_f32x16{};
  const int fr = lane & 31, fh = lane >> 5;

#pragma unroll
  for (int t = 0; t < AHEAD; ++t)
    if (t < T) C3D_ISSUE(t)
  for (int t = 0; t < T; ++t) {
    // steps issued beyond t: min(AHEAD - 1, T - 1 - t); wait until only theirs are in flight
    const int after = T - 1 - t;
    if (after >= AHEAD - 1) c3_wait_vm<(AHEAD - 1) * LPS>();
    else if constexpr (AHEAD > 2) {
      if (after == 1) c3_wait_vm<LPS>();
      else if (after == 2) c3_wait_vm<2 * LPS>();
      else if (after == 3) c3_wait_vm<(AHEAD > 4 ? 3 : 0) * LPS>();
      else if (after == 4) c3_wait_vm<(AHEAD > 5 ? 4 : 0) * LPS>();
      else if (after == 5) c3_wait_vm<(AHEAD > 6 ? 5 : 0) * LPS>();
      else if (after == 6) c3_wait_vm<(AHEAD > 7 ? 6 : 0) * LPS>();
      else c3_wait_vm<0>();
    } else {
      c3_wait_vm<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the stage refilled below are done
    __builtin_amdgcn_s_barrier();
    if (t + AHEAD < T) C3D_ISSUE(t + AHEAD)  // into stage (t + AHEAD) % NBUF, last read at step t + AHEAD - NBUF <= t - 1
    const unsigned char* A = c3_smem + (t % NBUF) * STAGE;
    const unsigned char* B = A + BM * RB;
    c3_bf16x8 af[BK / 16][2], bf[BK / 16][2];
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[kk][i] = *reinterpret_cast<const c3_bf16x8*>(A + c3_swz<RB>(wm * 64 + i * 32 + fr, 2 * kk + fh));
        bf[kk][i] = *reinterpret_cast<const c3_bf16x8*>(B + c3_swz<RB>(wn * 64 + i * 32 + fr, 2 * kk + fh));
      }
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kk][i], bf[kk][j], acc[i][j], 0, 0, 0);
  }
#undef C3D_ISSUE
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // every wave is done with the ring: the epilogue reuses it

  constexpr int OLD = BN * 2 + 16;
  unsigned char* O = c3_smem;
  float ssum[2] = {0.f, 0.f}, ssq[2] = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
        const int col = wn * 64 + j * 32 + fr;
        const bool valid = m0 + row < M;
        const uint16_t b = c3_f2bf(acc[i][j][e]);
        *reinterpret_cast<uint16_t*>(O + row * OLD + col * 2) = b;
        const float v = valid ? c3_bf2f(b) : 0.f;
        ssum[j] += v;
        ssq[j] = fmaf(v, v, ssq[j]);
      }
  float* red = reinterpret_cast<float*>(c3_smem + BM * OLD);
  if (part) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      ssum[j] += __shfl_xor(ssum[j], 32);
      ssq[j] += __shfl_xor(ssq[j], 32);
    }
    if (fh == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        red[(wm * 2 + 0) * BN + wn * 64 + j * 32 + fr] = ssum[j];
        red[(wm * 2 + 1) * BN + wn * 64 + j * 32 + fr] = ssq[j];
      }
    }
  }
  __syncthreads();
  if (part) {
    for (int c = tid; c < 2 * BN; c += C3_T) {
      const int which = c / BN, col = c - which * BN;
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < WM; ++g) v += red[(g * 2 + which) * BN + col];
      part[(long long)mt * 2 * K + which * K + n0 + col] = v;
    }
  }
  constexpr int RC = BN / 8;
#pragma unroll
  for (int i = 0; i < BM * RC / C3_T; ++i) {
    const int e = tid + i * C3_T, row = e / RC, ch = e - row * RC;
    if (m0 + row < M)
      *reinterpret_cast<c3_u32x4*>(y + (long long)(m0 + row) * K + n0 + ch * 8) =
          *reinterpret_cast<const c3_u32x4*>(O + row * OLD + ch * 16);
  }
}

// w'[c][2-r][2-s][k] = w[k][r][s][c] (bf16, channels-last filters): the
// stride-1 data gradient as a forward convolution of dY.  Also casts the fp32
// master filter when src32 is given (one launch for cast + flip).
__global__ __launch_bounds__(256) void k_conv3x3_wflip(const float* __restrict__ src32,
                                                       const uint16_t* __restrict__ src16, uint16_t* __restrict__ dst,
                                                       int K, int C) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)K * 9 * C) return;
  const int k = (int)(i % K);  // destination [c][tap'][k]: k fastest (coalesced stores)
  const long long rest = i / K;
  const int tp = (int)(rest % 9), c = (int)(rest / 9);
  const int tap = 8 - tp;  // (2 - r, 2 - s)
  const long long srci = ((long long)k * 9 + tap) * C + c;
  dst[i] = src32 ? c3_f2bf(src32[srci]) : src16[srci];
}

// fp32 channels-last filter [K][3][3][C] -> bf16 (same layout).
__global__ __launch_bounds__(256) void k_conv3x3_wcast(const float* __restrict__ src, uint16_t* __restrict__ dst,
                                                       long long n) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= n) return;
  const float4 v = *reinterpret_cast<const float4*>(src + i);
  uint2 o;
  o.x = (uint32_t)c3_f2bf(v.x) | ((uint32_t)c3_f2bf(v.y) << 16);
  o.y = (uint32_t)c3_f2bf(v.z) | ((uint32_t)c3_f2bf(v.w) << 16);
  *reinterpret_cast<uint2*>(dst + i) = o;
}

template <int WM, int WN, int S, int BK, int PF, int R = 3, int NB = 2, bool PERSIST = false>
int launch_fwd(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int OH, int OW, int K,
               hipStream_t s) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  const long long M = (long long)N * OH * OW;
  long long blocks = ((M + BM - 1) / BM) * (K / BN);
  if (blocks > 0x7fffffffLL || C % BK) return -1;
  const size_t stage = NB * (BM + BN) * (2 * BK), epi = BM * (BN * 2 + 16) + WM * 2 * BN * 4;
  const size_t lds = stage > epi ? stage : epi;
  if (PERSIST) {  // resident grid: CUs x workgroups per CU
    static int resident = 0;
    if (!resident) {
      int per_cu = 0, dev = 0, cus = 0;
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu, (const void*)k_conv3x3_fwd<WM, WN, S, BK, PF, R, NB, PERSIST>, C3_T, lds);
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      resident = (per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 256);
    }
    if (blocks > resident) blocks = resident;
  }
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv3x3_fwd<WM, WN, S, BK, PF, R, NB, PERSIST>), dim3((unsigned)blocks), dim3(C3_T), lds, s,
                     reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const uint16_t*>(w),
                     reinterpret_cast<uint16_t*>(y), part, N, H, W, C, OH, OW, K);
  return (int)hipGetLastError();
}

template <int WM, int WN, int S, int NBUF, int AHEAD>
int launch_dma(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int OH, int OW, int K,
               hipStream_t s) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  const long long M = (long long)N * OH * OW;
  const long long blocks = ((M + BM - 1) / BM) * (K / BN);
  if (blocks > 0x7fffffffLL || C % 32) return -1;
  const size_t stage = NBUF * (BM + BN) * 64, epi = BM * (BN * 2 + 16) + WM * 2 * BN * 4;
  const size_t lds = stage > epi ? stage : epi;
  static bool attr = false;
  if (!attr) {  // rings above 64 KB
    (void)hipFuncSetAttribute((const void*)k_conv3x3_fwd_dma<WM, WN, S, NBUF, AHEAD>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    attr = true;
  }
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv3x3_fwd_dma<WM, WN, S, NBUF, AHEAD>), dim3((unsigned)blocks), dim3(C3_T), lds, s,
                     reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const uint16_t*>(w),
                     reinterpret_cast<uint16_t*>(y), part, N, H, W, C, OH, OW, K);
  return (int)hipGetLastError();
}

// channel depth of a K step: 64 (128-byte rows, 64 KB of staging per
// 128 x 128 block) or 32 (half the LDS, twice the steps); the default and
// the per-variant timings: profiles/resnet50_r6.md
int g_c3_bk = 64, g_c3_pf = 1;

template <int WM, int WN, int S>
int launch_bk(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int OH, int OW, int K,
              hipStream_t s) {
  if (g_c3_pf == 3) return launch_dma<WM, WN, S, 4, 3>(x, w, y, part, N, H, W, C, OH, OW, K, s);
  if (g_c3_pf == 4) return launch_dma<WM, WN, S, 6, 5>(x, w, y, part, N, H, W, C, OH, OW, K, s);
  if (g_c3_pf == 5) return launch_dma<WM, WN, S, 8, 7>(x, w, y, part, N, H, W, C, OH, OW, K, s);
  if (g_c3_pf == 1)
    return g_c3_bk == 32 ? launch_fwd<WM, WN, S, 32, 1>(x, w, y, part, N, H, W, C, OH, OW, K, s)
                         : launch_fwd<WM, WN, S, 64, 1>(x, w, y, part, N, H, W, C, OH, OW, K, s);
  return g_c3_bk == 32 ? launch_fwd<WM, WN, S, 32, 2>(x, w, y, part, N, H, W, C, OH, OW, K, s)
                       : launch_fwd<WM, WN, S, 64, 2>(x, w, y, part, N, H, W, C, OH, OW, K, s);
}

// 1x1: register staging, BK 64, one step in flight (a 1x1 conv has C / 64
// K steps -- one to 32 -- so there is little to pipeline); g_c1_nb LDS
// buffers (pto_conv1x1_set_variant, the timing tool's knob)
int g_c1_nb = 1;
template <int WM, int WN, int S>
int launch_1x1(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int OH, int OW, int K,
               hipStream_t s) {
  if (g_c1_nb == 3) return launch_fwd<WM, WN, S, 64, 1, 1, 1, true>(x, w, y, part, N, H, W, C, OH, OW, K, s);
  return g_c1_nb == 1 ? launch_fwd<WM, WN, S, 64, 1, 1, 1>(x, w, y, part, N, H, W, C, OH, OW, K, s)
                      : launch_fwd<WM, WN, S, 64, 1, 1, 2>(x, w, y, part, N, H, W, C, OH, OW, K, s);
}

}  // namespace

#define PTO_API extern "C" __attribute__((visibility("default")))

// Tile shape for K output channels: 256 x 64 at K = 64, 128 x 128 up to
// K = 256, 64 x 256 above (fewer, wider column tiles where M is small).
// Variant knobs for the timing tool (tools/conv3x3_bench.py): K-step depth
// (32 / 64 channels) and register prefetch depth (1 / 2 steps); pf = 3 / 4 / 5:
// the LDS-DMA ring (k_conv3x3_fwd_dma, BK 32 whatever bk says) with 4 / 6 / 8
// stages, 3 / 5 / 7 steps in flight.
PTO_API int pto_conv3x3_set_variant(int bk, int pf) {
  if ((bk != 32 && bk != 64) || pf < 1 || pf > 5) return -1;
  g_c3_bk = bk;
  g_c3_pf = pf;
  return 0;
}

PTO_API int pto_conv3x3_tile_m(int K) { return K == 64 ? 256 : (K <= 256 ? 128 : 64); }

// y[N][OH][OW][K] = conv3x3(x[N][H][W][C], w[K][3][3][C]), pad 1, stride
// 1 or 2, bf16 channels-last; part (optional): [ceil(M / tile_m)][2][K]
// per-tile channel sums / sums of squares of the rounded outputs.
PTO_API int pto_conv3x3_fwd(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int K,
                            int stride, hipStream_t s) {
  if (N < 1 || H < 1 || W < 1 || C < 64 || C % 64 || K < 64 || K % 64 || (stride != 1 && stride != 2)) return -1;
  if ((((uintptr_t)x) | ((uintptr_t)w) | ((uintptr_t)y)) & 15) return -1;
  const int OH = (H + 2 - 3) / stride + 1, OW = (W + 2 - 3) / stride + 1;
  if ((long long)N * H * W * C >= (1LL << 31) || (long long)N * OH * OW * K >= (1LL << 31)) return -1;
  const int tm = pto_conv3x3_tile_m(K);
  if (tm == 256) return stride == 1 ? launch_bk<4, 1, 1>(x, w, y, part, N, H, W, C, OH, OW, K, s)
                                    : launch_bk<4, 1, 2>(x, w, y, part, N, H, W, C, OH, OW, K, s);
  if (tm == 128) {
    if (K % 128) return -1;
    return stride == 1 ? launch_bk<2, 2, 1>(x, w, y, part, N, H, W, C, OH, OW, K, s)
                       : launch_bk<2, 2, 2>(x, w, y, part, N, H, W, C, OH, OW, K, s);
  }
  if (K % 256) return -1;
  return stride == 1 ? launch_bk<1, 4, 1>(x, w, y, part, N, H, W, C, OH, OW, K, s)
                     : launch_bk<1, 4, 2>(x, w, y, part, N, H, W, C, OH, OW, K, s);
}

// 1 / 2: LDS staging buffers, one tile per workgroup; 3: one buffer and a
// resident grid walking the tiles
PTO_API int pto_conv1x1_set_variant(int nb) {
  if (nb < 1 || nb > 3) return -1;
  g_c1_nb = nb;
  return 0;
}

// y[N][OH][OW][K] = conv1x1(x[N][H][W][C], w[K][C]), stride 1 or 2 (pixel
// (oh S, ow S)), bf16 channels-last; part as for pto_conv3x3_fwd (same tile
// rows: pto_conv3x3_tile_m(K)).
PTO_API int pto_conv1x1_fwd(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int K,
                            int stride, hipStream_t s) {
  if (N < 1 || H < 1 || W < 1 || C < 64 || C % 64 || K < 64 || K % 64 || (stride != 1 && stride != 2)) return -1;
  if ((((uintptr_t)x) | ((uintptr_t)w) | ((uintptr_t)y)) & 15) return -1;
  const int OH = (H - 1) / stride + 1, OW = (W - 1) / stride + 1;
  if ((long long)N * H * W * C >= (1LL << 31) || (long long)N * OH * OW * K >= (1LL << 31)) return -1;
  const int tm = pto_conv3x3_tile_m(K);
  if (tm == 256) return stride == 1 ? launch_1x1<4, 1, 1>(x, w, y, part, N, H, W, C, OH, OW, K, s)
                                    : launch_1x1<4, 1, 2>(x, w, y, part, N, H, W, C, OH, OW, K, s);
  if (tm == 128) {
    if (K % 128) return -1;
    return stride == 1 ? launch_1x1<2, 2, 1>(x, w, y, part, N, H, W, C, OH, OW, K, s)
                       : launch_1x1<2, 2, 2>(x, w, y, part, N, H, W, C, OH, OW, K, s);
  }
  if (K % 256) return -1;
  return stride == 1 ? launch_1x1<1, 4, 1>(x, w, y, part, N, H, W, C, OH, OW, K, s)
                     : launch_1x1<1, 4, 2>(x, w, y, part, N, H, W, C, OH, OW, K, s);
}

// bf16 copy of an fp32 channels-last filter (n = K * 9 * C, n % 4 == 0).
PTO_API int pto_conv3x3_wcast(const float* src, void* dst, long long n, hipStream_t s) {
  if (n <= 0 || n % 4 || ((((uintptr_t)src) | ((uintptr_t)dst)) & 15)) return -1;
  hipLaunchKernelGGL(k_conv3x3_wcast, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, s, src,
                     reinterpret_cast<uint16_t*>(dst), n);
  return (int)hipGetLastError();
}

// dst[C][3][3][K] = flip(src[K][3][3][C]) (src fp32 when src32, else bf16).
PTO_API int pto_conv3x3_wflip(const float* src32, const void* src16, void* dst, int K, int C, hipStream_t s) {
  if (K < 1 || C < 1 || (!src32 && !src16)) return -1;
  const long long n = (long long)K * 9 * C;
  hipLaunchKernelGGL(k_conv3x3_wflip, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src32,
                     reinterpret_cast<const uint16_t*>(src16), reinterpret_cast<uint16_t*>(dst), K, C);
  return (int)hipGetLastError();
}
