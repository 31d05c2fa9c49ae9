// Fused fp32 kernels for the reference MNIST CNN training step on gfx950.
//
// Workload parity: reference examples/mnist/mnist.py:17-43 (Net + SGD step);
// op inventory K1..K10 in SURVEY.md §2.9.  The training step is 4 launches
// (train/fused_step.py):
//
//   F12  conv1+bias+ReLU+maxpool (VALU) and conv2+bias+ReLU+maxpool (MFMA
//        implicit GEMM, pool in registers), k_conv12_fwd2_t
//   F3   fc1+bias+ReLU (MFMA, split-K over 16 waves), k_linear_fwd_vec16
//   F4dx fc2+log_softmax+NLL+dlogits+dh1 on the matrix cores, then
//        d(a2p) = dh1 W1 per tile, k_fc2_ce_dx_mf
//   B    the whole backward (+ every parameter update in the one-process
//        schedule), k_bwd_all
//
// The single-op kernels (k_conv1_fwd, k_conv2_fwd, k_fc2_ce, k_conv2_bwd,
// k_conv1_bwd, ...) serve the evaluation pass and the autograd module path
// (ops/nn.py).
//
// Pool/ReLU backward never materialises a scattered tensor: each pooled
// output stores a 1-byte argmax code (0..3 = window position, 4 = no
// gradient because the pooled ReLU output is 0), and every backward kernel
// expands (pooled grad, code) on the fly.
//
// Latency rule used everywhere below: every operand a kernel needs was just
// written by the previous launch (usually on another XCD, so it is served
// from the Infinity Cache at ~1 us), hence each kernel issues ALL of its
// loads before consuming any of them — 1-3 dependent memory rounds per
// kernel instead of one per loop iteration.
//
// Batch cursor: the training data lives in HBM as [n_batches][B][...]; the
// kernels that read x / labels take a device pointer to the current batch
// index (`bidx`, advanced by the SGD launch), so a captured HIP graph walks
// the dataset without any copy kernels.
#include <stdlib.h>

#include "mfma_f32.h"
#include "sgd_f32.h"
#include "xgmi_ar.h"

// Phase timestamps for the timing probes under tools/probes (which define
// PTO_STAMP before including this file); nothing in the shipped library.
#ifndef PTO_STAMP
#define PTO_STAMP(k) ((void)0)
#define PTO_STAMP_SCOPE()
#endif

namespace {

constexpr int C1 = 20, C2 = 50, P1 = 12, F1OUT = 500, F1IN = 800, NCLS = 10;
constexpr int A1P = C1 * P1 * P1;  // 2880 floats of pooled conv1 output per sample

// torch semantics: relu() then max_pool2d(2,2): first strict max wins, a
// pooled value of 0 passes no gradient (relu'(0) = 0).
PTO_DEV void relu_pool4(const float v[4], float& out, uint8_t& code) {
  float m = v[0];
  int a = 0;
#pragma unroll
  for (int r = 1; r < 4; ++r)
    if (v[r] > m) { m = v[r]; a = r; }
  if (m > 0.f) { out = m; code = (uint8_t)a; }
  else { out = 0.f; code = 4; }
}

PTO_DEV const float* batch_ptr(const float* base, const long long* bidx, int per_batch) {
  return bidx ? base + (size_t)(*bidx) * per_batch : base;
}

// "Fused optimizer" schedule of the single-process step (no gradient
// all-reduce between backward and the update): the optimizer runs inside
// launches that already exist instead of a separate SGD launch.
//   * fc + conv2 parameters: updated inside k_bwd_all by the block that
//     finishes their gradient (no later launch of the step reads them).
//   * conv1 parameters: their grads are final only when k_bwd_all ends, and
//     F12 of the NEXT step is their first reader.  F12 applies the pending
//     update on the fly while staging the weights (LazyConv1), and F4dx of
//     that step (which does not read conv1) commits it: p, m written, g
//     zeroed (Conv1Commit).  `pending` (set by k_bwd_all) says whether an
//     update is owed; the host flushes it before anyone reads the parameters.
//   * batch cursor: advanced by k_bwd_all (nothing later in the step reads
//     it: F12 copied the images out for the backward).
struct LazyConv1 {
  const float* g;       // flat conv1 grads: weights [0, 500), bias [bias_off, +20)
  const float* m;       // flat conv1 momentum, same layout
  const int* pending;   // nullptr: plain forward
  SgdArgs a;
  int bias_off;
  float* xout;          // nullptr, or [B][784]: the batch's images copied out for B1 (no cursor hop there)
  float* w2out;         // nullptr, or [50][500]: conv2.weight as read here (k_bwd_all's dgrad reads it)
  const float* rep;     // extra gradient replicas (k_bwd_all): g + sum_r rep[r*rep_stride + i], r < nrep-1
  int nrep, rep_stride;
};
constexpr int C1_MAXREP = 256;  // max conv1 gradient replicas (launchers check)
constexpr int REP_CHUNK = 16;   // replica loads the readers keep in flight at once
struct Conv1Commit {
  float* p;             // flat conv1 range [0, n) of params / grads / momentum
  float* g;
  float* m;
  int n;                // multiple of 4
  const int* pending;   // nullptr: no commit
  SgdArgs a;
  float* rep;           // extra gradient replicas, summed into the update and re-zeroed
  int nrep, rep_stride;
  int* zero_word;       // F4dx: reset to 0 (the overlapped step's conv-role counter), or nullptr
};

// Conv1Commit's update of 4 elements at i: the gradient is the sum of the
// primary slot and the replicas; all of them are zeroed.
PTO_DEV void commit4(const Conv1Commit& cm, int i, float lr) {
  if (cm.nrep <= 1) {
    sgd_flat4(cm.p, cm.g, cm.m, i, lr, cm.a);
    return;
  }
  // the parameter / momentum loads first: in flight with the gradient and
  // replica loads (after the replica zeroing stores they were a second
  // round trip -- the compiler cannot move them above possibly aliasing stores)
  float4 pv = *reinterpret_cast<float4*>(cm.p + i);
  float4 mv = *reinterpret_cast<float4*>(cm.m + i);
  float4 gs = *reinterpret_cast<const float4*>(cm.g + i);
  for (int r0 = 0; r0 < cm.nrep - 1; r0 += REP_CHUNK) {
    float4 v[REP_CHUNK];  // a chunk of replica loads in flight before the first add
#pragma unroll
    for (int r = 0; r < REP_CHUNK; ++r)
      v[r] = *reinterpret_cast<const float4*>(cm.rep + (size_t)min(r0 + r, cm.nrep - 2) * cm.rep_stride + i);
#pragma unroll
    for (int r = 0; r < REP_CHUNK; ++r) {
      if (r0 + r >= cm.nrep - 1) break;
      gs.x += v[r].x; gs.y += v[r].y; gs.z += v[r].z; gs.w += v[r].w;
      *reinterpret_cast<float4*>(cm.rep + (size_t)(r0 + r) * cm.rep_stride + i) = float4{0.f, 0.f, 0.f, 0.f};
    }
  }
  sgd_elem(pv.x, gs.x, mv.x, lr, cm.a.mom, cm.a.wd, cm.a.gscale, cm.a.nesterov);
  sgd_elem(pv.y, gs.y, mv.y, lr, cm.a.mom, cm.a.wd, cm.a.gscale, cm.a.nesterov);
  sgd_elem(pv.z, gs.z, mv.z, lr, cm.a.mom, cm.a.wd, cm.a.gscale, cm.a.nesterov);
  sgd_elem(pv.w, gs.w, mv.w, lr, cm.a.mom, cm.a.wd, cm.a.gscale, cm.a.nesterov);
  *reinterpret_cast<float4*>(cm.p + i) = pv;
  *reinterpret_cast<float4*>(cm.m + i) = mv;
  *reinterpret_cast<float4*>(cm.g + i) = float4{0.f, 0.f, 0.f, 0.f};
}

// s0 + the nrep-1 extra conv1 gradient replicas at index i (s0 if !live),
// added one by one in replica order starting from the primary slot s0 --
// the association commit4 and the xGMI fold use, so the lazily applied and
// the committed update are bit-identical (deterministic resume).  REP_CHUNK
// loads are issued before the first add (clamped addresses, branch-free): a
// plain runtime-bound loop compiled to one dependent memory round trip per
// replica, ~1 us of F12's critical path at nrep = 8.
PTO_DEV float rep_sum(const float* __restrict__ rep, int nrep, int stride, int i, bool live, float s0) {
  float s = s0;
  for (int r0 = 0; r0 < nrep - 1; r0 += REP_CHUNK) {
    float v[REP_CHUNK];
#pragma unroll
    for (int r = 0; r < REP_CHUNK; ++r) v[r] = rep[(size_t)min(r0 + r, nrep - 2) * stride + i];
#pragma unroll
    for (int r = 0; r < REP_CHUNK; ++r) s += (live && r0 + r < nrep - 1) ? v[r] : 0.f;
  }
  return s;
}

// ---------------------------------------------------------------- F1 ----
// thread = (sample, 4-channel group, pooled pixel); 6x6 input patch in
// registers, 4 channels x 4 window positions x 25 taps.
__global__ __launch_bounds__(256) void k_conv1_fwd(const float* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ bias, float* __restrict__ out,
                                                   uint8_t* __restrict__ code, int B,
                                                   const long long* __restrict__ bidx) {
  __shared__ float ws[C1 * 25];
  __shared__ float bs[C1];
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const bool active = idx < B * 720;
  const int b = idx / 720, rem = idx - b * 720, cg = rem / 144, pix = rem - cg * 144;
  const int ph = pix / 12, pw = pix - ph * 12;
  // issue the patch loads before the weight staging barrier
  float p[6][6];
  x = batch_ptr(x, bidx, B * 784);
  const float* xb = x + (active ? b * 784 + (2 * ph) * 28 + 2 * pw : 0);
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int c = 0; c < 6; ++c) p[r][c] = xb[r * 28 + c];
  for (int i = threadIdx.x; i < C1 * 25; i += 256) ws[i] = w[i];
  if (threadIdx.x < C1) bs[threadIdx.x] = bias[threadIdx.x];
  __syncthreads();
  if (!active) return;
#pragma unroll
  for (int cc = 0; cc < 4; ++cc) {
    const int oc = cg * 4 + cc;
    const float* wc = ws + oc * 25;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int dy = q >> 1, dx = q & 1;
      float s = bs[oc];
#pragma unroll
      for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) s = fmaf(p[dy + kh][dx + kw], wc[kh * 5 + kw], s);
      v[q] = s;
    }
    float o;
    uint8_t cd;
    relu_pool4(v, o, cd);
    const int oi = ((b * C1 + oc) * P1 + ph) * P1 + pw;
    out[oi] = o;
    code[oi] = cd;
  }
}

// ---------------------------------------------------------------- F2 ----
// Implicit GEMM: rows m = (sample, pooled pixel, window pos), cols = out
// channel, K = (ic, kh, kw) = 500.  Block = (sample, 16-channel tile); wave
// w = pooled row t (16 rows = 4 pooled pixels x 4 window positions), laid
// out so that lane l's 4 accumulator registers ARE one pooling window ->
// ReLU+maxpool happen in registers.
// K order per group G (25 groups): lane group g takes (ic,kh) row R=4G+g
// and MFMA j takes kw=j, so K=500 is covered exactly by 125 MFMAs.
// Both operands are staged in LDS with coalesced float4 loads: the weight
// tile (16 x 500, row stride 501 -> conflict-free column reads) and the
// whole pooled conv1 map of the sample (20 x 12 x 12).
constexpr int WS_LD = 502;  // n*502 mod 32 are the 16 even banks: B reads (n, 5g) conflict-free
__global__ __launch_bounds__(256) void k_conv2_fwd(const float* __restrict__ a1p, const float* __restrict__ w2,
                                                   const float* __restrict__ b2, float* __restrict__ a2p,
                                                   uint8_t* __restrict__ code2, int B) {
  __shared__ float ws[16 * WS_LD];
  __shared__ __attribute__((aligned(16))) float in_s[A1P];
  const int b = blockIdx.x >> 2, nt = blockIdx.x & 3;
  const int tid = threadIdx.x;
  {
    const int nrows = min(16, C2 - nt * 16);  // 16,16,16,2
    const float4* wsrc = reinterpret_cast<const float4*>(w2 + nt * 16 * 500);
    const float4* isrc = reinterpret_cast<const float4*>(a1p + b * A1P);
    float4 wv[8], iv[3];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + 256 * q;  // float4 index inside the 16x500 tile
      wv[q] = (e < nrows * 125) ? wsrc[e] : float4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int e = tid + 256 * q;
      iv[q] = (e < A1P / 4) ? isrc[e] : float4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + 256 * q;
      if (e < 2000) {
        const int row = e / 125, col = (e - row * 125) * 4;
        float* d = ws + row * WS_LD + col;
        d[0] = wv[q].x; d[1] = wv[q].y; d[2] = wv[q].z; d[3] = wv[q].w;
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int e = tid + 256 * q;
      if (e < A1P / 4) reinterpret_cast<float4*>(in_s)[e] = iv[q];
    }
  }
  __syncthreads();
  const int t = tid >> 6, lane = tid & 63;
  const int i = lane & 15, g = lane >> 4;
  const int pw = i >> 2, dy = (i >> 1) & 1, dx = i & 1;
  const int n = nt * 16 + (lane & 15);
  const float* wl = ws + (lane & 15) * WS_LD + 5 * g;
  const float* il = in_s + (2 * t + dy) * 12 + 2 * pw + dx;
  f32x4 acc0 = zero4(), acc1 = zero4();
#pragma unroll
  for (int G = 0; G < 25; ++G) {
    const int R = 4 * G + g;
    const int ic = R / 5, kh = R - ic * 5;
    const float* arow = il + ic * 144 + kh * 12;
    const float* brow = wl + 20 * G;
    acc0 = mfma16x16x4(arow[0], brow[0], acc0);
    acc1 = mfma16x16x4(arow[1], brow[1], acc1);
    acc0 = mfma16x16x4(arow[2], brow[2], acc0);
    acc1 = mfma16x16x4(arow[3], brow[3], acc1);
    acc0 = mfma16x16x4(arow[4], brow[4], acc0);
  }
  const f32x4 acc = acc0 + acc1;
  if (n >= C2 || b >= B) return;
  const float bn = b2[n];
  float v[4] = {acc[0] + bn, acc[1] + bn, acc[2] + bn, acc[3] + bn};
  float o;
  uint8_t cd;
  relu_pool4(v, o, cd);
  const int oi = b * F1IN + n * 16 + t * 4 + (lane >> 4);
  a2p[oi] = o;
  code2[oi] = cd;
}

// -------------------------------------------------------------- F1+F2 ----
// conv1 and conv2 forward in ONE launch.  Block = (sample, 16-channel conv2
// tile), 1024 threads; each block recomputes the sample's whole pooled conv1
// map straight into LDS (2880 outputs x 100 FMAs: cheaper than a kernel
// boundary) and the nt == 0 block also writes it (+ argmax codes) to HBM for
// the backward pass.
//  * conv1: a lane task is (channel pair, pooled pixel): 100 packed FMAs
//    (v_pk_fma_f32, the pair's weights interleaved in LDS), the 6x6 input
//    patch read as float2 pairs.  20 full wave tasks (pair x 64-pixel chunk,
//    wave-uniform weights, broadcast b128 reads) + 3 tail tasks (4 pairs x
//    the last 16 pixels).
//  * conv2 implicit GEMM (k_conv2_fwd's lane maps): K split over the four
//    wave sets (7+6+6+6 groups of 5 MFMAs), partial tiles combined through
//    LDS, so each SIMD interleaves independent MFMA chains.
//  * lazy conv1 update (one-process schedule, LazyConv1), the image copy
//    for the backward (xout) and the conv2.weight snapshot (w2out).
//  * ARM != 0 (overlapped multi-GPU step, fused_step.py "ddp-xgmi"): the
//    PREVIOUS step's gradient exchange runs as two roles ahead of the conv
//    blocks in the grid (protocol ARM-1):
//      cv.nblk blocks  the conv exchange (xgmi_ar.h ar_role_oneshot_sgd:
//                      one-shot all-reduce + SGD of conv2/conv1, 100 KB);
//                      the conv blocks wait on cv.ready (one lane, bounded)
//                      before reading conv1/conv2, then read them with
//                      system-scope loads.  No launch of its own between
//                      the backward and this forward any more.
//      ar.nblk blocks  the fc exchange (ar_role_sgd), which nothing here
//                      reads: it runs concurrently with the convolutions.
//    Role blocks come first in the grid, so they are resident before any
//    conv block can wait on them.  B == 0: the roles alone (the closing
//    launch of a captured run).  The kernel is capped at 64 VGPRs (8 waves
//    per SIMD) so a role block fits on a CU next to a conv block.
struct ArRole {
  const pto_ar::ArPeers* peers;
  long long off, n4;
  int rank, world, chan, nblk;
  uint32_t* epochs;
  int* err;
  long long timeout;
  pto_ar::ArSgd f;
  int* ready;  // conv role: one add per workgroup once its parameters are stored
};

// Read access to a parameter tensor.  SYS: system-scope buffer loads (sc0
// sc1: miss this CU's L1 and serve the line written through by a role
// workgroup of the SAME launch, wherever it ran); otherwise plain loads.
template <bool SYS>
struct ParamView {
  const float* p;
  __amdgpu_buffer_rsrc_t r;
  PTO_DEV ParamView(const float* base, int n) : p(base) {
    if constexpr (SYS) r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, n * 4, 0x00020000);
  }
  PTO_DEV float operator[](int i) const {
    if constexpr (SYS)
      return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, i * 4, 0, pto_ar::AUX_SYS));
    else
      return p[i];
  }
  PTO_DEV float4 v4(int i4) const {
    if constexpr (SYS)
      return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, i4 * 16, 0, pto_ar::AUX_SYS));
    else
      return reinterpret_cast<const float4*>(p)[i4];
  }
};

// A conv workgroup of the overlapped step waits here (one lane) until every
// conv-role workgroup of its launch has published (ar_role_oneshot_sgd), or
// the exchange failed, or the bounded spin ran out (err bit 16).  Every role
// workgroup publishes even on failure, so the spin ends in every case.
PTO_DEV void wait_conv_role(const ArRole& cv) {
  const long long t0 = wall_clock64();
  for (;;) {
    // the counter and the error word in flight together: one round trip per poll
    const int r = __hip_atomic_load(cv.ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int ev = __hip_atomic_load(cv.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (r >= cv.nblk || ev != 0) break;
    if (wall_clock64() - t0 > cv.timeout) {
      atomicOr(cv.err, 16);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
constexpr int W1PLD = 52;  // a channel pair's 25 interleaved taps, padded to whole float4
template <int NTH, int ARM = 0>
__global__ __launch_bounds__(NTH, ARM ? 2 * NTH / 256 : 1) void k_conv12_fwd2_t(
    const float* __restrict__ x, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2, float* __restrict__ a1p, uint8_t* __restrict__ code1,
    float* __restrict__ a2p, uint8_t* __restrict__ code2, int B, const long long* __restrict__ bidx, LazyConv1 lz,
    ArRole ar, ArRole cv) {
  // role blocks FIRST in the grid: they are dispatched before the conv
  // blocks, so their latency chains start at once (and the conv blocks that
  // wait on the conv role can never hold the CU slots it needs)
  int bx = (int)blockIdx.x;
  if constexpr (ARM != 0) {
    if (bx < cv.nblk + ar.nblk) {
      PTO_STAMP_SCOPE();
      __shared__ float4 ar_lds[NTH];
      if (bx < cv.nblk)
        pto_ar::ar_role_oneshot_sgd<ARM == 2, NTH>(cv.peers, cv.off, cv.n4, cv.rank, cv.world, cv.chan, cv.epochs,
                                                   cv.err, cv.timeout, cv.f, bx, ar_lds, cv.ready);
      else
        pto_ar::ar_role_sgd<ARM == 2, NTH>(ar.peers, ar.off, ar.n4, ar.rank, ar.world, ar.chan, ar.epochs, ar.err,
                                           ar.timeout, ar.f, bx - cv.nblk, ar_lds);
      return;
    }
    bx -= cv.nblk + ar.nblk;
  }
  constexpr bool SYS = ARM != 0;  // conv parameters written by this launch's conv role
  __shared__ float ws[16 * WS_LD];
  __shared__ __attribute__((aligned(16))) float in_s[A1P];
  __shared__ __attribute__((aligned(16))) float xs[784];
  __shared__ float b1s[C1];
  // the full tasks' channel pairs interleaved, (w[2p][k], w[2p+1][k]) per
  // tap: the b128 loads land as the packed FMA's weight pairs directly
  // (from per-channel rows the compiler spent ~43 v_mov per task pairing them)
  __shared__ __attribute__((aligned(16))) float w1p[(C1 / 2) * W1PLD];
  constexpr int NWV = NTH / 64, NPART = NTH / 256;  // waves; K parts of the conv2 GEMM
  __shared__ __attribute__((aligned(16))) float red[(NPART - 1) * 1024];
  PTO_STAMP_SCOPE();
  const int b = bx >> 2, nt = bx & 3;
  const int tid = threadIdx.x;
  {
    x = batch_ptr(x, bidx, B * 784);
    const float4 xv = tid < 196 ? reinterpret_cast<const float4*>(x + b * 784)[tid] : float4{0.f, 0.f, 0.f, 0.f};
    if constexpr (ARM != 0) {
      if (tid == 0) wait_conv_role(cv);
      __syncthreads();
      PTO_STAMP(5);
    }
    const int nrows = min(16, C2 - nt * 16);
    const ParamView<SYS> wsrc(w2 + nt * 16 * 500, nrows * 500);
    float4 wv[2048 / NTH];
#pragma unroll
    for (int q = 0; q < 2048 / NTH; ++q) {
      const int e = tid + NTH * q;
      wv[q] = (e < nrows * 125) ? wsrc.v4(e) : float4{0.f, 0.f, 0.f, 0.f};
    }
    constexpr int QW1 = (C1 * 26 + NTH - 1) / NTH;
    float wq[QW1], gq[QW1], mq[QW1];
    const ParamView<SYS> w1v(w1, C1 * 25), b1v(b1, C1);
#pragma unroll
    for (int q = 0; q < QW1; ++q) {
      const int e = tid + NTH * q;
      wq[q] = e < C1 * 25 ? w1v[e] : (e < C1 * 26 ? b1v[e - C1 * 25] : 0.f);
    }
    int pend = 0;
    float lr = 0.f;
    if (lz.pending) {
      pend = *lz.pending;
      lr = *lz.a.lr;
#pragma unroll
      for (int q = 0; q < QW1; ++q) {
        const int e = tid + NTH * q;
        const int fi = e < C1 * 25 ? e : lz.bias_off + (e - C1 * 25);
        const float gsum = rep_sum(lz.rep, lz.nrep, lz.rep_stride, e < C1 * 26 ? fi : 0, e < C1 * 26,
                                   e < C1 * 26 ? lz.g[fi] : 0.f);
        gq[q] = gsum;
        mq[q] = e < C1 * 26 ? lz.m[fi] : 0.f;
      }
    }
    if (pend) {
#pragma unroll
      for (int q = 0; q < QW1; ++q) sgd_elem(wq[q], gq[q], mq[q], lr, lz.a.mom, lz.a.wd, lz.a.gscale, lz.a.nesterov);
    }
#pragma unroll
    for (int q = 0; q < 2048 / NTH; ++q) {
      const int e = tid + NTH * q;
      if (e < 2000) {
        const int row = e / 125, col = (e - row * 125) * 4;
        float* d = ws + row * WS_LD + col;
        d[0] = wv[q].x; d[1] = wv[q].y; d[2] = wv[q].z; d[3] = wv[q].w;
      }
    }
    if (tid < 196) {
      reinterpret_cast<float4*>(xs)[tid] = xv;
      if (lz.xout && nt == 0) reinterpret_cast<float4*>(lz.xout + b * 784)[tid] = xv;
    }
    if (lz.w2out && b == 0) {  // conv2.weight snapshot: rows nt*16.. (one writer per row)
#pragma unroll
      for (int q = 0; q < 2048 / NTH; ++q) {
        const int e = tid + NTH * q;
        if (e < nrows * 125) reinterpret_cast<float4*>(lz.w2out + nt * 16 * 500)[e] = wv[q];
      }
    }
#pragma unroll
    for (int q = 0; q < QW1; ++q) {
      const int e = tid + NTH * q;
      if (e < C1 * 25) {
        const int oc = e / 25, k = e - oc * 25;
        w1p[(oc >> 1) * W1PLD + 2 * k + (oc & 1)] = wq[q];
      } else if (e < C1 * 26) {
        b1s[e - C1 * 25] = wq[q];
      }
    }
  }
  __syncthreads();
  PTO_STAMP(1);
  const int wid = tid >> 6, lane = tid & 63;
  // conv1 + bias + ReLU + pool as (channel pair, pooled pixel) lane tasks,
  // every one the same 100 packed FMAs: 20 full wave tasks (10 pairs x the
  // two 64-pixel chunks, weights wave-uniform) + 3 tail tasks for pixels
  // 128..143 (lane = 4 pairs x 16 pixels, per-lane weight rows).  23 tasks
  // on 16 waves: at most 6 per SIMD (the per-channel tail tasks of unpacked
  // FMAs made it 25 tasks, up to 7 per SIMD).
  static_assert(NTH == 1024, "F12 is laid out for 16 waves");
  constexpr int CPT = 2;
  constexpr int NPAIR = C1 / CPT, NFULL = 2 * NPAIR, NTASK = NFULL + (NPAIR + 3) / 4;
  for (int si = 0; si < 2; ++si) {
    const int task = wid + NWV * si;
    if (task >= NTASK) break;
    int cg, pix;
    bool live = true;
    if (task < NFULL) {
      cg = task >> 1;
      pix = (task & 1) * 64 + lane;
    } else {
      cg = (task - NFULL) * 4 + (lane >> 4);
      pix = 128 + (lane & 15);
      live = cg < NPAIR;
      cg = min(cg, NPAIR - 1);
    }
    static_assert(CPT == 2, "w1p interleaves channel pairs");
    float wp[W1PLD], bz[CPT];
#pragma unroll
    for (int j = 0; j < W1PLD / 4; ++j) {
      const float4 v = *reinterpret_cast<const float4*>(w1p + cg * W1PLD + 4 * j);
      wp[4 * j] = v.x; wp[4 * j + 1] = v.y; wp[4 * j + 2] = v.z; wp[4 * j + 3] = v.w;
    }
#pragma unroll
    for (int cc = 0; cc < CPT; ++cc) bz[cc] = b1s[cg * CPT + cc];
    if (!live) continue;
    const int ph = pix / 12, pw = pix - ph * 12;
    float p[6][6];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int c = 0; c < 6; c += 2) {
        const float2 v = *reinterpret_cast<const float2*>(xs + (2 * ph + r) * 28 + 2 * pw + c);
        p[r][c] = v.x;
        p[r][c + 1] = v.y;
      }
    // the task's two channels as one packed pair: every tap is one
    // v_pk_fma_f32 (input pixel broadcast to both halves, the two channels'
    // weights as the pair), 100 instead of 200 FMA issues per lane; each
    // half is the same fmaf chain as a scalar sum (bitwise equal)
    static_assert(CPT == 2, "conv1 full tasks pack two channels");
    f32x2 s2[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int dy = q >> 1, dx = q & 1;
      f32x2 acc2 = f32x2{bz[0], bz[1]};
#pragma unroll
      for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const float pv = p[dy + kh][dx + kw];
          acc2 = __builtin_elementwise_fma(f32x2{pv, pv}, f32x2{wp[2 * (kh * 5 + kw)], wp[2 * (kh * 5 + kw) + 1]},
                                           acc2);
        }
      s2[q] = acc2;
    }
#pragma unroll
    for (int cc = 0; cc < CPT; ++cc) {
      const int oc = cg * CPT + cc;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = s2[q][cc];
      float o;
      uint8_t cd;
      relu_pool4(v, o, cd);
      in_s[oc * 144 + pix] = o;
      if (nt == 0) {
        a1p[b * A1P + oc * 144 + pix] = o;
        code1[b * A1P + oc * 144 + pix] = cd;
      }
    }
  }
  __syncthreads();
  PTO_STAMP(2);
  // conv2 implicit GEMM (k_conv2_fwd's lane maps), K (25 groups of 5 MFMAs)
  // split over NPART wave sets: 13+12 (512 threads) or 7+6+6+6 (1024)
  const int t = wid & 3, half = wid >> 2;
  const int i = lane & 15, g = lane >> 4;
  const int pw = i >> 2, dy = (i >> 1) & 1, dx = i & 1;
  const int n = nt * 16 + (lane & 15);
  const float* wl = ws + (lane & 15) * WS_LD + 5 * g;
  const float* il = in_s + (2 * t + dy) * 12 + 2 * pw + dx;
  f32x4 acc0 = zero4(), acc1 = zero4();
  auto group = [&](int G) {
    const int R = 4 * G + g;
    const int ic = R / 5, kh = R - ic * 5;
    const float* arow = il + ic * 144 + kh * 12;
    const float* brow = wl + 20 * G;
    acc0 = mfma16x16x4(arow[0], brow[0], acc0);
    acc1 = mfma16x16x4(arow[1], brow[1], acc1);
    acc0 = mfma16x16x4(arow[2], brow[2], acc0);
    acc1 = mfma16x16x4(arow[3], brow[3], acc1);
    acc0 = mfma16x16x4(arow[4], brow[4], acc0);
  };
  if (NPART == 2) {
    if (half == 0) {
#pragma unroll
      for (int G = 0; G < 13; ++G) group(G);
    } else {
#pragma unroll
      for (int G = 13; G < 25; ++G) group(G);
    }
  } else {
    if (half == 0) {
#pragma unroll
      for (int G = 0; G < 7; ++G) group(G);
    } else {
      const int g0 = 7 + 6 * (half - 1);
#pragma unroll
      for (int G = 0; G < 6; ++G) group(g0 + G);
    }
  }
  f32x4 acc = acc0 + acc1;
  if (half != 0) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) red[(half - 1) * 1024 + t * 256 + rr * 64 + lane] = acc[rr];
  }
  __syncthreads();
  PTO_STAMP(3);
  if (half != 0) return;
#pragma unroll
  for (int pp = 0; pp < NPART - 1; ++pp)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) acc[rr] += red[pp * 1024 + t * 256 + rr * 64 + lane];
  if (n >= C2 || b >= B) return;
  const float bn = ParamView<SYS>(b2, C2)[n];
  float v[4] = {acc[0] + bn, acc[1] + bn, acc[2] + bn, acc[3] + bn};
  float o;
  uint8_t cd;
  relu_pool4(v, o, cd);
  const int oi = b * F1IN + n * 16 + t * 4 + (lane >> 4);
  a2p[oi] = o;
  code2[oi] = cd;
}

// ---------------------------------------------------------------- F3 ----
struct EpiBiasRelu {
  const float* bias; float* out; int ld; bool relu;
  PTO_DEV void operator()(int m, int n, float v) const {
    v += bias ? bias[n] : 0.f;
    out[m * ld + n] = relu ? fmaxf(v, 0.f) : v;
  }
};
struct EpiStore {
  float* out; int ld;
  PTO_DEV void operator()(int m, int n, float v) const { out[m * ld + n] = v; }
};


// y[M,N] = act(x[M,K] @ w[N,K]^T + b): generic fp32 linear (fc1 and the
// nn.Module path).  One 16x16 output tile per block, K split over 4 waves.
__global__ __launch_bounds__(256) void k_linear_fwd(const float* __restrict__ x, const float* __restrict__ w,
                                                    const float* __restrict__ bias, float* __restrict__ y, int M,
                                                    int N, int K, int relu) {
  __shared__ float red[4 * 256];
  block_gemm_splitk4<LAY_ROWK, LAY_ROWK>(x, K, w, K, M, N, K, blockIdx.x, red,
                                          EpiBiasRelu{bias, y, N, relu != 0});
}

// float4 operand loads, 16 waves (1024 threads, 4 waves per SIMD): each wave
// owns a 64-deep K slice (NG = 4 groups, all 8 loads per lane in flight at
// once), so the serial chain per wave is one memory round trip + 16 MFMAs
// (fc1 at B=64: 128 blocks).  Requires K % 4 == 0 and 16-byte aligned x / w
// (checked by the launcher).
// XCD-aware tile order: workgroup i runs on XCD i % 8, so tile index
// (i % 8) * (T / 8) + i / 8 puts T/8 consecutive tiles -- the m-tiles that
// share one weight tile -- on one XCD, and each weight tile is fetched into
// one L2 instead of up to four.  Identity unless T % 8 == 0.
// Split-K partial tiles through LDS: wave w's accumulator element rr of
// lane l (row (l >> 4)*4 + rr, column l & 15) goes to
// red[w*RED_W + rr*RED_RR + l] -- consecutive lanes, consecutive banks on the
// write (a row-major [row][16] slot put a write's four 16-lane groups on the
// same 16 banks), and the RED_RR = 64 + 16 skew puts the reducing threads'
// four rr values on four different 16-bank groups on the read (with 64 they
// all land on one: 4-way conflicts moved from the write to the read).
// red_slot(t) is where the reducing thread t (row t >> 4, column t & 15)
// finds it.
constexpr int RED_RR = 80, RED_W = 4 * RED_RR;
PTO_DEV int red_slot(int t) { return ((t >> 4) & 3) * RED_RR + (t >> 6) * 16 + (t & 15); }

PTO_DEV int xcd_tile(int i, int T, bool on) { return (on && !(T & 7)) ? (i & 7) * (T >> 3) + (i >> 3) : i; }

__global__ __launch_bounds__(1024) void k_linear_fwd_vec16(const float* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ bias, float* __restrict__ y,
                                                           int M, int N, int K, int relu) {
  __shared__ float red[16 * RED_W];
  PTO_STAMP_SCOPE();
  const int mtiles = (M + 15) >> 4;
  const int tile = xcd_tile(blockIdx.x, gridDim.x, true);
  const int mt = tile % mtiles, nt = tile / mtiles;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kc = (((K + 15) / 16) + 15) & ~15;
  const f32x4 acc = wave_tile_16x16<LAY_ROWK, LAY_ROWK, 4, true, true>(x, K, w, K, M, N, K, mt * 16, nt * 16,
                                                                       wv * kc, (wv + 1) * kc);
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) red[wv * RED_W + rr * RED_RR + lane] = acc[rr];
  PTO_STAMP(1);  // wave 0's operands arrived and its MFMAs issued
  __syncthreads();
  PTO_STAMP(2);  // every wave's partial tile in LDS
  const int t = threadIdx.x;
  if (t < 256) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) v += red[q * RED_W + red_slot(t)];
    const int m = mt * 16 + (t >> 4), n = nt * 16 + (t & 15);
    if (m < M && n < N) EpiBiasRelu{bias, y, N, relu != 0}(m, n, v);
  }
}

// fc1 forward WITHOUT bias / ReLU, K split over two workgroups per 16x16
// tile: 2 x 128 workgroups (16 waves of 32-deep K slices by default, one
// memory round trip each) at B = 64 instead of 128 of 16, so every CU holds one tile-half
// and pulls half the operand bytes through its L1 (F3 spent ~3 us of its
// ~4.5 us span getting its 128 KB per CU of operands in:
// profiles/mnist_step_pmc_r6.md).  Both halves are added into h (zero on
// entry: k_bwd_all re-zeroes it) by hardware fp32 atomics -- exactly two
// addends onto +0, so the sum is the same in either arrival order; F4dx,
// the only reader, applies bias + ReLU while staging it and writes h1 out for
// the backward.  XCD-aware: XCD x runs n-tiles 4x..4x+3 (its W1 rows fetched
// into one L2), all m-tiles, both halves.
template <int NW>
__global__ __launch_bounds__(NW * 64) void k_fc1_fwd_split2(const float* __restrict__ x, const float* __restrict__ w,
                                                          float* __restrict__ h, int M) {
  // NW waves per workgroup, each a KW-deep slice of the 400-deep K half in
  // one memory round (KW / 16 k-groups of loads in flight)
  constexpr int KW = ((F1IN / 2 + NW - 1) / NW + 15) / 16 * 16;
  __shared__ float red[NW * RED_W];
  PTO_STAMP_SCOPE();
  const int mtiles = (M + 15) >> 4;
  const int i = blockIdx.x, xcd = i & 7, j = i >> 3;
  const int nt = 4 * xcd + j / (2 * mtiles), mt = (j >> 1) % mtiles, half = j & 1;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int KH = F1IN / 2;
  const int kb = half * KH + wv * KW, ke = min(kb + KW, (half + 1) * KH);
  const f32x4 acc = wave_tile_16x16<LAY_ROWK, LAY_ROWK, KW / 16, true, true>(x, F1IN, w, F1IN, M, F1OUT, F1IN,
                                                                             mt * 16, nt * 16, kb, ke);
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) red[wv * RED_W + rr * RED_RR + lane] = acc[rr];
  PTO_STAMP(1);
  __syncthreads();
  PTO_STAMP(2);
  const int t = threadIdx.x;
  if (t < 256) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) v += red[q * RED_W + red_slot(t)];
    const int m = mt * 16 + (t >> 4), n = nt * 16 + (t & 15);
    if (m < M && n < F1OUT) atomicAdd(h + m * F1OUT + n, v);
  }
}

// dx[M,K] = dy[M,N] @ w[N,K]   (B operand: w as [k=N rows][n=K cols])
__global__ __launch_bounds__(256) void k_linear_bwd_data(const float* __restrict__ dy, const float* __restrict__ w,
                                                         float* __restrict__ dx, int M, int N, int K) {
  __shared__ float red[4 * 256];
  block_gemm_splitk4<LAY_ROWK, LAY_KROW>(dy, N, w, K, M, K, N, blockIdx.x, red, EpiStore{dx, K});
}

// dw[N,K] = dy[M,N]^T @ x[M,K]  (reduction over the batch)
__global__ __launch_bounds__(256) void k_linear_bwd_weight(const float* __restrict__ dy, const float* __restrict__ x,
                                                           float* __restrict__ dw, int M, int N, int K) {
  block_gemm_4tiles<LAY_KROW, LAY_KROW>(dy, N, x, K, N, K, M, blockIdx.x, EpiStore{dw, K});
}

// db[N] = sum_m dy[m, n]
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ dy, float* __restrict__ db, int M, int N) {
  __shared__ float red[256];
  block_colsum64(dy, N, M, N, blockIdx.x * 64, red, db);
}

__global__ __launch_bounds__(256) void k_relu_bwd(const float* __restrict__ g, const float* __restrict__ y,
                                                  float* __restrict__ out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = y[i] > 0.f ? g[i] : 0.f;
}

// ---------------------------------------------------------------- F4 ----
// One wave per row: fc2 (500->10) + log_softmax + NLL + dlogits + dh1
// (= dlogits @ W2, masked by ReLU).  `inv_b` = 1/B for a mean loss.  All 99
// loads of a lane (8 activations, 80 weights, 10 biases, the label) are
// issued before the first FMA.
PTO_DEV void fc2_ce_row(int row, int lane, const float* __restrict__ h1, const float* __restrict__ w,
                        const float* __restrict__ bias, const int64_t* __restrict__ labels,
                        float* __restrict__ logp, float* __restrict__ loss_rows, float* __restrict__ dlogits,
                        float* __restrict__ dh1, int B, float inv_b, const long long* __restrict__ bidx) {
  float h[8], wv[NCLS][8], bz[NCLS];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = lane + 64 * j;
    h[j] = k < F1OUT ? h1[row * F1OUT + k] : 0.f;
#pragma unroll
    for (int c = 0; c < NCLS; ++c) wv[c][j] = k < F1OUT ? w[c * F1OUT + k] : 0.f;
  }
#pragma unroll
  for (int c = 0; c < NCLS; ++c) bz[c] = bias[c];
  int y = 0;
  if (labels) {
    if (bidx) labels += (size_t)(*bidx) * B;
    y = (int)labels[row];
  }
  float z[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s = fmaf(h[j], wv[c][j], s);
    z[c] = s;
  }
  {
    // recursive halving (10 sums padded to 16): 8+4+2+1 shuffles leave lane l
    // with class idx = bits 5..2 of l summed over 16 lanes, two butterflies
    // finish it, and each class is broadcast back with one readlane:
    // 17 shuffles + 10 readlanes instead of 60 shuffles.
    float h8[8], h4[4], h2[2], h1;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool up = lane & 32;
      const float a0 = z[k], a1 = k + 8 < NCLS ? z[k + 8] : 0.f;
      h8[k] = (up ? a1 : a0) + __shfl_xor(up ? a0 : a1, 32, 64);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool up = lane & 16;
      h4[k] = (up ? h8[k + 4] : h8[k]) + __shfl_xor(up ? h8[k] : h8[k + 4], 16, 64);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bool up = lane & 8;
      h2[k] = (up ? h4[k + 2] : h4[k]) + __shfl_xor(up ? h4[k] : h4[k + 2], 8, 64);
    }
    {
      const bool up = lane & 4;
      h1 = (up ? h2[1] : h2[0]) + __shfl_xor(up ? h2[0] : h2[1], 4, 64);
    }
    h1 += __shfl_xor(h1, 2, 64);
    h1 += __shfl_xor(h1, 1, 64);
#pragma unroll
    for (int c = 0; c < NCLS; ++c) {
      const int src = ((c >> 3) & 1) * 32 + ((c >> 2) & 1) * 16 + ((c >> 1) & 1) * 8 + (c & 1) * 4;
      z[c] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h1), src));
    }
  }
#pragma unroll
  for (int c = 0; c < NCLS; ++c) z[c] += bz[c];
  float mx = z[0];
#pragma unroll
  for (int c = 1; c < NCLS; ++c) mx = fmaxf(mx, z[c]);
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < NCLS; ++c) se += __expf(z[c] - mx);
  const float lse = mx + __logf(se);
  float dl[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) dl[c] = (__expf(z[c] - lse) - (c == y ? 1.f : 0.f)) * inv_b;
  if (lane < NCLS) {
    float zl = z[0], dd = dl[0];
#pragma unroll
    for (int c = 1; c < NCLS; ++c)
      if (lane == c) { zl = z[c]; dd = dl[c]; }
    if (logp) logp[row * NCLS + lane] = zl - lse;
    if (dlogits) dlogits[row * NCLS + lane] = dd;
  }
  if (lane == 0 && loss_rows) {
    float zy = z[0];
#pragma unroll
    for (int c = 1; c < NCLS; ++c)
      if (c == y) zy = z[c];
    loss_rows[row] = lse - zy;
  }
  if (!dh1) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = lane + 64 * j;
    if (k < F1OUT) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < NCLS; ++c) s = fmaf(dl[c], wv[c][j], s);
      dh1[row * F1OUT + k] = h[j] > 0.f ? s : 0.f;
    }
  }
}

__global__ __launch_bounds__(256) void k_fc2_ce(const float* __restrict__ h1, const float* __restrict__ w,
                                                const float* __restrict__ bias, const int64_t* __restrict__ labels,
                                                float* __restrict__ logp, float* __restrict__ loss_rows,
                                                float* __restrict__ dlogits, float* __restrict__ dh1, int B,
                                                float inv_b, const long long* __restrict__ bidx) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B) return;
  fc2_ce_row(row, lane, h1, w, bias, labels, logp, loss_rows, dlogits, dh1, B, inv_b, bidx);
}

constexpr int FDX_WAVES = 16;
// dL tile row stride: rows r*20 floats apart put the dh1 phase's float4 A
// reads (16 rows per 16-lane group) on 16 distinct 4-bank groups (16: 4-way)
constexpr int DLS_LD = 20;

// F4dx: F4 + d(a2p) in one launch.  Block (mt, nt) = 16 waves: the fc2 +
// log_softmax + NLL + dlogits + dh1 head of its 16 rows (recomputed per
// column tile -- ~1 us of dependent latency either way -- so the F4 -> B3
// launch boundary disappears; the nt == 0 blocks store loss/dlogits/dh1),
// then the d(a2p) tile [16 rows, 16 cols] = dh1 W1 split-K over the waves.
// The head runs on the matrix cores (a per-wave VALU head read all of W2
// with 80 scalar loads per lane, ~1600 VMEM instructions per block,
// profiles/fdx_mfma_head_r2.md): the block stages its 16 h1 rows and W2 into
// LDS with one round of float4 loads and runs two tiny GEMMs:
//   Z[16 x 16]   = h1_tile[16 x 500] W2^T   (split-K over the 16 waves)
//   dh1[16 x 500] = dL[16 x 16] W2[16 x 500] (2 column tiles per wave, K=16)
// with the softmax between them done by 256 threads, 16 lanes per row.
// dh1 overwrites the h1 tile in place (each element is read for its ReLU
// mask and written by the same lane), then the d(a2p) tile is as before.
// Requires 16-byte aligned h1 and W2 (checked by the launcher).
// The NEXT step's images, staged by F4dx's last STAGE_BLOCKS workgroups
// into a buffer at a fixed address (xnext), which the next F12 reads with no
// batch cursor: F12 had to load the cursor (written by the previous
// backward) before it could even address its images -- two dependent
// memory round trips at the head of the step.  With F12 reading a fixed
// address the step measured 34.91-34.98 vs 35.96-36.00 us
// (profiles/mnist_step_pmc_r6.md); a plain prefetch of the next batch into
// the caches did not help, the dependent cursor load was the cost.  The
// copy takes batch (cursor + 1) % nb: every schedule advances the cursor
// after F4dx (k_bwd_all, k_ddp_sgd or the exchange epilogue).
struct BatchStage {
  const float* x;  // [nb][n4 * 4] images (nullptr: no staging)
  float* xnext;    // [n4 * 4]
  long long nb;
  int n4;
};
constexpr int STAGE_BLOCKS = 4;

__global__ __launch_bounds__(FDX_WAVES * 64) void k_fc2_ce_dx_mf(
    const float* __restrict__ h1, const float* __restrict__ w2, const float* __restrict__ b2,
    const int64_t* __restrict__ labels, const float* __restrict__ w1, float* __restrict__ loss_rows,
    float* __restrict__ dlogits, float* __restrict__ dh1, float* __restrict__ da2p, int B, float inv_b,
    const long long* __restrict__ bidx, Conv1Commit cm, BatchStage st, const float* __restrict__ b1,
    float* __restrict__ h1out) {
  // LDS row stride.  500 keeps the dh1 phase's scalar accesses (rows r and
  // r + 4 in one 32-lane group, 4*500 = 16 mod 32 banks apart) conflict-free;
  // 504 would make the float4 operand reads conflict-free instead but the
  // dh1 phase 2-way (measured: more conflict cycles, same time)
  constexpr int HLD = F1OUT;
  __shared__ __attribute__((aligned(16))) float hs[16 * HLD];
  __shared__ __attribute__((aligned(16))) float w2s[NCLS * HLD];
  __shared__ float red[FDX_WAVES * RED_W];
  __shared__ __attribute__((aligned(16))) float dls[16 * DLS_LD];
  const int mtiles = (B + 15) >> 4, ntiles = (F1IN + 15) >> 4;
  const int t = threadIdx.x;
  PTO_STAMP_SCOPE();
  if (blockIdx.x > (unsigned)(mtiles * ntiles)) {  // next-batch staging (launcher: st.xnext && bidx)
    const long long nb = (*bidx + 1) % st.nb;
    const float4* src = reinterpret_cast<const float4*>(st.x) + nb * st.n4;
    float4* dst = reinterpret_cast<float4*>(st.xnext);
    const int j0 = (blockIdx.x - mtiles * ntiles - 1) * (FDX_WAVES * 64) + t;
    constexpr int STRIDE = STAGE_BLOCKS * FDX_WAVES * 64;  // 4 x 4096 float4 >= B = 64's 12,544
    // four named float4s, not an array: with `float4 v[4]` and the guarded
    // stores the compiler kept v in scratch, which gave the whole kernel a
    // private segment (80 bytes per lane)
    for (int i0 = j0; i0 < st.n4; i0 += 4 * STRIDE) {
      const int i1 = i0 + STRIDE, i2 = i0 + 2 * STRIDE, i3 = i0 + 3 * STRIDE;
      const float4 v0 = src[i0];
      const float4 v1 = src[i1 < st.n4 ? i1 : i0];
      const float4 v2 = src[i2 < st.n4 ? i2 : i0];
      const float4 v3 = src[i3 < st.n4 ? i3 : i0];
      dst[i0] = v0;
      if (i1 < st.n4) dst[i1] = v1;
      if (i2 < st.n4) dst[i2] = v2;
      if (i3 < st.n4) dst[i3] = v3;
    }
    return;
  }
  if (blockIdx.x == (unsigned)(mtiles * ntiles)) {
    if (cm.zero_word && t == 0) *cm.zero_word = 0;  // every waiter of the previous launch has finished
    if (cm.pending) {
      const int pend = *cm.pending;
      const float lr = *cm.a.lr;  // in flight with the flag
      if (pend)
        for (int i = 4 * t; i < cm.n; i += 4 * FDX_WAVES * 64) commit4(cm, i, lr);
    }
    return;
  }
  const int tile = xcd_tile(blockIdx.x, mtiles * ntiles, true);
  const int mt = tile % mtiles, nt = tile / mtiles;
  const int w = t >> 6, lane = t & 63;
  const int r = lane & 15, gq = lane >> 4;
  constexpr int KC = ((F1OUT + FDX_WAVES - 1) / FDX_WAVES + 15) & ~15;  // 32
  constexpr int NGK = KC / 16;
  constexpr int H4 = 16 * F1OUT / 4, W4 = NCLS * F1OUT / 4;  // 2000, 1250 float4
  constexpr int NT = FDX_WAVES * 64;
  static_assert(F1OUT % 4 == 0 && H4 <= 2 * NT && W4 <= 2 * NT, "staging assumes two float4 rounds");
  const int kb = w * KC, kend = min((w + 1) * KC, F1OUT);
  // ---- one round of loads: h1 tile + W2 (float4), W1 slice, label, bias
  const int nrow = min(16, B - mt * 16);
  const float4* hg = reinterpret_cast<const float4*>(h1 + (size_t)mt * 16 * F1OUT);
  const float4* wg = reinterpret_cast<const float4*>(w2);
  // a zero RVALUE: with an lvalue zero, `ok ? *p : z4` is an lvalue
  // conditional, which the compiler lowers to a flat load from a select
  // between p and a scratch copy of the zero
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const int h4n = nrow * (F1OUT / 4);
  float4 hv0 = t < h4n ? hg[t] : float4(z4);
  float4 hv1 = (t + NT < H4 && t + NT < h4n) ? hg[t + NT] : float4(z4);
  // split fc1 (b1 != nullptr): h1 holds the raw split-K sum; relu(h + b1)
  // is formed here, the bias loaded in the same round
  float4 bb0 = z4, bb1 = z4;
  if (b1) {
    const float4* b4 = reinterpret_cast<const float4*>(b1);
    constexpr int RB = F1OUT / 4;
    bb0 = b4[t % RB];
    bb1 = b4[(t + NT) % RB];
  }
  const float4 wv0 = t < W4 ? wg[t] : float4(z4);
  const float4 wv1 = t + NT < W4 ? wg[t + NT] : float4(z4);
  float bw[NGK][4];
#pragma unroll
  for (int q = 0; q < NGK; ++q) load4<LAY_KROW>(w1, F1IN, nt * 16 + r, F1IN, kb + 16 * q + 4 * gq, kend, bw[q]);
  const int hm = t >> 4, hn = t & 15;  // softmax thread -> (row, class), t < 256
  const int grow = mt * 16 + hm;
  int y = 0;
  float bias = 0.f;
  if (t < 256) {
    if (grow < B && labels) y = (int)labels[(bidx ? (size_t)(*bidx) * B : 0) + grow];
    if (hn < NCLS) bias = b2[hn];
  }
  if (b1) {
    auto act = [](float4 a, float4 c) {
      return make_float4(fmaxf(a.x + c.x, 0.f), fmaxf(a.y + c.y, 0.f), fmaxf(a.z + c.z, 0.f), fmaxf(a.w + c.w, 0.f));
    };
    hv0 = t < h4n ? act(hv0, bb0) : float4(z4);
    hv1 = (t + NT < H4 && t + NT < h4n) ? act(hv1, bb1) : float4(z4);
    if (nt == 0) {  // h1 for the backward's fc2 weight gradient, one writer per row
      float4* ho = reinterpret_cast<float4*>(h1out + (size_t)mt * 16 * F1OUT);
      if (t < h4n) ho[t] = hv0;
      if (t + NT < H4 && t + NT < h4n) ho[t + NT] = hv1;
    }
  }
  float4* hs4 = reinterpret_cast<float4*>(hs);
  float4* ws4 = reinterpret_cast<float4*>(w2s);
  constexpr int R4 = F1OUT / 4;  // float4 per row
  auto pad4 = [](int e) { return (e / R4) * (HLD / 4) + e % R4; };
  hs4[pad4(t)] = hv0;
  if (t + NT < H4) hs4[pad4(t + NT)] = hv1;
  if (t < W4) ws4[pad4(t)] = wv0;
  if (t + NT < W4) ws4[pad4(t + NT)] = wv1;
  __syncthreads();
  PTO_STAMP(1);
  // ---- Z partial: rows r of the tile x classes r (<10), K slice of wave w
  {
    f32x4 acc0 = zero4(), acc1 = zero4();
#pragma unroll
    for (int q = 0; q < NGK; ++q) {
      // branch-free: reads clamped into the staged rows, the A value of a
      // k past the end zeroed after the read (class rows >= 10 only feed
      // unused output columns)
      const int k0 = kb + 16 * q + 4 * gq, kc = min(k0, F1OUT - 4);
      const float4 at = *reinterpret_cast<const float4*>(hs + r * HLD + kc);
      const float4 a = k0 < F1OUT ? at : float4(z4);
      const float4 b = *reinterpret_cast<const float4*>(w2s + min(r, NCLS - 1) * HLD + kc);
      acc0 = mfma16x16x4(a.x, b.x, acc0);
      acc1 = mfma16x16x4(a.y, b.y, acc1);
      acc0 = mfma16x16x4(a.z, b.z, acc0);
      acc1 = mfma16x16x4(a.w, b.w, acc1);
    }
    const f32x4 acc = acc0 + acc1;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) red[w * RED_W + rr * RED_RR + lane] = acc[rr];
  }
  __syncthreads();
  PTO_STAMP(2);
  // ---- log_softmax + NLL + dlogits: 16 lanes per row (waves 0..3)
  if (t < 256) {
    float z = bias;
#pragma unroll
    for (int q = 0; q < FDX_WAVES; ++q) z += red[q * RED_W + red_slot(t)];
    const bool cls = hn < NCLS;
    float mx = cls ? z : -INFINITY;
    mx = row16_max(mx);
    float se = cls ? __expf(z - mx) : 0.f;
    se = row16_sum(se);
    const float lse = mx + __logf(se);
    const bool live = grow < B;
    const float dl = (cls && live) ? (__expf(z - lse) - (hn == y ? 1.f : 0.f)) * inv_b : 0.f;
    dls[hm * DLS_LD + hn] = dl;
    const float zy = __shfl(z, (lane & 48) | (y & 15), 64);
    if (nt == 0 && live) {
      if (cls) dlogits[grow * NCLS + hn] = dl;
      if (hn == 0) loss_rows[grow] = lse - zy;
    }
  }
  __syncthreads();
  PTO_STAMP(3);
  // ---- dh1 = (dL W2) * [h1 > 0], column tiles 2w and 2w + 1, in place:
  // exactly the K slice [KC*w, KC*w + 32) this wave reads in the d(a2p)
  // phase (and read in the Z phase), so no block barrier between the two --
  // the wave's own LDS stores precede its reads.
  // Branch-free operand reads (classes >= 10 have dL = 0 exactly, so their
  // W2 row is clamped to a valid one; columns >= 500 read column 499 and are
  // not written), all issued before the two interleaved 4-MFMA chains
  {
    const float4 a = *reinterpret_cast<const float4*>(dls + r * DLS_LD + 4 * gq);
    float bb[2][4], hv[2][4];
    bool cok[2];
    int cc[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int col = (2 * w + hh) * 16 + r;
      cok[hh] = col < F1OUT;
      cc[hh] = cok[hh] ? col : F1OUT - 1;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // classes 10..15 read rows 2..7 (the rows lane group gq - 2 reads for
        // the same j: same address, a broadcast) rather than all row 9,
        // whose banks overlap rows 0, 2, 3 and 6
        const int c = 4 * gq + j;
        bb[hh][j] = w2s[(c < NCLS ? c : c - 8) * HLD + cc[hh]];
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) hv[hh][rr] = hs[(gq * 4 + rr) * HLD + cc[hh]];
    }
    f32x4 acc[2] = {zero4(), zero4()};
    const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) acc[hh] = mfma16x16x4(av[j], bb[hh][j], acc[hh]);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      if (!cok[hh]) continue;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = gq * 4 + rr;
        const float v = hv[hh][rr] > 0.f ? acc[hh][rr] : 0.f;
        hs[row * HLD + cc[hh]] = v;
        if (nt == 0 && mt * 16 + row < B) dh1[(mt * 16 + row) * F1OUT + cc[hh]] = v;
      }
    }
  }
  static_assert(KC == 32 && 2 * 16 * FDX_WAVES >= F1OUT, "wave w's dh1 tiles are its d(a2p) K slice");
  PTO_STAMP(4);
  // ---- d(a2p) tile [16 rows, 16 cols] = dh1 W1, split-K over the waves
  {
    f32x4 acc0 = zero4(), acc1 = zero4();
#pragma unroll
    for (int q = 0; q < NGK; ++q) {
      // unconditional float4 read: a k past the row's end is clamped into
      // the row (finite values that meet bw = 0 there)
      const float4 av = *reinterpret_cast<const float4*>(hs + r * HLD + min(kb + 16 * q + 4 * gq, F1OUT - 4));
      acc0 = mfma16x16x4(av.x, bw[q][0], acc0);
      acc1 = mfma16x16x4(av.y, bw[q][1], acc1);
      acc0 = mfma16x16x4(av.z, bw[q][2], acc0);
      acc1 = mfma16x16x4(av.w, bw[q][3], acc1);
    }
    const f32x4 acc = acc0 + acc1;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) red[w * RED_W + rr * RED_RR + lane] = acc[rr];
  }
  __syncthreads();
  PTO_STAMP(5);
  if (t < 256) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < FDX_WAVES; ++q) v += red[q * RED_W + red_slot(t)];
    const int m = mt * 16 + (t >> 4), n = nt * 16 + (t & 15);
    if (m < B && n < F1IN) da2p[m * F1IN + n] = v;
  }
}

// ---------------------------------------------------------------- B2 ----
// conv2 backward.  g = d(a2p) [B,800] (pooled grad), code2 = argmax codes.
//  part A: dW2[oc][ic,kh,kw] += sum_{b,pos} dY2 * a1p-patch  (split-K over
//          sample chunks, fp32 atomics; tile = 16 oc x 16 (ic,kh,kw)).
//          K order: lane group g = pooled pixel 4G+g, MFMA j = window pos j,
//          so the (grad, code) expansion is one load pair per 4 MFMAs.
//          Loads for 4 samples (96 per lane) are in flight at once.
//  part B: d(a1p) via col2im.  Block = (sample, 5-input-channel group):
//          T[pos][ic,kh,kw] = sum_oc dY2[oc][pos] W2[oc][ic,kh,kw] (MFMA,
//          64 x 125 x 52) into LDS, then each output pixel gathers <=25 T
//          entries.  Deterministic, no atomics, 3.4x fewer MFMAs than the
//          dense full-convolution GEMM.
//  part C: db2[oc] = sum of unmasked pooled grads (one wave per channel).
constexpr int B2_CHUNK = 7;  // samples per weight-grad block (7: LDS <= 40 KB -> 4 blocks/CU, all parts co-resident)
constexpr int B2_ICG = 10;   // input-channel pairs per sample in the dgrad part
// LDS of a dgrad block: R1 = T [64][65] (first the W2 slice [50][68]) +
// R2 = dY2^T [50][68] (c2_dgrad_block)
constexpr int B2_DLD = 68;  // dY^T row stride (64 positions + 4): conflict-free writes and GEMM reads
constexpr int B2_LDS_FLOATS = 64 * 65 + C2 * B2_DLD;

// Recursive-halving wave reduction of 26 (padded to 32) per-lane sums: at
// each step a lane keeps half of its live accumulators (chosen by its lane
// bit) and receives its partner's copy of them: 16+8+4+2+1+1 = 32 exchanges
// instead of 6 x 26.  Bits 5 and 4 by v_permlane32/16_swap (which move
// exactly the halves each side keeps), bits 3..0 by DPP (bit 2's partner is
// lane ^ 7, see lane_mirror8) -- no LDS-crossbar round trips.  The 26 wave
// totals are written to out[0..25].
PTO_DEV void wave_halving26(const float acc[26], int lane, float* out) {
  float h16[16], h8[8], h4[4], h2[2], h1;
#pragma unroll
  for (int k = 0; k < 16; ++k) h16[k] = halve32(acc[k], k + 16 < 26 ? acc[k + 16] : 0.f);
#pragma unroll
  for (int k = 0; k < 8; ++k) h8[k] = halve16(h16[k], h16[k + 8]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool up = lane & 8;
    h4[k] = (up ? h8[k + 4] : h8[k]) + lane_xor8(up ? h8[k] : h8[k + 4]);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const bool up = lane & 4;
    h2[k] = (up ? h4[k + 2] : h4[k]) + lane_mirror8(up ? h4[k] : h4[k + 2]);
  }
  {
    const bool up = lane & 2;
    h1 = (up ? h2[1] : h2[0]) + lane_xor2(up ? h2[0] : h2[1]);
  }
  h1 += lane_xor1(h1);
  const int idx = ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 + ((lane >> 2) & 1) * 2 +
                  ((lane >> 1) & 1);
  if (!(lane & 1) && idx < 26) out[idx] = h1;
}

// conv2 weight-gradient block (part A of the conv2 backward): NTW 16-column
// K-tiles x all 64 (padded) output channels x a chunk of CH samples, fp32
// atomics into gw2 (or, deterministic mode, the chunk's partial tile).
// ONE staging round: the block's 16*NTW (ic,kh,kw) columns touch at most
// NCH input channels, so for every sample of the chunk it stages NCH x 144
// pooled conv1 values + the 800 pooled grads + 800 codes with coalesced
// 16-byte loads, then runs its MFMAs from LDS.  NTW = 2 shares that staging
// (and every A-operand read) between two column tiles.
// Staged a1p planes of the wgrad blocks: 12 rows at stride WG_RS, channel
// planes WG_PS apart (dwords).  The MFMA loop's patch reads are ds_read2_b32
// (banks = dword mod 32 per 32-lane half): with the dense 12 / 144 layout
// the lanes' (tap, pooled column) addresses wrapped onto each other (+4
// conflict cycles per read2, ~2e5 per launch); 20 / 260 is the layout
// tools/lds_bank_model.py finds conflict-free for all 32 column tiles.
constexpr int WG_RS = 20, WG_PS = 260;
static_assert(WG_RS % 4 == 0 && WG_PS % 4 == 0 && WG_PS >= 12 * WG_RS, "float4-staged planes");
template <int NTW>
constexpr int wgrad_nch() { return NTW == 1 ? 2 : 3; }  // 16 cols span <= 2 channels, 32 cols <= 3
template <int CH, int NTW>
constexpr int wgrad_lds_floats() { return CH * (wgrad_nch<NTW>() * WG_PS + F1IN + F1IN / 4); }
template <int CH, int NTW = 1>
PTO_DEV void c2_wgrad_block(int bid, float* smem, const float* __restrict__ g2, const uint8_t* __restrict__ code2,
                            const float* __restrict__ a1p, float* __restrict__ gw2, int B,
                            float* __restrict__ part = nullptr) {
  constexpr int NT = 32 / NTW;           // column tiles of one sample chunk
  constexpr int NCH = wgrad_nch<NTW>();  // input channels staged per sample
  static_assert(32 % NTW == 0, "500 columns = 32 tiles of 16");
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nt = bid % NT, chunk = bid / NT;
  const int col0 = nt * 16 * NTW;
  const int oc = wv * 16 + (lane & 15);
  const int g = lane >> 4;
  const int ic0 = col0 / 25;
  int koff[NTW];
  bool kvalid[NTW];
#pragma unroll
  for (int u = 0; u < NTW; ++u) {
    const int kk = col0 + 16 * u + (lane & 15);
    kvalid[u] = kk < 500;
    const int ic = kvalid[u] ? kk / 25 : ic0, r25 = kvalid[u] ? kk - ic * 25 : 0;
    const int kh = r25 / 5, kw = r25 - kh * 5;
    koff[u] = (ic - ic0) * WG_PS + kh * WG_RS + kw;
  }
  const bool ocvalid = oc < C2;
  const int b0 = chunk * CH, nb = min(B, b0 + CH) - b0;
  float* as = smem;                                           // [CH][NCH][12 x WG_RS, WG_PS]
  float* gs = smem + CH * NCH * WG_PS;                        // [CH][800]
  uint8_t* cs = reinterpret_cast<uint8_t*>(gs + CH * F1IN);  // [CH][800] bytes
  const int tid = threadIdx.x;
  {
    constexpr int A4 = NCH * 36;  // float4 per sample
    constexpr int NVA = (CH * A4 + 255) / 256, NVG = (CH * (F1IN / 4) + 255) / 256;
    float4 va[NVA], vg[NVG];
    uint32_t vc[NVG];
#pragma unroll
    for (int q = 0; q < NVA; ++q) {
      const int e = tid + 256 * q;  // float4 index over [s][ch][36]
      const int smp = e / A4, rr = e - smp * A4, ch = rr / 36, off = (rr - ch * 36) * 4;
      const bool ok = e < nb * A4 && ic0 + ch < C1;
      va[q] = ok ? *reinterpret_cast<const float4*>(a1p + (b0 + smp) * A1P + (ic0 + ch) * 144 + off)
                 : float4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < NVG; ++q) {
      const int e = tid + 256 * q;
      const bool ok = e < nb * (F1IN / 4);
      vg[q] = ok ? reinterpret_cast<const float4*>(g2 + b0 * F1IN)[e] : float4{0.f, 0.f, 0.f, 0.f};
      vc[q] = ok ? reinterpret_cast<const uint32_t*>(code2 + b0 * F1IN)[e] : 0x04040404u;
    }
#pragma unroll
    for (int q = 0; q < NVA; ++q) {
      const int e = tid + 256 * q;
      if (e < CH * A4) {
        const int sc = e / 36, f4 = e - sc * 36, row = f4 / 3;  // (sample, channel) plane, row of 3 float4
        *reinterpret_cast<float4*>(as + sc * WG_PS + row * WG_RS + 4 * (f4 - row * 3)) = va[q];
      }
    }
#pragma unroll
    for (int q = 0; q < NVG; ++q) {
      const int e = tid + 256 * q;
      if (e < CH * (F1IN / 4)) {
        // Transposed + swizzled: the loaded quad holds pooled pixels (G, g =
        // 0..3) of channel oc; slot (oc, g) holds the 4 G values of pooled
        // column g contiguously (one ds_read_b128 / one ds_read_b32 per
        // sample in the MFMA loop instead of 4 + 4), at quad g ^ ((oc >> 2) &
        // 3) of the channel's 16 floats: the 16 channels of a b128 read
        // group then cover all 64 banks once, and the 64 code dwords too
        const int smp = e / (F1IN / 4), r = e - smp * (F1IN / 4), oc_ = r >> 2, G = r & 3;
        const int sw = (oc_ >> 2) & 3;
        const float vv[4] = {vg[q].x, vg[q].y, vg[q].z, vg[q].w};
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const int o = smp * F1IN + oc_ * 16 + 4 * (gg ^ sw) + G;
          gs[o] = vv[gg];
          cs[o] = (uint8_t)(vc[q] >> (8 * gg));
        }
      }
    }
  }
  __syncthreads();
  PTO_STAMP(1);
  // K order: lane group g = pooled pixel 4G+g, MFMA j = window position j,
  // so one (grad, code) expansion feeds 4 MFMAs per column tile.
  // Branch-free operand reads over all CH staged samples (the slots of
  // samples past nb were staged as zero grads with code 4); columns
  // kk >= 500 read column offset 0 -- finite values whose output columns are
  // never stored -- so every read of a sample can be issued before its
  // MFMAs (exec-masked reads compiled to one LDS round trip per pixel
  // group).  Waves 0-2 run rows 0..47 on the matrix cores; wave 3 runs rows
  // 48, 49 on the VALU.
  if (wv == C2 / 16) {
    // rows 48..49 (the only valid rows of the 4th 16-row tile) on the VALU:
    // lane = column c (16) x row 48 + rr (2) x sample half h (2); per
    // (sample, pooled pixel) one (grad, code) pair and the one patch value
    // its code selects -- a quarter of the FLOPs of the zero-padded MFMA
    // tile, and no MFMA issue on this wave's SIMD
    static_assert(C2 % 16 == 2, "VALU tail covers exactly 2 rows");
    const int c = lane & 15, rr = (lane >> 4) & 1, h = lane >> 5;
    const int ocx = C2 - 2 + rr;
    const int xsw = (ocx >> 2) & 3;
    float sum[NTW];
#pragma unroll
    for (int u = 0; u < NTW; ++u) sum[u] = 0.f;
#pragma unroll
    for (int i = 0; i < (CH + 1) / 2; ++i) {
      const int smp = 2 * i + h;
      if (smp >= CH) break;
#pragma unroll
      for (int pp = 0; pp < 16; ++pp) {
        const int G = pp >> 2, gq = pp & 3;
        const int o = smp * F1IN + ocx * 16 + 4 * (gq ^ xsw) + G;
        const float gv = gs[o];
        const int cd = cs[o];
        const int po = (cd >> 1) * WG_RS + (cd & 1);  // window position of the code (cd 4: masked)
#pragma unroll
        for (int u = 0; u < NTW; ++u) {
          const float* ap = as + smp * (NCH * WG_PS) + koff[u] + 2 * WG_RS * G + 2 * gq;
          const float bvx = ap[cd < 4 ? po : 0];
          sum[u] = fmaf(cd < 4 ? gv : 0.f, bvx, sum[u]);
        }
      }
    }
    PTO_STAMP(2);
#pragma unroll
    for (int u = 0; u < NTW; ++u) {
      const float v = lane_sum32(sum[u]);
      const int n = col0 + 16 * u + c;
      if (h == 0 && n < 500) {
        if (part)
          part[chunk * (C2 * 500) + ocx * 500 + n] = v;
        else
          atomicAdd(gw2 + ocx * 500 + n, v);
      }
    }
    return;
  }
  f32x4 acc0[NTW], acc1[NTW];
#pragma unroll
  for (int u = 0; u < NTW; ++u) acc0[u] = acc1[u] = zero4();
  const int goff = oc * 16 + 4 * (g ^ ((oc >> 2) & 3));
#pragma unroll
  for (int smp = 0; smp < CH; ++smp) {
    float gv[4], bv[NTW][4][4];
    int cd[4];
    const float4 g4 = *reinterpret_cast<const float4*>(gs + smp * F1IN + goff);
    const uint32_t c4 = *reinterpret_cast<const uint32_t*>(cs + smp * F1IN + goff);
    gv[0] = g4.x; gv[1] = g4.y; gv[2] = g4.z; gv[3] = g4.w;
#pragma unroll
    for (int G = 0; G < 4; ++G) {
      cd[G] = (c4 >> (8 * G)) & 0xff;
#pragma unroll
      for (int u = 0; u < NTW; ++u) {
        const float* ap = as + smp * (NCH * WG_PS) + koff[u] + 2 * WG_RS * G + 2 * g;
        bv[u][G][0] = ap[0];
        bv[u][G][1] = ap[1];
        bv[u][G][2] = ap[WG_RS];
        bv[u][G][3] = ap[WG_RS + 1];
      }
    }
#pragma unroll
    for (int G = 0; G < 4; ++G) {
      const float a0 = cd[G] == 0 ? gv[G] : 0.f, a1 = cd[G] == 1 ? gv[G] : 0.f;
      const float a2 = cd[G] == 2 ? gv[G] : 0.f, a3 = cd[G] == 3 ? gv[G] : 0.f;
#pragma unroll
      for (int u = 0; u < NTW; ++u) {
        acc0[u] = mfma16x16x4(a0, bv[u][G][0], acc0[u]);
        acc1[u] = mfma16x16x4(a1, bv[u][G][1], acc1[u]);
        acc0[u] = mfma16x16x4(a2, bv[u][G][2], acc0[u]);
        acc1[u] = mfma16x16x4(a3, bv[u][G][3], acc1[u]);
      }
    }
  }
  PTO_STAMP(2);
#pragma unroll
  for (int u = 0; u < NTW; ++u) {
    const f32x4 acc = acc0[u] + acc1[u];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = wv * 16 + (lane >> 4) * 4 + rr;
      const int n = col0 + 16 * u + (lane & 15);
      if (n < 500) {
        if (part)  // deterministic mode: this chunk's partial tile, summed in chunk order by the last arriver
          part[chunk * (C2 * 500) + m * 500 + n] = acc[rr];
        else
          atomicAdd(gw2 + m * 500 + n, acc[rr]);
      }
    }
  }
}

// conv2 data-gradient block (part B): (sample, input-channel pair) ->
// d(a1p) by col2im (stored when da1p != nullptr) and, with gw1 != nullptr,
// conv1's weight/bias gradient of those two channels (fp32 atomics).
PTO_DEV void c2_dgrad_block(int bid, float* smem, const float* __restrict__ g2, const uint8_t* __restrict__ code2,
                            const float* __restrict__ w2, float* __restrict__ da1p, int B, const float* __restrict__ x,
                            const long long* __restrict__ bidx, const uint8_t* __restrict__ code1,
                            float* __restrict__ gw1, float* __restrict__ gb1, bool det) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // ---- part B: data gradient via col2im.  Block = (sample, pair of input
  // channels): 640 blocks at B=64, so each block's serial chain (one
  // staging round -> dY2 expansion -> 64x64x52 GEMM -> col2im) is short.
  // Staged: the W2 slice of the two channels (50 x 50, coalesced) + the
  // sample's pooled grads and codes.
  const int b = bid / B2_ICG, icg = bid - b * B2_ICG;
  constexpr int WLD = 68;   // 64 + 4: the 4 k-rows of a wave hit disjoint banks
  // T is kept transposed, T^T [col][pos] at row stride 68: the GEMM's
  // accumulator rows (4 column rows per lane group, 4*68 = 16 mod 64 banks
  // apart) store conflict-free, and col2im's reads of one tap column at 64
  // distinct positions are one contiguous row.  ([pos][col] at stride 65
  // stored with 4-way conflicts: 4 position rows 4 banks apart.)
  constexpr int TLD = 68;
  // Two LDS regions, each reused once the phase that reads it is over
  // (30 KB in all):
  //   R1: W2 slice [50][68]                     -> after the GEMM: T^T [50][68]
  //       -> after col2im: the conv1 wave partials
  //   R2: expanded dY2^T [50][68]               -> after the GEMM: input
  //       image [784] + conv1 codes [2][144] (held in registers until then)
  //       + d(a1p) of the two channels [288]
  // The W2 slice's pad columns 50..63 are never written: they only feed T
  // columns col2im does not read; the K rows past 50 are masked at the read.
  constexpr int R1 = 64 * 65;
  static_assert(50 * WLD <= R1 && 50 * TLD <= R1, "W2 slice and T^T fit R1");
  float* ws = smem;                      // R1
  float* ts = smem;                      // R1 after the GEMM
  float* dys = smem + R1;                // R2
  float* xs = dys;                       // R2 after the GEMM
  uint8_t* c1s = reinterpret_cast<uint8_t*>(xs + 784);
  float* dsum = xs + 784 + 72;
  const bool fuse1 = gw1 != nullptr;
  const int r = lane & 15, gg = lane >> 4;
  const int tid = threadIdx.x;
  float4 xv = float4{0.f, 0.f, 0.f, 0.f};
  uint32_t c1v = 0;
  if (fuse1) {  // issued with the other loads, stored to LDS after the GEMM
    const float* xb = batch_ptr(x, bidx, B * 784) + b * 784;
    if (tid < 196) xv = reinterpret_cast<const float4*>(xb)[tid];
    if (tid < 72) c1v = reinterpret_cast<const uint32_t*>(code1 + (b * C1 + icg * 2) * 144)[tid];
  }
  {
    // the W2 slice as float2 (rows of 50 floats at a 2000-B stride, slice
    // start 200*icg B: 8-byte aligned; launchers check w2)
    constexpr int NW = (C2 * 25 + 255) / 256;  // 5
    float2 wv_[NW];
    const float2* wb = reinterpret_cast<const float2*>(w2 + icg * 50);
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const int e = tid + 256 * q, k = e / 25, n2 = e - k * 25;
      wv_[q] = e < C2 * 25 ? wb[k * 250 + n2] : float2{0.f, 0.f};
    }
    float4 gv4 = float4{0.f, 0.f, 0.f, 0.f};
    uint32_t cv = 0;
    if (tid < F1IN / 4) {
      gv4 = reinterpret_cast<const float4*>(g2 + b * F1IN)[tid];
      cv = reinterpret_cast<const uint32_t*>(code2 + b * F1IN)[tid];
    }
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const int e = tid + 256 * q, k = e / 25, n2 = e - k * 25;
      if (e < C2 * 25) *reinterpret_cast<float2*>(ws + k * WLD + 2 * n2) = wv_[q];
    }
    // dY^T [oc][pos] expanded straight from the registers: thread t < 200
    // holds pooled row ph = t & 3 of channel oc = t >> 2 (4 grads + 4 codes)
    // and writes conv2-output rows 2ph and 2ph+1 (16 positions, 4 float4)
    if (tid < F1IN / 4) {
      const int oc = tid >> 2, ph = tid & 3;
      const float gq[4] = {gv4.x, gv4.y, gv4.z, gv4.w};
      float e[2][8];
#pragma unroll
      for (int pw = 0; pw < 4; ++pw) {
        const int cd = (cv >> (8 * pw)) & 0xff;
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
          for (int dx = 0; dx < 2; ++dx) e[dy][2 * pw + dx] = cd == dy * 2 + dx ? gq[pw] : 0.f;
      }
      float4* row = reinterpret_cast<float4*>(dys + oc * B2_DLD + 16 * ph);
      row[0] = float4{e[0][0], e[0][1], e[0][2], e[0][3]};
      row[1] = float4{e[0][4], e[0][5], e[0][6], e[0][7]};
      row[2] = float4{e[1][0], e[1][1], e[1][2], e[1][3]};
      row[3] = float4{e[1][4], e[1][5], e[1][6], e[1][7]};
    }
  }
  __syncthreads();
  PTO_STAMP(1);
  {
    // T^T = W2slice^T dY^T: rows = T columns, columns = positions.
    // T columns 0..47 on the matrix cores (3 row tiles); the 2 valid
    // columns of the 4th tile (48, 49) on the VALU: lane = position (16) x
    // column (2) x K half (2), 25 FMAs, one shuffle -- a 13-MFMA tile that
    // was 7/8 padding
    static_assert(2 * 25 - 48 == 2, "VALU tail covers T columns 48, 49");
    constexpr int NQ = 3;
    f32x4 acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = zero4();
#pragma unroll
    for (int k0 = 0; k0 < 4; ++k0) {
      if (k0 == 3) {
        // K tail (k = 48..51): one k per lane group, so 4 MFMAs instead of
        // 16 with three quarters of their K padding (profiles/conv2_ktail_ab_r1.md)
        const int k = 48 + gg;
        const float a = k < C2 ? dys[k * B2_DLD + wv * 16 + r] : 0.f;
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[q] = mfma16x16x4(k < C2 ? ws[k * WLD + q * 16 + r] : 0.f, a, acc[q]);
        break;
      }
      float av[4], bv[NQ][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = 16 * k0 + 4 * gg + j;
        av[j] = dys[k * B2_DLD + wv * 16 + r];
#pragma unroll
        for (int q = 0; q < NQ; ++q) bv[q][j] = ws[k * WLD + q * 16 + r];
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[q] = mfma16x16x4(bv[q][j], av[j], acc[q]);
    }
    float tail;
    {
      const int pos = wv * 16 + r, cc = 48 + (gg & 1), k0 = (gg >> 1) * 25;
      float tv = 0.f;
#pragma unroll
      for (int k = 0; k < 25; ++k) tv = fmaf(dys[(k0 + k) * B2_DLD + pos], ws[(k0 + k) * WLD + cc], tv);
      tail = lane_sum32(tv);
    }
    __syncthreads();  // ts aliases ws, xs aliases dys: every wave's GEMM reads are done
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        ts[(q * 16 + gg * 4 + rr) * TLD + wv * 16 + r] = acc[q][rr];
    if (gg < 2) ts[(48 + gg) * TLD + wv * 16 + r] = tail;
    if (fuse1) {
      if (tid < 196) reinterpret_cast<float4*>(xs)[tid] = xv;
      if (tid < 72) reinterpret_cast<uint32_t*>(c1s)[tid] = c1v;
    }
  }
  __syncthreads();
  PTO_STAMP(3);
  {
    // 288 outputs on 256 threads: one full output per thread, then the last
    // 32 outputs split 8 ways over all threads (<= 4 taps each, 3-step
    // shuffle sum) instead of a second full round on half a wave.  Taps
    // outside the 8x8 map read position 0 of the same T column (same
    // address as any lane reading it: a broadcast) and are dropped by a
    // select, so all of a thread's reads issue back to back
    {
      const int o = tid, icl = o / 144, pix = o - icl * 144;
      const int y = pix / 12, xx = pix - y * 12;
      float tv[25];
#pragma unroll
      for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const int sy = y - kh, sx = xx - kw;
          const bool ok = (unsigned)sy < 8u && (unsigned)sx < 8u;
          tv[kh * 5 + kw] = ts[(icl * 25 + kh * 5 + kw) * TLD + (ok ? sy * 8 + sx : 0)];
          tv[kh * 5 + kw] = ok ? tv[kh * 5 + kw] : 0.f;
        }
      float sacc = 0.f;
#pragma unroll
      for (int t = 0; t < 25; ++t) sacc += tv[t];
      if (da1p) da1p[b * A1P + (icg * 2 + icl) * 144 + pix] = sacc;
      dsum[o] = sacc;
    }
    {
      const int o = 256 + (tid >> 3), part = tid & 7, pix = o - 144;  // icl = 1
      const int y = pix / 12, xx = pix - y * 12;
      float tv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int tt = part + 8 * i;
        const int kh = tt / 5, kw = tt - kh * 5, sy = y - kh, sx = xx - kw;
        const bool ok = tt < 25 && (unsigned)sy < 8u && (unsigned)sx < 8u;
        tv[i] = ts[(25 + (tt < 25 ? tt : 0)) * TLD + (ok ? sy * 8 + sx : 0)];
        tv[i] = ok ? tv[i] : 0.f;
      }
      float sacc = tv[0];  // tap order, as the sequential sum over valid taps
      sacc += tv[1];
      sacc += tv[2];
      sacc += tv[3];
      sacc += lane_mirror8(sacc);  // sum over the 8 lanes of the output
      sacc += lane_xor2(sacc);
      sacc += lane_xor1(sacc);
      if (part == 0) {
        if (da1p) da1p[b * A1P + (icg * 2 + 1) * 144 + pix] = sacc;
        dsum[o] = sacc;
      }
    }
  }
  if (!fuse1) return;
  // ---- conv1 weight+bias grad of this sample's 2 channels (replaces the
  // separate conv1-backward launch): thread = (channel, tap, pixel
  // quarter); pooled grad expanded through the conv1 argmax code.
  __syncthreads();
  PTO_STAMP(4);
  float* part = ws;  // [4][26] wave totals (free after the GEMM)
  {
    // pixel-major: wave w owns channel w>>1 and 72 of its 144 pooled pixels
    // (lanes 0..63, then lanes 0..7 again); a lane expands its pixel's
    // (grad, code) once and accumulates the 25 taps + bias in registers;
    // the 26 sums are reduced across the wave by recursive halving
    const int icl = wv >> 1, p0 = (wv & 1) * 72;
    float acc[26];
#pragma unroll
    for (int k = 0; k < 26; ++k) acc[k] = 0.f;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int pl = lane + 64 * it;
      if (pl < 72) {
        const int pix = p0 + pl;
        const int cd = c1s[icl * 144 + pix];
        const float v = cd < 4 ? dsum[icl * 144 + pix] : 0.f;
        const int oh = 2 * (pix / 12) + ((cd >> 1) & 1), ow = 2 * (pix % 12) + (cd & 1);
        const float* xp = xs + oh * 28 + ow;
#pragma unroll
        for (int kh = 0; kh < 5; ++kh)
#pragma unroll
          for (int kw = 0; kw < 5; ++kw) acc[kh * 5 + kw] = fmaf(v, xp[kh * 28 + kw], acc[kh * 5 + kw]);
        acc[25] += v;
      }
    }
    wave_halving26(acc, lane, part + wv * 26);
  }
  __syncthreads();
  PTO_STAMP(5);
  if (tid < 52) {
    const int icl = tid / 26, k = tid - icl * 26, oc1 = icg * 2 + icl;
    const float v = part[(2 * icl) * 26 + k] + part[(2 * icl + 1) * 26 + k];
    if (det) {  // deterministic mode: one slot per sample, every element written once
      if (k < 25) gw1[oc1 * 25 + k] = v;
      else gb1[oc1] = v;
    } else {
      if (k < 25) atomicAdd(gw1 + oc1 * 25 + k, v);
      else atomicAdd(gb1 + oc1, v);
    }
  }
}

// db2[oc] = sum of the unmasked pooled grads of channel oc (one wave; the
// result is in every lane).
PTO_DEV float c2_bias_sum(int oc, const float* __restrict__ g2, const uint8_t* __restrict__ code2, int B) {
  const int lane = threadIdx.x & 63;
  float s = 0.f;
  for (int i0 = 0; i0 < B * 16; i0 += 64 * 8) {
    float gv[8];
    int cd[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = i0 + q * 64 + lane;
      const int idx = (i >> 4) * F1IN + oc * 16 + (i & 15);
      const bool ok = i < B * 16;
      gv[q] = ok ? g2[idx] : 0.f;
      cd[q] = ok ? (int)code2[idx] : 4;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) s += cd[q] < 4 ? gv[q] : 0.f;
  }
  return wave_sum(s);
}

__global__ __launch_bounds__(256) void k_conv2_bwd(const float* __restrict__ g2, const uint8_t* __restrict__ code2,
                                                   const float* __restrict__ a1p, const float* __restrict__ w2,
                                                   float* __restrict__ gw2, float* __restrict__ gb2,
                                                   float* __restrict__ da1p, int B, int nA, int nB, int nC,
                                                   const float* __restrict__ x, const long long* __restrict__ bidx,
                                                   const uint8_t* __restrict__ code1, float* __restrict__ gw1,
                                                   float* __restrict__ gb1) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int bid = blockIdx.x;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (bid < nA) {
    c2_wgrad_block<B2_CHUNK>(bid, smem, g2, code2, a1p, gw2, B);
    return;
  }
  bid -= nA;
  if (bid < nB) {
    c2_dgrad_block(bid, smem, g2, code2, w2, da1p, B, x, bidx, code1, gw1, gb1, false);
    return;
  }
  bid -= nB;
  if (bid < nC) {
    // ---- part C: conv2 bias grad, one wave per output channel
    const int oc = bid * 4 + wv;
    if (oc >= C2) return;
    const float s = c2_bias_sum(oc, g2, code2, B);
    if (lane == 0) gb2[oc] = s;
  }
}

// One wave: a 16x16 tile of dW1 = dh1^T a2p (K = B) consumed straight from
// the MMA accumulators by SGD on fc1.weight (pw/mw: its param/momentum
// rows); the gradient itself is never stored.  The wave's p/m elements are
// loaded before the MMA chain so their latency overlaps the operand loads.
PTO_DEV void dw1_sgd_tile(int tile, const float* __restrict__ dh1, const float* __restrict__ a2p,
                          float* __restrict__ pw, float* __restrict__ mw, int B, const SgdArgs& a) {
  constexpr int MT = (F1OUT + 15) / 16, NT = (F1IN + 15) / 16;
  if (tile >= MT * NT) return;
  const int mt = tile % MT, nt = tile / MT, lane = threadIdx.x & 63;
  const int n = nt * 16 + (lane & 15);
  float pv[4], mv[4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int r = mt * 16 + (lane >> 4) * 4 + rr;
    const bool ok = r < F1OUT && n < F1IN;
    pv[rr] = ok ? pw[r * F1IN + n] : 0.f;
    mv[rr] = ok ? mw[r * F1IN + n] : 0.f;
  }
  const float lr = *a.lr;
  // 4 k-groups per memory round (K = B = 64 exactly, 32 loads per lane in
  // flight; 8 groups with half of them masked off was slower)
  const f32x4 acc =
      wave_tile_16x16<LAY_KROW, LAY_KROW, 4>(dh1, F1OUT, a2p, F1IN, F1OUT, F1IN, B, mt * 16, nt * 16, 0, B);
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int r = mt * 16 + (lane >> 4) * 4 + rr;
    if (r < F1OUT && n < F1IN) {
      sgd_elem(pv[rr], acc[rr], mv[rr], lr, a.mom, a.wd, a.gscale, a.nesterov);
      pw[r * F1IN + n] = pv[rr];
      mw[r * F1IN + n] = mv[rr];
    }
  }
}

// One wave: the two dW1 tiles (mt, 2j) and (mt, 2j+1) side by side -- they
// share the dh1 operand (16 loads per lane instead of 32 for two tiles) and
// their four MFMA chains interleave, so a wave holds two tiles for about
// the latency of one (the serial form, PTO_BWD_DTPW 2, measured 2.4 us
// slower).  Each tile's accumulation order is wave_tile_16x16's (chains
// acc0/acc1 over k, summed at the end), so the results are bitwise those of
// dw1_sgd_tile / the grads-only store.  SGD: sgd_elem on fc1.weight;
// grads-only (gout != nullptr): the gradient is stored instead.
PTO_DEV void dw1_tile_pair(int pair, const float* __restrict__ dh1, const float* __restrict__ a2p,
                           float* __restrict__ pw, float* __restrict__ mw, float* __restrict__ gout, int B,
                           const SgdArgs& a) {
  constexpr int MT = (F1OUT + 15) / 16, NT = (F1IN + 15) / 16;
  static_assert(NT % 2 == 0 && F1IN % 16 == 0, "dW1 column tiles pair up with no column tail");
  if (pair >= MT * NT / 2) return;
  const int mt = pair % MT, nt0 = 2 * (pair / MT), lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  float pv[2][4], mv[2][4];
  if (!gout) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = mt * 16 + g * 4 + rr, n = (nt0 + t) * 16 + r;
        const bool ok = row < F1OUT;
        pv[t][rr] = ok ? pw[row * F1IN + n] : 0.f;
        mv[t][rr] = ok ? mw[row * F1IN + n] : 0.f;
      }
  }
  f32x4 acc[2][2] = {{zero4(), zero4()}, {zero4(), zero4()}};
  constexpr int NG = 4;
  for (int k = 0; k < B; k += 16 * NG) {
    float av[NG][4], bv[2][NG][4];
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      load4<LAY_KROW>(dh1, F1OUT, mt * 16 + r, F1OUT, k + 16 * q + 4 * g, B, av[q]);
#pragma unroll
      for (int t = 0; t < 2; ++t) load4<LAY_KROW>(a2p, F1IN, (nt0 + t) * 16 + r, F1IN, k + 16 * q + 4 * g, B, bv[t][q]);
    }
#pragma unroll
    for (int q = 0; q < NG; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[t][j & 1] = mfma16x16x4(av[q][j], bv[t][q][j], acc[t][j & 1]);
  }
  const float lr = gout ? 0.f : *a.lr;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const f32x4 s = acc[t][0] + acc[t][1];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = mt * 16 + g * 4 + rr, n = (nt0 + t) * 16 + r;
      if (row >= F1OUT) continue;
      if (gout) {
        gout[row * F1IN + n] = s[rr];
      } else {
        sgd_elem(pv[t][rr], s[rr], mv[t][rr], lr, a.mom, a.wd, a.gscale, a.nesterov);
        pw[row * F1IN + n] = pv[t][rr];
        mw[row * F1IN + n] = mv[t][rr];
      }
    }
  }
}

// ---------------------------------------------------------------- B1 ----
// conv1 weight+bias grad.  Block = (out channel, chunk of 4 samples = 576
// pooled pixels); a thread owns up to 3 pooled pixels: their (grad, code)
// pairs are loaded in one round, the 25-tap input patches at the winning
// positions in a second round; 26 register accumulators, block reduction,
// 26 atomics per block (16 blocks per channel at B=64).
constexpr int B1_CHUNK = 4;
PTO_DEV void conv1_bwd_block(int vb, const float* __restrict__ g1, const uint8_t* __restrict__ code1,
                             const float* __restrict__ x, float* __restrict__ gw1, float* __restrict__ gb1, int B,
                             const long long* __restrict__ bidx) {
  // One memory round: the chunk's 4 input images (12.5 KB, coalesced
  // float4) go to LDS together with each thread's (grad, code) pairs; the
  // 25-tap patches are then read from LDS.
  __shared__ __attribute__((aligned(16))) float xs[B1_CHUNK * 784];
  __shared__ float part[4][26];
  x = batch_ptr(x, bidx, B * 784);
  const int oc = vb % C1, chunk = vb / C1;
  const int b0 = chunk * B1_CHUNK, nb = min(B, b0 + B1_CHUNK) - b0;
  const int nitems = nb * 144;
  constexpr int PER = (B1_CHUNK * 144 + 255) / 256;
  constexpr int XPER = (B1_CHUNK * 196 + 255) / 256;
  float gv[PER];
  int cd[PER];
  float4 xv[XPER];
#pragma unroll
  for (int q = 0; q < XPER; ++q) {
    const int e = threadIdx.x + 256 * q;
    xv[q] = e < nb * 196 ? reinterpret_cast<const float4*>(x + b0 * 784)[e] : float4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int it = threadIdx.x + 256 * q;
    const bool ok = it < nitems;
    const int idx = ok ? ((b0 + it / 144) * C1 + oc) * 144 + it % 144 : 0;
    gv[q] = ok ? g1[idx] : 0.f;
    cd[q] = ok ? (int)code1[idx] : 4;
  }
#pragma unroll
  for (int q = 0; q < XPER; ++q) {
    const int e = threadIdx.x + 256 * q;
    if (e < B1_CHUNK * 196) reinterpret_cast<float4*>(xs)[e] = xv[q];
  }
  __syncthreads();
  float acc[26];
#pragma unroll
  for (int k = 0; k < 26; ++k) acc[k] = 0.f;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int it = threadIdx.x + 256 * q;
    if (cd[q] >= 4) continue;
    const int smp = it / 144, pix = it - smp * 144;
    const int oh = 2 * (pix / 12) + (cd[q] >> 1), ow = 2 * (pix % 12) + (cd[q] & 1);
    const float* xp = xs + smp * 784 + oh * 28 + ow;
    const float gq = gv[q];
#pragma unroll
    for (int kh = 0; kh < 5; ++kh)
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) acc[kh * 5 + kw] = fmaf(gq, xp[kh * 28 + kw], acc[kh * 5 + kw]);
    acc[25] += gq;
  }
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  wave_halving26(acc, lane, part[wv]);
  __syncthreads();
  if (threadIdx.x < 26) {
    const int q = threadIdx.x;
    const float s = part[0][q] + part[1][q] + part[2][q] + part[3][q];
    if (q < 25) atomicAdd(gw1 + oc * 25 + q, s);
    else atomicAdd(gb1 + oc, s);
  }
}

__global__ __launch_bounds__(256) void k_conv1_bwd(const float* __restrict__ g1, const uint8_t* __restrict__ code1,
                                                   const float* __restrict__ x, float* __restrict__ gw1,
                                                   float* __restrict__ gb1, int B,
                                                   const long long* __restrict__ bidx) {
  conv1_bwd_block(blockIdx.x, g1, code1, x, gw1, gb1, B, bidx);
}

// ------------------------------------------------------ B (all-in-one) ----
// The whole backward + optimizer of the single-process step in ONE launch
// (F12 -> F3 -> F4dx -> B: four launches per step).  Every block range
// consumes only what F4dx / F12 produced, and every parameter is updated by
// the block that finishes its gradient:
//   A  conv2 wgrad (split-K over sample chunks, fp32 atomics).  Per 16-column
//      tile an arrival counter: the chunk block that arrives LAST (after its
//      own atomics have been performed: vmcnt(0)) consumes the finished tile
//      with atomic exchanges (read the memory-side sum, re-zero it for the
//      next step) and applies SGD to conv2.weight -- a stream-K style fixup,
//      no separate optimizer pass.  Nobody else in this launch reads
//      conv2.weight: the dgrad blocks read F12's snapshot of it (w2f).
//   B  conv2 dgrad via col2im, with conv1's wgrad of the same sample/channel
//      pair fused (atomics; conv1's update stays "owed": applied by the next
//      F12, committed by the next F4dx).  d(a1p) is never stored.
//   C  conv2 bias: one wave per channel sums and updates.
//   D  dW1 = dh1^T a2p tiles consumed by SGD on fc1.weight.
//   F  dW2 (fc2) tiles, db1, db2 with SGD epilogues.
// Block 0 advances the batch cursor and marks conv1's update as owed.
// dW1 tiles (16 x 16 of fc1.weight's gradient) per wave of a k_bwd_all D
// block.  A grid of 256-thread blocks starts at ~3.6 ns per block
// (tools/dispatch_ramp_probe.py: 1422 blocks take 4.6-5.4 us just to all be
// running, 711 x 512 threads 2.4 us), and k_bwd_all's 1,422 blocks also
// exceed its 1,280 resident slots, so its D blocks -- last in the grid --
// both start last and wait for slots; fewer, longer D blocks shrink the grid
// (profiles/mnist_step_pmc_r6.md).
#ifndef PTO_BWD_DTPW  // probe builds (tools/bwd_roles_probe.py --dtpw) sweep it
#define PTO_BWD_DTPW 1  // 2-4 measured slower (profiles/mnist_step_pmc_r6.md)
#endif
constexpr int BWD_DTPW = PTO_BWD_DTPW;
// BwdAllArgs::dpair = 1: every D wave holds a PAIR of dW1 tiles side by
// side (dw1_tile_pair: shared dh1 operand, interleaved chains), 200 D blocks
// instead of 400, so the whole 1,222-block grid is resident at once (5 x 256
// slots).  Bitwise equal, but not faster: D alone 5.4 -> 6.7 us, k_bwd_all
// 13.83-13.93 vs 13.96-13.97 us, step 35.99-36.06 vs 36.19-36.25 us
// (profiles/mnist_step_pmc_r6.md).  Host switch PTO_BWD_DPAIR (default 0).
static int bwd_dpair() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PTO_BWD_DPAIR");
    v = (e && BWD_DTPW == 1) ? (atoi(e) != 0) : 0;
  }
  return v;
}
// Role order of k_bwd_all's grid (role ids C 0, F 1, A 2, B 3, D 4).  Order
// 0: the short independent ranges first, then conv2 wgrad, conv2 dgrad,
// dW1 (dgrad-first and dW1-before-dgrad measured 0.9 and 1.4 us slower in
// round 2, profiles/bwd_all_r2.md; re-swept in round 6 with the probe's
// PTO_BWD_ORDER builds, profiles/mnist_step_pmc_r6.md).
#ifndef PTO_BWD_ORDER
#define PTO_BWD_ORDER 0
#endif
__host__ __device__ constexpr int bwd_order(int i) {
  constexpr int o[6][5] = {{0, 1, 2, 3, 4}, {3, 2, 4, 0, 1}, {3, 2, 0, 1, 4}, {2, 3, 0, 1, 4},
                           {3, 4, 2, 0, 1}, {0, 1, 3, 2, 4}};
  return o[PTO_BWD_ORDER][i];
}
constexpr int bwd_n_dw1_blocks(bool pair) {
  return pair ? ((((F1OUT + 15) / 16) * ((F1IN + 15) / 16) / 2) + 3) / 4
              : ((((F1OUT + 15) / 16) * ((F1IN + 15) / 16) + 3) / 4 + BWD_DTPW - 1) / BWD_DTPW;
}

struct BwdAllArgs {
  const float* g2;         // d(a2p) [B][800]
  const uint8_t* code2;
  const float* a1p;
  const float* w2f;        // conv2.weight as F12 read it (snapshot)
  const float* x;          // the batch's images (F12's copy)
  const uint8_t* code1;
  float* gw1;              // conv1 weight/bias grads (atomics, zero on entry)
  float* gb1;
  float* p2w; float* g2w; float* m2w;  // conv2.weight: param, grad (zero on entry, re-zeroed here), momentum
  int* ctr;                // [32] arrival counters, zero on entry and on exit
  float* p2b; float* m2b;  // conv2.bias
  const float* dh1; const float* a2p; const float* h1; const float* dl;
  float* p1w; float* m1w;  // fc1.weight
  float* p1b; float* m1b;  // fc1.bias
  float* pfw; float* mfw;  // fc2.weight
  float* pfb; float* mfb;  // fc2.bias
  SgdArgs a;
  long long* bidx;
  long long nbatches;
  int* pending;
  int B, nA, nB, nC, nD, nF;
  int dpair;               // D role: dW1 tile pairs per wave (bwd_dpair())
  // deterministic mode (wpart != nullptr): no floating-point atomics.  The
  // conv2 wgrad chunks store partial tiles into wpart[chunk] and the last
  // arriver per tile sums them in chunk order; conv1 grads go to one
  // replica per sample (nrep == B), each element stored once.
  float* wpart;
  // conv1 grads are accumulated into nrep replicas (sample b -> b % nrep;
  // replica 0 = gw1/gb1, replica r >= 1 at c1rep + (r-1)*rep_stride, same
  // layout as the flat conv1 range: weights at 0, bias at bias_off), so
  // each address sees B/nrep atomic adds instead of B (same-address adds
  // serialise at the memory side); readers sum the replicas
  float* c1rep;
  int nrep, rep_stride, bias_off;
  // grads_only (multi-GPU step): every gradient is written to the flat grad
  // buffer (g2w/gw1/gb1 accumulated atomically, the rest stored) and no
  // parameter is touched -- the all-reduce's SGD epilogue updates them;
  // the cursor is advanced only if bidx is given (the overlapped xGMI step,
  // whose exchange runs inside the next forward)
  int grads_only;
  float* g2b; float* g1w; float* g1b; float* gfw; float* gfb;  // grad slots of conv2.bias, fc1.w/b, fc2.w/b
  float* hz;  // split fc1's accumulation buffer, re-zeroed here for the next F3 (nz floats, or nullptr)
  int nz;
};

struct EpiSgd {
  float* p; float* m; int ld; float lr; const SgdArgs* a;
  PTO_DEV void operator()(int r, int c, float g) const {
    const int i = r * ld + c;
    float pv = p[i], mv = m[i];
    sgd_elem(pv, g, mv, lr, a->mom, a->wd, a->gscale, a->nesterov);
    p[i] = pv;
    m[i] = mv;
  }
};

template <int CH, int NTW>
__global__ __launch_bounds__(256) void k_bwd_all(BwdAllArgs A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int s_last;
  int bid = blockIdx.x;
  PTO_STAMP_SCOPE();
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (bid == 0 && threadIdx.x == 0) {  // no block of this launch reads the cursor
    if (A.bidx) *A.bidx = (*A.bidx + 1) % A.nbatches;
    if (A.pending) *A.pending = 1;
  }
  if (A.hz) {  // F4dx, its only reader, has finished with it
    const int i = bid * 256 + (int)threadIdx.x;
    if (i < A.nz) A.hz[i] = 0.f;
  }
  // block order (role ranges of the grid): bwd_order(); a grid of
  // 1,422 blocks takes ~5 us just to start (tools/dispatch_ramp_probe.py),
  // so the order decides which roles start late
  int role = 4;
  {
    const int cnt[5] = {A.nC, A.nF, A.nA, A.nB, A.nD};  // role ids: C F A B D
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int r = bwd_order(i);
      if (bid < cnt[r]) {
        role = r;
        break;
      }
      bid -= cnt[r];
    }
  }
  if (role == 0) {  // C
    const int oc = bid * 4 + wv;
    if (oc >= C2) return;
    const float g = c2_bias_sum(oc, A.g2, A.code2, A.B);
    if (lane == 0 && A.grads_only) A.g2b[oc] = g;
    else if (lane == 0) {
      float pv = A.p2b[oc], mv = A.m2b[oc];
      sgd_elem(pv, g, mv, *A.a.lr, A.a.mom, A.a.wd, A.a.gscale, A.a.nesterov);
      A.p2b[oc] = pv;
      A.m2b[oc] = mv;
    }
    return;
  }
  if (role == 1) {  // F
    const float lr = *A.a.lr;
    constexpr int NWF = (((NCLS + 15) / 16) * ((F1OUT + 15) / 16) + 3) / 4;
    if (A.grads_only) {
      if (bid < NWF) {
        block_gemm_4tiles<LAY_KROW, LAY_KROW>(A.dl, NCLS, A.h1, F1OUT, NCLS, F1OUT, A.B, bid, EpiStore{A.gfw, F1OUT});
        return;
      }
      bid -= NWF;
      if (bid < 8) block_colsum64(A.dh1, F1OUT, A.B, F1OUT, bid * 64, smem, A.g1b);
      else block_colsum64(A.dl, NCLS, A.B, NCLS, 0, smem, A.gfb);
      return;
    }
    if (bid < NWF) {
      block_gemm_4tiles<LAY_KROW, LAY_KROW>(A.dl, NCLS, A.h1, F1OUT, NCLS, F1OUT, A.B, bid,
                                            EpiSgd{A.pfw, A.mfw, F1OUT, lr, &A.a});
      return;
    }
    bid -= NWF;
    if (bid < 8) block_colsum64_epi(A.dh1, F1OUT, A.B, F1OUT, bid * 64, smem, EpiSgd{A.p1b, A.m1b, 0, lr, &A.a});
    else block_colsum64_epi(A.dl, NCLS, A.B, NCLS, 0, smem, EpiSgd{A.pfb, A.mfb, 0, lr, &A.a});
    return;
  }
  if (role == 2) {  // A
    const bool det = A.wpart != nullptr;
    c2_wgrad_block<CH, NTW>(bid, smem, A.g2, A.code2, A.a1p, A.g2w, A.B, A.wpart);
    if (A.grads_only && !det) return;
    // arrival: every lane's atomics have been performed at the memory side
    // (deterministic mode: the partial-tile stores are written back first)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    PTO_STAMP(3);
    constexpr int NT = 32 / NTW, TC = 16 * NTW;  // column tiles per chunk, columns per tile
    const int nt = bid % NT, nchunk = A.nA / NT;
    if (threadIdx.x == 0) {
      if (det) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const int old = __hip_atomic_fetch_add(A.ctr + nt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == nchunk - 1;
      if (s_last) {
        __hip_atomic_store(A.ctr + nt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (det) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
    }
    __syncthreads();
    PTO_STAMP(4);
    if (!s_last) return;
    constexpr int NQ = (C2 * TC + 255) / 256;  // tile elements per thread
    int idx[NQ];
    float gv[NQ], pv[NQ], mv[NQ];
    if (det) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int e = threadIdx.x + 256 * q, row = e / TC, col = nt * TC + (e % TC);
        idx[q] = (e < C2 * TC && col < 500) ? row * 500 + col : -1;
        float g = 0.f;
        if (idx[q] >= 0)
          for (int c = 0; c < nchunk; ++c) g += A.wpart[c * (C2 * 500) + idx[q]];  // chunk order
        gv[q] = g;
      }
      if (A.grads_only) {
#pragma unroll
        for (int q = 0; q < NQ; ++q)
          if (idx[q] >= 0) A.g2w[idx[q]] = gv[q];
        return;
      }
    }
    const float lr = *A.a.lr;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {  // 50 rows x TC columns
      const int e = threadIdx.x + 256 * q, row = e / TC, col = nt * TC + (e % TC);
      idx[q] = (e < C2 * TC && col < 500) ? row * 500 + col : -1;
      if (idx[q] >= 0) {
        if (!det) gv[q] = atomicExch(A.g2w + idx[q], 0.f);
        pv[q] = A.p2w[idx[q]];
        mv[q] = A.m2w[idx[q]];
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (idx[q] >= 0) {
        sgd_elem(pv[q], gv[q], mv[q], lr, A.a.mom, A.a.wd, A.a.gscale, A.a.nesterov);
        A.p2w[idx[q]] = pv[q];
        A.m2w[idx[q]] = mv[q];
      }
    return;
  }
  if (role == 3) {  // B
    const int r = (bid / B2_ICG) % A.nrep;
    float* gw1 = r == 0 ? A.gw1 : A.c1rep + (r - 1) * A.rep_stride;
    float* gb1 = r == 0 ? A.gb1 : A.c1rep + (r - 1) * A.rep_stride + A.bias_off;
    c2_dgrad_block(bid, smem, A.g2, A.code2, A.w2f, nullptr, A.B, A.x, nullptr, A.code1, gw1, gb1,
                   A.wpart != nullptr);
    return;
  }
  if (role == 4) {  // D
    if (A.dpair) {  // two dW1 tiles per wave, side by side
      dw1_tile_pair(bid * 4 + wv, A.dh1, A.a2p, A.p1w, A.m1w, A.grads_only ? A.g1w : nullptr, A.B, A.a);
      return;
    }
    // BWD_DTPW dW1 tiles per wave, one after the other (no barriers in this role)
#pragma unroll
    for (int j = 0; j < BWD_DTPW; ++j) {
      const int vb = bid * BWD_DTPW + j;
      if (A.grads_only)
        block_gemm_4tiles<LAY_KROW, LAY_KROW, EpiStore, 4>(A.dh1, F1OUT, A.a2p, F1IN, F1OUT, F1IN, A.B, vb,
                                                          EpiStore{A.g1w, F1IN});
      else
        dw1_sgd_tile(vb * 4 + wv, A.dh1, A.a2p, A.p1w, A.m1w, A.B, A.a);
    }
    return;
  }
}

// Host-side flush of an owed conv1 update (before the parameters are read
// or replaced): commit it and clear `pending`.  One block.
__global__ __launch_bounds__(256) void k_conv1_commit(Conv1Commit cm, int* __restrict__ pending) {
  const int pend = *cm.pending;
  const float lr = *cm.a.lr;  // in flight with the flag (one round trip, not two)
  if (!pend) return;
  for (int i = 4 * threadIdx.x; i < cm.n; i += 1024) commit4(cm, i, lr);
  __syncthreads();
  if (threadIdx.x == 0) *pending = 0;
}

// The RCCL schedule's optimizer launch (ddp-rccl).  The all-reduce covers
// the flat gradient buffer AND the conv1 replica tail allocated right after
// it (one message), so k_bwd_all spreads conv1's same-address atomics over
// C1_REPLICAS copies on this schedule too; this launch folds them in replica
// order (commit4's association), applies SGD to the flat params/momentum,
// zeroes the atomically accumulated range [zero_from, n) and the replicas,
// and advances the batch cursor.  One float4 per thread.
__global__ __launch_bounds__(256) void k_ddp_sgd(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                 int n, int c1, int zero_from, float* __restrict__ rep, int nrep,
                                                 SgdArgs a, long long* __restrict__ bidx, long long nbatches) {
  if (bidx && blockIdx.x == 0 && threadIdx.x == 0) *bidx = (*bidx + 1) % nbatches;
  const int i = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= n) return;
  const float lr = *a.lr;
  if (i >= c1) {
    const Conv1Commit cm{p + c1, g + c1, m + c1, n - c1, nullptr, a, rep, nrep, n - c1};
    commit4(cm, i - c1, lr);
  } else {
    sgd_flat4(p, g, m, i, lr, a, i >= zero_from);
  }
}

// conv1 data gradient (only needed when the input requires grad, e.g. the
// nn.Module path under autograd checks).  dx[b][y][x] = sum dY1 * w.
__global__ __launch_bounds__(256) void k_conv1_bwd_data(const float* __restrict__ g1,
                                                        const uint8_t* __restrict__ code1,
                                                        const float* __restrict__ w, float* __restrict__ dx, int B) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * 784) return;
  const int b = idx / 784, pix = idx - b * 784, y = pix / 28, xx = pix - (pix / 28) * 28;
  float s = 0.f;
  for (int oc = 0; oc < C1; ++oc)
    for (int kh = 0; kh < 5; ++kh) {
      const int oh = y - kh;
      if (oh < 0 || oh >= 24) continue;
      for (int kw = 0; kw < 5; ++kw) {
        const int ow = xx - kw;
        if (ow < 0 || ow >= 24) continue;
        const int pi = ((b * C1 + oc) * 12 + (oh >> 1)) * 12 + (ow >> 1);
        if (code1[pi] == ((oh & 1) * 2 + (ow & 1))) s = fmaf(g1[pi], w[oc * 25 + kh * 5 + kw], s);
      }
    }
  dx[idx] = s;
}

// Eval head: fused argmax + correct count + summed NLL (K11) over the
// log-probabilities written by k_fc2_ce.  stats = [loss_sum, correct].
__global__ __launch_bounds__(256) void k_eval_head(const float* __restrict__ logp, const int64_t* __restrict__ labels,
                                                   float* __restrict__ stats, int B) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  float loss = 0.f, corr = 0.f;
  if (row < B) {
    const float* z = logp + row * NCLS;
    int am = 0;
    float mv = z[0];
    for (int c = 1; c < NCLS; ++c)
      if (z[c] > mv) { mv = z[c]; am = c; }
    const int y = (int)labels[row];
    loss = -z[y];
    corr = (am == y) ? 1.f : 0.f;
  }
  loss = wave_sum(loss);
  corr = wave_sum(corr);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(stats, loss);
    atomicAdd(stats + 1, corr);
  }
}

}  // namespace

// ======================================================================
// C ABI launchers (loaded with ctypes; every launcher is graph-capturable:
// no allocation, no sync, everything on the caller's stream).
// ======================================================================
#define PTO_API extern "C" __attribute__((visibility("default")))
#define LAUNCH_CHECK() return (int)hipGetLastError()

PTO_API int pto_conv1_fwd(const float* x, const float* w, const float* b, float* out, uint8_t* code, int B,
                          const long long* bidx, hipStream_t s) {
  hipLaunchKernelGGL(k_conv1_fwd, dim3((B * 720 + 255) / 256), dim3(256), 0, s, x, w, b, out, code, B, bidx);
  LAUNCH_CHECK();
}

PTO_API int pto_conv2_fwd(const float* a1p, const float* w, const float* b, float* out, uint8_t* code, int B,
                          hipStream_t s) {
  hipLaunchKernelGGL(k_conv2_fwd, dim3(B * 4), dim3(256), 0, s, a1p, w, b, out, code, B);
  LAUNCH_CHECK();
}

static SgdArgs sgd_args(const float* lr, float mom, float wd, float gscale, int nesterov) {
  SgdArgs a;
  a.lr = lr;
  a.mom = mom;
  a.wd = wd;
  a.gscale = gscale;
  a.nesterov = nesterov;
  a.variant = 0;
  return a;
}

// F12: conv1 + conv2 forward.  g1f/m1f/pending non-null: conv1's owed SGD
// update is applied on the fly (flat conv1 grads/momentum, weights at 0,
// bias at bias_off, `nrep` gradient replicas at rep + r*rep_stride); xout:
// the batch's images copied out for the backward; w2out: the conv2.weight
// snapshot k_bwd_all's dgrad blocks read.
PTO_API int pto_conv12_fwd_lazy_x(const float* x, const float* w1, const float* b1, const float* w2,
                                  const float* b2, float* a1p, uint8_t* code1, float* a2p, uint8_t* code2, int B,
                                  const long long* bidx, const float* g1f, const float* m1f, int bias_off,
                                  const int* pending, const float* lr, float mom, float wd, float gscale, int nesterov,
                                  float* xout, float* w2out, const float* rep, int nrep, int rep_stride,
                                  hipStream_t s) {
  if (nrep < 1 || nrep > C1_MAXREP || (nrep > 1 && !rep) || (pending && (!g1f || !m1f || !lr))) return -1;
  LazyConv1 lz{g1f, m1f, pending, sgd_args(lr, mom, wd, gscale, nesterov), bias_off, xout, w2out, rep, nrep,
               rep_stride};
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv12_fwd2_t<1024, 0>), dim3(B * 4), dim3(1024), 0, s, x, w1, b1, w2, b2, a1p,
                     code1, a2p, code2, B, bidx, lz, ArRole{}, ArRole{});
  LAUNCH_CHECK();
}

extern "C" long long pto_ar_timeout_ticks();

// F12 (plain forward: no lazy conv1 update) + the previous step's gradient
// exchange of the overlapped multi-GPU step as two roles of the same launch
// (protocol: 0 coherent, 1 fenced -- the one the XgmiAllReduce instance of
// `peers` uses; shared peers table, epochs and error word):
//   conv role  one-shot all-reduce + SGD of [cv_off, cv_off + cv_n) on
//              channel cv_chan; the gradient replicas of [rep_from, rep_from
//              + rep_stride) are part of the registered buffer (replica r >=
//              1 at float index rep_base + (r-1)*rep_stride) and every rank
//              reads every rank's; gradient and replicas zeroed after its
//              second barrier; the conv blocks wait on *ready
//   fc role    rank-split all-reduce + SGD of [fc_off, fc_off + fc_n) on
//              channel fc_chan, local gradient zeroed from fc_zero_from
// B == 0: the two roles alone (the closing exchange of a captured run).
PTO_API int pto_conv12_fwd_ar(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                              float* a1p, uint8_t* code1, float* a2p, uint8_t* code2, int B, const long long* bidx,
                              float* xout, const void* peers, int rank, int world, void* epochs, void* err,
                              int protocol, float* p, float* m, const float* lr, float mom, float wd, float gscale,
                              int nesterov, long long fc_off, long long fc_n, int fc_chan, long long fc_zero_from,
                              long long cv_off, long long cv_n, int cv_chan, long long rep_base, int nrep,
                              int rep_stride, long long rep_from, int* ready, hipStream_t s) {
  using namespace pto_ar;
  if (fc_n <= AR_ONESHOT_MAX || fc_n % 4 || fc_off % 4 || fc_n > (1LL << 29) || cv_n > AR_ONESHOT_MAX || cv_n < 4 ||
      cv_n % 4 || cv_off % 4 || world < 1 || world > AR_MAX_RANKS || fc_chan < 0 || fc_chan >= AR_CHANNELS ||
      cv_chan < 0 || cv_chan >= AR_CHANNELS || fc_chan == cv_chan || rank < 0 || rank >= world || !p || !m || !lr ||
      !peers || !ready || protocol < 0 || protocol > 1 || B < 0 || ((((uintptr_t)p) | ((uintptr_t)m)) & 15))
    return -1;
  if (nrep < 1 || nrep > AR_MAX_REP || (nrep > 1 && (rep_stride % 4 || rep_from % 4 || rep_base % 4 ||
                                                      rep_base < cv_off + cv_n || rep_from < cv_off ||
                                                      rep_from + rep_stride > cv_off + cv_n)))
    return -1;
  LazyConv1 lz{nullptr, nullptr, nullptr, sgd_args(lr, mom, wd, gscale, nesterov), 0, xout, nullptr, nullptr, 1, 0};
  ArRole ar{}, cv{};
  for (ArRole* r : {&ar, &cv}) {
    r->peers = reinterpret_cast<const ArPeers*>(peers);
    r->rank = rank;
    r->world = world;
    r->epochs = reinterpret_cast<uint32_t*>(epochs);
    r->err = reinterpret_cast<int*>(err);
    r->timeout = pto_ar_timeout_ticks();
    r->f = ArSgd{};
    r->f.p = p;
    r->f.m = m;
    r->f.a = sgd_args(lr, mom, wd, gscale, nesterov);
    r->f.nbatches = 1;
    r->f.nrep = 1;
    r->ready = ready;
  }
  ar.off = fc_off;
  ar.n4 = fc_n / 4;
  ar.chan = fc_chan;
  ar.nblk = role_blocks(fc_n, world, 1024);
  ar.f.zero_from = fc_zero_from;
  cv.off = cv_off;
  cv.n4 = cv_n / 4;
  cv.chan = cv_chan;
  cv.nblk = oneshot_role_blocks(cv_n, world, 1024);
  cv.f.zero_from = cv_off;
  cv.f.nrep = nrep;
  cv.f.rep_stride = rep_stride;
  cv.f.rep_from = rep_from;
  cv.f.rep_base = rep_base;
  if (ar.nblk > AR_MAX_BLOCKS || cv.nblk > AR_MAX_BLOCKS) return -1;
  const dim3 g((unsigned)(B * 4 + ar.nblk + cv.nblk));
  if (protocol)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv12_fwd2_t<1024, 2>), g, dim3(1024), 0, s, x, w1, b1, w2, b2, a1p, code1,
                       a2p, code2, B, bidx, lz, ar, cv);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv12_fwd2_t<1024, 1>), g, dim3(1024), 0, s, x, w1, b1, w2, b2, a1p, code1,
                       a2p, code2, B, bidx, lz, ar, cv);
  LAUNCH_CHECK();
}

PTO_API int pto_linear_fwd(const float* x, const float* w, const float* b, float* y, int M, int N, int K, int relu,
                           hipStream_t s) {
  const int tiles = ((M + 15) / 16) * ((N + 15) / 16);
  const bool vec = (K % 4) == 0 && ((((uintptr_t)x) | ((uintptr_t)w)) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(k_linear_fwd_vec16, dim3(tiles), dim3(1024), 0, s, x, w, b, y, M, N, K, relu);
  else
    hipLaunchKernelGGL(k_linear_fwd, dim3(tiles), dim3(256), 0, s, x, w, b, y, M, N, K, relu);
  LAUNCH_CHECK();
}

// fc1 forward of the training step, split-K over two workgroups per tile
// (k_fc1_fwd_split2): h += x W^T (h zero on entry), no bias / ReLU (F4dx
// applies them, k_bwd_all re-zeroes h).
PTO_API int pto_fc1_fwd_split(const float* x, const float* w, float* h, int M, hipStream_t s) {
  if (M < 1 || !x || !w || !h || ((((uintptr_t)x) | ((uintptr_t)w)) & 15)) return -1;
  static const int nw = [] {
    const char* e = getenv("PTO_FC1_NW");
    const int v = e ? atoi(e) : 16;  // 16 waves of 32-deep slices: 34.13-34.19 vs 34.34-34.40 us/step with 8
    return (v == 4 || v == 8) ? v : 16;
  }();
  const dim3 g(((M + 15) / 16) * 64);
  if (nw == 4)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fc1_fwd_split2<4>), g, dim3(256), 0, s, x, w, h, M);
  else if (nw == 16)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fc1_fwd_split2<16>), g, dim3(1024), 0, s, x, w, h, M);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fc1_fwd_split2<8>), g, dim3(512), 0, s, x, w, h, M);
  LAUNCH_CHECK();
}

PTO_API int pto_linear_bwd(const float* dy, const float* x, const float* w, float* dx, float* dw, float* db, int M,
                           int N, int K, hipStream_t s) {
  if (dx) {
    const int tiles = ((M + 15) / 16) * ((K + 15) / 16);
    hipLaunchKernelGGL(k_linear_bwd_data, dim3(tiles), dim3(256), 0, s, dy, w, dx, M, N, K);
  }
  if (dw) {
    const int tiles = ((N + 15) / 16) * ((K + 15) / 16);
    hipLaunchKernelGGL(k_linear_bwd_weight, dim3((tiles + 3) / 4), dim3(256), 0, s, dy, x, dw, M, N, K);
  }
  if (db) hipLaunchKernelGGL(k_colsum, dim3((N + 63) / 64), dim3(256), 0, s, dy, db, M, N);
  LAUNCH_CHECK();
}

PTO_API int pto_relu_bwd(const float* g, const float* y, float* out, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_relu_bwd, dim3((n + 255) / 256), dim3(256), 0, s, g, y, out, n);
  LAUNCH_CHECK();
}

PTO_API int pto_fc2_ce(const float* h1, const float* w, const float* b, const int64_t* labels, float* logp,
                       float* loss_rows, float* dlogits, float* dh1, int B, float inv_b, const long long* bidx,
                       hipStream_t s) {
  hipLaunchKernelGGL(k_fc2_ce, dim3((B + 3) / 4), dim3(256), 0, s, h1, w, b, labels, logp, loss_rows, dlogits, dh1,
                     B, inv_b, bidx);
  LAUNCH_CHECK();
}

PTO_API int pto_conv1_commit(float* p1, float* g1, float* m1, int n1, int* pending, const float* lr, float mom,
                             float wd, float gscale, int nesterov, float* rep, int nrep, int rep_stride,
                             hipStream_t s) {
  if (n1 % 4 || rep_stride % 4 || ((((uintptr_t)p1) | ((uintptr_t)g1) | ((uintptr_t)m1) | ((uintptr_t)rep)) & 15))
    return -1;
  Conv1Commit cm{p1, g1, m1, n1, pending, sgd_args(lr, mom, wd, gscale, nesterov), rep, nrep, rep_stride};
  hipLaunchKernelGGL(k_conv1_commit, dim3(1), dim3(256), 0, s, cm, pending);
  LAUNCH_CHECK();
}

// ddp-rccl optimizer launch (k_ddp_sgd): flat buffers of n floats, conv1
// range [c1, n), replicas r >= 1 at rep + (r-1)*(n-c1).
PTO_API int pto_mnist_ddp_sgd(float* p, float* g, float* m, int n, int c1, int zero_from, float* rep, int nrep,
                              const float* lr, float mom, float wd, float gscale, int nesterov, long long* bidx,
                              long long nbatches, hipStream_t s) {
  if (n % 4 || c1 % 4 || zero_from % 4 || c1 < 0 || c1 >= n || !lr || nrep < 1 || nrep > C1_MAXREP ||
      (nrep > 1 && !rep) || (bidx && nbatches < 1))
    return -1;
  if ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)rep)) & 15) return -1;
  hipLaunchKernelGGL(k_ddp_sgd, dim3((n / 4 + 255) / 256), dim3(256), 0, s, p, g, m, n, c1, zero_from, rep, nrep,
                     sgd_args(lr, mom, wd, gscale, nesterov), bidx, nbatches);
  LAUNCH_CHECK();
}

// parts: bit0 = weight grad (atomic-accumulated: gw2 must be zeroed by the
// caller), bit1 = data grad, bit2 = bias grad.
// With gw1 != nullptr the dgrad part also accumulates conv1's weight/bias
// grads (gw1/gb1 zeroed by the caller) from x (+ batch cursor) and code1.
PTO_API int pto_conv2_bwd(const float* g2, const uint8_t* code2, const float* a1p, const float* w2, float* gw2,
                          float* gb2, float* da1p, int B, int parts, const float* x, const long long* bidx,
                          const uint8_t* code1, float* gw1, float* gb1, hipStream_t s) {
  if ((parts & 2) && (((uintptr_t)w2) & 7)) return -1;  // float2 staging of the W2 slice
  const int nA = (parts & 1) ? ((B + B2_CHUNK - 1) / B2_CHUNK) * 32 : 0;
  const int nB = (parts & 2) ? B * B2_ICG : 0;
  const int nC = (parts & 4) ? (C2 + 3) / 4 : 0;
  const size_t ldsA = (parts & 1) ? wgrad_lds_floats<B2_CHUNK, 1>() * sizeof(float) : 0;
  const size_t ldsB = (parts & 2) ? B2_LDS_FLOATS * sizeof(float) : 0;
  const size_t lds = ldsA > ldsB ? ldsA : ldsB;
  if (nA + nB + nC == 0) return 0;
  hipLaunchKernelGGL(k_conv2_bwd, dim3(nA + nB + nC), dim3(256), lds, s, g2, code2, a1p, w2, gw2, gb2, da1p, B, nA,
                     nB, nC, x, bidx, code1, (parts & 2) ? gw1 : nullptr, gb1);
  LAUNCH_CHECK();
}

// F4dx (k_fc2_ce_dx_mf) + one extra block committing conv1's owed update
// (pending != nullptr; flat range p1/g1/m1 of n1 floats + replicas) and
// resetting *zero_word (non-null: the overlapped step's conv-role counter,
// which the previous F12 launch's conv blocks waited on) + STAGE_BLOCKS
// blocks copying the next batch's images (st_x [st_nb][B * 784], batch
// (*bidx + 1) % st_nb) into st_xnext, the next F12's input (optional).
PTO_API int pto_fc2_ce_dx(const float* h1, const float* w2, const float* b2, const int64_t* labels, const float* w1,
                          float* loss_rows, float* dlogits, float* dh1, float* da2p, int B, float inv_b,
                          const long long* bidx, float* p1, float* g1, float* m1, int n1, const int* pending,
                          const float* lr, float mom, float wd, float gscale, int nesterov, float* rep, int nrep,
                          int rep_stride, int* zero_word, const float* st_x, float* st_xnext, long long st_nb,
                          const float* b1, float* h1out, hipStream_t s) {
  if (b1 && (!h1out || ((((uintptr_t)b1) | ((uintptr_t)h1out)) & 15))) return -1;
  if (n1 % 4 || rep_stride % 4 || ((((uintptr_t)p1) | ((uintptr_t)g1) | ((uintptr_t)m1) | ((uintptr_t)rep)) & 15))
    return -1;
  if ((((uintptr_t)h1) | ((uintptr_t)w2)) & 15) return -1;  // float4 staging of the h1 tile and W2
  if (nrep < 1 || nrep > C1_MAXREP || (nrep > 1 && !rep)) return -1;
  if (st_xnext && (!st_x || !bidx || st_nb < 1 || ((((uintptr_t)st_x) | ((uintptr_t)st_xnext)) & 15))) return -1;
  Conv1Commit cm{p1, g1, m1, n1, pending, sgd_args(lr, mom, wd, gscale, nesterov), rep, nrep, rep_stride, zero_word};
  const BatchStage st{st_x, st_xnext, st_nb, B * 784 / 4};
  const int nblk = ((B + 15) / 16) * ((F1IN + 15) / 16);
  hipLaunchKernelGGL(k_fc2_ce_dx_mf, dim3(nblk + 1 + (st_xnext ? STAGE_BLOCKS : 0)), dim3(FDX_WAVES * 64), 0, s, h1,
                     w2, b2, labels, w1, loss_rows, dlogits, dh1, da2p, B, inv_b, bidx, cm, st, b1, h1out);
  LAUNCH_CHECK();
}

// gw1/gb1 are atomic-accumulated: zeroed by the caller.
PTO_API int pto_conv1_bwd(const float* g1, const uint8_t* code1, const float* x, float* gw1, float* gb1, int B,
                          const long long* bidx, hipStream_t s) {
  const int nblk = C1 * ((B + B1_CHUNK - 1) / B1_CHUNK);
  hipLaunchKernelGGL(k_conv1_bwd, dim3(nblk), dim3(256), 0, s, g1, code1, x, gw1, gb1, B, bidx);
  LAUNCH_CHECK();
}

PTO_API int pto_conv1_bwd_data(const float* g1, const uint8_t* code1, const float* w, float* dx, int B,
                               hipStream_t s) {
  hipLaunchKernelGGL(k_conv1_bwd_data, dim3((B * 784 + 255) / 256), dim3(256), 0, s, g1, code1, w, dx, B);
  LAUNCH_CHECK();
}

PTO_API int pto_eval_head(const float* logp, const int64_t* labels, float* stats, int B, hipStream_t s) {
  hipLaunchKernelGGL(k_eval_head, dim3((B + 255) / 256), dim3(256), 0, s, logp, labels, stats, B);
  LAUNCH_CHECK();
}

// Samples per conv2-wgrad block of k_bwd_all: 5 -> 29.7 KB of LDS with the
// padded 20/260 a1p planes, 5 blocks per CU next to the 29.5 KB dgrad blocks
// (6 needs 35.6 KB: 4 blocks per CU; role probe, all roles: 13.99 vs 14.63 us,
// profiles/lds_conflicts_r3.md; the round-2 sweep over 4..8 with the dense
// planes picked 6, profiles/bwd_all_r2.md).
#ifndef PTO_BWD_WCHUNK  // probe builds (tools/bwd_roles_probe.py --chunk) sweep it
#define PTO_BWD_WCHUNK 5
#endif
constexpr int BWD_WCHUNK = PTO_BWD_WCHUNK;
// 16-column tiles per conv2-wgrad block of k_bwd_all.  2 shares the staged
// grads/codes (and the A-operand reads) between two tiles but halves the
// wgrad blocks: k_bwd_all 16.5 -> 18.4 us (r3), so 1
constexpr int BWD_WNTW = 1;

// The all-in-one backward (+ optimizer) launch (k_bwd_all).  Flat-buffer
// views: p/g/m + offsets of each parameter (elements); ctr: 32 zeroed ints.
PTO_API int pto_bwd_all(const float* g2, const uint8_t* code2, const float* a1p, const float* w2f, const float* x,
                        const uint8_t* code1, const float* dh1, const float* a2p, const float* h1, const float* dl,
                        float* p, float* g, float* m, long long off_fc2w, long long off_fc2b, long long off_fc1w,
                        long long off_fc1b, long long off_c2w, long long off_c2b, long long off_c1w,
                        long long off_c1b, int* ctr, long long* bidx, long long nbatches, int* pending, int B,
                        const float* lr, float mom, float wd, float gscale, int nesterov, float* c1rep, int nrep,
                        int rep_stride, int grads_only, float* wpart, float* hz, int nz, hipStream_t s) {
  if (!ctr) return -1;
  if (((uintptr_t)(grads_only ? p + off_c2w : w2f)) & 7) return -1;  // float2 staging of the W2 slice
  if (!grads_only && (!bidx || !pending || !w2f)) return -1;
  if (bidx && nbatches < 1) return -1;
  if (B < 1 || nrep < 1 || nrep > C1_MAXREP || (nrep > 1 && !c1rep)) return -1;
  if (wpart && nrep != B) return -1;  // deterministic mode: one conv1 replica per sample
  BwdAllArgs A;
  A.g2 = g2; A.code2 = code2; A.a1p = a1p; A.w2f = w2f; A.x = x; A.code1 = code1;
  A.gw1 = g + off_c1w; A.gb1 = g + off_c1b;
  A.p2w = p + off_c2w; A.g2w = g + off_c2w; A.m2w = m + off_c2w; A.ctr = ctr;
  A.p2b = p + off_c2b; A.m2b = m + off_c2b;
  A.dh1 = dh1; A.a2p = a2p; A.h1 = h1; A.dl = dl;
  A.p1w = p + off_fc1w; A.m1w = m + off_fc1w;
  A.p1b = p + off_fc1b; A.m1b = m + off_fc1b;
  A.pfw = p + off_fc2w; A.mfw = m + off_fc2w;
  A.pfb = p + off_fc2b; A.mfb = m + off_fc2b;
  A.a = sgd_args(lr, mom, wd, gscale, nesterov);
  A.c1rep = c1rep;
  A.nrep = nrep;
  A.rep_stride = rep_stride;
  A.bias_off = (int)(off_c1b - off_c1w);
  A.grads_only = grads_only;
  A.g2b = g + off_c2b; A.g1w = g + off_fc1w; A.g1b = g + off_fc1b; A.gfw = g + off_fc2w; A.gfb = g + off_fc2b;
  if (grads_only) A.w2f = p + off_c2w;  // nothing updates conv2.weight in this launch
  A.bidx = bidx; A.nbatches = nbatches; A.pending = pending; A.B = B;
  A.nA = ((B + BWD_WCHUNK - 1) / BWD_WCHUNK) * (32 / BWD_WNTW);
  A.nB = B * B2_ICG;
  A.nC = (C2 + 3) / 4;
  A.dpair = bwd_dpair();
  A.nD = bwd_n_dw1_blocks(A.dpair);
  A.nF = (((NCLS + 15) / 16) * ((F1OUT + 15) / 16) + 3) / 4 + 9;
  A.wpart = wpart;
  A.hz = hz;
  A.nz = hz ? nz : 0;
  if ((long long)A.nz > (long long)(A.nA + A.nB + A.nC + A.nD + A.nF) * 256) return -1;  // one element per thread
  const size_t ldsA = wgrad_lds_floats<BWD_WCHUNK, BWD_WNTW>() * sizeof(float);
  const size_t ldsB = B2_LDS_FLOATS * sizeof(float);
  const size_t lds = ldsA > ldsB ? ldsA : ldsB;
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_bwd_all<BWD_WCHUNK, BWD_WNTW>), dim3(A.nA + A.nB + A.nC + A.nD + A.nF), dim3(256), lds, s, A);
  LAUNCH_CHECK();
}
