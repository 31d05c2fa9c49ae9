// Single-node gradient all-reduce over xGMI peer memory (IPC-mapped HBM
// of the other ranks), for the small/medium DDP buckets where RCCL's
// per-collective latency dominates (MNIST: 1.7 MB of fp32 gradients per
// step; RCCL ring/tree setup costs tens of microseconds for that size).
//
// Algorithm: two-stage "pull" all-reduce, every write local:
//   barrier 1   every rank's input is complete (stream order) and published
//   stage 1     rank r sums chunk r of ALL ranks' inputs (fixed rank order, so
//               every rank ends with bit-identical results) -> own tmp[chunk r]
//   barrier 2   all partial sums published
//   stage 2     rank r pulls chunk q from rank q's tmp for every q -> own input
// Per rank that is 2 x (W-1)/W x bytes read over xGMI (the same as a
// reduce-scatter + all-gather ring) but in ONE launch with two barriers,
// no ring steps.  The barriers are per workgroup: workgroup b of every rank
// owns the same sub-range of every chunk, so block b only waits for block b
// of the peers (no grid-wide sync).
//
// Hazards covered by construction: a rank only overwrites its input in
// stage 2 (after every peer finished reading it in stage 1 = barrier 2),
// and only overwrites tmp in the NEXT call's stage 1 (after barrier 1 of
// that call, which peers only reach once their previous launch, including
// its stage-2 reads of this tmp, has completed).
//
// Visibility: two protocols (pto_ar_set_protocol, chosen at setup; the
// trainer's autotune verifies the one it keeps against RCCL on the real
// links, falling back from 0 to 1 to RCCL).
//
//   0 "coherent" (default): NO cache-maintenance fences.  Every byte a peer
//     reads that this launch writes (the folded gradient, the stage-1 partial
//     sums in tmp) is stored WRITE-THROUGH at system scope (buffer stores
//     with sc0 sc1); every storing wave drains (s_waitcnt vmcnt(0): the
//     stores are acknowledged at system scope) and the workgroup barrier
//     orders that before the one-lane flag store (system-scope relaxed store
//     into the peer's uncached flag page).  Every load of peer-written bytes
//     is a system-coherent buffer load (sc0 sc1: misses in this CU's L1 and
//     this XCD's L2), so no acquire is needed (the system-scope analogue of
//     MI355X_MICROARCH.md "Valid forms": sc1 payload + drained flag, sc1
//     loads).  The gradient bytes written by the PREVIOUS kernel on the
//     stream (k_bwd_all) are in HBM once that kernel has ended: the end-of-
//     kernel release writes every XCD's dirty L2 lines back (at least agent
//     scope, which on the 8-XCD part is an L2 write-back, or the next kernel
//     on another XCD could not read them), and a peer's sc0 sc1 loads read
//     HBM.  Cost per barrier: one flag round trip, no L2 walk.
//   1 "fenced": plain stores and loads; producer = stores -> s_waitcnt
//     vmcnt(0) -> barrier -> release fence (system: L2 write-back) ->
//     s_waitcnt vmcnt(0) -> relaxed system flag store; consumer = relaxed poll
//     -> system acquire (L1/L2 invalidate) -> s_waitcnt -> barrier -> loads.
//     One write-back + one invalidate per workgroup per barrier (18.8 us per
//     call at world 1, profiles/ddp_step_r3.md).
// Flags live in uncached memory; every spin is bounded (pto_ar_set_timeout_ms,
// default 500 ms) and reports a timeout through *err instead of hanging the
// device.
//
// Failure semantics (a peer died or stalled): the first barrier that times
// out sets *err; from then on every barrier of this rank -- in this launch
// and in every later launch -- returns at once without waiting or
// publishing, so a dead peer costs ONE timeout, not one per barrier, and
// the peers still waiting on this rank time out too (the whole job fails
// together and restarts from its checkpoint).  A workgroup whose barrier
// failed skips the rest of the kernel: no partial sums from incomplete peer
// data are written, no parameter is updated, no gradient is zeroed.  The
// host reads *err after every run() chunk (FusedMnistTrainer.check_comm) and
// exits with the retryable code 138.
//
// Two independent "channels" (flag sets + epochs) let two buckets be in
// flight at once on different streams.
//
// Small buckets (<= AR_ONESHOT_MAX floats, e.g. MNIST's 100 KB conv bucket,
// which sits on the step's critical path) use a one-shot variant instead:
// barrier 1, every rank reads the WHOLE range from all ranks and reduces it
// in rank order (bit-identical everywhere; one element per thread, kept in
// registers), barrier 2 (nobody reads my input any more), then the local
// write / optimizer epilogue.  One remote round trip instead of two, no tmp.
//
// Optimizer epilogue (k_xgmi_allreduce<true>): stage 2 does not store the
// reduced gradient; it applies SGD-momentum to the local parameters and
// momentum with it (same element formula as the multi-tensor SGD launch,
// sgd_f32.h) and zeroes the local gradient from `zero_from` on (the
// atomically accumulated range).  The DDP step then needs no optimizer
// launch.  Zeroing is safe in stage 2: every
// peer read this rank's gradient in its stage 1, before barrier 2.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "sgd_f32.h"

#define PTO_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int AR_MAX_RANKS = 8;
// workgroups per launch: ceil(chunk / AR_THREADS) up to this cap, so every
// thread handles ONE float4 per stage down to world 1-2 on MNIST's 1.7 MB
constexpr int AR_MAX_BLOCKS = 256;
constexpr int AR_CHANNELS = 2;
constexpr int AR_THREADS = 512;
constexpr int AR_MAX_REP = 256;  // gradient replicas folded before barrier 1 (launcher check)
constexpr int AR_REP_CHUNK = 16;  // replica loads in flight at once
// stage-1 sums of this rank's own chunk kept in registers for stage 2 (the
// same thread handles element j of the chunk in both stages): iterations
// beyond this re-read them from tmp
constexpr int AR_CARRY = 4;
constexpr long long AR_ONESHOT_MAX = 65536;  // floats (256 KB): one-shot path
constexpr long long AR_TICKS_PER_MS = 100000LL;  // wall_clock64 runs at 100 MHz
long long g_timeout_ticks = 500 * AR_TICKS_PER_MS;  // pto_ar_set_timeout_ms
int g_protocol = 0;  // pto_ar_set_protocol: 0 coherent (write-through + sc0 sc1 loads), 1 fenced

// buffer-instruction cache bits (aux operand): sc0 | sc1 = system scope
constexpr int AUX_SYS = 1 | 16;

// global (not flat) views of generic pointers: flag words and the local
// parameter/momentum/gradient float4 groups
using gu32 = __attribute__((address_space(1))) uint32_t;
using v4f = __attribute__((ext_vector_type(4))) float;
using gv4f = __attribute__((address_space(1))) v4f;
__device__ __forceinline__ gu32* G(uint32_t* p) { return (gu32*)p; }
__device__ __forceinline__ float4 gld4(const float* p) {
  const v4f v = *(const gv4f*)p;
  return float4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ void gst4(float* p, float4 a) { *(gv4f*)p = v4f{a.x, a.y, a.z, a.w}; }

struct ArPeers {
  float* in[AR_MAX_RANKS];
  float* tmp[AR_MAX_RANKS];
  uint32_t* flags[AR_MAX_RANKS];
};

__host__ __device__ constexpr int flag_index(int chan, int phase, int block, int src) {
  return ((chan * 2 + phase) * AR_MAX_BLOCKS + block) * AR_MAX_RANKS + src;
}
constexpr int AR_FLAG_WORDS = AR_CHANNELS * 2 * AR_MAX_BLOCKS * AR_MAX_RANKS;

// float4 access to a buffer that peers read or write.  COHERENT: system-
// scope buffer loads/stores (sc0 sc1), i.e. write-through stores and loads
// that miss in L1/L2; otherwise plain accesses (the fenced protocol's
// release/acquire provide visibility).  The descriptor covers `bytes` from
// `base` (the launcher keeps every range below 2 GB).
struct Buf {
  __amdgpu_buffer_rsrc_t r;
  float* p;
};
__device__ __forceinline__ Buf mkbuf(float* base, long long bytes) {
  return Buf{__builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000), base};
}
template <bool COHERENT>
__device__ __forceinline__ float4 ld4(const Buf& b, long long i4) {
  if constexpr (COHERENT) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(b.r, (int)(i4 * 16), 0, AUX_SYS);
    return __builtin_bit_cast(float4, v);
  } else {
    return reinterpret_cast<const float4*>(b.p)[i4];
  }
}
template <bool COHERENT>
__device__ __forceinline__ void st4(const Buf& b, long long i4, float4 v) {
  if constexpr (COHERENT) {
    using u4 = __attribute__((ext_vector_type(4))) unsigned int;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), b.r, (int)(i4 * 16), 0, AUX_SYS);
  } else {
    reinterpret_cast<float4*>(b.p)[i4] = v;
  }
}

// Returns false (for every thread of the block) if the barrier failed: a
// peer did not arrive within `timeout` ticks, or an earlier barrier of this
// rank already failed (*err != 0).  s_fail is per phase, so a fast thread
// resetting phase 1's word cannot race a slow thread still reading phase 0's.
// FENCED: system release before the flag store, system acquire after the
// wait; otherwise the drained write-through stores need no release and the
// consumer's sc0 sc1 loads no acquire.
template <bool FENCED>
__device__ __forceinline__ bool block_barrier(const ArPeers* __restrict__ P, int chan, int phase, int rank, int world, uint32_t e,
                                              long long timeout, int* err) {
  __shared__ int s_fail[2];
  const int t = threadIdx.x, b = blockIdx.x;
  if (t == 0) s_fail[phase] = 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave: its stores acknowledged
  __syncthreads();
  if (t < world) {
    bool dead = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    if (!dead) {
      if constexpr (FENCED) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: write back this XCD's L2
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_store(G(P->flags[t] + flag_index(chan, phase, b, rank)), e, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      gu32* f = G(P->flags[rank] + flag_index(chan, phase, b, t));
      const long long t0 = wall_clock64();
      while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != e) {
        if (wall_clock64() - t0 > timeout) {
          atomicOr(err, 1 << phase);
          dead = true;
          break;
        }
        // another block (or an earlier launch) already gave up: stop now
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
          dead = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if constexpr (FENCED) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // invalidate L1/L2 before reading peer data
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler order only: no loads above the poll
      }
    }
    if (dead) s_fail[phase] = 1;
  }
  __syncthreads();
  return s_fail[phase] == 0;
}

// Fused optimizer epilogue of the all-reduce: own parameters/momentum (same
// flat layout as the gradient buffer), hyper-parameters, zero range, and an
// optional batch cursor advanced once the update is done.
struct ArSgd {
  float* p;
  float* m;
  SgdArgs a;
  long long zero_from;  // float index: own gradient zeroed from here on
  long long* bidx;      // nullptr: no cursor
  long long nbatches;
  // optional gradient replicas of the float range [rep_from, rep_from +
  // rep_stride) (k_bwd_all's conv1 replicas, multi-GPU step): replica r >= 1
  // at rep + (r-1)*rep_stride.  Folded into the local gradient (and zeroed)
  // by the workgroup that owns the element, BEFORE barrier 1, so every peer
  // reads folded values.
  float* rep;
  int nrep, rep_stride;
  long long rep_from;
};

// Fold the local replicas into float4 element i4 (float offset 4*i4 from the
// buffer base) of the local gradient, if it lies in the replicated range.
// Every replica load is issued before the first add; the folded value is
// stored through `g` (write-through under the coherent protocol: peers read
// it).
template <bool COHERENT>
__device__ __forceinline__ void fold_rep(const ArSgd& f, const Buf& g, long long off, long long i4) {
  const long long fi = off + 4 * i4;  // float index in the whole buffer (rep_from's frame)
  if (!f.rep || f.nrep <= 1 || fi < f.rep_from || fi >= f.rep_from + f.rep_stride) return;
  const long long k = fi - f.rep_from;
  float4 a = gld4(g.p + 4 * i4);
  for (int r0 = 0; r0 < f.nrep - 1; r0 += AR_REP_CHUNK) {  // replica order
    float4 v[AR_REP_CHUNK];
#pragma unroll
    for (int r = 0; r < AR_REP_CHUNK; ++r)
      v[r] = gld4(f.rep + (long long)min(r0 + r, f.nrep - 2) * f.rep_stride + k);
#pragma unroll
    for (int r = 0; r < AR_REP_CHUNK; ++r) {
      if (r0 + r >= f.nrep - 1) break;
      a.x += v[r].x; a.y += v[r].y; a.z += v[r].z; a.w += v[r].w;
      gst4(f.rep + (long long)(r0 + r) * f.rep_stride + k, float4{0.f, 0.f, 0.f, 0.f});
    }
  }
  st4<COHERENT>(g, i4, a);
}

// SGD on float4 group i (float index) of the local parameters/momentum.
__device__ __forceinline__ void sgd4(const ArSgd& f, long long i, float4 g, float4& pv, float4& mv, float lr) {
  sgd_elem(pv.x, g.x, mv.x, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
  sgd_elem(pv.y, g.y, mv.y, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
  sgd_elem(pv.z, g.z, mv.z, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
  sgd_elem(pv.w, g.w, mv.w, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
  gst4(f.p + i, pv);
  gst4(f.m + i, mv);
}

__device__ __forceinline__ float4 add4(float4 a, float4 b) { return float4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }

// n4 float4 elements starting at float offset `off` of every rank's buffers.
template <bool SGD, bool FENCED>
__global__ __launch_bounds__(AR_THREADS) void k_xgmi_allreduce(const ArPeers* __restrict__ peers, long long off,
                                                               long long n4, int rank, int world, int chan,
                                                               uint32_t* __restrict__ epochs, int* err, long long timeout,
                                                               ArSgd f) {
  constexpr bool CO = !FENCED;
  __shared__ uint32_t s_epoch;
  const ArPeers* __restrict__ P = peers;
  if (threadIdx.x == 0) s_epoch = epochs[chan * AR_MAX_BLOCKS + blockIdx.x] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  if (threadIdx.x == 0) epochs[chan * AR_MAX_BLOCKS + blockIdx.x] = e;
  const long long cs = (n4 + world - 1) / world;  // chunk length (float4)
  const long long stride = (long long)gridDim.x * AR_THREADS;
  const long long j0 = (long long)blockIdx.x * AR_THREADS + threadIdx.x;
  const long long bytes = n4 * 16;
  float* const my_in = P->in[rank];
  if (f.rep && f.nrep > 1 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
    // the elements this workgroup's peers will read: the same sub-range of every chunk
    const Buf g = mkbuf(my_in + off, bytes);
    for (int q = 0; q < world; ++q)
      for (long long j = j0; j < cs && q * cs + j < n4; j += stride) fold_rep<CO>(f, g, off, q * cs + j);
  }

  if (!block_barrier<FENCED>(P, chan, 0, rank, world, e, timeout, err)) return;
  // stage 1: reduce my chunk over all ranks (rank order 0..W-1 everywhere);
  // the first AR_CARRY iterations' sums stay in registers for stage 2, tmp
  // gets them only if a peer (or a later iteration) reads them
  float4 own[AR_CARRY];
  {
    const long long c0 = (long long)rank * cs, c1 = min(n4, c0 + cs);
    int it = 0;
    for (long long i = c0 + j0; i < c1; i += stride, ++it) {
      float4 v[AR_MAX_RANKS];
#pragma unroll
      for (int q = 0; q < AR_MAX_RANKS; ++q)
        if (q < world) v[q] = ld4<CO>(mkbuf(P->in[q] + off, bytes), i);
      float4 a = v[0];
#pragma unroll
      for (int q = 1; q < AR_MAX_RANKS; ++q)
        if (q < world) a = add4(a, v[q]);
#pragma unroll
      for (int c = 0; c < AR_CARRY; ++c)
        if (c == it) own[c] = a;
      if (world > 1 || it >= AR_CARRY) st4<CO>(mkbuf(P->tmp[rank] + off, bytes), i, a);
    }
  }
  const float lr = SGD ? *f.a.lr : 0.f;
  if (!block_barrier<FENCED>(P, chan, 1, rank, world, e, timeout, err)) return;
  // stage 2: gather every chunk into my input (or: update my parameters)
  int it = 0;
  for (long long j = j0; j < cs; j += stride, ++it) {
    float4 v[AR_MAX_RANKS];
#pragma unroll
    for (int q = 0; q < AR_MAX_RANKS; ++q)
      if (q < world && (long long)q * cs + j < n4) {
        if (q == rank && it < AR_CARRY) {
#pragma unroll
          for (int c = 0; c < AR_CARRY; ++c)
            if (c == it) v[q] = own[c];
        } else {
          v[q] = ld4<CO>(mkbuf(P->tmp[q] + off, bytes), q * cs + j);
        }
      }
#pragma unroll
    for (int q = 0; q < AR_MAX_RANKS; ++q)
      if (q < world && (long long)q * cs + j < n4) {
        if constexpr (SGD) {
          const long long i = off + 4 * (q * cs + j);
          float4 pv = gld4(f.p + i);
          float4 mv = gld4(f.m + i);
          sgd4(f, i, v[q], pv, mv, lr);
          if (i >= f.zero_from) gst4(my_in + i, float4{0.f, 0.f, 0.f, 0.f});
        } else {
          gst4(my_in + off + 4 * (q * cs + j), v[q]);
        }
      }
  }
  if (SGD && f.bidx && blockIdx.x == 0 && threadIdx.x == 0) *f.bidx = (*f.bidx + 1) % f.nbatches;
}

// One-shot variant: n4 <= gridDim.x * AR_THREADS (one float4 per thread).
template <bool SGD, bool FENCED>
__global__ __launch_bounds__(AR_THREADS) void k_xgmi_allreduce_1shot(const ArPeers* __restrict__ peers,
                                                                     long long off, long long n4, int rank,
                                                                     int world, int chan,
                                                                     uint32_t* __restrict__ epochs, int* err,
                                                                     long long timeout, ArSgd f) {
  constexpr bool CO = !FENCED;
  __shared__ uint32_t s_epoch;
  const ArPeers* __restrict__ P = peers;
  if (threadIdx.x == 0) s_epoch = epochs[chan * AR_MAX_BLOCKS + blockIdx.x] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  if (threadIdx.x == 0) epochs[chan * AR_MAX_BLOCKS + blockIdx.x] = e;
  const long long i = (long long)blockIdx.x * AR_THREADS + threadIdx.x;
  const bool act = i < n4;
  const long long bytes = n4 * 16;
  float* const my_in = P->in[rank];
  if (act && f.rep && f.nrep > 1 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
    fold_rep<CO>(f, mkbuf(my_in + off, bytes), off, i);
  if (!block_barrier<FENCED>(P, chan, 0, rank, world, e, timeout, err)) return;
  float4 a = {0.f, 0.f, 0.f, 0.f};
  if (act) {
    float4 v[AR_MAX_RANKS];
#pragma unroll
    for (int q = 0; q < AR_MAX_RANKS; ++q)
      if (q < world) v[q] = ld4<CO>(mkbuf(P->in[q] + off, bytes), i);
    a = v[0];
#pragma unroll
    for (int q = 1; q < AR_MAX_RANKS; ++q)
      if (q < world) a = add4(a, v[q]);
  }
  // every peer is done reading my input (on failure: nothing is written)
  if (!block_barrier<FENCED>(P, chan, 1, rank, world, e, timeout, err)) return;
  if (act) {
    if constexpr (SGD) {
      const float lr = *f.a.lr;
      const long long j = off + 4 * i;
      float4 pv = gld4(f.p + j);
      float4 mv = gld4(f.m + j);
      sgd4(f, j, a, pv, mv, lr);
      if (j >= f.zero_from) gst4(my_in + j, float4{0.f, 0.f, 0.f, 0.f});
    } else {
      gst4(my_in + off + 4 * i, a);
    }
  }
  if (SGD && f.bidx && blockIdx.x == 0 && threadIdx.x == 0) *f.bidx = (*f.bidx + 1) % f.nbatches;
}

// Workgroups used for n floats (identical on every rank: derived from n, W).
int blocks_for(long long n, int world) {
  if (n <= AR_ONESHOT_MAX) return (int)((n / 4 + AR_THREADS - 1) / AR_THREADS);
  const long long cs = ((n / 4) + world - 1) / world;
  long long b = (cs + AR_THREADS - 1) / AR_THREADS;
  if (b < 1) b = 1;
  if (b > AR_MAX_BLOCKS) b = AR_MAX_BLOCKS;
  return (int)b;
}

template <bool SGD>
int launch(const void* peers, long long off, long long n, int rank, int world, int chan, void* epochs, void* err,
           const ArSgd& f, hipStream_t s) {
  const ArPeers* P = reinterpret_cast<const ArPeers*>(peers);
  uint32_t* ep = reinterpret_cast<uint32_t*>(epochs);
  int* er = reinterpret_cast<int*>(err);
  const long long n4 = n / 4;
  if (n <= AR_ONESHOT_MAX) {
    const dim3 g((unsigned)((n4 + AR_THREADS - 1) / AR_THREADS));
    if (g_protocol)
      hipLaunchKernelGGL(HIP_KERNEL_NAME(k_xgmi_allreduce_1shot<SGD, true>), g, dim3(AR_THREADS), 0, s, P, off, n4,
                         rank, world, chan, ep, er, g_timeout_ticks, f);
    else
      hipLaunchKernelGGL(HIP_KERNEL_NAME(k_xgmi_allreduce_1shot<SGD, false>), g, dim3(AR_THREADS), 0, s, P, off, n4,
                         rank, world, chan, ep, er, g_timeout_ticks, f);
    return (int)hipGetLastError();
  }
  const dim3 g((unsigned)blocks_for(n, world));
  if (g_protocol)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_xgmi_allreduce<SGD, true>), g, dim3(AR_THREADS), 0, s, P, off, n4, rank,
                       world, chan, ep, er, g_timeout_ticks, f);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_xgmi_allreduce<SGD, false>), g, dim3(AR_THREADS), 0, s, P, off, n4, rank,
                       world, chan, ep, er, g_timeout_ticks, f);
  return (int)hipGetLastError();
}

}  // namespace

// ---------------------------------------------------------------- host API
PTO_API int pto_ar_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }
PTO_API int pto_ar_flag_bytes(int) { return AR_FLAG_WORDS * (int)sizeof(uint32_t); }
PTO_API int pto_ar_max_ranks() { return AR_MAX_RANKS; }
PTO_API int pto_ar_peers_bytes() { return (int)sizeof(ArPeers); }
PTO_API int pto_ar_epoch_words() { return AR_CHANNELS * AR_MAX_BLOCKS; }
// Barrier spin bound for launches issued (or graph-captured) from now on.
PTO_API int pto_ar_set_timeout_ms(int ms) {
  if (ms < 1) return -1;
  g_timeout_ticks = (long long)ms * AR_TICKS_PER_MS;
  return 0;
}
// Visibility protocol for launches issued (or graph-captured) from now on:
// 0 coherent (default), 1 fenced (see the file header).  Every rank of a
// group must use the same one.
PTO_API int pto_ar_set_protocol(int p) {
  if (p < 0 || p > 1) return -1;
  g_protocol = p;
  return 0;
}
PTO_API int pto_ar_get_protocol() { return g_protocol; }

// Flags: uncached device memory, zeroed.
PTO_API int pto_ar_alloc_flags(void** out) {
  hipError_t e = hipExtMallocWithFlags(out, (size_t)AR_FLAG_WORDS * sizeof(uint32_t), hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*out, 0, (size_t)AR_FLAG_WORDS * sizeof(uint32_t));
}
PTO_API int pto_ar_free(void* p) { return (int)hipFree(p); }

// IPC handle of the allocation containing ptr, plus ptr's byte offset in it.
PTO_API int pto_ar_get_ipc_handle(void* ptr, void* handle_out, long long* offset_out) {
  void* base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, ptr);
  if (e != hipSuccess) return (int)e;
  *offset_out = (long long)((char*)ptr - (char*)base);
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle_out), base);
}
PTO_API int pto_ar_open_ipc_handle(const void* handle, void** ptr_out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof h);
  return (int)hipIpcOpenMemHandle(ptr_out, h, hipIpcMemLazyEnablePeerAccess);
}
PTO_API int pto_ar_close_ipc_handle(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

PTO_API int pto_ar_blocks(long long n, int world) { return blocks_for(n, world); }

// Largest range (floats) one call may cover: the buffer descriptors of the
// coherent protocol address it with 32-bit byte offsets.
constexpr long long AR_MAX_FLOATS = (1LL << 29) - 4;

// In-place SUM all-reduce of n floats at float offset `off` of the registered
// input buffers.  peers: device copy of ArPeers.  Requires n % 4 == 0,
// off % 4 == 0, 1 <= world <= 8 (world 1: the one-process measurement of the
// multi-GPU step, no peers), chan < 2.
PTO_API int pto_ar_allreduce(const void* peers, long long off, long long n, int rank, int world, int chan,
                             void* epochs, void* err, hipStream_t s) {
  if (n % 4 || off % 4 || n > AR_MAX_FLOATS || world < 1 || world > AR_MAX_RANKS || chan < 0 ||
      chan >= AR_CHANNELS || rank < 0 || rank >= world)
    return -1;
  if (n == 0) return 0;
  return launch<false>(peers, off, n, rank, world, chan, epochs, err, ArSgd{}, s);
}

// All-reduce + SGD-momentum epilogue over the same range: p/m are this rank's
// flat parameter/momentum buffers (gradient layout, 16-byte aligned); the
// reduced gradient is scaled by gscale (1/world: DDP's mean), consumed by
// the update and not stored; the local gradient is zeroed from float index
// zero_from on; bidx (optional) advances mod nbatches after the update.
PTO_API int pto_ar_allreduce_sgd(const void* peers, long long off, long long n, int rank, int world, int chan,
                                 void* epochs, void* err, float* p, float* m, const float* lr, float mom, float wd,
                                 float gscale, int nesterov, long long zero_from, long long* bidx,
                                 long long nbatches, float* rep, int nrep, int rep_stride, long long rep_from,
                                 hipStream_t s) {
  if (n % 4 || off % 4 || n > AR_MAX_FLOATS || world < 1 || world > AR_MAX_RANKS || chan < 0 ||
      chan >= AR_CHANNELS || rank < 0 || rank >= world || !p || !m || !lr ||
      ((((uintptr_t)p) | ((uintptr_t)m)) & 15) || (bidx && nbatches < 1))
    return -1;
  if (rep && (nrep < 1 || nrep > AR_MAX_REP || rep_stride % 4 || rep_from % 4 || (((uintptr_t)rep) & 15)))
    return -1;
  if (n == 0) return 0;
  ArSgd f;
  f.p = p;
  f.m = m;
  f.a.lr = lr;
  f.a.mom = mom;
  f.a.wd = wd;
  f.a.gscale = gscale;
  f.a.nesterov = nesterov;
  f.zero_from = zero_from;
  f.bidx = bidx;
  f.nbatches = nbatches;
  f.rep = rep;
  f.nrep = rep ? nrep : 1;
  f.rep_stride = rep_stride;
  f.rep_from = rep_from;
  return launch<true>(peers, off, n, rank, world, chan, epochs, err, f, s);
}
