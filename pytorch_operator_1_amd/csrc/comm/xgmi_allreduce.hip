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
// Visibility (MI355X_MICROARCH.md "inter-workgroup visibility", applied at
// system scope because readers are other devices): producer = stores ->
// s_waitcnt vmcnt(0) -> barrier -> release fence (system: L2 write-back) ->
// s_waitcnt vmcnt(0) -> relaxed system flag store; consumer = relaxed poll ->
// system acquire (L1/L2 invalidate) -> s_waitcnt -> barrier -> loads.
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
// (64 left a 3-round dependent chain per stage at world 1: 18.8 us)
constexpr int AR_MAX_BLOCKS = 256;
constexpr int AR_CHANNELS = 2;
constexpr int AR_THREADS = 512;
constexpr int AR_MAX_REP = 256;  // gradient replicas folded before barrier 1 (launcher check)
constexpr int AR_REP_CHUNK = 16;  // replica loads in flight at once
constexpr long long AR_ONESHOT_MAX = 65536;  // floats (256 KB): one-shot path
constexpr long long AR_TICKS_PER_MS = 100000LL;  // wall_clock64 runs at 100 MHz
long long g_timeout_ticks = 500 * AR_TICKS_PER_MS;  // pto_ar_set_timeout_ms

struct ArPeers {
  float* in[AR_MAX_RANKS];
  float* tmp[AR_MAX_RANKS];
  uint32_t* flags[AR_MAX_RANKS];
};

__host__ __device__ constexpr int flag_index(int chan, int phase, int block, int src) {
  return ((chan * 2 + phase) * AR_MAX_BLOCKS + block) * AR_MAX_RANKS + src;
}
constexpr int AR_FLAG_WORDS = AR_CHANNELS * 2 * AR_MAX_BLOCKS * AR_MAX_RANKS;

// Returns false (for every thread of the block) if the barrier failed: a
// peer did not arrive within `timeout` ticks, or an earlier barrier of this
// rank already failed (*err != 0).  s_fail is per phase, so a fast thread
// resetting phase 1's word cannot race a slow thread still reading phase 0's.
__device__ __forceinline__ bool block_barrier(const ArPeers& P, int chan, int phase, int rank, int world, uint32_t e,
                                              long long timeout, int* err) {
  __shared__ int s_fail[2];
  const int t = threadIdx.x, b = blockIdx.x;
  if (t == 0) s_fail[phase] = 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t < world) {
    bool dead = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    if (!dead) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: write back this XCD's L2
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(P.flags[t] + flag_index(chan, phase, b, rank), e, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      uint32_t* f = P.flags[rank] + flag_index(chan, phase, b, t);
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
        __builtin_amdgcn_s_sleep(2);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // invalidate L1/L2 before reading peer data
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

// Fold the local replicas into float4 element (float offset fi) of the local
// gradient g, if fi lies in the replicated range.  Every replica load is
// issued before the first add.
__device__ __forceinline__ void fold_rep(const ArSgd& f, float* g, long long fi) {
  if (!f.rep || f.nrep <= 1 || fi < f.rep_from || fi >= f.rep_from + f.rep_stride) return;
  const long long k = fi - f.rep_from;
  float4 a = *reinterpret_cast<const float4*>(g + fi);
  for (int r0 = 0; r0 < f.nrep - 1; r0 += AR_REP_CHUNK) {  // replica order
    float4 v[AR_REP_CHUNK];
#pragma unroll
    for (int r = 0; r < AR_REP_CHUNK; ++r)
      v[r] = *reinterpret_cast<const float4*>(f.rep + (long long)min(r0 + r, f.nrep - 2) * f.rep_stride + k);
#pragma unroll
    for (int r = 0; r < AR_REP_CHUNK; ++r) {
      if (r0 + r >= f.nrep - 1) break;
      a.x += v[r].x; a.y += v[r].y; a.z += v[r].z; a.w += v[r].w;
      *reinterpret_cast<float4*>(f.rep + (long long)(r0 + r) * f.rep_stride + k) = float4{0.f, 0.f, 0.f, 0.f};
    }
  }
  *reinterpret_cast<float4*>(g + fi) = a;
}

// n4 float4 elements starting at float offset `off` of every rank's buffers.
template <bool SGD>
__global__ __launch_bounds__(AR_THREADS) void k_xgmi_allreduce(const ArPeers* __restrict__ peers, long long off,
                                                               long long n4, int rank, int world, int chan,
                                                               uint32_t* __restrict__ epochs, int* err, long long timeout,
                                                               ArSgd f) {
  __shared__ uint32_t s_epoch;
  const ArPeers P = *peers;
  if (threadIdx.x == 0) s_epoch = epochs[chan * AR_MAX_BLOCKS + blockIdx.x] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  if (threadIdx.x == 0) epochs[chan * AR_MAX_BLOCKS + blockIdx.x] = e;
  const long long cs = (n4 + world - 1) / world;  // chunk length (float4)
  const long long stride = (long long)gridDim.x * AR_THREADS;
  if (f.rep && f.nrep > 1 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
    // the elements this workgroup's peers will read: the same sub-range of every chunk
    for (int q = 0; q < world; ++q)
      for (long long j = (long long)blockIdx.x * AR_THREADS + threadIdx.x; j < cs && q * cs + j < n4; j += stride)
        fold_rep(f, P.in[rank], off + 4 * (q * cs + j));
  }

  if (!block_barrier(P, chan, 0, rank, world, e, timeout, err)) return;
  // stage 1: reduce my chunk over all ranks (rank order 0..W-1 everywhere)
  {
    const long long c0 = (long long)rank * cs, c1 = min(n4, c0 + cs);
    for (long long i = c0 + (long long)blockIdx.x * AR_THREADS + threadIdx.x; i < c1; i += stride) {
      float4 v[AR_MAX_RANKS];
#pragma unroll
      for (int q = 0; q < AR_MAX_RANKS; ++q)
        if (q < world) v[q] = reinterpret_cast<const float4*>(P.in[q] + off)[i];
      float4 a = v[0];
#pragma unroll
      for (int q = 1; q < AR_MAX_RANKS; ++q)
        if (q < world) {
          a.x += v[q].x;
          a.y += v[q].y;
          a.z += v[q].z;
          a.w += v[q].w;
        }
      reinterpret_cast<float4*>(P.tmp[rank] + off)[i] = a;
    }
  }
  if (!block_barrier(P, chan, 1, rank, world, e, timeout, err)) return;
  // stage 2: gather every chunk into my input (or: update my parameters)
  const float lr = SGD ? *f.a.lr : 0.f;
  for (long long j = (long long)blockIdx.x * AR_THREADS + threadIdx.x; j < cs; j += stride) {
    float4 v[AR_MAX_RANKS];
#pragma unroll
    for (int q = 0; q < AR_MAX_RANKS; ++q)
      if (q < world && (long long)q * cs + j < n4) v[q] = reinterpret_cast<const float4*>(P.tmp[q] + off)[q * cs + j];
#pragma unroll
    for (int q = 0; q < AR_MAX_RANKS; ++q)
      if (q < world && (long long)q * cs + j < n4) {
        if constexpr (SGD) {
          const long long i = off + 4 * (q * cs + j);
          float4 pv = *reinterpret_cast<float4*>(f.p + i);
          float4 mv = *reinterpret_cast<float4*>(f.m + i);
          sgd_elem(pv.x, v[q].x, mv.x, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
          sgd_elem(pv.y, v[q].y, mv.y, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
          sgd_elem(pv.z, v[q].z, mv.z, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
          sgd_elem(pv.w, v[q].w, mv.w, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
          *reinterpret_cast<float4*>(f.p + i) = pv;
          *reinterpret_cast<float4*>(f.m + i) = mv;
          if (i >= f.zero_from) *reinterpret_cast<float4*>(P.in[rank] + i) = float4{0.f, 0.f, 0.f, 0.f};
        } else {
          reinterpret_cast<float4*>(P.in[rank] + off)[q * cs + j] = v[q];
        }
      }
  }
  if (SGD && f.bidx && blockIdx.x == 0 && threadIdx.x == 0) *f.bidx = (*f.bidx + 1) % f.nbatches;
}

// One-shot variant: n4 <= gridDim.x * AR_THREADS (one float4 per thread).
template <bool SGD>
__global__ __launch_bounds__(AR_THREADS) void k_xgmi_allreduce_1shot(const ArPeers* __restrict__ peers,
                                                                     long long off, long long n4, int rank,
                                                                     int world, int chan,
                                                                     uint32_t* __restrict__ epochs, int* err,
                                                                     long long timeout, ArSgd f) {
  __shared__ uint32_t s_epoch;
  const ArPeers P = *peers;
  if (threadIdx.x == 0) s_epoch = epochs[chan * AR_MAX_BLOCKS + blockIdx.x] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  if (threadIdx.x == 0) epochs[chan * AR_MAX_BLOCKS + blockIdx.x] = e;
  const long long i = (long long)blockIdx.x * AR_THREADS + threadIdx.x;
  const bool act = i < n4;
  if (act && f.rep && f.nrep > 1 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
    fold_rep(f, P.in[rank], off + 4 * i);
  if (!block_barrier(P, chan, 0, rank, world, e, timeout, err)) return;
  float4 a = {0.f, 0.f, 0.f, 0.f};
  if (act) {
    float4 v[AR_MAX_RANKS];
#pragma unroll
    for (int q = 0; q < AR_MAX_RANKS; ++q)
      if (q < world) v[q] = reinterpret_cast<const float4*>(P.in[q] + off)[i];
    a = v[0];
#pragma unroll
    for (int q = 1; q < AR_MAX_RANKS; ++q)
      if (q < world) {
        a.x += v[q].x;
        a.y += v[q].y;
        a.z += v[q].z;
        a.w += v[q].w;
      }
  }
  // every peer is done reading my input (on failure: nothing is written)
  if (!block_barrier(P, chan, 1, rank, world, e, timeout, err)) return;
  if (act) {
    if constexpr (SGD) {
      const float lr = *f.a.lr;
      const long long j = off + 4 * i;
      float4 pv = *reinterpret_cast<float4*>(f.p + j);
      float4 mv = *reinterpret_cast<float4*>(f.m + j);
      sgd_elem(pv.x, a.x, mv.x, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
      sgd_elem(pv.y, a.y, mv.y, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
      sgd_elem(pv.z, a.z, mv.z, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
      sgd_elem(pv.w, a.w, mv.w, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
      *reinterpret_cast<float4*>(f.p + j) = pv;
      *reinterpret_cast<float4*>(f.m + j) = mv;
      if (j >= f.zero_from) *reinterpret_cast<float4*>(P.in[rank] + j) = float4{0.f, 0.f, 0.f, 0.f};
    } else {
      reinterpret_cast<float4*>(P.in[rank] + off)[i] = a;
    }
  }
  if (SGD && f.bidx && blockIdx.x == 0 && threadIdx.x == 0) *f.bidx = (*f.bidx + 1) % f.nbatches;
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

// Workgroups used for n floats (identical on every rank: derived from n, W).
PTO_API int pto_ar_blocks(long long n, int world) {
  if (n <= AR_ONESHOT_MAX) return (int)((n / 4 + AR_THREADS - 1) / AR_THREADS);
  const long long cs = ((n / 4) + world - 1) / world;
  long long b = (cs + AR_THREADS - 1) / AR_THREADS;
  if (b < 1) b = 1;
  if (b > AR_MAX_BLOCKS) b = AR_MAX_BLOCKS;
  return (int)b;
}

// In-place SUM all-reduce of n floats at float offset `off` of the registered
// input buffers.  peers: device copy of ArPeers.  Requires n % 4 == 0,
// off % 4 == 0, 1 <= world <= 8 (world 1: the one-process measurement of the
// multi-GPU step, no peers), chan < 2.
PTO_API int pto_ar_allreduce(const void* peers, long long off, long long n, int rank, int world, int chan,
                             void* epochs, void* err, hipStream_t s) {
  if (n % 4 || off % 4 || world < 1 || world > AR_MAX_RANKS || chan < 0 || chan >= AR_CHANNELS || rank < 0 ||
      rank >= world)
    return -1;
  if (n == 0) return 0;
  if (n <= AR_ONESHOT_MAX) {
    hipLaunchKernelGGL(k_xgmi_allreduce_1shot<false>, dim3((unsigned)((n / 4 + AR_THREADS - 1) / AR_THREADS)),
                       dim3(AR_THREADS), 0, s, reinterpret_cast<const ArPeers*>(peers), off, n / 4, rank, world, chan,
                       reinterpret_cast<uint32_t*>(epochs), reinterpret_cast<int*>(err), g_timeout_ticks, ArSgd{});
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(k_xgmi_allreduce<false>, dim3(pto_ar_blocks(n, world)), dim3(AR_THREADS), 0, s,
                     reinterpret_cast<const ArPeers*>(peers), off, n / 4, rank, world, chan,
                     reinterpret_cast<uint32_t*>(epochs), reinterpret_cast<int*>(err), g_timeout_ticks, ArSgd{});
  return (int)hipGetLastError();
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
  if (n % 4 || off % 4 || world < 1 || world > AR_MAX_RANKS || chan < 0 || chan >= AR_CHANNELS || rank < 0 ||
      rank >= world || !p || !m || !lr || ((((uintptr_t)p) | ((uintptr_t)m)) & 15) || (bidx && nbatches < 1))
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
  if (n <= AR_ONESHOT_MAX) {
    hipLaunchKernelGGL(k_xgmi_allreduce_1shot<true>, dim3((unsigned)((n / 4 + AR_THREADS - 1) / AR_THREADS)),
                       dim3(AR_THREADS), 0, s, reinterpret_cast<const ArPeers*>(peers), off, n / 4, rank, world, chan,
                       reinterpret_cast<uint32_t*>(epochs), reinterpret_cast<int*>(err), g_timeout_ticks, f);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(k_xgmi_allreduce<true>, dim3(pto_ar_blocks(n, world)), dim3(AR_THREADS), 0, s,
                     reinterpret_cast<const ArPeers*>(peers), off, n / 4, rank, world, chan,
                     reinterpret_cast<uint32_t*>(epochs), reinterpret_cast<int*>(err), g_timeout_ticks, f);
  return (int)hipGetLastError();
}
