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
// Small buckets (<= AR_ONESHOT_MAX floats; MNIST's 100 KB conv bucket runs
// the rank-split form of it, ar_role_oneshot_sgd) use a one-shot variant:
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

#include "xgmi_ar.h"

#define PTO_API extern "C" __attribute__((visibility("default")))

namespace {

using namespace pto_ar;

long long g_timeout_ticks = 500 * AR_TICKS_PER_MS;  // pto_ar_set_timeout_ms
int g_protocol = 0;  // pto_ar_set_protocol: 0 coherent (write-through + sc0 sc1 loads), 1 fenced

template <bool SGD, bool FENCED>
__global__ __launch_bounds__(AR_THREADS) void k_xgmi_allreduce(const ArPeers* __restrict__ peers, long long off,
                                                               long long n4, int rank, int world, int chan,
                                                               uint32_t* __restrict__ epochs, int* err, long long timeout,
                                                               ArSgd f) {
  ar_twostage<SGD, FENCED, AR_THREADS>(peers, off, n4, rank, world, chan, epochs, err, timeout, f, blockIdx.x,
                                       gridDim.x);
}

template <bool SGD, bool FENCED>
__global__ __launch_bounds__(AR_THREADS) void k_xgmi_allreduce_1shot(const ArPeers* __restrict__ peers,
                                                                     long long off, long long n4, int rank,
                                                                     int world, int chan,
                                                                     uint32_t* __restrict__ epochs, int* err,
                                                                     long long timeout, ArSgd f) {
  ar_oneshot<SGD, FENCED, AR_THREADS>(peers, off, n4, rank, world, chan, epochs, err, timeout, f, blockIdx.x);
}

// The fc / conv all-reduce roles of the overlapped MNIST step as launches of
// their own: EXACTLY the decompositions of the roles inside the F12 launch
// (1024-thread workgroups, ar_role_sgd / ar_role_oneshot_sgd), so a rank
// that runs a step's exchange stand-alone interoperates with a peer that ran
// the same exchange inside its F12 (block b covers the same elements and
// advances the same epoch either way).
constexpr int AR_ROLE_THREADS = 1024;
template <bool FENCED>
__global__ __launch_bounds__(AR_ROLE_THREADS) void k_xgmi_allreduce_role(const ArPeers* __restrict__ peers, long long off,
                                                                          long long n4, int rank, int world, int chan,
                                                                          uint32_t* __restrict__ epochs, int* err,
                                                                          long long timeout, ArSgd f) {
  __shared__ float4 lds[AR_ROLE_THREADS];
  ar_role_sgd<FENCED, AR_ROLE_THREADS>(peers, off, n4, rank, world, chan, epochs, err, timeout, f, blockIdx.x, lds);
}

template <bool FENCED>
__global__ __launch_bounds__(AR_ROLE_THREADS) void k_xgmi_oneshot_role(const ArPeers* __restrict__ peers, long long off,
                                                                       long long n4, int rank, int world, int chan,
                                                                       uint32_t* __restrict__ epochs, int* err,
                                                                       long long timeout, ArSgd f, int* ready) {
  __shared__ float4 lds[AR_ROLE_THREADS];
  ar_role_oneshot_sgd<FENCED, AR_ROLE_THREADS>(peers, off, n4, rank, world, chan, epochs, err, timeout, f, blockIdx.x,
                                               lds, ready);
}

// ------------------------------------------------------ parameter hash --
// Cross-rank consistency check of a data-parallel run (fused_step.py): a
// 64-bit hash of this rank's parameters, published into the hash ring of
// EVERY rank's flag page, so each rank's host can compare its own hash with
// every peer's for the same sequence number (XgmiAllReduce.check_hashes).
// Replicas updated by the same all-reduced gradient hold bit-identical
// parameters; a lost or stale peer read anywhere shows up as a mismatch.
// The hash is a SUM over 32-bit words of a 64-bit mix of (index, bits), so
// workgroups combine with one 64-bit atomic add each, in any order.  The
// workgroup whose arrival is last (ticket counter; every adder drained its
// atomic first) publishes {seq, hash} -- hash stored, drained, then seq
// stored, so a reader that sees seq also sees the hash -- and re-arms the
// accumulator and the ticket for the next call.
// st: [0] accumulator, [1] ticket, [2] sequence number (int64, zeroed at setup).
__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x += 0x9e3779b97f4a7c15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}
constexpr int HASH_THREADS = 256;
__global__ __launch_bounds__(HASH_THREADS) void k_param_hash(const ArPeers* __restrict__ P, const uint4* __restrict__ p,
                                                             long long n4, int rank, int world,
                                                             unsigned long long* __restrict__ st) {
  __shared__ unsigned long long red[HASH_THREADS / 64];
  __shared__ int s_last;
  unsigned long long h = 0;
  for (long long i = (long long)blockIdx.x * HASH_THREADS + threadIdx.x; i < n4; i += (long long)gridDim.x * HASH_THREADS) {
    const uint4 v = p[i];
    const unsigned long long k = (unsigned long long)i << 34;
    h += mix64(k | v.x) + mix64(k | (1ULL << 32) | v.y) + mix64(k | (2ULL << 32) | v.z) + mix64(k | (3ULL << 32) | v.w);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = 0;
    for (int w = 0; w < HASH_THREADS / 64; ++w) b += red[w];
    atomicAdd(st, b);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the add performed before the ticket
    const unsigned long long old = atomicAdd(st + 1, 1ULL);
    s_last = old == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last || threadIdx.x >= world) return;
  // last arriver: lanes 0..world-1 publish into rank t's page
  const unsigned long long tot = __hip_atomic_load(st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long seq = st[2] + 1;
  const int t = threadIdx.x;
  uint32_t* e = P->flags[t] + AR_FLAG_WORDS + ((int)(seq % AR_HASH_RING) * AR_MAX_RANKS + rank) * 4;
  __hip_atomic_store(G(e + 2), (uint32_t)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(G(e + 3), (uint32_t)(tot >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(G(e + 1), (uint32_t)(seq >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(G(e + 0), (uint32_t)seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (t == 0) {
    st[0] = 0;
    st[1] = 0;
    st[2] = seq;
  }
}

template <bool FENCED>
__global__ __launch_bounds__(AR_THREADS) void k_xgmi_allreduce_bf16(const ArPeers* __restrict__ peers, long long off,
                                                                    long long nv, int rank, int world, int chan,
                                                                    uint32_t* __restrict__ epochs, int* err,
                                                                    long long timeout) {
  ar_twostage_bf16<FENCED, AR_THREADS>(peers, off, nv, rank, world, chan, epochs, err, timeout, blockIdx.x,
                                       gridDim.x);
}

template <bool FENCED>
__global__ __launch_bounds__(AR_THREADS) void k_xgmi_allreduce_bf16_1shot(const ArPeers* __restrict__ peers,
                                                                          long long off, long long nv, int rank,
                                                                          int world, int chan,
                                                                          uint32_t* __restrict__ epochs, int* err,
                                                                          long long timeout) {
  ar_oneshot_bf16<FENCED, AR_THREADS>(peers, off, nv, rank, world, chan, epochs, err, timeout, blockIdx.x);
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
PTO_API int pto_ar_flag_bytes(int) { return AR_PAGE_WORDS * (int)sizeof(uint32_t); }
PTO_API int pto_ar_hash_offset_words() { return AR_FLAG_WORDS; }
PTO_API int pto_ar_hash_ring() { return AR_HASH_RING; }
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
PTO_API long long pto_ar_timeout_ticks() { return g_timeout_ticks; }

// Flags: uncached device memory, zeroed.
PTO_API int pto_ar_alloc_flags(void** out) {
  // (ordinary device memory measured the same barrier latency at world 1:
  // profiles/exchange_r5.md)
  hipError_t e = hipExtMallocWithFlags(out, (size_t)AR_PAGE_WORDS * sizeof(uint32_t), hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*out, 0, (size_t)AR_PAGE_WORDS * sizeof(uint32_t));
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

// Publish a 64-bit hash of n floats at p (16-byte aligned, n % 4 == 0) into
// every rank's hash ring (k_param_hash).  st: 3 zeroed int64 of this rank.
PTO_API int pto_ar_param_hash(const void* peers, const float* p, long long n, int rank, int world, void* st,
                              hipStream_t s) {
  if (!peers || !p || !st || n % 4 || n <= 0 || (((uintptr_t)p) & 15) || world < 1 || world > AR_MAX_RANKS ||
      rank < 0 || rank >= world)
    return -1;
  const long long n4 = n / 4;
  const long long nb_need = (n4 + HASH_THREADS - 1) / HASH_THREADS;
  const int nb = (int)(nb_need < 64 ? nb_need : 64);
  hipLaunchKernelGGL(k_param_hash, dim3(nb), dim3(HASH_THREADS), 0, s, reinterpret_cast<const ArPeers*>(peers),
                     reinterpret_cast<const uint4*>(p), n4, rank, world,
                     reinterpret_cast<unsigned long long*>(st));
  return (int)hipGetLastError();
}

// Copy nwords 32-bit words of device memory (e.g. this rank's flag page)
// into host memory (synchronous).
PTO_API int pto_ar_read_words(const void* src, void* dst, long long nwords) {
  return (int)hipMemcpy(dst, src, (size_t)nwords * 4, hipMemcpyDeviceToHost);
}
// The same, queued on stream s (dst: pinned host memory).
PTO_API int pto_ar_read_words_async(const void* src, void* dst, long long nwords, hipStream_t s) {
  return (int)hipMemcpyAsync(dst, src, (size_t)nwords * 4, hipMemcpyDeviceToHost, s);
}

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

// In-place SUM all-reduce of n bf16 values at element offset `off` of the
// registered (bf16) input buffers: n % 8 == 0, off % 8 == 0.  A range of at
// most AR_ONESHOT_MAX * 2 bf16 (the same 256 KB) takes the one-shot path.
PTO_API int pto_ar_allreduce_bf16(const void* peers, long long off, long long n, int rank, int world, int chan,
                                  void* epochs, void* err, hipStream_t s) {
  if (n % 8 || off % 8 || n > 2 * AR_MAX_FLOATS || world < 1 || world > AR_MAX_RANKS || chan < 0 ||
      chan >= AR_CHANNELS || rank < 0 || rank >= world)
    return -1;
  if (n == 0) return 0;
  const ArPeers* P = reinterpret_cast<const ArPeers*>(peers);
  uint32_t* ep = reinterpret_cast<uint32_t*>(epochs);
  int* er = reinterpret_cast<int*>(err);
  const long long nv = n / 8;
  if (n <= 2 * AR_ONESHOT_MAX) {
    const dim3 g((unsigned)((nv + AR_THREADS - 1) / AR_THREADS));
    if (g_protocol)
      hipLaunchKernelGGL(HIP_KERNEL_NAME(k_xgmi_allreduce_bf16_1shot<true>), g, dim3(AR_THREADS), 0, s, P, off, nv,
                         rank, world, chan, ep, er, g_timeout_ticks);
    else
      hipLaunchKernelGGL(HIP_KERNEL_NAME(k_xgmi_allreduce_bf16_1shot<false>), g, dim3(AR_THREADS), 0, s, P, off, nv,
                         rank, world, chan, ep, er, g_timeout_ticks);
    return (int)hipGetLastError();
  }
  // as many workgroups as the fp32 path uses for the same bytes
  const dim3 g((unsigned)blocks_for(n / 2, world));
  if (g_protocol)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_xgmi_allreduce_bf16<true>), g, dim3(AR_THREADS), 0, s, P, off, nv, rank,
                       world, chan, ep, er, g_timeout_ticks);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_xgmi_allreduce_bf16<false>), g, dim3(AR_THREADS), 0, s, P, off, nv, rank,
                       world, chan, ep, er, g_timeout_ticks);
  return (int)hipGetLastError();
}

// Stand-alone launch of the all-reduce-with-SGD ROLE (same arguments as
// the fc role of pto_conv12_fwd_ar, same workgroup decomposition).
PTO_API int pto_ar_role_sgd(const void* peers, long long off, long long n, int rank, int world, int chan, void* epochs,
                            void* err, int protocol, float* p, float* m, const float* lr, float mom, float wd,
                            float gscale, int nesterov, long long zero_from, hipStream_t s) {
  if (n <= AR_ONESHOT_MAX || n % 4 || off % 4 || n > AR_MAX_FLOATS || world < 1 || world > AR_MAX_RANKS ||
      chan < 0 || chan >= AR_CHANNELS || rank < 0 || rank >= world || !p || !m || !lr || !peers || protocol < 0 ||
      protocol > 1 || ((((uintptr_t)p) | ((uintptr_t)m)) & 15))
    return -1;
  ArSgd f{};
  f.p = p;
  f.m = m;
  f.a.lr = lr;
  f.a.mom = mom;
  f.a.wd = wd;
  f.a.gscale = gscale;
  f.a.nesterov = nesterov;
  f.zero_from = zero_from;
  f.nbatches = 1;
  f.nrep = 1;
  const ArPeers* P = reinterpret_cast<const ArPeers*>(peers);
  const int nb = role_blocks(n, world, AR_ROLE_THREADS);
  if (nb > AR_MAX_BLOCKS) return -1;
  const dim3 g((unsigned)nb);
  if (protocol)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_xgmi_allreduce_role<true>), g, dim3(AR_ROLE_THREADS), 0, s, P, off, n / 4,
                       rank, world, chan, reinterpret_cast<uint32_t*>(epochs), reinterpret_cast<int*>(err),
                       g_timeout_ticks, f);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_xgmi_allreduce_role<false>), g, dim3(AR_ROLE_THREADS), 0, s, P, off, n / 4,
                       rank, world, chan, reinterpret_cast<uint32_t*>(epochs), reinterpret_cast<int*>(err),
                       g_timeout_ticks, f);
  return (int)hipGetLastError();
}

// Stand-alone launch of the conv role (ar_role_oneshot_sgd: one-shot
// all-reduce + SGD of [off, off + n) with the gradient replicas of
// [rep_from, rep_from + rep_stride) at float index rep_base of the registered
// buffer, gradient and replicas zeroed after the second barrier, one add to
// *ready per workgroup) with
// the decomposition it has inside the MNIST forward launch, so a rank that
// closes a step's exchange here pairs block by block with a peer that runs
// it inside its next forward.
PTO_API int pto_ar_oneshot_role_sgd(const void* peers, long long off, long long n, int rank, int world, int chan,
                                    void* epochs, void* err, int protocol, float* p, float* m, const float* lr,
                                    float mom, float wd, float gscale, int nesterov, long long rep_base, int nrep,
                                    int rep_stride, long long rep_from, int* ready, hipStream_t s) {
  if (n > AR_ONESHOT_MAX || n < 4 || n % 4 || off % 4 || world < 1 || world > AR_MAX_RANKS || chan < 0 ||
      chan >= AR_CHANNELS || rank < 0 || rank >= world || !p || !m || !lr || !peers || !ready || protocol < 0 ||
      protocol > 1 || ((((uintptr_t)p) | ((uintptr_t)m)) & 15))
    return -1;
  if (nrep < 1 || nrep > AR_MAX_REP || (nrep > 1 && (rep_stride % 4 || rep_from % 4 || rep_base % 4 ||
                                                      rep_base < off + n || rep_from < off ||
                                                      rep_from + rep_stride > off + n)))
    return -1;
  ArSgd f{};
  f.p = p;
  f.m = m;
  f.a.lr = lr;
  f.a.mom = mom;
  f.a.wd = wd;
  f.a.gscale = gscale;
  f.a.nesterov = nesterov;
  f.zero_from = off;
  f.nbatches = 1;
  f.nrep = nrep;
  f.rep_stride = rep_stride;
  f.rep_from = rep_from;
  f.rep_base = rep_base;
  const ArPeers* P = reinterpret_cast<const ArPeers*>(peers);
  const int nb = oneshot_role_blocks(n, world, AR_ROLE_THREADS);
  if (nb > AR_MAX_BLOCKS) return -1;
  if (protocol)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_xgmi_oneshot_role<true>), dim3(nb), dim3(AR_ROLE_THREADS), 0, s, P, off,
                       n / 4, rank, world, chan, reinterpret_cast<uint32_t*>(epochs), reinterpret_cast<int*>(err),
                       g_timeout_ticks, f, ready);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_xgmi_oneshot_role<false>), dim3(nb), dim3(AR_ROLE_THREADS), 0, s, P, off,
                       n / 4, rank, world, chan, reinterpret_cast<uint32_t*>(epochs), reinterpret_cast<int*>(err),
                       g_timeout_ticks, f, ready);
  return (int)hipGetLastError();
}
PTO_API int pto_ar_oneshot_role_blocks(long long n, int world) { return oneshot_role_blocks(n, world, AR_ROLE_THREADS); }
