// Device side of the xGMI peer all-reduce (protocol, barriers, stages):
// shared by the stand-alone kernels (xgmi_allreduce.hip) and the kernels
// that run an all-reduce as extra workgroups next to their own work (the
// MNIST forward launch of the overlapped multi-GPU step, mnist_kernels.hip).
// The algorithm, the two visibility protocols and the failure semantics are
// described in xgmi_allreduce.hip's header.  Every function takes the
// block's index among the all-reduce's workgroups (`blk` of `nblk`) and the
// workgroup size NT, so the same stages run in a launch of their own or as
// a role inside another kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sgd_f32.h"

// Phase timestamps for the timing probes under tools/probes (which define
// PTO_STAMP before including the kernel sources); nothing in the shipped
// library.
#ifndef PTO_STAMP
#define PTO_STAMP(k) ((void)0)
#define PTO_STAMP_SCOPE()
#endif

namespace pto_ar {

constexpr int AR_MAX_RANKS = 8;
// workgroups per launch: ceil(chunk / AR_THREADS) up to this cap, so every
// thread handles ONE float4 per stage down to world 1-2 on MNIST's 1.7 MB
constexpr int AR_MAX_BLOCKS = 256;
// channels 0 and 1: the stand-alone all-reduces and the fc role of the
// overlapped MNIST step; channel 2: that step's conv role (ar_role_oneshot_sgd)
constexpr int AR_CHANNELS = 3;
constexpr int AR_THREADS = 512;  // workgroup size of the stand-alone kernels
constexpr int AR_MAX_REP = 256;  // gradient replicas folded before barrier 1 (launcher check)
constexpr int AR_REP_CHUNK = 16;  // replica loads in flight at once
// stage-1 sums of this rank's own chunk kept in registers for stage 2 (the
// same thread handles element j of the chunk in both stages): iterations
// beyond this re-read them from tmp
constexpr int AR_CARRY = 4;
constexpr long long AR_ONESHOT_MAX = 65536;  // floats (256 KB): one-shot path
constexpr long long AR_TICKS_PER_MS = 100000LL;  // wall_clock64 runs at 100 MHz

// buffer-instruction cache bits (aux operand): sc0 | sc1 = system scope
constexpr int AUX_SYS = 1 | 16;

// global (not flat) views of generic pointers: flag words and the local
// parameter/momentum/gradient float4 groups
using gu32 = __attribute__((address_space(1))) uint32_t;
using v4f = __attribute__((ext_vector_type(4))) float;
using gv4f = __attribute__((address_space(1))) v4f;
using v4u = __attribute__((ext_vector_type(4))) unsigned int;
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
// parameter-hash ring after the flags (k_param_hash): AR_HASH_RING entries per
// source rank, each {seq lo, seq hi, hash lo, hash hi}; entry (seq % RING) of
// rank q is written by rank q into EVERY rank's page
constexpr int AR_HASH_RING = 4;
constexpr int AR_HASH_WORDS = AR_HASH_RING * AR_MAX_RANKS * 4;
constexpr int AR_PAGE_WORDS = AR_FLAG_WORDS + AR_HASH_WORDS;

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
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), b.r, (int)(i4 * 16), 0, AUX_SYS);
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
// DRAIN = false: no store of this workgroup precedes the barrier (nothing
// to publish), so the arriving lanes do not wait for the workgroup's
// outstanding loads -- e.g. the SGD operands prefetched just before.
// err0 >= 0: the caller's copy of *err (loaded with its other operands at
// entry), so the arriving lanes store their flag without a round trip to
// *err first; a failure of another workgroup since then is still seen in
// the wait loop.
template <bool FENCED, bool DRAIN = true>
__device__ __forceinline__ bool block_barrier(const ArPeers* __restrict__ P, int chan, int phase, int b, int rank,
                                              int world, uint32_t e, long long timeout, int* err, int err0 = -1) {
  __shared__ int s_fail[2];
  const int t = threadIdx.x;
  if (t == 0) s_fail[phase] = 0;
  if constexpr (DRAIN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave: its stores acknowledged
  __syncthreads();
  if (t < world) {
    bool dead = (err0 >= 0 ? err0 : __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0;
    if (!dead) {
      if constexpr (FENCED) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: write back this XCD's L2
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_store(G(P->flags[t] + flag_index(chan, phase, b, rank)), e, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      gu32* f = G(P->flags[rank] + flag_index(chan, phase, b, t));
      const long long t0 = wall_clock64();
      for (;;) {
        // the flag and the error word in flight together: one round trip
        // per poll
        const uint32_t v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const int ev = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v == e) break;
        // another block (or an earlier launch) already gave up: stop now
        if (ev != 0) {
          dead = true;
          break;
        }
        if (wall_clock64() - t0 > timeout) {
          atomicOr(err, 1 << phase);
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

// The waiting half of a barrier whose arrival was an atomic INCREMENT of
// every peer's flag slot (not a store of the epoch): the arrival needs no
// epoch and no error word, so it goes out at workgroup entry; the slot's
// count equals the epoch as long as every call of the channel arrives this
// way.  Lanes < world poll their source's slot until it reaches e.
template <bool FENCED>
__device__ __forceinline__ bool block_wait(const ArPeers* __restrict__ P, int chan, int phase, int b, int rank,
                                           int world, uint32_t e, long long timeout, int* err) {
  __shared__ int s_failw;
  const int t = threadIdx.x;
  if (t == 0) s_failw = 0;
  __syncthreads();
  if (t < world) {
    bool dead = false;
    gu32* f = G(P->flags[rank] + flag_index(chan, phase, b, t));
    const long long t0 = wall_clock64();
    for (;;) {
      const uint32_t v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const int ev = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v == e) break;
      if (ev != 0) {
        dead = true;
        break;
      }
      if (wall_clock64() - t0 > timeout) {
        atomicOr(err, 1 << phase);
        dead = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if constexpr (FENCED) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (dead) s_failw = 1;
  }
  __syncthreads();
  return s_failw == 0;
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
  // ar_role_oneshot_sgd: the replicas live in the registered buffer itself,
  // replica 1 at this float index (peers read them; `rep` is unused)
  long long rep_base;
};

// Fold the local replicas into float4 element i4 (float offset 4*i4 from the
// buffer base) of the local gradient, if it lies in the replicated range.
// Every replica load is issued before the first add; the folded value is
// stored through `g` (write-through under the coherent protocol: peers read
// it).
// CHUNK: replica loads in flight at once (a role inside a 64-VGPR kernel
// uses 8: the MNIST step's 7 extra replicas in one round, 32 VGPRs).
template <bool COHERENT, int CHUNK = AR_REP_CHUNK>
__device__ __forceinline__ void fold_rep(const ArSgd& f, const Buf& g, long long off, long long i4) {
  const long long fi = off + 4 * i4;  // float index in the whole buffer (rep_from's frame)
  if (!f.rep || f.nrep <= 1 || fi < f.rep_from || fi >= f.rep_from + f.rep_stride) return;
  const long long k = fi - f.rep_from;
  float4 a = gld4(g.p + 4 * i4);
  for (int r0 = 0; r0 < f.nrep - 1; r0 += CHUNK) {  // replica order
    float4 v[CHUNK];
#pragma unroll
    for (int r = 0; r < CHUNK; ++r)
      v[r] = gld4(f.rep + (long long)min(r0 + r, f.nrep - 2) * f.rep_stride + k);
#pragma unroll
    for (int r = 0; r < CHUNK; ++r) {
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
// Workgroup `blk` of the `nblk` that run it, NT threads each.  LEAN: the
// register-light form for a role inside a register-capped kernel (no
// gradient replicas, no register carry of the own chunk, one rank's float4
// in flight at a time in stage 2).
template <bool SGD, bool FENCED, int NT, bool LEAN = false>
__device__ __forceinline__ void ar_twostage(const ArPeers* __restrict__ peers, long long off, long long n4, int rank,
                                            int world, int chan, uint32_t* __restrict__ epochs, int* err,
                                            long long timeout, const ArSgd& f, int blk, int nblk) {
  constexpr bool CO = !FENCED;
  __shared__ uint32_t s_epoch;
  const ArPeers* __restrict__ P = peers;
  if (threadIdx.x == 0) s_epoch = epochs[chan * AR_MAX_BLOCKS + blk] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  if (threadIdx.x == 0) epochs[chan * AR_MAX_BLOCKS + blk] = e;
  const long long cs = (n4 + world - 1) / world;  // chunk length (float4)
  const long long stride = (long long)nblk * NT;
  const long long j0 = (long long)blk * NT + threadIdx.x;
  const long long bytes = n4 * 16;
  float* const my_in = P->in[rank];
  constexpr int CARRY = LEAN ? 0 : AR_CARRY;
  if constexpr (!LEAN) {
    if (f.rep && f.nrep > 1 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      // the elements this workgroup's peers will read: the same sub-range of every chunk
      const Buf g = mkbuf(my_in + off, bytes);
      for (int q = 0; q < world; ++q)
        for (long long j = j0; j < cs && q * cs + j < n4; j += stride) fold_rep<CO>(f, g, off, q * cs + j);
    }
  }

  if (!block_barrier<FENCED>(P, chan, 0, blk, rank, world, e, timeout, err)) return;
  // stage 1: reduce my chunk over all ranks (rank order 0..W-1 everywhere);
  // the first CARRY iterations' sums stay in registers for stage 2, tmp
  // gets them only if a peer (or a later iteration) reads them
  float4 own[CARRY > 0 ? CARRY : 1];
  {
    const long long c0 = (long long)rank * cs, c1 = min(n4, c0 + cs);
    int it = 0;
    for (long long i = c0 + j0; i < c1; i += stride, ++it) {
      float4 a;
      if constexpr (LEAN) {
        // up to 4 ranks' loads in flight at once (a rank-by-rank chain would
        // pay one cross-GPU round trip per rank), summed in rank order
        a = ld4<CO>(mkbuf(P->in[0] + off, bytes), i);
#pragma unroll
        for (int q0 = 1; q0 < AR_MAX_RANKS; q0 += 2) {
          float4 v[2];
#pragma unroll
          for (int k = 0; k < 2; ++k)
            if (q0 + k < world) v[k] = ld4<CO>(mkbuf(P->in[q0 + k] + off, bytes), i);
#pragma unroll
          for (int k = 0; k < 2; ++k)
            if (q0 + k < world) a = add4(a, v[k]);
        }
      } else {
        float4 v[AR_MAX_RANKS];
#pragma unroll
        for (int q = 0; q < AR_MAX_RANKS; ++q)
          if (q < world) v[q] = ld4<CO>(mkbuf(P->in[q] + off, bytes), i);
        a = v[0];
#pragma unroll
        for (int q = 1; q < AR_MAX_RANKS; ++q)
          if (q < world) a = add4(a, v[q]);
      }
#pragma unroll
      for (int c = 0; c < CARRY; ++c)
        if (c == it) own[c] = a;
      if (world > 1 || it >= CARRY) st4<CO>(mkbuf(P->tmp[rank] + off, bytes), i, a);
    }
  }
  const float lr = SGD ? *f.a.lr : 0.f;
  if (!block_barrier<FENCED>(P, chan, 1, blk, rank, world, e, timeout, err)) return;
  // stage 2: gather every chunk into my input (or: update my parameters)
  if constexpr (LEAN) {
    // one rank's chunk element per round (the register cap of the host
    // kernel); its peer load and the local p/m loads go out together
    for (long long j = j0; j < cs; j += stride)
      for (int q = 0; q < world; ++q) {
        const long long k = q * cs + j;
        if (k >= n4) break;
        const float4 v = ld4<CO>(mkbuf(P->tmp[q] + off, bytes), k);
        if constexpr (SGD) {
          const long long i = off + 4 * k;
          float4 pv = gld4(f.p + i);
          float4 mv = gld4(f.m + i);
          sgd4(f, i, v, pv, mv, lr);
          if (i >= f.zero_from) gst4(my_in + i, float4{0.f, 0.f, 0.f, 0.f});
        } else {
          gst4(my_in + off + 4 * k, v);
        }
      }
    if (SGD && f.bidx && blk == 0 && threadIdx.x == 0) *f.bidx = (*f.bidx + 1) % f.nbatches;
    return;
  }
  int it = 0;
  for (long long j = j0; j < cs; j += stride, ++it) {
    float4 v[AR_MAX_RANKS];
#pragma unroll
    for (int q = 0; q < AR_MAX_RANKS; ++q)
      if (q < world && (long long)q * cs + j < n4) {
        if (q == rank && it < CARRY) {
#pragma unroll
          for (int c = 0; c < CARRY; ++c)
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
  if (SGD && f.bidx && blk == 0 && threadIdx.x == 0) *f.bidx = (*f.bidx + 1) % f.nbatches;
}

// One-shot variant: n4 <= nblk * NT (one float4 per thread).
template <bool SGD, bool FENCED, int NT>
__device__ __forceinline__ void ar_oneshot(const ArPeers* __restrict__ peers, long long off, long long n4, int rank,
                                           int world, int chan, uint32_t* __restrict__ epochs, int* err,
                                           long long timeout, const ArSgd& f, int blk) {
  constexpr bool CO = !FENCED;
  __shared__ uint32_t s_epoch;
  const ArPeers* __restrict__ P = peers;
  if (threadIdx.x == 0) s_epoch = epochs[chan * AR_MAX_BLOCKS + blk] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  if (threadIdx.x == 0) epochs[chan * AR_MAX_BLOCKS + blk] = e;
  const long long i = (long long)blk * NT + threadIdx.x;
  const bool act = i < n4;
  const long long bytes = n4 * 16;
  float* const my_in = P->in[rank];
  // the SGD epilogue's local operands (parameters, momentum, lr: nobody
  // else writes them during the launch) are loaded before the barrier, so
  // after it only the peer loads stand between the flag and the update
  float4 pv = {0.f, 0.f, 0.f, 0.f}, mv = {0.f, 0.f, 0.f, 0.f};
  float lr = 0.f;
  if constexpr (SGD) {
    if (act) {
      pv = gld4(f.p + off + 4 * i);
      mv = gld4(f.m + off + 4 * i);
    }
    lr = *f.a.lr;
  }
  if (act && f.rep && f.nrep > 1 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
    fold_rep<CO>(f, mkbuf(my_in + off, bytes), off, i);
  if (!block_barrier<FENCED>(P, chan, 0, blk, rank, world, e, timeout, err)) return;
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
  if (!block_barrier<FENCED>(P, chan, 1, blk, rank, world, e, timeout, err)) return;
  if (act) {
    if constexpr (SGD) {
      const long long j = off + 4 * i;
      sgd4(f, j, a, pv, mv, lr);
      if (j >= f.zero_from) gst4(my_in + j, float4{0.f, 0.f, 0.f, 0.f});
    } else {
      gst4(my_in + off + 4 * i, a);
    }
  }
  if (SGD && f.bidx && blk == 0 && threadIdx.x == 0) *f.bidx = (*f.bidx + 1) % f.nbatches;
}

// ------------------------------------------------------- rank-split role --
// The all-reduce + SGD as a ROLE inside a register-capped kernel (the MNIST
// forward launch, <= 64 VGPRs): every thread has exactly ONE float4 in
// flight per stage, whatever the world size, because the block's NT threads
// are split into W groups of S = NT / W, group q handling rank q:
//   stage 1  thread (q, s) loads rank q's element s of this block's
//            sub-range of MY chunk into LDS; the first S threads sum the W
//            values in rank order (only this rank computes its chunk's sum,
//            so the order is fixed) and store it write-through into tmp;
//   stage 2  thread (q, s) loads element s of the sub-range of chunk q from
//            rank q's tmp, applies SGD to the local parameter/momentum.
// Block b covers sub-range [b*S, b*S + S) of every chunk on every rank (the
// pairing the per-block barriers rely on), so nblk = ceil(chunk / S) ~ n4 /
// NT blocks at any W -- more blocks, not more serial rounds, as W grows.
// lds: NT float4 of scratch.  No replica fold, no cursor.
__host__ __device__ inline int role_blocks(long long n, int world, int nt) {
  const long long cs = ((n / 4) + world - 1) / world, S = nt / world;
  return (int)((cs + S - 1) / S);
}
template <bool FENCED, int NT>
__device__ __forceinline__ void ar_role_sgd(const ArPeers* __restrict__ P, long long off, long long n4, int rank,
                                            int world, int chan, uint32_t* __restrict__ epochs, int* err,
                                            long long timeout, const ArSgd& f, int blk, float4* lds) {
  constexpr bool CO = !FENCED;
  __shared__ uint32_t s_epoch;
  if (threadIdx.x == 0) s_epoch = epochs[chan * AR_MAX_BLOCKS + blk] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  if (threadIdx.x == 0) epochs[chan * AR_MAX_BLOCKS + blk] = e;
  const long long cs = (n4 + world - 1) / world;
  const int S = NT / world;
  const int q = threadIdx.x / S, sidx = threadIdx.x - q * S;
  const bool in_group = q < world;
  const long long j = (long long)blk * S + sidx;  // element of every chunk this thread covers
  const long long bytes = n4 * 16;
  // barrier 0: every peer's input is complete (its backward has ended) and
  // every peer has finished its previous call of this role, including the
  // stage-2 reads of tmp that stage 1 below overwrites.  (Round 4 skipped it
  // under the coherent protocol because a stand-alone conv exchange always
  // preceded this role; the conv exchange now runs NEXT TO it, as
  // ar_role_oneshot_sgd in the same launch, so nothing else orders it.)
  // Nothing is stored before it: no drain, and *err was read at entry.
  const int err0 = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!block_barrier<FENCED, false>(P, chan, 0, blk, rank, world, e, timeout, err, err0)) return;
  // stage 1: my chunk's element j from rank q -> LDS, then rank-order sums
  const long long i1 = (long long)rank * cs + j;
  const bool v1 = in_group && j < cs && i1 < n4;
  if (v1) lds[q * S + sidx] = ld4<CO>(mkbuf(P->in[q] + off, bytes), i1);
  __syncthreads();
  if (q == 0 && v1) {
    float4 a = lds[sidx];
    for (int r = 1; r < world; ++r) a = add4(a, lds[r * S + sidx]);
    st4<CO>(mkbuf(P->tmp[rank] + off, bytes), i1, a);
  }
  const float lr = *f.a.lr;
  // stage 2's local SGD operands before the barrier (only this thread
  // writes them), so after it only the peer load is on the chain
  const long long k = (long long)q * cs + j;
  const bool v2 = in_group && j < cs && k < n4;
  float4 pv = {0.f, 0.f, 0.f, 0.f}, mv = {0.f, 0.f, 0.f, 0.f};
  if (v2) {
    pv = gld4(f.p + off + 4 * k);
    mv = gld4(f.m + off + 4 * k);
  }
  if (!block_barrier<FENCED>(P, chan, 1, blk, rank, world, e, timeout, err)) return;
  // stage 2: element j of chunk q from rank q's partial sums
  if (v2) {
    const float4 v = ld4<CO>(mkbuf(P->tmp[q] + off, bytes), k);
    const long long i = off + 4 * k;
    sgd4(f, i, v, pv, mv, lr);
    if (i >= f.zero_from) gst4(P->in[rank] + i, float4{0.f, 0.f, 0.f, 0.f});
  }
}

// ------------------------------------------------ one-shot rank-split role --
// The conv exchange of the overlapped MNIST step (<= AR_ONESHOT_MAX floats:
// conv2 + conv1, 100 KB) as a ROLE of the NEXT step's forward launch, whose
// conv workgroups wait on `ready` before they read the parameters it
// updates -- so the exchange no longer costs a launch of its own between the
// backward and that forward (fused_step.py, "ddp-xgmi" overlap).
// Register-light like ar_role_sgd (the host kernel is capped at 64 VGPRs):
// the block's NT threads are W groups of S = NT / W; block b covers float4
// groups [b*S, b*S + S) of the range on every rank (same pairing on every
// rank), and thread (q, s) reads rank q's group s.  Per workgroup:
//   barrier 0  every peer's backward has ended (its gradient is complete).
//              Nothing of this call precedes it, so the lanes arrive at
//              workgroup entry by an atomic increment of every peer's slot
//              (no drain, no epoch read first) and wait while the epoch and
//              the SGD operands are being loaded.
//   stage 1    thread (q, s) loads rank q's gradient group and, inside the
//              replicated range (rep_off: the gradient replicas of the
//              backward's atomics live in the SAME registered buffer, replica
//              r >= 1 at rep_off + (r-1)*rep_stride), rank q's replicas,
//              summed in replica order -- no local fold store and no drain
//              before the barrier; q = 0 sums the W values in rank order
//              (bit-identical on every rank), applies SGD, stores the
//              parameter WRITE-THROUGH (system scope: the waiting conv
//              workgroups on other XCDs read it with system-scope loads; no
//              L2 of this XCD keeps a stale copy) and the momentum plainly
//              (only the next launch reads it)
//   publish    every wave drains its stores (vmcnt 0), workgroup barrier,
//              ONE agent-scope add to *ready.  Done on failure too (nothing
//              was written then and *err is set), so the waiting conv
//              workgroups are always released and the grid drains.
//   barrier 1  every peer has read this rank's gradient and replicas
//   q = 0      zero this rank's gradient group and its replicas: the next
//              backward accumulates into them (a run() ends with zero conv
//              gradients)
// Hazards: a rank writes its gradient range and replicas only after
// barrier 1 (every peer's stage-1 read of this call is done).  The conv
// workgroups read the updated parameters only after *ready counts every
// role workgroup; the next writer of those parameters is the next call of
// this role, a later launch.  *ready is reset by a later launch of the same
// step (the MNIST F4dx launch).
template <bool FENCED, int NT>
__device__ __forceinline__ void ar_role_oneshot_sgd(const ArPeers* __restrict__ P, long long off, long long n4,
                                                    int rank, int world, int chan, uint32_t* __restrict__ epochs,
                                                    int* err, long long timeout, const ArSgd& f, int blk,
                                                    float4* lds, int* ready) {
  constexpr bool CO = !FENCED;
  // barrier 0 arrival first thing: nothing of this call precedes it (the
  // gradient it announces was written by the previous launch), so no drain,
  // no epoch and no error word are needed to send it (block_wait).  A rank
  // whose exchange already failed still announces its raw gradient; it is
  // absent from barrier 1, where its peers then fail too.
  if (threadIdx.x < world)
    __hip_atomic_fetch_add(G(P->flags[threadIdx.x] + flag_index(chan, 0, blk, rank)), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  __shared__ uint32_t s_epoch;
  if (threadIdx.x == 0) s_epoch = epochs[chan * AR_MAX_BLOCKS + blk] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  if (threadIdx.x == 0) epochs[chan * AR_MAX_BLOCKS + blk] = e;
  const int S = NT / world;
  const int q = threadIdx.x / S, sidx = threadIdx.x - q * S;
  const long long j = (long long)blk * S + sidx;
  const bool valid = q < world && j < n4;
  const bool own = q == 0 && valid;  // this thread updates element group j
  // replicated range: [f.rep_from, f.rep_from + rep_stride) (float index)
  const long long fi = off + 4 * j;
  const bool repl = valid && f.nrep > 1 && fi >= f.rep_from && fi < f.rep_from + f.rep_stride;
  const long long rep_base = f.rep_base;
  const long long span = f.nrep > 1 ? rep_base + (long long)(f.nrep - 1) * f.rep_stride : off + 4 * n4;
  float4 pv = {0.f, 0.f, 0.f, 0.f}, mv = {0.f, 0.f, 0.f, 0.f};
  float lr = 0.f;
  if (own) {
    pv = gld4(f.p + fi);
    mv = gld4(f.m + fi);
    lr = *f.a.lr;
  }
  const bool ok = block_wait<FENCED>(P, chan, 0, blk, rank, world, e, timeout, err);
  PTO_STAMP(1);
  if (ok) {
    if (valid) {
      const Buf g = mkbuf(P->in[q], span * 4);
      float4 a = ld4<CO>(g, fi / 4);
      if (repl) {
        const long long k4 = (rep_base + (fi - f.rep_from)) / 4, st4 = f.rep_stride / 4;
        for (int r0 = 0; r0 < f.nrep - 1; r0 += 8) {  // replica order, 8 loads in flight
          float4 v[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] = ld4<CO>(g, k4 + (long long)min(r0 + r, f.nrep - 2) * st4);
#pragma unroll
          for (int r = 0; r < 8; ++r)
            if (r0 + r < f.nrep - 1) a = add4(a, v[r]);
        }
      }
      lds[q * S + sidx] = a;
    }
    __syncthreads();
    if (own) {
      float4 a = lds[sidx];
      for (int r = 1; r < world; ++r) a = add4(a, lds[r * S + sidx]);
      sgd_elem(pv.x, a.x, mv.x, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
      sgd_elem(pv.y, a.y, mv.y, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
      sgd_elem(pv.z, a.z, mv.z, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
      sgd_elem(pv.w, a.w, mv.w, lr, f.a.mom, f.a.wd, f.a.gscale, f.a.nesterov);
      st4<true>(mkbuf(f.p + off, n4 * 16), j, pv);
      gst4(f.m + fi, mv);
    }
  }
  PTO_STAMP(2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave: its parameter stores acknowledged
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  PTO_STAMP(3);
  if (!ok) return;
  if (!block_barrier<FENCED>(P, chan, 1, blk, rank, world, e, timeout, err)) return;
  PTO_STAMP(4);
  if (own) {
    float* const my = P->in[rank];
    gst4(my + fi, float4{0.f, 0.f, 0.f, 0.f});
    if (repl)
      for (int r = 0; r < f.nrep - 1; ++r)
        gst4(my + rep_base + (long long)r * f.rep_stride + (fi - f.rep_from), float4{0.f, 0.f, 0.f, 0.f});
  }
}
__host__ __device__ inline int oneshot_role_blocks(long long n, int world, int nt) {
  const long long S = nt / world;
  return (int)(((n / 4) + S - 1) / S);
}

// ---------------------------------------------------------------- bf16 --
// Plain SUM all-reduce of bf16 gradient buckets (the large-model DDP comm
// hook, parallel/ddp.py): 16-byte vectors of 8 bf16, summed in fp32 in rank
// order and rounded to bf16 once (stage 1 / the one-shot sum), so every rank
// ends with bit-identical values.  Same barriers, protocols and failure
// semantics as the fp32 path; no optimizer epilogue.
struct F8 {
  float v[8];
};
__device__ __forceinline__ F8 bf16x8_to_f32(v4u x) {
  F8 r;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    r.v[2 * k] = __uint_as_float(x[k] << 16);
    r.v[2 * k + 1] = __uint_as_float(x[k] & 0xffff0000u);
  }
  return r;
}
__device__ __forceinline__ uint32_t f32_to_bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  if (f != f) return 0x7fc0u;  // NaN stays a quiet NaN
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ v4u f32_to_bf16x8(const F8& a) {
  v4u r;
#pragma unroll
  for (int k = 0; k < 4; ++k) r[k] = f32_to_bf16_rne(a.v[2 * k]) | (f32_to_bf16_rne(a.v[2 * k + 1]) << 16);
  return r;
}
template <bool COHERENT>
__device__ __forceinline__ v4u ldv(const Buf& b, long long i) {
  if constexpr (COHERENT) return __builtin_amdgcn_raw_buffer_load_b128(b.r, (int)(i * 16), 0, AUX_SYS);
  else return reinterpret_cast<const v4u*>(b.p)[i];
}
template <bool COHERENT>
__device__ __forceinline__ void stv(const Buf& b, long long i, v4u v) {
  if constexpr (COHERENT) __builtin_amdgcn_raw_buffer_store_b128(v, b.r, (int)(i * 16), 0, AUX_SYS);
  else reinterpret_cast<v4u*>(b.p)[i] = v;
}
// byte-offset view of a registered buffer (`off` in elements of `esize` bytes)
__device__ __forceinline__ float* at(float* base, long long off, int esize) {
  return reinterpret_cast<float*>(reinterpret_cast<char*>(base) + off * esize);
}
// nv vectors of 8 bf16 starting at element `off` of every rank's buffers.
template <bool FENCED, int NT>
__device__ __forceinline__ void ar_twostage_bf16(const ArPeers* __restrict__ P, long long off, long long nv, int rank,
                                                 int world, int chan, uint32_t* __restrict__ epochs, int* err,
                                                 long long timeout, int blk, int nblk) {
  constexpr bool CO = !FENCED;
  __shared__ uint32_t s_epoch;
  if (threadIdx.x == 0) s_epoch = epochs[chan * AR_MAX_BLOCKS + blk] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  if (threadIdx.x == 0) epochs[chan * AR_MAX_BLOCKS + blk] = e;
  const long long cs = (nv + world - 1) / world;
  const long long stride = (long long)nblk * NT;
  const long long j0 = (long long)blk * NT + threadIdx.x;
  const long long bytes = nv * 16;
  if (!block_barrier<FENCED>(P, chan, 0, blk, rank, world, e, timeout, err)) return;
  {
    const long long c0 = (long long)rank * cs, c1 = min(nv, c0 + cs);
    for (long long i = c0 + j0; i < c1; i += stride) {
      v4u raw[AR_MAX_RANKS];
#pragma unroll
      for (int q = 0; q < AR_MAX_RANKS; ++q)
        if (q < world) raw[q] = ldv<CO>(mkbuf(at(P->in[q], off, 2), bytes), i);
      F8 a = bf16x8_to_f32(raw[0]);
#pragma unroll
      for (int q = 1; q < AR_MAX_RANKS; ++q)
        if (q < world) {
          const F8 b = bf16x8_to_f32(raw[q]);
#pragma unroll
          for (int k = 0; k < 8; ++k) a.v[k] += b.v[k];
        }
      stv<CO>(mkbuf(at(P->tmp[rank], off, 2), bytes), i, f32_to_bf16x8(a));
    }
  }
  if (!block_barrier<FENCED>(P, chan, 1, blk, rank, world, e, timeout, err)) return;
  float* const my_in = at(P->in[rank], off, 2);
  for (long long j = j0; j < cs; j += stride) {
    v4u v[AR_MAX_RANKS];
#pragma unroll
    for (int q = 0; q < AR_MAX_RANKS; ++q)
      if (q < world && (long long)q * cs + j < nv) v[q] = ldv<CO>(mkbuf(at(P->tmp[q], off, 2), bytes), q * cs + j);
#pragma unroll
    for (int q = 0; q < AR_MAX_RANKS; ++q)
      if (q < world && (long long)q * cs + j < nv) reinterpret_cast<v4u*>(my_in)[q * cs + j] = v[q];
  }
}

// One-shot variant: nv <= nblk * NT (one vector per thread).
template <bool FENCED, int NT>
__device__ __forceinline__ void ar_oneshot_bf16(const ArPeers* __restrict__ P, long long off, long long nv, int rank,
                                                int world, int chan, uint32_t* __restrict__ epochs, int* err,
                                                long long timeout, int blk) {
  constexpr bool CO = !FENCED;
  __shared__ uint32_t s_epoch;
  if (threadIdx.x == 0) s_epoch = epochs[chan * AR_MAX_BLOCKS + blk] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  if (threadIdx.x == 0) epochs[chan * AR_MAX_BLOCKS + blk] = e;
  const long long i = (long long)blk * NT + threadIdx.x;
  const bool act = i < nv;
  const long long bytes = nv * 16;
  if (!block_barrier<FENCED>(P, chan, 0, blk, rank, world, e, timeout, err)) return;
  F8 a{};
  if (act) {
    v4u raw[AR_MAX_RANKS];
#pragma unroll
    for (int q = 0; q < AR_MAX_RANKS; ++q)
      if (q < world) raw[q] = ldv<CO>(mkbuf(at(P->in[q], off, 2), bytes), i);
    a = bf16x8_to_f32(raw[0]);
#pragma unroll
    for (int q = 1; q < AR_MAX_RANKS; ++q)
      if (q < world) {
        const F8 b = bf16x8_to_f32(raw[q]);
#pragma unroll
        for (int k = 0; k < 8; ++k) a.v[k] += b.v[k];
      }
  }
  if (!block_barrier<FENCED>(P, chan, 1, blk, rank, world, e, timeout, err)) return;
  if (act) reinterpret_cast<v4u*>(at(P->in[rank], off, 2))[i] = f32_to_bf16x8(a);
}

// Workgroups of NT threads an all-reduce of n floats uses (identical on every
// rank: derived from n, W).
__host__ __device__ inline int blocks_for(long long n, int world, int nt = AR_THREADS) {
  if (n <= AR_ONESHOT_MAX) return (int)((n / 4 + nt - 1) / nt);
  const long long cs = ((n / 4) + world - 1) / world;
  long long b = (cs + nt - 1) / nt;
  if (b < 1) b = 1;
  if (b > AR_MAX_BLOCKS) b = AR_MAX_BLOCKS;
  return (int)b;
}

}  // namespace pto_ar
