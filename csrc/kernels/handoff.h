// In-launch hand-off of a BatchNorm finalize to the apply blocks of the same grid.
//
// Why: a BatchNorm finalize (per-channel partials -> coefficients) is a few KB of reading and a
// few hundred flops, yet as its own kernel it costs ~7 us of a training step (launch, ramp and the
// dependency boundary on both sides; bench/ab_step.py arm bn_set_skip_finalize:1 measured 0.65 ms
// over ResNet-50's 89 finalizes).  Fused, the finalize runs in the first blocks of the apply
// kernel's grid and the apply blocks wait for its coefficients inside the launch.
//
// Protocol (MI355X guide §6 Guideline 16, form R2: the data IS the flag):
//   * every handed-off coefficient travels as an 8-byte granule {tag = 1, fp32 bits}, written
//     by ONE aligned 8-byte write-through store (relaxed agent-scope atomic store = sc1); no
//     counter, no fence (a counter every block touches serialises at ~45 ns per block - measured:
//     +70-120 us per launch);
//   * blocks [0, nfin) are the finalize blocks; every other block of the grid reads the granules
//     its coefficients need ONCE per block (relaxed agent-scope 8-byte loads = sc1, L1-bypassing;
//     tag and value arrive in one load, so nothing can be stale) and stages them in LDS;
//   * the apply grid keeps its full size (capping it to what is co-resident with the finalize
//     blocks measured slower than the launch it saves), so correctness may not rest on dispatch
//     order: a block whose wait exceeds kHelpPolls runs the finalize items itself ("helping").
//     The finalize of an item is deterministic, so every block that runs it stores the same
//     coefficients (idempotent); the one read-modify-write side effect - the forward running
//     statistics and num_batches_tracked - is done by whoever wins that item's claim word (one
//     atomic exchange per item, on its own address: no contention).  Whatever the order, some
//     running block publishes every item;
//   * tags and claims are zeroed once per training step: bn_handoff_begin() (ops/bn.py
//     begin_step) memsets the arena region the previous step used; each fused launch takes a
//     fresh range of it, so a granule is written by one launch between two zeroings (a graph
//     replay replays that memset too).  Outside a step the launches run unfused.
// A wait that still exceeds its final bound adds to an error word (bn_handoff_errors(); never
// expected) and proceeds.
#pragma once

#include "common.h"

namespace dpt {

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

struct BnHandoff {
  unsigned* err = nullptr;    // bounded-spin time-outs
  unsigned* claim = nullptr;  // [nfin] one word per finalize item (forward running statistics)
  int nfin = 0;               // blocks [0, nfin) run the finalize (0: not fused)
  int idle_fin = 0;           // test only (bn_set_handoff_idle_finalizers): the finalize blocks
                              // exit at once, so every apply block must help
};

// The claim of finalize item `claim` (one lane): true for exactly one caller per step.
__device__ __forceinline__ bool handoff_claim(unsigned* claim) {
  return __hip_atomic_exchange((gu32*)claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
}

// granule store: ONE aligned 8-byte write-through store {tag 1 | value}
__device__ __forceinline__ void put_gran(unsigned long long* g, float v) {
  __hip_atomic_store((gu64*)g, (1ull << 32) | (unsigned long long)__builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// polls (s_sleep 2 + an L2 round trip each, ~1 us) before a waiting block helps with the finalize
constexpr unsigned kHelpPolls = 256;
// ~2^22 polls: > 0.2 s, far beyond any finalize - only then the error word
constexpr unsigned kHandoffSpins = 1u << 22;

__device__ __forceinline__ unsigned long long gran_ld(const unsigned long long* g) {
  return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// granule load: re-read until the tag is set (bounded)
__device__ __forceinline__ float get_gran(const unsigned long long* g, unsigned* err) {
  unsigned long long v = gran_ld(g);
  for (unsigned it = 0; (v >> 32) != 1ull; ++it) {
    if (it == kHandoffSpins) {
      __hip_atomic_fetch_add((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
    v = gran_ld(g);
  }
  return __builtin_bit_cast(float, (unsigned)v);
}

// Whole block: wait for the n granules [g, g + n) of this launch; after kHelpPolls without them run
// every finalize item (fin(i), i < h.nfin: block-wide code) and wait again.  stage: copy the values
// to lds[0, n) (the callers stage when C <= kStageC, else each thread reads its own granules).
constexpr int kStageC = 512;
template <typename Fin>
__device__ __forceinline__ void handoff_acquire(const unsigned long long* g, int n, float* lds, bool stage,
                                                const BnHandoff& h, Fin&& fin) {
  bool ready = true;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    unsigned long long v = gran_ld(g + i);
    for (unsigned it = 0; (v >> 32) != 1ull && it < kHelpPolls; ++it) {
      __builtin_amdgcn_s_sleep(2);
      v = gran_ld(g + i);
    }
    if ((v >> 32) != 1ull) {
      ready = false;
      break;
    }
    if (stage) lds[i] = __builtin_bit_cast(float, (unsigned)v);
  }
  if (__syncthreads_or(!ready)) {  // block-uniform
#pragma nounroll
    for (int i = 0; i < h.nfin; ++i) fin(__builtin_amdgcn_readfirstlane(i));  // keeps the helper lean
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (stage)
      for (int i = threadIdx.x; i < n; i += blockDim.x) lds[i] = get_gran(g + i, h.err);
  }
  __syncthreads();
}

}  // namespace dpt
