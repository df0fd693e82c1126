// Agent-coherent access helpers and the hierarchical grid barrier shared by the persistent kernels
// (decoder_persist.hip, the BiLSTM in encoder.hip).
//
// Memory model: cross-workgroup data is written with agent-scope relaxed atomic stores (sc1:
// write-through past the per-XCD L2) and read with agent-scope loads (sc1, L1 bypass); every wave
// drains its stores (vmcnt(0)) before the barrier arrival. Barrier waits give up after 0.2 s
// (error word set, every workgroup exits): a launch that is not co-resident fails loudly.
#pragma once
#include "common.h"

constexpr unsigned long long BAR_TIMEOUT = 20000000ull;  // s_memrealtime ticks (100 MHz): 0.2 s

// ------------------------------------------------------------------ coherent access helpers
__device__ __forceinline__ float ldc(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ldci(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stc(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stci(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte agent-coherent load at byte offset `off` from a wave-uniform base (buffer load, sc1)
template <int AUX = 16>
__device__ __forceinline__ f32x4 ldc4(const float* base, int off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
}


// LDS-only workgroup barrier: unlike __syncthreads() (whose workgroup-scope fences wait for every
// outstanding global load, vmcnt(0)), global loads already in flight stay in flight
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Hierarchical grid barrier, split so that loads for the next phase can be issued between the
// arrival and the wait. arrive: every wave drains its stores (sc1 write-through), then thread 0
// counts the workgroup in at its XCD group counter (blockIdx % 8); the last arrival of a group counts it in at
// the global counter; the 8th XCD writes the go word.
// nwg: workgroups taking part (a multiple of 8; default the whole grid)
__device__ __forceinline__ void gsync_arrive(unsigned* bar, unsigned& gen, unsigned nwg = 0) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ++gen;
  if (threadIdx.x == 0) {
    unsigned* xc = bar + 64 + (blockIdx.x & 7) * 32;
    const unsigned per = (nwg ? nwg : gridDim.x) / 8;
    if (__hip_atomic_fetch_add(xc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == per * gen - 1)
      if (__hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 8u * gen - 1)
        __hip_atomic_store(bar + 32, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// wait for the go word; false = timed out (error word set, the caller exits)
__device__ __forceinline__ bool gsync_wait(unsigned* bar, unsigned gen, int* flag) {
  if (threadIdx.x == 0) {
    int good = 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(bar + 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > BAR_TIMEOUT) {
        __hip_atomic_fetch_or(bar + 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        good = 0;
        break;
      }
    }
    *flag = good;
  }
  lds_barrier();
  return *flag;
}

