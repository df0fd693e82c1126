// Microbenchmark for a persistent (one launch per chunk of decoder steps) design: the cost of a
// grid-wide barrier across 256 co-resident workgroups, and of a decoder_rnn-sized GEMM phase
// (4096 gate rows x K = 2560, B = 32) whose weight fragments stay in VGPRs across iterations.
// Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/persist_bench.hip -o tools/persist_bench
#include "../tts_amd/csrc/common.h"

#include <cstdio>
#include <vector>

__device__ unsigned g_err;
__device__ int g_skew;  // > 0: each workgroup waits up to g_skew ticks (s_memtime) before arriving

// per-(workgroup, iteration) arrival skew, as a phase of uneven work would give
__device__ __forceinline__ void arrive_skew(int i) {
  const int sk = *(volatile int*)&g_skew;
  if (sk <= 0) return;
  const unsigned h = (blockIdx.x * 2654435761u) ^ ((unsigned)i * 40503u);
  const unsigned long long d = (h >> 8) % (unsigned)sk, t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < d) {}
}

// mode bit 0: agent acquire fence after the barrier; bit 1: s_sleep in the spin
__device__ __forceinline__ bool grid_sync(unsigned* ctr, unsigned& target, int mode, int* ok) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    target += gridDim.x;
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int good = 1;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {  // 0.2 s: give up, every WG exits
        atomicOr(&g_err, 1u);
        good = 0;
        break;
      }
      if (mode & 2) __builtin_amdgcn_s_sleep(1);
    }
    if (mode & 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    *ok = good;
  }
  __syncthreads();
  return *ok;
}

__global__ __launch_bounds__(256) void bar_kernel(unsigned* ctr, int iters, int mode) {
  __shared__ int ok;
  unsigned target = 0;
  for (int i = 0; i < iters; ++i)
    if (!grid_sync(ctr, target, mode, &ok)) return;
}

__device__ __forceinline__ bool spin_timeout(unsigned long long t0) {
  if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {
    atomicOr(&g_err, 1u);
    return true;
  }
  return false;
}

// (B) hierarchical: per-XCD counters (workgroups are dispatched round-robin over the 8 XCDs), the
// last arriver of an XCD bumps the global counter, the last global arriver bumps a go flag
__global__ __launch_bounds__(256) void bar_hier_kernel(unsigned* ctr, int iters) {
  __shared__ int ok;
  const int xcd = blockIdx.x & 7;
  const unsigned per = gridDim.x / 8;
  unsigned* xc = ctr + 64 + xcd * 32;  // own 128-B line per XCD
  unsigned* gc = ctr;
  unsigned* go = ctr + 32;
  for (int i = 0; i < iters; ++i) {
    arrive_skew(i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      int good = 1;
      const unsigned old = __hip_atomic_fetch_add(xc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == per * (i + 1) - 1) {
        const unsigned g = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (g == 8u * (i + 1) - 1) __hip_atomic_store(go, (unsigned)(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(i + 1))
        if (spin_timeout(t0)) {
          good = 0;
          break;
        }
      ok = good;
    }
    __syncthreads();
    if (!ok) return;
  }
}

// (F) per-XCD counters, the last arriver of an XCD writes its XCD's slot of one 8-slot line; every
// workgroup polls that line (lanes 0-7) until all slots hold the generation (no second atomic)
__global__ __launch_bounds__(256) void bar_hier8_kernel(unsigned* ctr, int iters) {
  __shared__ int ok;
  const int xcd = blockIdx.x & 7;
  const unsigned per = gridDim.x / 8;
  unsigned* xc = ctr + 64 + xcd * 32;
  unsigned* line = ctr + 32;
  for (int i = 0; i < iters; ++i) {
    arrive_skew(i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(xc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == per * (i + 1) - 1) __hip_atomic_store(line + xcd, (unsigned)(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x < 64) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      int good = 1;
      const int l = threadIdx.x & 7;
      while (true) {
        unsigned v = __hip_atomic_load(line + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__builtin_amdgcn_ballot_w64(v < (unsigned)(i + 1)) == 0) break;
        if (spin_timeout(t0)) {
          good = 0;
          break;
        }
      }
      if (threadIdx.x == 0) ok = good;
    }
    __syncthreads();
    if (!ok) return;
  }
}
// (G) NC counters (each on its own 128-B line), arrival = one add that returns nothing (no atomic
// round trip on the arriving workgroup's chain); lanes 0..NC-1 of wave 0 poll every counter until
// each holds its share of the generation (no leader, no go word)
template <int NC>
__global__ __launch_bounds__(256) void bar_ctrs_kernel(unsigned* ctr, int iters) {
  __shared__ int ok;
  const unsigned per = gridDim.x / NC;
  unsigned* mine = ctr + 64 + (blockIdx.x % NC) * 32;
  for (int i = 0; i < iters; ++i) {
    arrive_skew(i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(mine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < 64) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      int good = 1;
      const int l = threadIdx.x % NC;
      const unsigned want = per * (unsigned)(i + 1);
      while (true) {
        unsigned v = __hip_atomic_load(ctr + 64 + l * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__builtin_amdgcn_ballot_w64(v < want) == 0) break;
        if (spin_timeout(t0)) {
          good = 0;
          break;
        }
      }
      if (threadIdx.x == 0) ok = good;
    }
    __syncthreads();
    if (!ok) return;
  }
}

// (H) per-XCD counters (returning add); the last arriver of an XCD adds to the global counter
// without waiting for the result, and every workgroup polls the global counter itself (8 arrivals
// per generation): one atomic round trip and the go-word store fewer on the last arriver's chain
__global__ __launch_bounds__(256) void bar_hier2_kernel(unsigned* ctr, int iters) {
  __shared__ int ok;
  const int xcd = blockIdx.x & 7;
  const unsigned per = gridDim.x / 8;
  unsigned* xc = ctr + 64 + xcd * 32;
  unsigned* gc = ctr;
  for (int i = 0; i < iters; ++i) {
    arrive_skew(i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      int good = 1;
      const unsigned old = __hip_atomic_fetch_add(xc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == per * (i + 1) - 1) __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(gc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 8u * (i + 1))
        if (spin_timeout(t0)) {
          good = 0;
          break;
        }
      ok = good;
    }
    __syncthreads();
    if (!ok) return;
  }
}

// (P) the hierarchical barrier with K go-word polls in flight (issued about RT / K apart): the
// release is seen within ~RT / K of landing instead of up to one load round trip later
__device__ __forceinline__ unsigned ald(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 4 go-word polls in flight (issued about s_sleep SLP apart, then each reissued as soon as it has
// been checked: vmcnt(3) waits for the oldest only); true once the word holds gen, false after
// `rounds` rounds of 4 (the caller then polls with its timeout check)
template <int SLP>
__device__ __forceinline__ bool poll4(const unsigned* go, unsigned gen, int rounds) {
  unsigned a, b, c, d;
  int hit;
  asm volatile(
      "global_load_dword %[a], %[p], off sc1\n"
      "s_sleep %[slp]\n"
      "global_load_dword %[b], %[p], off sc1\n"
      "s_sleep %[slp]\n"
      "global_load_dword %[c], %[p], off sc1\n"
      "s_sleep %[slp]\n"
      "global_load_dword %[d], %[p], off sc1\n"
      "s_mov_b32 %[hit], 0\n"
      "1:\n"
      "s_waitcnt vmcnt(3)\n"
      "v_cmp_le_u32 vcc, %[g], %[a]\n"
      "s_nop 4\n"
      "s_cbranch_vccnz 2f\n"
      "global_load_dword %[a], %[p], off sc1\n"
      "s_waitcnt vmcnt(3)\n"
      "v_cmp_le_u32 vcc, %[g], %[b]\n"
      "s_nop 4\n"
      "s_cbranch_vccnz 2f\n"
      "global_load_dword %[b], %[p], off sc1\n"
      "s_waitcnt vmcnt(3)\n"
      "v_cmp_le_u32 vcc, %[g], %[c]\n"
      "s_nop 4\n"
      "s_cbranch_vccnz 2f\n"
      "global_load_dword %[c], %[p], off sc1\n"
      "s_waitcnt vmcnt(3)\n"
      "v_cmp_le_u32 vcc, %[g], %[d]\n"
      "s_nop 4\n"
      "s_cbranch_vccnz 2f\n"
      "global_load_dword %[d], %[p], off sc1\n"
      "s_sub_u32 %[n], %[n], 1\n"
      "s_cmp_gt_i32 %[n], 0\n"
      "s_cbranch_scc1 1b\n"
      "s_branch 3f\n"
      "2:\n"
      "s_mov_b32 %[hit], 1\n"
      "3:\n"
      "s_waitcnt vmcnt(0)\n"
      : [a] "=&v"(a), [b] "=&v"(b), [c] "=&v"(c), [d] "=&v"(d), [hit] "=&s"(hit), [n] "+s"(rounds)
      : [p] "v"(go), [g] "v"(gen), [slp] "i"(SLP)
      : "vcc", "scc", "memory");
  return hit != 0;
}

template <int SLP>
__global__ __launch_bounds__(256) void bar_asm_kernel(unsigned* ctr, int iters) {
  __shared__ int ok;
  const int xcd = blockIdx.x & 7;
  const unsigned per = gridDim.x / 8;
  unsigned* xc = ctr + 64 + xcd * 32;
  unsigned* gc = ctr;
  unsigned* go = ctr + 32;
  for (int i = 0; i < iters; ++i) {
    arrive_skew(i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      int good = 1;
      const unsigned gen = (unsigned)(i + 1);
      const unsigned old = __hip_atomic_fetch_add(xc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == per * gen - 1) {
        const unsigned g = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (g == 8u * gen - 1) __hip_atomic_store(go, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (!poll4<SLP>(go, gen, 64)) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen)
          if (spin_timeout(t0)) {
            good = 0;
            break;
          }
      }
      ok = good;
    }
    __syncthreads();
    if (!ok) return;
  }
}

template <int K, int SLP>
__global__ __launch_bounds__(256) void bar_pipe_kernel(unsigned* ctr, int iters) {
  __shared__ int ok;
  const int xcd = blockIdx.x & 7;
  const unsigned per = gridDim.x / 8;
  unsigned* xc = ctr + 64 + xcd * 32;
  unsigned* gc = ctr;
  unsigned* go = ctr + 32;
  for (int i = 0; i < iters; ++i) {
    arrive_skew(i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      int good = 1;
      const unsigned gen = (unsigned)(i + 1);
      const unsigned old = __hip_atomic_fetch_add(xc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == per * gen - 1) {
        const unsigned g = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (g == 8u * gen - 1) __hip_atomic_store(go, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      unsigned v[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        v[k] = ald(go);
        if (k + 1 < K) __builtin_amdgcn_s_sleep(SLP);
      }
      bool done = false;
      while (!done) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          if (v[k] >= gen) {
            done = true;
            break;
          }
          v[k] = ald(go);
        }
        if (!done && spin_timeout(t0)) {
          good = 0;
          break;
        }
      }
      ok = good;
    }
    __syncthreads();
    if (!ok) return;
  }
}

// (T) the hierarchical barrier with NC first-level counters (workgroup g -> counter g % NC, STRIDE
// words apart) feeding the global counter (NC arrivals), then the go word: fewer arrivals contend
// on each counter when the whole grid arrives at once
template <int NC, int STRIDE>
__global__ __launch_bounds__(256) void bar_tree_kernel(unsigned* ctr, int iters) {
  __shared__ int ok;
  const unsigned per = gridDim.x / NC;
  unsigned* xc = ctr + 1024 + (blockIdx.x % NC) * STRIDE;
  unsigned* gc = ctr;
  unsigned* go = ctr + 32;
  for (int i = 0; i < iters; ++i) {
    arrive_skew(i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      int good = 1;
      const unsigned gen = (unsigned)(i + 1);
      if (__hip_atomic_fetch_add(xc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == per * gen - 1)
        if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)NC * gen - 1)
          __hip_atomic_store(go, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen)
        if (spin_timeout(t0)) {
          good = 0;
          break;
        }
      ok = good;
    }
    __syncthreads();
    if (!ok) return;
  }
}

// (X) a 32-workgroup barrier: one counter + go word, participants either the 32 workgroups of XCD 0
// (blockIdx % 8 == 0, SAME = 1) or workgroups 0..31 (spread over the 8 XCDs); the rest exit
template <int SAME>
__global__ __launch_bounds__(256) void bar32_kernel(unsigned* ctr, int iters) {
  __shared__ int ok;
  if (SAME ? (blockIdx.x & 7) != 0 : blockIdx.x >= 32) return;
  unsigned* xc = ctr + 64;
  unsigned* go = ctr + 32;
  for (int i = 0; i < iters; ++i) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      int good = 1;
      const unsigned gen = (unsigned)(i + 1);
      if (__hip_atomic_fetch_add(xc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 32u * gen - 1)
        __hip_atomic_store(go, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen)
        if (spin_timeout(t0)) {
          good = 0;
          break;
        }
      ok = good;
    }
    __syncthreads();
    if (!ok) return;
  }
}

// (C) flag array, no atomics: each workgroup stores its generation to its own slot; wave 0 polls
// all slots (4 per lane) until the minimum reaches the generation
__global__ __launch_bounds__(256) void bar_flags_kernel(unsigned* flags, int iters) {
  __shared__ int ok;
  for (int i = 0; i < iters; ++i) {
    arrive_skew(i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flags + blockIdx.x, (unsigned)(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < 64) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      int good = 1;
      while (true) {
        unsigned m = 0xffffffffu;
        for (int j = threadIdx.x; j < (int)gridDim.x; j += 64)
          m = min(m, __hip_atomic_load(flags + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        for (int off = 32; off > 0; off >>= 1) m = min(m, (unsigned)__shfl_xor((int)m, off, 64));
        if (m >= (unsigned)(i + 1)) break;
        if (spin_timeout(t0)) {
          good = 0;
          break;
        }
      }
      if (threadIdx.x == 0) ok = good;
    }
    __syncthreads();
    if (!ok) return;
  }
}

// (E) one counter, but waiters poll a separate go flag written by the last arriver
__global__ __launch_bounds__(256) void bar_go_kernel(unsigned* ctr, int iters) {
  __shared__ int ok;
  unsigned* go = ctr + 32;
  for (int i = 0; i < iters; ++i) {
    arrive_skew(i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      int good = 1;
      const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == gridDim.x * (i + 1) - 1) __hip_atomic_store(go, (unsigned)(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(i + 1))
        if (spin_timeout(t0)) {
          good = 0;
          break;
        }
      ok = good;
    }
    __syncthreads();
    if (!ok) return;
  }
}

__global__ void empty_kernel() {}

constexpr int KC = 160;  // 2560 / 16
constexpr int NWV = 8;   // waves per workgroup
constexpr int NKW = KC / NWV;  // k-chunks per wave

// MODE bit 2: activation loads with sc1 (device-coherent) instead of plain loads
template <int MT, int MODE>
__global__ __launch_bounds__(64 * NWV) void k4_kernel(const f32x4* __restrict__ W, const f32x4* act, float* out,
                                                 unsigned* ctr, int iters) {
  __shared__ int ok;
  __shared__ f32x4 red[NWV][MT][64];
  const int tile = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  f32x4 w[NKW];
#pragma unroll
  for (int i = 0; i < NKW; ++i) w[i] = W[((long)tile * KC + wave * NKW + i) * 64 + lane];
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)act, 0, 0x7fffffff, 0x00020000);
  auto ld = [&](int i, int mt) {
    const int idx = (mt * KC + wave * NKW + i) * 64 + lane;
    if constexpr (MODE & 4) return __builtin_amdgcn_raw_buffer_load_b128(rs, idx * 16, 0, 16);
    else return act[idx];
  };
  unsigned target = 0;
  for (int it = 0; it < iters; ++it) {
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int G = 4;
    f32x4 a[2][G][MT];
#pragma unroll
    for (int i = 0; i < G; ++i)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a[0][i][mt] = ld(i, mt);
#pragma unroll
    for (int i0 = 0; i0 < NKW; i0 += G) {
      const int cur = (i0 / G) & 1;
      if (i0 + G < NKW) {
#pragma unroll
        for (int i = 0; i < G; ++i)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) a[cur ^ 1][i][mt] = ld(i0 + G + i, mt);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < G; ++i)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[mt] = MFMA16(a[cur][i][mt][s], w[i0 + i][s], acc[mt]);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[wave][mt][lane] = acc[mt];
    __syncthreads();
    if (wave < MT) {
      f32x4 r = red[0][wave][lane];
#pragma unroll
      for (int v = 1; v < NWV; ++v) r += red[v][wave][lane];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __hip_atomic_store(out + ((long)(wave * 16 + 4 * (lane >> 4) + j) * 4096 + tile * 16 + (lane & 15)), r[j],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!grid_sync(ctr, target, MODE, &ok)) return;
  }
}

static hipStream_t S;

template <typename F>
static float timed(F launch) {
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  launch();  // warm
  HIP_OK(hipStreamSynchronize(S));
  HIP_OK(hipEventRecord(e0, S));
  launch();
  HIP_OK(hipEventRecord(e1, S));
  HIP_OK(hipEventSynchronize(e1));
  float ms;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  return ms;
}

static bool check_err(const char* what) {
  unsigned e = 0;
  HIP_OK(hipMemcpyFromSymbol(&e, HIP_SYMBOL(g_err), 4));
  if (e) {
    printf("%s: barrier timeout (not all workgroups co-resident?)\n", what);
    unsigned z = 0;
    HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_err), &z, 4));
    return false;
  }
  return true;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  HIP_OK(hipStreamCreate(&S));
  unsigned* ctr;
  HIP_OK(hipMalloc(&ctr, 4));
  const int NWG = 256;
  const size_t lds_force = 96 * 1024;  // one workgroup per CU
  HIP_OK(hipFuncSetAttribute((const void*)bar_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_force));
  for (int mode : {0, 1, 2, 3}) {
    const int iters = 2000;
    float ms = timed([&] {
      HIP_OK(hipMemsetAsync(ctr, 0, 4, S));
      int it = iters, md = mode;
      void* args[] = {&ctr, &it, &md};
      HIP_OK(hipLaunchCooperativeKernel((const void*)bar_kernel, dim3(NWG), dim3(256), args, lds_force, S));
    });
    if (!check_err("barrier")) return 1;
    printf("grid barrier, 256 WGs, mode %d (fence %d, sleep %d): %.3f us per barrier\n", mode, mode & 1,
           (mode >> 1) & 1, ms * 1000.f / iters);
  }
  unsigned* big;
  HIP_OK(hipMalloc(&big, 80 * 1024 * 4));
  for (int sk : {0, 1000})
  for (int v : {0, 15, 20, 21}) {
    HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_skew), &sk, 4));
    const void* f = v == 0 ? (const void*)bar_hier_kernel : v == 1 ? (const void*)bar_flags_kernel
                  : v == 2 ? (const void*)bar_go_kernel : v == 3 ? (const void*)bar_hier8_kernel
                  : v == 4 ? (const void*)bar_ctrs_kernel<8> : v == 5 ? (const void*)bar_ctrs_kernel<16>
                  : v == 6 ? (const void*)bar_hier2_kernel : v == 7 ? (const void*)bar_pipe_kernel<2, 4>
                  : v == 8 ? (const void*)bar_pipe_kernel<4, 2> : v == 9 ? (const void*)bar_pipe_kernel<4, 0>
                  : v == 10 ? (const void*)bar_pipe_kernel<8, 1> : v == 11 ? (const void*)bar_asm_kernel<2>
                  : v == 12 ? (const void*)bar_asm_kernel<4> : v == 13 ? (const void*)bar_asm_kernel<8>
                  : v == 14 ? (const void*)bar_tree_kernel<8, 1024> : v == 15 ? (const void*)bar_tree_kernel<16, 32>
                  : v == 16 ? (const void*)bar_tree_kernel<16, 1024> : v == 17 ? (const void*)bar_tree_kernel<32, 32>
                  : v == 18 ? (const void*)bar_tree_kernel<32, 1024> : v == 19 ? (const void*)bar_tree_kernel<64, 1024>
                  : v == 20 ? (const void*)bar32_kernel<1> : (const void*)bar32_kernel<0>;
    const char* nm = v == 0 ? "hierarchical" : v == 1 ? "flag array" : v == 2 ? "counter + go flag"
                   : v == 3 ? "xcd ctr + 8-slot line" : v == 4 ? "8 ctrs, poll all" : v == 5 ? "16 ctrs, poll all"
                   : v == 6 ? "xcd ctr, poll global" : v == 7 ? "hier, 2 polls s4" : v == 8 ? "hier, 4 polls s2"
                   : v == 9 ? "hier, 4 polls s0" : v == 10 ? "hier, 8 polls s1" : v == 11 ? "hier, asm 4 polls s2"
                   : v == 12 ? "hier, asm 4 polls s4" : v == 13 ? "hier, asm 4 polls s8"
                   : v == 14 ? "tree 8 x 4KB" : v == 15 ? "tree 16 x 128B" : v == 16 ? "tree 16 x 4KB"
                   : v == 17 ? "tree 32 x 128B" : v == 18 ? "tree 32 x 4KB" : v == 19 ? "tree 64 x 4KB"
                   : v == 20 ? "32 WGs of one XCD" : "32 WGs over 8 XCDs";
    HIP_OK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_force));
    if (sk) printf("(arrival skew up to %d memtime ticks)\n", sk);
    for (int nwg : {256}) {
      const int iters = 2000;
      float ms = timed([&] {
        HIP_OK(hipMemsetAsync(big, 0, 80 * 1024 * 4, S));
        int it = iters;
        void* args[] = {&big, &it};
        HIP_OK(hipLaunchCooperativeKernel(f, dim3(nwg), dim3(256), args, lds_force, S));
      });
      if (!check_err(nm)) return 1;
      printf("grid barrier %-18s %d WGs: %.3f us per barrier\n", nm, nwg, ms * 1000.f / iters);
    }
  }
  {
    hipGraph_t g;
    hipGraphExec_t ge;
    HIP_OK(hipStreamBeginCapture(S, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 100; ++i) empty_kernel<<<256, 256, 0, S>>>();
    HIP_OK(hipStreamEndCapture(S, &g));
    HIP_OK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    float ms = timed([&] { HIP_OK(hipGraphLaunch(ge, S)); });
    printf("empty kernel in a graph: %.3f us per launch\n", ms * 10.f);
  }
  // K4-sized phase with resident weights
  const int Bp = 32;
  std::vector<float> h((size_t)4096 * 2560);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 1e-3f * (float)((i * 2654435761u) % 1000) / 1000.f;
  f32x4* W;
  f32x4* act;
  float* out;
  HIP_OK(hipMalloc(&W, h.size() * 4));
  HIP_OK(hipMemcpy(W, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMalloc(&act, (size_t)Bp * 2560 * 4));
  HIP_OK(hipMemcpy(act, h.data(), (size_t)Bp * 2560 * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMalloc(&out, (size_t)Bp * 4096 * 4));
  auto run_k4 = [&](const void* f, int mt, int mode) {
    HIP_OK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_force));
    const int iters = 500;
    float ms = timed([&] {
      HIP_OK(hipMemsetAsync(ctr, 0, 4, S));
      int it = iters;
      void* args[] = {&W, &act, &out, &ctr, &it};
      HIP_OK(hipLaunchCooperativeKernel(f, dim3(NWG), dim3(64 * NWV), args, lds_force, S));
    });
    if (!check_err("k4")) exit(1);
    printf("K4 phase resident weights MT=%d mode %d: %.3f us per phase (incl. barrier)\n", mt, mode,
           ms * 1000.f / iters);
  };
  run_k4((const void*)k4_kernel<2, 1>, 2, 1);
  run_k4((const void*)k4_kernel<2, 4>, 2, 4);
  run_k4((const void*)k4_kernel<2, 3>, 2, 3);
  run_k4((const void*)k4_kernel<1, 1>, 1, 1);
  run_k4((const void*)k4_kernel<1, 4>, 1, 4);
  printf("done\n");
  return 0;
}
