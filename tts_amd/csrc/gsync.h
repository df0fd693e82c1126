// Agent-coherent access helpers and the grid barriers (counter and flag forms) shared by the persistent kernels
// (decoder_persist.hip, the BiLSTM and GE2E pipeline in encoder.hip).
//
// Memory model: cross-workgroup data is written with agent-scope relaxed atomic stores (sc1:
// write-through past the per-XCD L2) and read with agent-scope loads (sc1, L1 bypass); every wave
// drains its stores (vmcnt(0)) before the barrier arrival. Barrier waits give up after a limit
// (error word set, every workgroup exits): a launch that is not co-resident fails loudly.
//
// Why relaxed arrivals and a relaxed go-word poll suffice (no release / acquire fences):
//  * hardware: this is the hand-off form MI355X_MICROARCH.md ("Valid forms", inter-workgroup
//    visibility) lists in place of a release / acquire pair: EVERY store of the handed-off bytes is
//    sc1 (reaches the memory side, nothing dirty stays in an XCD L2 to write back) and is drained
//    (s_waitcnt vmcnt(0)) by its wave before the workgroup barrier that precedes the counter add,
//    and EVERY load of them is a global_/buffer_ sc1 load to registers issued after the poll and a
//    workgroup barrier (never L1-served, so no stale line needs invalidating). An agent-scope
//    release fetch_add would add buffer_wbl2 sc1 (~1.7 us per the guide) and an acquire load
//    buffer_inv sc1 (+1.7 us measured on this kernel) to every one of the ~5
//    barriers of a decoder step, for no data that is not already coherent;
//  * compiler: every point where ordering matters is a compiler barrier: the drain is an asm with
//    a "memory" clobber followed by __syncthreads(), and the wait ends in lds_barrier() (asm,
//    "memory" clobber), so no load or store is moved across the arrival or the wait.
// Plain (non-sc1) accesses of cross-workgroup data are therefore a bug in this scheme; every such
// access goes through ldc / ldci / ldc4 / stc / stci below.
// The wait limit sits in word BAR_TMO of each barrier block (BAR_WORDS words), written by arm_barrier at
// launch: TTS_BARRIER_TIMEOUT_MS (default 2000 ms). The cooperative launch itself guarantees
// co-residency; the limit only turns an over-admitted grid (occupancy API one workgroup per CU
// too high) into an error instead of a hang, so it is generous enough that a workgroup preempted
// by another queue on the same GPU does not trip it.
#pragma once
#include "common.h"
#include <hip/hip_ext.h>
#include "split16.h"

#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

constexpr int BAR_TMO = 48;  // word of the barrier block holding the wait limit (s_memrealtime ticks)
// words per barrier block: 0 global counter, 16 error word, 32 go word, BAR_TMO wait limit, then up
// to 16 first-level counters on their own 128-byte lines (words 64 + 32 c); the flag form uses the
// error word, the wait limit, go words 32 + 64 k (k < BAR_NGO) and arrival flags at BAR_FLAGS
constexpr int BAR_WORDS = 1024;

// entries zeroing `nblk` barrier blocks and writing their wait limit, for a caller's fill
inline void add_barrier_fills(FillList& f, unsigned* bar, int nblk) {
  static const unsigned ticks = [] {
    double ms = 2000.0;
    if (const char* e = std::getenv("TTS_BARRIER_TIMEOUT_MS")) ms = std::atof(e);
    ms = ms < 1.0 ? 1.0 : (ms > 40000.0 ? 40000.0 : ms);
    return (unsigned)(ms * 1e5);  // 100 MHz ticks
  }();
  for (int i = 0; i < nblk; ++i) {
    f.add(bar + i * BAR_WORDS, BAR_TMO * 4);
    f.add(bar + i * BAR_WORDS + BAR_TMO, 4, ticks);
    f.add(bar + i * BAR_WORDS + BAR_TMO + 1, (BAR_WORDS - BAR_TMO - 1) * 4);
  }
}

// zero `nblk` barrier blocks and write their wait limit (stream-ordered before the launch)
inline void arm_barrier(unsigned* bar, int nblk, hipStream_t s) {
  FillList f;
  add_barrier_fills(f, bar, nblk);
  launch_fills(f, s);
}

// gsync_arrive's first-level counters each take n / NC arrivals: n must be a multiple of NC
// (16 for n >= 256, else 8), or a counter never completes and every wait times out
inline bool gsync_count_ok(unsigned n) { return n > 0 && n % (n >= 256 ? 16u : 8u) == 0; }

// Launch a kernel whose workgroups meet at grid barriers. Every workgroup must be resident at
// once: that is checked here against the occupancy query, which is all a cooperative launch adds
// (MI355X_MICROARCH.md "coop-launch": same residency as a plain launch, +15-19 us of host time).
// hipLaunchCooperativeKernel also sets up HIP's cooperative queue, whose teardown at process exit
// collides with the HSA runtime rocprofv3 preloads (SIGSEGV in exit() after the profile is
// written), so the plain launch is the default. TTS_COOP_LAUNCH=1 restores it.
// ev0 / ev1 (optional): timing events taken from the launch itself (hipExtLaunchKernel), so that no
// event-record packet sits between the kernel and its neighbours on the stream
inline void launch_resident(const void* f, dim3 grid, dim3 block, void** args, size_t lds, hipStream_t s,
                            hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> fits;  // (kernel, device) -> workgroups it holds at once
  static const bool coop = [] {
    const char* e = std::getenv("TTS_COOP_LAUNCH");
    return e && std::atoi(e) != 0;
  }();
  int cap = 0, dev = 0;
  HIP_OK(hipGetDevice(&dev));
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = fits.find({f, dev});
    if (it == fits.end()) {
      int cus = 0, nb = 0;
      HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, (int)(block.x * block.y * block.z), lds));
      it = fits.emplace(std::make_pair(f, dev), nb * cus).first;
    }
    cap = it->second;
  }
  TTS_CHECK((long)grid.x * grid.y * grid.z <= cap, "grid-barrier kernel: grid larger than the device holds at once");
  TTS_CHECK(grid.y == 1 && grid.z == 1 && gsync_count_ok(grid.x),
            "grid-barrier kernel: a 1-D grid that is a multiple of the barrier's counter fan-in");
  if (coop) {
    if (ev0) HIP_OK(hipEventRecord(ev0, s));
    HIP_OK(hipLaunchCooperativeKernel(f, grid, block, args, (unsigned)lds, s));
    if (ev1) HIP_OK(hipEventRecord(ev1, s));
  } else if (ev0 || ev1) {
    HIP_OK(hipExtLaunchKernel(f, grid, block, args, lds, s, ev0, ev1, 0));
  } else {
    HIP_OK(hipLaunchKernel(f, grid, block, args, lds, s));
  }
}

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
// 16-byte agent-coherent store at byte offset `off` from a wave-uniform base (buffer store, sc1:
// write-through, one fabric write per lane instead of four 4-byte ones)
__device__ __forceinline__ void stc4(float* base, int off, f32x4 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);  // lax vector conversion: a bitcast
}

// 4 consecutive elements held by the 4 lanes of a DPP quad (lane q of the quad: element e0 + q,
// e0 % 4 == 0, every lane of the quad active): gathered into the quad's lane 0 and written as ONE
// 16-byte coherent store. TTS_NARROW_STORES keeps the per-lane 4-byte stores (A/B builds).
__device__ __forceinline__ void stc_quad(float* base, int e, float v) {
#ifdef TTS_NARROW_STORES
  stc(base + e, v);
#else
  const int b = __float_as_int(v);
  const f32x4 q = {__int_as_float(__builtin_amdgcn_mov_dpp(b, 0x00, 0xf, 0xf, true)),   // quad_perm(0,0,0,0)
                   __int_as_float(__builtin_amdgcn_mov_dpp(b, 0x55, 0xf, 0xf, true)),   // (1,1,1,1)
                   __int_as_float(__builtin_amdgcn_mov_dpp(b, 0xAA, 0xf, 0xf, true)),   // (2,2,2,2)
                   __int_as_float(__builtin_amdgcn_mov_dpp(b, 0xFF, 0xf, 0xf, true))};  // (3,3,3,3)
  if ((threadIdx.x & 3) == 0) stc4(base, e * 4, q);
#endif
}
// stc_quad's pre-split form (the persistent decoder's and the BiLSTM's split-f16 hand-offs): lanes
// 4 q .. 4 q + 3 hold 4 consecutive k of one row; lane 4 q stores their f16 hi halves then their lo
// halves, [hi 0..3 | lo 0..3] in the 16 bytes (split_fast: the bits split8 on the consumer gives)
__device__ __forceinline__ void stc_quad_x3(float* base, int e, float v) {
  _Float16 hi, lo;
  split_fast(v, hi, lo);
  const int p = (int)((unsigned)__builtin_bit_cast(unsigned short, hi) |
                      ((unsigned)__builtin_bit_cast(unsigned short, lo) << 16));
  const unsigned p0 = (unsigned)__builtin_amdgcn_mov_dpp(p, 0x00, 0xf, 0xf, true),
                 p1 = (unsigned)__builtin_amdgcn_mov_dpp(p, 0x55, 0xf, 0xf, true),
                 p2 = (unsigned)__builtin_amdgcn_mov_dpp(p, 0xAA, 0xf, 0xf, true),
                 p3 = (unsigned)__builtin_amdgcn_mov_dpp(p, 0xFF, 0xf, 0xf, true);
  const f32x4 q = {__uint_as_float((p0 & 0xffffu) | (p1 << 16)), __uint_as_float((p2 & 0xffffu) | (p3 << 16)),
                   __uint_as_float((p0 >> 16) | (p1 & 0xffff0000u)), __uint_as_float((p2 >> 16) | (p3 & 0xffff0000u))};
  if ((threadIdx.x & 3) == 0) stc4(base, e * 4, q);
}

// LDS-only workgroup barrier: unlike __syncthreads() (whose workgroup-scope fences wait for every
// outstanding global load, vmcnt(0)), global loads already in flight stay in flight

// Hierarchical grid barrier, split so that loads for the next phase can be issued between the
// arrival and the wait. arrive: every wave drains its stores (sc1 write-through), then thread 0
// counts the workgroup in at its first-level counter (blockIdx % NC; workgroups are dealt round-robin
// over the 8 XCDs, so a counter's workgroups share an XCD); the last arrival at a counter counts it
// in at the global counter; the last of those writes the go word. NC = 16 for grids of 256 or more
// (16 arrivals per counter: tools/persist_bench.hip, 256 workgroups arriving together, 1.84 us
// against 2.14 us with one counter per XCD), 8 below.
// nwg: workgroups taking part (a multiple of NC, numbered from 0; default the whole grid)
__device__ __forceinline__ void gsync_arrive(unsigned* bar, unsigned& gen, unsigned nwg = 0) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ++gen;
  if (threadIdx.x == 0) {
    const unsigned n = nwg ? nwg : gridDim.x;
#ifdef TTS_BAR_NC8
    const unsigned nc = 8u;  // A/B builds: one counter per XCD
#else
    const unsigned nc = n >= 256 ? 16u : 8u;
#endif
    unsigned* xc = bar + 64 + (blockIdx.x % nc) * 32;
    if (__hip_atomic_fetch_add(xc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (n / nc) * gen - 1)
      if (__hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nc * gen - 1)
        __hip_atomic_store(bar + 32, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// Flag grid barrier (round 5; the persistent decoder's form, grids of at most 256 workgroups):
// arrival is ONE relaxed store per workgroup (its generation, to its own word of a 1 KB array at
// BAR_FLAGS) instead of two dependent atomic round trips; wave 0 of workgroup 0 polls the whole
// array (one 16-byte load per lane) and stores the go word to BAR_NGO lines (words 32 + 64 k), each
// workgroup polling copy blockIdx % BAR_NGO. tools/bar_bench.hip, 256 x 512 threads: 1.53 us per
// barrier against 1.84 us for gsync_arrive / gsync_wait, 2.10 against 2.45 us with a 1 KB hand-off
// around it. Every workgroup polling the array itself is slower (2.7 us: 256 pollers on 8 lines).
// The memory-model argument is gsync's: the stores before the arrival are drained sc1 stores.
// Users: the persistent decoder and the GE2E layer pipeline (whole grids). The BiLSTM's 64-workgroup
// recurrences keep gsync (tools/group_bar_bench.hip: counters 0.1 us per step ahead at that size).
// The block's physical place changes the cost (1.50-2.08 us per barrier): the decoder times
// candidate blocks once per workspace (decoder_persist.hip pick_barrier_blocks).
constexpr int BAR_FLAGS = 512;  // words 512 .. 767 of the barrier block
constexpr int BAR_NGO = 8;
// A barrier over a group of n workgroups (default the grid): idx = the workgroup's index in the
// group (default blockIdx.x), n <= 256; the group's index-0 workgroup releases it.
__device__ __forceinline__ void gflag_arrive(unsigned* bar, unsigned& gen, int idx = -1) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ++gen;
  if (idx < 0) idx = (int)blockIdx.x;
  if (threadIdx.x == 0) __hip_atomic_store(bar + BAR_FLAGS + idx, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool gflag_wait(unsigned* bar, unsigned gen, int* flag, int n = 0, int idx = -1) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (idx < 0) idx = (int)blockIdx.x;
  if (n <= 0) n = (int)gridDim.x;
  if (idx == 0) {
    if (threadIdx.x < 64) {
      const unsigned long long tmo = bar[BAR_TMO];
      const int w0 = 4 * (int)threadIdx.x;
      bool good = true;
      while (true) {
        const f32x4 v = ldc4(reinterpret_cast<const float*>(bar + BAR_FLAGS), w0 * 4);
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) ok = ok && (w0 + j >= n || __float_as_uint(v[j]) >= gen);
        if (__all(ok)) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > tmo) {
          good = false;
          break;
        }
      }
      if (good && threadIdx.x < BAR_NGO)
        __hip_atomic_store(bar + 32 + 64 * threadIdx.x, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (threadIdx.x == 0) {
        if (!good) __hip_atomic_fetch_or(bar + 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = good;
      }
    }
  } else if (threadIdx.x == 0) {
    const unsigned long long tmo = bar[BAR_TMO];
    const unsigned* go = bar + 32 + 64 * (idx % BAR_NGO);
    int good = 1;
    while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > tmo) {
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

// wait for the go word; false = timed out (error word set, the caller exits)
__device__ __forceinline__ bool gsync_wait(unsigned* bar, unsigned gen, int* flag) {
  if (threadIdx.x == 0) {
    int good = 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long tmo = bar[BAR_TMO];
    while (__hip_atomic_load(bar + 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > tmo) {
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

