// Barriers over workgroup groups, as the encoder BiLSTM runs them: a grid of 256
// workgroups x 256 threads in 4 independent groups of 64 (row group x direction), each step a
// hand-off of 256 B per workgroup (its 4 hidden units x 16 rows) read back whole (16 KB) by every
// workgroup of the group, then the group's barrier.
//   mode 0: gflag (the group's tile 0 polls the 64 flags and releases the group through 8 go lines)
//   mode 1: every workgroup polls its group's 64 flags itself (no go hop; 64 pollers on 2 lines)
//   mode 2: gsync counters (the round-4 form)
// Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/group_bar_bench.hip -o tools/group_bar_bench
#include "../tts_amd/csrc/gsync.h"

#include <cstdio>

#ifndef GB_NT
#define GB_NT 64
#endif
// NT workgroups per group (64: the encoder BiLSTM's 4 hidden units per workgroup; 16 / 32: 16 / 8
// units per workgroup), 16 KB of h per group either way (FPW floats published per workgroup)
constexpr int NT = GB_NT, NG = 4, FPW = 4096 / NT;

template <int MODE>
__global__ __launch_bounds__(256) void group_kernel(unsigned* bars, float* h, int steps, float* out) {
  __shared__ int flag;
  const int dom = blockIdx.x / NT, tl = blockIdx.x % NT;
  unsigned* bar = bars + dom * BAR_WORDS;
  float* hd = h + (size_t)dom * 2 * 4096;  // [2 step parities][NT workgroups][FPW floats]
  unsigned gen = 0;
  f32x4 acc = {0, 0, 0, 0};
  const int lane = threadIdx.x & 63;
  for (int s = 0; s < steps; ++s) {
    const float* hi = hd + (s & 1) * 4096;
    float* ho = hd + ((s + 1) & 1) * 4096;
    // read the group's whole h (16 KB): 256 threads x 4 x 16 B
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += ldc4(hi, ((j * 256 + threadIdx.x) * 16) % 16384);
    if (threadIdx.x < FPW / 4) stc4(ho, (tl * (FPW / 4) + threadIdx.x) * 16, acc * 0.5f);
    if (s + 1 == steps) break;
    if (MODE == 0) {
      gflag_arrive(bar, gen, tl);
      if (!gflag_wait(bar, gen, &flag, NT, tl)) return;
    } else if (MODE == 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      ++gen;
      if (threadIdx.x == 0) __hip_atomic_store(bar + BAR_FLAGS + tl, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (threadIdx.x < 64) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        bool good = true;
        while (true) {
          bool ok = true;
          if (lane < NT / 4) {
            const f32x4 v = ldc4(reinterpret_cast<const float*>(bar + BAR_FLAGS), lane * 16);
#pragma unroll
            for (int j = 0; j < 4; ++j) ok = ok && __float_as_uint(v[j]) >= gen;
          }
          if (__all(ok)) break;
          if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {
            good = false;
            break;
          }
        }
        if (threadIdx.x == 0) flag = good;
      }
      lds_barrier();
      if (!flag) return;
    } else {
      gsync_arrive(bar, gen, NT);
      if (!gsync_wait(bar, gen, &flag)) return;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? std::atoi(argv[1]) : 2000;
  unsigned* pool;
  float *h, *out;
  HIP_OK(hipMalloc(&pool, (size_t)16 * NG * BAR_WORDS * 4));
  HIP_OK(hipMalloc(&h, (size_t)NG * 2 * 4096 * 4));
  HIP_OK(hipMemset(h, 0, (size_t)NG * 2 * 4096 * 4));
  HIP_OK(hipMalloc(&out, 256 * 256 * 4));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  const void* ks[] = {(const void*)group_kernel<0>, (const void*)group_kernel<1>, (const void*)group_kernel<2>};
  const char* names[] = {"gflag (tile 0 releases)", "all poll the group's flags", "gsync counters"};
  for (const void* k : ks) HIP_OK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  for (int place = 0; place < 4; ++place)  // 4 consecutive-block placements of the 4 groups' blocks
    for (int m = 0; m < 3; ++m) {
      unsigned* bars = pool + (size_t)place * NG * BAR_WORDS;
      float best = 1e30f;
      for (int r = 0; r < 3; ++r) {
        HIP_OK(hipMemset(bars, 0, (size_t)NG * BAR_WORDS * 4));
        const unsigned tmo = 20000000u;
        for (int d = 0; d < NG; ++d) HIP_OK(hipMemcpy(bars + d * BAR_WORDS + BAR_TMO, &tmo, 4, hipMemcpyHostToDevice));
        int st = steps;
        void* args[] = {&bars, &h, &st, &out};
        HIP_OK(hipEventRecord(e0));
        HIP_OK(hipLaunchKernel(ks[m], dim3(NG * NT), dim3(256), args, 96 * 1024, 0));  // LDS: one workgroup per CU
        HIP_OK(hipEventRecord(e1));
        HIP_OK(hipEventSynchronize(e1));
        float ms = 0.f;
        HIP_OK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      unsigned err = 0;
      for (int d = 0; d < NG; ++d) {
        unsigned e = 0;
        HIP_OK(hipMemcpy(&e, bars + d * BAR_WORDS + 16, 4, hipMemcpyDeviceToHost));
        err |= e;
      }
      std::printf("{\"placement\": %d, \"mode\": %d, \"form\": \"%s\", \"us_per_step\": %.3f, \"err\": %u}\n", place, m,
                  names[m], best * 1000.f / steps, err);
      if (err) return 1;
    }
  return 0;
}
