// Grid-barrier forms for the persistent decoder's 256 x 512-thread grid:
// how long a barrier takes from the last arrival to every workgroup's release.
//   mode 0: gsync.h as the decoder runs it (16 first-level counters, a global counter, a go word)
//   mode 1: arrival flags: every workgroup stores its generation to its own word of a 1 KB array
//           (no atomics) and its wave 0 polls the whole array, one 16-byte load per lane
//   mode 2: arrival flags, polled by workgroup 0 only, which then stores a go word that the others poll
//   mode 3: as mode 1, with the flag words of one XCD's workgroups on one 128-byte line
//   mode 4: as mode 2, with mode 3's flag layout
//   mode 5: as mode 4, the go word stored to 8 lines (one per XCD), each workgroup polling its XCD's
//   mode 6: as mode 2, with mode 5's go-word copies
// + 8: a hand-off around each barrier: every workgroup stores 1 KB (sc1) before arriving and loads
//      another workgroup's 1 KB after the release (the decoder's phase-opening load)
// Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bar_bench.hip -o tools/bar_bench
#include "../tts_amd/csrc/gsync.h"

#include <cstdio>
#include <vector>

__device__ unsigned g_err;

__device__ __forceinline__ int flag_slot(int b, int m) {
  return (m == 3 || m == 4 || m == 5) ? (b % 8) * 32 + b / 8 : b;
}

// wave 0 polls the 256 flag words until all reach gen; false = timed out
__device__ __forceinline__ bool poll_flags(const unsigned* flags, unsigned gen) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    const f32x4 v = ldc4(reinterpret_cast<const float*>(flags), (int)threadIdx.x * 16);
    const unsigned m0 = __float_as_uint(v[0]) < __float_as_uint(v[1]) ? __float_as_uint(v[0]) : __float_as_uint(v[1]);
    const unsigned m1 = __float_as_uint(v[2]) < __float_as_uint(v[3]) ? __float_as_uint(v[2]) : __float_as_uint(v[3]);
    const bool ok = (m0 < m1 ? m0 : m1) >= gen;
    if (__all(ok)) return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) return false;
  }
}

// ring polling: 4 loads in flight, issued SL x 64 clocks apart, the oldest checked as the next is issued
__device__ __forceinline__ bool flags_ok(f32x4 v, unsigned gen) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 4; ++j) ok = ok && __float_as_uint(v[j]) >= gen;
  return __all(ok);
}
template <int SL>
__device__ __forceinline__ bool poll_flags_ring(const unsigned* flags, unsigned gen) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const float* f = reinterpret_cast<const float*>(flags);
  const int off = (int)threadIdx.x * 16;
  f32x4 a = ldc4(f, off);
  if (SL) __builtin_amdgcn_s_sleep(SL);
  f32x4 b = ldc4(f, off);
  if (SL) __builtin_amdgcn_s_sleep(SL);
  f32x4 c = ldc4(f, off);
  if (SL) __builtin_amdgcn_s_sleep(SL);
  while (true) {
    f32x4 d = ldc4(f, off);
    if (flags_ok(a, gen)) return true;
    if (SL) __builtin_amdgcn_s_sleep(SL);
    a = ldc4(f, off);
    if (flags_ok(b, gen)) return true;
    if (SL) __builtin_amdgcn_s_sleep(SL);
    b = ldc4(f, off);
    if (flags_ok(c, gen)) return true;
    if (SL) __builtin_amdgcn_s_sleep(SL);
    c = ldc4(f, off);
    if (flags_ok(d, gen)) return true;
    if (SL) __builtin_amdgcn_s_sleep(SL);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) return false;
  }
}
template <int SL>
__device__ __forceinline__ bool go_ring(const unsigned* go, unsigned gen) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  auto ld = [&]() { return __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  unsigned a = ld();
  if (SL) __builtin_amdgcn_s_sleep(SL);
  unsigned b = ld();
  if (SL) __builtin_amdgcn_s_sleep(SL);
  unsigned c = ld();
  if (SL) __builtin_amdgcn_s_sleep(SL);
  while (true) {
    unsigned d = ld();
    if (a >= gen) return true;
    if (SL) __builtin_amdgcn_s_sleep(SL);
    a = ld();
    if (b >= gen) return true;
    if (SL) __builtin_amdgcn_s_sleep(SL);
    b = ld();
    if (c >= gen) return true;
    if (SL) __builtin_amdgcn_s_sleep(SL);
    c = ld();
    if (d >= gen) return true;
    if (SL) __builtin_amdgcn_s_sleep(SL);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) return false;
  }
}

template <int SL>
__global__ __launch_bounds__(512) void ring_kernel(unsigned* bar, unsigned* flags, float* data, int iters, int hand,
                                                   float* out) {
  __shared__ int flag;
  unsigned gen = 0;
  f32x4 acc = {0, 0, 0, 0};
  for (int i = 0; i < iters; ++i) {
    if (hand && threadIdx.x < 64) stc4(data, (blockIdx.x * 64 + threadIdx.x) * 16, acc + (float)i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ++gen;
    if (threadIdx.x == 0) stci(reinterpret_cast<int*>(flags) + blockIdx.x, (int)gen);
    if (blockIdx.x == 0) {
      if (threadIdx.x < 64) {
        const bool good = poll_flags_ring<SL>(flags, gen);
        if (good && threadIdx.x < 8) stci(reinterpret_cast<int*>(bar) + 32 + 64 * threadIdx.x, (int)gen);
        if (threadIdx.x == 0) {
          flag = good;
          if (!good) atomicOr(&g_err, 1u);
        }
      }
    } else if (threadIdx.x == 0) {
      const bool good = go_ring<SL>(bar + 32 + 64 * (blockIdx.x % 8), gen);
      flag = good;
      if (!good) atomicOr(&g_err, 1u);
    }
    lds_barrier();
    if (!flag) return;
    if (hand && threadIdx.x < 64) acc += ldc4(data, (((blockIdx.x * 37 + i + 1) & 255) * 64 + threadIdx.x) * 16);
  }
  if (threadIdx.x < 64) out[blockIdx.x * 64 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

// atomic round trip from each XCD to candidate 4 KiB blocks: workgroup w (one per XCD) chases
// dependent agent-scope atomics through word 32 of block c; out[w][c] = ticks (100 MHz) for NCH loads, out[w][NC] = XCC id
constexpr int LAT_NC = 64, LAT_NCH = 64;
__global__ void lat_kernel(unsigned* pool, unsigned* out) {
  if (threadIdx.x != 0) return;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  for (int c = 0; c < LAT_NC; ++c) {
    const unsigned* p = pool + (size_t)c * 1024 + 32;
    unsigned v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // warm
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < LAT_NCH; ++i)  // atomics: performed past the XCD's L2 (a load would hit in it)
      v = __hip_atomic_fetch_add(const_cast<unsigned*>(p) + (v & 1), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * (LAT_NC + 1) + c] = (unsigned)(t1 - t0) + (v & 1);
  }
  out[blockIdx.x * (LAT_NC + 1) + LAT_NC] = xcc & 15u;
}

__global__ __launch_bounds__(512) void bar_kernel(unsigned* bar, unsigned* flags, float* data, int iters, int mode,
                                                  float* out, int ncp) {
  __shared__ int flag;
  unsigned gen = 0;
  f32x4 acc = {0, 0, 0, 0};
  const bool hand = mode & 8;
  const int m = mode & 7;
  const bool master = m == 2 || m >= 4, copies = m == 5 || m == 6;
  for (int i = 0; i < iters; ++i) {
    if (hand && threadIdx.x < 64) {
      const f32x4 v = acc + (float)i;
      stc4(data, (blockIdx.x * 64 + threadIdx.x) * 16, v);
    }
    if (m == 0) {
      gsync_arrive(bar, gen);
      if (!gsync_wait(bar, gen, &flag)) return;
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      ++gen;
      if (threadIdx.x == 0) stci(reinterpret_cast<int*>(flags) + flag_slot(blockIdx.x, m), (int)gen);
      if (master) {
        if (blockIdx.x == 0 && threadIdx.x < 64) {
          const bool good = poll_flags(flags, gen);
          if (good && (copies ? (int)threadIdx.x < ncp : threadIdx.x == 0))
            stci(reinterpret_cast<int*>(bar) + 32 + 64 * threadIdx.x, (int)gen);
          if (!good && threadIdx.x == 0) atomicOr(&g_err, 1u);
        }
        if (!gsync_wait(bar + (copies ? 64 * (blockIdx.x % ncp) : 0), gen, &flag)) return;
      } else {
        if (threadIdx.x < 64) {
          const bool good = poll_flags(flags, gen);
          if (threadIdx.x == 0) flag = good;
          if (!good && threadIdx.x == 0) atomicOr(&g_err, 1u);
        }
        lds_barrier();
        if (!flag) return;
      }
    }
    if (hand && threadIdx.x < 64) {
      const int src = (blockIdx.x * 37 + i + 1) & 255;
      acc += ldc4(data, (src * 64 + threadIdx.x) * 16);
    }
  }
  if (threadIdx.x < 64) out[blockIdx.x * 64 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 4000;
  unsigned *bar, *flags;
  float *data, *out;
  HIP_OK(hipMalloc(&bar, 64 * 64 * 4));
  HIP_OK(hipMalloc(&flags, 256 * 4));
  HIP_OK(hipMalloc(&data, 256 * 64 * 16));
  HIP_OK(hipMalloc(&out, 256 * 64 * 4));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  int nb = 0;
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)bar_kernel, 512, 0));
  int cus = 0;
  HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  if (nb * cus < 256) {
    std::printf("grid of 256 does not fit (%d x %d)\n", nb, cus);
    return 1;
  }
  const char* names[] = {"gsync (counters + go word)", "flags, all poll", "flags, wg0 polls + go word",
                         "flags, XCD lines, all poll", "flags XCD lines, wg0 polls + go word",
                         "flags XCD lines, wg0 polls + 8 go copies", "flags, wg0 polls + 8 go copies"};
  struct Cfg { int mode, ncp; };
  for (Cfg c : {Cfg{0, 1}, Cfg{6, 8}, Cfg{6, 16}, Cfg{6, 32}, Cfg{6, 64}, Cfg{8, 1}, Cfg{14, 8}, Cfg{14, 16},
                Cfg{14, 32}, Cfg{14, 64}}) {
    const int mode = c.mode, ncp = c.ncp;
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      HIP_OK(hipMemset(bar, 0, 64 * 64 * 4));
      const unsigned tmo = 20000000u;  // 0.2 s in 100 MHz ticks
      for (int k = 0; k < 64; ++k) HIP_OK(hipMemcpy(bar + 64 * k + BAR_TMO, &tmo, 4, hipMemcpyHostToDevice));
      HIP_OK(hipMemset(flags, 0, 256 * 4));
      HIP_OK(hipEventRecord(e0));
      hipLaunchKernelGGL(bar_kernel, dim3(256), dim3(512), 0, 0, bar, flags, data, iters, mode, out, ncp);
      HIP_OK(hipEventRecord(e1));
      HIP_OK(hipEventSynchronize(e1));
      float ms = 0.f;
      HIP_OK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    unsigned err = 0, berr = 0;
    HIP_OK(hipMemcpyFromSymbol(&err, HIP_SYMBOL(g_err), 4));
    for (int k = 0; k < 64; ++k) {
      unsigned e = 0;
      HIP_OK(hipMemcpy(&e, bar + 64 * k + 16, 4, hipMemcpyDeviceToHost));
      berr |= e;
    }
    std::printf("{\"mode\": %d, \"form\": \"%s\", \"handoff\": %d, \"go_copies\": %d, \"us_per_barrier\": %.3f, \"err\": %u}\n", mode,
                names[mode & 7], mode >> 3, ncp, best * 1000.f / iters, err | berr);
    if (err | berr) return 1;
  }
  {  // load latency matrix (XCD x candidate block)
    unsigned *pool, *lat;
    HIP_OK(hipMalloc(&pool, (size_t)LAT_NC * 4096));
    HIP_OK(hipMemset(pool, 0, (size_t)LAT_NC * 4096));
    HIP_OK(hipMalloc(&lat, 8 * (LAT_NC + 1) * 4));
    std::vector<unsigned> h(8 * (LAT_NC + 1));
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(lat_kernel, dim3(8), dim3(64), 0, 0, pool, lat);
      HIP_OK(hipDeviceSynchronize());
    }
    HIP_OK(hipMemcpy(h.data(), lat, h.size() * 4, hipMemcpyDeviceToHost));
    for (int w = 0; w < 8; ++w) {
      std::printf("{\"lat_xcc\": %u, \"ns_per_load\": [", h[w * (LAT_NC + 1) + LAT_NC]);
      for (int c = 0; c < LAT_NC; ++c) std::printf("%s%.0f", c ? ", " : "", h[w * (LAT_NC + 1) + c] * 10.0 / LAT_NCH);
      std::printf("]}\n");
    }
  }
  // placement: the flag barrier (mode 6, 8 go copies) on barrier blocks at different offsets of one
  // 64 MiB allocation (8 KiB steps, then 2 MiB steps): does the block's physical place matter?
  {
    unsigned* big;
    HIP_OK(hipMalloc(&big, 64u << 20));
    auto run_at = [&](size_t off_bytes, int hand) {
      unsigned* b = big + off_bytes / 4;
      unsigned* fl = b + 16 * 64;  // flags after the 64 go-copy lines (words 0 .. 1023)
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        HIP_OK(hipMemset(b, 0, 64 * 64 * 4 + 1024));
        const unsigned tmo = 20000000u;
        for (int k = 0; k < 8; ++k) HIP_OK(hipMemcpy(b + 64 * k + BAR_TMO, &tmo, 4, hipMemcpyHostToDevice));
        int it = iters / 2, md = 6 + 8 * hand, nc = 8;
        HIP_OK(hipEventRecord(e0));
        hipLaunchKernelGGL(bar_kernel, dim3(256), dim3(512), 0, 0, b, fl, data, it, md, out, nc);
        HIP_OK(hipEventRecord(e1));
        HIP_OK(hipEventSynchronize(e1));
        float ms = 0.f;
        HIP_OK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      return best * 1000.f / (iters / 2);
    };
    for (int hand = 0; hand < 2; ++hand) {
      std::printf("{\"placement\": \"8KiB steps\", \"handoff\": %d, \"us\": [", hand);
      for (int k = 0; k < 16; ++k) std::printf("%s%.3f", k ? ", " : "", run_at((size_t)k * 4096 * 2, hand));
      std::printf("]}\n{\"placement\": \"2MiB steps\", \"handoff\": %d, \"us\": [", hand);
      for (int k = 0; k < 16; ++k) std::printf("%s%.3f", k ? ", " : "", run_at((size_t)k * (2u << 20) + 8192 * 17, hand));
      std::printf("]}\n");
    }
    unsigned err = 0;
    HIP_OK(hipMemcpyFromSymbol(&err, HIP_SYMBOL(g_err), 4));
    if (err) return 1;
  }
  const void* rk[] = {(const void*)ring_kernel<0>, (const void*)ring_kernel<1>, (const void*)ring_kernel<2>,
                      (const void*)ring_kernel<4>};
  const int sls[] = {0, 1, 2, 4};
  for (int hand = 0; hand < 2; ++hand)
    for (int k = 0; k < 4; ++k) {
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        HIP_OK(hipMemset(bar, 0, 64 * 64 * 4));
        HIP_OK(hipMemset(flags, 0, 256 * 4));
        int it = iters, hd = hand;
        void* args[] = {&bar, &flags, &data, &it, &hd, &out};
        HIP_OK(hipEventRecord(e0));
        HIP_OK(hipLaunchKernel(rk[k], dim3(256), dim3(512), args, 0, 0));
        HIP_OK(hipEventRecord(e1));
        HIP_OK(hipEventSynchronize(e1));
        float ms = 0.f;
        HIP_OK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      unsigned err = 0;
      HIP_OK(hipMemcpyFromSymbol(&err, HIP_SYMBOL(g_err), 4));
      std::printf("{\"form\": \"flags, wg0 ring-polls + 8 go copies, ring polls\", \"sleep\": %d, \"handoff\": %d, "
                  "\"us_per_barrier\": %.3f, \"err\": %u}\n", sls[k], hand, best * 1000.f / iters, err);
      if (err) return 1;
    }
  return 0;
}
