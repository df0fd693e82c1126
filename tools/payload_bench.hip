// Next-round candidate: the decoder's P5 hand-off stream as 24-bit fixed point
// instead of fp32. 256 workgroups x 512 threads; every iteration each workgroup rewrites its slice of
// the block (sc1), a flag barrier, then every wave streams its part of the block, one k-step of loads
// ahead, splits each value into f16 hi / lo and feeds the split-f16 MFMA form (3 MFMAs per product),
// as gemm_x3_hatt_ctx does.
//   mode 0: fp32 payload, 16 values per lane per k-step in 4 x 16 B (192 KB block)
//   mode 1: 24-bit payload (value = int24 * 2^-23, |value| < 1), 16 values in 3 x 16 B (144 KB)
//   mode 2: barriers and rewrites only
//   mode 3: the fp32 block's bytes published pre-split ([hi 4 | lo 4] per 16 bytes): the f16 MFMA
//           operands come straight from the loads, no split on the consumer
//   mode 4: as 3 with the halves laid out so that each 16-byte load is one whole operand (the hi
//           of 8 k in one slot, their lo in the other): no operand moves either
//   mode 5: mode 3's layout read with 8-byte loads straight into the operand halves (hi of k 0..3
//           and of k 4..7 into one operand, their lo into the other): no moves, twice the loads
// Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/payload_bench.hip -o tools/payload_bench
#include "../tts_amd/csrc/gsync.h"
#include "../tts_amd/csrc/split16.h"

#include <cstdio>

constexpr int NKS = 6;

__device__ __forceinline__ int sx24(unsigned x) { return ((int)(x << 8)) >> 8; }

template <int MODE>
__global__ __launch_bounds__(512) void payload_kernel(unsigned* bar, float* act, int iters, float* out) {
  __shared__ int flag;
  unsigned gen = 0;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int NLD = MODE == 1 ? 3 : 4;       // 16-byte loads per lane per k-step (modes 0, 3: 4)
  constexpr int STEP = NLD * 16 * 64;          // bytes per wave per k-step
  constexpr int BLOCK = 8 * NKS * STEP;
  h8 wh, wl;
  for (int j = 0; j < 8; ++j) wh[j] = (_Float16)(0.01f * (j + 1)), wl[j] = (_Float16)(0.001f * j);
  f32x4 am = {0, 0, 0, 0}, ac = {0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    if (MODE != 2) {
      f32x4 x[2][NLD];
      auto ld = [&](f32x4 (&d)[NLD], int k) {
#pragma unroll
        for (int j = 0; j < NLD; ++j) d[j] = ldc4(act, wave * NKS * STEP + k * STEP + (j * 64 + lane) * 16);
      };
      // mode 5: y[buf][2 h] = hi operand, y[buf][2 h + 1] = lo operand of pair h, from 8-byte loads
      f32x4 y[2][NLD];
      auto ld5 = [&](f32x4 (&d)[NLD], int k) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int o0 = wave * NKS * STEP + k * STEP + ((2 * h) * 64 + lane) * 16;
          const int o1 = wave * NKS * STEP + k * STEP + ((2 * h + 1) * 64 + lane) * 16;
          const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)act, 0, 0x7fffffff, 0x00020000);
          typedef unsigned u2 __attribute__((ext_vector_type(2)));
          const u2 a0 = __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(r, o0, 0, 16));
          const u2 b0 = __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(r, o1, 0, 16));
          const u2 a1 = __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(r, o0 + 8, 0, 16));
          const u2 b1 = __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(r, o1 + 8, 0, 16));
          d[2 * h] = f32x4{__uint_as_float(a0[0]), __uint_as_float(a0[1]), __uint_as_float(b0[0]), __uint_as_float(b0[1])};
          d[2 * h + 1] = f32x4{__uint_as_float(a1[0]), __uint_as_float(a1[1]), __uint_as_float(b1[0]), __uint_as_float(b1[1])};
        }
      };
      if constexpr (MODE == 5) ld5(y[0], 0);
      else ld(x[0], 0);
#pragma unroll
      for (int k = 0; k < NKS; ++k) {
        if (k + 1 < NKS) {
          if constexpr (MODE == 5) ld5(y[(k + 1) & 1], k + 1);
          else ld(x[(k + 1) & 1], k + 1);
        }
        if constexpr (MODE == 5) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f32x4 a = y[k & 1][2 * h], b = y[k & 1][2 * h + 1];
            mfma_x3(wh, wl, __builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), am, ac);
          }
          continue;
        }
        if constexpr (MODE == 4) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
            mfma_x3(wh, wl, __builtin_bit_cast(h8, x[k & 1][2 * h]), __builtin_bit_cast(h8, x[k & 1][2 * h + 1]), am, ac);
          continue;
        }
        if constexpr (MODE == 3) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f32x4 a = x[k & 1][2 * h], b = x[k & 1][2 * h + 1];
            const f32x4 hi4 = {a[0], a[1], b[0], b[1]}, lo4 = {a[2], a[3], b[2], b[3]};
            const h8 xh = __builtin_bit_cast(h8, hi4), xl = __builtin_bit_cast(h8, lo4);
            mfma_x3(wh, wl, xh, xl, am, ac);
          }
          continue;
        }
        float v[16];
        if constexpr (MODE == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) v[4 * j + q] = x[k & 1][j][q];
        } else {
          unsigned d[12];
#pragma unroll
          for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) d[4 * j + q] = __float_as_uint(x[k & 1][j][q]);
#pragma unroll
          for (int g = 0; g < 4; ++g) {  // 3 dwords -> 4 values
            const unsigned a = d[3 * g], b = d[3 * g + 1], c = d[3 * g + 2];
            const int i0 = sx24(a), i1 = sx24(__builtin_amdgcn_alignbit(b, a, 24)),
                      i2 = sx24(__builtin_amdgcn_alignbit(c, b, 16)), i3 = ((int)c) >> 8;
            v[4 * g] = (float)i0 * (1.f / 8388608.f);
            v[4 * g + 1] = (float)i1 * (1.f / 8388608.f);
            v[4 * g + 2] = (float)i2 * (1.f / 8388608.f);
            v[4 * g + 3] = (float)i3 * (1.f / 8388608.f);
          }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float e[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = v[8 * h + j];
          h8 xh, xl;
          split8(e, xh, xl);
          mfma_x3(wh, wl, xh, xl, am, ac);
        }
      }
    }
    // producers: each workgroup rewrites its 1/256 of the block (sc1)
    if (threadIdx.x * 16 < BLOCK / 256) stc4(act, (blockIdx.x * (BLOCK / 256) + threadIdx.x * 16), am * 0.f);
    gflag_arrive(bar, gen);
    if (!gflag_wait(bar, gen, &flag)) return;
  }
  out[blockIdx.x * 512 + threadIdx.x] = am[0] + ac[1];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  unsigned* pool;
  float *act, *out;
  HIP_OK(hipMalloc(&pool, 16 * BAR_WORDS * 4));
  HIP_OK(hipMalloc(&act, 192 * 1024));
  HIP_OK(hipMemset(act, 0, 192 * 1024));
  HIP_OK(hipMalloc(&out, 256 * 512 * 4));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  const void* ks[] = {(const void*)payload_kernel<0>, (const void*)payload_kernel<1>, (const void*)payload_kernel<2>,
                      (const void*)payload_kernel<3>, (const void*)payload_kernel<4>,
                      (const void*)payload_kernel<5>};
  const char* names[] = {"fp32 payload (192 KB)", "24-bit payload (144 KB) + unpack", "barriers + rewrites only",
                         "pre-split payload (192 KB, no consumer split)", "pre-split, whole-operand slots (no moves)",
                         "pre-split, 8-byte loads into the operands (no moves)"};
  // the fastest of 4 barrier-block placements, then 2 passes over the modes
  int best_slot = 0;
  float best_t = 1e30f;
  for (int pass = 0; pass < 3; ++pass)
    for (int m = (pass == 0 ? 2 : 0); m < 6; ++m) {
      for (int slot = 0; slot < (pass == 0 ? 4 : 1); ++slot) {
        unsigned* bar = pool + (pass == 0 ? slot : best_slot) * BAR_WORDS;
        float best = 1e30f;
        for (int r = 0; r < 3; ++r) {
          HIP_OK(hipMemset(bar, 0, BAR_WORDS * 4));
          const unsigned tmo = 20000000u;
          HIP_OK(hipMemcpy(bar + BAR_TMO, &tmo, 4, hipMemcpyHostToDevice));
          int it = iters;
          void* args[] = {&bar, &act, &it, &out};
          HIP_OK(hipEventRecord(e0));
          HIP_OK(hipLaunchKernel(ks[m], dim3(256), dim3(512), args, 0, 0));
          HIP_OK(hipEventRecord(e1));
          HIP_OK(hipEventSynchronize(e1));
          float ms = 0.f;
          HIP_OK(hipEventElapsedTime(&ms, e0, e1));
          best = ms < best ? ms : best;
        }
        unsigned err = 0;
        HIP_OK(hipMemcpy(&err, bar + 16, 4, hipMemcpyDeviceToHost));
        if (err) return 1;
        const float us = best * 1000.f / iters;
        if (pass == 0) {
          if (us < best_t) best_t = us, best_slot = slot;
          continue;
        }
        std::printf("{\"mode\": %d, \"what\": \"%s\", \"us_per_iteration\": %.3f}\n", m, names[m], us);
      }
      if (pass == 0) break;
    }
  return 0;
}
