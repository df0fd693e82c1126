// P5-like broadcast stream: 256 workgroups x 512 threads, every workgroup reads
// the same 192 KB activation block with sc1 loads, one k-step of loads ahead per wave (as the
// decoder's gemm_x3_hatt_ctx), between flag barriers. Does the order in which the 32 workgroups of
// an XCD walk the block matter (all on the same lines at once vs rotated starts)?
//   mode 0: every workgroup walks k-steps 0 .. NKS-1
//   mode 1: workgroup g starts at k-step (g / 8) % NKS (the XCD's workgroups spread over the lines)
//   mode 2: barriers only (the floor to subtract)
//   mode 3: two k-steps of loads ahead (mode 0 order)
//   mode 4: mode 0 without the rewrite (the block stays valid in every XCD's L2)
//   mode 5: mode 0 with plain loads (not a valid hand-off: L1 may serve stale lines; timing only)
//   mode 6: mode 0, and wave 0 of each workgroup first touches its 1/32 share of the block's lines
//           (workgroups g and g + 8 k share an XCD: share (g / 8) % 32), so that each XCD's L2
//           requests all of the block at once instead of line by line behind the k-steps
//   mode 7: rewrite, barrier, each XCD's workgroups touch the whole block (full 128-byte lines,
//           8 lanes x 16 B each, 1/32 of the lines per workgroup), barrier, then mode 0's stream
//   mode 8: as mode 7 with one 4-byte load per line
//   mode 9: as mode 7 without the touch (its baseline: two barriers per iteration)
// Every workgroup rewrites its 1/256 of the block before each barrier, so the lines the next pass
// reads were last written by another XCD (as the decoder's hand-offs).
// Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_bench.hip -o tools/stream_bench
#include "../tts_amd/csrc/gsync.h"

#include <cstdio>
#include <vector>

constexpr int NKS = 6;                 // k-steps per wave (4 h_att + 2 ctx)
constexpr int STEP_BYTES = 4096;       // per wave per k-step: 2 m-tiles x 2 x 16 B x 64 lanes
constexpr int WAVE_BYTES = NKS * STEP_BYTES;
constexpr int BLOCK_BYTES = 8 * WAVE_BYTES;  // 192 KB

template <int AUX = 16>
__device__ __forceinline__ void ld_step(f32x4 (&x)[4], const float* base, int wave, int k, int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) x[j] = ldc4<AUX>(base, wave * WAVE_BYTES + k * STEP_BYTES + (j * 64 + lane) * 16);
}

template <int MODE>
__global__ __launch_bounds__(512) void stream_kernel(unsigned* bar, float* act, int iters, float* out) {
  __shared__ int flag;
  unsigned gen = 0;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rot = MODE == 1 ? (int)(blockIdx.x / 8) % NKS : 0;
  f32x4 acc = {0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    if (MODE >= 7) {  // rewrite, barrier, touch (or not), barrier; the stream below
      if (threadIdx.x < 48) stc4(act, (blockIdx.x * 48 + threadIdx.x) * 16, acc * 1e-30f);
      gflag_arrive(bar, gen);
      if (!gflag_wait(bar, gen, &flag)) return;
      const int sh = (int)(blockIdx.x / 8) % 32;  // 1536 lines, 48 per workgroup of an XCD
      if (MODE == 7 && wave < 6) {                // 6 waves x 8 lines x 8 lanes x 16 B
        const f32x4 t = ldc4(act, ((sh + 32 * (8 * wave + lane / 8)) * 128) + (lane & 7) * 16);
        acc += t * 1e-30f;
      }
      if (MODE == 8 && wave == 0 && lane < 48) acc[0] += ldc(act + (sh + 32 * lane) * 32) * 1e-30f;
      gflag_arrive(bar, gen);
      if (!gflag_wait(bar, gen, &flag)) return;
    }
    if (MODE == 0 || MODE == 1 || MODE == 4 || MODE == 5 || MODE == 6 || MODE >= 7) {
      constexpr int AUX = MODE == 5 ? 0 : 16;
      if (MODE == 6 && wave == 0) {
        // 1536 lines of 128 B; this workgroup's share: lines sh + 32 i, i < 48; lane L of load j
        // reads 16 B of line sh + 32 (8 j + L / 8) (8 lanes per line)
        const int sh = (int)(blockIdx.x / 8) % 32;
        f32x4 t = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 6; ++j) t += ldc4(act, ((sh + 32 * (8 * j + lane / 8)) * 128) + (lane & 7) * 16);
        acc += t * 1e-30f;
      }
      f32x4 x[2][4];
      ld_step<AUX>(x[0], act, wave, rot, lane);
#pragma unroll
      for (int k = 0; k < NKS; ++k) {
        if (k + 1 < NKS) {
          int kk = k + 1 + rot;
          kk = kk >= NKS ? kk - NKS : kk;
          ld_step<AUX>(x[(k + 1) & 1], act, wave, kk, lane);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = acc * 0.999f + x[k & 1][j];
      }
    } else if (MODE == 3) {
      f32x4 x[3][4];
      ld_step(x[0], act, wave, 0, lane);
      ld_step(x[1], act, wave, 1, lane);
#pragma unroll
      for (int k = 0; k < NKS; ++k) {
        if (k + 2 < NKS) ld_step(x[(k + 2) % 3], act, wave, k + 2, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = acc * 0.999f + x[k % 3][j];
      }
    }
    // producers: every workgroup rewrites its 768-byte slice of the block (sc1), as P3 / P4 do
    if (MODE != 2 && MODE != 4 && MODE < 7 && threadIdx.x < 48) stc4(act, (blockIdx.x * 48 + threadIdx.x) * 16, acc * 1e-30f);
    gflag_arrive(bar, gen);
    if (!gflag_wait(bar, gen, &flag)) return;
  }
  out[blockIdx.x * 512 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  unsigned* bar;
  float *act, *out;
  HIP_OK(hipMalloc(&bar, BAR_WORDS * 4));
  HIP_OK(hipMalloc(&act, BLOCK_BYTES));
  HIP_OK(hipMemset(act, 0, BLOCK_BYTES));
  HIP_OK(hipMalloc(&out, 256 * 512 * 4));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  const void* ks[] = {(const void*)stream_kernel<0>, (const void*)stream_kernel<1>, (const void*)stream_kernel<2>,
                      (const void*)stream_kernel<3>, (const void*)stream_kernel<4>, (const void*)stream_kernel<5>,
                      (const void*)stream_kernel<6>, (const void*)stream_kernel<7>, (const void*)stream_kernel<8>,
                      (const void*)stream_kernel<9>};
  const char* names[] = {"same order", "rotated start per XCD slot", "barriers only", "two k-steps ahead",
                         "no rewrite (L2-valid block)", "plain loads (timing only)", "XCD-shared line touch first",
                         "touch full lines one barrier ahead", "touch one dword per line one barrier ahead",
                         "two barriers, no touch (baseline of 7 / 8)"};
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 10; ++m) {
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
      std::printf("{\"mode\": %d, \"what\": \"%s\", \"us_per_iteration\": %.3f, \"err\": %u}\n", m, names[m],
                  best * 1000.f / iters, err);
      if (err) return 1;
    }
  return 0;
}
