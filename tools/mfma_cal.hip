// Calibration of the MFMA PMC counters (VERDICT r04 "Calibrate the MFMA counter"): kernels with a
// known number of MFMAs per wave, run under the same rocprofv3 --pmc sets as the library's kernels
// (tools/mfma_cal.sh), so that tools/pmc_kernels.py can be checked to read 1.0 on a kernel that
// keeps every SIMD's MFMA pipe busy and the known duty elsewhere.
//
//   kernel            per wave                                          expected pipe share
//   cal_f16_full      N x v_mfma_f32_16x16x32_f16, 4 independent accs   1.0  (one wave per SIMD)
//   cal_f16_half      N x (MFMA + ~16 cycles of dependent VALU)         ~0.5
//   cal_f16k16_full   N x v_mfma_f32_16x16x16_f16, 4 independent accs  1.0 (its cycles per MFMA)
//   cal_f32_full      N x v_mfma_f32_16x16x4_f32, 4 independent accs    1.0
//
// Grid: 256 workgroups x 256 threads (4 waves: one per SIMD on every CU). Each kernel writes its
// accumulators (so nothing is dead code) and prints the expected MFMA count per launch; the
// measured SQ_INSTS_VALU_MFMA_MOPS_* x 512 / FLOP per MFMA must equal it.
// Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_cal.hip -o tools/mfma_cal
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define HIP_OK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

constexpr int N = 20000;  // MFMAs per wave (per accumulator chain: N / 4)

__global__ __launch_bounds__(256) void cal_f16_full(float* out, float seed) {
  h8 a, b;
  for (int i = 0; i < 8; ++i) a[i] = (_Float16)(seed * (threadIdx.x + i)), b[i] = (_Float16)(seed - i);
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < N / 4; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c3, 0, 0, 0);
  }
  const f32x4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// one MFMA, then VALU work that depends on its result (so the next MFMA waits for it): the pipe
// is busy for about half of the wave's cycles
__global__ __launch_bounds__(256) void cal_f16_half(float* out, float seed) {
  h8 a, b;
  for (int i = 0; i < 8; ++i) a[i] = (_Float16)(seed * (threadIdx.x + i)), b[i] = (_Float16)(seed - i);
  f32x4 c = {0, 0, 0, 0};
  float x = seed;
  for (int i = 0; i < N; ++i) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    x = __builtin_fmaf(x, c[0], 1.0f);
#pragma unroll
    for (int k = 0; k < 3; ++k) x = __builtin_fmaf(x, x, 0.5f);
    a[0] = (_Float16)x;
  }
  out[blockIdx.x * 256 + threadIdx.x] = c[0] + c[1] + c[2] + c[3] + x;
}

// the K = 16 f16 MFMA (half the work of the K = 32 form): does it take half the cycles on gfx950?
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void cal_f16k16_full(float* out, float seed) {
  h4 a, b;
  for (int i = 0; i < 4; ++i) a[i] = (_Float16)(seed * (threadIdx.x + i)), b[i] = (_Float16)(seed - i);
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < N / 4; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c3, 0, 0, 0);
  }
  const f32x4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ __launch_bounds__(256) void cal_f32_full(float* out, float seed) {
  const float a = seed * threadIdx.x, b = seed - 1.f;
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < N / 4; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
  }
  const f32x4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

int main() {
  float* out;
  HIP_OK(hipMalloc(&out, 256 * 256 * 4));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  const long waves = 256L * 4;
  struct K {
    const char* name;
    void (*f)(float*, float);
    double flop_per_mfma;
  } ks[] = {{"cal_f16_full", cal_f16_full, 16.0 * 16 * 32 * 2},
            {"cal_f16_half", cal_f16_half, 16.0 * 16 * 32 * 2},
            {"cal_f16k16_full", cal_f16k16_full, 16.0 * 16 * 16 * 2},
            {"cal_f32_full", cal_f32_full, 16.0 * 16 * 4 * 2}};
  for (const K& k : ks) {
    for (int rep = 0; rep < 12; ++rep) {
      HIP_OK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(256), dim3(256), 0, 0, out, 0.001f);
      HIP_OK(hipEventRecord(e1));
      HIP_OK(hipEventSynchronize(e1));
      float ms = 0.f;
      HIP_OK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 11)
        std::printf("{\"kernel\": \"%s\", \"mfma_per_launch\": %ld, \"flop_per_launch\": %.6e, \"ms\": %.4f, "
                    "\"tflops\": %.1f}\n",
                    k.name, waves * N, waves * N * k.flop_per_mfma, ms, waves * N * k.flop_per_mfma / ms * 1e-9);
    }
  }
  HIP_OK(hipDeviceSynchronize());
  return 0;
}
