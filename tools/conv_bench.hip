// Microbenchmark for the generic MFMA conv kernel at the postnet / encoder shapes of the C2
// workload (32 LJ-length utterances). Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/conv_bench.hip -o tools/conv_bench
#include "../tts_amd/csrc/conv.hip"

#include <cstdio>
#include <functional>
#include <vector>

static const int kM[32] = {832, 164, 833, 443, 699, 490, 723, 154, 651, 760, 389, 710, 223, 857, 796, 454,
                           605, 645, 553, 403, 742, 608, 728, 677, 764, 525, 831, 511, 459, 596, 677, 610};
static hipStream_t S;

static float time_graph(const std::function<void()>& body, int per_graph = 4, int reps = 5) {
  hipGraph_t g;
  hipGraphExec_t ge;
  HIP_OK(hipStreamBeginCapture(S, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < per_graph; ++i) body();
  HIP_OK(hipStreamEndCapture(S, &g));
  HIP_OK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  HIP_OK(hipGraphLaunch(ge, S));
  HIP_OK(hipStreamSynchronize(S));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  HIP_OK(hipEventRecord(e0, S));
  for (int r = 0; r < reps; ++r) HIP_OK(hipGraphLaunch(ge, S));
  HIP_OK(hipEventRecord(e1, S));
  HIP_OK(hipEventSynchronize(e1));
  float ms;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  HIP_OK(hipGraphExecDestroy(ge));
  HIP_OK(hipGraphDestroy(g));
  return ms * 1000.f / (per_graph * reps);
}

static float* dalloc(size_t n) {
  float* p;
  HIP_OK(hipMalloc(&p, n * 4));
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = 0.01f * (float)((i * 2654435761u) % 1000) / 1000.f - 0.005f;
  HIP_OK(hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice));
  return p;
}

template <int MI, int NI, int WM, int WN, int KT>
static void variant(const char* name, const ConvArgs& a, int TQ, int TC, double flop) {
  const int span = (a.K - 1) * a.dil;
  const size_t lds = (size_t)(2 * ((16 * (TQ + span + 1) + 3) & ~3) + 16 * a.K) * 4;
  dim3 grid((a.max_q + TQ - 1) / TQ, a.Cout_pad / TC, a.B * a.nphase);
  const float us = time_graph([&] { conv_mfma_kernel<MI, NI, WM, WN, KT><<<grid, 256, lds, S>>>(a); });
  printf("%-40s %8.1f us  %6.1f TF/s\n", name, us, flop / (us * 1e-6) / 1e12);
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  HIP_OK(hipStreamCreate(&S));
  int* lens;
  HIP_OK(hipMalloc(&lens, 32 * 4));
  HIP_OK(hipMemcpy(lens, kM, 32 * 4, hipMemcpyHostToDevice));
  const int Mmax = 857;
  double frames = 0;
  for (int b = 0; b < 32; ++b) frames += kM[b];
  // postnet 512 -> 512, k5, tanh: activations (B, 512, Mmax) channel-major
  {
    ConvArgs a{};
    float* x = dalloc((size_t)32 * 512 * Mmax);
    float* y = dalloc((size_t)32 * 512 * Mmax);
    a.src[0] = ConvSrc{x, (long)512 * Mmax, Mmax, 1, 512, 0};
    a.src[1] = a.src[0];
    a.Cin = 512;
    a.K = 5;
    a.dil = 1;
    a.pad_mode = 0;
    a.lens = lens;
    a.len_add = 0;
    a.in_mul = a.q_mul = 1;
    a.rep_pad = 0;
    a.nphase = 1;
    a.pad_left[0] = 2;
    a.w_phase_stride = 0;
    a.W = dalloc((size_t)512 * 512 * 5);
    a.bias = dalloc(512);
    a.Cout = a.Cout_pad = 512;
    a.out = y;
    a.ob = (long)512 * Mmax;
    a.oc = Mmax;
    a.ot = 1;
    a.out_mul = 1;
    a.epi_act = 2;
    a.resid = nullptr;
    a.max_q = Mmax;
    a.B = 32;
    const double flop = 2.0 * 512 * 512 * 5 * frames;
    variant<4, 2, 2, 2, 0>("postnet 512->512 k5 128x64 (current)", a, 64, 128, flop);
    variant<4, 2, 2, 2, 5>("postnet 512->512 k5 128x64 ring5", a, 64, 128, flop);
    variant<2, 2, 2, 2, 5>("postnet 512->512 k5 64x64 ring5", a, 64, 64, flop);
    variant<4, 4, 2, 2, 5>("postnet 512->512 k5 128x128 ring5", a, 128, 128, flop);
    variant<2, 4, 2, 2, 5>("postnet 512->512 k5 64x128 ring5", a, 128, 64, flop);
    variant<4, 4, 2, 2, 0>("postnet 512->512 k5 128x128", a, 128, 128, flop);
  }
  printf("done\n");
  return 0;
}
