// Microbenchmark for the fused ResidualStack block kernel at the MB-MelGAN stage shapes of the
// C2 workload (32 LJ-length utterances, M from tests/golden/lj_profile.json). Not part of the
// library:  hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/voc_bench.hip -o tools/voc_bench
#include "../tts_amd/csrc/resblock.hip"

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

template <int C, int TQ, int WM, int WN>
static void variant(const char* name, ResArgs a) {
  double flop = 0;
  for (int b = 0; b < 32; ++b) flop += 2.0 * C * 5 * C * (double)(kM[b] * a.mul);
  float tot = 0;
  for (int dil : {1, 3, 9, 27}) {
    a.dil = dil;
    tot += time_graph([&] { launch_rb<C, TQ, WM, WN>(a, S); });
  }
  printf("C=%3d %-22s 4 blocks %8.1f us  %6.1f TF/s\n", C, name, tot, 4 * flop / (tot * 1e-6) / 1e12);
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  HIP_OK(hipStreamCreate(&S));
  int* lens;
  HIP_OK(hipMalloc(&lens, 32 * 4));
  HIP_OK(hipMemcpy(lens, kM, 32 * 4, hipMemcpyHostToDevice));
  int Mmax = 0;
  for (int b = 0; b < 32; ++b) Mmax = std::max(Mmax, kM[b]);
  for (int stage = 0; stage < 3; ++stage) {
    const int C = 192 >> stage, mul = stage == 0 ? 8 : stage == 1 ? 32 : 64;
    const int Ls = Mmax * mul;
    ResArgs a{};
    a.x = dalloc((size_t)32 * C * Ls);
    a.y = dalloc((size_t)32 * C * Ls);
    a.sb = (long)C * Ls;
    a.Ls = Ls;
    a.lens = lens;
    a.len_add = 0;
    a.mul = mul;
    a.Wd = dalloc((size_t)3 * C * C);
    a.bd = dalloc(C);
    a.Wf = dalloc((size_t)2 * C * C);
    a.bf = dalloc(C);
    a.max_q = Ls;
    a.B = 32;
    if (C == 192) {
      variant<192, 32, 4, 1>("TQ32 4x1 (current)", a);
      variant<192, 64, 4, 2>("TQ64 4x2 (8 waves)", a);
      variant<192, 32, 4, 2>("TQ32 4x2 (8 waves)", a);
    } else if (C == 96) {
      variant<96, 64, 2, 2>("TQ64 2x2 (current)", a);
      variant<96, 128, 2, 4>("TQ128 2x4 (8 waves)", a);
      variant<96, 64, 2, 4>("TQ64 2x4 (8 waves)", a);
    } else {
      variant<48, 128, 1, 4>("TQ128 1x4 (current)", a);
      variant<48, 64, 1, 4>("TQ64 1x4", a);
      variant<48, 128, 1, 8>("TQ128 1x8 (8 waves)", a);
    }
    HIP_OK(hipFree((void*)a.x));
    HIP_OK(hipFree(a.y));
  }
  printf("done\n");
  return 0;
}
