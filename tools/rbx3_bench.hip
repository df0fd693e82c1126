// Split-f16 ResidualStack block: correctness against a double-precision CPU restatement of the
// block (melgan.py:35-39) on ragged utterances, then timing against the fp32 kernel at the
// MB-MelGAN stage shapes of the C2 workload. Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/rbx3_bench.hip -o tools/rbx3_bench
#include "../tts_amd/csrc/resblock.hip"
#ifdef RB_TRACE
__device__ unsigned long long* rb_trace;
#endif
#include "../tts_amd/csrc/resblock_x3.hip"

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <functional>
#include <random>
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

template <class T>
static T* dup(const std::vector<T>& h) {
  T* p;
  HIP_OK(hipMalloc(&p, h.size() * sizeof(T)));
  HIP_OK(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

static double lrelu_d(double v) { return v >= 0 ? v : 0.2 * v; }
static int g_variant = 0;  // check(): 0 the library tile, 1..3 the CPB sweep variants

// CPU block on utterance b: x (C, Ls) -> y (C, L)
static void cpu_block(const float* x, int C, int Ls, int L, int d, const std::vector<float>& wd,
                      const std::vector<float>& bd, const std::vector<float>& wf, const std::vector<float>& bf,
                      std::vector<double>& y) {
  std::vector<double> h((size_t)C * L);
  auto refl = [&](int i) { return i < 0 ? -i : (i >= L ? 2 * (L - 1) - i : i); };
  for (int co = 0; co < C; ++co)
    for (int p = 0; p < L; ++p) {
      double s = bd[co];
      for (int ci = 0; ci < C; ++ci)
        for (int k = 0; k < 3; ++k) s += (double)wd[((size_t)co * C + ci) * 3 + k] * lrelu_d(x[(size_t)ci * Ls + refl(p + (k - 1) * d)]);
      h[(size_t)co * L + p] = lrelu_d(s);
    }
  y.assign((size_t)C * L, 0.0);
  for (int co = 0; co < C; ++co)
    for (int p = 0; p < L; ++p) {
      double s = bf[co];
      for (int k = 0; k < C; ++k) s += (double)wf[(size_t)co * 2 * C + k] * h[(size_t)k * L + p];
      for (int k = 0; k < C; ++k) s += (double)wf[(size_t)co * 2 * C + C + k] * x[(size_t)k * Ls + p];
      y[(size_t)co * L + p] = s;
    }
}

static int check(int C, int d, float xscale) {
  std::mt19937 rng(C * 100 + d);
  std::normal_distribution<float> nd(0.f, 1.f);
  const int B = 3, lens[3] = {301, d < 7 ? 7 : 60, 130}, Ls = 320;  // reflection needs L > d
  std::vector<float> x((size_t)B * C * Ls), wd((size_t)C * C * 3), bd(C), wf((size_t)C * 2 * C), bf(C);
  for (auto& v : x) v = xscale * nd(rng);
  const float sw = 1.f / std::sqrt(3.f * C);
  for (auto& v : wd) v = sw * nd(rng);
  for (auto& v : wf) v = sw * nd(rng);
  for (auto& v : bd) v = 0.1f * nd(rng);
  for (auto& v : bf) v = 0.1f * nd(rng);
  std::vector<uint16_t> wd16, wf16;
  pack_resblock_x3(wd, wf, C, wd16, wf16);
  ResArgs a{};
  a.x = dup(x);
  std::vector<float> y0((size_t)B * C * Ls, 0.f);
  a.y = dup(y0);
  a.sb = (long)C * Ls;
  a.Ls = Ls;
  a.lens = dup(std::vector<int>(lens, lens + B));
  a.len_add = 0;
  a.mul = 1;
  a.dil = d;
  a.bd = dup(bd);
  a.bf = dup(bf);
  a.Wd16 = dup(wd16);
  a.Wf16 = dup(wf16);
  a.oflow = dup(std::vector<unsigned>(1, 0));
  a.max_q = 301;
  a.B = B;
  if (g_variant == 1) launch_rbx3<192, 48, 12, 1, 3, 2>(a, lens, S);
  else if (g_variant == 2) launch_rbx3<192, 48, 12, 1, 3, 3>(a, lens, S);
  else if (g_variant == 3) launch_rbx3<96, 64, 6, 1, 3, 3>(a, lens, S);
  else launch_resblock_x3(a, lens, C, S);
  HIP_OK(hipStreamSynchronize(S));
  std::vector<float> y((size_t)B * C * Ls);
  HIP_OK(hipMemcpy(y.data(), a.y, y.size() * 4, hipMemcpyDeviceToHost));
  unsigned of = 0;
  HIP_OK(hipMemcpy(&of, a.oflow, 4, hipMemcpyDeviceToHost));
  double err = 0, mag = 0;
  bool untouched = true;
  for (int b = 0; b < B; ++b) {
    std::vector<double> ref;
    cpu_block(&x[(size_t)b * C * Ls], C, Ls, lens[b], d, wd, bd, wf, bf, ref);
    for (int co = 0; co < C; ++co) {
      for (int p = 0; p < lens[b]; ++p) {
        err = std::max(err, std::fabs(y[((size_t)b * C + co) * Ls + p] - ref[(size_t)co * lens[b] + p]));
        mag = std::max(mag, std::fabs(ref[(size_t)co * lens[b] + p]));
      }
      for (int p = lens[b]; p < Ls; ++p) untouched &= y[((size_t)b * C + co) * Ls + p] == 0.f;
    }
  }
  const bool ok = err <= 4e-6 * std::max(1.0, mag) && untouched && of == (xscale > 1e4f ? 1u : 0u);
  printf("check C=%3d d=%2d |x|~%-8g max|err| %.3e (max|y| %.3e) tail untouched %d oflow %u  %s\n", C, d, xscale, err,
         mag, (int)untouched, of, ok ? "OK" : "FAIL");
  return ok ? 0 : 1;
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  HIP_OK(hipStreamCreate(&S));
  const int prof_C = argc > 1 ? std::atoi(argv[1]) : 0;  // profiling mode: one stage, library tile only
  int fails = 0;
  if (!prof_C) {
  for (int C : {48, 96, 192})
    for (int d : {1, 9, 27}) fails += check(C, d, 1.f);
  for (int C : {32, 64, 128, 256}) fails += check(C, 3, 1.f);  // the full-band MelGAN stages
  fails += check(96, 3, 1e-3f);
  // CPB variants (several chunks per barrier): bit-identical to the library tile by construction;
  // checked against the CPU block like it
  g_variant = 1;
  for (int d : {1, 27}) fails += check(192, d, 1.f);
  g_variant = 2;
  for (int d : {1, 27}) fails += check(192, d, 1.f);
  g_variant = 3;
  for (int d : {1, 27}) fails += check(96, d, 1.f);
  g_variant = 0;
  fails += check(96, 3, 1e5f);  // out of the f16 range: must raise the flag
  }
  int* lens;
  HIP_OK(hipMalloc(&lens, 32 * 4));
  HIP_OK(hipMemcpy(lens, kM, 32 * 4, hipMemcpyHostToDevice));
  int Mmax = 0;
  for (int b = 0; b < 32; ++b) Mmax = std::max(Mmax, kM[b]);
  for (int stage = 0; stage < 3; ++stage) {
    if (prof_C && (192 >> stage) != std::abs(prof_C)) continue;
    const int C = 192 >> stage, mul = stage == 0 ? 8 : stage == 1 ? 32 : 64;
    const int Ls = Mmax * mul;
    // random operands (DVFS: constant or zero data clocks higher, MI355X_MICROARCH.md)
    auto rnd = [](size_t n, float sc) {
      std::vector<float> v(n);
      uint32_t s = 12345u + (uint32_t)n;
      for (auto& x : v) {
        s = s * 1664525u + 1013904223u;
        x = sc * ((float)(s >> 8) * (1.f / 8388608.f) - 1.f);
      }
      return v;
    };
    std::vector<float> big = rnd((size_t)32 * C * Ls, 1.f), w = rnd((size_t)3 * C * C, 0.05f), bb(C, 0.f);
    std::vector<uint16_t> wd16, wf16;
    pack_resblock_x3(rnd((size_t)C * C * 3, 0.05f), rnd((size_t)C * 2 * C, 0.05f), C, wd16, wf16);
    ResArgs a{};
    a.x = dup(big);
    a.y = dup(big);
    a.sb = (long)C * Ls;
    a.Ls = Ls;
    a.lens = lens;
    a.mul = mul;
    a.Wd = dup(w);
    a.Wf = dup(w);
    a.bd = a.bf = dup(bb);
    a.Wd16 = dup(wd16);
    a.Wf16 = dup(wf16);
    a.oflow = dup(std::vector<unsigned>(1, 0));
    a.max_q = Ls;
    a.B = 32;
    double flop = 0;
    for (int b = 0; b < 32; ++b) flop += 2.0 * C * 5 * C * (double)(kM[b] * mul);
    auto timeit = [&](const char* name, const std::function<void()>& f) {
      float t = 0;
      for (int dil : {1, 3, 9, 27}) {
        a.dil = dil;
        t += time_graph(f);
      }
      printf("C=%3d  4 blocks %-26s %8.1f us (%6.1f TF/s fp32-equivalent)\n", C, name, t, 4 * flop / (t * 1e-6) / 1e12);
    };
#ifdef RB_TRACE
    if (prof_C < 0) {  // phase stamps of the first 4 tiles of every workgroup, dilation 9
      if (C != -prof_C) continue;
      a.dil = 9;
      std::vector<unsigned long long> h((size_t)256 * 4 * 8, 0);
      unsigned long long* dtr = dup(h);
      HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(rb_trace), &dtr, sizeof(dtr)));
      launch_resblock_x3(a, kM, C, S);
      HIP_OK(hipStreamSynchronize(S));
      HIP_OK(hipMemcpy(h.data(), dtr, h.size() * 8, hipMemcpyDeviceToHost));
      double seg[5] = {0};
      int n = 0;
      for (int w = 0; w < 256; ++w)
        for (int i = 1; i < 3; ++i) {  // tiles 1, 2: steady state
          const unsigned long long* r = &h[((size_t)w * 4 + i) * 8];
          const unsigned long long* rn = &h[((size_t)w * 4 + i + 1) * 8];
          if (!r[0] || !r[5] || !rn[0]) continue;
          seg[0] += (r[1] - r[0]) * 0.01;
          seg[1] += (r[2] - r[1]) * 0.01;
          seg[2] += (r[3] - r[2]) * 0.01;
          seg[3] += (r[5] - r[3]) * 0.01;
          seg[4] += (rn[0] - r[5]) * 0.01;
          ++n;
        }
      printf("C=%d trace (us per tile, mean of %d): phase 1 %.2f, h split %.2f, phase 2 %.2f, stores+sync %.2f, "
             "next-tile store+sync %.2f\n", C, n, seg[0] / n, seg[1] / n, seg[2] / n, seg[3] / n, seg[4] / n);
      continue;
    }
#endif
    if (prof_C) {
      a.dil = 9;
      for (int i = 0; i < 5; ++i) launch_resblock_x3(a, kM, C, S);
      HIP_OK(hipStreamSynchronize(S));
      continue;
    }
    timeit("fp32", [&] { launch_resblock(a, C, S); });
    timeit("split-f16 (library tile)", [&] { launch_resblock_x3(a, kM, C, S); });
    if (C == 192) {
      timeit("x3 TQ64 12x1", [&] { launch_rbx3<192, 64, 12, 1, 3>(a, kM, S); });
      timeit("x3 TQ48 12x1 (NI3)", [&] { launch_rbx3<192, 48, 12, 1, 3>(a, kM, S); });
      timeit("x3 TQ32 12x1 (NI2)", [&] { launch_rbx3<192, 32, 12, 1, 3>(a, kM, S); });
      timeit("x3 TQ64 4x2 (MI3 NI2)", [&] { launch_rbx3<192, 64, 4, 2, 3>(a, kM, S); });
      timeit("x3 TQ64 4x1 (MI3 NI4)", [&] { launch_rbx3<192, 64, 4, 1, 3>(a, kM, S); });
      timeit("x3 TQ64 6x2 (MI2 NI2)", [&] { launch_rbx3<192, 64, 6, 2, 3>(a, kM, S); });
      timeit("x3 TQ48 12x1 CPB2", [&] { launch_rbx3<192, 48, 12, 1, 3, 2>(a, kM, S); });
      timeit("x3 TQ48 12x1 CPB3", [&] { launch_rbx3<192, 48, 12, 1, 3, 3>(a, kM, S); });
      timeit("x3 TQ64 12x1 R6", [&] { launch_rbx3<192, 64, 12, 1, 6>(a, kM, S); });
      timeit("x3 TQ64 6x1 (MI2 NI4)", [&] { launch_rbx3<192, 64, 6, 1, 3>(a, kM, S); });
    } else if (C == 96) {
      timeit("x3 TQ128 6x2", [&] { launch_rbx3<96, 128, 6, 2, 3>(a, kM, S); });
      timeit("x3 TQ96 6x2 (NI3)", [&] { launch_rbx3<96, 96, 6, 2, 3>(a, kM, S); });
      timeit("x3 TQ64 6x2 (NI2)", [&] { launch_rbx3<96, 64, 6, 2, 3>(a, kM, S); });
      timeit("x3 TQ96 2x2 (MI3 NI3)", [&] { launch_rbx3<96, 96, 2, 2, 3>(a, kM, S); });
      timeit("x3 TQ128 2x4 (MI3 NI2)", [&] { launch_rbx3<96, 128, 2, 4, 3>(a, kM, S); });
      timeit("x3 TQ64 6x2 CPB3 (NI2)", [&] { launch_rbx3<96, 64, 6, 2, 3, 3>(a, kM, S); });
      timeit("x3 TQ64 6x1 CPB3 (NI4)", [&] { launch_rbx3<96, 64, 6, 1, 3, 3>(a, kM, S); });
      timeit("x3 TQ128 3x4 (MI2 NI2)", [&] { launch_rbx3<96, 128, 3, 4, 3>(a, kM, S); });
      timeit("x3 TQ128 3x2 (MI2 NI4)", [&] { launch_rbx3<96, 128, 3, 2, 3>(a, kM, S); });
      timeit("x3 TQ96 3x2 (MI2 NI3)", [&] { launch_rbx3<96, 96, 3, 2, 3>(a, kM, S); });
    } else {
      timeit("x3 TQ128 3x4", [&] { launch_rbx3<48, 128, 3, 4, 3>(a, kM, S); });
      timeit("x3 TQ192 3x4 (NI3)", [&] { launch_rbx3<48, 192, 3, 4, 3>(a, kM, S); });
      timeit("x3 TQ160 3x4 (NI5/2)", [&] { launch_rbx3<48, 160, 3, 2, 3>(a, kM, S); });
      timeit("x3 TQ144 3x3 (NI3)", [&] { launch_rbx3<48, 144, 3, 3, 3>(a, kM, S); });
      timeit("x3 TQ192 1x4 (MI3 NI3)", [&] { launch_rbx3<48, 192, 1, 4, 3>(a, kM, S); });
      timeit("x3 TQ128 1x8 (MI3 NI1)", [&] { launch_rbx3<48, 128, 1, 8, 3>(a, kM, S); });
    }
  }
  printf(fails ? "FAILED\n" : "all checks passed\n");
  return fails ? 1 : 0;
}
