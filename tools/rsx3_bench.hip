// Fused ResidualStack blocks 0-2 (resstack_x3.hip) against three resblock_x3 launches at the
// MB-MelGAN C = 48 stage of the C2 workload: agreement check (the same split-f16 arithmetic per
// row, up to the MFMA orientation of phase 2), then timing. Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/rsx3_bench.hip -o tools/rsx3_bench
// Diagnostic builds: -DRS_NO_MFMA (operand traffic only), -DRS_NO_LDS (MFMAs on stale registers).
#include "../tts_amd/csrc/resblock_x3.hip"
#ifdef RS_TRACE
__device__ unsigned long long* rs_trace;
#endif
#include "../tts_amd/csrc/resstack_x3.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
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

template <class T>
static T* dup(const std::vector<T>& h) {
  T* p;
  HIP_OK(hipMalloc(&p, h.size() * sizeof(T)));
  HIP_OK(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

static std::vector<float> rnd(size_t n, float sc, uint32_t seed) {
  std::vector<float> v(n);
  uint32_t s = seed;
  for (auto& x : v) {
    s = s * 1664525u + 1013904223u;
    x = sc * ((float)(s >> 8) * (1.f / 8388608.f) - 1.f);
  }
  return v;
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  HIP_OK(hipStreamCreate(&S));
  const int nB = argc > 1 ? std::atoi(argv[1]) : 32;
  const int C = argc > 2 ? std::atoi(argv[2]) : 48;  // 48 (mul 64) or 96 (mul 32)
  const int mul = C == 48 ? 64 : 32, pad = argc > 3 ? std::atoi(argv[3]) : 2;  // inference padding
  int Mmax = 0;
  std::vector<int> hl(kM, kM + nB);
  for (int b = 0; b < nB; ++b) Mmax = std::max(Mmax, kM[b]);
  const int Ls = (Mmax + 2 * pad) * mul;
  int* lens = dup(hl);
  const float* x = dup(rnd((size_t)nB * C * Ls, 1.f, 7u));
  float* y1 = dup(std::vector<float>((size_t)nB * C * Ls, 0.f));
  float* y2 = dup(std::vector<float>((size_t)nB * C * Ls, 0.f));
  float* t1 = dup(std::vector<float>((size_t)nB * C * Ls, 0.f));
  unsigned* of = dup(std::vector<unsigned>(1, 0));
  const int dil[3] = {1, 3, 9};
  StackArgs sa{};
  ResArgs ra[3]{};
  for (int k = 0; k < 3; ++k) {
    std::vector<uint16_t> wd16, wf16, wd16p;
    const std::vector<float> wd = rnd((size_t)C * C * 3, 0.08f, 11u + k);
    pack_resblock_x3(wd, rnd((size_t)C * 2 * C, 0.08f, 21u + k), C, wd16, wf16);
    const float* bd = dup(rnd(C, 0.1f, 31u + k));
    const float* bf = dup(rnd(C, 0.1f, 41u + k));
    sa.dil[k] = dil[k];
    const void* wd_plain = dup(wd16);
    if (C % 32 == 16) pack_resblock_x3p(wd, C, wd16p);  // the stack's packed phase-1 order
    sa.wd16[k] = C % 32 == 16 ? dup(wd16p) : wd_plain;
    sa.wf16[k] = dup(wf16);
    sa.bd[k] = bd;
    sa.bf[k] = bf;
    ResArgs& r = ra[k];
    r.sb = (long)C * Ls;
    r.Ls = Ls;
    r.lens = lens;
    r.len_add = 2 * pad;
    r.mul = mul;
    r.dil = dil[k];
    r.bd = bd;
    r.bf = bf;
    r.Wd16 = wd_plain;
    r.Wf16 = sa.wf16[k];
    r.oflow = of;
    r.max_q = (Mmax + 2 * pad) * mul;
    r.B = nB;
  }
  ra[0].x = x;
  ra[0].y = t1;
  ra[1].x = t1;
  ra[1].y = y1;
  ra[2].x = y1;
  ra[2].y = t1;  // sequential result in t1
  sa.x = x;
  sa.y = y2;
  sa.sb = (long)C * Ls;
  sa.Ls = Ls;
  sa.lens = lens;
  sa.len_add = 2 * pad;
  sa.mul = mul;
  sa.B = nB;
  sa.oflow = of;
  auto seq = [&] {
    for (int k = 0; k < 3; ++k) launch_resblock_x3(ra[k], hl.data(), C, S);
  };
  auto fused = [&] { launch_resstack_x3(sa, hl.data(), C, S); };
#ifdef RS_TRACE
  // the stamp buffer is set before any traced launch (every launch writes through it)
  std::vector<unsigned long long> h((size_t)256 * RS_TRACE_TILES * 16, 0);
  unsigned long long* dtr = dup(h);
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(rs_trace), &dtr, sizeof(dtr)));
#endif
  seq();
  fused();
  HIP_OK(hipStreamSynchronize(S));
  std::vector<float> a((size_t)nB * C * Ls), b(a.size());
  HIP_OK(hipMemcpy(a.data(), t1, a.size() * 4, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(b.data(), y2, b.size() * 4, hipMemcpyDeviceToHost));
  unsigned hof = 0;
  HIP_OK(hipMemcpy(&hof, of, 4, hipMemcpyDeviceToHost));
  long diff = 0, n = 0;
  double md = 0, mag = 0;
  for (int bb = 0; bb < nB; ++bb) {
    const int L = (hl[bb] + 2 * pad) * mul;
    for (int c = 0; c < C; ++c)
      for (int p = 0; p < L; ++p) {
        const size_t i = ((size_t)bb * C + c) * Ls + p;
        ++n;
        if (a[i] != b[i]) ++diff;
        md = std::max(md, (double)std::fabs(a[i] - b[i]));
        mag = std::max(mag, (double)std::fabs(a[i]));
      }
  }
  printf("fused vs 3 launches: %ld of %ld values differ, max|diff| %.3e (max|y| %.3e), oflow %u\n", diff, n, md, mag, hof);
#ifdef RS_TRACE
  {  // per-segment means over tiles 1..2 of every workgroup (steady state)
    HIP_OK(hipMemset(dtr, 0, h.size() * 8));
    fused();
    HIP_OK(hipStreamSynchronize(S));
    HIP_OK(hipMemcpy(h.data(), dtr, h.size() * 8, hipMemcpyDeviceToHost));
    const int pts[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 14, 15};
    const char* nm[] = {"setup", "b0 ph1", "b0 ph2", "b0 xwr", "b1 setup", "b1 ph1", "b1 ph2", "b1 xwr",
                        "b2 setup", "b2 ph1", "b2 ph2", "b2 store", "next stage"};
    double seg[13] = {0};
    int n = 0;
    for (int w = 0; w < 256; ++w)
      for (int i = 1; i < 3; ++i) {
        const unsigned long long* r = &h[((size_t)w * RS_TRACE_TILES + i) * 16];
        bool ok = true;
        for (int k : pts) ok &= r[k] != 0;
        if (!ok) continue;
        for (int k = 0; k < 13; ++k) seg[k] += (double)(r[pts[k + 1]] - r[pts[k]]) * 0.01;
        ++n;
      }
    printf("trace (us per tile, mean of %d tiles):", n);
    double tot = 0;
    for (int k = 0; k < 13; ++k) {
      printf(" %s %.2f,", nm[k], seg[k] / n);
      tot += seg[k] / n;
    }
    printf(" total %.2f\n", tot);
  }
#endif
  const float ts = time_graph(seq), tf = time_graph(fused);
  printf("B=%d C=%d blocks 0-2: 3 x resblock_x3 %.1f us, fused %.1f us\n", nB, C, ts, tf);
#define VAR(TQ, WN, NI) printf("  fused TQ %d WN %d NI %d: %.1f us\n", TQ, WN, NI, time_graph([&] { \
    StackArgs v = sa; v.ext[2] = 0; v.ext[1] = 9; v.ext[0] = 12; launch_rsx3<48, TQ, WN, NI>(v, hl.data(), S); }))
  if (C == 48) {
    VAR(208, 4, 4);
    VAR(192, 4, 4);
    VAR(176, 4, 4);
  }
  // the fused kernel's blocks 0-1 keep phase 2 untransposed (their output goes to LDS), the
  // resblock_x3 launches transpose every block: the MFMA's internal order differs, ~1 ulp
  return md <= 1e-6 * std::max(1.0, mag) ? 0 : 1;
}
