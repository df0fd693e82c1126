// Split-f16 generic conv (conv_x3.hip): correctness against the fp32 MFMA conv (conv.hip, itself
// parity-tested against the oracle) over padding modes, phases, two sources, time-major sources,
// activations and epilogues on ragged utterances; then timing of both at the C2 shapes
// (Tacotron2 encoder / postnet, MB-MelGAN conv_in and ConvTranspose stages). Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/cx3_bench.hip -o tools/cx3_bench
#include "../tts_amd/csrc/conv.hip"
#include "../tts_amd/csrc/conv_x3.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

static const int kM[32] = {832, 164, 833, 443, 699, 490, 723, 154, 651, 760, 389, 710, 223, 857, 796, 454,
                           605, 645, 553, 403, 742, 608, 728, 677, 764, 525, 831, 511, 459, 596, 677, 610};
static const int kT[32] = {151, 40, 158, 83, 131, 92, 134, 30, 122, 142, 75, 132, 44, 168, 149, 86,
                           112, 120, 104, 76, 139, 114, 136, 127, 143, 98, 155, 96, 86, 111, 127, 114};
static hipStream_t S;

template <class T>
static T* dup(const std::vector<T>& h) {
  T* p;
  HIP_OK(hipMalloc(&p, std::max<size_t>(h.size(), 1) * sizeof(T)));
  if (!h.empty()) HIP_OK(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

static std::vector<float> rnd(size_t n, float sc, uint32_t seed) {
  std::vector<float> v(n);
  uint32_t s = seed * 2654435761u + 12345u;
  for (auto& x : v) {
    s = s * 1664525u + 1013904223u;
    x = sc * ((float)(s >> 8) * (1.f / 8388608.f) - 1.f);
  }
  return v;
}

// fp32 kernel weights: tap-major inside 16-channel chunks, then the 16x16x4 fragment swizzle
static std::vector<float> pack_f32(const std::vector<float>& Wm, int Cin, int Cout, int Cout_pad, int K, int nph) {
  const int Kd = Cin * K;
  std::vector<float> Wt(Wm.size());
  for (size_t r = 0; r < (size_t)nph * Cout; ++r)
    for (int ci = 0; ci < Cin; ++ci)
      for (int k = 0; k < K; ++k) Wt[r * Kd + (size_t)(ci / 16) * 16 * K + k * 16 + ci % 16] = Wm[r * Kd + (size_t)ci * K + k];
  const size_t per = (size_t)Cout_pad * Kd;
  std::vector<float> sw(per * nph);
  for (int ph = 0; ph < nph; ++ph) swizzle_rows16(Wt.data() + (size_t)ph * Cout * Kd, Cout, Cout_pad, Kd, sw.data() + ph * per);
  return sw;
}

struct Case {
  std::string name;
  int Cin, Cout, K, nph, B;
  const int* lens;
  int in_mul;  // input length = lens * in_mul; output positions per phase = the same
  int pad_mode, rep_pad, act, epi, two_src, time_major, resid;
};

struct Built {
  ConvArgs a;
  float* out;
  size_t out_elems;
  int tile;
  double flop;
  ConvArgs am;  // nph > 1: the phase-merged form (merged_u)
};

static Built build(const Case& c, uint32_t seed, float xscale) {
  const int B = c.B;
  int Lmax = 0;
  double sumL = 0;
  for (int b = 0; b < B; ++b) Lmax = std::max(Lmax, c.lens[b] * c.in_mul), sumL += c.lens[b] * c.in_mul;
  const int Lsrc = Lmax;  // source positions (rep_pad: raw length)
  const int pl = c.nph > 1 ? 1 : (c.K - 1) / 2;
  ConvArgs a{};
  const int C0 = c.two_src ? c.Cin / 2 : c.Cin;
  auto xs = rnd((size_t)B * c.Cin * Lsrc, xscale, seed);
  float* x = dup(xs);
  if (c.time_major) {
    a.src[0] = ConvSrc{x, (long)c.Cin * Lsrc, 1, c.Cin, C0, c.act};
  } else {
    a.src[0] = ConvSrc{x, (long)c.Cin * Lsrc, Lsrc, 1, C0, c.act};
  }
  a.src[1] = a.src[0];
  if (c.two_src) {
    a.src[1].ptr = x + (c.time_major ? C0 : (long)C0 * Lsrc);
    a.src[1].C = c.Cin - C0;
    a.src[1].act = 0;
  }
  a.nsrc = c.two_src ? 2 : 1;
  a.Cin = c.Cin;
  a.K = c.K;
  a.dil = 1;
  a.pad_mode = c.pad_mode;
  a.lens = dup(std::vector<int>(c.lens, c.lens + B));
  a.len_add = 2 * c.rep_pad;
  a.in_mul = a.q_mul = c.in_mul;
  a.rep_pad = c.rep_pad;
  a.nphase = c.nph;
  for (int p = 0; p < 8; ++p) a.pad_left[p] = c.nph > 1 ? (p < c.nph / 2 ? 1 : 0) : pl;
  const int tile = conv_tile_for_cout(c.Cout);
  const int TC = conv_tile_tc(tile);
  a.Cout = c.Cout;
  a.Cout_pad = (c.Cout + TC - 1) / TC * TC;
  auto Wm = rnd((size_t)c.nph * c.Cout * c.Cin * c.K, 1.f / std::sqrt((float)c.Cin * c.K), seed + 1);
  a.W = dup(pack_f32(Wm, c.Cin, c.Cout, a.Cout_pad, c.K, c.nph));
  a.w_phase_stride = (long)a.Cout_pad * c.Cin * c.K;
  a.W16 = dup(pack_conv_x3(Wm, c.Cin, c.Cout, c.K, c.nph, &a.w16_phase_stride));
  a.oflow = dup(std::vector<unsigned>(1, 0));
  a.bias = dup(rnd(c.Cout, 0.1f, seed + 2));
  const int Lout = (Lmax + 2 * c.rep_pad) * c.nph;
  const size_t oe = (size_t)B * c.Cout * Lout;
  float* out = dup(std::vector<float>(oe, 0.f));
  a.out = out;
  a.ob = (long)c.Cout * Lout;
  a.oc = Lout;
  a.ot = 1;
  a.out_mul = c.nph;
  a.epi_act = c.epi;
  if (c.resid) {
    a.resid = dup(rnd(oe, 1.f, seed + 3));
    a.rb = a.ob;
    a.rc = a.oc;
    a.rt = 1;
  }
  a.max_q = Lmax + 2 * c.rep_pad;
  a.B = B;
  Built r{a, out, oe, tile, 2.0 * c.Cout * c.Cin * c.K * sumL * c.nph, a};
  if (c.nph > 1) {
    ConvArgs& m = r.am;
    long st;
    m.W16 = dup(pack_conv_x3(merge_convT_phases(Wm, c.nph, c.Cin, c.Cout), c.Cin, c.nph * c.Cout, 2, 1, &st));
    m.w16_phase_stride = st;
    std::vector<float> hb(c.Cout), bm((size_t)c.nph * c.Cout);
    HIP_OK(hipMemcpy(hb.data(), a.bias, c.Cout * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < bm.size(); ++i) bm[i] = hb[i / c.nph];
    m.bias = dup(bm);
    m.Cout = m.Cout_pad = c.nph * c.Cout;
    m.nphase = 1;
    m.pad_left[0] = 1;
    m.out_mul = 1;
    m.max_q = Lmax + 1;
    m.merged_u = c.nph;
  }
  return r;
}

static float time_it(const std::function<void()>& f, int reps = 10) {
  f();
  HIP_OK(hipStreamSynchronize(S));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  HIP_OK(hipEventRecord(e0, S));
  for (int r = 0; r < reps; ++r) f();
  HIP_OK(hipEventRecord(e1, S));
  HIP_OK(hipEventSynchronize(e1));
  float ms;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / reps;
}

static int check(const Case& c, float xscale = 1.f) {
  Built r = build(c, 7 + c.Cin + c.Cout + c.K, xscale);
  launch_conv(r.a, r.tile, S);
  HIP_OK(hipStreamSynchronize(S));
  std::vector<float> ref(r.out_elems), got(r.out_elems);
  HIP_OK(hipMemcpy(ref.data(), r.out, r.out_elems * 4, hipMemcpyDeviceToHost));
  HIP_OK(hipMemset(r.out, 0, r.out_elems * 4));
  launch_conv_x3(r.a, S);
  HIP_OK(hipStreamSynchronize(S));
  HIP_OK(hipMemcpy(got.data(), r.out, r.out_elems * 4, hipMemcpyDeviceToHost));
  unsigned of = 0;
  HIP_OK(hipMemcpy(&of, r.a.oflow, 4, hipMemcpyDeviceToHost));
  double err = 0, mag = 0;
  for (size_t i = 0; i < r.out_elems; ++i) {  // untouched tails: both zero, else counted here
    err = std::max(err, (double)std::fabs(got[i] - ref[i]));
    mag = std::max(mag, (double)std::fabs(ref[i]));
  }
  const bool want_of = xscale > 1e4f;
  bool ok = (want_of || err <= 4e-6 * std::max(1.0, mag)) && (of != 0) == want_of;
  printf("check %-28s max|err| %.3e (max|y| %.3e) oflow %u  %s\n", c.name.c_str(), err, mag, of, ok ? "OK" : "FAIL");
  if (c.nph > 1) {
    HIP_OK(hipMemset(r.out, 0, r.out_elems * 4));
    launch_conv_x3(r.am, S);
    HIP_OK(hipStreamSynchronize(S));
    HIP_OK(hipMemcpy(got.data(), r.out, r.out_elems * 4, hipMemcpyDeviceToHost));
    double e2 = 0;
    for (size_t i = 0; i < r.out_elems; ++i) e2 = std::max(e2, (double)std::fabs(got[i] - ref[i]));
    const bool ok2 = e2 <= 4e-6 * std::max(1.0, mag);
    printf("check %-28s max|err| %.3e (phase-merged)  %s\n", c.name.c_str(), e2, ok2 ? "OK" : "FAIL");
    ok = ok && ok2;
  }
  return ok ? 0 : 1;
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  HIP_OK(hipStreamCreate(&S));
  const bool prof = argc > 1 && std::string(argv[1]) == "prof";
  static const int small[3] = {37, 5, 70};
  int fails = 0;
  if (!prof) {
    // name, Cin, Cout, K, nph, B, lens, in_mul, pad_mode, rep_pad, act, epi, two_src, time_major, resid
    fails += check({"k5 512->512 relu tmajor", 512, 512, 5, 1, 3, small, 1, 0, 0, 0, 1, 0, 1, 0});
    fails += check({"k5 80->512 tanh", 80, 512, 5, 1, 3, small, 1, 0, 0, 0, 2, 0, 0, 0});
    fails += check({"k5 80->512 tanh tmajor", 80, 512, 5, 1, 3, small, 1, 0, 0, 0, 2, 0, 1, 0});
    fails += check({"k5 512->80 resid", 512, 80, 5, 1, 3, small, 1, 0, 0, 0, 0, 0, 0, 1});
    fails += check({"k1 512->2048", 512, 2048, 1, 1, 3, small, 1, 0, 0, 0, 0, 0, 0, 0});
    fails += check({"k1 512->128 tmajor", 512, 128, 1, 1, 3, small, 1, 0, 0, 0, 0, 0, 1, 0});
    fails += check({"k7 80->384 reflect rep2", 80, 384, 7, 1, 3, small, 1, 1, 2, 0, 0, 0, 0, 0});
    fails += check({"k7 80->384 reflect", 80, 384, 7, 1, 3, small, 1, 1, 0, 0, 0, 0, 0, 0});
    fails += check({"convT 384->192 x8 lrelu", 384, 192, 2, 8, 3, small, 1, 0, 0, 1, 0, 0, 0, 0});
    fails += check({"convT 192->96 x4 lrelu", 192, 96, 2, 4, 3, small, 8, 0, 0, 1, 0, 0, 0, 0});
    fails += check({"convT 96->48 x2 lrelu", 96, 48, 2, 2, 3, small, 32, 0, 0, 1, 0, 0, 0, 0});
    fails += check({"k3 256->64 clamp lrelu", 256, 64, 3, 1, 3, small, 2, 2, 0, 1, 1, 0, 0, 0});
    fails += check({"k5 192->384 gate pair", 192, 384, 5, 1, 3, small, 1, 0, 0, 0, 3, 0, 0, 0});
    fails += check({"k5 512->512 range", 512, 512, 5, 1, 3, small, 1, 0, 0, 0, 1, 0, 0, 0}, 1e5f);
  }
  // C2 shapes: Tacotron2 on the 32 LJ token / frame lengths, MB-MelGAN stages
  struct Shape {
    Case c;
    const char* what;
  };
  std::vector<Shape> shapes = {
      {{"enc k5 512->512", 512, 512, 5, 1, 32, kT, 1, 0, 0, 0, 1, 0, 0, 0}, "encoder conv (x3 per call)"},
      {{"lstm_in k1 512->2048", 512, 2048, 1, 1, 32, kT, 1, 0, 0, 0, 0, 0, 0, 0}, "BiLSTM input projection"},
      {{"post k5 80->512", 80, 512, 5, 1, 32, kM, 1, 0, 0, 0, 2, 0, 1, 0}, "postnet 0"},
      {{"post k5 512->512", 512, 512, 5, 1, 32, kM, 1, 0, 0, 0, 2, 0, 0, 0}, "postnet 1-3 (x3 per call)"},
      {{"post k5 512->80", 512, 80, 5, 1, 32, kM, 1, 0, 0, 0, 0, 0, 0, 1}, "postnet 4"},
      {{"mg k7 80->384", 80, 384, 7, 1, 32, kM, 1, 1, 0, 0, 0, 0, 0, 0}, "MB-MelGAN conv_in"},
      {{"mg convT 384->192 x8", 384, 192, 2, 8, 32, kM, 1, 0, 0, 1, 0, 0, 0, 0}, "upsample 1"},
      {{"mg convT 192->96 x4", 192, 96, 2, 4, 32, kM, 8, 0, 0, 1, 0, 0, 0, 0}, "upsample 2"},
      {{"mg convT 96->48 x2", 96, 48, 2, 2, 32, kM, 32, 0, 0, 1, 0, 0, 0, 0}, "upsample 3"},
  };
  for (auto& sh : shapes) {
    Built r = build(sh.c, 99, 1.f);
    if (prof) {
      for (int i = 0; i < 3; ++i) launch_conv_x3(sh.c.nph > 1 ? r.am : r.a, S);
      HIP_OK(hipStreamSynchronize(S));
      continue;
    }
    const float t32 = time_it([&] { launch_conv(r.a, r.tile, S); });
    const float tx3 = time_it([&] { launch_conv_x3(r.a, S); });
    printf("%-24s fp32 %8.1f us (%6.1f TF/s)   x3 %8.1f us (%6.1f TF/s fp32-equiv)  %s\n", sh.c.name.c_str(), t32,
           r.flop / (t32 * 1e-6) / 1e12, tx3, r.flop / (tx3 * 1e-6) / 1e12, sh.what);
    if (sh.c.nph > 1) {
      const float tm = time_it([&] { launch_conv_x3(r.am, S); });
      printf("%-24s                              x3 %8.1f us (%6.1f TF/s fp32-equiv)  phase-merged\n", sh.c.name.c_str(),
             tm, r.flop / (tm * 1e-6) / 1e12);
    }
  }
  if (argc > 1 && std::string(argv[1]) == "sweep") {
    // tile shapes beside the library's choice on the C2 shapes; every variant's output must equal
    // the library tile's bit for bit (the same k-step order per output element)
    struct V {
      const char* name;
      int tc;
      std::function<void(const ConvArgs&)> run;
    };
    std::vector<V> vs = {
        {"128x48 (2,3,4,1)", 128, [](const ConvArgs& a) { cx_taps<2, 3, 4, 1, 2>(a, S); }},
        {"128x64 (2,4,4,1)", 128, [](const ConvArgs& a) { cx_taps<2, 4, 4, 1, 2>(a, S); }},
        {"64x128 (2,4,2,2)", 64, [](const ConvArgs& a) { cx_taps<2, 4, 2, 2, 1>(a, S); }},
        {"192x64 (3,4,4,1)", 192, [](const ConvArgs& a) { cx_taps<3, 4, 4, 1, 2>(a, S); }},
        {"96x128 (3,4,2,2)", 96, [](const ConvArgs& a) { cx_taps<3, 4, 2, 2, 1>(a, S); }},
        {"128x32 (2,2,4,1)", 128, [](const ConvArgs& a) { cx_taps<2, 2, 4, 1, 2>(a, S); }},
        {"256x32 (2,2,8,1)", 256, [](const ConvArgs& a) { cx_taps<2, 2, 8, 1, 2>(a, S); }},
        {"128x64 (1,4,8,1)", 128, [](const ConvArgs& a) { cx_taps<1, 4, 8, 1, 2>(a, S); }},
    };
    for (auto& sh : shapes) {
      if (sh.c.Cout == 80 || sh.c.Cout == 48) continue;
      Built r = build(sh.c, 99, 1.f);
      const ConvArgs& a = sh.c.nph > 1 ? r.am : r.a;
      launch_conv_x3(a, S);
      HIP_OK(hipStreamSynchronize(S));
      std::vector<float> ref(r.out_elems), got(r.out_elems);
      HIP_OK(hipMemcpy(ref.data(), r.out, r.out_elems * 4, hipMemcpyDeviceToHost));
      const float tl = time_it([&] { launch_conv_x3(a, S); });
      printf("%-24s library %8.1f us\n", sh.c.name.c_str(), tl);
      for (auto& v : vs) {
        if (a.Cout % v.tc) continue;
        HIP_OK(hipMemset(r.out, 0, r.out_elems * 4));
        v.run(a);
        HIP_OK(hipStreamSynchronize(S));
        HIP_OK(hipMemcpy(got.data(), r.out, r.out_elems * 4, hipMemcpyDeviceToHost));
        const bool same = std::memcmp(got.data(), ref.data(), r.out_elems * 4) == 0;
        const float t = time_it([&] { v.run(a); });
        printf("%-24s %-18s %8.1f us  %s\n", "", v.name, t, same ? "same bits" : "DIFFERENT");
        fails += !same;
      }
    }
  }
  printf(fails ? "FAILED\n" : "all checks passed\n");
  return fails ? 1 : 0;
}
