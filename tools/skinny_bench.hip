// Microbenchmark for the decoder's skinny GEMM kernels (K4 / K5 / K2 shapes) and the raw
// weight-stream rate, timed as graph replays of back-to-back launches. Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../tts_amd/csrc tools/skinny_bench.hip -o /tmp/sb
#define ATTN_TRACE_BUF 1
#define SK_TRACE_BUF 1
#include "../tts_amd/csrc/decoder.hip"
#include <algorithm>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

static float* dalloc(size_t n, float v = 0.01f) {
  float* p;
  HIP_OK(hipMalloc(&p, n * 4));
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = v * (float)((i * 2654435761u) % 1000) / 1000.f;
  HIP_OK(hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice));
  return p;
}

// raw stream of a wave's weight slice: all NCH loads issued at once, one wait
template <int NCH, int KS>
__global__ __launch_bounds__(KS * 64) void wstream_all(const f32x4* W, int nkc, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const f32x4* p = W + ((long)blockIdx.x * nkc + w * NCH) * 64 + lane;
  f32x4 r[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) r[i] = p[(long)i * 64];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) s += r[i][0] + r[i][1] + r[i][2] + r[i][3];
  if (s == 12345.f) out[0] = s;
}

// same, groups of U with a two-deep register pipeline (the SkPipe structure without X)
template <int NCH, int KS, int U>
__global__ __launch_bounds__(KS * 64) void wstream_pipe(const f32x4* W, int nkc, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const f32x4* p = W + ((long)blockIdx.x * nkc + w * NCH) * 64 + lane;
  f32x4 a[U], b[U];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) a[u] = p[(long)u * 64];
  for (int k = 0; k < NCH; k += 2 * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = p[(long)min(k + U + u, NCH - 1) * 64];
#pragma unroll
    for (int u = 0; u < U; ++u) s += a[u][0] + a[u][1] + a[u][2] + a[u][3];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = p[(long)min(k + 2 * U + u, NCH - 1) * 64];
#pragma unroll
    for (int u = 0; u < U; ++u) s += b[u][0] + b[u][1] + b[u][2] + b[u][3];
  }
  if (s == 12345.f) out[0] = s;
}


// structural model of the skinny k-loop: ring of D chunks, W (1 KiB) + MT X loads per chunk,
// MFMAs optional, X optional
template <int MT, int D, int KS, bool MMA, bool XL>
__global__ __launch_bounds__(KS * 64) void ring_model(const f32x4* W, const float* X, int ldx, int nkc, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int per = nkc / KS, lo = w * per, hi = lo + per;
  const f32x4* wp = W + (long)blockIdx.x * nkc * 64 + lane;
  const float* xp = X + (long)(lane & 15) * ldx + 4 * (lane >> 4);
  f32x4 wr[D], xr[D][MT];
  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto load1 = [&](int u, int kc_in) {
    const int kc = min(kc_in, hi - 1);
    wr[u] = wp[(long)kc * 64];
    if (XL) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) xr[u][mt] = *reinterpret_cast<const f32x4*>(xp + kc * 16 + (long)mt * 16 * ldx);
    } else {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) xr[u][mt] = f32x4{1.f, 1.f, 1.f, 1.f};
    }
  };
#pragma unroll
  for (int u = 0; u < D; ++u) load1(u, lo + u);
  for (int kc0 = lo; kc0 < hi; kc0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      if (kc0 + u < hi) {
        if (MMA) {
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[mt] = MFMA16(xr[u][mt][s], wr[u][s], acc[mt]);
        } else {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[mt] += xr[u][mt] + wr[u];
        }
      }
      load1(u, kc0 + D + u);
    }
  }
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < MT; ++i) sum += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (sum == 12345.f) out[0] = sum;
}

// MFMA issue only: per wave NCH chunks of MT*4 dependent-pair MFMAs on register operands
template <int MT, int KS>
__global__ __launch_bounds__(KS * 64) void mfma_only(int nch, float* out) {
  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 a = f32x4{1.f, 2.f, 3.f, (float)threadIdx.x};
  for (int c = 0; c < nch; ++c) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = MFMA16(a[s], a[3 - s], acc[mt]);
  }
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < MT; ++i) sum += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (sum == 12345.f) out[0] = sum;
}

__global__ void empty_kernel(float* out) {
  if (threadIdx.x == 1000) out[0] = 1.f;
}

static hipStream_t S;

static float time_graph(const std::function<void()>& body, int per_graph = 40, int reps = 10) {
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

// one traced launch: per-phase averages over workgroups (us)
static void sk_report(const char* name, int nwg, const std::function<void()>& launch) {
  std::vector<unsigned long long> tr(1024 * 8, 0);
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(sk_trace), tr.data(), tr.size() * 8));
  time_graph(launch, 20, 2);  // warm replays; the buffer keeps the last launch
  HIP_OK(hipStreamSynchronize(S));
  HIP_OK(hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(sk_trace), tr.size() * 8));
  unsigned long long tmin = ~0ull, tmax = 0;
  for (int w = 0; w < nwg; ++w) tmin = std::min(tmin, tr[w * 8]);
  double ph[6] = {0};
  int n = 0;
  for (int w = 0; w < nwg; ++w) {
    const unsigned long long* t = &tr[w * 8];
    if (!t[5]) continue;
    ++n;
    ph[0] += (double)(t[0] - tmin);
    ph[1] += (double)(t[1] - t[0]);
    ph[2] += (double)(t[2] - t[1]);
    ph[3] += (double)(t[3] - t[2]);
    ph[4] += (double)((t[4] ? t[4] : t[5]) - t[3]);
    ph[5] += (double)(t[5] - (t[4] ? t[4] : t[3]));
    tmax = std::max(tmax, t[5]);
  }
  printf("   %s: start %.2f | issue %.2f gemm %.2f reduce %.2f epi %.2f pq/tail %.2f | span %.2f us (%d wg)\n", name,
         ph[0] / n / 100, ph[1] / n / 100, ph[2] / n / 100, ph[3] / n / 100, ph[4] / n / 100, ph[5] / n / 100,
         (double)(tmax - tmin) / 100, n);
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  HIP_OK(hipStreamCreate(&S));
  const int B = argc > 1 ? atoi(argv[1]) : 32;
  const int MT = (B + 15) / 16, Bp = MT * 16;
  float* dummy = dalloc(16);
  // control block
  int* ctl;
  HIP_OK(hipMalloc(&ctl, (4 + 4 * 64) * 4));
  HIP_OK(hipMemset(ctl, 0, (4 + 4 * 64) * 4));
  DecDev d{};
  d.ctl = reinterpret_cast<DecCtl*>(ctl);
  d.done = ctl + 4;
  d.steps = ctl + 68;
  d.status = ctl + 132;
  d.max_steps = ctl + 196;
  d.B = B;
  d.S_cap = 1;
  d.T_max = 1;
  float* dec_out = dalloc((size_t)B * 80 * 7);
  d.dec_out = dec_out;
  // activations / weights
  float* hatt = dalloc((size_t)Bp * 1024);
  float* ctx = dalloc((size_t)Bp * 512);
  float* hd0 = dalloc((size_t)Bp * 1024);
  float* hd1 = dalloc((size_t)Bp * 1024);
  float* cst = dalloc((size_t)Bp * 1024);
  float* gatt = dalloc((size_t)Bp * 4096);
  float* pb = dalloc((size_t)Bp * 256);
  float* y = dalloc((size_t)Bp * 560);
  float* pq = dalloc((size_t)256 * Bp * 128);
  float* spart = dalloc((size_t)64 * Bp);
  float* Wdec = dalloc((size_t)4096 * 2560);
  float* Wpre = dalloc((size_t)4096 * 1536);
  float* Wproj = dalloc((size_t)560 * 1536);
  float* Watt = dalloc((size_t)4096 * 256);
  float* WqT = dalloc((size_t)1024 * 128);
  float* bias = dalloc(4096);
  float* stw = dalloc(1584);
  printf("B=%d MT=%d\n", B, MT);
  printf("empty kernel (1 WG)              %7.2f us\n", time_graph([&] { empty_kernel<<<1, 64, 0, S>>>(dummy); }));
  printf("empty kernel (256 WG x 256)      %7.2f us\n", time_graph([&] { empty_kernel<<<256, 256, 0, S>>>(dummy); }));

  const double wbytes = 4096.0 * 2560 * 4;
  auto rep = [&](const char* name, float us, double bytes) {
    printf("%-34s %7.2f us  %7.1f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
  };
  const f32x4* Wv = reinterpret_cast<const f32x4*>(Wdec);
  rep("W stream all-at-once KS=4 (40)", time_graph([&] { wstream_all<40, 4><<<256, 256, 0, S>>>(Wv, 160, dummy); }), wbytes);
  rep("W stream all-at-once KS=8 (20)", time_graph([&] { wstream_all<20, 8><<<256, 512, 0, S>>>(Wv, 160, dummy); }), wbytes);
  rep("W stream all-at-once KS=16 (10)", time_graph([&] { wstream_all<10, 16><<<256, 1024, 0, S>>>(Wv, 160, dummy); }), wbytes);
  rep("W stream pipe KS=4 U=4", time_graph([&] { wstream_pipe<40, 4, 4><<<256, 256, 0, S>>>(Wv, 160, dummy); }), wbytes);
  rep("W stream pipe KS=4 U=8", time_graph([&] { wstream_pipe<40, 4, 8><<<256, 256, 0, S>>>(Wv, 160, dummy); }), wbytes);
  rep("W stream all KS=4 (80) 128 WG", time_graph([&] { wstream_all<80, 4><<<128, 256, 0, S>>>(Wv, 320, dummy); }), wbytes);
  rep("W stream all KS=8 (40) 128 WG", time_graph([&] { wstream_all<40, 8><<<128, 512, 0, S>>>(Wv, 320, dummy); }), wbytes);
  rep("W stream all KS=16 (40) 64 WG", time_graph([&] { wstream_all<40, 16><<<64, 1024, 0, S>>>(Wv, 640, dummy); }), wbytes);
  rep("W stream all 8MB KS=4 (40) 48WG", time_graph([&] { wstream_all<40, 4><<<48, 256, 0, S>>>(Wv, 160, dummy); }), wbytes * 48 / 256);
  rep("W stream pipe KS=8 U=4", time_graph([&] { wstream_pipe<20, 8, 4><<<256, 512, 0, S>>>(Wv, 160, dummy); }), wbytes);

  rep("MFMA only MT=2 40ch KS=4", time_graph([&] { mfma_only<2, 4><<<256, 256, 0, S>>>(40, dummy); }), wbytes);
  rep("MFMA only MT=1 40ch KS=4", time_graph([&] { mfma_only<1, 4><<<256, 256, 0, S>>>(40, dummy); }), wbytes);
  rep("MFMA only MT=2 20ch KS=8", time_graph([&] { mfma_only<2, 8><<<256, 512, 0, S>>>(20, dummy); }), wbytes);
  rep("ring W only D=4", time_graph([&] { ring_model<2, 4, 4, false, false><<<256, 256, 0, S>>>(Wv, hatt, 1024, 160, dummy); }), wbytes);
  rep("ring W+X D=4", time_graph([&] { ring_model<2, 4, 4, false, true><<<256, 256, 0, S>>>(Wv, hatt, 1024, 160, dummy); }), wbytes);
  rep("ring W+X D=12", time_graph([&] { ring_model<2, 12, 4, false, true><<<256, 256, 0, S>>>(Wv, hatt, 1024, 160, dummy); }), wbytes);
  rep("ring W+X ld16 D=4", time_graph([&] { ring_model<2, 4, 4, false, true><<<256, 256, 0, S>>>(Wv, hatt, 16, 160, dummy); }), wbytes);
  rep("ring W+MMA D=4", time_graph([&] { ring_model<2, 4, 4, true, false><<<256, 256, 0, S>>>(Wv, hatt, 1024, 160, dummy); }), wbytes);
  rep("ring W+MMA D=12", time_graph([&] { ring_model<2, 12, 4, true, false><<<256, 256, 0, S>>>(Wv, hatt, 1024, 160, dummy); }), wbytes);
  rep("ring W+X+MMA D=4", time_graph([&] { ring_model<2, 4, 4, true, true><<<256, 256, 0, S>>>(Wv, hatt, 1024, 160, dummy); }), wbytes);
  rep("ring W+X+MMA D=12", time_graph([&] { ring_model<2, 12, 4, true, true><<<256, 256, 0, S>>>(Wv, hatt, 1024, 160, dummy); }), wbytes);
  rep("ring W+X+MMA ld16 D=4", time_graph([&] { ring_model<2, 4, 4, true, true><<<256, 256, 0, S>>>(Wv, hatt, 16, 160, dummy); }), wbytes);
  rep("ring W+X+MMA KS=8 D=4", time_graph([&] { ring_model<2, 4, 8, true, true><<<256, 512, 0, S>>>(Wv, hatt, 1024, 160, dummy); }), wbytes);

  // K4: decoder_rnn LSTM, K = 1024 + 512 + 1024
  SkArgs a4{};
  a4.njobs = 1;
  a4.MT = MT;
  {
    SkJob& J = a4.job[0];
    J.seg[0] = {hatt, 16 * 1024, 1024};
    J.seg[1] = {ctx, 16 * 512, 512};
    J.seg[2] = {hd0, 16 * 1024, 1024};
    J.nseg = 3;
    J.K = 2560;
    J.W = Wdec;
    J.ntiles = 256;
    J.epi = EPI_LSTM;
    J.bias = bias;
    J.h_out = hd1;
    J.c_state = cst;
    J.hc_ld = 1024;
  }
  auto k4 = [&](auto kern, int KS, const char* name) {
    const size_t lds = skinny_lds(1, KS, Bp);
    rep(name, time_graph([&] { kern<<<256, KS * 64, lds, S>>>(a4, d, 0); }), wbytes);
  };
  if (MT == 2) {
    k4(skinny_kernel<1, 4, 2, 4>, 4, "K4 <1,4> D=4");
    k4(skinny_kernel<1, 4, 2, 8>, 4, "K4 <1,4> D=8");
    k4(skinny_kernel<1, 4, 2, 12>, 4, "K4 <1,4> D=12");
    k4(skinny_kernel<1, 4, 2, 16>, 4, "K4 <1,4> D=16");
    k4(skinny_kernel<1, 4, 2, 20>, 4, "K4 <1,4> D=20");
    k4(skinny_kernel<1, 8, 2, 4>, 8, "K4 <1,8> D=4");
    k4(skinny_kernel<1, 8, 2, 8>, 8, "K4 <1,8> D=8");
    k4(skinny_kernel<1, 8, 2, 10>, 8, "K4 <1,8> D=10");
    k4(skinny_kernel<1, 16, 2, 4>, 16, "K4 <1,16> D=4");
    SkArgs keep = a4;
    a4.job[0].epi = EPI_STORE;
    a4.job[0].out = gatt;
    a4.job[0].out_ld = 4096;
    k4(skinny_kernel<1, 4, 2, 12>, 4, "K4 store-epi <1,4> D=12");
    k4(skinny_kernel<1, 8, 2, 8>, 8, "K4 store-epi <1,8> U=2");
    a4 = keep;
  }
  // K5: projection (stopnet tile + 10 frame tiles) || att-pre store (256 tiles), K = 1536
  SkArgs pj{}, ap{};
  pj.njobs = ap.njobs = 1;
  pj.MT = ap.MT = MT;
  {
    SkJob& J = pj.job[0];
    J.seg[0] = {hd1, 16 * 1024, 1024};
    J.seg[1] = {ctx, 16 * 512, 512};
    J.nseg = 2;
    J.K = 1536;
    J.W = Wproj;
    J.ntiles = 11;
    J.epi = EPI_STORE;
    J.bias = bias;
    J.out = y;
    J.out_ld = 560;
    J.out_frag = 1;
    J.frames_r = 2;
    J.lead_stop = 1;
    J.stop_part = spart;
    SkJob& J2 = ap.job[0];
    J2.seg[0] = {ctx, 16 * 512, 512};
    J2.seg[1] = {hatt, 16 * 1024, 1024};
    J2.nseg = 2;
    J2.K = 1536;
    J2.W = Wpre;
    J2.ntiles = 256;
    J2.epi = EPI_STORE;
    J2.bias = bias;
    J2.out = gatt;
    J2.out_ld = 4096;
  }
  SkArgs both5 = pj;
  both5.njobs = 2;
  both5.job[1] = ap.job[0];
  SkArgs both4 = a4;
  both4.njobs = 2;
  both4.job[1] = ap.job[0];
  const double bpj = 11.0 * 16 * 1536 * 4, bap = 256.0 * 16 * 1536 * 4;
  if (MT == 2) {
    rep("proj <1,4>", time_graph([&] { skinny_kernel<1, 4, 2, 0><<<11, 256, skinny_lds(1, 4, Bp), S>>>(pj, d, 0); }), bpj);
    rep("proj <1,8>", time_graph([&] { skinny_kernel<1, 8, 2, 0><<<11, 512, skinny_lds(1, 8, Bp), S>>>(pj, d, 0); }), bpj);
    rep("proj <1,16>", time_graph([&] { skinny_kernel<1, 16, 2, 0><<<11, 1024, skinny_lds(1, 16, Bp), S>>>(pj, d, 0); }), bpj);
    rep("att-pre <1,4>", time_graph([&] { skinny_kernel<1, 4, 2, 0><<<256, 256, skinny_lds(1, 4, Bp), S>>>(ap, d, 0); }), bap);
    rep("att-pre <1,8>", time_graph([&] { skinny_kernel<1, 8, 2, 0><<<256, 512, skinny_lds(1, 8, Bp), S>>>(ap, d, 0); }), bap);
    rep("proj + att-pre <1,8>", time_graph([&] { skinny_kernel<1, 8, 2, 0><<<267, 512, skinny_lds(1, 8, Bp), S>>>(both5, d, 0); }), bpj + bap);
    rep("proj + att-pre <1,4>", time_graph([&] { skinny_kernel<1, 4, 2, 0><<<267, 256, skinny_lds(1, 4, Bp), S>>>(both5, d, 0); }), bpj + bap);
    rep("K4 + att-pre <1,4>", time_graph([&] { skinny_kernel<1, 4, 2, 0><<<512, 256, skinny_lds(1, 4, Bp), S>>>(both4, d, 0); }), wbytes + bap);
    rep("K4 ; proj+att-pre <1,8>", time_graph([&] {
          skinny_kernel<1, 4, 2, 0><<<256, 256, skinny_lds(1, 4, Bp), S>>>(a4, d, 0);
          skinny_kernel<1, 8, 2, 0><<<267, 512, skinny_lds(1, 8, Bp), S>>>(both5, d, 0);
        }), wbytes + bpj + bap);
    rep("K4+att-pre ; proj <1,16>", time_graph([&] {
          skinny_kernel<1, 4, 2, 0><<<512, 256, skinny_lds(1, 4, Bp), S>>>(both4, d, 0);
          skinny_kernel<1, 16, 2, 0><<<11, 1024, skinny_lds(1, 16, Bp), S>>>(pj, d, 0);
        }), wbytes + bpj + bap);
    rep("K4+att-pre ; proj <1,8>", time_graph([&] {
          skinny_kernel<1, 4, 2, 0><<<512, 256, skinny_lds(1, 4, Bp), S>>>(both4, d, 0);
          skinny_kernel<1, 8, 2, 0><<<11, 512, skinny_lds(1, 8, Bp), S>>>(pj, d, 0);
        }), wbytes + bpj + bap);
  }
  // K2: attention LSTM prenet part K = 256 + pq partials
  SkArgs a2{};
  a2.njobs = 1;
  a2.MT = MT;
  {
    SkJob& J = a2.job[0];
    J.seg[0] = {pb, 16 * 256, 256};
    J.nseg = 1;
    J.K = 256;
    J.W = Watt;
    J.ntiles = 256;
    J.epi = EPI_LSTM;
    J.addin = gatt;
    J.addin_ld = 4096;
    J.h_out = hatt;
    J.c_state = cst;
    J.hc_ld = 1024;
    J.WqT = WqT;
    J.pq_part = pq;
    J.pq_cap = 256;
  }
  const double b2 = 4096.0 * 256 * 4;
  if (MT == 2) {
    sk_report("K2 <4,4>", 64, [&] { skinny_kernel<4, 4, 2, 0><<<64, 1024, skinny_lds(4, 4, Bp), S>>>(a2, d, 0); });
    sk_report("K4 <1,4>", 256, [&] { skinny_kernel<1, 4, 2, 0><<<256, 256, skinny_lds(1, 4, Bp), S>>>(a4, d, 0); });
    sk_report("proj <1,4>", 11, [&] { skinny_kernel<1, 4, 2, 0><<<11, 256, skinny_lds(1, 4, Bp), S>>>(pj, d, 0); });
    sk_report("proj+att-pre <1,4>", 267, [&] { skinny_kernel<1, 4, 2, 0><<<267, 256, skinny_lds(1, 4, Bp), S>>>(both5, d, 0); });
    rep("K2 <1,4> D=4 (pq 256)", time_graph([&] { skinny_kernel<1, 4, 2, 4><<<256, 256, skinny_lds(1, 4, Bp), S>>>(a2, d, 0); }), b2);
    rep("K2 <2,4> D=4 (pq 128)", time_graph([&] { skinny_kernel<2, 4, 2, 4><<<128, 512, skinny_lds(2, 4, Bp), S>>>(a2, d, 0); }), b2);
    rep("K2 <4,2> D=4", time_graph([&] { skinny_kernel<4, 2, 2, 4><<<64, 512, skinny_lds(4, 2, Bp), S>>>(a2, d, 0); }), b2);
    rep("K2 <4,2> D=8", time_graph([&] { skinny_kernel<4, 2, 2, 8><<<64, 512, skinny_lds(4, 2, Bp), S>>>(a2, d, 0); }), b2);
    rep("K2 <4,1> D=16", time_graph([&] { skinny_kernel<4, 1, 2, 16><<<64, 256, skinny_lds(4, 1, Bp), S>>>(a2, d, 0); }), b2);
    rep("K2 <4,4> D=4", time_graph([&] { skinny_kernel<4, 4, 2, 4><<<64, 1024, skinny_lds(4, 4, Bp), S>>>(a2, d, 0); }), b2);
    rep("K2 <4,4> D=2", time_graph([&] { skinny_kernel<4, 4, 2, 2><<<64, 1024, skinny_lds(4, 4, Bp), S>>>(a2, d, 0); }), b2);
  }
  // K3: attention over T_max positions
  for (int T : {16, 64, 168}) {
    int* lens;
    HIP_OK(hipMalloc(&lens, 64 * 4));
    std::vector<int> hl(64, T);
    HIP_OK(hipMemcpy(lens, hl.data(), 64 * 4, hipMemcpyHostToDevice));
    DecDev da = d;
    da.lens = lens;
    da.T_max = T;
    da.S_cap = 1;
    float* align = dalloc((size_t)B * T);
    da.align_out = align;
    AttnArgs p{};
    p.pq_part = pq;
    p.npq = 128;
    p.Bp = Bp;
    p.alpha = dalloc((size_t)B * T);
    p.alpha_cum = dalloc((size_t)B * T);
    p.Wloc = dalloc(32 * 62);
    p.WdT = dalloc(32 * 128);
    p.v = dalloc(128);
    p.bv = 0.1f;
    p.penc = dalloc((size_t)B * T * 128);
    p.energy = dalloc((size_t)B * T);
    p.enc = dalloc((size_t)B * T * 512);
    p.ctx = dalloc((size_t)Bp * 512);
    const int nch = (T + 15) / 16;
    p.part_s = dalloc((size_t)B * nch);
    p.part_m = dalloc((size_t)B * nch);
    p.part_u = dalloc((size_t)B * nch * 512);
    unsigned* cnt;
    HIP_OK(hipMalloc(&cnt, 64 * 4));
    HIP_OK(hipMemset(cnt, 0, 64 * 4));
    p.counter = cnt;
    p.nchmax = nch;
    for (int sm = 0; sm < 2; ++sm) {
      p.softmax = sm;
      char name[64];
      snprintf(name, sizeof(name), "K3 attention T=%d %s", T, sm ? "softmax" : "sigmoid");
      rep(name, time_graph([&] { launch_attention(p, da, 0, S); }), 1.0);
      rep("   256 thr, 16 pos", time_graph([&] { attn_kernel<256, 16><<<dim3(nch, B), 256, 0, S>>>(p, da, 0); }), 1.0);
      rep("   512 thr, 16 pos", time_graph([&] { attn_kernel<512, 16><<<dim3(nch, B), 512, 0, S>>>(p, da, 0); }), 1.0);
      rep("   512 thr, 32 pos", time_graph([&] { attn_kernel<512, 32><<<dim3((T + 31) / 32, B), 512, 0, S>>>(p, da, 0); }), 1.0);
      // one traced launch: phase durations (us) averaged over workgroups
      std::vector<unsigned long long> tr(64 * 64 * 9, 0);
      HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(attn_trace), tr.data(), tr.size() * 8));
      time_graph([&] { launch_attention(p, da, 0, S); }, 20, 2);
      HIP_OK(hipStreamSynchronize(S));
      HIP_OK(hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(attn_trace), tr.size() * 8));
      const int nwg = nch * B;
      unsigned long long tmin = ~0ull, tmax = 0;
      double ph[9] = {0};
      int nlast = 0;
      double cph[3] = {0};
      for (int w = 0; w < nwg; ++w) {
        const unsigned long long* t = &tr[(long)w * 9];
        tmin = std::min(tmin, t[0]);
        for (int k = 1; k <= 6; ++k) ph[k] += (double)(t[k] - t[k - 1]) / nwg;
        if (t[8]) {
          ++nlast;
          cph[0] += t[7] - t[6];
          cph[1] += t[8] - t[7];
          tmax = std::max(tmax, t[8]);
        }
      }
      double st = 0;
      for (int w = 0; w < nwg; ++w) st += (double)(tr[(long)w * 9] - tmin) / nwg;
      printf("   start skew avg %.2f | load %.2f pq %.2f conv %.2f energy %.2f ctx+store %.2f publish %.2f | combine-load %.2f finish %.2f | span %.2f us\n",
             st / 100, ph[1] / 100, ph[2] / 100, ph[3] / 100, ph[4] / 100, ph[5] / 100, ph[6] / 100,
             cph[0] / nlast / 100, cph[1] / nlast / 100, (double)(tmax - tmin) / 100);
    }
  }
  HIP_OK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
