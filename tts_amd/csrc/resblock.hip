// Fused MelGAN ResidualStack block on gfx950 (TTS/vocoder/layers/melgan.py:5-39):
//   h = conv_k3_dil_d(ReflectionPad(d)(LeakyReLU(x))) + b_d
//   y = shortcut(x) + conv1x1(LeakyReLU(h))  ==  [W_1x1 | W_sc] . [lrelu(h); x] + (b_1x1 + b_sc)
// One workgroup owns ALL C output channels for TQ time positions, so the hidden activation h
// never leaves the CU: phase 1 accumulates h in MFMA registers over 16-channel chunks of the
// reflect-padded, LReLU'd input (double-buffered staging; the raw centre columns are kept in LDS
// for the shortcut), phase 2 runs the concatenated 1x1 GEMM (K = 2C) straight from LDS. Versus two
// launches this saves writing and re-reading h (B*C*L floats) plus the second staging pass.
#include "common.h"

constexpr int RB_DMAX = 27;  // largest dilation (3^3, num_res_blocks <= 4)

template <int C, int TQ, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void resblock_kernel(ResArgs a) {
  constexpr int NTHR = 64 * WM * WN;
  static_assert(WM * WN == 4 || WM * WN == 8, "4 or 8 waves");
  constexpr int MI = C / 16 / WM;
  constexpr int NI = TQ / 16 / WN;
  static_assert(MI * 16 * WM == C && NI * 16 * WN == TQ, "tile split");
  constexpr int ROWMAX = TQ + 2 * RB_DMAX + 1;
  constexpr int SPT = (16 * ROWMAX + NTHR - 1) / NTHR;
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int b = blockIdx.y;
  const int L = (a.lens[b] + a.len_add) * a.mul;
  const int q0 = blockIdx.x * TQ;
  if (q0 >= L) return;
  const int d = a.dil;
  const int ROW = TQ + 2 * d + 1;
  const int XS = (16 * ROW + 3) & ~3;
  float* X0 = smem;
  float* X1 = smem + XS;
  float* HX = smem + 2 * XS;                           // [2C][TQ]: lrelu(h) then raw x (centre)

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int qb = wn * 16 * NI + (lane & 15);
  const int g4 = 4 * (lane >> 4);
  const int mt0 = wm * MI;

  const float* xb = a.x + (long)b * a.sb;
  const int i0 = q0 - d;
  const bool interior = i0 >= 0 && i0 + TQ + 2 * d <= L;
  int sc_[SPT], sp_[SPT];
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int e = tid + NTHR * j;
    sc_[j] = e / ROW;
    sp_[j] = e - sc_[j] * ROW;
  }
  float st[SPT];
  // clamped (always valid) addresses, no per-element guard: a guarded load becomes an exec-masked
  // branch per element; slots past 16 x (TQ + 2d) are loaded but never stored
  auto stage_load = [&](int chunk) {
    const float* bp = xb + (long)(chunk * 16) * a.Ls;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int c = min(sc_[j], 15);
      int i = i0 + sp_[j];
      if (!interior) {  // reflection (torch ReflectionPad1d)
        if (i < 0) i = -i;
        if (i >= L) i = 2 * (L - 1) - i;
      }
      i = i < 0 ? 0 : (i >= L ? L - 1 : i);
      st[j] = bp[(long)c * a.Ls + i];
    }
  };
  auto stage_store = [&](float* X, int chunk) {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int e = tid + NTHR * j;
      if (e < 16 * ROW) {
        X[e] = lrelu02(st[j]);
        const int p = sp_[j] - d;
        if (p >= 0 && p < TQ) HX[(C + chunk * 16 + sc_[j]) * TQ + p] = st[j];  // raw x for the shortcut
      }
    }
  };

  // Weight fragments come from L2 (every workgroup streams all of Wd and Wf): a ring of 3
  // k-chunks per wave keeps one whole staging chunk of weights in flight. The ring runs over
  // the concatenated sequence [Wd chunks 0..NKC1) [Wf chunks 0..NKC2), so phase 2's first
  // weights are already loaded when phase 1 ends.
  constexpr int NKC1 = 3 * C / 16;
  constexpr int NKC2 = 2 * C / 16;
  const f32x4* Wd = reinterpret_cast<const f32x4*>(a.Wd);
  const f32x4* Wf = reinterpret_cast<const f32x4*>(a.Wf);
  f32x4 ring[3][MI];
  auto wload = [&](f32x4 (&r)[MI], int seq) {
    const bool p1 = seq < NKC1;
    const f32x4* base = p1 ? Wd : Wf;
    const int nk = p1 ? NKC1 : NKC2;
    const int kc = p1 ? seq : min(seq - NKC1, NKC2 - 1);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) r[mi] = base[((long)(mt0 + mi) * nk + kc) * 64 + lane];
  };

  // ---------------- phase 1: h = Wd . lrelu(x) (K = 3C) ----------------
  f32x4 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  stage_load(0);
#pragma unroll
  for (int u = 0; u < 3; ++u) wload(ring[u], u);
  stage_store(X0, 0);
  __syncthreads();
  constexpr int NCH = C / 16;
  for (int chunk = 0; chunk < NCH; ++chunk) {
    float* X = (chunk & 1) ? X1 : X0;
    if (chunk + 1 < NCH) stage_load(chunk + 1);
    // keep the scheduler from sinking the staging loads to their stores (that made them synchronous)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kq = 0; kq < 3; ++kq) {
      // all 4 x NI operand reads of this k-chunk first (one LDS wait), tap offsets in registers
      float bv[4][NI];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) bv[s][ni] = X[(g4 + s) * ROW + kq * d + qb + ni * 16];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = MFMA16(ring[kq][mi][s], bv[s][ni], acc[mi][ni]);
      // reload this ring slot in place, after its MFMAs (no register rotation, no vmcnt(0))
      wload(ring[kq], (chunk + 1) * 3 + kq);
    }
    if (chunk + 1 < NCH) stage_store((chunk & 1) ? X0 : X1, chunk + 1);
    __syncthreads();
  }
  // h -> lrelu(h + b_d) into HX[0:C)
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = (mt0 + mi) * 16 + g4 + j;
      const float bd = a.bd[co];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) HX[co * TQ + qb + ni * 16] = lrelu02(acc[mi][ni][j] + bd);
    }
  }
  __syncthreads();
  // ---------------- phase 2: y = [W1 | Wsc] . [lrelu(h); x] (K = 2C) ----------------
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kc0 = 0; kc0 < NKC2; kc0 += 3) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int kc = kc0 + u;
      if (kc >= NKC2) break;  // C/8 chunks need not be a multiple of 3 (wave-uniform)
      const float* hrow = HX + (kc * 16 + g4) * TQ + qb;
      float bv[4][NI];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) bv[s][ni] = hrow[s * TQ + ni * 16];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = MFMA16(ring[u][mi][s], bv[s][ni], acc[mi][ni]);
      wload(ring[u], NKC1 + kc + 3);
    }
  }
  float* yb = a.y + (long)b * a.sb;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = (mt0 + mi) * 16 + g4 + j;
      const float bf = a.bf[co];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int q = q0 + qb + ni * 16;
        if (q < L) yb[(long)co * a.Ls + q] = acc[mi][ni][j] + bf;
      }
    }
  }
}

template <int C, int TQ, int WM, int WN>
static void launch_rb(const ResArgs& a, hipStream_t s) {
  const int ROW = TQ + 2 * a.dil + 1;
  const size_t lds = ((size_t)2 * ((16 * ROW + 3) & ~3) + (size_t)2 * C * TQ) * 4;
  dim3 grid((a.max_q + TQ - 1) / TQ, a.B);
  resblock_kernel<C, TQ, WM, WN><<<grid, 64 * WM * WN, lds, s>>>(a);
}

void launch_resblock(const ResArgs& a, int C, hipStream_t s) {
  TTS_CHECK(a.dil >= 1 && a.dil <= RB_DMAX, "resblock: dilation must be in [1, 27] (num_res_blocks <= 4)");
  if (a.max_q <= 0 || a.B <= 0) return;
  // tiles from tools/voc_bench.hip (C2 shapes)
  switch (C) {
    case 192: launch_rb<192, 32, 4, 1>(a, s); break;
    case 96: launch_rb<96, 64, 2, 2>(a, s); break;
    case 48: launch_rb<48, 128, 1, 8>(a, s); break;
    case 256: launch_rb<256, 32, 4, 1>(a, s); break;
    case 128: launch_rb<128, 64, 2, 2>(a, s); break;
    case 64: launch_rb<64, 128, 1, 8>(a, s); break;
    case 32: launch_rb<32, 64, 1, 4>(a, s); break;
    default: TTS_CHECK(false, "resblock: unsupported channel count");
  }
  HIP_OK(hipGetLastError());
}
