// Tacotron2 autoregressive decoder step kernels (gfx950).
//
// One reference decoder step (TTS/tts/layers/tacotron2.py:354-369 -> decode :259-298) becomes a
// chain of 7 stream-ordered launches, captured once into a hipGraph of CHUNK steps and
// replayed; the step index lives in device memory (DecCtl::base + j) so the same graph serves
// every chunk, and the reference's per-step host sync (`if stop_token > ...`, :362) becomes a
// device-side done flag per utterance plus an all_done word that turns every later kernel
// into an early exit.
//
//   K1a  stop(t-1) from the projection kernel's partial dots + done flags
//        || prenet layer 1 (common_layers.py:76-82)
//   K1b  prenet layer 2
//   K2   attention_rnn LSTMCell (only the K=256 prenet part; the ctx/h part was precomputed
//        by K4 of the previous step) + partial query projection (common_layers.py:272)
//   K3a  location-sensitive energies over T chunks (common_layers.py:268-278, 90-110)
//   K3b  sigmoid/softmax norm, alpha_cum, alignment, context (common_layers.py:347-366)
//   K4   decoder_rnn LSTMCell (tacotron2.py:279-282) || next step's attention_rnn ctx/h part
//   K5   linear_projection (tacotron2.py:286-289) + frame store + stopnet partial dots (:291-295)
//
// All GEMMs are "skinny" (M = batch <= 64): v_mfma_f32_16x16x4_f32 with M = 16 utterances,
// N = 16 gate rows, weights pre-swizzled into fragment order (one contiguous 1 KiB read per
// wave instruction), K split across the waves of a workgroup and reduced through LDS in a
// fixed order (deterministic).
//
// Every kernel here is latency-bound (microseconds of work, ~1 us per dependent trip to
// MALL/HBM), so each one issues all of its independent global loads first -- including before
// the all_done early-exit test -- never guards a load with a per-element condition (indices are
// clamped instead, cdna_hip_programming.md §5 trap (c)), and the GEMM k-loop is a two-stage
// register pipeline: fragments for k-group g+1 are in flight while group g's MFMAs issue.
#include "common.h"
#include "decoder.h"

template <int MT, int U>
struct SkFrag {
  f32x4 w[U];
  f32x4 x[U][MT];
};

// Per-wave k-loop state. Segment bases, boundaries and strides are resolved once into
// registers: reading SkJob fields inside the loop made hipcc emit a dependent load plus
// `s_waitcnt vmcnt(0)` before every weight load, draining the pipeline.
template <int MT, int NTHR = 256>
struct SkPipe {
  // 1024-thread workgroups are capped at 128 VGPRs: shallower groups, the 4 waves per SIMD hide latency
  static constexpr int U = (NTHR >= 1024 || MT > 2) ? 2 : 4;
  using Frag = SkFrag<MT, U>;
  const f32x4* Wv;
  const float* xb0;
  long d01, d12;  // element offsets xb1 - xb0, xb2 - xb1
  int ld0, dl01, dl12, e0, e1;
  int kc_lo, kc_hi;
  __device__ __forceinline__ void init(const SkJob& J, int tile, int w, int KS, int lane) {
    const int nkc = J.K / 16;
    kc_lo = (w * nkc) / KS;
    kc_hi = ((w + 1) * nkc) / KS;
    Wv = reinterpret_cast<const f32x4*>(J.W) + (long)tile * nkc * 64 + lane;
    const int row = lane & 15, kl = 4 * (lane >> 4);
    // read every field by value first: selecting between member addresses forces the
    // kernarg struct into scratch
    const int ns = J.nseg;
    const float* p0 = J.seg[0].ptr;
    const float* p1 = J.seg[1].ptr;
    const float* p2 = J.seg[2].ptr;
    const int l0 = J.seg[0].ld, l1 = J.seg[1].ld, l2 = J.seg[2].ld;
    const int k0 = J.seg[0].K, k1 = J.seg[1].K;
    const int ld1 = ns > 1 ? l1 : l0;
    const int ld2 = ns > 2 ? l2 : ld1;
    ld0 = l0;
    dl01 = ld1 - ld0;
    dl12 = ld2 - ld1;
    e0 = k0 / 16;
    e1 = ns > 1 ? e0 + k1 / 16 : (1 << 30);
    if (ns < 2) e0 = 1 << 30;
    xb0 = p0 + (long)row * ld0 + kl;
    const float* xb1 = (ns > 1 ? p1 : p0) + (long)row * ld1 + kl - (long)e0 * 16;
    const float* xb2 = (ns > 2 ? p2 : p0) + (long)row * ld2 + kl - (long)e1 * 16;
    d01 = xb1 - xb0;
    d12 = xb2 - xb1;
  }
  // load k-group [kc0, kc0+U) (indices clamped to the last chunk: always valid addresses)
  __device__ __forceinline__ void load(SkFrag<MT, U>& F, int kc0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kc = min(kc0 + u, kc_hi - 1);
      F.w[u] = Wv[(long)kc * 64];
      // segment select as conditional adds of deltas (a 3-way pointer select became a
      // scratch lookup table)
      const long d = (kc >= e0 ? d01 : 0l) + (kc >= e1 ? d12 : 0l);
      const float* xp = xb0 + d + kc * 16;
      const int ld = ld0 + (kc >= e0 ? dl01 : 0) + (kc >= e1 ? dl12 : 0);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) F.x[u][mt] = *reinterpret_cast<const f32x4*>(xp + (long)mt * 16 * ld);
    }
  }
  __device__ __forceinline__ void mma(const SkFrag<MT, U>& F, int nvalid, f32x4 (&acc)[MT]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < nvalid) {  // wave-uniform
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[mt] = MFMA16(F.x[u][mt][s], F.w[u][s], acc[mt]);
      }
    }
  }
  // first group's loads: issue before anything that waits on memory
  __device__ __forceinline__ void prefetch(Frag& A) { load(A, kc_lo); }
  __device__ __forceinline__ void run(Frag& A, Frag& B, f32x4 (&acc)[MT]) {
    for (int kc0 = kc_lo; kc0 < kc_hi; kc0 += 2 * U) {
      if (kc0 + U < kc_hi) load(B, kc0 + U);
      mma(A, kc_hi - kc0, acc);
      if (kc0 + U >= kc_hi) break;
      if (kc0 + 2 * U < kc_hi) load(A, kc0 + 2 * U);
      mma(B, kc_hi - kc0 - U, acc);
    }
  }
};

// partial sums in LDS: [wave][m][17]
template <int MT>
__device__ __forceinline__ void skinny_to_lds(float* part, int w, int lane, const f32x4 (&acc)[MT]) {
  constexpr int Bp = MT * 16;
  float* p = part + (long)w * Bp * 17;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) p[(mt * 16 + 4 * (lane >> 4) + j) * 17 + (lane & 15)] = acc[mt][j];
}

template <int KS, int Bp>
__device__ __forceinline__ float skinny_sum(const float* part, int m, int n) {
  float s = part[m * 17 + n];
#pragma unroll
  for (int w = 1; w < KS; ++w) s += part[(w * Bp + m) * 17 + n];
  return s;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// stopnet h-part: stop_part[ntiles][m] = w_h . h_dec[m]   (one extra workgroup of the projection)
template <int MT>
__device__ void stop_h_role(const SkJob& J, int nthr) {
  constexpr int Bp = MT * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = nthr / 64;
  float w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = J.stop_wh[lane + 64 * i];
  for (int m = wave; m < Bp; m += nw) {
    const float* h = J.stop_h + (long)m * 1024;
    float x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = h[lane + 64 * i];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s = fmaf(w[i], x[i], s);
    s = wave_sum(s);
    if (lane == 0) J.stop_part[(long)J.ntiles * Bp + m] = s;
  }
}

// --------------------------------------------------------------------------------------
// generic skinny kernel: NT tiles per workgroup, KS waves per tile, MT batch tiles of 16
// --------------------------------------------------------------------------------------
// body of one workgroup for job J (always called with a constant job index so J's fields stay
// scalar loads from the kernarg segment; a runtime-selected reference made hipcc copy the whole
// argument struct to scratch)
template <int NT, int KS, int MT>
__device__ __forceinline__ void skinny_body(const SkJob& J, const DecDev& D, int jstep, int wg, float* smem) {
  constexpr int Bp = MT * 16;
  constexpr int nthr = NT * KS * 64;
  constexpr int SITEMS = (NT * Bp * 16 + nthr - 1) / nthr;  // store items per thread (<= 4)
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int grp = wave / KS, w = wave % KS;
  const int all_done = D.ctl->all_done;
  if (J.stop_h && wg == J.ntiles / NT) {
    if (!all_done) stop_h_role<MT>(J, nthr);
    return;
  }
  const int tile = wg * NT + grp;
  SkPipe<MT, nthr> pipe;
  typename SkPipe<MT, nthr>::Frag fa, fb;
  pipe.init(J, tile, w, KS, lane);
  pipe.prefetch(fa);
  // epilogue operands, fetched under the GEMM
  float eb[SITEMS];
  float lb[4] = {0.f, 0.f, 0.f, 0.f}, la[4] = {0.f, 0.f, 0.f, 0.f}, lc = 0.f;
  float wq[4 * NT];
  if (J.epi == EPI_STORE) {
#pragma unroll
    for (int i = 0; i < SITEMS; ++i) {
      const int idx = min(tid + i * nthr, NT * Bp * 16 - 1);
      const int g = idx / (Bp * 16), n = idx % 16;
      eb[i] = J.bias ? J.bias[(wg * NT + g) * 16 + n] : 0.f;
    }
  } else {
    const int idx = min(tid, NT * Bp * 4 - 1);
    const int g = idx / (Bp * 4), rem = idx % (Bp * 4);
    const int m = rem / 4, u = rem % 4;
    const int tl = wg * NT + g;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int col = tl * 16 + q * 4 + u;
      if (J.bias) lb[q] = J.bias[col];
      if (J.addin) la[q] = J.addin[(long)m * J.addin_ld + col];
    }
    lc = J.c_state[(long)m * J.hc_ld + tl * 4 + u];
    if (J.pq_part) {
      const int a = tid % 128;
#pragma unroll
      for (int u2 = 0; u2 < 4 * NT; ++u2) wq[u2] = J.WqT[(long)(wg * NT * 4 + u2) * 128 + a];
    }
  }
  if (all_done) return;
  const int t = D.ctl->base + jstep;

  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  pipe.run(fa, fb, acc);
  float* part = smem + (long)grp * KS * Bp * 17;
  float* extra = smem + (long)NT * KS * Bp * 17;  // [NT][Bp][16]
  skinny_to_lds<MT>(part, w, lane, acc);
  __syncthreads();

  if (J.epi == EPI_STORE) {
#pragma unroll
    for (int i = 0; i < SITEMS; ++i) {
      const int idx = tid + i * nthr;
      if (idx >= NT * Bp * 16) break;
      const int g = idx / (Bp * 16), rem = idx % (Bp * 16);
      const int m = rem / 16, n = rem % 16;
      const int col = (wg * NT + g) * 16 + n;
      float v = skinny_sum<KS, Bp>(smem + (long)g * KS * Bp * 17, m, n) + eb[i];
      if (J.act == 1) v = fmaxf(v, 0.f);
      J.out[(long)m * J.out_ld + col] = v;
      if (J.frames_r > 0 && m < D.B && col < 80 * J.frames_r && t < D.S_cap && !D.done[m])
        D.dec_out[((long)m * D.S_cap + t) * J.frames_r * 80 + col] = v;
      if (J.stop_part) extra[idx] = v * J.stop_wy[col];
    }
    if (J.stop_part) {
      __syncthreads();
      for (int idx = tid; idx < NT * Bp; idx += nthr) {
        const int g = idx / Bp, m = idx % Bp;
        const float* e = extra + ((long)g * Bp + m) * 16;
        float s = e[0];
#pragma unroll
        for (int n = 1; n < 16; ++n) s += e[n];
        J.stop_part[(long)(wg * NT + g) * Bp + m] = s;
      }
    }
  } else {  // EPI_LSTM: tile rows are gate-major [i0..i3 f0..f3 g0..g3 o0..o3] of 4 units
    float* hs = extra;  // [Bp][4*NT]
    if (tid < NT * Bp * 4) {
      const int g = tid / (Bp * 4), rem = tid % (Bp * 4);
      const int m = rem / 4, u = rem % 4;
      const int tl = wg * NT + g;
      const float* pg = smem + (long)g * KS * Bp * 17;
      float pre[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) pre[q] = skinny_sum<KS, Bp>(pg, m, q * 4 + u) + lb[q] + la[q];
      const long ci = (long)m * J.hc_ld + tl * 4 + u;
      const float ig = 1.f / (1.f + expf(-pre[0]));
      const float fg = 1.f / (1.f + expf(-pre[1]));
      const float gg = tanhf(pre[2]);
      const float og = 1.f / (1.f + expf(-pre[3]));
      const float c = fg * lc + ig * gg;
      const float h = og * tanhf(c);
      J.c_state[ci] = c;
      J.h_out[ci] = h;
      hs[m * 4 * NT + g * 4 + u] = h;
    }
    if (J.pq_part) {  // partial query projection over this workgroup's 4*NT hidden units
      __syncthreads();
      for (int idx = tid; idx < Bp * 128; idx += nthr) {
        const int m = idx / 128, a = idx % 128;
        float s = 0.f;
#pragma unroll
        for (int u = 0; u < 4 * NT; ++u) s = fmaf(wq[u], hs[m * 4 * NT + u], s);
        J.pq_part[((long)wg * Bp + m) * 128 + a] = s;
      }
    }
  }
}

template <int NT, int KS, int MT>
__global__ __launch_bounds__(NT * KS * 64) void skinny_kernel(SkArgs A, DecDev D, int jstep) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int n0 = A.job[0].ntiles / NT;
  if (A.njobs > 1 && (int)blockIdx.x >= n0)
    skinny_body<NT, KS, MT>(A.job[1], D, jstep, (int)blockIdx.x - n0, smem);
  else
    skinny_body<NT, KS, MT>(A.job[0], D, jstep, (int)blockIdx.x, smem);
}

// --------------------------------------------------------------------------------------
// K1a: stop decision for step t-1 (one workgroup) || prenet layer 1 (16 workgroups)
// --------------------------------------------------------------------------------------
constexpr int NPARTS_MAX = 64;

template <int MT>
__global__ __launch_bounds__(256) void prenet1_stop_kernel(SkArgs A, DecDev D, StopArgs S, int jstep) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int Bp = MT * 16;
  if (blockIdx.x == A.job[0].ntiles) {
    // ---- stop role: logit = sum of the projection kernel's partial dots + b_s; sigma;
    //      reference stop rule (tacotron2.py:357-366): stop iff sigma > thr and t > 0,
    //      else stop when max_decoder_steps outputs exist. One thread per utterance.
    __shared__ int dflag[64];
    const int m = min(tid, Bp - 1);
    float pv[NPARTS_MAX];
#pragma unroll
    for (int p = 0; p < NPARTS_MAX; ++p) pv[p] = S.part[(long)min(p, S.nparts - 1) * S.Bp + m];
    const int dn0 = D.done[m];
    const int mx = D.max_steps[m];
    const int all_done = D.ctl->all_done;
    const int t = D.ctl->base + jstep;
    if (all_done) return;
    if (tid < D.B) {
      int dn = dn0;
      if (t >= 1 && !dn) {
        float s = 0.f;
#pragma unroll
        for (int p = 0; p < NPARTS_MAX; ++p)
          if (p < S.nparts) s += pv[p];
        const float logit = s + S.bs;
        const float sg = 1.f / (1.f + expf(-logit));
        if (t - 1 < D.S_cap) D.stop_out[(long)m * D.S_cap + (t - 1)] = sg;
        const bool st = (sg > S.threshold) && (t - 1) > 0;
        if (st || t >= mx) {
          D.done[m] = 1;
          D.steps[m] = t;
          D.status[m] = st ? 1 : 2;
          dn = 1;
        }
      }
      dflag[m] = dn;
    }
    __syncthreads();
    if (tid == 0) {
      int all = 1;
      for (int k = 0; k < D.B; ++k) all &= dflag[k];
      D.ctl->all_done = all;
    }
    return;
  }
  // ---- prenet layer 1: relu(W1 . memory) with memory = y[:, 80(r-1):80r] (go frame = 0) ----
  const SkJob& J = A.job[0];
  const int tile = blockIdx.x;
  SkPipe<MT> pipe;
  typename SkPipe<MT>::Frag fa, fb;
  pipe.init(J, tile, wave, 4, lane);
  pipe.prefetch(fa);
  if (D.ctl->all_done) return;
  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  pipe.run(fa, fb, acc);
  skinny_to_lds<MT>(smem, wave, lane, acc);
  __syncthreads();
  for (int idx = tid; idx < Bp * 16; idx += 256) {
    const int m = idx / 16, n = idx % 16;
    const float v = skinny_sum<4, Bp>(smem, m, n);
    J.out[(long)m * J.out_ld + tile * 16 + n] = fmaxf(v, 0.f);
  }
}

// --------------------------------------------------------------------------------------
// K3a: energies e[b][t] for a chunk of TCH encoder positions
// --------------------------------------------------------------------------------------
constexpr int TCH = 16;
constexpr int LOCK = 31, LOCF = 32, ADIM = 128, NPQ = 64;

__global__ __launch_bounds__(256) void attn_energy_kernel(AttnArgs P, DecDev D) {
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * TCH;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int a = tid & 127, grp = tid >> 7;
  __shared__ float red[2][ADIM];
  __shared__ float A0[TCH + LOCK], A1[TCH + LOCK];
  __shared__ float Wl[LOCF * 2 * LOCK];
  __shared__ float f[LOCF][TCH];
  __shared__ float er[2][TCH];
  const int Bp = P.Bp;
  const int T = D.lens[b];
  const int Tm1 = max(T - 1, 0);
  // -- every independent global load up front (clamped indices, no guarded loads) --
  float pen[TCH / 2];
#pragma unroll
  for (int i = 0; i < TCH / 2; ++i) {
    const int t = min(t0 + grp * (TCH / 2) + i, Tm1);
    pen[i] = P.penc[((long)b * D.T_max + t) * ADIM + a];
  }
  float wd[LOCF];
#pragma unroll
  for (int c = 0; c < LOCF; ++c) wd[c] = P.WdT[c * ADIM + a];
  const float va = P.v[a];
  float pp[NPQ / 2];
#pragma unroll
  for (int i = 0; i < NPQ / 2; ++i) pp[i] = P.pq_part[((long)(grp * (NPQ / 2) + i) * Bp + b) * ADIM + a];
  float a0 = 0.f, a1 = 0.f;
  {
    const int pos = t0 - (LOCK - 1) / 2 + min(tid, TCH + LOCK - 2);
    const int pc = min(max(pos, 0), Tm1);
    a0 = P.alpha[(long)b * D.T_max + pc];
    a1 = P.alpha_cum[(long)b * D.T_max + pc];
    if (pos < 0 || pos >= T) a0 = a1 = 0.f;
  }
  float wl[(LOCF * 2 * LOCK + 255) / 256];
#pragma unroll
  for (int i = 0; i < (LOCF * 2 * LOCK + 255) / 256; ++i) wl[i] = P.Wloc[min(tid + 256 * i, LOCF * 2 * LOCK - 1)];
  if (D.ctl->all_done || D.done[b] || t0 >= T) return;
  if (tid < TCH + LOCK - 1) {
    A0[tid] = a0;
    A1[tid] = a1;
  }
#pragma unroll
  for (int i = 0; i < (LOCF * 2 * LOCK + 255) / 256; ++i)
    if (tid + 256 * i < LOCF * 2 * LOCK) Wl[tid + 256 * i] = wl[i];
  // query projection = sum of the attention-LSTM kernel's 64 partials (fixed order)
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPQ / 2; ++i) s += pp[i];
  red[grp][a] = s;
  __syncthreads();
  const float pqa = red[0][a] + red[1][a];
  // location conv: f[c][tt] = sum_i sum_k Wl[c][i][k] * A_i[tt + k]
  for (int idx = tid; idx < LOCF * TCH; idx += 256) {
    const int c = idx / TCH, tt = idx % TCH;
    float sc = 0.f;
    const float* w0 = Wl + c * 2 * LOCK;
#pragma unroll
    for (int k = 0; k < LOCK; ++k) sc = fmaf(w0[k], A0[tt + k], sc);
#pragma unroll
    for (int k = 0; k < LOCK; ++k) sc = fmaf(w0[LOCK + k], A1[tt + k], sc);
    f[c][tt] = sc;
  }
  __syncthreads();
  // loc = W_dense . f ; e = v . tanh(pq + loc + penc) + b_v
#pragma unroll
  for (int i = 0; i < TCH / 2; ++i) {
    const int tt = grp * (TCH / 2) + i;
    float l = 0.f;
#pragma unroll
    for (int c = 0; c < LOCF; ++c) l = fmaf(wd[c], f[c][tt], l);
    float z = (t0 + tt < T) ? tanhf(pqa + l + pen[i]) * va : 0.f;
    z = wave_sum(z);
    if (lane == 0) er[wave & 1][tt] = z;
  }
  __syncthreads();
  if (tid < TCH && t0 + tid < T) P.energy[(long)b * D.T_max + t0 + tid] = er[0][tid] + er[1][tid] + P.bv;
}

// --------------------------------------------------------------------------------------
// K3b: normalisation, alignment, alpha_cum and the context vector (slice of 128 dims)
// --------------------------------------------------------------------------------------
__device__ __forceinline__ float block_reduce(float v, float* wred, bool is_max) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float o = __shfl_xor(v, off, 64);
    v = is_max ? fmaxf(v, o) : v + o;
  }
  __syncthreads();
  if (lane == 0) wred[wave] = v;
  __syncthreads();
  return is_max ? fmaxf(fmaxf(wred[0], wred[1]), fmaxf(wred[2], wred[3]))
                : (wred[0] + wred[1]) + (wred[2] + wred[3]);
}

constexpr int CTX_PRE = 4;  // encoder rows per thread prefetched before the normalisation

__global__ __launch_bounds__(256) void attn_context_kernel(AttnArgs P, DecDev D, int jstep) {
  const int b = blockIdx.y, slice = blockIdx.x;
  const int tid = threadIdx.x;
  extern __shared__ __attribute__((aligned(16))) float al[];  // [T_max]
  __shared__ float wred[4];
  __shared__ f32x4 cr[8][32];
  const int T = D.lens[b];
  const int Tm1 = max(T - 1, 0);
  const int d4 = tid & 31, g = tid >> 5;
  const f32x4* enc = reinterpret_cast<const f32x4*>(P.enc + (long)b * D.T_max * 512 + slice * 128) + d4;
  // prefetch: first energies and the first encoder rows of this thread's context slice
  const float* e = P.energy + (long)b * D.T_max;
  float e0 = e[min(tid, Tm1)];
  f32x4 ep[CTX_PRE];
#pragma unroll
  for (int i = 0; i < CTX_PRE; ++i) ep[i] = enc[(long)min(g + 8 * i, Tm1) * 128];
  if (D.ctl->all_done || D.done[b]) return;
  const int t_step = D.ctl->base + jstep;
  if (tid < T) al[tid] = e0;
  for (int t = tid + 256; t < T; t += 256) al[t] = e[t];
  __syncthreads();
  float mx = 0.f;
  if (P.softmax) {
    float m = -INFINITY;
    for (int t = tid; t < T; t += 256) m = fmaxf(m, al[t]);
    mx = block_reduce(m, wred, true);
  }
  float s = 0.f;
  for (int t = tid; t < T; t += 256) {
    const float x = al[t];
    const float v = P.softmax ? expf(x - mx) : 1.f / (1.f + expf(-x));
    al[t] = v;
    s += v;
  }
  const float S = block_reduce(s, wred, false);
  for (int t = tid; t < T; t += 256) {
    const float a = al[t] / S;
    al[t] = a;
    if (slice == 0) {
      P.alpha[(long)b * D.T_max + t] = a;
      P.alpha_cum[(long)b * D.T_max + t] += a;
      if (t_step < D.S_cap) D.align_out[((long)b * D.S_cap + t_step) * D.T_max + t] = a;
    }
  }
  __syncthreads();
  // context slice: ctx[b][slice*128 + d] = sum_t a_t * enc[b][t][slice*128 + d]
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < CTX_PRE; ++i)
    if (g + 8 * i < T) c += al[g + 8 * i] * ep[i];
  int t = g + 8 * CTX_PRE;
  for (; t + 24 < T; t += 32) {
    const f32x4 x0 = enc[(long)t * 128], x1 = enc[(long)(t + 8) * 128];
    const f32x4 x2 = enc[(long)(t + 16) * 128], x3 = enc[(long)(t + 24) * 128];
    c += al[t] * x0;
    c += al[t + 8] * x1;
    c += al[t + 16] * x2;
    c += al[t + 24] * x3;
  }
  for (; t < T; t += 8) c += al[t] * enc[(long)t * 128];
  cr[g][d4] = c;
  __syncthreads();
  if (tid < 32) {
    f32x4 r = cr[0][tid];
#pragma unroll
    for (int k = 1; k < 8; ++k) r += cr[k][tid];
    *reinterpret_cast<f32x4*>(P.ctx + (long)b * 512 + slice * 128 + 4 * tid) = r;
  }
}

__global__ void dec_advance_kernel(DecCtl* ctl, int n) {
  if (threadIdx.x == 0) ctl->base += n;
}

// --------------------------------------------------------------------------------------
// host launchers
// --------------------------------------------------------------------------------------
static size_t skinny_lds(int NT, int KS, int Bp) {
  return ((size_t)NT * KS * Bp * 17 + (size_t)NT * Bp * 16) * 4;
}

template <int NT, int KS>
static void launch_skinny_nt(const SkArgs& a, const DecDev& d, int jstep, int nwg, hipStream_t s) {
  const size_t lds = skinny_lds(NT, KS, a.MT * 16);
  switch (a.MT) {
    case 1: skinny_kernel<NT, KS, 1><<<nwg, NT * KS * 64, lds, s>>>(a, d, jstep); break;
    case 2: skinny_kernel<NT, KS, 2><<<nwg, NT * KS * 64, lds, s>>>(a, d, jstep); break;
    case 3: skinny_kernel<NT, KS, 3><<<nwg, NT * KS * 64, lds, s>>>(a, d, jstep); break;
    default: skinny_kernel<NT, KS, 4><<<nwg, NT * KS * 64, lds, s>>>(a, d, jstep); break;
  }
}

void launch_skinny(const SkArgs& a, const DecDev& d, int jstep, int NT, int KS, hipStream_t s) {
  TTS_CHECK(a.MT >= 1 && a.MT <= 4, "skinny: MT in [1,4]");
  for (int j = 0; j < a.njobs; ++j) {
    TTS_CHECK(a.job[j].ntiles % NT == 0, "skinny: ntiles % NT");
    if (a.job[j].epi == EPI_LSTM) TTS_CHECK(NT * a.MT * 16 * 4 <= NT * KS * 64, "skinny: LSTM items per thread");
  }
  int nwg = a.job[0].ntiles / NT + (a.njobs > 1 ? a.job[1].ntiles / NT : 0);
  if (a.njobs == 1 && a.job[0].stop_h) nwg += 1;
  if (NT == 1 && KS == 4) launch_skinny_nt<1, 4>(a, d, jstep, nwg, s);
  else if (NT == 1 && KS == 16) launch_skinny_nt<1, 16>(a, d, jstep, nwg, s);
  else if (NT == 4 && KS == 4) launch_skinny_nt<4, 4>(a, d, jstep, nwg, s);
  else TTS_CHECK(false, "skinny: unsupported tile config");
  HIP_OK(hipGetLastError());
}

void launch_prenet1_stop(const SkArgs& a, const DecDev& d, const StopArgs& st, int jstep, hipStream_t s) {
  TTS_CHECK(a.MT >= 1 && a.MT <= 4, "prenet: MT in [1,4]");
  TTS_CHECK(st.nparts >= 1 && st.nparts <= NPARTS_MAX, "stop: too many partials (r_init <= 12)");
  const size_t lds = skinny_lds(1, 4, a.MT * 16);
  const int g = a.job[0].ntiles + 1;
  switch (a.MT) {
    case 1: prenet1_stop_kernel<1><<<g, 256, lds, s>>>(a, d, st, jstep); break;
    case 2: prenet1_stop_kernel<2><<<g, 256, lds, s>>>(a, d, st, jstep); break;
    case 3: prenet1_stop_kernel<3><<<g, 256, lds, s>>>(a, d, st, jstep); break;
    default: prenet1_stop_kernel<4><<<g, 256, lds, s>>>(a, d, st, jstep); break;
  }
  HIP_OK(hipGetLastError());
}

void launch_attention(const AttnArgs& p, const DecDev& d, int jstep, hipStream_t s) {
  TTS_CHECK(p.npq == NPQ, "attention: expects 64 query partials");
  dim3 g1((d.T_max + TCH - 1) / TCH, d.B);
  attn_energy_kernel<<<g1, 256, 0, s>>>(p, d);
  HIP_OK(hipGetLastError());
  dim3 g2(4, d.B);
  attn_context_kernel<<<g2, 256, (size_t)d.T_max * 4, s>>>(p, d, jstep);
  HIP_OK(hipGetLastError());
}

void launch_dec_advance(DecCtl* ctl, int n, hipStream_t s) {
  dec_advance_kernel<<<1, 64, 0, s>>>(ctl, n);
  HIP_OK(hipGetLastError());
}
