// Tacotron2 autoregressive decoder step kernels (gfx950).
//
// One reference decoder step (TTS/tts/layers/tacotron2.py:354-369 -> decode :259-298) becomes a
// chain of 7 stream-ordered launches, captured once into a hipGraph of CHUNK steps and
// replayed; the step index lives in device memory (DecCtl::base + j) so the same graph serves
// every chunk, and the reference's per-step host sync (`if stop_token > ...`, :362) becomes a
// device-side done flag per utterance plus an all_done word that turns every later kernel
// into an early exit.
//
//   K1a  stop(t-1) + per-utterance done flags  ||  prenet layer 1 (common_layers.py:76-82)
//   K1b  prenet layer 2
//   K2   attention_rnn LSTMCell (only the K=256 prenet part; the ctx/h part was precomputed
//        by K4 of the previous step) + partial query projection (common_layers.py:272)
//   K3a  location-sensitive energies over T chunks (common_layers.py:268-278, 90-110)
//   K3b  sigmoid/softmax norm, alpha_cum, alignment, context (common_layers.py:347-366)
//   K4   decoder_rnn LSTMCell (tacotron2.py:279-282) || next step's attention_rnn ctx/h part
//   K5   linear_projection (tacotron2.py:286-289) + frame store
//
// All GEMMs are "skinny" (M = batch <= 64): v_mfma_f32_16x16x4_f32 with M = 16 utterances,
// N = 16 gate rows, weights pre-swizzled into fragment order (one contiguous 1 KiB read per
// wave instruction), K split across the waves of a workgroup and reduced through LDS in a
// fixed order (deterministic).
#include "common.h"
#include "decoder.h"

// --------------------------------------------------------------------------------------
// skinny GEMM core: partial[wave][m][n] for one 16-row tile over this wave's K range
// --------------------------------------------------------------------------------------
__device__ __forceinline__ void skinny_accumulate(const SkJob& J, int tile, int w, int KS, int MT,
                                                  int lane, f32x4 (&acc)[4]) {
  const int nkc = J.K / 16;
  const int kc_lo = (w * nkc) / KS, kc_hi = ((w + 1) * nkc) / KS;
  const f32x4* Wv = reinterpret_cast<const f32x4*>(J.W) + (long)tile * nkc * 64 + lane;
  const int row = lane & 15;
  const int kl = 4 * (lane >> 4);
  int seg_start = 0;
  for (int sgi = 0; sgi < J.nseg; ++sgi) {
    const SkSeg S = J.seg[sgi];
    const int s_lo = seg_start / 16, s_hi = (seg_start + S.K) / 16;
    const int lo = kc_lo > s_lo ? kc_lo : s_lo;
    const int hi = kc_hi < s_hi ? kc_hi : s_hi;
    const float* xb = S.ptr + (long)row * S.ld + kl - seg_start;
    for (int kc = lo; kc < hi; ++kc) {
      const f32x4 wv = Wv[(long)kc * 64];
      f32x4 xv[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        if (mt < MT) xv[mt] = *reinterpret_cast<const f32x4*>(xb + (long)mt * 16 * S.ld + kc * 16);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        if (mt < MT) {
          acc[mt] = MFMA16(xv[mt][0], wv[0], acc[mt]);
          acc[mt] = MFMA16(xv[mt][1], wv[1], acc[mt]);
          acc[mt] = MFMA16(xv[mt][2], wv[2], acc[mt]);
          acc[mt] = MFMA16(xv[mt][3], wv[3], acc[mt]);
        }
      }
    }
    seg_start += S.K;
  }
}

// part layout in LDS: [grp][w][m][17]
__device__ __forceinline__ void skinny_to_lds(float* part, int KS, int Bp, int w, int lane, int MT,
                                              const f32x4 (&acc)[4]) {
  float* p = part + (long)w * Bp * 17;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    if (mt < MT) {
#pragma unroll
      for (int j = 0; j < 4; ++j) p[(mt * 16 + 4 * (lane >> 4) + j) * 17 + (lane & 15)] = acc[mt][j];
    }
  }
}

__device__ __forceinline__ float skinny_sum(const float* part, int KS, int Bp, int m, int n) {
  float s = part[m * 17 + n];
  for (int w = 1; w < KS; ++w) s += part[((long)w * Bp + m) * 17 + n];
  return s;
}

// frame / stop bookkeeping shared by the epilogues
__device__ __forceinline__ int dec_step(const DecDev& D, int j) { return D.ctl->base + j; }

// --------------------------------------------------------------------------------------
// generic skinny kernel: NT tiles per workgroup, KS waves per tile
// --------------------------------------------------------------------------------------
template <int NT, int KS>
__global__ __launch_bounds__(NT * KS * 64) void skinny_kernel(SkArgs A, DecDev D, int jstep) {
  if (D.ctl->all_done) return;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int grp = wave / KS, w = wave % KS;
  int wg = blockIdx.x, ji = 0;
  if (A.njobs > 1 && wg >= A.job[0].ntiles / NT) {
    wg -= A.job[0].ntiles / NT;
    ji = 1;
  }
  const SkJob& J = A.job[ji];
  const int Bp = A.MT * 16;
  const int tile = wg * NT + grp;
  float* part = smem + (long)grp * KS * Bp * 17;

  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  skinny_accumulate(J, tile, w, KS, A.MT, lane, acc);
  skinny_to_lds(part, KS, Bp, w, lane, A.MT, acc);
  __syncthreads();

  const int nthr = NT * KS * 64;
  if (J.epi == EPI_STORE) {
    const int t = dec_step(D, jstep);
    for (int idx = tid; idx < NT * Bp * 16; idx += nthr) {
      const int g = idx / (Bp * 16), rem = idx % (Bp * 16);
      const int m = rem / 16, n = rem % 16;
      const int col = (wg * NT + g) * 16 + n;
      float v = skinny_sum(smem + (long)g * KS * Bp * 17, KS, Bp, m, n);
      if (J.bias) v += J.bias[col];
      if (J.addin) v += J.addin[(long)m * J.addin_ld + col];
      if (J.act == 1) v = fmaxf(v, 0.f);
      J.out[(long)m * J.out_ld + col] = v;
      if (J.frames_r > 0 && m < D.B && col < 80 * J.frames_r && t < D.S_cap && !D.done[m])
        D.dec_out[((long)m * D.S_cap + t) * J.frames_r * 80 + col] = v;
    }
  } else {  // EPI_LSTM: tile rows are gate-major [i0..i3 f0..f3 g0..g3 o0..o3] of 4 units
    float* hs = smem + (long)NT * KS * Bp * 17;  // [Bp][4*NT]
    for (int idx = tid; idx < NT * Bp * 4; idx += nthr) {
      const int g = idx / (Bp * 4), rem = idx % (Bp * 4);
      const int m = rem / 4, u = rem % 4;
      const int tl = wg * NT + g;
      const float* pg = smem + (long)g * KS * Bp * 17;
      float pre[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = tl * 16 + q * 4 + u;
        float v = skinny_sum(pg, KS, Bp, m, q * 4 + u);
        if (J.bias) v += J.bias[col];
        if (J.addin) v += J.addin[(long)m * J.addin_ld + col];
        pre[q] = v;
      }
      const int unit = tl * 4 + u;
      const long ci = (long)m * J.hc_ld + unit;
      const float ig = 1.f / (1.f + expf(-pre[0]));
      const float fg = 1.f / (1.f + expf(-pre[1]));
      const float gg = tanhf(pre[2]);
      const float og = 1.f / (1.f + expf(-pre[3]));
      const float c = fg * J.c_state[ci] + ig * gg;
      const float h = og * tanhf(c);
      J.c_state[ci] = c;
      J.h_out[ci] = h;
      hs[m * 4 * NT + g * 4 + u] = h;
    }
    if (J.pq_part) {  // partial query projection over this workgroup's 4*NT hidden units
      __syncthreads();
      const int unit0 = wg * NT * 4;
      for (int idx = tid; idx < Bp * 128; idx += nthr) {
        const int m = idx / 128, a = idx % 128;
        float s = 0.f;
        for (int u = 0; u < 4 * NT; ++u) s = fmaf(J.WqT[(long)(unit0 + u) * 128 + a], hs[m * 4 * NT + u], s);
        J.pq_part[((long)wg * Bp + m) * 128 + a] = s;
      }
    }
  }
}

// --------------------------------------------------------------------------------------
// K1a: stop decision for step t-1 (one workgroup) || prenet layer 1 (16 workgroups)
// --------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prenet1_stop_kernel(SkArgs A, DecDev D, StopArgs S, int jstep) {
  if (D.ctl->all_done) return;
  const int t = dec_step(D, jstep);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Bp = A.MT * 16;
  if (blockIdx.x == A.job[0].ntiles) {
    // ---- stop role: logit = w_s . [h_dec, y_full] + b_s; sigma; reference stop rule ----
    for (int m = wave; m < D.B; m += 4) {
      float s = 0.f;
      for (int k = lane; k < 1024; k += 64) s = fmaf(S.ws[k], S.hdec[(long)m * 1024 + k], s);
      for (int k = lane; k < S.ny; k += 64) s = fmaf(S.ws[1024 + k], S.y[(long)m * S.y_ld + k], s);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
      if (lane == 0 && t >= 1 && t <= D.S_cap && !D.done[m]) {
        const float logit = s + S.bs;
        const float sg = 1.f / (1.f + expf(-logit));
        D.stop_out[(long)m * D.S_cap + (t - 1)] = sg;
        const bool st = (sg > S.threshold) && (t - 1) > 0;
        if (st || t >= D.max_steps[m]) {
          D.done[m] = 1;
          D.steps[m] = t;
          D.status[m] = st ? 1 : 2;
        }
      }
    }
    __syncthreads();
    if (tid == 0) {
      int all = 1;
      for (int m = 0; m < D.B; ++m) all &= D.done[m];
      D.ctl->all_done = all;
    }
    return;
  }
  // ---- prenet layer 1: relu(W1 . memory) with memory = y[:, 80(r-1):80r] (go frame = 0) ----
  const SkJob& J = A.job[0];
  const int tile = blockIdx.x;
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  skinny_accumulate(J, tile, wave, 4, A.MT, lane, acc);
  skinny_to_lds(smem, 4, Bp, wave, lane, A.MT, acc);
  __syncthreads();
  for (int idx = tid; idx < Bp * 16; idx += 256) {
    const int m = idx / 16, n = idx % 16;
    const float v = skinny_sum(smem, 4, Bp, m, n);
    J.out[(long)m * J.out_ld + tile * 16 + n] = fmaxf(v, 0.f);
  }
}

// --------------------------------------------------------------------------------------
// K3a: energies e[b][t] for a chunk of TCH encoder positions
// --------------------------------------------------------------------------------------
constexpr int TCH = 16;
constexpr int LOCK = 31, LOCF = 32, ADIM = 128;

__global__ __launch_bounds__(256) void attn_energy_kernel(AttnArgs P, DecDev D) {
  if (D.ctl->all_done) return;
  const int b = blockIdx.y;
  if (D.done[b]) return;
  const int T = D.lens[b];
  const int t0 = blockIdx.x * TCH;
  if (t0 >= T) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ float pq[ADIM];
  __shared__ float red[2][ADIM];
  __shared__ float A0[TCH + LOCK], A1[TCH + LOCK];
  __shared__ float Wl[LOCF * 2 * LOCK];
  __shared__ float f[LOCF][TCH];
  __shared__ float er[2][TCH];
  const int Bp = P.Bp;
  {  // 1. query projection = sum of K2 partials (fixed order)
    const int a = tid & 127, h = tid >> 7;
    float s = 0.f;
    for (int p = h; p < P.npq; p += 2) s += P.pq_part[((long)p * Bp + b) * ADIM + a];
    red[h][a] = s;
  }
  for (int i = tid; i < TCH + LOCK - 1; i += 256) {
    const int pos = t0 - (LOCK - 1) / 2 + i;
    const bool ok = pos >= 0 && pos < T;
    A0[i] = ok ? P.alpha[(long)b * D.T_max + pos] : 0.f;
    A1[i] = ok ? P.alpha_cum[(long)b * D.T_max + pos] : 0.f;
  }
  for (int i = tid; i < LOCF * 2 * LOCK; i += 256) Wl[i] = P.Wloc[i];
  __syncthreads();
  if (tid < ADIM) pq[tid] = red[0][tid] + red[1][tid];
  // 2. location conv: f[c][tt] = sum_i sum_k Wl[c][i][k] * A_i[tt + k]
  for (int idx = tid; idx < LOCF * TCH; idx += 256) {
    const int c = idx / TCH, tt = idx % TCH;
    float s = 0.f;
    const float* w0 = Wl + c * 2 * LOCK;
    for (int k = 0; k < LOCK; ++k) s = fmaf(w0[k], A0[tt + k], s);
    for (int k = 0; k < LOCK; ++k) s = fmaf(w0[LOCK + k], A1[tt + k], s);
    f[c][tt] = s;
  }
  __syncthreads();
  // 3. loc = W_dense . f ; e = v . tanh(pq + loc + penc) + b_v
  const int a = tid & 127, grp = tid >> 7;
  float wd[LOCF];
#pragma unroll
  for (int c = 0; c < LOCF; ++c) wd[c] = P.Wdense[a * LOCF + c];
  const float va = P.v[a], pqa = pq[a];
  for (int i = 0; i < TCH / 2; ++i) {
    const int tt = grp * (TCH / 2) + i;
    const int t = t0 + tt;
    float z = 0.f;
    if (t < T) {
      float l = 0.f;
#pragma unroll
      for (int c = 0; c < LOCF; ++c) l = fmaf(wd[c], f[c][tt], l);
      z = tanhf(pqa + l + P.penc[((long)b * D.T_max + t) * ADIM + a]) * va;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) z += __shfl_xor(z, off, 64);
    if (lane == 0) er[wave & 1][tt] = z;
  }
  __syncthreads();
  if (tid < TCH && t0 + tid < T) P.energy[(long)b * D.T_max + t0 + tid] = er[0][tid] + er[1][tid] + P.bv;
}

// --------------------------------------------------------------------------------------
// K3b: normalisation, alignment, alpha_cum and the context vector (slice of 128 dims)
// --------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_context_kernel(AttnArgs P, DecDev D, int jstep) {
  if (D.ctl->all_done) return;
  const int b = blockIdx.y, slice = blockIdx.x;
  if (D.done[b]) return;
  const int T = D.lens[b];
  const int t_step = dec_step(D, jstep);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  extern __shared__ __attribute__((aligned(16))) float al[];  // [T_max]
  __shared__ float wred[4];
  __shared__ float bc[2];
  const float* e = P.energy + (long)b * D.T_max;
  float mx = -INFINITY;
  if (P.softmax) {
    for (int t = tid; t < T; t += 256) mx = fmaxf(mx, e[t]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    if (lane == 0) wred[wave] = mx;
    __syncthreads();
    if (tid == 0) bc[0] = fmaxf(fmaxf(wred[0], wred[1]), fmaxf(wred[2], wred[3]));
    __syncthreads();
    mx = bc[0];
  }
  float s = 0.f;
  for (int t = tid; t < T; t += 256) {
    const float v = P.softmax ? expf(e[t] - mx) : 1.f / (1.f + expf(-e[t]));
    al[t] = v;
    s += v;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  __syncthreads();
  if (lane == 0) wred[wave] = s;
  __syncthreads();
  if (tid == 0) bc[1] = (wred[0] + wred[1]) + (wred[2] + wred[3]);
  __syncthreads();
  const float S = bc[1];
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
  const int d = tid & 127, h = tid >> 7;
  const float* enc = P.enc + (long)b * D.T_max * 512 + slice * 128 + d;
  float c = 0.f;
  for (int t = h; t < T; t += 2) c = fmaf(al[t], enc[(long)t * 512], c);
  __shared__ float cr[2][128];
  cr[h][d] = c;
  __syncthreads();
  if (tid < 128) P.ctx[(long)b * 512 + slice * 128 + tid] = cr[0][tid] + cr[1][tid];
}

__global__ void dec_advance_kernel(DecCtl* ctl, int n) {
  if (threadIdx.x == 0) ctl->base += n;
}

// --------------------------------------------------------------------------------------
// host launchers
// --------------------------------------------------------------------------------------
static size_t skinny_lds(int NT, int KS, int Bp, bool lstm) {
  return (size_t)NT * KS * Bp * 17 * 4 + (lstm ? (size_t)Bp * 4 * NT * 4 : 0);
}

void launch_skinny(const SkArgs& a, const DecDev& d, int jstep, int NT, int KS, hipStream_t s) {
  int nwg = a.job[0].ntiles / NT + (a.njobs > 1 ? a.job[1].ntiles / NT : 0);
  bool lstm = a.job[0].epi == EPI_LSTM || (a.njobs > 1 && a.job[1].epi == EPI_LSTM);
  const size_t lds = skinny_lds(NT, KS, a.MT * 16, lstm);
  if (NT == 1 && KS == 4) skinny_kernel<1, 4><<<nwg, 256, lds, s>>>(a, d, jstep);
  else if (NT == 1 && KS == 16) skinny_kernel<1, 16><<<nwg, 1024, lds, s>>>(a, d, jstep);
  else if (NT == 4 && KS == 4) skinny_kernel<4, 4><<<nwg, 1024, lds, s>>>(a, d, jstep);
  else TTS_CHECK(false, "skinny: unsupported tile config");
  HIP_OK(hipGetLastError());
}

void launch_prenet1_stop(const SkArgs& a, const DecDev& d, const StopArgs& st, int jstep, hipStream_t s) {
  const size_t lds = skinny_lds(1, 4, a.MT * 16, false);
  prenet1_stop_kernel<<<a.job[0].ntiles + 1, 256, lds, s>>>(a, d, st, jstep);
  HIP_OK(hipGetLastError());
}

void launch_attention(const AttnArgs& p, const DecDev& d, int jstep, hipStream_t s) {
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
