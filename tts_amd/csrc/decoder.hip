// Tacotron2 autoregressive decoder step kernels (gfx950).
//
// One reference decoder step (TTS/tts/layers/tacotron2.py:354-369 -> decode :259-298) becomes a
// chain of 5 stream-ordered launches, captured once into a hipGraph of CHUNK steps and
// replayed; the step index lives in device memory (DecCtl::base + j) so the same graph serves
// every chunk, and the reference's per-step host sync (`if stop_token > ...`, :362) becomes a
// device-side done flag per utterance plus an all_done word that turns every later kernel
// into an early exit.
//
//   K1   stop(t-1) from the projection kernel's partial dots + done flags
//        || prenet layers 1 and 2 (common_layers.py:76-82)
//   K2   attention_rnn LSTMCell (only the K=256 prenet part; the ctx/h part was precomputed
//        by K5 of the previous step) + partial query projection (common_layers.py:272)
//   K3   location-sensitive energies over T chunks (common_layers.py:268-278, 90-110), chunk
//        partial contexts, last-arriving chunk normalises (sigmoid/softmax), updates alpha_cum,
//        writes the alignment row and the context (common_layers.py:347-366)
//   K4   decoder_rnn LSTMCell (tacotron2.py:279-282)
//   K5   linear_projection (tacotron2.py:286-289) + frame store + stopnet partial dots (:291-295)
//        || next step's attention_rnn ctx/h part (+ biases)
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

#ifdef SK_TRACE_BUF
// phase timestamps (s_memrealtime, 100 MHz) per workgroup of skinny launches: bench tool only
__device__ unsigned long long sk_trace[1024 * 8];
#define SK_TRACE(k) \
  if (threadIdx.x == 0) sk_trace[(long)blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define SK_TRACE(k)
#endif

template <int MT, int D>
struct SkFrag {
  f32x4 w[D];
  f32x4 x[D][MT];
};

// Per-wave k-loop state. Segment bases, boundaries and strides are resolved once into
// registers: reading SkJob fields inside the loop made hipcc emit a dependent load plus
// `s_waitcnt vmcnt(0)` before every weight load, draining the pipeline.
//
// The k-loop is a rolling ring of D chunks: chunk i's MFMAs are followed by the load of chunk
// i + D into the same registers, so D chunks stay in flight at all times. At M = 32 the MFMAs of
// one chunk take ~256 cycles per wave and a loaded HBM round trip several microseconds; a
// two-group pipeline stalled once per group, the ring overlaps the weight stream with the MFMA
// stream (tools/skinny_bench.hip).
template <int MT, int NTHR = 256, int DD = 0>
struct SkPipe {
  // measured best at B = 32 (tools/skinny_bench.hip): deeper rings thrash the memory pipeline
  static constexpr int D = DD > 0 ? DD : NTHR >= 1024 ? 2 : 4;
  using Frag = SkFrag<MT, D>;
  const f32x4* Wv;
  const float* xb0;
  long d01, d12;  // element offsets xb1 - xb0, xb2 - xb1
  int ms0, dm01, dm12, e0, e1;
  int kc_lo, kc_hi;
  __device__ __forceinline__ void init(const SkJob& J, int tile, int w, int KS, int lane) {
    const int nkc = J.K / 16;
    kc_lo = (w * nkc) / KS;
    kc_hi = ((w + 1) * nkc) / KS;
    Wv = reinterpret_cast<const f32x4*>(J.W) + (long)tile * nkc * 64 + lane;
    // read every field by value first: selecting between member addresses forces the
    // kernarg struct into scratch
    const int ns = J.nseg;
    const float* p0 = J.seg[0].ptr;
    const float* p1 = J.seg[1].ptr;
    const float* p2 = J.seg[2].ptr;
    const int l0 = J.seg[0].ms, l1 = J.seg[1].ms, l2 = J.seg[2].ms;
    const int k0 = J.seg[0].K, k1 = J.seg[1].K;
    const int ms1 = ns > 1 ? l1 : l0;
    const int ms2 = ns > 2 ? l2 : ms1;
    ms0 = l0;
    dm01 = ms1 - ms0;
    dm12 = ms2 - ms1;
    e0 = k0 / 16;
    e1 = ns > 1 ? e0 + k1 / 16 : (1 << 30);
    if (ns < 2) e0 = 1 << 30;
    // fragment order: chunk kc of 16-row block mt at ptr + mt*ms + kc*256, lane's float4 at +4*lane
    xb0 = p0 + 4 * lane;
    const float* xb1 = (ns > 1 ? p1 : p0) + 4 * lane - (long)e0 * 256;
    const float* xb2 = (ns > 2 ? p2 : p0) + 4 * lane - (long)e1 * 256;
    d01 = xb1 - xb0;
    d12 = xb2 - xb1;
  }
  // load chunk kc into ring slot u (index clamped to the last chunk: always a valid address;
  // the ring's tail re-reads that chunk from cache instead of branching around the loads)
  __device__ __forceinline__ void load1(Frag& F, int u, int kc_in) {
    const int kc = min(kc_in, kc_hi - 1);
    F.w[u] = Wv[(long)kc * 64];
    // segment select as conditional adds of deltas (a 3-way pointer select became a
    // scratch lookup table)
    const long d = (kc >= e0 ? d01 : 0l) + (kc >= e1 ? d12 : 0l);
    const float* xp = xb0 + d + (long)kc * 256;
    const int ms = ms0 + (kc >= e0 ? dm01 : 0) + (kc >= e1 ? dm12 : 0);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) F.x[u][mt] = *reinterpret_cast<const f32x4*>(xp + (long)mt * ms);
  }
  __device__ __forceinline__ void mma1(const Frag& F, int u, f32x4 (&acc)[MT]) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = MFMA16(F.x[u][mt][s], F.w[u][s], acc[mt]);
  }
  // the ring's first D loads: issue before anything that waits on memory
  __device__ __forceinline__ void prefetch(Frag& F) {
#pragma unroll
    for (int u = 0; u < D; ++u) load1(F, u, kc_lo + u);
  }
  __device__ __forceinline__ void run(Frag& F, f32x4 (&acc)[MT]) {
    for (int kc0 = kc_lo; kc0 < kc_hi; kc0 += D) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        if (kc0 + u < kc_hi) mma1(F, u, acc);  // wave-uniform
        load1(F, u, kc0 + D + u);
      }
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

// --------------------------------------------------------------------------------------
// generic skinny kernel: NT tiles per workgroup, KS waves per tile, MT batch tiles of 16
// --------------------------------------------------------------------------------------
// body of one workgroup for job J (always called with a constant job index so J's fields stay
// scalar loads from the kernarg segment; a runtime-selected reference made hipcc copy the whole
// argument struct to scratch)
template <int NT, int KS, int MT, int DD = 0>
__device__ __forceinline__ void skinny_body(const SkJob& J, const DecDev& D, int jstep, int wg, float* smem) {
  constexpr int Bp = MT * 16;
  constexpr int nthr = NT * KS * 64;
  constexpr int SITEMS = (NT * Bp * 16 + nthr - 1) / nthr;  // store items per thread
  constexpr int LITEMS = (NT * Bp * 4 + nthr - 1) / nthr;   // LSTM (utterance, unit) items per thread
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int grp = wave / KS, w = wave % KS;
  const int all_done = D.ctl->all_done;
  const int tile = wg * NT + grp;
  SkPipe<MT, nthr, DD> pipe;
  typename SkPipe<MT, nthr, DD>::Frag fa;
  pipe.init(J, tile, w, KS, lane);
  SK_TRACE(0);
  pipe.prefetch(fa);
  // epilogue operands, fetched under the GEMM (indices clamped: no guarded loads); a 1024-thread
  // workgroup at MT = 4 is out of registers for that and fetches them after the k-loop
  constexpr bool EPRE = !(nthr >= 1024 && MT >= 4);
  float eb[SITEMS];
  float lb[LITEMS][4], la[LITEMS][4], lc[LITEMS];
  auto load_epi = [&]() {
    if (J.epi == EPI_STORE) {
#pragma unroll
      for (int i = 0; i < SITEMS; ++i) {
        const int idx = min(tid + i * nthr, NT * Bp * 16 - 1);
        const int g = idx / (Bp * 16), n = idx % 16;
        eb[i] = J.bias ? J.bias[(wg * NT + g) * 16 + n] : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < LITEMS; ++i) {
        const int idx = min(tid + i * nthr, NT * Bp * 4 - 1);
        const int g = idx / (Bp * 4), rem = idx % (Bp * 4);
        const int m = rem / 4, u = rem % 4;
        const int tl = wg * NT + g;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int col = tl * 16 + q * 4 + u;
          lb[i][q] = J.bias ? J.bias[col] : 0.f;
          la[i][q] = J.addin ? J.addin[(long)m * J.addin_ld + col] : 0.f;
        }
        lc[i] = J.c_state[(long)m * J.hc_ld + tl * 4 + u];
      }
    }
  };
  if (EPRE) load_epi();
  // query-projection weights of this workgroup's 4*NT units for attention dim tid % 128
  float wqv[4 * NT];
  auto load_wq = [&]() {
    if (J.pq_part) {
      const float* wq = J.WqT + (long)(wg * NT * 4) * 128 + tid % 128;
#pragma unroll
      for (int u = 0; u < 4 * NT; ++u) wqv[u] = wq[(long)u * 128];
    }
  };
  if (EPRE) load_wq();
  SK_TRACE(1);
  if (all_done) return;
  const int t = D.ctl->base + jstep;

  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  pipe.run(fa, acc);
  SK_TRACE(2);
  if (!EPRE) {
    load_epi();
    load_wq();
  }
  float* part = smem + (long)grp * KS * Bp * 17;
  float* extra = smem + (long)NT * KS * Bp * 17;  // [NT][Bp][16]
  skinny_to_lds<MT>(part, w, lane, acc);
  __syncthreads();
  SK_TRACE(3);

  if (J.epi == EPI_STORE) {
#pragma unroll
    for (int i = 0; i < SITEMS; ++i) {
      const int idx = tid + i * nthr;
      if (idx >= NT * Bp * 16) break;
      const int g = idx / (Bp * 16), rem = idx % (Bp * 16);
      const int m = rem / 16, n = rem % 16;
      int col = (wg * NT + g) * 16 + n;
      float v = skinny_sum<KS, Bp>(smem + (long)g * KS * Bp * 17, m, n) + eb[i];
      if (J.act == 1) v = fmaxf(v, 0.f);
      if (J.lead_stop) {
        if (col < 16) {
          if (n == 0) J.stop_part[m] = v;
          continue;
        }
        col -= 16;
      }
      J.out[J.out_frag ? frag_idx(m, col, J.out_ld) : (long)m * J.out_ld + col] = v;
      if (J.frames_r > 0 && m < D.B && col < 80 * J.frames_r && t < D.S_cap && !D.done[m])
        D.dec_out[((long)m * D.S_cap + t) * J.frames_r * 80 + col] = v;
    }
  } else {  // EPI_LSTM: tile rows are gate-major [i0..i3 f0..f3 g0..g3 o0..o3] of 4 units
    float* hs = extra;  // [Bp][4*NT]
#pragma unroll
    for (int i = 0; i < LITEMS; ++i) {
      const int idx = tid + i * nthr;
      if (idx >= NT * Bp * 4) break;
      const int g = idx / (Bp * 4), rem = idx % (Bp * 4);
      const int m = rem / 4, u = rem % 4;
      const int tl = wg * NT + g;
      const float* pg = smem + (long)g * KS * Bp * 17;
      float pre[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) pre[q] = skinny_sum<KS, Bp>(pg, m, q * 4 + u) + lb[i][q] + la[i][q];
      const long ci = (long)m * J.hc_ld + tl * 4 + u;
      const float ig = 1.f / (1.f + expf(-pre[0]));
      const float fg = 1.f / (1.f + expf(-pre[1]));
      const float gg = tanhf(pre[2]);
      const float og = 1.f / (1.f + expf(-pre[3]));
      const float c = fg * lc[i] + ig * gg;
      const float h = og * tanhf(c);
      J.c_state[ci] = c;
      J.h_out[frag_idx(m, tl * 4 + u, J.hc_ld)] = h;
      hs[m * 4 * NT + g * 4 + u] = h;
    }
    SK_TRACE(4);
    if (J.pq_part) {  // partial query projection over this workgroup's 4*NT hidden units
      static_assert(nthr % 128 == 0, "pq: one attention dim per thread");
      const int a = tid % 128;
      __syncthreads();
      for (int m = tid / 128; m < Bp; m += nthr / 128) {
        float s = 0.f;
#pragma unroll
        for (int u = 0; u < 4 * NT; ++u) s = fmaf(wqv[u], hs[m * 4 * NT + u], s);
        J.pq_part[((long)wg * Bp + m) * 128 + a] = s;
      }
    }
  }
  SK_TRACE(5);
}

// grid = job0 tiles/NT  [+ job1 tiles/NT]
template <int NT, int KS, int MT, int DD = 0>
__global__ __launch_bounds__(NT * KS * 64) void skinny_kernel(SkArgs A, DecDev D, int jstep) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int n0 = A.job[0].ntiles / NT;
  const int n1 = A.njobs > 1 ? A.job[1].ntiles / NT : 0;
  const int bx = blockIdx.x;
  if (bx < n0) {
    skinny_body<NT, KS, MT, DD>(A.job[0], D, jstep, bx, smem);
  } else if (bx < n0 + n1) {
    skinny_body<NT, KS, MT, DD>(A.job[1], D, jstep, bx - n0, smem);
  }
}

// --------------------------------------------------------------------------------------
// K1: prenet (both layers) || stop decision for step t-1.
//   Workgroups 0..15: each recomputes prenet layer 1 for all utterances (16 waves, one 16-wide
//   tile each, K = 80) into LDS, then its own 16 columns of layer 2 (K = 256 split over the 16
//   waves, operand from LDS). Recomputing layer 1 (0.65 M MAC) per workgroup is cheaper than the
//   launch boundary it removes.
//   Workgroup 16: stop logit from the projection launch's stopnet tile; sigma;
//   reference stop rule (tacotron2.py:357-366): stop iff sigma > thr and t > 0, else stop when
//   max_decoder_steps outputs exist.
// --------------------------------------------------------------------------------------
constexpr int P1LD = 260;  // LDS row stride of the layer-1 activations (bank-conflict padding)

template <int MT>
__global__ __launch_bounds__(1024) void prenet_stop_kernel(SkArgs A, DecDev D, StopArgs S, int jstep) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int Bp = MT * 16;
  if (blockIdx.x == 16) {
    __shared__ int dflag[64];
    const int m = min(tid, Bp - 1);
    const float pv = S.part[m];
    const int dn0 = D.done[m];
    const int mx = D.max_steps[m];
    const int all_done = D.ctl->all_done;
    const int t = D.ctl->base + jstep;
    if (all_done) return;
    if (tid < D.B) {
      int dn = dn0;
      if (t >= 1 && !dn) {
        const float logit = pv;
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
      int last = -1;
      for (int k = 0; k < D.B; ++k)
        if (!dflag[k]) last = k;
      D.ctl->all_done = last < 0;
      D.ctl->active_tiles = last / 16 + 1;
    }
    return;
  }
  const SkJob& J1 = A.job[0];  // layer 1: 16 tiles, K = 80, X = y[:, 80(r-1):80r]
  const SkJob& J2 = A.job[1];  // layer 2: tile blockIdx.x, K = 256, X from LDS
  float* P1 = smem;                           // [Bp][P1LD]
  float* part = smem + Bp * P1LD;             // [16][Bp][17]
  const int n2 = blockIdx.x;
  // layer-2 weight fragment of this wave (one k-chunk per wave) and layer-1 pipeline, issued first
  const f32x4 w2 = reinterpret_cast<const f32x4*>(J2.W)[((long)n2 * 16 + wave) * 64 + lane];
  SkPipe<MT, 1024> pipe;
  typename SkPipe<MT, 1024>::Frag fa;
  pipe.init(J1, wave, 0, 1, lane);
  pipe.prefetch(fa);
  if (D.ctl->all_done) return;
  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  pipe.run(fa, acc);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      P1[(mt * 16 + 4 * (lane >> 4) + j) * P1LD + wave * 16 + (lane & 15)] = fmaxf(acc[mt][j], 0.f);
  __syncthreads();
  // layer 2, k-chunk `wave`
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    const int row = lane & 15, kl = 4 * (lane >> 4);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const f32x4 xv = *reinterpret_cast<const f32x4*>(P1 + (mt * 16 + row) * P1LD + wave * 16 + kl);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[mt] = MFMA16(xv[s], w2[s], acc[mt]);
    }
  }
  skinny_to_lds<MT>(part, wave, lane, acc);
  __syncthreads();
  for (int idx = tid; idx < Bp * 16; idx += 1024) {
    const int m = idx / 16, n = idx % 16;
    const float v = skinny_sum<16, Bp>(part, m, n);
    J2.out[frag_idx(m, n2 * 16 + n, J2.out_ld)] = fmaxf(v, 0.f);
  }
}

// --------------------------------------------------------------------------------------
// K3: location-sensitive attention in one launch.
//   Workgroup (chunk of TCH encoder positions, utterance): energies e_t (common_layers.py:268-278,
//   90-110), then chunk-local sigmoid(e) / exp(e - m_chunk), the chunk sum and the chunk's
//   unnormalised context sum_t s_t enc_t. The last workgroup of the utterance to arrive
//   (agent-scope release/acquire counter, cdna_hip_programming.md §6 Guideline 16 split-K recipe)
//   combines: S = sum of chunk sums, ctx = sum U_c / S, alpha_t = s_t / S, alpha_cum += alpha,
//   alignment row (common_layers.py:347-366).
// --------------------------------------------------------------------------------------
constexpr int TCH = 16;
constexpr int LOCK = 31, LOCF = 32, ADIM = 128, NPQ = 128;

#ifdef ATTN_TRACE_BUF
// phase timestamps (s_memrealtime, 100 MHz) of every workgroup, tools/skinny_bench.hip only
__device__ unsigned long long attn_trace[64 * 64 * 9];
#define ATTN_TRACE(k) \
  if (threadIdx.x == 0) attn_trace[((long)b * P.nchmax + ch) * 9 + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define ATTN_TRACE(k)
#endif

// one workgroup of NT threads (256 or 512): utterance b, positions [TC ch, TC ch + TC)
template <int NT, int TC>
__device__ __forceinline__ void attn_body(const AttnArgs& P, const DecDev& D, int jstep, int b, int ch) {
  constexpr int NG = NT / ADIM;           // thread groups over the attention dims
  constexpr int PPG = TC / NG;           // positions per group in the energy phase
  constexpr int DPT = 512 / NT;           // encoder dims per thread (context)
  constexpr int OPT = (LOCF * TC) / NT;  // location-conv outputs per thread
  constexpr int LPP = NT / TC;           // lanes per position in the energy reduction
  constexpr int NWL = (LOCF * 2 * LOCK + NT - 1) / NT;
  static_assert(NG >= 2 && OPT >= 1 && OPT <= 2 && LPP <= 64, "attention geometry");
  ATTN_TRACE(0);
  const int t0 = ch * TC;
  const int tid = threadIdx.x;
  const int a = tid % ADIM, grp = tid / ADIM;
  __shared__ float red[NG][ADIM];
  __shared__ float A0[TC + LOCK], A1[TC + LOCK];
  __shared__ float Wl[LOCF * 2 * LOCK];
  __shared__ __attribute__((aligned(16))) float f[TC][LOCF + 4];  // [position][filter]
  __shared__ float zb[TC][ADIM + 4];
  __shared__ float sv[TC];
  __shared__ int is_last;
  const int Bp = P.Bp;
  const int T = D.lens[b];
  const int Tm1 = max(T - 1, 0);
  // -- every independent global load up front (clamped indices, no guarded loads) --
  float pen[PPG];
#pragma unroll
  for (int i = 0; i < PPG; ++i) {
    const int t = min(t0 + grp * PPG + i, Tm1);
    pen[i] = P.penc[((long)b * D.T_max + t) * ADIM + a];
  }
  float wd[LOCF];
#pragma unroll
  for (int c = 0; c < LOCF; ++c) wd[c] = P.WdT[c * ADIM + a];
  const float va = P.v[a];
  float pp[NPQ / NG];
#pragma unroll
  for (int i = 0; i < NPQ / NG; ++i) pp[i] = P.pq_part[((long)(grp * (NPQ / NG) + i) * Bp + b) * ADIM + a];
  float a0, a1;
  {
    const int pos = t0 - (LOCK - 1) / 2 + min(tid, TC + LOCK - 2);
    const int pc = min(max(pos, 0), Tm1);
    a0 = P.alpha[(long)b * D.T_max + pc];
    a1 = P.alpha_cum[(long)b * D.T_max + pc];
    if (pos < 0 || pos >= T) a0 = a1 = 0.f;
  }
  float wl[NWL];
#pragma unroll
  for (int i = 0; i < NWL; ++i) wl[i] = P.Wloc[min(tid + NT * i, LOCF * 2 * LOCK - 1)];
  // encoder rows of this chunk for the partial context: dims DPT*tid .. DPT*tid + DPT-1
  float ev[TC][DPT];
#pragma unroll
  for (int i = 0; i < TC; ++i) {
    const float* er = P.enc + ((long)b * D.T_max + min(t0 + i, Tm1)) * 512 + DPT * tid;
    if constexpr (DPT == 2) {
      const float2 v2 = *reinterpret_cast<const float2*>(er);
      ev[i][0] = v2.x;
      ev[i][1] = v2.y;
    } else {
      ev[i][0] = er[0];
    }
  }
  if (D.ctl->all_done || D.done[b] || t0 >= T) return;
  const int t_step = D.ctl->base + jstep;
  if (tid < TC + LOCK - 1) {
    A0[tid] = a0;
    A1[tid] = a1;
  }
#pragma unroll
  for (int i = 0; i < NWL; ++i)
    if (tid + NT * i < LOCF * 2 * LOCK) Wl[tid + NT * i] = wl[i];
  // query projection = sum of the attention-LSTM kernel's partials (fixed order)
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPQ / NG; ++i) s += pp[i];
  red[grp][a] = s;
  __syncthreads();
  ATTN_TRACE(1);
  float pqa = red[0][a];
#pragma unroll
  for (int g = 1; g < NG; ++g) pqa += red[g][a];
  // location conv: f[tt][c] = sum_i sum_k Wl[c][i][k] * A_i[tt + k]; OPT adjacent positions of
  // one filter per thread, the window sliding in registers (one A read per tap)
  {
    const int c = tid / (TC / OPT), tt = (tid % (TC / OPT)) * OPT;
    const float* w0 = Wl + c * 2 * LOCK;
    float acc[OPT];
#pragma unroll
    for (int o = 0; o < OPT; ++o) acc[o] = 0.f;
#pragma unroll
    for (int ci = 0; ci < 2; ++ci) {
      const float* Ai = ci ? A1 : A0;
      float win[OPT];
#pragma unroll
      for (int o = 0; o < OPT; ++o) win[o] = Ai[tt + o];
#pragma unroll
      for (int k = 0; k < LOCK; ++k) {
        const float w = w0[ci * LOCK + k];
#pragma unroll
        for (int o = 0; o < OPT; ++o) acc[o] = fmaf(w, win[o], acc[o]);
#pragma unroll
        for (int o = 0; o + 1 < OPT; ++o) win[o] = win[o + 1];
        win[OPT - 1] = Ai[tt + k + OPT];
      }
    }
#pragma unroll
    for (int o = 0; o < OPT; ++o) f[tt + o][c] = acc[o];
  }
  __syncthreads();
  ATTN_TRACE(2);
  // loc = W_dense . f ; e = v . tanh(pq + loc + penc) + b_v. Each thread owns one attention dim
  // for PPG positions; the sum over dims goes through LDS (position-major, LPP lanes per
  // position) instead of serial 64-lane shuffle reductions
#pragma unroll
  for (int i = 0; i < PPG; ++i) {
    const int tt = grp * PPG + i;
    float l = 0.f;
#pragma unroll
    for (int c4 = 0; c4 < LOCF / 4; ++c4) {
      const f32x4 fv = *reinterpret_cast<const f32x4*>(&f[tt][c4 * 4]);
#pragma unroll
      for (int q = 0; q < 4; ++q) l = fmaf(wd[c4 * 4 + q], fv[q], l);
    }
    zb[tt][a] = tanhf(pqa + l + pen[i]) * va;
  }
  __syncthreads();
  ATTN_TRACE(3);
  const int nvalid = min(TC, T - t0);
  const long pidx = (long)b * P.nchmax + ch;
  {
    const int pos = tid / LPP, j = tid % LPP;
    float z = 0.f;
#pragma unroll
    for (int q = 0; q < ADIM / LPP; ++q) z += zb[pos][j * (ADIM / LPP) + q];
#pragma unroll
    for (int off = LPP / 2; off > 0; off >>= 1) z += __shfl_xor(z, off, 64);
    if (j == 0) {
      const float e = z + P.bv;
      if (pos < nvalid)
        __hip_atomic_store(P.energy + (long)b * D.T_max + t0 + pos, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sv[pos] = e;
    }
  }
  __syncthreads();
  ATTN_TRACE(4);
  // chunk-local normalisation terms
  float m_c = -INFINITY;
  if (P.softmax)
    for (int i = 0; i < nvalid; ++i) m_c = fmaxf(m_c, sv[i]);
  float sl[TC];
  float S_c = 0.f;
#pragma unroll
  for (int i = 0; i < TC; ++i) {
    const float e = sv[i];
    const float x = P.softmax ? expf(e - m_c) : 1.f / (1.f + expf(-e));
    sl[i] = i < nvalid ? x : 0.f;
    S_c += sl[i];
  }
  // unnormalised partial context of this chunk
  float u[DPT];
#pragma unroll
  for (int q = 0; q < DPT; ++q) {
    u[q] = 0.f;
#pragma unroll
    for (int i = 0; i < TC; ++i) u[q] = fmaf(sl[i], ev[i][q], u[q]);
  }
  // ---- publish: sc1 (write-through) stores need no release fence (cdna_hip_programming.md
  // §5 split-K item 2); every wave drains, barrier, then one relaxed agent-scope ticket ----
  if constexpr (DPT == 2) {
    union {
      float2 f;
      unsigned long long u;
    } pk;
    pk.f = make_float2(u[0], u[1]);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(P.part_u + pidx * 512) + tid, pk.u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else {
    __hip_atomic_store(P.part_u + pidx * 512 + tid, u[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid == 0) {
    __hip_atomic_store(P.part_s + pidx, S_c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(P.part_m + pidx, m_c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ATTN_TRACE(5);
  const int nch = (T + TC - 1) / TC;
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add(&P.counter[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = (prev == (unsigned)(nch - 1));
    if (is_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  ATTN_TRACE(6);
  if (!is_last) return;
  // ---- combine (one workgroup per utterance): chunk partials in batches of CB, all loads of a
  // batch in flight together (clamped), online rescaling for softmax ----
  const long pb = (long)b * P.nchmax;
  constexpr int CB = 16;
  float m = -INFINITY, S = 0.f;
  float cx[DPT];
#pragma unroll
  for (int q = 0; q < DPT; ++q) cx[q] = 0.f;
  for (int cb = 0; cb < nch; cb += CB) {
    float pm[CB], ps[CB], pu[CB][DPT];
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const long c = pb + min(cb + i, nch - 1);
      pm[i] = P.part_m[c];
      ps[i] = P.part_s[c];
      if constexpr (DPT == 2) {
        const float2 v2 = *reinterpret_cast<const float2*>(P.part_u + c * 512 + 2 * tid);
        pu[i][0] = v2.x;
        pu[i][1] = v2.y;
      } else {
        pu[i][0] = P.part_u[c * 512 + tid];
      }
    }
    float wc[CB];
    if (P.softmax) {
      float mb = m;
#pragma unroll
      for (int i = 0; i < CB; ++i)
        if (cb + i < nch) mb = fmaxf(mb, pm[i]);
      const float sc = (m == -INFINITY) ? 0.f : expf(m - mb);
      S *= sc;
#pragma unroll
      for (int q = 0; q < DPT; ++q) cx[q] *= sc;
      m = mb;
#pragma unroll
      for (int i = 0; i < CB; ++i) wc[i] = (cb + i < nch) ? expf(pm[i] - m) : 0.f;
    } else {
#pragma unroll
      for (int i = 0; i < CB; ++i) wc[i] = (cb + i < nch) ? 1.f : 0.f;
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      S = fmaf(ps[i], wc[i], S);
#pragma unroll
      for (int q = 0; q < DPT; ++q) cx[q] = fmaf(pu[i][q], wc[i], cx[q]);
    }
  }
  ATTN_TRACE(7);
#pragma unroll
  for (int q = 0; q < DPT; ++q) P.ctx[frag_idx(b, DPT * tid + q, 512)] = cx[q] / S;
  const float* en = P.energy + (long)b * D.T_max;
  for (int t = tid; t < T; t += NT) {
    const float e = en[t];
    const float al = (P.softmax ? expf(e - m) : 1.f / (1.f + expf(-e))) / S;
    P.alpha[(long)b * D.T_max + t] = al;
    P.alpha_cum[(long)b * D.T_max + t] += al;
    if (t_step < D.S_cap) D.align_out[((long)b * D.S_cap + t_step) * D.T_max + t] = al;
  }
  if (tid == 0) P.counter[b] = 0u;  // next step (ordered by the kernel boundary)
  ATTN_TRACE(8);
}

template <int NT, int TC>
__global__ __launch_bounds__(NT) void attn_kernel(AttnArgs P, DecDev D, int jstep) {
  attn_body<NT, TC>(P, D, jstep, blockIdx.y, blockIdx.x);
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
    TTS_CHECK(!a.job[j].pq_part || a.job[j].ntiles / NT <= a.job[j].pq_cap, "skinny: query partial buffer too small");
  }
  int nwg = a.job[0].ntiles / NT + (a.njobs > 1 ? a.job[1].ntiles / NT : 0);
  if (NT == 1 && KS == 4) launch_skinny_nt<1, 4>(a, d, jstep, nwg, s);
  else if (NT == 1 && KS == 8) launch_skinny_nt<1, 8>(a, d, jstep, nwg, s);
  else if (NT == 1 && KS == 16) launch_skinny_nt<1, 16>(a, d, jstep, nwg, s);
  else if (NT == 2 && KS == 4) launch_skinny_nt<2, 4>(a, d, jstep, nwg, s);
  else TTS_CHECK(false, "skinny: unsupported tile config");
  HIP_OK(hipGetLastError());
}

void launch_prenet_stop(const SkArgs& a, const DecDev& d, const StopArgs& st, int jstep, hipStream_t s) {
  TTS_CHECK(a.MT >= 1 && a.MT <= 4, "prenet: MT in [1,4]");
  TTS_CHECK(a.njobs == 2 && a.job[0].ntiles == 16 && a.job[1].ntiles == 16 && a.job[1].K == 256,
            "prenet: expects 256-wide layers");
  const int Bp = a.MT * 16;
  const size_t lds = ((size_t)Bp * P1LD + (size_t)16 * Bp * 17) * 4;
  switch (a.MT) {
    case 1: prenet_stop_kernel<1><<<17, 1024, lds, s>>>(a, d, st, jstep); break;
    case 2: prenet_stop_kernel<2><<<17, 1024, lds, s>>>(a, d, st, jstep); break;
    case 3: prenet_stop_kernel<3><<<17, 1024, lds, s>>>(a, d, st, jstep); break;
    default: prenet_stop_kernel<4><<<17, 1024, lds, s>>>(a, d, st, jstep); break;
  }
  HIP_OK(hipGetLastError());
}

void launch_attention(const AttnArgs& p, const DecDev& d, int jstep, hipStream_t s) {
  TTS_CHECK(p.npq == NPQ, "attention: expects 128 query partials");
  TTS_CHECK(p.nchmax * TCH >= d.T_max, "attention: partial buffers too small");
  dim3 g((d.T_max + TCH - 1) / TCH, d.B);
  // 512-thread workgroups shorten the chain when few chunks run; past ~200 workgroups the
  // 256-thread form is faster (tools/skinny_bench.hip, B = 32: T 64 11.7 vs 12.3 us, T 168 15.8 vs 14.9)
  if ((long)g.x * g.y <= 200)
    attn_kernel<512, TCH><<<g, 512, 0, s>>>(p, d, jstep);
  else
    attn_kernel<256, TCH><<<g, 256, 0, s>>>(p, d, jstep);
  HIP_OK(hipGetLastError());
}

void launch_dec_advance(DecCtl* ctl, int n, hipStream_t s) {
  dec_advance_kernel<<<1, 64, 0, s>>>(ctl, n);
  HIP_OK(hipGetLastError());
}
