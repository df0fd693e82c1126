// Persistent Tacotron2 decoder (gfx950): the autoregressive loop as ONE cooperative launch per
// batch-tile count, 256 workgroups (one per CU) x 8 waves, phases separated by a grid barrier.
//
// Why: with the 5-launch graph (decoder.hip) every step re-streams ~72 MB of LSTM / projection
// weights from MALL/HBM (the decoder_rnn launch alone is ~10 us of a 54 us step). Here the weights
// stay on chip for the whole decode:
//   decoder_rnn   [W_ih | W_hh] (41.9 MB)  VGPRs: workgroup g owns gate tile g, 20 k-chunks per wave
//   attention_rnn ctx/h part   (25.2 MB)   LDS:   96 KB per workgroup (tile g)
// and a hierarchical grid barrier (16 first-level counters, then 16 arrivals on a global counter,
// one go word; tools/persist_bench.hip: 1.8-2.1 us) replaces each launch boundary (1.7 us + cold
// start).
//
// One decoder step t (TTS/tts/layers/tacotron2.py:354-369 -> decode :259-298), 5 phases:
//   P1  stop decision for t-1 (workgroup 255; tacotron2.py:357-366)
//       || prenet layer 2 (workgroups 0-15). Layer 1 was folded into the previous projection:
//       the prenet reads the LAST frame y[:, 80(r-1):80r] of the projection, and layer 1 has no
//       bias, so relu(W1 y) = relu(W1 W_p,last [h|ctx] + W1 b_p,last): 16 extra projection tiles
//   P3  attention_rnn LSTMCell prenet part (K = 256) + cell + partial query projections
//       (workgroups 0-127, 8 units each) || frames of step t-1 to dec_out (workgroups 128-255)
//   P4  location-sensitive attention, work item = (utterance, 32 positions); the last arriving
//       item of an utterance combines (same protocol as decoder.hip K3)
//   P5  decoder_rnn LSTMCell (tile g, K = 2560, weights in VGPRs)
//   P6  next step's attention_rnn ctx/h part (tile g, weights in LDS)
//       || projection + stop tile + folded prenet layer 1, K split in 2 halves (workgroups
//       0 .. 2*ntj-1); consumers add the two halves and the bias
//
// Memory model: cross-workgroup data is written with agent-scope relaxed atomic stores (sc1:
// write-through past the non-coherent per-XCD L2) and read with agent-scope loads (sc1), every
// wave drains its stores (vmcnt(0)) before the barrier arrival; no L2 invalidation is needed.
// Barrier waits give up after TTS_BARRIER_TIMEOUT_MS (default 2 s; error word set, every
// workgroup exits): a launch that was not fully co-resident fails loudly instead of hanging.
#include "common.h"
#include "decoder.h"
#include "gsync.h"
#include "split16.h"

#include <algorithm>
#include <cstdio>
#include <type_traits>
#include <vector>

namespace {
constexpr int PW = 256, PT = 512, NWV = 8;
// the step's grid barriers: gsync.h's flag barrier (one store per arrival, workgroup 0 releases);
// -DTTS_BAR_COUNTERS builds the counter form for A/B
#ifdef TTS_BAR_COUNTERS
#define BAR_ARRIVE gsync_arrive
#define BAR_WAIT gsync_wait
#else
static_assert(PW <= 256, "gflag barrier: one flag word per workgroup, 256 at most");
#define BAR_ARRIVE gflag_arrive
#define BAR_WAIT gflag_wait
#endif
constexpr int DEC_NC = 20;   // 160 k-chunks / 8 waves
constexpr int ATTP_NC = 8;   // 4 tiles x 16 chunks / 8 waves
constexpr int PJ_NC = 6;     // 48 / 8
constexpr int NATT = 64;           // attention_rnn workgroups (P3): 4 gate tiles = 16 units each
constexpr int PJ_WG0 = 0;          // first projection workgroup (P6); jobs sit on the attention_rnn
                                   // workgroups, which have no attention item
constexpr int PTC = 32;      // attention positions per work item
constexpr int IW0 = NATT;    // attention items live on workgroups IW0 .. PW-1 (round-robin)
constexpr int YROWS = 64;    // rows per projection half (independent of the batch tile: the MT = 1
                             // launch reads what the MT = 2 launch left)
// encoder rows (of 8 per thread) an attention item keeps in registers across steps: 4 where the
// kernel stays within 256 VGPRs without spills (split-f16 variants without forward attention), 0
// elsewhere (and for 48 / 64-row batch tiles, whose accumulators need the registers); pec_arr
// sizes the (unused) array of the latter
constexpr int pec_of(int VAR, int MT) { return ((VAR & 8) && !(VAR & 2) && MT <= 2) ? 4 : 0; }
constexpr int pec_arr(int VAR, int MT) { return pec_of(VAR, MT) > 0 ? pec_of(VAR, MT) : 1; }
// pre-split hand-offs (VAR 8: location attention, every decoder GEMM on the split-f16 MFMA): h_att,
// ctx and h_dec are published as their f16 hi / lo halves, [hi 0..3 | lo 0..3] in the 16 bytes a
// fragment quad takes in fp32, so the streaming consumers feed the loads to the MFMA without
// splitting (the split is done once, by the producer; tools/payload_bench.hip mode 3: 0.42 us less
// per streamed 192 KB block). The variants with fp32 readers of these buffers keep fp32.
#ifdef TTS_NO_PRESPLIT
constexpr bool presplit_of(int) { return false; }
#else
constexpr bool presplit_of(int VAR) { return VAR == 8; }
#endif
template <bool PS>
__device__ __forceinline__ void stc_quad_h(float* base, int e, float v) {
  if constexpr (PS) stc_quad_x3(base, e, v);
  else stc_quad(base, e, v);
}
constexpr int LOCK_ = 31, ADIM_ = 128, NPQ_ = NATT;  // NPQ_: query-projection partials
// LDS layouts chosen for bank-conflict-free access (64 banks x 4 B; ds_read_b32 / ds_write_b32 bank
// = dword index mod 32 within a 32-lane group, ds_read_b128 = mod 64 within a 16-lane group):
// * RS: row stride of the wave-partial reduction scratch [wave][row][RS]. Writers put row
//   4 (lane >> 4) + j, column lane & 15 (rows r and r + 4 in one 32-lane group: 20 * 4 = 80 = 16 mod
//   32, disjoint halves); the LSTM cells read row tid >> 2 (8 rows per group), column 4 q + (tid & 3):
//   20 m mod 32 = {0, 20, 8, 28, 16, 4, 24, 12} + 0..3, disjoint. Stride 17 gave 2-way conflicts on
//   the cell reads.
// * WCLD: row stride of the folded location filter Wcomb [64 taps][WCLD]: lanes 0-15 read tap j,
//   lanes 16-31 tap j + 1 of the same 16 dims; WCLD = 16 mod 32 puts them on disjoint banks (128
//   put both halves on the same 16 banks: 2-way).
// * split-f16 weight / operand fragments in LDS as [k-step][hi 64 lanes | lo 64 lanes] planes: a
//   lane's 16-byte read is contiguous with its neighbours' (the interleaved [lane][hi | lo] form
//   strides lanes 32 B apart: 2-way on every ds_read_b128 / ds_write_b128).
#ifndef TTS_RS
#define TTS_RS 20
#endif
#ifndef TTS_WCLD
#define TTS_WCLD 144
#endif
#ifndef TTS_X3_PLANES
#define TTS_X3_PLANES 1
#endif
constexpr int RS = TTS_RS, WCLD = TTS_WCLD;
// LDS index (in 16-byte units) of the hi (h = 0) / lo (h = 1) half of lane `lane`'s split fragment of k-step ks
__device__ __forceinline__ int x3i(int ks, int lane, int h) {
  return TTS_X3_PLANES ? (ks * 128 + h * 64 + lane) : ((ks * 64 + lane) * 2 + h);
}
}  // namespace

// Opaque copies of lane / wave indices, taken at the start of each phase: without them the
// compiler hoists every loop-invariant address of every phase out of the step loop and keeps them
// all live (hundreds of VGPRs / SGPRs, spilled to scratch).
__device__ __forceinline__ int opaque_v(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ int opaque_s(int v) {
  asm volatile("" : "+s"(v));
  return v;
}
constexpr int ACT_AUX = 16;  // sc1; measured: plain / sc0 / sc0|sc1 loads are no faster

// partial sums of one wave's MT accumulators into LDS [wave][m][RS]
template <int MT>
__device__ __forceinline__ void acc_to_lds(float* part, int w, int lane, const f32x4 (&acc)[MT]) {
  constexpr int Bp = MT * 16;
  float* p = part + w * Bp * RS;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) p[(mt * 16 + 4 * (lane >> 4) + j) * RS + (lane & 15)] = acc[mt][j];
}
// chunk c (m-tiles CM c .. CM c + CM - 1) of a wave's MT accumulators into LDS [wave][CM * 16][RS]:
// reductions over the waves go in chunks of at most 2 m-tiles (32 rows, the scratch's size), so
// MT = 3, 4 (48 / 64 rows) reuse the MT = 2 scratch; rows past MT stay stale and are not read
template <int MT, int CM>
__device__ __forceinline__ void acc_chunk_to_lds(float* part, int w, int lane, const f32x4 (&acc)[MT], int c) {
  float* p = part + w * CM * 16 * RS;
#pragma unroll
  for (int mt = 0; mt < CM; ++mt)
    if (c * CM + mt < MT)
#pragma unroll
      for (int j = 0; j < 4; ++j) p[(mt * 16 + 4 * (lane >> 4) + j) * RS + (lane & 15)] = acc[c * CM + mt][j];
}
template <int KS, int Bp>
__device__ __forceinline__ float lds_sum(const float* part, int m, int n) {
  float s = part[m * RS + n];
#pragma unroll
  for (int w = 1; w < KS; ++w) s += part[(w * Bp + m) * RS + n];
  return s;
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// sum over the 16 lanes of a DPP row (every lane of the row gets the row sum)
__device__ __forceinline__ float row16_sum(float v) {
  auto dpp = [](float x, auto ctrl) {
    // every lane of every row is enabled and these patterns never read outside the row, so the
    // old value is never used: mov_dpp (bound_ctrl) needs no zero-initialised destination
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), decltype(ctrl)::value, 0xf, 0xf, true));
  };
  v += dpp(v, std::integral_constant<int, 0xB1>{});   // quad_perm(1,0,3,2)
  v += dpp(v, std::integral_constant<int, 0x4E>{});   // quad_perm(2,3,0,1)
  v += dpp(v, std::integral_constant<int, 0x124>{});  // row_ror:4
  v += dpp(v, std::integral_constant<int, 0x128>{});  // row_ror:8
  return v;
}
// sum over all 64 lanes (uniform result)
__device__ __forceinline__ float wave64_sum(float v) {
  v = row16_sum(v);
  const int b = __float_as_int(v);
  return __int_as_float(__builtin_amdgcn_readlane(b, 0)) + __int_as_float(__builtin_amdgcn_readlane(b, 16)) +
         __int_as_float(__builtin_amdgcn_readlane(b, 32)) + __int_as_float(__builtin_amdgcn_readlane(b, 48));
}

// ------------------------------------------------------------------ attention work item
// utterance b, positions [PTC ch, PTC ch + PTC): energies (common_layers.py:268-278, 90-110),
// chunk partials, last arriver normalises and writes alpha, alpha_cum, alignment and context
// (common_layers.py:347-366). NT = 512 threads: 4 groups over the 128 attention dims, 8 positions
// per thread.
// location_dense(location_conv(alpha, alpha_cum)) is linear with no biases, so it is applied as
// ONE 62-tap filter per attention dim: Wcomb[i*31 + k][a] = sum_c W_dense[a][c] W_conv[c][i][k]
// (folded in double at load; read from LDS), slid over the alpha window in registers.

// attention item timestamps (P.atrace, optional): [8 steps][256 items][8]
// The phase / item stamps are compiled in only with -DTTS_PHASE_TRACE (tools/build_variants.sh,
// TTS_PTRACE=<file> with TTSHIP_LIB pointing at that build): in the default build their conditions
// and pointers held ~10 SGPRs across the step loop, in a kernel whose SGPRs already spill to VGPR
// lanes, and every phase start paid the lane reads and writes
#ifdef TTS_PHASE_TRACE
#define ATRACE(k)                                                                             \
  if (P.atrace && threadIdx.x == 0 && (unsigned)(t - P.trace_t0) < 8u)                         \
  P.atrace[(((long)(t - P.trace_t0) * PW + b * P.nchmax + ch) * 8) + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define ATRACE(k)
#endif

// Location features of item (b, ch) for this step, computed one phase early (P1, from the alpha /
// alpha_cum the previous step's combine wrote): L[i] = location term + processed input at position
// t0 + 16 (i >> 2) + 4 (lane >> 4) + (i & 3), attention dim 16 wave + (lane & 15). Sums
// loc + penc before the query is added: (pq + (loc + penc)) instead of the reference's
// ((pq + loc) + penc), a one-ulp reassociation inside the tanh argument.
// T: the utterance's length (D.lens[b], read by the caller: for a workgroup's first item once per
// launch, so that the window loads below do not wait for it)
__device__ __forceinline__ void attn_loc(const PArgs& P, int b, int ch, int T, float* Aw, const float* wcomb,
                                         float (&L)[8]) {
  const DecDev& D = P.D;
  const int t0 = ch * PTC;
  const int tid = opaque_v(threadIdx.x);
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int a = 16 * wave + (lane & 15);
  const int Tm1 = max(T - 1, 0);
  float aw;
  {
    const int q = tid & 63, ci = (tid >> 6) & 1;  // threads 0-127 fill the two windows
    const int pos = t0 - (LOCK_ - 1) / 2 + q;
    const int pc = min(max(pos, 0), Tm1);
    aw = ldc((ci ? P.acum : P.alpha) + (long)b * D.T_max + pc);
    if (pos < 0 || pos >= T) aw = 0.f;
  }
  float pen[8];  // (position tile mt, row r) -> position 16 mt + 4 (lane >> 4) + r
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int pos = 16 * (i >> 2) + 4 * (lane >> 4) + (i & 3);
    pen[i] = P.penc[((long)b * D.T_max + min(t0 + pos, Tm1)) * ADIM_ + a];
  }
  if (P.spk_penc) {  // processed inputs of the speaker columns: W_in,s s, constant over positions
    const float ps = P.spk_penc[(long)b * P.spk_ld + a];
#pragma unroll
    for (int i = 0; i < 8; ++i) pen[i] += ps;
  }
  if (tid < 128) Aw[tid] = aw;
  lds_barrier();
  // location_dense(location_conv(.)) on MFMA: E[pos][dim] = sum_j X[pos][j] Wcomb[j][dim],
  // X[pos][ci*31 + k] = window_ci[pos + k]; K = 62 taps padded to 64 (Wcomb rows 62, 63 are 0)
  f32x4 le[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int st = 0; st < 16; ++st) {
    const int j = 4 * st + (lane >> 4);
    const int ci = j >= LOCK_ ? 1 : 0;
    const int k = j - LOCK_ * ci;
    const bool valid = j < 2 * LOCK_;
    const float w = wcomb[j * WCLD + a];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const float x = valid ? Aw[ci * 64 + 16 * mt + (lane & 15) + k] : 0.f;
      le[mt] = MFMA16(x, w, le[mt]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) L[i] = le[i >> 2][i & 3] + pen[i];
  lds_barrier();  // window reads done before the scratch is reused
}

// ekeep: (deferred alignment pass) LDS slot [32 energies | valid flag] of this item, kept until P6;
// null: the last arriver runs the alignment pass itself (decoder variants, many items per workgroup)
template <int MT, int VAR>
__device__ __forceinline__ void pattn_item(const PArgs& P, int t, int b, int ch, int Tb, float* sm, const float* wcomb,
                                           int* is_last, float (&L)[8], bool haveL,
                                           f32x4 (&evc)[pec_arr(VAR, MT)], bool load_ev, float* ekeep) {
  constexpr int PEC = pec_of(VAR, MT);
  constexpr bool WIN = VAR & 1, FWD = (VAR & 2) != 0;  // compiled-in decoder variants
  constexpr int NT = PT, TC = PTC;
  constexpr int NPT = NPQ_ / 16;  // query partials per thread (16 groups)
  constexpr int Bp = MT * 16;
  static_assert(TC == 32 && NT == 512, "attention item geometry: 2 position tiles x 8 dim tiles");
  const DecDev& D = P.D;
  const int t0 = ch * TC;
  float* red = sm;              // [16][ADIM] query-partial group sums
  float* Aw = red + 16 * ADIM_; // [2][64]: alpha / alpha_cum windows, alpha[t0 - 15 + q]
  float* esum = Aw + 128;       // [8 waves][TC] partial energies
  float* sv = esum + 8 * TC;    // [TC] energies
  float* sw = sv + TC;          // [TC] normalised weights
  float* swf = sw + TC;         // [TC] forward-attention weights
  if (!haveL) attn_loc(P, b, ch, Tb, Aw, wcomb, L);  // items beyond a workgroup's first
  const int tid = opaque_v(threadIdx.x);
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // attention dims 16 wave .. 16 wave + 15
  const int a = 16 * wave + (lane & 15);                       // this lane's dim in the MFMA output
  // ---- independent loads first (clamped indices), in the order they are consumed: vmcnt is an
  //      in-order counter, so waiting for an early load does not wait for the later ones. The
  //      query partials (the phase's critical hand-off) go out before anything whose value is
  //      needed to form an address: reading the utterance length first put a full load round
  //      trip (~0.5 us) in front of them ----
  const int a4 = tid & 31, pg = tid >> 5;  // query partials: 16-byte loads, dims 4 a4 .. 4 a4 + 3
  f32x4 pp[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) pp[i] = ldc4(P.pq, ((((pg * NPT + i) * Bp + b) * ADIM_) + 4 * a4) * 4);
  const int dn = ldci(D.done + b);
  const float va = P.v[a];
  __builtin_amdgcn_sched_barrier(0);
  const int T = Tb;
  const int Tm1 = max(T - 1, 0);
  ATRACE(0);
  if (t0 >= T || dn) return;  // workgroup-uniform
  {
    f32x4 s4 = pp[0];
#pragma unroll
    for (int i = 1; i < NPT; ++i) s4 += pp[i];
    *reinterpret_cast<f32x4*>(&red[pg * ADIM_ + 4 * a4]) = s4;
  }
  lds_barrier();
  ATRACE(1);
  // encoder rows for the partial context, consumed after the energies: thread (eg = tid / 128,
  // cq = tid % 128) holds channels 4 cq .. 4 cq + 3 of positions 8 eg .. 8 eg + 7, one 16-byte
  // buffer load each (row offsets in SGPRs: eg is wave-uniform). The encoder output is constant
  // over the decode, so a workgroup's first item keeps its first PEC rows in registers for the
  // whole launch (loaded on its first step; all 8 would push the kernel past 256 VGPRs); the rest
  // load every step, once the first batch of loads has drained
  constexpr int EPG = TC / 4;  // positions per thread group
  const int eg = tid >> 7, cq = tid & 127;
  f32x4 ev4[EPG];
  {
    const __amdgpu_buffer_rsrc_t er =
        __builtin_amdgcn_make_buffer_rsrc((void*)(P.enc + (long)b * D.T_max * 512), 0, 0x7fffffff, 0x00020000);
    auto ld = [&](int i) {
      return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
          er, cq * 16, __builtin_amdgcn_readfirstlane(min(t0 + EPG * eg + i, Tm1) * 2048), 0));
    };
    if (load_ev) {
#pragma unroll
      for (int i = 0; i < PEC; ++i) evc[i] = ld(i);
    }
#pragma unroll
    for (int i = PEC; i < EPG; ++i) ev4[i] = ld(i);
#pragma unroll
    for (int i = 0; i < PEC; ++i) ev4[i] = evc[i];
  }
  float pqa = red[a];
#pragma unroll
  for (int g = 1; g < 16; ++g) pqa += red[g * ADIM_ + a];
  ATRACE(2);
  // e = v . tanh(pq + loc + penc): the 16 dims of a DPP row summed in registers, the 8 waves
  // (dim tiles) through LDS
  {
    float z[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = row16_sum(tanh_e(pqa + L[i]) * va);
    if ((lane & 15) == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) esum[wave * TC + 16 * (i >> 2) + 4 * (lane >> 4) + (i & 3)] = z[i];
    }
  }
  lds_barrier();
  ATRACE(3);
  const int nvalid = min(TC, T - t0);
  const long pidx = (long)b * P.nchmax + ch;
  // attention windowing (common_layers.py:286-300): energies outside [lo, hi) around the previous
  // step's argmax become -inf; on the first step (win_idx == -1) position 0 takes the max energy
  int wlo = 0, whi = T, widx = 0;
  if ((WIN && P.win)) {
    widx = ldci(P.win_idx + b);
    if (widx - 2 > 0) wlo = widx - 2;
    if (widx + 6 < T) whi = widx + 6;
  }
  if (tid < TC) {
    float e = P.bv;
#pragma unroll
    for (int w = 0; w < 8; ++w) e += esum[w * TC + tid];
    if ((WIN && P.win) && (t0 + tid < wlo || t0 + tid >= whi)) e = -INFINITY;
    sv[tid] = e;
  }
  lds_barrier();
  if ((WIN && P.win) && widx == -1 && ch == 0) {  // the first window [0, 5) lies in chunk 0
    if (tid == 0) {
      float mx = -INFINITY;
      for (int i = 0; i < nvalid; ++i) mx = fmaxf(mx, sv[i]);
      sv[0] = mx;
    }
    lds_barrier();
  }
  if (ekeep) {  // the alignment pass runs in P6 from these (only the last arriver's combine reads
                // other chunks, and it needs their partials, not their energies)
    if (tid < TC) ekeep[tid] = sv[tid];
    if (tid == 0) ekeep[TC] = 1.f;
  } else if (tid < nvalid) {
    stc(P.energy + (long)b * D.T_max + t0 + tid, sv[tid]);
  }
  ATRACE(4);
  // chunk-local normalisation terms (computed once, shared through LDS)
  float m_c = -INFINITY;
  if (P.softmax) {
#pragma unroll
    for (int i = 0; i < TC; ++i)
      if (i < nvalid) m_c = fmaxf(m_c, sv[i]);
  }
  // forward attention (common_layers.py:302-323): w = ((1-u) a[t] + u a[t-1] + 1e-8) * raw with
  // raw = sigmoid(e) or exp(e - m_c); the normaliser of raw cancels in the renormalisation
  const float fu = (FWD && P.fwd) ? ldc(P.fwd_u + b) : 0.f;
  auto fwd_prev = [&](int pos) {  // previous forward alignment (init [1, 1e-7, ...], :236-241)
    if (pos < 0) return 0.f;
    return t == 0 ? (pos == 0 ? 1.f : 1e-7f) : ldc(P.alpha + (long)b * D.T_max + pos);
  };
  if (tid < TC) {
    const float e = sv[tid];
    float x = P.softmax ? (m_c == -INFINITY ? 0.f : expf(e - m_c)) : sigm_f(e);
    if (tid >= nvalid) x = 0.f;
    sw[tid] = x;
    if ((FWD && P.fwd)) {
      const int pos = t0 + tid;
      swf[tid] = tid < nvalid ? ((1.f - fu) * fwd_prev(pos) + fu * fwd_prev(pos - 1) + 1e-8f) * x : 0.f;
    }
  }
  lds_barrier();
  const float* wsel = (FWD && P.fwd) ? swf : sw;
  // chunk sums of the weights: only thread 0 publishes them, so wave 0 alone sums them (one
  // position per lane and a wave reduction instead of a 32-term loop in every thread)
  float S_c = 0.f, F_c = 0.f;
  if (wave == 0) {
    S_c = wave64_sum(lane < TC ? sw[lane] : 0.f);
    if ((FWD && P.fwd)) F_c = wave64_sum(lane < TC ? swf[lane] : 0.f);
  }
  // partial context: 4 channels x 8 positions per thread, then the 4 position groups summed
  // through LDS (the query-partial scratch `red`, [4][512], is free since the energies)
  float u;
  {
    f32x4 u4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < EPG; ++i) {
      const float wv = wsel[EPG * eg + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) u4[j] = fmaf(wv, ev4[i][j], u4[j]);
    }
    *reinterpret_cast<f32x4*>(&red[eg * 512 + 4 * cq]) = u4;
    lds_barrier();
    u = (red[tid] + red[512 + tid]) + (red[1024 + tid] + red[1536 + tid]);
  }
  stc_quad(P.part_u, (int)pidx * 512 + tid, u);
  if (tid == 0) {
    stc(P.part_s + pidx, S_c);
    stc(P.part_m + pidx, m_c);
    if ((FWD && P.fwd)) stc(P.part_f + pidx, F_c);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ATRACE(5);
  const int nch = (T + TC - 1) / TC;
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add(&P.counter[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *is_last = (prev == (unsigned)(nch - 1));
  }
  lds_barrier();
  ATRACE(6);
  if (!*is_last) return;
  // the alignment pass's first loads (position tid), issued ahead of the combine's: they do not
  // depend on it, and vmcnt is in order, so they land while the partials are summed
  const long ab = (long)b * D.T_max;
  const int tt0 = min(tid, Tm1);
  const float e_first = ekeep ? 0.f : ldc(P.energy + ab + tt0);
  const float acum_first = ekeep ? 0.f : ldc(P.acum + ab + tt0);
  // combine: chunk partials in batches of 8, all loads of a batch in flight (clamped)
  const long pb0 = (long)b * P.nchmax;
  constexpr int CB = 8;
  float m = -INFINITY, S = 0.f, Fz = 0.f, cx = 0.f;
  for (int cb = 0; cb < nch; cb += CB) {
    float pm[CB], ps[CB], pf[CB], pu[CB];
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const long c = pb0 + min(cb + i, nch - 1);
      pm[i] = ldc(P.part_m + c);
      ps[i] = ldc(P.part_s + c);
      pf[i] = (FWD && P.fwd) ? ldc(P.part_f + c) : 0.f;
      pu[i] = ldc(P.part_u + c * 512 + tid);
    }
    float wc[CB];
    if (P.softmax) {
      float mb = m;
#pragma unroll
      for (int i = 0; i < CB; ++i)
        if (cb + i < nch) mb = fmaxf(mb, pm[i]);
      const float sc = (m == -INFINITY) ? 0.f : expf(m - mb);
      S *= sc;
      Fz *= sc;
      cx *= sc;
      m = mb;
#pragma unroll
      for (int i = 0; i < CB; ++i) wc[i] = (cb + i < nch && pm[i] != -INFINITY) ? expf(pm[i] - m) : 0.f;
    } else {
#pragma unroll
      for (int i = 0; i < CB; ++i) wc[i] = (cb + i < nch) ? 1.f : 0.f;
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      S = fmaf(ps[i], wc[i], S);
      Fz = fmaf(pf[i], wc[i], Fz);
      cx = fmaf(pu[i], wc[i], cx);
    }
  }
  float ctx_v = cx / ((FWD && P.fwd) ? Fz : S);
  stc_quad_h<presplit_of(VAR)>(P.ctx, (int)frag_idx(b, tid, 512), ctx_v);
  ATRACE(7);
  if (ekeep) {  // deferred alignment pass: publish the normaliser, the items finish in P6
    if (tid == 0) {
      stc(P.anorm + 2 * b, S);
      stc(P.anorm + 2 * b + 1, m);
      __hip_atomic_store(&P.counter[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  float bestv = -INFINITY;
  int besti = 0x7fffffff;
  // forward_attn_mask (common_layers.py:309-318): argmax of the shifted previous alignment
  // (1 + first argmax of a[0 .. T-2]; 0 when that max is 0) and the max of the unmasked one
  float prv_m = 0.f, vmax = 0.f;
  int prv_i = 0x7fffffff;
  for (int tt = tid; tt < T; tt += NT) {
    const float e = tt == tid ? e_first : ldc(P.energy + ab + tt);
    if ((WIN && P.win) && (e > bestv || (e == bestv && tt < besti))) {
      bestv = e;
      besti = tt;
    }
    const float raw = P.softmax ? (e == -INFINITY ? 0.f : expf(e - m)) : 1.f / (1.f + expf(-e));
    const float al = raw / S;
    stc(P.acum + ab + tt, (tt == tid ? acum_first : ldc(P.acum + ab + tt)) + al);  // location state: raw alignment
    if ((FWD && P.fwd)) {  // forward alignment into the energy slot (alpha is still read as a[t-1] here)
      const float ap = fwd_prev(tt);
      const float fa = ((1.f - fu) * ap + fu * fwd_prev(tt - 1) + 1e-8f) * raw / Fz;
      stc(P.energy + ab + tt, fa);
      if (P.fwd_mask) {
        vmax = fmaxf(vmax, fa);
        if (tt <= T - 2 && ap > prv_m) {  // strictly greater: the first index of the max
          prv_m = ap;
          prv_i = tt;
        }
      }
    } else {
      stc(P.alpha + ab + tt, al);
      if (t < D.S_cap) D.align_out[((long)b * D.S_cap + t) * D.T_max + tt] = al;
    }
  }
  if ((FWD && P.fwd)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // mask: keep [lo, n + 2] (lo = n - 1, or T - 1 when n = 0: Python's a[:-1] = 0), then
    // a[n - 2] (negative index wraps) = 0.01 max, renormalise; the context is recomputed from the
    // at most 5 surviving positions
    int lo = 0, hi = T - 1, pp = -1;
    float vz = 0.f, zsum = 1.f;
    if (P.fwd_mask) {
      for (int off = 32; off > 0; off >>= 1) {
        const float ov = __shfl_xor(prv_m, off, 64);
        const int oi = __shfl_xor(prv_i, off, 64);
        if (ov > prv_m || (ov == prv_m && oi < prv_i)) {
          prv_m = ov;
          prv_i = oi;
        }
        vmax = fmaxf(vmax, __shfl_xor(vmax, off, 64));
      }
      float* rv = red;
      int* ri = reinterpret_cast<int*>(red + 16);
      float* rm = red + 32;
      if (lane == 0) {
        rv[tid >> 6] = prv_m;
        ri[tid >> 6] = prv_i;
        rm[tid >> 6] = vmax;
      }
      lds_barrier();
      float pv = rv[0], vm = rm[0];
      int pi = ri[0];
      for (int w = 1; w < NT / 64; ++w) {
        if (rv[w] > pv || (rv[w] == pv && ri[w] < pi)) {
          pv = rv[w];
          pi = ri[w];
        }
        vm = fmaxf(vm, rm[w]);
      }
      const int n = pv > 0.f ? pi + 1 : 0;
      lo = n >= 1 ? n - 1 : T - 1;
      hi = min(n + 2, T - 1);
      pp = n - 2 < 0 ? n - 2 + T : n - 2;
      vz = 0.01f * vm;
      zsum = 0.f;
      for (int j = lo; j <= hi; ++j)
        if (j != pp) zsum += ldc(P.energy + ab + j);
      if (pp >= 0) zsum += vz;
      lds_barrier();  // the reduction scratch is reused below
    }
    for (int tt = tid; tt < T; tt += NT) {
      float af = ldc(P.energy + ab + tt);
      if (P.fwd_mask) af = tt == pp ? vz / zsum : (tt >= lo && tt <= hi ? af / zsum : 0.f);
      stc(P.alpha + ab + tt, af);
      if (t < D.S_cap) D.align_out[((long)b * D.S_cap + t) * D.T_max + tt] = af;
    }
    if (P.fwd_mask) {
      const float* eb = P.enc + (long)b * D.T_max * 512 + tid;
      float c2 = 0.f;
      for (int j = lo; j <= hi; ++j)
        if (j != pp) c2 = fmaf(ldc(P.energy + ab + j) / zsum, eb[(long)j * 512], c2);
      if (pp >= 0) c2 = fmaf(vz / zsum, eb[(long)pp * 512], c2);
      ctx_v = c2;
      stc(P.ctx + frag_idx(b, tid, 512), ctx_v);
    }
  }
  if ((WIN && P.win) || ((FWD && P.fwd) && P.trans)) {
    // block reductions over the 512 threads: window argmax (first index of the max energy) and the
    // transition agent u = sigmoid(ta . [context, query] + b) for the next step
    float tdot = 0.f;
    if ((FWD && P.fwd) && P.trans) {
      tdot = P.ta_w[tid] * ctx_v;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int q = tid + k * NT;
        tdot = fmaf(P.ta_w[512 + q], ldc(P.hatt + frag_idx(b, q, 1024)), tdot);
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      const float ov = __shfl_xor(bestv, off, 64);
      const int oi = __shfl_xor(besti, off, 64);
      if (ov > bestv || (ov == bestv && oi < besti)) {
        bestv = ov;
        besti = oi;
      }
      tdot += __shfl_xor(tdot, off, 64);
    }
    float* rv = red;  // the query-partial scratch is free by now
    int* ri = reinterpret_cast<int*>(red + 16);
    float* rt = red + 32;
    lds_barrier();
    if (lane == 0) {
      rv[tid >> 6] = bestv;
      ri[tid >> 6] = besti;
      rt[tid >> 6] = tdot;
    }
    lds_barrier();
    if (tid == 0) {
      float bv = rv[0], ts = rt[0];
      int bi = ri[0];
      for (int w = 1; w < NT / 64; ++w) {
        if (rv[w] > bv || (rv[w] == bv && ri[w] < bi)) {
          bv = rv[w];
          bi = ri[w];
        }
        ts += rt[w];
      }
      if ((WIN && P.win)) stci(P.win_idx + b, bi);
      if ((FWD && P.fwd) && P.trans) stc(P.fwd_u + b, 1.f / (1.f + expf(-(ts + P.ta_b))));
    }
  }
  if (tid == 0) __hip_atomic_store(&P.counter[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// Graves attention item (common_layers.py:150-193, eval: no dropout; mask None at B = 1): utterance
// b, positions [PTC ch, PTC ch + PTC). gbk = N_a.2(hidden) from the P3g hidden row, the mixture
// (softmax(g) + eps, softplus(b) + eps, mu_prev + softplus(k)), alpha_j = F(j + 1) - F(j) with
// F(i) = sum_k g_k / (1 + sigmoid((mu_k - i - 0.5) / sig_k)) (0 -> 1e-8), the partial context
// (alpha is not normalised); the last arriver sums the partials and carries mu to the next step.
__device__ __forceinline__ float softplus_t(float x) { return x > 20.f ? x : log1pf(expf(x)); }

template <int MT>
__device__ __forceinline__ void graves_item(const PArgs& P, int t, int b, int ch, float* sm, int* is_last) {
  constexpr int NT = PT, TC = PTC;
  const DecDev& D = P.D;
  const int t0 = ch * TC;
  const int tid = opaque_v(threadIdx.x);
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = D.lens[b];
  const int K = P.gK;
  float* red = sm;             // [48][8] wave partials of gbk
  float* gbk = red + 48 * 8;   // [48]
  float* sw = gbk + 48;        // [TC] alpha of this chunk
  const int dn = ldci(D.done + b);
  const float hv0 = ldc(P.gh + (long)b * 1024 + tid), hv1 = ldc(P.gh + (long)b * 1024 + tid + NT);
  if (t0 >= T || dn) return;  // workgroup-uniform
  for (int o = 0; o < 3 * K; ++o) {
    const float v = wave64_sum(fmaf(P.na2_w[(long)o * 1024 + tid], hv0, P.na2_w[(long)o * 1024 + tid + NT] * hv1));
    if (lane == 0) red[o * 8 + wave] = v;
  }
  lds_barrier();
  if (tid < 3 * K) {
    float v = P.na2_b[tid];
#pragma unroll
    for (int w = 0; w < 8; ++w) v += red[tid * 8 + w];
    gbk[tid] = v;
  }
  lds_barrier();
  // mixture parameters (every thread, K <= 16)
  float gm = -INFINITY;
  for (int k = 0; k < K; ++k) gm = fmaxf(gm, gbk[k]);
  float gs = 0.f;
  for (int k = 0; k < K; ++k) gs += expf(gbk[k] - gm);
  const long pidx = (long)b * P.nchmax + ch;
  const int nvalid = min(TC, T - t0);
  if (tid < TC) {
    float al = 0.f;
    if (tid < nvalid) {
      const float j0 = (float)(t0 + tid) + 0.5f, j1 = j0 + 1.f;
      float f0 = 0.f, f1 = 0.f;
      for (int k = 0; k < K; ++k) {
        const float gk = expf(gbk[k] - gm) / gs + 1e-5f;
        const float sg = softplus_t(gbk[K + k]) + 1e-5f;
        const float mu = ldc(P.gmu + (long)b * 16 + k) + softplus_t(gbk[2 * K + k]);
        f0 += gk * (1.f / (1.f + 1.f / (1.f + expf(-((mu - j0) / sg)))));
        f1 += gk * (1.f / (1.f + 1.f / (1.f + expf(-((mu - j1) / sg)))));
      }
      al = f1 - f0;
      if (al == 0.f) al = 1e-8f;
      if (t < D.S_cap) D.align_out[((long)b * D.S_cap + t) * D.T_max + t0 + tid] = al;
    }
    sw[tid] = al;
  }
  lds_barrier();
  {
    const float* eb = P.enc + ((long)b * D.T_max + t0) * 512 + tid;
    float u = 0.f;
    for (int i = 0; i < nvalid; ++i) u = fmaf(sw[i], eb[(long)i * 512], u);
    stc_quad(P.part_u, (int)pidx * 512 + tid, u);
    if (P.spk_scale && wave == 0) {  // chunk sum of the weights: the speaker columns' context factor
      const float s_c = wave64_sum(lane < nvalid ? sw[lane] : 0.f);
      if (lane == 0) stc(P.part_s + pidx, s_c);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int nch = (T + TC - 1) / TC;
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add(&P.counter[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *is_last = (prev == (unsigned)(nch - 1));
  }
  lds_barrier();
  if (!*is_last) return;
  const long pb0 = (long)b * P.nchmax;
  float cx = 0.f;
  for (int c = 0; c < nch; ++c) cx += ldc(P.part_u + (pb0 + c) * 512 + tid);
  stc(P.ctx + frag_idx(b, tid, 512), cx);
  if (P.spk_scale && tid == 0) {  // context of the speaker columns = (sum_j alpha_j) s
    float sa = 0.f;
    for (int c = 0; c < nch; ++c) sa += ldc(P.part_s + pb0 + c);
    stc(P.anorm + 2 * b, sa);
  }
  if (tid < K) stc(P.gmu + (long)b * 16 + tid, ldc(P.gmu + (long)b * 16 + tid) + softplus_t(gbk[2 * K + tid]));
  if (tid == 0) __hip_atomic_store(&P.counter[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// acc[MT] += act[:, chunks kc0 .. kc0+NC) . W^T for one fragment-order activation with nk 16-column
// chunks; wf(i) gives the weight fragment of local chunk i (registers or LDS). Activation loads
// run G chunks ahead (two register stages).
template <int MT, int NC, int G, class WF>
__device__ __forceinline__ void gemm_seg(f32x4 (&acc)[MT], const float* base, int nk, int kc0, int lane, WF wf) {
  static_assert(NC % G == 0, "chunk groups");
  auto ld = [&](int kc, int mt) { return ldc4<ACT_AUX>(base, ((mt * nk + kc) * 64 + lane) * 16); };
  f32x4 x[2][G][MT];
#pragma unroll
  for (int i = 0; i < G; ++i)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) x[0][i][mt] = ld(kc0 + i, mt);
#pragma unroll
  for (int i0 = 0; i0 < NC; i0 += G) {
    const int cur = (i0 / G) & 1;
    if (i0 + G < NC) {
#pragma unroll
      for (int i = 0; i < G; ++i)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) x[cur ^ 1][i][mt] = ld(kc0 + i0 + G + i, mt);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const f32x4 w = wf(i0 + i);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = MFMA16(x[cur][i][mt][q], w[q], acc[mt]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Split-f16 forms of gemm_seg / gemm_seg2 over k-steps ks0 .. ks0 + NKS - 1 (32 columns each) of
// an fp32 fragment-order activation with nk 16-column chunks per 16-row block. The activation is
// split in registers: lane L of k-step ks holds row L & 15, k = 32 ks + 8 (L >> 4) + 0..7, i.e.
// chunk 2 ks + (L >> 5) at fragment lanes l1 and l1 + 16. wf(k, hi, lo) yields the B fragment
// (split weights) of the k-th step. Adds to the accumulators; one k-step of loads in flight.
template <int MT>
__device__ __forceinline__ void ld_x3_step(f32x4 (&x)[MT][2], const float* base, int nk, int ks, int lane) {
  const int l1 = 32 * ((lane >> 4) & 1) + (lane & 15);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int c = mt * nk + 2 * ks + (lane >> 5);
    x[mt][0] = ldc4<ACT_AUX>(base, (c * 64 + l1) * 16);
    x[mt][1] = ldc4<ACT_AUX>(base, (c * 64 + l1 + 16) * 16);
  }
}
// PS: the chunk was published pre-split (stc_quad_x3): x[0] holds k 0..3 as [hi | lo], x[1] k 4..7
template <bool PS>
__device__ __forceinline__ void split_x3_step(const f32x4 (&x)[2], h8& xh, h8& xl) {
  if constexpr (PS) {
    xh = __builtin_bit_cast(h8, (f32x4{x[0][0], x[0][1], x[1][0], x[1][1]}));
    xl = __builtin_bit_cast(h8, (f32x4{x[0][2], x[0][3], x[1][2], x[1][3]}));
  } else {
    const float v[8] = {x[0][0], x[0][1], x[0][2], x[0][3], x[1][0], x[1][1], x[1][2], x[1][3]};
    split8(v, xh, xl);
  }
}
template <int MT, int NKS, bool PS = false, class WF>
__device__ __forceinline__ void gemm_x3(f32x4 (&acc)[MT], const float* base, int nk, int ks0, int lane, WF wf) {
  f32x4 x[2][MT][2];
  ld_x3_step<MT>(x[0], base, nk, ks0, lane);
  f32x4 am[MT], ac[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) am[mt] = ac[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < NKS; ++k) {
    if (k + 1 < NKS) ld_x3_step<MT>(x[(k + 1) & 1], base, nk, ks0 + k + 1, lane);
    h8 bh, bl;
    wf(k, bh, bl);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      h8 xh, xl;
      split_x3_step<PS>(x[k & 1][mt], xh, xl);
      mfma_x3(xh, xl, bh, bl, am[mt], ac[mt]);
    }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[mt][j] += x3_value(am[mt][j], ac[mt][j]);
}
template <int MT, int NKS, bool PS = false, class WF1, class WF2>
__device__ __forceinline__ void gemm_x3_pair(f32x4 (&acc1)[MT], f32x4 (&acc2)[MT], const float* base, int nk, int ks0,
                                             int lane, WF1 wf1, WF2 wf2) {
  f32x4 x[2][MT][2];
  ld_x3_step<MT>(x[0], base, nk, ks0, lane);
  f32x4 am1[MT], ac1[MT], am2[MT], ac2[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) am1[mt] = ac1[mt] = am2[mt] = ac2[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < NKS; ++k) {
    if (k + 1 < NKS) ld_x3_step<MT>(x[(k + 1) & 1], base, nk, ks0 + k + 1, lane);
    h8 b1h, b1l, b2h, b2l;
    wf1(k, b1h, b1l);
    wf2(k, b2h, b2l);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      h8 xh, xl;
      split_x3_step<PS>(x[k & 1][mt], xh, xl);
      mfma_x3(xh, xl, b1h, b1l, am1[mt], ac1[mt]);
      mfma_x3(xh, xl, b2h, b2l, am2[mt], ac2[mt]);
    }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc1[mt][j] += x3_value(am1[mt][j], ac1[mt][j]);
      acc2[mt][j] += x3_value(am2[mt][j], ac2[mt][j]);
    }
}

// P5 of the attention-item workgroups (split-f16): the h_att parts (NKA k-steps from `a`, weights
// wa1 / wa2) then the ctx parts (NKC k-steps from `c`, weights wc1 / wc2) of both LSTMs, one
// pipeline: every activation chunk is read once and the first ctx k-step's loads are in flight
// under the last h_att k-step
template <int MT, int NKA, int NKC, bool PS = false, class WA1, class WA2, class WC1, class WC2>
__device__ __forceinline__ void gemm_x3_hatt_ctx(f32x4 (&acc1)[MT], f32x4 (&acc2)[MT], const float* a, int nka,
                                                 int ksa, const float* c, int nkc, int ksc, int lane, WA1 wa1,
                                                 WA2 wa2, WC1 wc1, WC2 wc2) {
  constexpr int NS = NKA + NKC;
  auto ld = [&](f32x4 (&x)[MT][2], int k) {
    if (k < NKA) ld_x3_step<MT>(x, a, nka, ksa + k, lane);
    else ld_x3_step<MT>(x, c, nkc, ksc + k - NKA, lane);
  };
  f32x4 x[2][MT][2];
  ld(x[0], 0);
  f32x4 am1[MT], ac1[MT], am2[MT], ac2[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) am1[mt] = ac1[mt] = am2[mt] = ac2[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    if (k + 1 < NS) ld(x[(k + 1) & 1], k + 1);
    h8 b1h, b1l, b2h, b2l;
    if (k < NKA) wa1(k, b1h, b1l), wa2(k, b2h, b2l);
    else wc1(k - NKA, b1h, b1l), wc2(k - NKA, b2h, b2l);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      h8 xh, xl;
      split_x3_step<PS>(x[k & 1][mt], xh, xl);
      mfma_x3(xh, xl, b1h, b1l, am1[mt], ac1[mt]);
      mfma_x3(xh, xl, b2h, b2l, am2[mt], ac2[mt]);
    }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc1[mt][j] += x3_value(am1[mt][j], ac1[mt][j]);
      acc2[mt][j] += x3_value(am2[mt][j], ac2[mt][j]);
    }
}

// m-tiles O .. O + N - 1 of an accumulator array: the split-f16 GEMM helpers keep MT-sized operand
// and accumulator temporaries, so batch tiles of 48 / 64 rows run them in passes of at most 2 m-tiles
// (32 rows; the activation base moves by 2 m-tiles, nk 16-column chunks of 256 floats each) and stay
// within 256 VGPRs
template <int O, int N, int M>
__device__ __forceinline__ f32x4 (&msub(f32x4 (&a)[M]))[N] {
  static_assert(O + N <= M, "m-tile range");
  return *reinterpret_cast<f32x4(*)[N]>(&a[O]);
}
#define X3_PASSES(MT_, CALL)                       \
  do {                                             \
    if constexpr ((MT_) <= 2) {                    \
      constexpr int NM = (MT_), MO = 0;            \
      CALL;                                        \
    } else {                                       \
      {                                            \
        constexpr int NM = 2, MO = 0;              \
        CALL;                                      \
      }                                            \
      {                                            \
        constexpr int NM = (MT_) - 2, MO = 2;      \
        CALL;                                      \
      }                                            \
    }                                              \
  } while (0)

// gemm_seg for two accumulator sets over the SAME activation chunks (one load per chunk feeds both)
template <int MT, int NC, int G, class WF1, class WF2>
__device__ __forceinline__ void gemm_seg2(f32x4 (&acc1)[MT], f32x4 (&acc2)[MT], const float* base, int nk, int kc0,
                                          int lane, WF1 wf1, WF2 wf2) {
  static_assert(NC % G == 0, "chunk groups");
  auto ld = [&](int kc, int mt) { return ldc4<ACT_AUX>(base, ((mt * nk + kc) * 64 + lane) * 16); };
  f32x4 x[2][G][MT];
#pragma unroll
  for (int i = 0; i < G; ++i)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) x[0][i][mt] = ld(kc0 + i, mt);
#pragma unroll
  for (int i0 = 0; i0 < NC; i0 += G) {
    const int cur = (i0 / G) & 1;
    if (i0 + G < NC) {
#pragma unroll
      for (int i = 0; i < G; ++i)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) x[cur ^ 1][i][mt] = ld(kc0 + i0 + G + i, mt);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const f32x4 w1 = wf1(i0 + i);
      const f32x4 w2 = wf2(i0 + i);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          acc1[mt] = MFMA16(x[cur][i][mt][q], w1[q], acc1[mt]);
          acc2[mt] = MFMA16(x[cur][i][mt][q], w2[q], acc2[mt]);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ------------------------------------------------------------------ the persistent kernel
// LDS: [att-pre weights 96 x 1 KiB][Wcomb 64 x 128][scratch: GEMM reduction + hs | attention]
constexpr size_t P_LDS_APRE = 96 * 64 * 16;
constexpr size_t P_LDS_WC = 64 * WCLD * 4;
constexpr size_t P_LDS_SCRATCH = 8 * 32 * RS * 4 + 64 * 17 * 4;  // red0 | hs; >= attention scratch (~2.5K floats)
constexpr int PDEF_MAXIT = 8;  // attention items per workgroup the deferred alignment pass keeps
constexpr size_t P_LDS_EKEEP = PDEF_MAXIT * (32 + 1) * 4;
constexpr size_t P_LDS = P_LDS_APRE + P_LDS_WC + P_LDS_SCRATCH + P_LDS_EKEEP;

// phase timestamps of every workgroup for 8 steps (P.trace, optional): [step][16][256]
// (0-9 phase boundaries, 10-15 points inside P5)
#ifdef TTS_PHASE_TRACE
#define PTRACE(k)                                                                              \
  if (P.trace && threadIdx.x == 0 && (unsigned)(t - P.trace_t0) < 8u)                          \
  P.trace[((long)(t - P.trace_t0) * 16 + (k)) * PW + blockIdx.x] = __builtin_amdgcn_s_memrealtime()
#else
#define PTRACE(k)
#endif

template <int MT, int VAR>
__global__ __launch_bounds__(PT) void persist_decoder_kernel(PArgs P) {
  constexpr bool GRAVES = (VAR & 4) != 0;  // Graves attention replaces the location-sensitive one
  constexpr bool X3P = (VAR & 8) != 0;     // P3's attention_rnn prenet part on the split-f16 MFMA
  constexpr bool DEFER = (VAR & 7) == 0;   // plain location attention: alignment pass deferred to P6
  constexpr bool PS = presplit_of(VAR);    // h_att, ctx, h_dec published pre-split
  extern __shared__ __attribute__((aligned(16))) f32x4 smem4[];
  __shared__ int sflag, is_last;
  constexpr int Bp = MT * 16;
  constexpr int CM = MT < 2 ? MT : 2;            // m-tiles per LDS reduction chunk
  constexpr int CB = CM * 16;                    // rows per chunk
  constexpr int NCK = (MT + CM - 1) / CM;        // chunks (1 for MT <= 2)
  constexpr int JR = (X3P && MT > 2) ? 4 : 2;    // projection jobs per tile (row blocks / K halves)
  const DecDev& D = P.D;
  f32x4* Wap = smem4;                                              // [96][64]
  float* wcomb = reinterpret_cast<float*>(smem4) + 96 * 64 * 4;    // [64][WCLD]
  float* scr = wcomb + 64 * WCLD;
  float* red0 = scr;                   // [8][CB][RS]
  float* hs = red0 + 8 * 32 * RS;      // [Bp][17]
  float* ekeep0 = scr + P_LDS_SCRATCH / 4;  // [PDEF_MAXIT][PTC + 1]: deferred alignment pass
  const int g = blockIdx.x, tid0 = threadIdx.x, lane0 = tid0 & 63;
  const int wave0 = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  const int YP = P.ntj * 16;

  // ---- one-time: resident weights ----
  int tid = tid0, lane = lane0, wave = wave0;
  {
    const f32x4* src = reinterpret_cast<const f32x4*>(P.apre_w) + (long)g * 96 * 64;
    // split-f16 variant: the same bytes hold split B fragments [48 k-steps][64 lanes][hi | lo]
    const f32x4* srcx = reinterpret_cast<const f32x4*>(P.apre_x3) + (long)g * 96 * 64;
    for (int i = tid; i < 96 * 64; i += PT) {
      if (X3P) Wap[x3i(i >> 7, (i >> 1) & 63, i & 1)] = srcx[i];
      else Wap[i] = src[i];
    }
    if (g >= IW0)  // attention_rnn workgroups use this area as P3 staging instead
      for (int i = tid; i < 64 * 128; i += PT) wcomb[(i >> 7) * WCLD + (i & 127)] = P.Wcomb[i];
  }
  // decoder_rnn weights of this wave: K = [h_att 64 chunks | ctx 32 | h_dec 64]; wave w keeps
  // h_att chunks 8w..8w+7 (wd[0..7]), ctx chunks 4w..4w+3 (wd[8..11]), h_dec chunks 8w..8w+7
  // (wd[12..19]), so that each part can run in the phase where its input becomes final
  f32x4 wd[X3P ? 1 : DEC_NC];
  // split-f16 variant: slots 0-3 h_att k-steps 4w..4w+3, 4-5 ctx k-steps 32+2w, +1, 6-9 h_dec
  // k-steps 48+4w..+3 (the same K ranges as the fp32 chunks, 32 columns per k-step)
  h8 wdx[X3P ? 10 : 1][2];
  if constexpr (X3P) {
    const h8* src = reinterpret_cast<const h8*>(P.dec_x3) + ((long)g * 80 * 64 + lane) * 2;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int ks = i < 4 ? 4 * wave + i : (i < 6 ? 32 + 2 * wave + (i - 4) : 48 + 4 * wave + (i - 6));
      wdx[i][0] = src[(long)ks * 128];
      wdx[i][1] = src[(long)ks * 128 + 1];
    }
  } else {
    const f32x4* src = reinterpret_cast<const f32x4*>(P.dec_w) + (long)g * 160 * 64 + lane;
#pragma unroll
    for (int i = 0; i < 8; ++i) wd[i] = src[(long)(8 * wave + i) * 64];
#pragma unroll
    for (int i = 0; i < 4; ++i) wd[8 + i] = src[(long)(64 + 4 * wave + i) * 64];
#pragma unroll
    for (int i = 0; i < 8; ++i) wd[12 + i] = src[(long)(96 + 8 * wave + i) * 64];
  }
  const h8* Wapx = reinterpret_cast<const h8*>(Wap);
  auto wdx_f = [&](int base) { return [&, base](int k, h8& hi, h8& lo) { hi = wdx[base + k][0], lo = wdx[base + k][1]; }; };
  auto wap_f = [&](int ks0) {
    return [&, ks0](int k, h8& hi, h8& lo) {
      hi = Wapx[x3i(ks0 + k, lane, 0)];
      lo = Wapx[x3i(ks0 + k, lane, 1)];
    };
  };
  // epilogue constants: decoder_rnn biases of this thread's (row, unit) item, attention_rnn
  // ctx/h-part bias of its column
  float db[NCK][4];
#pragma unroll
  for (int c = 0; c < NCK; ++c)
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // + the row's speaker part (W_dec,s s, api.hip spk_bias_kernel)
      db[c][q] = P.dec_b[g * 16 + q * 4 + (tid & 3)];
      if (P.spk_dec && !(GRAVES && P.spk_scale))  // scaled per step below otherwise
        db[c][q] += P.spk_dec[(long)min(c * CB + (tid >> 2), Bp - 1) * P.spk_ld + g * 16 + q * 4 + (tid & 3)];
    }
  const float apb = P.apre_b[g * 16 + (tid & 15)];
  // Graves attention with speaker embeddings: its weights do not sum to 1, so the speaker columns'
  // share of the context is (sum_j alpha_j) s; every speaker bias the context feeds (attention_rnn
  // and decoder_rnn gates, the projection and the rows folded through it) scales by that per-row
  // sum of the step the context belongs to (published in P.anorm by the combine)
  const bool sscale = GRAVES && P.spk_scale;
  auto spk_sum = [&](int m) { return m < D.B ? ldc(P.anorm + 2 * m) : 0.f; };
  auto pjb1 = [&](int m, int col) {
    const float v = P.pjb_rows[(long)m * P.spk_ld + col];
    return sscale ? P.pj_b[col] + spk_sum(m) * v : v;
  };
  auto pjb4 = [&](int m, int col) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(P.pjb_rows + (long)m * P.spk_ld + col);
    return sscale ? *reinterpret_cast<const f32x4*>(P.pj_b + col) + spk_sum(m) * v : v;
  };
  __syncthreads();

  unsigned gen = 0;
  // the first attention item's utterance length, constant over the launch
  const int it_first = g - IW0;
  const int T_first = (it_first >= 0 && it_first < D.B * P.nchmax) ? D.lens[it_first / P.nchmax] : 0;
  float Lr[8];  // location features of the first attention item (attn_loc in P1, used in P4)
  f32x4 evc[pec_arr(VAR, MT)];  // encoder rows of the first attention item (loaded on its first step)
  if (P.diag && tid0 == 0) {  // placement diagnostics: which XCD this workgroup runs on
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    stci(reinterpret_cast<int*>(P.diag) + blockIdx.x, (int)(xcc & 15u));
  }
  const int t_first = D.ctl->base;
  int t = t_first;
  const int pj_jobs = (X3P && MT > 2 ? 4 : 2) * P.ntj;
  const int pj = g - PJ_WG0;  // projection job of this workgroup (P6), if 0 <= pj < pj_jobs
  const bool is_pj = pj >= 0 && pj < pj_jobs;
  // prenet layer-2 weight chunks of this wave
  // (workgroups 0-31: tile g & 15, k-chunks wave and 8 + wave: the whole K for 16 batch rows,
  // so P3 reads one pb copy)
  // are loaded per step at P1's start beside its hand-off loads (L2 hits): kept in registers for the
  // whole launch they held 8 VGPRs through P5's k-loop, where the kernel spilled to scratch
  // partial sums of this workgroup's decoder_rnn tile (accd) and attention_rnn ctx/h tile (acca),
  // accumulated across phases. Attention-item workgroups (g >= IW0): accd h_dec part in P3, h_att
  // part in P4 after the item, ctx part in P5; acca ctx part in P5, h_att part + epilogue in P6.
  // attention_rnn workgroups (g < IW0, no item): accd h_dec and both h_att parts in P4, ctx parts
  // and both epilogues in P5.
  f32x4 accd[MT], acca[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) accd[mt] = acca[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto dec_hdec_part = [&](const float* hd) {
    if constexpr (X3P)
      X3_PASSES(MT, (gemm_x3<NM, 4, PS>(msub<MO, NM>(accd), hd + MO * 64 * 256, 64, 4 * wave, lane, wdx_f(6))));
    else gemm_seg<MT, 8, 4>(accd, hd, 64, 8 * wave, lane, [&](int i) { return wd[12 + i]; });
  };
  // attention_rnn ctx/h tile g complete: reduce over the waves, add the biases, publish the next
  // step's gate addends, reset the accumulator
  auto att_epilogue = [&](float* red) {
#pragma unroll
    for (int c = 0; c < NCK; ++c) {
      acc_chunk_to_lds<MT, CM>(red, wave, lane, acca, c);
      lds_barrier();
      for (int idx = tid; idx < CB * 16; idx += PT) {
        const int m = c * CB + (idx >> 4), n = idx & 15;
        if (m >= Bp) break;
        float v = lds_sum<NWV, CB>(red, idx >> 4, n) + apb;
        if (P.spk_att) v += (sscale ? spk_sum(m) : 1.f) * P.spk_att[(long)m * P.spk_ld + g * 16 + n];  // speaker part of the new ctx
        stc_quad(P.gatt, m * 4096 + g * 16 + n, v);
      }
      if (NCK > 1) lds_barrier();
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acca[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // frames of step s (< S_cap) from the two projection halves (K5 frame store of decoder.hip):
  // written when the row was still decoding at step s, i.e. not done or done later than s
  auto write_frames = [&](int s, int wg0, int nwg) {
    if (s < 0 || s >= D.S_cap) return;
    const int FR = 80 * P.r;
    const int n = D.B * FR;
    for (int idx = (g - wg0) * PT + tid; idx < n; idx += nwg * PT) {
      const int m = idx / FR, c = idx - m * FR;
      if (!ldci(D.done + m) || ldci(D.steps + m) > s) {
        const float v = ldc(P.ypart + (long)m * YP + 16 + c) + (X3P ? 0.f : ldc(P.ypart + (long)(YROWS + m) * YP + 16 + c)) +
                        pjb1(m, 16 + c);
        D.dec_out[((long)m * D.S_cap + s) * FR + c] = v;
      }
    }
  };

  for (;; ++t) {
    PTRACE(0);
    float* hd_cur = (t & 1) ? P.hdec1 : P.hdec0;
    float* hd_nxt = (t & 1) ? P.hdec0 : P.hdec1;
    // ======== P1: prenet layer 2 (workgroups 0-31) || stop(t-1) (workgroup IW0 - 1) ========
    tid = opaque_v(tid0);
    lane = opaque_v(lane0);
    wave = opaque_s(wave0);
    if (g < 16 * MT) {  // prenet layer 2: tile g & 15, batch rows 16 (g >> 4) .. + 15, whole K
      const int tl2 = g & 15, mt = g >> 4;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4* w2p = reinterpret_cast<const f32x4*>(P.pre2_w) + ((long)tl2 * 16 + wave) * 64 + lane;
      const f32x4 w2 = w2p[0], w2b = w2p[8 * 64];
      // t = 0: the prenet input is the zero go-frame: layer 1 gives relu(b1') (BN prenet) or 0
      if (t > 0 || P.pre1_b0) {
        f32x4 x[2];
        const int m = mt * 16 + (lane & 15);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int kc = 8 * h + wave;
          const int col = P.nt_proj * 16 + kc * 16 + 4 * (lane >> 4);
          if (t > 0) {
            const f32x4 bb = pjb4(m, col);
            x[h] = X3P ? ldc4(P.ypart, (m * YP + col) * 4) + bb
                       : ldc4(P.ypart, (m * YP + col) * 4) + ldc4(P.ypart, ((YROWS + m) * YP + col) * 4) + bb;
          } else {
            x[h] = *reinterpret_cast<const f32x4*>(P.pre1_b0 + kc * 16 + 4 * (lane >> 4));
          }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int q = 0; q < 4; ++q) x[h][q] = fmaxf(x[h][q], 0.f);
#pragma unroll
          for (int q = 0; q < 4; ++q) acc = MFMA16(x[h][q], h ? w2b[q] : w2[q], acc);
        }
      }
      float* p = red0 + wave * 16 * RS;  // [wave][16 rows][RS]
#pragma unroll
      for (int j = 0; j < 4; ++j) p[(4 * (lane >> 4) + j) * RS + (lane & 15)] = acc[j];
      lds_barrier();
      if (tid < 256) {
        const int mm = tid >> 4, n = tid & 15;
        float v = red0[mm * RS + n];
#pragma unroll
        for (int w = 1; w < NWV; ++w) v += red0[(w * 16 + mm) * RS + n];
        if (P.pre2_b) v += P.pre2_b[tl2 * 16 + n];  // BN prenet layer-2 bias
        stc_quad(P.pb, (int)frag_idx(mt * 16 + mm, tl2 * 16 + n, 256), v);
      }
      lds_barrier();
    }
    // location features of this workgroup's first attention item for step t (alpha of t-1 is
    // final); items sit on workgroups IW0.. so that they miss the prenet workgroups
    const int it0 = g - IW0;
    if (!GRAVES && it0 >= 0 && it0 < D.B * P.nchmax)
      attn_loc(P, it0 / P.nchmax, it0 % P.nchmax, T_first, scr + 16 * ADIM_, wcomb, Lr);
    // stop decision: an attention_rnn workgroup that is not a prenet one (MT <= 2), or the last
    // item workgroup once every attention_rnn workgroup runs a prenet job (MT = 3, 4)
    if (g == (MT <= 2 ? IW0 - 1 : PW - 1)) {
      int dn = 1;
      if (tid < D.B) {
        const int m = tid;
        // every input of the decision in one round trip (the logit's loads used to wait for the
        // done flag's)
        dn = ldci(D.done + m);
        const float y0 = ldc(P.ypart + (long)m * YP), y1 = X3P ? 0.f : ldc(P.ypart + (long)(YROWS + m) * YP);
        const float yb = pjb1(m, 0);
        const int msteps = D.max_steps[m];
        if (t >= 1 && !dn) {
          const float logit = y0 + y1 + yb;
          const float sg = sigm(logit);
          if (t - 1 < D.S_cap) D.stop_out[(long)m * D.S_cap + (t - 1)] = sg;
          const bool st = (sg > P.thr) && (t - 1) > 0;
          if (st || t >= msteps) {
            stci(D.done + m, 1);
            stci(D.steps + m, t);
            stci(D.status + m, st ? 1 : 2);
            dn = 1;
          }
        }
      }
      if (tid < 64) {  // rows still decoding: one ballot over wave 0 (B <= 64), no serial scan
        const unsigned long long act = __ballot(tid < D.B && !dn);
        if (tid == 0) {
          const int last = act ? 63 - __builtin_clzll(act) : -1;
          stci(&D.ctl->all_done, act == 0);
          stci(&D.ctl->active_tiles, last / 16 + 1);
        }
      }
    }
    PTRACE(1);
    BAR_ARRIVE(P.bar, gen);
    // P3 operands that are already final: its epilogue's gate addends (written by P5 of the
    // previous step), c_att, the query-projection weights
    float ga[NCK][4], ca[NCK], wq[4];
    {
      const int idx = min(tid, 4 * CB * 4 - 1);
      const int gl = idx / (CB * 4), rem = idx % (CB * 4);
      const int u = rem & 3;
      const int tile = 4 * min(g, NATT - 1) + gl;
#pragma unroll
      for (int c = 0; c < NCK; ++c) {
        const int m = min(c * CB + (rem >> 2), Bp - 1);
#pragma unroll
        for (int q = 0; q < 4; ++q) ga[c][q] = ldc(P.gatt + (long)m * 4096 + tile * 16 + q * 4 + u);
        ca[c] = P.catt[(long)m * 1024 + tile * 4 + u];
      }
#pragma unroll
      // query-projection B operand: Wq^T rows 16 g + 4 q + (lane >> 4), attention dim 16 wave + (lane & 15)
      for (int q = 0; q < 4; ++q)
        wq[q] = P.WqT[(long)(16 * min(g, NATT - 1) + 4 * q + (lane >> 4)) * 128 + 16 * wave + (lane & 15)];
    }
    // attention_rnn prenet-part weights for P3: 4 tiles per workgroup, waves 2j, 2j+1 = tile j
    // K halves (8 k-chunks each)
    f32x4 wa[ATTP_NC];
    h8 wx[ATTP_NC / 2][2];  // split-f16: k-steps 4 (wave & 1) .. +3 of tile tl, [hi | lo]
    if constexpr (X3P) {
      const int tl = 4 * min(g, NATT - 1) + (wave >> 1);
      const h8* src = reinterpret_cast<const h8*>(P.attp_x3) + (((long)tl * 8 + 4 * (wave & 1)) * 64 + lane) * 2;
#pragma unroll
      for (int i = 0; i < ATTP_NC / 2; ++i) wx[i][0] = src[(long)i * 128], wx[i][1] = src[(long)i * 128 + 1];
    } else {
      const int tl = 4 * min(g, NATT - 1) + (wave >> 1);
      const f32x4* src = reinterpret_cast<const f32x4*>(P.attp_w) + ((long)tl * 16 + 8 * (wave & 1)) * 64 + lane;
#pragma unroll
      for (int i = 0; i < ATTP_NC; ++i) wa[i] = src[(long)i * 64];
    }
    if (!BAR_WAIT(P.bar, gen, &sflag)) return;
    PTRACE(2);
    tid = opaque_v(tid0);
    lane = opaque_v(lane0);
    wave = opaque_s(wave0);
    // loop exit: rows all done, the batch tile shrank (the next launch takes over), or past S_cap.
    // The exit words are a coherent load round trip (~0.5 us) after the barrier; the split-f16
    // attention_rnn workgroups (P3's critical path) evaluate them only after their first staging
    // pass, so that round trip overlaps their operand loads instead of preceding them (nothing
    // before that point writes anything outside LDS)
    const int ex_done = ldci(&D.ctl->all_done), ex_act = ldci(&D.ctl->active_tiles);
    // (the words pass through opaque copies at each test, so the compiler cannot hoist their
    // scalar conversion, and with it the wait for the load, above the operand loads)
    auto p3_exit = [&]() {
      const int done = opaque_v(ex_done), act = opaque_v(ex_act);
      if (done || act < MT || t > D.S_cap + 1) {
        write_frames(t - 1, 0, PW);
        if (g == 0 && tid == 0) {
          D.ctl->base = t;
          if (P.base_out) *P.base_out = t;
        }
        return true;
      }
      return false;
    };
    if (!(X3P && g < NATT) && p3_exit()) return;
    // ======== P3: attention_rnn (prenet part) + cell + query partials (workgroups 0 .. NATT-1)
    //            || frames(t-1) + the decoder_rnn h_dec part (item workgroups) ========
    if (g < NATT) {
      // relu(prenet output) staged once per workgroup in LDS (the Wcomb area: attention_rnn
      // workgroups have no attention item); wave w loads k-chunks 2w, 2w+1
      f32x4 acc[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (X3P) {
        // split-f16 A fragments [MT][8 k-steps][64 lanes][hi | lo]; wave w stages k-step w: lane L
        // holds row L & 15, k = 32 w + 8 (L >> 4) + 0..7, i.e. two fp32 fragments of pb's
        // 16-column chunk 2 w + (L >> 5), lanes l1 and l1 + 16 (frag_idx order)
        // (MT > 2: two passes of 2 m-tiles each, the staging area holds 32 rows)
        h8* xs = reinterpret_cast<h8*>(wcomb);
        const int l1 = 32 * ((lane >> 4) & 1) + (lane & 15);
        bool bad = false;
        // waves 2j, 2j+1: tile 4g + j, K halves (4 k-steps each)
        f32x4 am[MT], ac[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) am[mt] = ac[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ps = 0; ps < NCK; ++ps) {
          if (ps > 0) lds_barrier();  // the previous pass's operand reads are done
          f32x4 xv[CM][2];
#pragma unroll
          for (int mt = ps * CM; mt < min(MT, ps * CM + CM); ++mt) {
            const int c = mt * 16 + 2 * wave + (lane >> 5);
            xv[mt - ps * CM][0] = ldc4(P.pb, (c * 64 + l1) * 16);
            xv[mt - ps * CM][1] = ldc4(P.pb, (c * 64 + l1 + 16) * 16);
          }
          __builtin_amdgcn_sched_barrier(0);
          if (ps == 0 && p3_exit()) return;  // workgroup-uniform; the operand loads are in flight
#pragma unroll
          for (int mt = ps * CM; mt < min(MT, ps * CM + CM); ++mt) {
            const f32x4 x0 = xv[mt - ps * CM][0], x1 = xv[mt - ps * CM][1];
            float v[8];
            float mx = 0.f;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              v[q] = fmaxf(x0[q], 0.f), v[4 + q] = fmaxf(x1[q], 0.f);
              mx = fmaxf(mx, fmaxf(v[q], v[4 + q]));
            }
            bad |= !(mx < F16_RANGE);
            h8 hi, lo;
            split8(v, hi, lo);
            xs[x3i((mt - ps * CM) * 8 + wave, lane, 0)] = hi;
            xs[x3i((mt - ps * CM) * 8 + wave, lane, 1)] = lo;
          }
          lds_barrier();
          PTRACE(13);
#pragma unroll
          for (int i = 0; i < ATTP_NC / 2; ++i) {
            h8 xh[CM], xl[CM];
#pragma unroll
            for (int mt = ps * CM; mt < min(MT, ps * CM + CM); ++mt) {
              const int ks = 4 * (wave & 1) + i;
              xh[mt - ps * CM] = xs[x3i((mt - ps * CM) * 8 + ks, lane, 0)];
              xl[mt - ps * CM] = xs[x3i((mt - ps * CM) * 8 + ks, lane, 1)];
            }
#pragma unroll
            for (int mt = ps * CM; mt < min(MT, ps * CM + CM); ++mt)
              mfma_x3(xh[mt - ps * CM], xl[mt - ps * CM], wx[i][0], wx[i][1], am[mt], ac[mt]);
          }
        }
        if (bad) __hip_atomic_fetch_or(P.x3flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[mt][j] = x3_value(am[mt][j], ac[mt][j]);
      } else {
        f32x4* xs = reinterpret_cast<f32x4*>(wcomb);  // [CM * 16 chunks][64 lanes] per pass
#pragma unroll
        for (int ps = 0; ps < NCK; ++ps) {
          if (ps > 0) lds_barrier();
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int mt = ps * CM; mt < min(MT, ps * CM + CM); ++mt) {
              const int c = mt * 16 + 2 * wave + i;
              f32x4 x = ldc4(P.pb, (c * 64 + lane) * 16);
#pragma unroll
              for (int q = 0; q < 4; ++q) x[q] = fmaxf(x[q], 0.f);
              xs[(c - ps * CM * 16) * 64 + lane] = x;
            }
          lds_barrier();
          PTRACE(13);
          // waves 2j, 2j+1: tile 4g + j, K halves (8 chunks each)
#pragma unroll
          for (int i = 0; i < ATTP_NC; ++i) {
            f32x4 x[CM];
#pragma unroll
            for (int mt = ps * CM; mt < min(MT, ps * CM + CM); ++mt)
              x[mt - ps * CM] = xs[((mt - ps * CM) * 16 + 8 * (wave & 1) + i) * 64 + lane];
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
              for (int mt = ps * CM; mt < min(MT, ps * CM + CM); ++mt)
                acc[mt] = MFMA16(x[mt - ps * CM][q], wa[i][q], acc[mt]);
          }
        }
      }
      PTRACE(10);
#pragma unroll
      for (int ck = 0; ck < NCK; ++ck) {
        acc_chunk_to_lds<MT, CM>(red0 + (wave >> 1) * 2 * CB * RS, wave & 1, lane, acc, ck);
        lds_barrier();
        if (tid < 4 * CB * 4) {
          const int gl = tid / (CB * 4), rem = tid % (CB * 4);
          const int m = ck * CB + (rem >> 2), u = rem & 3;
          const int tile = 4 * g + gl;
          const float* pg = red0 + gl * 2 * CB * RS;
          if (m < Bp) {
            float pre[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) pre[q] = lds_sum<2, CB>(pg, rem >> 2, q * 4 + u) + ga[ck][q];
            const long ci = (long)m * 1024 + tile * 4 + u;
            const float c = sigm_f(pre[1]) * ca[ck] + sigm_f(pre[0]) * tanh_f(pre[2]);
            const float h = sigm_f(pre[3]) * tanh_f(c);
            P.catt[ci] = c;
            stc_quad_h<PS>(P.hatt, (int)frag_idx(m, tile * 4 + u, 1024), h);
            hs[m * 17 + gl * 4 + u] = h;
          }
        }
        lds_barrier();
      }
      PTRACE(11);
      if (!GRAVES) {  // partial query projection over this workgroup's 16 units
        // on the MFMA: wave w owns attention dims 16 w .. 16 w + 15, K = this workgroup's 16 units.
        // Transposed product (dims x rows): a lane ends with 4 consecutive dims of one batch row,
        // stored as one 16-byte write (the partials are the step's largest hand-off, 16 KB per
        // workgroup)
        f32x4 qa[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) qa[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
            qa[mt] = MFMA16(wq[q], hs[(mt * 16 + (lane & 15)) * 17 + 4 * q + (lane >> 4)], qa[mt]);
#ifdef TTS_PQ_NARROW
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int j = 0; j < 4; ++j) stc(P.pq + ((long)g * Bp + mt * 16 + (lane & 15)) * 128 + 16 * wave + 4 * (lane >> 4) + j, qa[mt][j]);
#else
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          stc4(P.pq, (((g * Bp + mt * 16 + (lane & 15)) * 128) + 16 * wave + 4 * (lane >> 4)) * 4, qa[mt]);
#endif
      }
      PTRACE(12);
    } else {
      dec_hdec_part(hd_cur);
      write_frames(t - 1, NATT, PW - NATT);
    }
    PTRACE(3);
    BAR_ARRIVE(P.bar, gen);
    if (!BAR_WAIT(P.bar, gen, &sflag)) return;
    if constexpr (GRAVES) {
      // ======== P3g: N_a hidden = relu(W1 h_att + b1), 16 units per workgroup IW0 .. IW0+63 ========
      tid = opaque_v(tid0);
      lane = opaque_v(lane0);
      wave = opaque_s(wave0);
      const int gt = g - IW0;
      if (gt >= 0 && gt < 64) {
        f32x4 wn[8];
        const f32x4* src = reinterpret_cast<const f32x4*>(P.na1_w) + ((long)gt * 64 + 8 * wave) * 64 + lane;
#pragma unroll
        for (int i = 0; i < 8; ++i) wn[i] = src[(long)i * 64];
        f32x4 acc[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        gemm_seg<MT, 8, 2>(acc, P.hatt, 64, 8 * wave, lane, [&](int i) { return wn[i]; });
#pragma unroll
        for (int ck = 0; ck < NCK; ++ck) {
          acc_chunk_to_lds<MT, CM>(red0, wave, lane, acc, ck);
          lds_barrier();
          for (int idx = tid; idx < CB * 16; idx += PT) {
            const int m = ck * CB + (idx >> 4), n = idx & 15;
            if (m >= Bp) break;
            const float v = lds_sum<NWV, CB>(red0, idx >> 4, n) + P.na1_b[gt * 16 + n];
            stc(P.gh + (long)m * 1024 + gt * 16 + n, fmaxf(v, 0.f));
          }
          lds_barrier();
        }
      }
      BAR_ARRIVE(P.bar, gen);
      if (!BAR_WAIT(P.bar, gen, &sflag)) return;
    }
    PTRACE(4);
    // ======== P4: attention || the h_att parts of decoder_rnn and attention_rnn ========
    tid = opaque_v(tid0);
    lane = opaque_v(lane0);
    wave = opaque_s(wave0);
    {
      // The h_att parts run AFTER this workgroup's attention item: fp32 MFMA occupies the SIMD
      // (no co-issue with the attention's VALU work on the other wave), so under the item they
      // only lengthen the attention chain; after it they overlap the other items' tails.
      if (g >= IW0) {  // items, then the decoder_rnn h_att part (attention_rnn's waits for P6)
        PTRACE(15);
        const int nitems = D.B * P.nchmax;
        for (int it = g - IW0, k = 0; it < nitems; it += PW - IW0, ++k) {
          if (k == 0) PTRACE(14);
          float* ek = nullptr;
          if (DEFER && P.defer_align) {
            ek = ekeep0 + k * (PTC + 1);
            if (tid == 0) ek[PTC] = 0.f;  // set by the item when its utterance is still decoding
          }
          if constexpr (GRAVES) graves_item<MT>(P, t, it / P.nchmax, it % P.nchmax, scr, &is_last);
          else pattn_item<MT, VAR>(P, t, it / P.nchmax, it % P.nchmax, it < PW - IW0 ? T_first : D.lens[it / P.nchmax],
                                   scr, wcomb, &is_last, Lr, it < PW - IW0, evc, nitems > PW - IW0 || t == t_first, ek);
          lds_barrier();
        }
        // split-f16: the h_att part runs at the start of P5 instead (h_att is still in place), off
        // the chain of the utterances' last arrivers, whose combine and alignment pass end P4
        if constexpr (!X3P) gemm_seg<MT, 8, 2>(accd, P.hatt, 64, 8 * wave, lane, [&](int i) { return wd[i]; });
      } else {  // no item: both h_att parts and the decoder_rnn h_dec part
        if constexpr (X3P)
          X3_PASSES(MT, (gemm_x3_pair<NM, 4, PS>(msub<MO, NM>(accd), msub<MO, NM>(acca), P.hatt + MO * 64 * 256, 64,
                                             4 * wave, lane, wdx_f(0), wap_f(16 + 4 * wave))));
        else
          gemm_seg2<MT, 8, 2>(accd, acca, P.hatt, 64, 8 * wave, lane, [&](int i) { return wd[i]; },
                              [&](int i) { return Wap[(32 + 8 * wave + i) * 64 + lane]; });
        dec_hdec_part(hd_cur);
      }
    }
    PTRACE(5);
    BAR_ARRIVE(P.bar, gen);
    // P5 epilogue operand (own tile's c_dec), fetched during the barrier
    float cd[NCK];
#pragma unroll
    for (int c = 0; c < NCK; ++c) cd[c] = P.cdec[(long)min(c * CB + (tid >> 2), Bp - 1) * 1024 + g * 4 + (tid & 3)];
    if (!BAR_WAIT(P.bar, gen, &sflag)) return;
    PTRACE(6);
    // ======== P5: ctx parts, then the decoder_rnn cell (tile g) and the next step's
    //            attention_rnn ctx/h part (tile g, + biases) ========
    tid = opaque_v(tid0);
    lane = opaque_v(lane0);
    wave = opaque_s(wave0);
    {
      if constexpr (X3P) {
        if (g >= IW0)  // + both h_att parts (moved here from P4 / P6: h_att read once per step)
          X3_PASSES(MT, (gemm_x3_hatt_ctx<NM, 4, 2, PS>(msub<MO, NM>(accd), msub<MO, NM>(acca), P.hatt + MO * 64 * 256, 64,
                                                    4 * wave, P.ctx + MO * 32 * 256, 32, 2 * wave, lane, wdx_f(0),
                                                    wap_f(16 + 4 * wave), wdx_f(4), wap_f(2 * wave))));
        else
          X3_PASSES(MT, (gemm_x3_pair<NM, 2, PS>(msub<MO, NM>(accd), msub<MO, NM>(acca), P.ctx + MO * 32 * 256, 32,
                                             2 * wave, lane, wdx_f(4), wap_f(2 * wave))));
      }
      else
        gemm_seg2<MT, 4, 4>(accd, acca, P.ctx, 32, 4 * wave, lane, [&](int i) { return wd[8 + i]; },
                            [&](int i) { return Wap[(4 * wave + i) * 64 + lane]; });
      float* red1 = red0;  // two reductions back to back: [2][8][Bp][17] would not fit; reuse
#pragma unroll
      for (int ck = 0; ck < NCK; ++ck) {
        acc_chunk_to_lds<MT, CM>(red0, wave, lane, accd, ck);
        lds_barrier();
        const int m = ck * CB + (tid >> 2), u = tid & 3;
        if (tid < CB * 4 && m < Bp) {
          float pre[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) pre[q] = lds_sum<NWV, CB>(red0, tid >> 2, q * 4 + u) + db[ck][q];
          if (sscale) {
            const float sa = spk_sum(m);
#pragma unroll
            for (int q = 0; q < 4; ++q) pre[q] += sa * P.spk_dec[(long)m * P.spk_ld + g * 16 + q * 4 + u];
          }
          const long ci = (long)m * 1024 + g * 4 + u;
          const float c = sigm_f(pre[1]) * cd[ck] + sigm_f(pre[0]) * tanh_f(pre[2]);
          const float h = sigm_f(pre[3]) * tanh_f(c);
          P.cdec[ci] = c;
          stc_quad_h<PS>(hd_nxt, (int)frag_idx(m, g * 4 + u, 1024), h);
        }
        lds_barrier();
      }
      if (g < IW0) att_epilogue(red1);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) accd[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    PTRACE(7);
    BAR_ARRIVE(P.bar, gen);
    // projection weights for P6 (half pj & 1 of job tile pj >> 1, 6 k-chunks per wave)
    f32x4 wp[X3P ? 1 : PJ_NC];
    h8 wpx[X3P ? PJ_NC : 1][2];  // split-f16: the whole K for 16 rows, k-steps 6 wave .. + 5
    {
      const int q = min(max(pj, 0) / JR, P.ntj - 1), half = pj & 1;
      if constexpr (X3P) {
        (void)half;
        const h8* src = reinterpret_cast<const h8*>(P.pj_x3) + (((long)q * 48 + 6 * wave) * 64 + lane) * 2;
#pragma unroll
        for (int i = 0; i < PJ_NC; ++i) wpx[i][0] = src[(long)i * 128], wpx[i][1] = src[(long)i * 128 + 1];
      } else {
        const f32x4* src = reinterpret_cast<const f32x4*>(P.pj_w) + ((long)q * 96 + 48 * half + wave * PJ_NC) * 64 + lane;
#pragma unroll
        for (int i = 0; i < PJ_NC; ++i) wp[i] = src[(long)i * 64];
      }
    }
    if (!BAR_WAIT(P.bar, gen, &sflag)) return;
    PTRACE(8);
    // ======== P6: projection halves (workgroups PJ_WG0 ..) || attention_rnn h_att part (items) ========
    tid = opaque_v(tid0);
    lane = opaque_v(lane0);
    wave = opaque_s(wave0);
    if (X3P && is_pj && (pj % JR) < MT) {
      // split-f16: job pj = (tile pj / JR, batch rows 16 (pj % JR) .. + 15), the whole K, so ypart
      // holds one copy (P1, the stop decision and the frame writes read it once)
      const int mtb = pj % JR;
      f32x4 y[PJ_NC][1][2];
#pragma unroll
      for (int i = 0; i < PJ_NC; ++i) {
        const int ks = 6 * wave + i;
        if (ks < 32) ld_x3_step<1>(y[i], hd_nxt + (long)mtb * 64 * 256, 64, ks, lane);
        else ld_x3_step<1>(y[i], P.ctx + (long)mtb * 32 * 256, 32, ks - 32, lane);
      }
      f32x4 am = f32x4{0.f, 0.f, 0.f, 0.f}, ac = am;
#pragma unroll
      for (int i = 0; i < PJ_NC; ++i) {
        h8 xh, xl;
        split_x3_step<PS>(y[i][0], xh, xl);
        mfma_x3(xh, xl, wpx[i][0], wpx[i][1], am, ac);
      }
      float* p = red0 + wave * 16 * RS;  // [wave][16 rows][RS]
#pragma unroll
      for (int j = 0; j < 4; ++j) p[(4 * (lane >> 4) + j) * RS + (lane & 15)] = x3_value(am[j], ac[j]);
      lds_barrier();
      if (tid < 256) {
        const int mm = tid >> 4, n = tid & 15;
        float v = red0[mm * RS + n];
#pragma unroll
        for (int w = 1; w < NWV; ++w) v += red0[(w * 16 + mm) * RS + n];
        stc_quad(P.ypart, (mtb * 16 + mm) * YP + (pj / JR) * 16 + n, v);
      }
      lds_barrier();
    } else if (!X3P && is_pj) {
      f32x4 acc2[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc2[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kb = 48 * (pj & 1) + wave * PJ_NC;  // K = [h_dec 1024 | ctx 512]
      {
        f32x4 y[PJ_NC][MT];
#pragma unroll
        for (int i = 0; i < PJ_NC; ++i) {
          const int kc = kb + i;
          const float* base = kc < 64 ? hd_nxt : P.ctx;
          const int kl = kc < 64 ? kc : kc - 64;
          const int nk = kc < 64 ? 64 : 32;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) y[i][mt] = ldc4<ACT_AUX>(base, ((mt * nk + kl) * 64 + lane) * 16);
        }
#pragma unroll
        for (int i = 0; i < PJ_NC; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc2[mt] = MFMA16(y[i][mt][q], wp[i][q], acc2[mt]);
      }
#pragma unroll
      for (int ck = 0; ck < NCK; ++ck) {
        acc_chunk_to_lds<MT, CM>(red0, wave, lane, acc2, ck);
        lds_barrier();
        for (int idx = tid; idx < CB * 16; idx += PT) {
          const int m = ck * CB + (idx >> 4), n = idx & 15;
          if (m >= Bp) break;
          stc(P.ypart + (long)((pj & 1) * YROWS + m) * YP + (pj >> 1) * 16 + n, lds_sum<NWV, CB>(red0, idx >> 4, n));
        }
        lds_barrier();
      }
    }
    if (g >= IW0) {  // item workgroups: attention_rnn h_att part (h_att of step t is still in place)
      if constexpr (!X3P)  // split-f16: done in P5 beside the decoder_rnn h_att part
        gemm_seg<MT, 8, 2>(acca, P.hatt, 64, 8 * wave, lane, [&](int i) { return Wap[(32 + 8 * wave + i) * 64 + lane]; });
      att_epilogue(red0);
      if (DEFER && P.defer_align) {
        // deferred alignment pass (common_layers.py:347-357): this workgroup's items of step t, their
        // own positions; S and m came from each utterance's last arriver in P4. Off the step's
        // critical path: the item workgroups' P6 is short beside the projection jobs.
        const int nitems = D.B * P.nchmax;
        for (int it = g - IW0, k = 0; it < nitems; it += PW - IW0, ++k) {
          const float* ek = ekeep0 + k * (PTC + 1);
          const int b = it / P.nchmax, p0 = (it % P.nchmax) * PTC;
          const int T = D.lens[b];
          if (ek[PTC] == 0.f || tid >= min(PTC, T - p0)) continue;
          const long ab = (long)b * D.T_max + p0 + tid;
          const float S = ldc(P.anorm + 2 * b), m = ldc(P.anorm + 2 * b + 1);
          const float e = ek[tid];
          const float raw = P.softmax ? (e == -INFINITY ? 0.f : expf(e - m)) : 1.f / (1.f + expf(-e));
          const float al = raw / S;
          stc(P.acum + ab, ldc(P.acum + ab) + al);
          stc(P.alpha + ab, al);
          if (t < D.S_cap) D.align_out[((long)b * D.S_cap + t) * D.T_max + p0 + tid] = al;
        }
      }
    }
    PTRACE(9);
    BAR_ARRIVE(P.bar, gen);
    if (!BAR_WAIT(P.bar, gen, &sflag)) return;
  }
}

// host side ------------------------------------------------------------------------------
bool persist_supported(int device) {
  int cus = 0, coop = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, device) != hipSuccess) return false;
  return cus == PW && coop;
}

int persist_attn_tc() { return PTC; }

// ---- barrier-block placement (tools/bar_bench.hip placement sweep): the same flag barrier costs
// 1.53-1.58 or 1.78-1.92 us depending on where its 4 KiB block lies (alternating with address bit 13
// at 8 KiB steps; 2.15 against 2.32 us with a hand-off), i.e. on which memory stack the words sit
// relative to the releasing workgroup's XCD. The decoder saw it as a per-process 25.8 / 27.2 us
// step. Candidate blocks are timed once per workspace and the fastest serve the launches.
namespace {
__global__ __launch_bounds__(PT) void gflag_cal_kernel(unsigned* bar, int iters) {
  __shared__ int flag;
  unsigned gen = 0;
  for (int i = 0; i < iters; ++i) {
    gflag_arrive(bar, gen);
    if (!gflag_wait(bar, gen, &flag)) return;
  }
}
}  // namespace

void pick_barrier_blocks(unsigned* pool, int ncand, int nwant, int* slot, hipStream_t s) {
  for (int i = 0; i < nwant; ++i) slot[i] = i;
  const char* e = std::getenv("TTS_BAR_CALIBRATE");
  if ((e && std::atoi(e) == 0) || ncand <= nwant) return;
  const void* f = (const void*)gflag_cal_kernel;
  ensure_dyn_lds(f, (int)P_LDS);  // one workgroup per CU, as the decoder
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  std::vector<std::pair<float, int>> t;
  int iters = 200;
  for (int k = 0; k < ncand; ++k) {
    unsigned* b = pool + (size_t)k * BAR_WORDS;
    float best = 1e30f;
    for (int rep = 0; rep < 2; ++rep) {
      arm_barrier(b, 1, s);
      void* args[] = {&b, &iters};
      HIP_OK(hipEventRecord(e0, s));
      launch_resident(f, dim3(PW), dim3(PT), args, P_LDS, s);
      HIP_OK(hipEventRecord(e1, s));
      HIP_OK(hipEventSynchronize(e1));
      float ms = 0.f;
      HIP_OK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
    }
    unsigned err = 0;
    HIP_OK(hipMemcpy(&err, b + 16, 4, hipMemcpyDeviceToHost));
    if (err != 0) {  // not co-resident (another kernel on the device): keep the default blocks 0..nwant-1;
      HIP_OK(hipEventDestroy(e0));  // the decode's own barrier check reports a real residency failure
      HIP_OK(hipEventDestroy(e1));
      std::fprintf(stderr, "tts_amd: barrier-block calibration timed out; using the default blocks\n");
      return;
    }
    t.push_back({best, k});
  }
  HIP_OK(hipEventDestroy(e0));
  HIP_OK(hipEventDestroy(e1));
  std::stable_sort(t.begin(), t.end());
  for (int i = 0; i < nwant; ++i) slot[i] = t[i].second;
  if (std::getenv("TTS_DIAG_XCC")) {
    std::fprintf(stderr, "TTS_DIAG_XCC barrier blocks (us per barrier):");
    for (auto& x : t) std::fprintf(stderr, " %d:%.3f", x.second, x.first * 1000.f / iters);
    std::fprintf(stderr, "\n");
  }
}
#ifdef TTS_PHASE_TRACE
bool persist_trace_built() { return true; }
#else
bool persist_trace_built() { return false; }
#endif
bool persist_defer_ok(int nitems) { return nitems <= (PW - IW0) * PDEF_MAXIT; }

static int persist_var(const PArgs& a) {
  return (a.gK > 0 ? 4 : (a.win ? 1 : 0) | (a.fwd ? 2 : 0)) | (a.attp_x3 ? 8 : 0);
}
bool persist_presplit(const PArgs& a) { return presplit_of(persist_var(a)); }

void launch_persist_decoder(const PArgs& a, int MT, hipStream_t s, bool arm, hipEvent_t ev0, hipEvent_t ev1) {
  TTS_CHECK(MT >= 1 && MT <= 4, "persistent decoder: MT must be in [1, 4]");
  TTS_CHECK(PJ_WG0 + a.ntj * (MT > 2 ? 4 : 2) <= PW && a.ntj >= 17, "persistent decoder: projection job count");
  TTS_CHECK(a.D.B <= 64 && NATT * 4 * 4 == 1024, "persistent decoder: attention_rnn layout");
  TTS_CHECK(a.nchmax * PTC >= a.D.T_max, "persistent decoder: attention partial buffers too small");
  TTS_CHECK(a.D.B <= 16 * MT, "persistent decoder: rows beyond the batch tile");
  // decoder variants are compiled in only where used: VAR bit 0 windowing, bit 1 forward attention
  // (bit 2: Graves attention, exclusive of the others); bit 3: split-f16 P3 (attp_x3 given)
  TTS_CHECK(!a.attp_x3 || (a.x3flag && a.dec_x3 && a.apre_x3 && a.pj_x3),
            "persistent decoder: split-f16 weights incomplete or without a range flag");
  const int var = persist_var(a);
#define PDK(mt, v) (const void*)persist_decoder_kernel<mt, v>
#define PDK_ROW(mt) \
  {PDK(mt, 0), PDK(mt, 1), PDK(mt, 2), PDK(mt, 3), PDK(mt, 4), nullptr, nullptr, nullptr, PDK(mt, 8), PDK(mt, 9), \
   PDK(mt, 10), PDK(mt, 11), PDK(mt, 12)}
  static const void* const fns[4][13] = {PDK_ROW(1), PDK_ROW(2), PDK_ROW(3), PDK_ROW(4)};
#undef PDK_ROW
#undef PDK
  const void* f = fns[MT - 1][var];
  TTS_CHECK(f != nullptr, "persistent decoder: variant");
  ensure_dyn_lds(f, (int)P_LDS);
  if (arm) arm_barrier(a.bar, 1, s);
  PArgs copy = a;
  void* kargs[] = {&copy};
  launch_resident(f, dim3(PW), dim3(PT), kargs, P_LDS, s, ev0, ev1);
}
