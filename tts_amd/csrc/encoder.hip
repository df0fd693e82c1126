// Tacotron2 encoder pieces that are not convolutions (gfx950):
//  * embedding gather  (TTS/tts/models/tacotron2.py:61,144)
//  * BiLSTM recurrence (TTS/tts/layers/tacotron2.py:91-96,116-118, nn.LSTM bidirectional,
//    no packing at inference). The input projection x.W_ih^T + b_ih + b_hh for both directions
//    runs beforehand as one MFMA conv (K=1, Cout=2048); the step kernel below does the T
//    sequential steps with per-utterance lengths: the reverse direction starts at T_b - 1, never
//    in the padding (a padded reverse pass differs by 0.29 L-inf).
#include "common.h"
#include "decoder.h"  // frag_idx
#include "gsync.h"
#include "split16.h"

// row stride of the LDS gate-partial reductions [wave][row][LRS]: writers put rows r and r + 4 of a
// 32-lane group 80 = 16 (mod 32) banks apart, the cell threads read rows m = tid / 4 (8 per group)
// at columns 4 q + (tid & 3): 20 m mod 32 = {0, 20, 8, 28, 16, 4, 24, 12} + 0..3, no two alike
// (stride 17 put 2 lanes on one bank: 2-way conflicts on every read of the reduction)
constexpr int LRS = 20;

__global__ __launch_bounds__(256) void embed_gather_kernel(const int64_t* __restrict__ ids, int T_max,
                                                           const float* __restrict__ table, int num_rows,
                                                           int D, const int* lens, const int* rowmap,
                                                           float* __restrict__ out /* (B,T_max,D) */) {
  const int b = blockIdx.y, t = blockIdx.x;
  float* o = out + ((long)b * T_max + t) * D;
  const bool valid = t < lens[b];
  const long ib = rowmap ? rowmap[b] : b;  // ids row of output row b (the decode order's map)
  long id = valid ? ids[ib * T_max + t] : 0;
  if (id < 0 || id >= num_rows) id = 0;  // host validates ids; never read out of bounds
  for (int c = threadIdx.x; c < D; c += blockDim.x) o[c] = valid ? table[id * D + c] : 0.f;
}

// rowmap (optional, device): output row b takes ids row rowmap[b] (lens are in output order)
void launch_embed_gather(const int64_t* ids, int T_max, const float* table, int num_rows, int D,
                         const int* lens, int B, float* out, hipStream_t s, const int* rowmap) {
  if (B <= 0 || T_max <= 0) return;
  embed_gather_kernel<<<dim3(T_max, B), 256, 0, s>>>(ids, T_max, table, num_rows, D, lens, rowmap, out);
  HIP_OK(hipGetLastError());
}

// One BiLSTM time step for every utterance and both directions. The recurrent GEMM
// gates = h W_hh^T runs on MFMA over all B utterances at once (M = 16-row batch tiles), split by
// hidden units across 128 workgroups: workgroup (dir, tile) owns 4 hidden units = the i, f, g, o
// rows of one 16-row tile (gate-interleaved like the decoder LSTMs), so the cell update is its
// epilogue and W_hh is spread over the chip instead of streamed by one CU per utterance. One
// launch per step; h ping-pongs between two fragment-order buffers.
//   Whh : per dir, gate-interleaved tiles, swizzled [64 tiles][16 k-chunks][64 lanes][4]
//   Gin : (B, T_max, 2048) x W_ih^T + b_ih + b_hh, columns [dir][tile][gate][unit]
//   h   : [dir][Bp x 256] fragment order (frag_idx), c: [dir][Bp][256]
//   out : (B, T_max, 512) = [fwd h | bwd h]
template <int MT>
__global__ __launch_bounds__(256) void bilstm_step_kernel(const float* __restrict__ Whh,
                                                          const float* __restrict__ Gin, const int* lens,
                                                          int T_max, int B, int step,
                                                          const float* __restrict__ h_in, float* __restrict__ h_out,
                                                          float* __restrict__ c, float* __restrict__ out) {
  constexpr int Bp = MT * 16;
  constexpr int H = 256, NKC = H / 16, KPW = NKC / 4;  // 4 k-chunks per wave
  __shared__ float part[4 * Bp * LRS];
  const int dir = blockIdx.x >> 6, tl = blockIdx.x & 63;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const f32x4* Wv = reinterpret_cast<const f32x4*>(Whh) + ((long)(dir * 64 + tl) * NKC + wave * KPW) * 64 + lane;
  const float* hx = h_in + (long)dir * Bp * H + (long)(wave * KPW) * 256 + 4 * lane;
  f32x4 w[KPW], x[KPW][MT];
#pragma unroll
  for (int k = 0; k < KPW; ++k) {
    w[k] = Wv[(long)k * 64];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) x[k][mt] = *reinterpret_cast<const f32x4*>(hx + (long)mt * 16 * H + k * 256);
  }
  // epilogue operands (clamped indices; validity applied at the stores)
  const int m = min(tid >> 2, Bp - 1), u = tid & 3;
  const int Tm = lens[min(m, B - 1)];
  const bool valid = (tid >> 2) < Bp && m < B && step < Tm;
  const int t = min(max(dir ? Tm - 1 - step : step, 0), T_max - 1);
  const float* gp = Gin + ((long)min(m, B - 1) * T_max + t) * 2048 + dir * 1024 + tl * 16 + u;
  float gin[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) gin[q] = gp[q * 4];
  const long ci = ((long)dir * Bp + m) * H + tl * 4 + u;
  const float cprev = c[ci];
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < KPW; ++k)
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = MFMA16(x[k][mt][s4], w[k][s4], acc[mt]);
  float* p = part + wave * Bp * LRS;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) p[(mt * 16 + 4 * (lane >> 4) + j) * LRS + (lane & 15)] = acc[mt][j];
  __syncthreads();
  if (!valid) return;
  float pre[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n = q * 4 + u;
    pre[q] = part[m * LRS + n] + part[(Bp + m) * LRS + n] + part[(2 * Bp + m) * LRS + n] + part[(3 * Bp + m) * LRS + n] +
             gin[q];
  }
  const float ig = 1.f / (1.f + expf(-pre[0]));
  const float fg = 1.f / (1.f + expf(-pre[1]));
  const float gg = tanhf(pre[2]);
  const float og = 1.f / (1.f + expf(-pre[3]));
  const float cn = fg * cprev + ig * gg;
  const float hn = og * tanhf(cn);
  c[ci] = cn;
  h_out[(long)dir * Bp * H + frag_idx(m, tl * 4 + u, H)] = hn;
  out[((long)m * T_max + t) * 512 + dir * 256 + tl * 4 + u] = hn;
}

// The whole recurrence as ONE cooperative launch: workgroup (dir, tile) owns gate tile `tile` (4
// hidden units, gate-interleaved) of direction dir; its W_hh fragments stay in VGPRs, the cell
// state in a register of the thread that owns (row, unit), and a hierarchical grid barrier
// (gsync.h) per direction replaces the launch boundary between steps (per-step launches were
// host-enqueue bound at ~8 us per step). Used by the Tacotron2 encoder BiLSTM (H = 256, 2
// directions) and the GE2E speaker encoder LSTMs (H = 768, 1 direction).
//   Whh : [dir][H/4 tiles][H/16 k-chunks][64 lanes][4]   Gin : (B, T_max, NDIR*4H) incl. biases
//   hbuf: [2 ping-pong][dir][Bp x H] fragment order      out : (B, T_max, NDIR*H)
//   Whh16 (X3): the same tiles split-f16 (split16.h pack_split_a, [dir * H/4 + tile][H/32][64][16]);
//   h is loaded from the fp32 fragment buffer and split in registers (|h| <= 1: always in range)
// Row groups (RG > 1, round 4): the batch rows split into RG independent recurrences of MT tiles
// each, on RG x NDIR x NT workgroups (the encoder BiLSTM at B = 17..64: 2 x 2 x 64 = every CU),
// each group with its own h buffers and barrier: half the rows per step on every workgroup.
//   hbuf: [2 ping-pong][RG][dir][Bp x H]
constexpr int LSTM_NW = 8;  // waves per workgroup: the K = H reduction split 8 ways
template <int MT, int H, int NDIR, bool X3>
__global__ __launch_bounds__(64 * LSTM_NW) void lstm_persist_kernel(const float* __restrict__ Whh,
                                                           const uint16_t* __restrict__ Whh16,
                                                           const float* __restrict__ Gin, const int* lens,
                                                           int T_max, int B, float* hbuf, float* __restrict__ out,
                                                           unsigned* bar, int stall) {
  constexpr int Bp = MT * 16;
  constexpr int NT = H / 4;                   // gate tiles per direction
  constexpr int NW = LSTM_NW;
  constexpr int NKC = H / 16, KPW = NKC / NW;  // k-chunks, per wave
  constexpr int G = NDIR * 4 * H, O = NDIR * H;
  static_assert(NKC % NW == 0 && KPW % 2 == 0 && NT % 8 == 0 && NT <= 256, "LSTM geometry (gflag groups of <= 256)");
  __shared__ float part[NW * Bp * LRS];
  __shared__ int sflag;
  const int RG = gridDim.x / (NDIR * NT);      // row groups (the launcher sizes the grid)
  const int rg = blockIdx.x / (NDIR * NT);
  const int dir = (blockIdx.x / NT) % NDIR, tl = blockIdx.x % NT;
  const int dom = rg * NDIR + dir;             // this workgroup's recurrence: h buffers and barrier
  const int r0 = rg * Bp;                      // its first batch row
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int KSW = KPW / 2;  // split-f16 k-steps (32) per wave
  f32x4 w[X3 ? 1 : KPW];
  h8 wx[X3 ? KSW : 1][2];
  if constexpr (X3) {
    const h8* Wv = reinterpret_cast<const h8*>(Whh16) + (((long)(dir * NT + tl) * (H / 32) + wave * KSW) * 64 + lane) * 2;
#pragma unroll
    for (int k = 0; k < KSW; ++k) wx[k][0] = Wv[(long)k * 128], wx[k][1] = Wv[(long)k * 128 + 1];
  } else {
    const f32x4* Wv = reinterpret_cast<const f32x4*>(Whh) + ((long)(dir * NT + tl) * NKC + wave * KPW) * 64 + lane;
#pragma unroll
    for (int k = 0; k < KPW; ++k) w[k] = Wv[(long)k * 64];
  }
  const int m = min(tid >> 2, Bp - 1), u = tid & 3;
  const int ma = r0 + m;  // absolute batch row
  const bool row = (tid >> 2) < Bp && ma < B;
  const int Tm = lens[min(ma, B - 1)];
  const float* gbase = Gin + (long)min(ma, B - 1) * T_max * G + dir * 4 * H + tl * 16 + u;
  float cst = 0.f;
  unsigned gen = 0;
  // input-projection gates of a step do not depend on h: loaded one step ahead, under the barrier
  auto tpos = [&](int step) { return min(max(dir ? Tm - 1 - step : step, 0), T_max - 1); };
  float gin[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) gin[q] = gbase[(long)tpos(0) * G + q * 4];
  for (int step = 0; step < T_max; ++step) {
    // test hook (tts_test_stall_lstm(<recurrence>)): one workgroup of that recurrence leaves before
    // its second barrier, so the others time out and set that recurrence's error word
    if (step == 1 && dom == stall && tl == 0) return;
    const float* hi = hbuf + (size_t)(step & 1) * RG * NDIR * Bp * H + (long)dom * Bp * H;
    float* ho = hbuf + (size_t)((step + 1) & 1) * RG * NDIR * Bp * H + (long)dom * Bp * H;
    const int t = tpos(step);
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (X3) {
      // k-step ks: lane L holds row L & 15, k = 32 ks + 8 (L >> 4) + 0..7 = fp32 fragment chunk
      // 2 ks + (L >> 5), lanes l1 and l1 + 16 (frag_idx order)
      const int l1 = 32 * ((lane >> 4) & 1) + (lane & 15);
      f32x4 x[KSW][MT][2];
#pragma unroll
      for (int k = 0; k < KSW; ++k)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int c = mt * NKC + 2 * (wave * KSW + k) + (lane >> 5);
          x[k][mt][0] = ldc4(hi, (c * 64 + l1) * 16);
          x[k][mt][1] = ldc4(hi, (c * 64 + l1 + 16) * 16);
        }
      f32x4 am[MT], ac[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) am[mt] = ac[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KSW; ++k)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          // h was published pre-split (stc_quad_x3): k 0..3 as [hi | lo] in x[..][0], k 4..7 in x[..][1]
          const f32x4 &a = x[k][mt][0], &b = x[k][mt][1];
          const h8 xh = __builtin_bit_cast(h8, (f32x4{a[0], a[1], b[0], b[1]}));
          const h8 xl = __builtin_bit_cast(h8, (f32x4{a[2], a[3], b[2], b[3]}));
          mfma_x3(xh, xl, wx[k][0], wx[k][1], am[mt], ac[mt]);
        }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[mt][j] = x3_value(am[mt][j], ac[mt][j]);
    } else {
      f32x4 x[KPW][MT];
#pragma unroll
      for (int k = 0; k < KPW; ++k)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) x[k][mt] = ldc4(hi, ((mt * NKC + wave * KPW + k) * 64 + lane) * 16);
#pragma unroll
      for (int k = 0; k < KPW; ++k)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[mt] = MFMA16(x[k][mt][s4], w[k][s4], acc[mt]);
    }
    float* p = part + wave * Bp * LRS;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) p[(mt * 16 + 4 * (lane >> 4) + j) * LRS + (lane & 15)] = acc[mt][j];
    lds_barrier();
    if (row && step < Tm) {
      float pre[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = q * 4 + u;
        float sum = part[m * LRS + n];
#pragma unroll
        for (int w = 1; w < NW; ++w) sum += part[(w * Bp + m) * LRS + n];
        pre[q] = sum + gin[q];
      }
      cst = sigm_f(pre[1]) * cst + sigm_f(pre[0]) * tanh_f(pre[2]);
      const float hn = sigm_f(pre[3]) * tanh_f(cst);
      // lanes u = 0..3 of a quad: one 16-byte store (split-f16: pre-split, the consumers' MFMA operands)
      if constexpr (X3) stc_quad_x3(ho, (int)frag_idx(m, tl * 4 + u, H), hn);
      else stc_quad(ho, (int)frag_idx(m, tl * 4 + u, H), hn);
      out[((long)ma * T_max + t) * O + dir * H + tl * 4 + u] = hn;
    }
    if (step + 1 < T_max) {  // directions and row groups are independent: one barrier each
      unsigned* db = bar + dom * BAR_WORDS;
      // the recurrence's NT workgroups: counter form (tools/group_bar_bench.hip, 4 groups of 64
      // with the 16 KB h exchange: 2.41-2.51 us per step against 2.51-2.64 for the flag form,
      // which wins on the full 256-workgroup grid; the BiLSTM kernel itself reads the same with
      // either, 531 / 528 us); -DTTS_LSTM_BAR_FLAGS builds the flag form
#ifndef TTS_LSTM_BAR_FLAGS
      gsync_arrive(db, gen, NT);
#else
      gflag_arrive(db, gen, tl);
#endif
#pragma unroll
      for (int q = 0; q < 4; ++q) gin[q] = gbase[(long)tpos(step + 1) * G + q * 4];
#ifndef TTS_LSTM_BAR_FLAGS
      if (!gsync_wait(db, gen, &sflag)) return;
#else
      if (!gflag_wait(db, gen, &sflag, NT, tl)) return;
#endif
    }
  }
}

// returns the number of recurrences launched (row groups x directions, each with its own barrier
// block), 0 when a cooperative launch is unavailable
std::atomic<int> g_test_stall_lstm{-1};

template <int H, int NDIR>
// zero_out: the launch's fill also zeroes out (B, T_max, NDIR H): the padding past each length
static int launch_lstm_persist_t(const float* Gin, const float* Whh, const uint16_t* Whh16, const int* lens, int T_max,
                                 int B, float* hbuf, unsigned* bar, float* out, hipStream_t s, bool zero_out = false) {
  int dev = 0, coop = 0;
  HIP_OK(hipGetDevice(&dev));
  HIP_OK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
  if (!coop) return 0;
  // row groups: two recurrences of half the batch tiles each when every workgroup of both still
  // fits the device (the encoder BiLSTM, B > 16: 2 x 2 x 64 = 256); TTS_LSTM_RG=1 turns it off
  static const bool rg_on = [] {
    const char* e = std::getenv("TTS_LSTM_RG");
    return !e || std::atoi(e) != 1;
  }();
  const int MT0 = (B + 15) / 16;
  const int RG = (rg_on && MT0 % 2 == 0 && 2 * NDIR * (H / 4) <= device_cu_count()) ? 2 : 1;
  const int MT = MT0 / RG, Bp = MT * 16;
  {
    FillList f;  // state, barrier blocks and (zero_out) the output in one launch
    f.add(hbuf, (size_t)2 * RG * NDIR * Bp * H * 4);
    if (zero_out) f.add(out, (size_t)B * T_max * NDIR * H * 4);
    add_barrier_fills(f, bar, RG * NDIR);
    launch_fills(f, s);
  }
  int stall = g_test_stall_lstm.load();  // test hook (tts_test_stall_lstm), -1 in production
  void* args[] = {(void*)&Whh, (void*)&Whh16, (void*)&Gin, (void*)&lens, (void*)&T_max,
                  (void*)&B,   (void*)&hbuf,  (void*)&out, (void*)&bar, (void*)&stall};
#define LPK(mt, x) (const void*)lstm_persist_kernel<mt, H, NDIR, x>
  static const void* const fns[2][4] = {{LPK(1, false), LPK(2, false), LPK(3, false), LPK(4, false)},
                                        {LPK(1, true), LPK(2, true), LPK(3, true), LPK(4, true)}};
#undef LPK
  const void* f = fns[Whh16 ? 1 : 0][MT - 1];
  launch_resident(f, dim3(RG * NDIR * H / 4), dim3(64 * LSTM_NW), args, 0, s);
  return RG * NDIR;
}

// encoder BiLSTM (H = 256, both directions; zeroes out first): the number of recurrences (barrier
// blocks in `bar`), 0 = cooperative launch unavailable (nothing launched, out untouched)
int launch_bilstm_persist(const float* Gin, const float* Whh, const uint16_t* Whh16, const int* lens, int T_max,
                          int B, float* hbuf, unsigned* bar, float* out, hipStream_t s) {
  return launch_lstm_persist_t<256, 2>(Gin, Whh, Whh16, lens, T_max, B, hbuf, bar, out, s, true);
}

// GE2E speaker-encoder LSTM layer (H = 768, forward only); hbuf >= 2 x 64 x 768 floats, bar >= 512 words
bool launch_lstm768_persist(const float* Gin, const float* Whh, const uint16_t* Whh16, const int* lens, int T_max,
                            int B, float* hbuf, unsigned* bar, float* out, hipStream_t s) {
  TTS_CHECK(B >= 1 && B <= 64, "speaker encoder: 1..64 sequences per launch");
  return launch_lstm_persist_t<768, 1>(Gin, Whh, Whh16, lens, T_max, B, hbuf, bar, out, s) > 0;
}

void launch_bilstm(const float* Gin, const float* Whh, const int* lens, int T_max, int B, float* hbuf, float* cbuf,
                   float* out, hipStream_t s) {
  if (B <= 0 || T_max <= 0) return;
  TTS_CHECK(B <= 64, "bilstm: B <= 64");
  const int MT = (B + 15) / 16, Bp = MT * 16;
  HIP_OK(hipMemsetAsync(hbuf, 0, (size_t)2 * 2 * Bp * 256 * 4, s));
  HIP_OK(hipMemsetAsync(cbuf, 0, (size_t)2 * Bp * 256 * 4, s));
  for (int step = 0; step < T_max; ++step) {
    const float* hi = hbuf + (size_t)(step & 1) * 2 * Bp * 256;
    float* ho = hbuf + (size_t)((step + 1) & 1) * 2 * Bp * 256;
    switch (MT) {
      case 1: bilstm_step_kernel<1><<<128, 256, 0, s>>>(Whh, Gin, lens, T_max, B, step, hi, ho, cbuf, out); break;
      case 2: bilstm_step_kernel<2><<<128, 256, 0, s>>>(Whh, Gin, lens, T_max, B, step, hi, ho, cbuf, out); break;
      case 3: bilstm_step_kernel<3><<<128, 256, 0, s>>>(Whh, Gin, lens, T_max, B, step, hi, ho, cbuf, out); break;
      default: bilstm_step_kernel<4><<<128, 256, 0, s>>>(Whh, Gin, lens, T_max, B, step, hi, ho, cbuf, out); break;
    }
  }
  HIP_OK(hipGetLastError());
}

// GE2E layer pipeline (round 4): the nl 768-unit LSTM layers of the speaker encoder
// (TTS/speaker_encoder/model.py:7-58: LSTMWithProjection x nl, or one nl-layer nn.LSTM) in ONE
// persistent launch. Layer l computes time t = s - l in global step s, so a call takes T + nl - 1
// grid-barrier steps instead of nl x T, and the layers' input projections run inside the
// recurrence instead of as convs between layer launches:
//   gates^l_t = W_hh^l h^l_{t-1} + W_in^l h^{l-1}_t + b^l   (l >= 1; layer 0 reads its precomputed
//   input gates), W_in^l = W_ih^l W_proj^{l-1} (the projection folded on the host, fp64) or W_ih^l.
// h^{l-1}_t was written by layer l - 1 in step s - 1, like h^l_{t-1}: one barrier per step covers
// both edges. Workgroup (l, tile) owns hidden units 12 tile .. 12 tile + 11 (3 gate-interleaved
// 16-row tiles, lstm_tile_rows order); its 8 waves split the K range (layer >= 1: waves 0-3 the
// recurrent half, 4-7 the input half) for all 3 tiles, with every weight fragment in VGPRs, and
// combine through LDS; thread (m, unit) keeps the cell state. Split-f16 only (|h| <= 1, weights
// range-checked at pack time), B <= 16.
//   w16  : per layer [192 m-tiles][NKS k-steps][64][16] (split16.h pack_split_a), NKS = 24 / 48
//   hbuf : [2 ping-pong][nl][16 x 768] fragment order, pre-split (stc_quad_x3; zeroed by the launcher)
//   out  : (B, T_max, 768), the last layer's h
struct GePipeArgs {
  const uint16_t* w16[4];
  const float* bias[4];
  const float* gin0;  // (B, T_max, 3072) layer-0 input gates incl. biases, tile order
  const int* lens;
  int T_max, B, nl;
  float* hbuf;
  float* out;
  unsigned* bar;
};
constexpr int GP_TILES = 64, GP_NW = 8;

template <class T>
__device__ __forceinline__ T pick4(T v0, T v1, T v2, T v3, int i) {  // wave-uniform, no indexed kernarg
  return i == 0 ? v0 : (i == 1 ? v1 : (i == 2 ? v2 : v3));
}

__global__ __launch_bounds__(64 * GP_NW) void ge2e_pipe_kernel(GePipeArgs a) {
  constexpr int H = 768, KSH = H / 32;  // 24 k-steps per 768-wide operand
  __shared__ float part[GP_NW][3][16 * 17];  // (stride 17: see LRS; this kernel reads 3 tiles per row group)
  __shared__ int sflag;
  const int l = blockIdx.x / GP_TILES, tile = blockIdx.x % GP_TILES;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int KS = l == 0 ? KSH / GP_NW : 2 * KSH / GP_NW;  // k-steps per wave: 3 / 6
  const int nks = l == 0 ? KSH : 2 * KSH;
  const h8* W = reinterpret_cast<const h8*>(pick4(a.w16[0], a.w16[1], a.w16[2], a.w16[3], l));
  h8 w[6][3][2];
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int mi = 0; mi < 3; ++mi) {
      const int ks = wave * KS + (j < KS ? j : 0);
      const long f = (((long)(3 * tile + mi) * nks + ks) * 64 + lane) * 2;
      w[j][mi][0] = W[f];
      w[j][mi][1] = W[f + 1];
    }
  // epilogue threads: (batch row m, unit uu of the workgroup's 12)
  const bool eth = tid < 192;
  const int m = eth ? tid / 12 : 0, uu = tid % 12, mi_e = uu >> 2, u = uu & 3;
  const int Tm = m < a.B ? a.lens[m] : 0;
  const int unit = 12 * tile + uu, trow = (3 * tile + mi_e) * 16;
  const float* bl = pick4(a.bias[0], a.bias[1], a.bias[2], a.bias[3], l);
  float bq[4] = {0.f, 0.f, 0.f, 0.f};
  if (l > 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[q] = bl[trow + q * 4 + u];
  }
  const float* g0 = a.gin0 + (long)min(m, a.B - 1) * a.T_max * 3072 + trow + u;
  float gin[4] = {0.f, 0.f, 0.f, 0.f};
  auto load_gin = [&](int t) {
    const int tc = min(max(t, 0), a.T_max - 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) gin[q] = g0[(long)tc * 3072 + q * 4];
  };
  if (l == 0) load_gin(0);
  const int l1 = 32 * ((lane >> 4) & 1) + (lane & 15);
  const int S = a.T_max + a.nl - 1;
  float cst = 0.f;
  unsigned gen = 0;
  for (int s = 0; s < S; ++s) {
    const int t = s - l;
    if (t >= 0 && t < a.T_max) {
      const size_t slab = (size_t)16 * H;
      const float* hp = a.hbuf + ((size_t)(s & 1) * a.nl + l) * slab;
      const float* hin = a.hbuf + ((size_t)(s & 1) * a.nl + (l > 0 ? l - 1 : 0)) * slab;
      // this wave's operand: the recurrent half (k-steps < 24) or the input half, never both
      const bool inh = wave * KS >= KSH;
      const float* src = inh ? hin : hp;
      const int k0 = wave * KS - (inh ? KSH : 0);
      f32x4 x[6][2];
#pragma unroll
      for (int j = 0; j < 6; ++j)
        if (j < KS) {
          const int c = 2 * (k0 + j) + (lane >> 5);
          x[j][0] = ldc4(src, (c * 64 + l1) * 16);
          x[j][1] = ldc4(src, (c * 64 + l1 + 16) * 16);
        }
      f32x4 am[3], ac[3];
#pragma unroll
      for (int mi = 0; mi < 3; ++mi) am[mi] = ac[mi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 6; ++j)
        if (j < KS) {
          // published pre-split (stc_quad_x3): k 0..3 as [hi | lo] in x[j][0], k 4..7 in x[j][1]
          const h8 xh = __builtin_bit_cast(h8, (f32x4{x[j][0][0], x[j][0][1], x[j][1][0], x[j][1][1]}));
          const h8 xl = __builtin_bit_cast(h8, (f32x4{x[j][0][2], x[j][0][3], x[j][1][2], x[j][1][3]}));
#pragma unroll
          for (int mi = 0; mi < 3; ++mi) mfma_x3(xh, xl, w[j][mi][0], w[j][mi][1], am[mi], ac[mi]);
        }
#pragma unroll
      for (int mi = 0; mi < 3; ++mi)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          part[wave][mi][(4 * (lane >> 4) + jj) * 17 + (lane & 15)] = x3_value(am[mi][jj], ac[mi][jj]);
      lds_barrier();
      if (eth && m < a.B && t < Tm) {
        float pre[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = q * 4 + u;
          float sum = part[0][mi_e][m * 17 + n];
#pragma unroll
          for (int wv = 1; wv < GP_NW; ++wv) sum += part[wv][mi_e][m * 17 + n];
          pre[q] = sum + (l == 0 ? gin[q] : bq[q]);
        }
        cst = sigm_f(pre[1]) * cst + sigm_f(pre[0]) * tanh_f(pre[2]);
        const float hn = sigm_f(pre[3]) * tanh_f(cst);
        float* ho = a.hbuf + ((size_t)((s + 1) & 1) * a.nl + l) * slab;
        stc_quad_x3(ho, (int)frag_idx(m, unit, H), hn);  // a quad = 4 units of one row: one 16-byte store, pre-split
        if (l == a.nl - 1) a.out[((long)m * a.T_max + t) * H + unit] = hn;
      }
    }
    if (s + 1 < S) {
      gflag_arrive(a.bar, gen);
      if (l == 0) load_gin(t + 1);
      if (!gflag_wait(a.bar, gen, &sflag)) return;
    }
  }
}

// false: B or nl outside the pipeline's geometry (the caller runs the per-layer kernels)
bool launch_ge2e_pipe(const uint16_t* const* w16, const float* const* bias, int nl, const float* gin0, const int* lens,
                      int T_max, int B, float* hbuf, unsigned* bar, float* out, hipStream_t s) {
  if (B < 1 || B > 16 || nl < 1 || nl > 4 || GP_TILES * nl > device_cu_count()) return false;
  for (int l = 0; l < nl; ++l)
    if (!w16[l] || (l > 0 && !bias[l])) return false;
  GePipeArgs a{};
  for (int l = 0; l < 4; ++l) {
    a.w16[l] = w16[l < nl ? l : 0];
    a.bias[l] = l > 0 && l < nl ? bias[l] : nullptr;
  }
  a.gin0 = gin0;
  a.lens = lens;
  a.T_max = T_max;
  a.B = B;
  a.nl = nl;
  a.hbuf = hbuf;
  a.out = out;
  a.bar = bar;
  HIP_OK(hipMemsetAsync(hbuf, 0, (size_t)2 * nl * 16 * 768 * 4, s));
  arm_barrier(bar, 1, s);
  void* args[] = {(void*)&a};
  launch_resident((const void*)ge2e_pipe_kernel, dim3(GP_TILES * nl), dim3(64 * GP_NW), args, 0, s);
  return true;
}
