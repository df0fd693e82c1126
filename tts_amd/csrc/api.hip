// C-ABI of the ttship library: context, weight folding / packing, workspace, the
// graph-captured autoregressive decode loop, and the vocoder pipeline.
#include "common.h"
#include "decoder.h"
#include "gsync.h"
#include "split16.h"
#include "../../include/ttship.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

void launch_embed_gather(const int64_t* ids, int T_max, const float* table, int num_rows, int D,
                         const int* lens, int B, float* out, hipStream_t s, const int* rowmap = nullptr);
int launch_bilstm_persist(const float* Gin, const float* Whh, const uint16_t* Whh16, const int* lens, int T_max,
                          int B, float* hbuf, unsigned* bar, float* out, hipStream_t s);
void launch_glu_ln_res(const float* x, long xb, int C2, const float* gamma, const float* beta, const float* res,
                       long rb, float* out, long ob, const int* lens, int B, int T, hipStream_t s);
void launch_ln(float* x, long xb, int C, const float* gamma, const float* beta, const int* lens, int B, int T,
               hipStream_t s, bool relu = false);
void launch_glow_mha(const float* qkv, int H, int heads, int T, const int* lens, float* out, int B, hipStream_t s);
void launch_tds_depthwise(const float* x, int C, int T, const float* w, const float* bias, const int* lens, float* y,
                          int B, hipStream_t s);
void launch_glow_durations(const float* logw, int T, const int* lens, float length_scale, float* cum, int* ylen,
                           float* wceil, int B, hipStream_t s);
void launch_glow_expand(const float* o_mean, int C, int Tx, const int* xlens, const float* cum, const int* ylens,
                        int Ty, const float* noise, float noise_scale, float* y_mean, float* z, float* attn, int B,
                        hipStream_t s);
void launch_glow_squeeze(const float* x, int C, int T, const int* ylens, float* y, int K, int B, hipStream_t s);
void launch_glow_unsqueeze(const float* x, int C2, int K, const int* ylens, float* y, int T, int B, hipStream_t s);
void launch_pw_upsample(const float* in, long ib, int Lin_max, const int* lens, int len_add, int in_mul, int s,
                        const float* h, float* out, long ob, int Lout_max, int C, int B, hipStream_t st);
void launch_pw_first(const float* noise, long nb, const float* w, const float* bias, const int* lens, int len_add,
                     int hop, float* x, int Tmax, int B, hipStream_t st);
void launch_pw_layer(const float* x, const float* c, float* xn, float* skip, const float* W1, const float* b1,
                     const float* W2, const float* b2, const int* lens, const float* zeros, int len_add, int hop,
                     int Tmax, int dil, int first, int B, int variant, hipStream_t st);
void launch_pw_layer_x3(const float* x, const float* c, float* xn, float* skip, const void* W1x, const float* b1,
                        const void* W2x, const float* b2, const int* lens, const int* h_lens, int len_add, int hop,
                        int Tmax, int dil, int first, int B, unsigned* oflow, hipStream_t st);
void pack_pw_layer_x3(const std::vector<float>& m1, const std::vector<float>& m2, std::vector<uint16_t>& w1x,
                      std::vector<uint16_t>& w2x);
void launch_pw_out(const float* skip, float scale, const float* W3, const float* b3, const float* w4,
                   const float* b4, const int* lens, int len_add, int hop, int Tmax, float* out, int B,
                   hipStream_t st);
void launch_glow_speaker(const int* spk, const float* table, int c_in, int c_pad, float* g, int B, hipStream_t s);
void launch_glow_embed(const int64_t* ids, int T, const float* table, int rows, int D, const int* lens, float* out,
                       int B, hipStream_t s);
bool launch_ge2e_pipe(const uint16_t* const* w16, const float* const* bias, int nl, const float* gin0, const int* lens,
                      int T_max, int B, float* hbuf, unsigned* bar, float* out, hipStream_t s);
bool launch_lstm768_persist(const float* Gin, const float* Whh, const uint16_t* Whh16, const int* lens, int T_max,
                            int B, float* hbuf, unsigned* bar, float* out, hipStream_t s);
void launch_bilstm(const float* Gin, const float* Whh, const int* lens, int T_max, int B, float* hbuf, float* cbuf,
                   float* out,
                       hipStream_t s);

static thread_local std::string g_err;
void tts_set_error(const std::string& m) { g_err = m; }

namespace {

constexpr int CHUNK = 8;  // decoder steps per captured graph (even: parity of t == parity of j)
constexpr int BMAX = 64;  // utterances per call (Bp <= 64)

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  // grow-only; returns true when the address changed
  bool ensure(size_t n) {
    if (n <= bytes && p) return false;
    if (p) HIP_OK(hipFree(p));
    p = nullptr;
    HIP_OK(hipMalloc(&p, std::max<size_t>(n, 256)));
    bytes = std::max<size_t>(n, 256);
    return true;
  }
  template <class T>
  void upload(const std::vector<T>& v) {
    ensure(v.size() * sizeof(T));
    HIP_OK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  }
  void reset() {
    if (p) HIP_OK(hipFree(p));
    p = nullptr;
    bytes = 0;
  }
  float* f() const { return static_cast<float*>(p); }
  int* i() const { return static_cast<int*>(p); }
  const uint16_t* h() const { return static_cast<const uint16_t*>(p); }
};

// split-f16 A fragments (split16.h pack_split_a) of a row-major (rows x K) matrix, rows and K
// multiples of 16 and 32; the buffer stays empty when a weight is outside the f16 range (the
// kernels then take their fp32 path)
void upload_split_rows(DevBuf& d, const std::vector<float>& w, int rows, int K) {
  bool ok = rows % 16 == 0 && K % 32 == 0 && w.size() == (size_t)rows * K;
  for (float v : w) ok &= std::fabs(v) < F16_RANGE;
  if (!ok) {
    d.reset();
    return;
  }
  d.upload(pack_split_a(rows / 16, K / 32, [&](int m, int k) { return w[(size_t)m * K + k]; }));
}

struct HostT {
  std::vector<float> d;
  std::vector<int64_t> shape;
};
using HostMap = std::map<std::string, HostT>;

const HostT& need(const HostMap& m, const std::string& k, std::vector<int64_t> shape) {
  auto it = m.find(k);
  TTS_CHECK(it != m.end(), "missing tensor: " + k);
  if (!shape.empty()) {
    bool ok = it->second.shape == shape;
    if (!ok) {
      std::string s = "shape mismatch for " + k + ": got (";
      for (auto x : it->second.shape) s += std::to_string(x) + ",";
      s += ") expected (";
      for (auto x : shape) s += std::to_string(x) + ",";
      throw std::runtime_error(s + ")");
    }
  }
  return it->second;
}

struct ConvLayer {
  DevBuf W, bias;
  int Cin = 0, Cout = 0, Cout_pad = 0, K = 1, dil = 1, tile = 0, nphase = 1;
  int pad_left[8] = {0};
  long phase_stride = 0;
  DevBuf W16;             // split-f16 A fragments (conv_x3.hip); empty when the shape is not covered
  long w16_stride = 0;    // bytes per phase
};

// Wm: nphase blocks of [Cout][Cin*K] row-major
void pack_conv(ConvLayer& L, const std::vector<float>& Wm, const std::vector<float>& bias, int Cin, int Cout,
               int K, int dil, int nphase, const int* pad_left) {
  TTS_CHECK(Cin % 16 == 0, "conv Cin must be a multiple of 16");
  L.Cin = Cin;
  L.Cout = Cout;
  L.K = K;
  L.dil = dil;
  L.nphase = nphase;
  L.tile = conv_tile_for_cout(Cout);
  if (K == 1 && Cout % 64 == 0 && Cout <= 384) L.tile = TILE_64x64;  // short 1x1 convs: more workgroups
  const int TC = conv_tile_tc(L.tile);
  L.Cout_pad = (Cout + TC - 1) / TC * TC;
  const int Kdim = Cin * K;
  const size_t per = (size_t)L.Cout_pad * Kdim;
  // k order inside each 16-input-channel chunk: tap-major (k' = tap * 16 + ci % 16), so k-chunk
  // `tap` of a staging chunk reads LDS rows ci at column offset tap * dil (no offset table)
  std::vector<float> Wt(Wm.size());
  for (size_t r = 0; r < (size_t)nphase * Cout; ++r)
    for (int ci = 0; ci < Cin; ++ci)
      for (int k = 0; k < K; ++k)
        Wt[r * Kdim + (size_t)(ci / 16) * 16 * K + k * 16 + ci % 16] = Wm[r * Kdim + (size_t)ci * K + k];
  std::vector<float> sw(per * nphase);
  for (int ph = 0; ph < nphase; ++ph)
    swizzle_rows16(Wt.data() + (size_t)ph * Cout * Kdim, Cout, L.Cout_pad, Kdim, sw.data() + ph * per);
  L.phase_stride = (long)per;
  L.W.upload(sw);
  L.bias.upload(bias);
  for (int ph = 0; ph < nphase; ++ph) L.pad_left[ph] = pad_left[ph];
  // split-f16 weights when the shape is covered and every weight is inside the f16 range
  bool in_range = true;
  for (float v : Wm) in_range &= std::fabs(v) < F16_RANGE;
  if (conv_x3_supported(Cin, Cout, K, dil) && in_range) {
    const std::vector<uint16_t> w16 = pack_conv_x3(Wm, Cin, Cout, K, nphase, &L.w16_stride);
    L.W16.ensure(w16.size() * 2);
    HIP_OK(hipMemcpy(L.W16.p, w16.data(), w16.size() * 2, hipMemcpyHostToDevice));
  } else {
    L.W16.reset();
  }
}

// split-f16 weights only (a layer that has no fp32 form: the phase-merged ConvTranspose)
void pack_conv_x3_only(ConvLayer& L, const std::vector<float>& Wm, const std::vector<float>& bias, int Cin, int Cout,
                       int K) {
  TTS_CHECK(conv_x3_supported(Cin, Cout, K, 1), "conv_x3: shape not covered");
  L.Cin = Cin;
  L.Cout = L.Cout_pad = Cout;
  L.K = K;
  L.dil = 1;
  L.nphase = 1;
  L.pad_left[0] = (K - 1) / 2 + (K == 2 ? 1 : 0);
  for (float v : Wm) TTS_CHECK(std::fabs(v) < F16_RANGE, "conv_x3: weight outside the f16 range");
  const std::vector<uint16_t> w16 = pack_conv_x3(Wm, Cin, Cout, K, 1, &L.w16_stride);
  L.W16.ensure(w16.size() * 2);
  HIP_OK(hipMemcpy(L.W16.p, w16.data(), w16.size() * 2, hipMemcpyHostToDevice));
  L.bias.upload(bias);
}

struct ConvCall {
  ConvSrc s[2];
  int nsrc = 1;
  int pad_mode = 0;
  const int* lens = nullptr;
  int len_add = 0, in_mul = 1, q_mul = 1, rep_pad = 0, out_mul = 1;
  float* out = nullptr;
  long ob = 0;
  int oc = 0, ot = 0;
  int epi = 0;
  const float* resid = nullptr;
  long rb = 0;
  int rc = 0, rt = 0, resid_rows = 0;
  const float* aux = nullptr;
  long auxb = 0;              // epi 3: batch stride of the per-utterance gate bias in aux
  int max_q = 0, B = 0;
  unsigned* oflow = nullptr;  // set: run the split-f16 kernel where the layer has split weights
  int merged_u = 0;           // phase-merged ConvTranspose (layer from pack_conv_x3_only)
};

void run_conv(const ConvLayer& L, const ConvCall& c, hipStream_t st) {
  ConvArgs a{};
  a.src[0] = c.s[0];
  a.src[1] = c.nsrc > 1 ? c.s[1] : c.s[0];
  if (c.nsrc == 1) a.src[0].C = L.Cin;
  a.nsrc = c.nsrc;
  a.Cin = L.Cin;
  a.K = L.K;
  a.dil = L.dil;
  a.pad_mode = c.pad_mode;
  a.lens = c.lens;
  a.len_add = c.len_add;
  a.in_mul = c.in_mul;
  a.q_mul = c.q_mul;
  a.rep_pad = c.rep_pad;
  a.nphase = L.nphase;
  for (int i = 0; i < 8; ++i) a.pad_left[i] = L.pad_left[i];
  a.w_phase_stride = L.phase_stride;
  a.W = L.W.f();
  a.bias = L.bias.f();
  a.Cout = L.Cout;
  a.Cout_pad = L.Cout_pad;
  a.out = c.out;
  a.ob = c.ob;
  a.oc = c.oc;
  a.ot = c.ot;
  a.out_mul = c.out_mul;
  a.epi_act = c.epi;
  a.resid = c.resid;
  a.rb = c.rb;
  a.rc = c.rc;
  a.rt = c.rt;
  a.resid_rows = c.resid_rows;
  a.aux = c.aux;
  a.auxb = c.auxb;
  a.max_q = c.max_q;
  a.B = c.B;
  a.merged_u = c.merged_u;
  TTS_CHECK(!c.merged_u || (c.oflow && L.W16.p), "phase-merged ConvTranspose runs on split-f16 weights only");
  if (c.oflow && L.W16.p && c.nsrc == 1 && (c.s[0].sc != 1 || c.s[0].st % 4 == 0)) {
    a.W16 = L.W16.p;
    a.w16_phase_stride = L.w16_stride;
    a.oflow = c.oflow;
    launch_conv_x3(a, st);
    return;
  }
  launch_conv(a, L.tile, st);
}

ConvSrc src_of(const float* p, long sb, int sc, int st, int C, int act) {
  ConvSrc s;
  s.ptr = p;
  s.sb = sb;
  s.sc = sc;
  s.st = st;
  s.C = C;
  s.act = act;
  return s;
}

// ---------------------------------------------------------------- Tacotron2 -----------
struct TacoModel {
  bool ready = false;
  int num_chars = 0, r_init = 7, softmax = 0;
  DevBuf emb;
  ConvLayer enc[3], lstm_in, penc, post[5];
  DevBuf whhT;
  DevBuf whhT16;  // W_hh split-f16 for the persistent BiLSTM (empty if out of the f16 range)
  DevBuf pre1, pre2, att_p, att_pre, att_bias, dec_w, dec_bias, WqT, Wloc, Wdense, v, proj_w, proj_b;
  // split-f16 forms for the persistent decoder (P3 prenet part, P5 ctx parts); empty if out of range
  DevBuf att_p_x3, dec_x3, apre_x3, pj_x3;
  DevBuf Wcomb;  // location_dense . location_conv folded, [64 taps (62 used)][128 dims]
  float bv = 0.f;
  // persistent decoder: projection rows [stop tile | W_p] (+ bias) and prenet layer 1 on the host,
  // folded per r into pj_w / pj_b = [stop tile | first 80r rows of W_p | W1 W_p,last frame]
  std::vector<float> proj_rows, proj_bias, pre1_host;
  DevBuf pj_w, pj_b;
  int pj_r = -1;
  // multi-speaker (models/tacotron2.py:50-58, 152-155): the speaker vector s is constant over the
  // encoder positions and the attention weights of a step sum to 1, so every ctx-fed GEMM splits
  // into its 512 encoder columns plus W_s s, a per-utterance bias. Host copies of the speaker
  // columns (rows in the kernels' order), spk_dim x ... each; spk_wT = [spk_dim][NSPK] for pj_r.
  int spk_dim = 0, num_spk = 0;
  // decoder variants (common_layers.py:25-74, 196-372): BN prenet folded into the prenet weights
  // (+ biases), windowing / forward attention / transition agent flags
  bool prenet_bn = false, windowing = false, forward_attn = false, trans_agent = false, forward_attn_mask = false;
  std::vector<float> pre1_bias;  // b1' (BN), folded into the projection's prenet rows
  DevBuf pre1_b0, pre2_b, ta_w;
  float ta_b = 0.f;
  bool variant() const { return prenet_bn || windowing || forward_attn || graves; }
  // Graves attention (common_layers.py:113-193): N_a layer 1 as 64 swizzled 16-row tiles of the
  // P3g GEMM (K = 1024), its bias, layer 2 (3K x 1024, row-major) and bias
  bool graves = false;
  int graves_K = 0;
  DevBuf na1_w, na1_b, na2_w, na2_b;
  DevBuf spk_table;  // speaker_embedding.weight (num_spk, 512) when learned
  std::vector<float> spk_att_h, spk_dec_h, spk_penc_h, proj_spk;
  DevBuf spk_wT;
};

// Tacotron2 status words (TacoWS::stat on the device, tts_ctx::pinned on the host; one copy after
// the call): BiLSTM barrier errors (one per recurrence: 2 directions x up to 2 row groups),
// persistent-decoder barrier errors (one per launch), the decoder results (done, steps, status per
// decode row), the range flag, the launches' end steps
constexpr int PMAX_LAUNCH = 4;  // persistent decoder launches per decode (MT = 4, 3, 2, 1)
constexpr int PBAR_CAND = 16;   // candidate barrier blocks timed for them
constexpr int ENC_NDOM_MAX = 4;  // BiLSTM recurrences (barrier blocks) per launch
constexpr int TS_ENC = 16, TS_DEC = TS_ENC + ENC_NDOM_MAX, TS_RES = TS_DEC + PMAX_LAUNCH, TS_FLAG = TS_RES + 3 * BMAX,
              TS_END = TS_FLAG + 1, TS_VERR = TS_END + PMAX_LAUNCH, TS_N = TS_VERR + 1;
static_assert(TS_N <= 240, "status words fit the pinned block below check_encoder_barrier's words");

struct TacoWS {
  int B = 0, T_max = 0, S_cap = 0, r = 0, MT = 0;
  long gen = 0;
  DevBuf lens, mlens, x0, ca, cb, gin, enc, penc;
  DevBuf lh, lc;  // BiLSTM h (2 buffers x 2 directions, fragment order) and c
  DevBuf p1, pb, gatt, hatt, catt, hdec0, hdec1, cdec, ctx, y, pq, spart, alpha, acum, energy, ctl;
  DevBuf dec, align, stop, pa, pbb;
  DevBuf aps, apm, apu, acnt;  // attention chunk partials + per-utterance arrival counters
  DevBuf post, map;            // rows in decode order (longest first); map = [perm | inverse]
  DevBuf stat;                 // status words for the host, laid out as tts_ctx::pinned (TS_*)
  DevBuf ypart, pbar;          // persistent decoder: projection halves, grid-barrier words
  // the decoder launches' barrier blocks: PBAR_CAND candidates in pbar, the PMAX_LAUNCH fastest
  // picked once per allocation (pick_barrier_blocks)
  int pslot[PMAX_LAUNCH] = {0, 1, 2, 3};
  const void* pslot_base = nullptr;
  bool pslot_cal = false;      // pslot timed (after enter(), on the first persistent decode of these blocks)
  DevBuf anorm;                // persistent decoder: per-utterance attention normaliser (deferred alignment)
  DevBuf spk, spkid, spkb;     // speaker vectors (decode order), per-row biases [Bp][NSPK]
  DevBuf win_idx, fwd_u, apf;  // windowing argmax, transition probability, forward chunk sums
  DevBuf gh, gmu;              // Graves: N_a hidden (32 x 1024), mixture means (64 x 16)
  DevBuf trace, xdiag;         // TTS_PTRACE / TTS_DIAG_XCC diagnostics, on this context's device
  bool enc_persist = false;    // the last encoder ran the persistent BiLSTM (lc = its barrier words)
  int enc_ndom = 0;            // its recurrences (directions x row groups), one barrier block each
  // one CHUNK-step graph per batch-tile count MT' <= MT (the batch tile shrinks as the
  // longest-first rows finish); all share one configuration key
  hipGraphExec_t graphs[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  long graph_gen = -1;
  int gB = -1, gT = -1, gS = -1, gr = -1;
  float thr = 0.5f, gthr = -1.f;
};

struct MelganModel {
  bool ready = false;
  int in_ch = 80, out_ch = 4, base = 384, nres = 4, pqmf = 1, taps = 62;
  std::vector<int> ups;
  ConvLayer conv_in, conv_out;
  std::vector<ConvLayer> convT;
  std::vector<ConvLayer> convTm;  // phase-merged split-f16 form (conv_x3.hip merged_u), W16 only
  std::vector<ConvLayer> dconv, fused;  // [stage*nres + block]
  std::vector<DevBuf> rb_wd16, rb_wf16;  // split-f16 block weights (resblock_x3.hip), empty if C unsupported
  std::vector<DevBuf> rb_wd16p;          // phase-1 weights in the packed order (C % 32 == 16), for resstack_x3
  DevBuf G;
  DevBuf out_w, out_b;  // conv_out as [c][k][o] for the fused output + PQMF kernel
  int C_last = 0;
};

// what run_generator leaves when the output conv is left to the fused PQMF kernel
struct GenTail {
  const float* x = nullptr;  // last ResidualStack output (B, C, Ls), before LReLU
  int C = 0;
  long Ls = 0;
  int mul = 1;
};

struct MelganWS {
  DevBuf lens, xa, xb, bands;
};

}  // namespace

// GE2E speaker encoder (TTS/speaker_encoder/model.py:5-80): 3 x [LSTM(in -> 768), Linear(768 -> 256,
// no bias)] (use_lstm_with_projection) or one 3-layer LSTM + Linear(bias) + ReLU on the last hidden
// state; the embedding is the L2-normalised output at each sequence's last frame.
struct Ge2eModel {
  bool ready = false;
  int in_dim = 40, in_pad = 48, proj = 256, H = 768, nl = 3, with_proj = 1;
  ConvLayer gin[4];      // input projections (K = 1, Cout = 4H gate-interleaved tiles, b_ih + b_hh)
  DevBuf whh[4];         // W_hh, swizzled tiles
  DevBuf whh16[4];       // W_hh split-f16 (empty if out of the f16 range)
  ConvLayer proj_l[4];   // with_proj: Linear(768 -> proj) per layer as a K = 1 conv
  DevBuf lin_w, lin_b;   // without projection: final Linear (proj x H) + bias
  // layer pipeline (encoder.hip ge2e_pipe_kernel): layer l >= 1 as split-f16 [W_hh | W_in] rows
  // (W_in = W_ih^l W_proj^{l-1} folded in fp64, or W_ih^l) and b_ih + b_hh, tile order
  DevBuf wpipe[4], bpipe[4];
  bool pipe_ok = false;
};

struct Ge2eWS {
  DevBuf x, lens, g, o, p, bar, hbuf;
};

// Glow-TTS (TTS/tts/models/glow_tts.py, the reference configs' gated-conv encoder, mean_only,
// num_sqz 2, num_splits 4, dilation 1; optional speaker conditioning)
struct GlowModel {
  bool ready = false;
  int num_chars = 0, H = 192, Fdp = 256, C = 80, enc_layers = 9, flows = 12, wn_layers = 4;
  DevBuf emb;                                   // scaled by sqrt(H)
  std::vector<ConvLayer> enc_conv;              // H -> 2H, k5
  std::vector<DevBuf> enc_g, enc_b;             // LayerNorm(2H)
  // time-depth-separable encoder (configs/glow_tts_tdsep.json): ConvLayerNorm prenet, then per
  // layer time_conv (H -> 2H, BN folded, rows interleaved for the GLU epilogue), depthwise k5 (BN
  // folded) + swish, time_conv2 (BN folded) + residual
  bool tdsep = false, tfm = false;
  // transformer encoder: per layer q|k|v as one 1x1 conv (H -> 3H), o (1x1), FFN k3 (H -> 768 -> H)
  std::vector<ConvLayer> tfm_qkv, tfm_o, tfm_f1, tfm_f2;
  std::vector<DevBuf> tfm_g1, tfm_b1, tfm_g2, tfm_b2;
  std::vector<ConvLayer> pre_conv, tds_tc, tds_tc2;
  std::vector<DevBuf> pre_g, pre_b, tds_dw, tds_dwb;
  ConvLayer pre_proj;
  ConvLayer proj_m, dp1, dp2, dp_proj;
  DevBuf dp_g1, dp_b1, dp_g2, dp_b2;
  // per flow block (index = block): start (C -> H), WN in (H -> 2H, k5, rows interleaved), res+skip
  // (H -> 2H, last layer H -> H skip), end (H -> 2C, rows interleaved) whose epilogue also applies
  // the inverse InvConvNear + ActNorm from invtab (2C x {w[4], bias, exp(-logs)})
  std::vector<ConvLayer> start, end;
  std::vector<DevBuf> invtab;
  std::vector<ConvLayer> wn_in, wn_rs;  // [block * wn_layers + i]
  // speaker conditioning (glow_tts.py:97-99,159-161; encoder.py:131-135; glow.py:87-91,119-130):
  // c_in channels of g padded to c_pad (multiple of 16); the duration predictor's conv_1 reads
  // [x; g] (g broadcast over time by a time stride of 0); every block's cond_layer stacked into one
  // 1x1 conv (c_pad -> flows * wn_layers * 2H, rows interleaved like wn_in) whose output is the
  // per-utterance gate bias of each WN in-layer
  int c_in = 0, c_pad = 0, n_spk = 0;
  DevBuf emb_g;
  ConvLayer cond;
};

struct GlowWS {
  int B = 0, Tx = 0, Ty = 0;
  DevBuf ids, lens, klens, ylens, xa, xb, h2, hdp, logw, cum, wceil, om, z, sq, sq2, whs, wacts, big;
  DevBuf spk, ones, g, gcond;  // speaker ids, unit lengths, normalized g (B, c_pad), cond biases
  bool has_g = false;          // the last glow_encode was given speaker ids
  std::vector<int> h_ylens, h_klens, h_spk;
};

// ParallelWaveGAN generator (TTS/vocoder/models/parallel_wavegan_generator.py, setup_generator's
// configuration: 64 res / 128 gate / 64 skip / 80 aux channels, kernel 3)
struct PwganModel {
  bool ready = false;
  int layers = 30, stacks = 3;
  std::vector<int> ups;
  DevBuf first_w, first_b;
  ConvLayer conv_in;                 // 80 -> 80, k1, no bias
  std::vector<DevBuf> up_h;          // per factor s: 2s + 1 taps
  std::vector<DevBuf> W1, b1, W2, b2;  // per residual block (pw_layer_kernel layouts)
  std::vector<DevBuf> W1x, W2x;        // split-f16 forms (pw_layer_x3_kernel); empty if out of range
  DevBuf W3, b3, w4, b4;
};

struct PwganWS {
  DevBuf lens, ca, cb, xa, xb, skip, zeros;
};

// one submitted fused call: what its fp32 re-run needs if the split-f16 vocoder raised the range
// flag (the caller keeps d_post and d_wav untouched until the ticket is finished)
constexpr int NVT = 4, TK_PIN = 248;
struct VocTicket {
  int64_t id = 0;
  bool pending = false;       // not finished: the caller's stream is not yet ordered after the vocoder
  bool x3 = false;            // vocoder launched on split-f16 kernels: its range flag is to be looked at
  hipEvent_t ev = nullptr;    // recorded after the vocoder, the copy of its flag and the row packing
  const float* d_post = nullptr;
  int64_t st[3] = {0, 0, 0};
  std::vector<int32_t> lens;  // decoded mel lengths, caller order
  int B = 0, M = 0, pad = 0;
  float* d_wav = nullptr;
};

struct tts_ctx {
  std::recursive_mutex mu;  // held by every entry point (guarded_ctx)
  int device = 0;
  hipStream_t s = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr, ev_chunk[2] = {nullptr, nullptr};
  hipEvent_t ev_dec[PMAX_LAUNCH + 1] = {};  // around the persistent decoder launches
  hipEvent_t ev_status = nullptr;  // a fused call's decode status words are on the host
  int* pinned = nullptr;  // [256]: [0:4) chunk polling, [12] range flag, [TS_*]: status words of the last
                          // Tacotron2 call (one copy of TacoWS::stat), [240:244) BiLSTM barrier
                          // words, [TK_PIN + k]: range flag of the vocoder of ticket slot k
  bool flag_read = false; // the entry point already fetched the range flag into pinned[12]
  int dec_end[PMAX_LAUNCH] = {};  // step index after each persistent launch of the last decode
  int dec_path = 0;       // last decode: 0 = step graphs, 1 = persistent kernel
  bool dec_presplit = false;  // last persistent decode published h_att / ctx / h_dec pre-split
  // GEMM arithmetic: true = split-f16 MFMA kernels where built (fp32-accurate, split16.h), false =
  // fp32 MFMA everywhere (tts_set_gemm_mode; TTS_GEMM=f32 in the environment starts a context so)
  bool gemm_x3 = true;
  long x3_fallbacks = 0;  // calls re-run in fp32 because an operand left the f16 range
  DevBuf x3flag;          // range flag raised by split-f16 kernels during one call (with_x3_fallback)
  int dec_nlaunch = 0;
  HostMap taco_host, mg_host;
  TacoModel taco;
  TacoWS tws;
  MelganModel mg;
  MelganWS mws;
  HostMap ge2e_host;
  Ge2eModel ge2e;
  Ge2eWS gws;
  HostMap pw_host;
  PwganModel pw;
  PwganWS pws;
  HostMap glow_host;
  GlowModel glow;
  GlowWS glws;
  // last decode configuration (for tts_time_decoder_kernel)
  int last_B = 0, last_T = 0, last_S = 0, last_r = 0;
  // fused Tacotron2 + MB-MelGAN submissions whose vocoder may still run (tts_taco_mbmelgan_submit)
  VocTicket vt[NVT];
  int64_t next_ticket = 1;
  // the fused submissions' vocoders run on sv (TTS_VOC_STREAM=0: sv is s), behind their decode's
  // status event, so the next submission's Tacotron2 on s overlaps them. Each ticket slot has its own
  // device lengths and range flag (vslot: [NVT][BMAX] lengths, then NVT flags). Every other entry
  // joins sv first (enter); a fused submission's Tacotron2 does not (in_submit).
  hipStream_t sv = nullptr;
  hipEvent_t ev_sv = nullptr;  // after the last vocoder enqueued on sv
  bool sv_live = false;        // sv may hold work that s has not joined
  bool in_submit = false;
  DevBuf vslot;
  unsigned* flag_override = nullptr;  // range flag of the vocoder being enqueued (x3_flag)
  int* vlens_override = nullptr;      // device lengths of the vocoder being enqueued (run_generator)
};

int* vslot_lens(tts_ctx* c, int k) {
  c->vslot.ensure((size_t)NVT * (BMAX + 1) * 4);
  return reinterpret_cast<int*>(c->vslot.p) + k * BMAX;
}
unsigned* vslot_flag(tts_ctx* c, int k) {
  c->vslot.ensure((size_t)NVT * (BMAX + 1) * 4);
  return reinterpret_cast<unsigned*>(c->vslot.p) + NVT * BMAX + k;
}

// range flag for the split-f16 kernels of the current call, or null (fp32 kernels)
unsigned* x3_flag(tts_ctx* c) {
  if (!c->gemm_x3) return nullptr;
  if (c->flag_override) return c->flag_override;
  c->x3flag.ensure(4);
  return reinterpret_cast<unsigned*>(c->x3flag.p);
}

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    HIP_OK(hipGetDevice(&prev));
    if (prev != d) HIP_OK(hipSetDevice(d));
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// stream ordering with the caller's stream (nothing to wait for when all of its work is complete:
// a server loop's stream holds only waits on this context's own finished events)
void enter(tts_ctx* c, void* stream) {
  if (c->sv_live && !c->in_submit) {  // a fused submission's vocoder may still use the vocoder workspace
    HIP_OK(hipStreamWaitEvent(c->s, c->ev_sv, 0));
    c->sv_live = false;
  }
  if (hipStreamQuery((hipStream_t)stream) == hipSuccess) return;
  (void)hipGetLastError();  // hipErrorNotReady is not an error here; clear it for later launch checks
  HIP_OK(hipEventRecord(c->ev_in, (hipStream_t)stream));
  HIP_OK(hipStreamWaitEvent(c->s, c->ev_in, 0));
}
void leave(tts_ctx* c, void* stream) {
  HIP_OK(hipEventRecord(c->ev_out, c->s));
  HIP_OK(hipStreamWaitEvent((hipStream_t)stream, c->ev_out, 0));
}

std::vector<float> lstm_tile_rows(const std::vector<float>& W, int H, int K) {
  std::vector<float> out((size_t)4 * H * K);
  for (int t = 0; t < H / 4; ++t)
    for (int g = 0; g < 4; ++g)
      for (int u = 0; u < 4; ++u) {
        const size_t src = (size_t)(g * H + 4 * t + u) * K, dst = (size_t)(t * 16 + g * 4 + u) * K;
        std::memcpy(&out[dst], &W[src], K * sizeof(float));
      }
  return out;
}

// concatenate column blocks of matrices with equal row counts
std::vector<float> hcat(const std::vector<std::pair<const float*, int>>& parts, int rows, int ld_src_first = 0) {
  (void)ld_src_first;
  int K = 0;
  for (auto& p : parts) K += p.second;
  std::vector<float> out((size_t)rows * K);
  for (int r = 0; r < rows; ++r) {
    int off = 0;
    for (auto& p : parts) {
      std::memcpy(&out[(size_t)r * K + off], p.first + (size_t)r * p.second, p.second * sizeof(float));
      off += p.second;
    }
  }
  return out;
}

std::vector<float> slice_cols(const std::vector<float>& W, int rows, int K, int c0, int c1) {
  std::vector<float> out((size_t)rows * (c1 - c0));
  for (int r = 0; r < rows; ++r)
    std::memcpy(&out[(size_t)r * (c1 - c0)], &W[(size_t)r * K + c0], (c1 - c0) * sizeof(float));
  return out;
}

std::vector<float> swz(const std::vector<float>& Wm, int rows, int K) {
  const int rp = (rows + 15) / 16 * 16;
  std::vector<float> out((size_t)rp * K);
  swizzle_rows16(Wm.data(), rows, rp, K, out.data());
  return out;
}

void fold_convbn(const HostMap& m, const std::string& pfx, int Cin, int Cout, int K, std::vector<float>& Wm,
                 std::vector<float>& bias) {
  const auto& W = need(m, pfx + ".convolution1d.weight", {Cout, Cin, K}).d;
  const auto& b = need(m, pfx + ".convolution1d.bias", {Cout}).d;
  const auto& g = need(m, pfx + ".batch_normalization.weight", {Cout}).d;
  const auto& be = need(m, pfx + ".batch_normalization.bias", {Cout}).d;
  const auto& mu = need(m, pfx + ".batch_normalization.running_mean", {Cout}).d;
  const auto& var = need(m, pfx + ".batch_normalization.running_var", {Cout}).d;
  Wm.resize((size_t)Cout * Cin * K);
  bias.resize(Cout);
  for (int co = 0; co < Cout; ++co) {
    const double sc = (double)g[co] / std::sqrt((double)var[co] + 1e-5);
    for (int i = 0; i < Cin * K; ++i) Wm[(size_t)co * Cin * K + i] = (float)(W[(size_t)co * Cin * K + i] * sc);
    bias[co] = (float)(((double)b[co] - mu[co]) * sc + be[co]);
  }
}

void taco_finalize(tts_ctx* c, int num_chars, int r_init, int attn_norm) {
  auto& M = c->taco;
  M.graves = c->taco_host.count("decoder.attention.N_a.0.weight") > 0;
  if (M.graves) {
    // Graves attention has no location-sensitive tensors: zero stand-ins keep the shared packing
    // (processed inputs, query projection, location filters, energies) well defined; the Graves
    // variant of the persistent decoder never reads what they produce
    const auto it = c->taco_host.find("decoder.attention_rnn.weight_ih");
    TTS_CHECK(it != c->taco_host.end() && it->second.shape.size() == 2 && it->second.shape[1] > 256,
              "missing tensor: decoder.attention_rnn.weight_ih");
    const int64_t ES = it->second.shape[1] - 256;
    auto zero = [&](const std::string& k, std::vector<int64_t> shape) {
      size_t n = 1;
      for (auto d : shape) n *= (size_t)d;
      c->taco_host[k] = HostT{std::vector<float>(n, 0.f), shape};
    };
    zero("decoder.attention.inputs_layer.linear_layer.weight", {128, ES});
    zero("decoder.attention.query_layer.linear_layer.weight", {128, 1024});
    zero("decoder.attention.location_layer.location_conv1d.weight", {32, 2, 31});
    zero("decoder.attention.location_layer.location_dense.linear_layer.weight", {128, 32});
    zero("decoder.attention.v.linear_layer.weight", {1, 128});
    zero("decoder.attention.v.linear_layer.bias", {1});
  }
  const auto& h = c->taco_host;
  M.ready = false;
  if (M.graves) {
    const auto& w2 = need(h, "decoder.attention.N_a.2.weight", {}).d;
    M.graves_K = (int)(w2.size() / 1024 / 3);
    TTS_CHECK(M.graves_K >= 1 && M.graves_K <= 16 && (size_t)M.graves_K * 3 * 1024 == w2.size(),
              "Graves attention: N_a.2.weight must be (3K, 1024), K <= 16");
    std::vector<float> sw((size_t)1024 * 1024);
    swizzle_rows16(need(h, "decoder.attention.N_a.0.weight", {1024, 1024}).d.data(), 1024, 1024, 1024, sw.data());
    M.na1_w.upload(sw);
    M.na1_b.upload(need(h, "decoder.attention.N_a.0.bias", {1024}).d);
    M.na2_w.upload(w2);
    M.na2_b.upload(need(h, "decoder.attention.N_a.2.bias", {3 * M.graves_K}).d);
  }
  M.num_chars = num_chars;
  M.r_init = r_init;
  M.softmax = attn_norm;
  const int E = 512, H = 256, Q = 1024, D = 1024, P = 256, A = 128, F = 80;
  M.emb.upload(need(h, "embedding.weight", {num_chars, E}).d);
  // decoder_in_features = 512 + speaker dim (models/tacotron2.py:57-58), read off inputs_layer
  {
    auto it = h.find("decoder.attention.inputs_layer.linear_layer.weight");
    TTS_CHECK(it != h.end() && it->second.shape.size() == 2 && it->second.shape[1] >= E,
              "missing tensor: decoder.attention.inputs_layer.linear_layer.weight");
    M.spk_dim = (int)it->second.shape[1] - E;
    TTS_CHECK(M.spk_dim <= 1024, "speaker embedding dim must be <= 1024");
    auto st = h.find("speaker_embedding.weight");
    M.num_spk = 0;
    if (st != h.end()) {
      TTS_CHECK(st->second.shape.size() == 2 && st->second.shape[1] == M.spk_dim,
                "speaker_embedding.weight must be (num_speakers, decoder_in_features - 512)");
      M.num_spk = (int)st->second.shape[0];
      M.spk_table.upload(st->second.d);
    }
  }
  const int S = M.spk_dim, ES = E + S;
  int pl2[8] = {2}, pl0[8] = {0};
  for (int i = 0; i < 3; ++i) {
    std::vector<float> Wm, b;
    fold_convbn(h, "encoder.convolutions." + std::to_string(i), E, E, 5, Wm, b);
    pack_conv(M.enc[i], Wm, b, E, E, 5, 1, 1, pl2);
  }
  {  // BiLSTM input projection for both directions as one K=1 conv (Cout 2048), b_ih + b_hh folded
    // gate rows of both the input projection and W_hh in gate-interleaved tile order:
    // column dir*1024 + tile*16 + gate*4 + unit  (unit = 4*tile + u)
    std::vector<float> Wm((size_t)2048 * E), b(2048);
    std::vector<float> whh_all, whh_rows;
    for (int dir = 0; dir < 2; ++dir) {
      const std::string sfx = dir ? "_reverse" : "";
      const auto& wih = need(h, "encoder.lstm.weight_ih_l0" + sfx, {4 * H, E}).d;
      const auto& whh = need(h, "encoder.lstm.weight_hh_l0" + sfx, {4 * H, H}).d;
      const auto& bih = need(h, "encoder.lstm.bias_ih_l0" + sfx, {4 * H}).d;
      const auto& bhh = need(h, "encoder.lstm.bias_hh_l0" + sfx, {4 * H}).d;
      const auto wt = lstm_tile_rows(wih, H, E);
      std::memcpy(&Wm[(size_t)dir * 1024 * E], wt.data(), (size_t)1024 * E * 4);
      std::vector<float> bs(4 * H);
      for (int i = 0; i < 4 * H; ++i) bs[i] = bih[i] + bhh[i];
      const auto bt = lstm_tile_rows(bs, H, 1);
      std::copy(bt.begin(), bt.end(), b.begin() + dir * 1024);
      const auto rows = lstm_tile_rows(whh, H, H);
      const auto hs = swz(rows, 4 * H, H);
      whh_all.insert(whh_all.end(), hs.begin(), hs.end());
      whh_rows.insert(whh_rows.end(), rows.begin(), rows.end());
    }
    pack_conv(M.lstm_in, Wm, b, E, 2048, 1, 1, 1, pl0);
    M.whhT.upload(whh_all);
    upload_split_rows(M.whhT16, whh_rows, 2 * 4 * H, H);
  }
  {  // processed_inputs = inputs_layer(enc)  (common_layers.py:262-263), K=1 conv, no bias
    const auto& win_all = need(h, "decoder.attention.inputs_layer.linear_layer.weight", {A, ES}).d;
    const auto win = slice_cols(win_all, A, ES, 0, E);
    pack_conv(M.penc, win, std::vector<float>(A, 0.f), E, A, 1, 1, 1, pl0);
    M.spk_penc_h = slice_cols(win_all, A, ES, E, ES);
  }
  M.pre1_host = need(h, "decoder.prenet.linear_layers.0.linear_layer.weight", {P, F}).d;
  std::vector<float> w2 = need(h, "decoder.prenet.linear_layers.1.linear_layer.weight", {P, P}).d;
  // BN prenet (LinearBN, common_layers.py:25-46, eval): relu(s (W x - mu) + beta) = relu(W' x + b')
  M.prenet_bn = h.count("decoder.prenet.linear_layers.0.batch_normalization.weight") > 0;
  std::vector<float> b2;
  M.pre1_bias.assign(P, 0.f);
  if (M.prenet_bn) {
    for (int l = 0; l < 2; ++l) {
      const std::string bn = "decoder.prenet.linear_layers." + std::to_string(l) + ".batch_normalization.";
      const auto& g_ = need(h, bn + "weight", {P}).d;
      const auto& b_ = need(h, bn + "bias", {P}).d;
      const auto& mu = need(h, bn + "running_mean", {P}).d;
      const auto& var = need(h, bn + "running_var", {P}).d;
      std::vector<float>& W = l == 0 ? M.pre1_host : w2;
      const int din = l == 0 ? F : P;
      std::vector<float> bias(P);
      for (int o = 0; o < P; ++o) {
        const double sc = (double)g_[o] / std::sqrt((double)var[o] + 1e-5);
        for (int k = 0; k < din; ++k) W[(size_t)o * din + k] = (float)(sc * W[(size_t)o * din + k]);
        bias[o] = (float)((double)b_[o] - sc * mu[o]);
      }
      if (l == 0) M.pre1_bias = bias;
      else b2 = bias;
    }
    M.pre1_b0.upload(M.pre1_bias);
    M.pre2_b.upload(b2);
  }
  M.pre1.upload(swz(M.pre1_host, P, F));
  M.pre2.upload(swz(w2, P, P));
  // transition agent of forward attention (common_layers.py:215-217): ta over [context | query]
  M.trans_agent = h.count("decoder.attention.ta.weight") > 0;
  if (M.trans_agent) {
    M.ta_w.upload(need(h, "decoder.attention.ta.weight", {1, E + S + Q}).d);
    M.ta_b = need(h, "decoder.attention.ta.bias", {1}).d[0];
    TTS_CHECK(S == 0, "transition agent with speaker embeddings is not implemented");
  }
  {
    const auto& wih = need(h, "decoder.attention_rnn.weight_ih", {4 * Q, P + ES}).d;
    const auto& whh = need(h, "decoder.attention_rnn.weight_hh", {4 * Q, Q}).d;
    const auto& bih = need(h, "decoder.attention_rnn.bias_ih", {4 * Q}).d;
    const auto& bhh = need(h, "decoder.attention_rnn.bias_hh", {4 * Q}).d;
    auto wp = slice_cols(wih, 4 * Q, P + ES, 0, P);
    auto wc = slice_cols(wih, 4 * Q, P + ES, P, P + E);
    M.spk_att_h = S ? lstm_tile_rows(slice_cols(wih, 4 * Q, P + ES, P + E, P + ES), Q, S) : std::vector<float>();
    const auto wpt = lstm_tile_rows(wp, Q, P);
    M.att_p.upload(swz(wpt, 4 * Q, P));
    upload_split_rows(M.att_p_x3, wpt, 4 * Q, P);
    auto pre = hcat({{wc.data(), E}, {whh.data(), Q}}, 4 * Q);
    const auto pret = lstm_tile_rows(pre, Q, E + Q);
    M.att_pre.upload(swz(pret, 4 * Q, E + Q));
    upload_split_rows(M.apre_x3, pret, 4 * Q, E + Q);
    std::vector<float> bsum(4 * Q);
    for (int i = 0; i < 4 * Q; ++i) bsum[i] = bih[i] + bhh[i];
    M.att_bias.upload(lstm_tile_rows(bsum, Q, 1));
  }
  {
    const auto& wq = need(h, "decoder.attention.query_layer.linear_layer.weight", {A, Q}).d;
    std::vector<float> t((size_t)Q * A);
    for (int a = 0; a < A; ++a)
      for (int k = 0; k < Q; ++k) t[(size_t)k * A + a] = wq[(size_t)a * Q + k];
    M.WqT.upload(t);
    M.Wloc.upload(need(h, "decoder.attention.location_layer.location_conv1d.weight", {32, 2, 31}).d);
    {
      const auto& wd = need(h, "decoder.attention.location_layer.location_dense.linear_layer.weight", {A, 32}).d;
      std::vector<float> wdT((size_t)32 * A);
      for (int a = 0; a < A; ++a)
        for (int c = 0; c < 32; ++c) wdT[(size_t)c * A + a] = wd[(size_t)a * 32 + c];
      M.Wdense.upload(wdT);
      // location_dense(location_conv(.)) has no biases: one 62-tap filter per attention dim
      const auto& wl = need(h, "decoder.attention.location_layer.location_conv1d.weight", {32, 2, 31}).d;
      std::vector<float> wc((size_t)64 * A, 0.f);
      for (int j = 0; j < 62; ++j)
        for (int a = 0; a < A; ++a) {
          double acc = 0.0;
          for (int cf = 0; cf < 32; ++cf) acc += (double)wd[(size_t)a * 32 + cf] * wl[(size_t)cf * 62 + j];
          wc[(size_t)j * A + a] = (float)acc;
        }
      M.Wcomb.upload(wc);
    }
    M.v.upload(need(h, "decoder.attention.v.linear_layer.weight", {1, A}).d);
    M.bv = need(h, "decoder.attention.v.linear_layer.bias", {1}).d[0];
  }
  {
    const auto& wih_all = need(h, "decoder.decoder_rnn.weight_ih", {4 * D, Q + ES}).d;
    const auto& whh = need(h, "decoder.decoder_rnn.weight_hh", {4 * D, D}).d;
    const auto& bih = need(h, "decoder.decoder_rnn.bias_ih", {4 * D}).d;
    const auto& bhh = need(h, "decoder.decoder_rnn.bias_hh", {4 * D}).d;
    const auto wih = slice_cols(wih_all, 4 * D, Q + ES, 0, Q + E);
    M.spk_dec_h = S ? lstm_tile_rows(slice_cols(wih_all, 4 * D, Q + ES, Q + E, Q + ES), D, S) : std::vector<float>();
    auto w = hcat({{wih.data(), Q + E}, {whh.data(), D}}, 4 * D);
    const auto wt = lstm_tile_rows(w, D, Q + E + D);
    M.dec_w.upload(swz(wt, 4 * D, Q + E + D));
    upload_split_rows(M.dec_x3, wt, 4 * D, Q + E + D);
    std::vector<float> bsum(4 * D);
    for (int i = 0; i < 4 * D; ++i) bsum[i] = bih[i] + bhh[i];
    M.dec_bias.upload(lstm_tile_rows(bsum, D, 1));
  }
  {
    const int NP = F * r_init;
    const auto& wp_all = need(h, "decoder.linear_projection.linear_layer.weight", {NP, D + ES}).d;
    const auto& bp = need(h, "decoder.linear_projection.linear_layer.bias", {NP}).d;
    const auto& ws = need(h, "decoder.stopnet.1.linear_layer.weight", {1, D + NP}).d;
    const auto wp = slice_cols(wp_all, NP, D + ES, 0, D + E);
    // speaker columns of [stop tile | W_p] (stop row = sum_o w_y,o W_p,s[o]), same row order
    M.proj_spk.assign((size_t)(16 + NP) * S, 0.f);
    for (int o = 0; o < NP && S; ++o)
      for (int k = 0; k < S; ++k) {
        const float v = wp_all[(size_t)o * (D + ES) + D + E + k];
        M.proj_spk[(size_t)(16 + o) * S + k] = v;
      }
    for (int k = 0; k < S; ++k) {
      double acc = 0.0;
      for (int o = 0; o < NP; ++o) acc += (double)ws[D + o] * wp_all[(size_t)o * (D + ES) + D + E + k];
      M.proj_spk[k] = (float)acc;
    }

    // stopnet folded through the projection (tacotron2.py:286-295, the stopnet sees all r_init
    // frames): stop = [w_h + W_p,h^T w_y | W_p,ctx^T w_y] . [h | ctx] + (b_s + w_y . b_p)
    std::vector<double> sw(D + E, 0.0);
    for (int k = 0; k < D; ++k) sw[k] = ws[k];
    double sb = need(h, "decoder.stopnet.1.linear_layer.bias", {1}).d[0];
    for (int o = 0; o < NP; ++o) {
      const double wy = ws[D + o];
      for (int k = 0; k < D + E; ++k) sw[k] += wy * wp[(size_t)o * (D + E) + k];
      sb += wy * bp[o];
    }
    // projection weight with the stopnet tile in front: rows [w_stop, 0 x 15, W_p]
    std::vector<float> wx((size_t)(16 + NP) * (D + E), 0.f), bx(16 + NP, 0.f);
    for (int k = 0; k < D + E; ++k) wx[k] = (float)sw[k];
    std::copy(wp.begin(), wp.end(), wx.begin() + (size_t)16 * (D + E));
    bx[0] = (float)sb;
    std::copy(bp.begin(), bp.end(), bx.begin() + 16);
    M.proj_w.upload(swz(wx, 16 + NP, D + E));
    M.proj_b.upload(bx);
    M.proj_rows = std::move(wx);
    M.proj_bias = std::move(bx);
    M.pj_r = -1;
  }
  const int pc[6] = {F, 512, 512, 512, 512, F};
  for (int i = 0; i < 5; ++i) {
    std::vector<float> Wm, b;
    fold_convbn(h, "postnet.convolutions." + std::to_string(i), pc[i], pc[i + 1], 5, Wm, b);
    pack_conv(M.post[i], Wm, b, pc[i], pc[i + 1], 5, 1, 1, pl2);
  }
  HIP_OK(hipDeviceSynchronize());
  M.ready = true;
  c->tws.gen++;  // weights moved: captured graphs are stale
}

template <class T>
bool grow(DevBuf& b, size_t n, long& gen) {
  if (b.ensure(n * sizeof(T))) {
    gen++;
    return true;
  }
  return false;
}

void taco_workspace(tts_ctx* c, int B, int T_max, int S_cap, int r) {
  auto& W = c->tws;
  const int Bp = 16 * ((B + 15) / 16);
  long& g = W.gen;
  grow<int>(W.lens, BMAX, g);
  grow<int>(W.mlens, BMAX, g);
  grow<float>(W.x0, (size_t)B * T_max * 512, g);
  grow<float>(W.ca, (size_t)B * T_max * 512, g);
  grow<float>(W.cb, (size_t)B * T_max * 512, g);
  grow<float>(W.gin, (size_t)B * T_max * 2048, g);
  grow<float>(W.lh, (size_t)2 * 2 * 64 * 256, g);
  grow<float>(W.lc, (size_t)2 * 64 * 256, g);
  grow<float>(W.enc, (size_t)B * T_max * 512, g);
  grow<float>(W.penc, (size_t)B * T_max * 128, g);
  grow<float>(W.p1, (size_t)Bp * 256, g);
  grow<float>(W.pb, (size_t)2 * 64 * 256, g);  // persistent decoder: two K halves of prenet layer 2
  grow<float>(W.gatt, (size_t)Bp * 4096, g);
  grow<float>(W.hatt, (size_t)Bp * 1024, g);
  grow<float>(W.catt, (size_t)Bp * 1024, g);
  grow<float>(W.hdec0, (size_t)Bp * 1024, g);
  grow<float>(W.hdec1, (size_t)Bp * 1024, g);
  grow<float>(W.cdec, (size_t)Bp * 1024, g);
  grow<float>(W.ctx, (size_t)Bp * 512, g);
  grow<float>(W.y, (size_t)Bp * 80 * c->taco.r_init, g);
  grow<float>(W.pq, (size_t)128 * Bp * 128, g);
  grow<float>(W.spart, (size_t)Bp, g);
  grow<float>(W.alpha, (size_t)B * T_max, g);
  grow<float>(W.acum, (size_t)B * T_max, g);
  grow<float>(W.energy, (size_t)B * T_max, g);
  const int nch = (T_max + 15) / 16;
  grow<float>(W.aps, (size_t)B * nch, g);
  grow<float>(W.apf, (size_t)B * nch, g);
  grow<float>(W.apm, (size_t)B * nch, g);
  grow<float>(W.apu, (size_t)B * nch * 512, g);
  grow<unsigned>(W.acnt, BMAX, g);
  grow<int>(W.ctl, 4 + 4 * BMAX, g);
  grow<float>(W.dec, (size_t)B * S_cap * r * 80, g);
  grow<float>(W.align, (size_t)B * S_cap * T_max, g);
  grow<float>(W.stop, (size_t)B * S_cap, g);
  grow<float>(W.pa, (size_t)B * 512 * S_cap * r, g);
  grow<float>(W.pbb, (size_t)B * 512 * S_cap * r, g);
  grow<float>(W.post, (size_t)B * S_cap * r * 80, g);
  grow<int>(W.map, 2 * BMAX, g);
  grow<int>(W.stat, 256, g);
  grow<float>(W.ypart, (size_t)2 * 64 * (1 + 5 * c->taco.r_init + 16) * 16, g);
  grow<unsigned>(W.pbar, PBAR_CAND * BAR_WORDS, g);  // candidate barrier blocks, one picked per launch (MT = 4 .. 1)
  if (W.pslot_base != W.pbar.p) {  // new candidate blocks: calibrated lazily by the first persistent decode
    for (int i = 0; i < PMAX_LAUNCH; ++i) W.pslot[i] = i;
    W.pslot_base = W.pbar.p;
    W.pslot_cal = false;
  }
  grow<float>(W.anorm, (size_t)2 * BMAX, g);
  grow<float>(W.spk, (size_t)64 * 1024, g);
  grow<int>(W.win_idx, 64, g);
  grow<float>(W.gh, 64 * 1024, g);
  grow<float>(W.gmu, 64 * 16, g);
  grow<float>(W.fwd_u, 64, g);
  grow<int64_t>(W.spkid, 64, g);
  W.B = B;
  W.T_max = T_max;
  W.S_cap = S_cap;
  W.r = r;
  W.MT = Bp / 16;
}

DecDev make_dev(tts_ctx* c, int Bact) {
  auto& W = c->tws;
  DecDev d{};
  int* ci = W.ctl.i();
  d.ctl = reinterpret_cast<DecCtl*>(ci);
  d.done = ci + 4;
  d.steps = ci + 4 + BMAX;
  d.status = ci + 4 + 2 * BMAX;
  d.max_steps = ci + 4 + 3 * BMAX;
  d.lens = W.lens.i();
  d.dec_out = W.dec.f();
  d.align_out = W.align.f();
  d.stop_out = W.stop.f();
  d.S_cap = W.S_cap;
  d.T_max = W.T_max;
  d.B = Bact;
  return d;
}

// columns [k0, k0 + K) of a fragment-order activation with Ktot columns
SkSeg seg(const float* base, int Ktot, int k0, int K) {
  SkSeg s;
  s.ptr = base + (long)(k0 / 16) * 256;
  s.ms = 16 * Ktot;
  s.K = K;
  return s;
}

SkJob job0() {
  SkJob j;
  std::memset(&j, 0, sizeof(j));
  return j;
}

// the 5 launches of decoder step j of a chunk (parity j & 1 selects the h_dec buffer) over the
// first MT batch tiles (rows >= 16*MT must all be finished)
void enqueue_step(tts_ctx* c, int j, int which_only, hipStream_t s, int MT) {
  auto& M = c->taco;
  auto& W = c->tws;
  const DecDev d = make_dev(c, std::min(W.B, 16 * MT));
  const int r = W.r, YLD = 80 * M.r_init;
  float* hd_cur = (j & 1) ? W.hdec1.f() : W.hdec0.f();
  float* hd_nxt = (j & 1) ? W.hdec0.f() : W.hdec1.f();
  if (which_only < 0 || which_only == 1) {  // K1: prenet layers 1+2 || stop(t-1)
    SkArgs a{};
    a.njobs = 2;
    a.MT = MT;
    SkJob& J = a.job[0] = job0();  // layer 1 (result kept in LDS)
    J.seg[0] = seg(W.y.f(), YLD, 80 * (r - 1), 80);
    J.nseg = 1;
    J.K = 80;
    J.W = M.pre1.f();
    J.ntiles = 16;
    SkJob& J2 = a.job[1] = job0();  // layer 2
    J2.K = 256;
    J2.W = M.pre2.f();
    J2.ntiles = 16;
    J2.out = W.pb.f();
    J2.out_ld = 256;
    J2.out_frag = 1;
    StopArgs st{};
    st.part = W.spart.f();
    st.threshold = W.thr;
    launch_prenet_stop(a, d, st, j, s);
  }
  if (which_only < 0 || which_only == 3) {  // K2: attention_rnn + partial query projection
    SkArgs a{};
    a.njobs = 1;
    a.MT = MT;
    SkJob& J = a.job[0] = job0();
    J.seg[0] = seg(W.pb.f(), 256, 0, 256);
    J.nseg = 1;
    J.K = 256;
    J.W = M.att_p.f();
    J.ntiles = 256;
    J.epi = EPI_LSTM;
    J.addin = W.gatt.f();
    J.addin_ld = 4096;
    J.h_out = W.hatt.f();
    J.c_state = W.catt.f();
    J.hc_ld = 1024;
    J.WqT = M.WqT.f();
    J.pq_part = W.pq.f();
    J.pq_cap = 128;
    launch_skinny(a, d, j, 2, 4, s);  // 128 workgroups of 8 units: 128 query partials
  }
  if (which_only < 0 || which_only == 4) {  // K3: attention
    AttnArgs p{};
    p.pq_part = W.pq.f();
    p.npq = 128;
    p.Bp = MT * 16;
    p.alpha = W.alpha.f();
    p.alpha_cum = W.acum.f();
    p.Wloc = M.Wloc.f();
    p.WdT = M.Wdense.f();
    p.v = M.v.f();
    p.bv = M.bv;
    p.penc = W.penc.f();
    p.energy = W.energy.f();
    p.enc = W.enc.f();
    p.ctx = W.ctx.f();
    p.part_s = W.aps.f();
    p.part_m = W.apm.f();
    p.part_u = W.apu.f();
    p.counter = reinterpret_cast<unsigned*>(W.acnt.p);
    p.nchmax = (W.T_max + 15) / 16;
    p.softmax = M.softmax;
    launch_attention(p, d, j, s);
  }
  if (which_only < 0 || which_only == 0) {  // K4: decoder_rnn LSTMCell
    SkArgs a{};
    a.njobs = 1;
    a.MT = MT;
    SkJob& J = a.job[0] = job0();
    J.seg[0] = seg(W.hatt.f(), 1024, 0, 1024);
    J.seg[1] = seg(W.ctx.f(), 512, 0, 512);
    J.seg[2] = seg(hd_cur, 1024, 0, 1024);
    J.nseg = 3;
    J.K = 2560;
    J.W = M.dec_w.f();
    J.ntiles = 256;
    J.epi = EPI_LSTM;
    J.bias = M.dec_bias.f();
    J.h_out = hd_nxt;
    J.c_state = W.cdec.f();
    J.hc_ld = 1024;
    launch_skinny(a, d, j, 1, 4, s);
  }
  if (which_only < 0 || which_only == 5) {  // K5: projection + stop logit || next attention_rnn ctx/h part
    SkArgs a{};
    a.njobs = 2;
    a.MT = MT;
    SkJob& J = a.job[0] = job0();
    J.seg[0] = seg(hd_nxt, 1024, 0, 1024);
    J.seg[1] = seg(W.ctx.f(), 512, 0, 512);
    J.nseg = 2;
    J.K = 1536;
    J.W = M.proj_w.f();
    J.ntiles = 1 + 5 * r;  // stopnet tile + the first r frames (tacotron2.py:297)
    J.epi = EPI_STORE;
    J.bias = M.proj_b.f();
    J.out = W.y.f();
    J.out_ld = YLD;
    J.out_frag = 1;
    J.frames_r = r;
    J.lead_stop = 1;
    J.stop_part = W.spart.f();
    SkJob& J2 = a.job[1] = job0();  // (+ biases)
    J2.seg[0] = seg(W.ctx.f(), 512, 0, 512);
    J2.seg[1] = seg(W.hatt.f(), 1024, 0, 1024);
    J2.nseg = 2;
    J2.K = 1536;
    J2.W = M.att_pre.f();
    J2.ntiles = 256;
    J2.epi = EPI_STORE;
    J2.bias = M.att_bias.f();
    J2.out = W.gatt.f();
    J2.out_ld = 4096;
    launch_skinny(a, d, j, 1, 4, s);
  }
}

__global__ void bcast_rows_kernel(const float* src, int n, float* dst, int rows) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n * rows; i += gridDim.x * blockDim.x)
    dst[i] = src[i % n];
}

// Per-row biases of the persistent decoder, one column per thread:
//   out[m][n] = base[n] + sum_e spk[m][e] WT[e][n]   (m < B; rows B..Bp-1 get base[n])
// base = 0 on the attention_rnn / decoder_rnn / processed-inputs columns, the projection bias on
// the projection columns [pj0, N). With no speaker (Es = 0) only the projection columns are built.
constexpr int SPK_BMAX = 64;
// Per-row speaker biases W_s s (+ the projection bias for the projection columns): out[m][n] for
// rows m < Bp. Workgroup = 64 columns x 4 waves, wave q summing the speaker dims e = q, q + 4, ...
// (the speaker values are wave-uniform scalar loads), the 4 partials added in a fixed order
// through LDS. Round 4: the previous form (one column per thread over all dims, 64 accumulators
// predicated on B) ran ~40 workgroups for ~400 us per call.
template <int MB>
__global__ __launch_bounds__(256) void spk_bias_kernel(const float* __restrict__ spk, int B, int Es,
                                                       const float* __restrict__ WT, int N,
                                                       const float* __restrict__ pjb, int pj0, int Bp,
                                                       float* __restrict__ out) {
  __shared__ float red[3][MB][64];
  const int c = threadIdx.x & 63;
  const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n = blockIdx.x * 64 + c;
  const int nc = min(n, N - 1);
  float acc[MB];
#pragma unroll
  for (int m = 0; m < MB; ++m) acc[m] = 0.f;
  for (int e = q; e < Es; e += 4) {
    const float w = WT[(long)e * N + nc];
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const float sv = m < B ? spk[m * Es + e] : 0.f;  // wave-uniform
      acc[m] = fmaf(sv, w, acc[m]);
    }
  }
  if (q > 0) {
#pragma unroll
    for (int m = 0; m < MB; ++m) red[q - 1][m][c] = acc[m];
  }
  __syncthreads();
  if (q != 0 || n >= N) return;
  const float base = n >= pj0 ? pjb[n - pj0] : 0.f;
#pragma unroll
  for (int m = 0; m < MB; ++m)
    if (m < Bp) out[(long)m * N + n] = base + (m < B ? ((acc[m] + red[0][m][c]) + red[1][m][c]) + red[2][m][c] : 0.f);
  for (int m = MB; m < Bp; ++m) out[(long)m * N + n] = base;  // rows past the speaker rows (Bp > MB)
}

// rowmap (optional, device): encoder row b reads ids row rowmap[b] (the decode order)
void run_encoder(tts_ctx* c, const int64_t* ids, int B, int T_max, float* enc_out, hipStream_t s,
                 const int* rowmap = nullptr) {
  auto& M = c->taco;
  auto& W = c->tws;
  const int* lens = W.lens.i();
  launch_embed_gather(ids, T_max, M.emb.f(), M.num_chars, 512, lens, B, W.x0.f(), s, rowmap);
  ConvCall cc;
  cc.lens = lens;
  cc.B = B;
  cc.oflow = x3_flag(c);
  cc.max_q = T_max;
  cc.pad_mode = 0;
  cc.epi = 1;
  cc.s[0] = src_of(W.x0.f(), (long)T_max * 512, 1, 512, 512, 0);
  cc.out = W.ca.f();
  cc.ob = (long)512 * T_max;
  cc.oc = T_max;
  cc.ot = 1;
  run_conv(M.enc[0], cc, s);
  cc.s[0] = src_of(W.ca.f(), (long)512 * T_max, T_max, 1, 512, 0);
  cc.out = W.cb.f();
  run_conv(M.enc[1], cc, s);
  cc.s[0] = src_of(W.cb.f(), (long)512 * T_max, T_max, 1, 512, 0);
  cc.out = W.ca.f();
  run_conv(M.enc[2], cc, s);
  cc.s[0] = src_of(W.ca.f(), (long)512 * T_max, T_max, 1, 512, 0);
  cc.out = W.gin.f();  // (B, T_max, 2048): time-major, so one step's gates of a tile are contiguous
  cc.ob = (long)2048 * T_max;
  cc.oc = 1;
  cc.ot = 2048;
  cc.epi = 0;
  run_conv(M.lstm_in, cc, s);
  // one cooperative launch for the whole recurrence (W.lc then holds its grid-barrier words; its
  // fill zeroes enc_out too); per-step launches when cooperative launch is unavailable or
  // TTS_ENCODER=steps
  const char* e = std::getenv("TTS_ENCODER");
  W.enc_ndom = (e && std::string(e) == "steps")
                   ? 0
                   : launch_bilstm_persist(W.gin.f(), M.whhT.f(), c->gemm_x3 ? M.whhT16.h() : nullptr, lens, T_max, B,
                                           W.lh.f(), reinterpret_cast<unsigned*>(W.lc.p), enc_out, s);
  W.enc_persist = W.enc_ndom > 0;
  if (!W.enc_persist) {
    HIP_OK(hipMemsetAsync(enc_out, 0, (size_t)B * T_max * 512 * 4, s));
    launch_bilstm(W.gin.f(), M.whhT.f(), lens, T_max, B, W.lh.f(), W.lc.f(), enc_out, s);
  }
}

// a persistent BiLSTM whose grid barrier timed out set its error word. The words are read on the
// library stream (ordered after the BiLSTM launch and its arm fill; c->s is non-blocking, so a
// null-stream copy would not be), then the stream is drained before they are looked at.
void check_encoder_barrier(tts_ctx* c) {
  if (!c->tws.enc_persist) return;
  int* pw = c->pinned + 240;  // one error word per recurrence (2 directions x up to 2 row groups)
  const int nd = std::min(c->tws.enc_ndom, ENC_NDOM_MAX);
  pw[0] = pw[1] = pw[2] = pw[3] = 0;
  const unsigned* words = reinterpret_cast<const unsigned*>(c->tws.lc.p);
  for (int i = 0; i < nd; ++i) HIP_OK(hipMemcpyAsync(&pw[i], words + i * BAR_WORDS + 16, 4, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  TTS_CHECK(pw[0] == 0 && pw[1] == 0 && pw[2] == 0 && pw[3] == 0, "persistent BiLSTM: grid barrier timed out (workgroups not co-resident) or preempted past TTS_BARRIER_TIMEOUT_MS; retrying the call is safe)");
}

void run_postnet(tts_ctx* c, const float* dec, long dec_b, const int* mlens, int B, int Mmax_alloc, int max_q,
                 float* out, long out_b, hipStream_t s) {
  auto& M = c->taco;
  auto& W = c->tws;
  ConvCall cc;
  cc.lens = mlens;
  cc.B = B;
  cc.oflow = x3_flag(c);
  cc.max_q = max_q;
  cc.pad_mode = 0;
  cc.epi = 2;
  cc.s[0] = src_of(dec, dec_b, 1, 80, 80, 0);
  cc.out = W.pa.f();
  cc.ob = (long)512 * Mmax_alloc;
  cc.oc = Mmax_alloc;
  cc.ot = 1;
  run_conv(M.post[0], cc, s);
  float* bufs[2] = {W.pa.f(), W.pbb.f()};
  for (int i = 1; i < 4; ++i) {
    cc.s[0] = src_of(bufs[(i - 1) & 1], (long)512 * Mmax_alloc, Mmax_alloc, 1, 512, 0);
    cc.out = bufs[i & 1];
    run_conv(M.post[i], cc, s);
  }
  cc.s[0] = src_of(bufs[1], (long)512 * Mmax_alloc, Mmax_alloc, 1, 512, 0);
  cc.out = out;
  cc.ob = out_b;
  cc.oc = 1;
  cc.ot = 80;
  cc.epi = 0;
  cc.resid = dec;
  cc.rb = dec_b;
  cc.rc = 1;
  cc.rt = 80;
  run_conv(M.post[4], cc, s);
}

template <class T>
__global__ void gather_rows_kernel(const T* __restrict__ src, T* __restrict__ dst, const int* __restrict__ map,
                                   long row) {
  const long i = blockIdx.y;
  const T* sr = src + (long)map[i] * row;
  T* dr = dst + i * row;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < row; e += (long)gridDim.x * blockDim.x) dr[e] = sr[e];
}

// dst row i <- src row map[i], i < B
template <class T>
void gather_rows(const T* src, T* dst, const int* d_map, long row, int B, hipStream_t s) {
  if (row <= 0 || B <= 0) return;
  dim3 g((unsigned)std::min<long>((row + 255) / 256, 64), B);
  gather_rows_kernel<T><<<g, 256, 0, s>>>(src, dst, d_map, row);
  HIP_OK(hipGetLastError());
}

// the decoder's four outputs scattered back to the caller's row order in one launch (entry z)
struct Gather4 {
  const float* src[4];
  float* dst[4];
  long row[4];
};
__global__ void gather4_rows_kernel(Gather4 g, const int* __restrict__ map) {
  const int z = blockIdx.z;
  const long row = g.row[z], i = blockIdx.y;
  const float* __restrict__ sr = g.src[z] + (long)map[i] * row;
  float* __restrict__ dr = g.dst[z] + i * row;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < row; e += (long)gridDim.x * blockDim.x) dr[e] = sr[e];
}
void gather4_rows(const Gather4& g, const int* d_map, int B, hipStream_t s) {
  long mx = 0;
  for (int z = 0; z < 4; ++z) mx = std::max(mx, g.row[z]);
  if (mx <= 0 || B <= 0) return;
  gather4_rows_kernel<<<dim3((unsigned)std::min<long>((mx + 255) / 256, 64), B, 4), 256, 0, s>>>(g, d_map);
  HIP_OK(hipGetLastError());
}

// Per-call host arguments as kernel arguments (one launch instead of three pageable uploads):
// decode order and its inverse, lengths in decode order, and the decoder control block
// [base, all_done, active_tiles, pad | done | steps | status | max_steps] (DecCtl + BMAX each)
struct TacoSetup {
  int B, MT;
  int perm[BMAX], inv[BMAX], lens[BMAX], max_steps[BMAX];
};
__global__ void taco_setup_kernel(TacoSetup a, int* map, int* lens, int* ctl, unsigned* zero_flag) {
  if (zero_flag && threadIdx.x == 0) *zero_flag = 0u;  // a fused call's range flag (no separate fill)
  for (int e = threadIdx.x; e < 4 + 4 * BMAX; e += blockDim.x) {
    const int ms = e - 4 - 3 * BMAX;
    ctl[e] = e == 2 ? a.MT : (ms >= 0 && ms < a.B ? a.max_steps[ms] : 0);
  }
  const int i = threadIdx.x;
  if (i < a.B) {
    map[i] = a.perm[i];
    map[BMAX + i] = a.inv[i];
    lens[i] = a.lens[i];
  }
}

// element (m, k) of a fragment-order activation; ps: published pre-split (decoder_persist.hip
// stc_quad_x3: the f16 hi / lo halves of k & ~3 .. + 3 as [hi 4 | lo 4] in their 16 bytes), read back
// as hi + 2^-11 lo, the value the decoder's split-f16 GEMMs consumed
__device__ __forceinline__ float frag_value(const float* p, int m, int k, int K, int ps) {
  if (!ps) return p[frag_idx(m, k, K)];
  const _Float16* q = reinterpret_cast<const _Float16*>(p + frag_idx(m, k & ~3, K));
  return (float)q[k & 3] + (float)q[4 + (k & 3)] * SPLIT_INV;
}

// decoder state in the caller's row order (tts_taco_decoder_state): fragment-order activations
// (h_att, h_dec, ctx) and row-major cells / attention rows of decode row inv[b] -> row b
__global__ void taco_state_kernel(const float* hatt, const float* catt, const float* hdec, const float* cdec,
                                  const float* ctx, const float* alpha, const float* acum, const int* inv, int T_max,
                                  int ps, float* o_ha, float* o_ca, float* o_hd, float* o_cd, float* o_ctx,
                                  float* o_al, float* o_ac) {
  const int b = blockIdx.y, m = inv[b];
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < 1024; k += gridDim.x * blockDim.x) {
    if (o_ha) o_ha[(long)b * 1024 + k] = frag_value(hatt, m, k, 1024, ps);
    if (o_ca) o_ca[(long)b * 1024 + k] = catt[(long)m * 1024 + k];
    if (o_hd) o_hd[(long)b * 1024 + k] = frag_value(hdec, m, k, 1024, ps);
    if (o_cd) o_cd[(long)b * 1024 + k] = cdec[(long)m * 1024 + k];
    if (o_ctx && k < 512) o_ctx[(long)b * 512 + k] = frag_value(ctx, m, k, 512, ps);
  }
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < T_max; k += gridDim.x * blockDim.x) {
    if (o_al) o_al[(long)b * T_max + k] = alpha[(long)m * T_max + k];
    if (o_ac) o_ac[(long)b * T_max + k] = acum[(long)m * T_max + k];
  }
}

// decode-order mel lengths for the postnet (steps * r), from the decoder results on the device
__global__ void taco_mlens_kernel(const int* ctl, int B, int r, int* mlens) {
  const int i = threadIdx.x;
  if (i < B) mlens[i] = ctl[4 + BMAX + i] * r;
}

// gather every status word the host checks after a Tacotron2 call into one block (TS_* layout)
struct DecSlots {
  int v[PMAX_LAUNCH];
};
// A fused call (vlens set) also writes the vocoder's mel lengths in caller order, steps * r of
// decode row inv[b], raised to Lmin where shorter (TS_VERR: the call fails)
__global__ void taco_status_kernel(const unsigned* enc_bar, int nenc, const unsigned* dec_bar, DecSlots dslot, int ndec,
                                   const int* ctl, const unsigned* flag, int* st, int B, const int* inv, int r,
                                   int Lmin, int* vlens) {
  const int i = threadIdx.x;
  int short_row = 0;
  if (vlens && i < B) {
    int L = ctl[4 + BMAX + inv[i]] * r;
    if (L < Lmin) {
      short_row = 1;
      L = Lmin;
    }
    vlens[i] = L;
  }
  short_row = __syncthreads_or(short_row);
  if (i == 0) st[TS_VERR] = short_row;
  if (i < 3 * BMAX) st[TS_RES + i] = ctl[4 + i];
  if (i < ENC_NDOM_MAX) st[TS_ENC + i] = enc_bar && i < nenc ? (int)enc_bar[i * BAR_WORDS + 16] : 0;
  if (i < PMAX_LAUNCH) {
    st[TS_DEC + i] = dec_bar && i < ndec ? (int)dec_bar[dslot.v[i] * BAR_WORDS + 16] : 0;
  }
  if (i == 0) st[TS_FLAG] = flag ? (int)*flag : 0;
}

// CHUNK-step graph for batch tile count MT (captured once per configuration)
hipGraphExec_t step_graph(tts_ctx* c, int MT, hipStream_t s) {
  auto& W = c->tws;
  if (W.graphs[MT]) return W.graphs[MT];
  hipGraph_t g;
  HIP_OK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  try {
    for (int j = 0; j < CHUNK; ++j) enqueue_step(c, j, -1, s, MT);
    launch_dec_advance(reinterpret_cast<DecCtl*>(W.ctl.p), CHUNK, s);
  } catch (...) {
    hipGraph_t tmp;
    (void)hipStreamEndCapture(s, &tmp);
    throw;
  }
  HIP_OK(hipStreamEndCapture(s, &g));
  HIP_OK(hipGraphInstantiate(&W.graphs[MT], g, nullptr, nullptr, 0));
  HIP_OK(hipGraphDestroy(g));
  return W.graphs[MT];
}

// projection job tiles of the persistent decoder for reduction factor r: the stop tile, the
// 5r tiles of the first r frames, and prenet layer 1 folded through the last frame's rows
// (relu(W1 y_last) = relu(W1 W_p,last [h|ctx] + W1 b_p,last); layer 1 has no bias), fold in double
void build_pj(tts_ctx* c, int r) {
  auto& M = c->taco;
  if (M.pj_r == r) return;
  const int K = 1536, F = 80, P = 256;
  const int rows_p = 16 + F * r;
  std::vector<float> rows((size_t)(rows_p + P) * K), bias(rows_p + P);
  std::memcpy(rows.data(), M.proj_rows.data(), (size_t)rows_p * K * sizeof(float));
  std::memcpy(bias.data(), M.proj_bias.data(), (size_t)rows_p * sizeof(float));
  const float* wl = M.proj_rows.data() + (size_t)(16 + F * (r - 1)) * K;  // W_p rows of the last frame
  const float* bl = M.proj_bias.data() + 16 + F * (r - 1);
  std::vector<double> acc(K);
  for (int k = 0; k < P; ++k) {
    std::fill(acc.begin(), acc.end(), 0.0);
    double bs = 0.0;
    for (int i = 0; i < F; ++i) {
      const double w1 = M.pre1_host[(size_t)k * F + i];
      const float* row = wl + (size_t)i * K;
      for (int j = 0; j < K; ++j) acc[j] += w1 * row[j];
      bs += w1 * bl[i];
    }
    float* dst = rows.data() + (size_t)(rows_p + k) * K;
    for (int j = 0; j < K; ++j) dst[j] = (float)acc[j];
    bias[rows_p + k] = (float)(bs + (M.pre1_bias.empty() ? 0.0 : (double)M.pre1_bias[k]));
  }
  M.pj_w.upload(swz(rows, rows_p + P, K));
  upload_split_rows(M.pj_x3, rows, rows_p + P, K);
  M.pj_b.upload(bias);
  if (M.spk_dim) {
    // speaker columns, transposed [Es][att 4096 | dec 4096 | penc 128 | pj rows_p + P]
    const int S = M.spk_dim, N = 4096 + 4096 + 128 + rows_p + P;
    std::vector<float> wt((size_t)S * N);
    auto put = [&](const std::vector<float>& rm, int n0, int nrows) {
      for (int i = 0; i < nrows; ++i)
        for (int e = 0; e < S; ++e) wt[(size_t)e * N + n0 + i] = rm[(size_t)i * S + e];
    };
    put(M.spk_att_h, 0, 4096);
    put(M.spk_dec_h, 4096, 4096);
    put(M.spk_penc_h, 8192, 128);
    put(M.proj_spk, 8320, rows_p);
    const float* sl = M.proj_spk.data() + (size_t)(16 + F * (r - 1)) * S;  // last frame's rows
    for (int k = 0; k < P; ++k)
      for (int e = 0; e < S; ++e) {
        double acc = 0.0;
        for (int i = 0; i < F; ++i) acc += (double)M.pre1_host[(size_t)k * F + i] * sl[(size_t)i * S + e];
        wt[(size_t)e * N + 8320 + rows_p + k] = (float)acc;
      }
    M.spk_wT.upload(wt);
  }
  M.pj_r = r;
}

bool use_persistent(tts_ctx* c) {
  const char* e = std::getenv("TTS_DECODER");
  if (e && std::string(e) == "graph") return false;
  return c->tws.MT <= PMAX_LAUNCH && persist_supported(c->device);
}

// the whole decode as one cooperative launch per batch-tile count (decoder_persist.hip)
void run_persistent(tts_ctx* c, int r, float thr, hipStream_t s) {
  auto& M = c->taco;
  auto& W = c->tws;
  build_pj(c, r);
  PArgs a{};
  a.dec_w = M.dec_w.f();
  a.dec_b = M.dec_bias.f();
  a.apre_w = M.att_pre.f();
  a.apre_b = M.att_bias.f();
  a.attp_w = M.att_p.f();
  a.x3flag = x3_flag(c);  // null in fp32 mode
  // split-f16 decoder GEMM parts: only with every split weight set in range, and Q = 1024,
  // E = 512, prenet 256 (the kernel's fixed geometry, checked by build_pj's callers)
  const bool dx3 = a.x3flag && M.att_p_x3.p && M.dec_x3.p && M.apre_x3.p && M.pj_x3.p && !std::getenv("TTS_DECODER_F32");
  a.attp_x3 = dx3 ? M.att_p_x3.h() : nullptr;
  a.dec_x3 = dx3 ? M.dec_x3.h() : nullptr;
  a.apre_x3 = dx3 ? M.apre_x3.h() : nullptr;
  a.pj_x3 = dx3 ? M.pj_x3.h() : nullptr;
  a.pj_w = M.pj_w.f();
  a.pj_b = M.pj_b.f();
  {  // per-row biases: projection (always), speaker columns when the model has them
    const int YP = (1 + 5 * r + 16) * 16;
    const int N = M.spk_dim ? 8320 + YP : YP;
    const int pj0 = M.spk_dim ? 8320 : 0;
    const int Bp = W.MT * 16;
    grow<float>(W.spkb, (size_t)64 * (8320 + 112 * 16), W.gen);
    TTS_CHECK(W.B <= SPK_BMAX || !M.spk_dim, "multi-speaker decoding: at most 64 utterances per call");
    const int Bs = M.spk_dim ? W.B : 0;
    TTS_CHECK(M.spk_dim <= 512, "speaker vectors of at most 512 dims");
    // Graves with speakers: the projection columns hold W_s s alone; the kernel adds the bias and
    // scales W_s s by the step's sum of attention weights (PArgs::spk_scale)
    a.spk_scale = M.graves && M.spk_dim ? 1 : 0;
    {
      const float* wt = M.spk_dim ? M.spk_wT.f() : nullptr;
      const int es = M.spk_dim, p0 = a.spk_scale ? N : pj0;
      const dim3 g((N + 63) / 64);
      if (Bs <= 16) spk_bias_kernel<16><<<g, 256, 0, s>>>(W.spk.f(), Bs, es, wt, N, M.pj_b.f(), p0, Bp, W.spkb.f());
      else if (Bs <= 32) spk_bias_kernel<32><<<g, 256, 0, s>>>(W.spk.f(), Bs, es, wt, N, M.pj_b.f(), p0, Bp, W.spkb.f());
      else spk_bias_kernel<64><<<g, 256, 0, s>>>(W.spk.f(), Bs, es, wt, N, M.pj_b.f(), p0, Bp, W.spkb.f());
    }
    HIP_OK(hipGetLastError());
    a.spk_ld = N;
    a.pjb_rows = W.spkb.f() + pj0;
    a.spk_att = M.spk_dim ? W.spkb.f() : nullptr;
    a.spk_dec = M.spk_dim ? W.spkb.f() + 4096 : nullptr;
    a.spk_penc = M.spk_dim ? W.spkb.f() + 8192 : nullptr;
  }
  // decoder variants
  a.pre1_b0 = M.prenet_bn ? M.pre1_b0.f() : nullptr;
  a.pre2_b = M.prenet_bn ? M.pre2_b.f() : nullptr;
  a.win = M.windowing;
  a.fwd = M.forward_attn;
  a.trans = M.forward_attn && M.trans_agent;
  a.fwd_mask = M.forward_attn && M.forward_attn_mask;
  a.ta_w = M.trans_agent ? M.ta_w.f() : nullptr;
  a.ta_b = M.ta_b;
  a.win_idx = W.win_idx.i();
  a.fwd_u = W.fwd_u.f();
  a.part_f = W.apf.f();
  if (M.windowing) HIP_OK(hipMemsetAsync(W.win_idx.p, 0xff, 64 * 4, s));  // -1: before the first step
  a.gK = M.graves ? M.graves_K : 0;
  a.na1_w = M.na1_w.f();
  a.na1_b = M.na1_b.f();
  a.na2_w = M.na2_w.f();
  a.na2_b = M.na2_b.f();
  a.gh = W.gh.f();
  a.gmu = W.gmu.f();
  if (M.graves) HIP_OK(hipMemsetAsync(W.gmu.p, 0, 64 * 16 * 4, s));  // mu_prev = 0 (common_layers.py:143)
  if (M.forward_attn) {
    static const std::vector<float> half(64, 0.5f);  // u = 0.5 (common_layers.py:241)
    HIP_OK(hipMemcpyAsync(W.fwd_u.p, half.data(), 64 * 4, hipMemcpyHostToDevice, s));
  }
  a.pre2_w = M.pre2.f();
  a.WqT = M.WqT.f();
  a.Wcomb = M.Wcomb.f();
  a.v = M.v.f();
  a.bv = M.bv;
  a.nt_proj = 1 + 5 * r;
  a.ntj = a.nt_proj + 16;
  a.r = r;
  a.penc = W.penc.f();
  a.enc = W.enc.f();
  a.ypart = W.ypart.f();
  a.pb = W.pb.f();
  a.gatt = W.gatt.f();
  a.hatt = W.hatt.f();
  a.catt = W.catt.f();
  a.hdec0 = W.hdec0.f();
  a.hdec1 = W.hdec1.f();
  a.cdec = W.cdec.f();
  a.ctx = W.ctx.f();
  a.pq = W.pq.f();
  a.alpha = W.alpha.f();
  a.acum = W.acum.f();
  a.energy = W.energy.f();
  a.part_s = W.aps.f();
  a.part_m = W.apm.f();
  a.part_u = W.apu.f();
  a.counter = reinterpret_cast<unsigned*>(W.acnt.p);
  a.nchmax = (W.T_max + persist_attn_tc() - 1) / persist_attn_tc();
  a.anorm = W.anorm.f();
  a.defer_align = persist_defer_ok(W.B * a.nchmax) && !std::getenv("TTS_ALIGN_IN_P4");
  a.softmax = M.softmax;
  a.thr = thr;
  a.bar = reinterpret_cast<unsigned*>(W.pbar.p);
  // TTS_PTRACE=<file>: phase timestamps of 8 steps from step TTS_PTRACE_T0 (default 100)
  DevBuf& trace_buf = W.trace;
  const char* tr = std::getenv("TTS_PTRACE");
  TTS_CHECK(!tr || persist_trace_built(), "TTS_PTRACE needs a library built with -DTTS_PHASE_TRACE "
                                          "(tools/build_variants.sh trace -DTTS_PHASE_TRACE; TTSHIP_LIB=tools/var/lib_trace.so)");
  if (tr) {
    trace_buf.ensure((size_t)8 * 24 * 256 * 8);
    HIP_OK(hipMemsetAsync(trace_buf.p, 0, (size_t)8 * 24 * 256 * 8, s));
    a.trace = static_cast<unsigned long long*>(trace_buf.p);
    a.atrace = a.trace + (size_t)8 * 16 * 256;
    const char* t0 = std::getenv("TTS_PTRACE_T0");
    a.trace_t0 = t0 ? std::atoi(t0) : 100;
  }
  // TTS_PTRACE_LAUNCH: which launch of the MT cascade is traced (default 0, the first)
  const int trace_li = [] {
    const char* e = std::getenv("TTS_PTRACE_LAUNCH");
    return e ? std::atoi(e) : 0;
  }();
  unsigned long long* const trace_p = a.trace;
  unsigned long long* const atrace_p = a.atrace;
  static const bool xdiag = std::getenv("TTS_DIAG_XCC") != nullptr;
  DevBuf& xdiag_buf = W.xdiag;
  if (xdiag) xdiag_buf.ensure((size_t)PMAX_LAUNCH * 256 * 4);
  c->dec_nlaunch = 0;
  c->dec_presplit = persist_presplit(a);
  for (int mt = W.MT; mt >= 1; --mt) {
    const int li = W.MT - mt;  // launch index: its barrier block (armed in taco_infer's state fill)
    a.bar = reinterpret_cast<unsigned*>(W.pbar.p) + BAR_WORDS * W.pslot[li];
    a.base_out = W.stat.i() + TS_END + li;
    a.D = make_dev(c, std::min(W.B, 16 * mt));
    a.trace = li == trace_li ? trace_p : nullptr;
    a.atrace = li == trace_li ? atrace_p : nullptr;
    a.diag = xdiag ? static_cast<unsigned*>(xdiag_buf.p) + 256 * li : nullptr;
    // launch timing from the dispatches themselves: ev_dec[0] at the first launch's start, ev_dec[i + 1]
    // at launch i's end (event-record packets between the launches cost ~5 us of idle each)
    launch_persist_decoder(a, mt, s, false, li == 0 ? c->ev_dec[0] : nullptr, c->ev_dec[li + 1]);
    if (tr && li == trace_li) {  // one launch is traced
      HIP_OK(hipStreamSynchronize(s));
      std::vector<unsigned long long> h((size_t)8 * 24 * 256);
      HIP_OK(hipMemcpy(h.data(), trace_buf.p, h.size() * 8, hipMemcpyDeviceToHost));
      if (FILE* fp = std::fopen(tr, "wb")) {
        std::fwrite(h.data(), 8, h.size(), fp);
        std::fclose(fp);
      }
      a.trace = nullptr;
      a.atrace = nullptr;
      tr = nullptr;
    }
    c->dec_nlaunch++;
  }
  a.diag = nullptr;
  if (xdiag) {  // TTS_DIAG_XCC: print each launch's workgroup -> XCD map and the hand-off addresses
    HIP_OK(hipStreamSynchronize(s));
    std::vector<unsigned> h((size_t)PMAX_LAUNCH * 256);
    HIP_OK(hipMemcpy(h.data(), xdiag_buf.p, h.size() * 4, hipMemcpyDeviceToHost));
    for (int li = 0; li < c->dec_nlaunch; ++li) {
      std::fprintf(stderr, "TTS_DIAG_XCC launch %d: wg0 xcc %u, wg0..15:", li, h[li * 256]);
      for (int k = 0; k < 16; ++k) std::fprintf(stderr, " %u", h[li * 256 + k]);
      std::fprintf(stderr, "\n");
    }
    std::fprintf(stderr, "TTS_DIAG_XCC addresses: bar %p pq %p hatt %p ctx %p hdec0 %p pb %p\n", (void*)W.pbar.p,
                 (void*)a.pq, (void*)a.hatt, (void*)a.ctx, (void*)a.hdec0, (void*)a.pb);
  }
}

// the vocoder half of a fused Tacotron2 + MB-MelGAN call: the decode's status kernel writes the
// vocoder's lengths into vlens (device, caller order), and enqueue() launches the vocoder on them
// before the host waits for the status words, so the GPU runs both models back to back
constexpr const char* VOC_SHORT_MSG =
    "MB-MelGAN: a decoded mel is shorter than the vocoder's reflection pads allow (ReflectionPad1d(3): mel frames "
    "+ 2*padding must be >= 4; a residual stack's dilation must be < the first stage's length)";
struct FusedVoc {
  int* vlens;
  int Lmin;
  std::function<void()> enqueue;
};

void taco_infer(tts_ctx* c, const int64_t* ids, const int32_t* h_lens, int B, int T_max, int r,
                const int32_t* h_max_steps, int S_cap, float thr, float* d_dec, float* d_post, float* d_align,
                float* d_stop, int32_t* h_steps, int32_t* h_status, void* stream,
                const int64_t* d_spk_ids = nullptr, const float* d_spk_emb = nullptr, const FusedVoc* fv = nullptr) {
  auto& M = c->taco;
  TTS_CHECK(M.ready, "tacotron2 weights not finalized");
  TTS_CHECK(B >= 1 && B <= BMAX, "B must be in [1, 64]");
  TTS_CHECK(T_max >= 1 && T_max <= 4096, "T_max must be in [1, 4096]");
  TTS_CHECK(r >= 1 && r <= M.r_init, "r must be in [1, r_init]");
  int max_ms = 0;
  for (int b = 0; b < B; ++b) {
    TTS_CHECK(h_lens[b] >= 1 && h_lens[b] <= T_max, "lens out of range");
    TTS_CHECK(h_max_steps[b] >= 1, "max_decoder_steps must be >= 1");
    max_ms = std::max(max_ms, (int)h_max_steps[b]);
  }
  TTS_CHECK(S_cap >= max_ms, "S_cap < max(max_steps)");
  taco_workspace(c, B, T_max, S_cap, r);
  auto& W = c->tws;
  hipStream_t s = c->s;
  enter(c, stream);
  // Decode order: longest expected first (max_decoder_steps, then text length), so the rows still
  // decoding at the end sit in the first batch tiles and the step can shrink to fewer tiles.
  // Every row is independent, so the order changes nothing but speed; outputs are scattered back.
  std::vector<int> perm(B), inv(B);
  for (int b = 0; b < B; ++b) perm[b] = b;
  std::stable_sort(perm.begin(), perm.end(), [&](int x, int y) {
    if (h_max_steps[x] != h_max_steps[y]) return h_max_steps[x] > h_max_steps[y];
    return h_lens[x] > h_lens[y];
  });
  for (int i = 0; i < B; ++i) inv[perm[i]] = i;
  // decode order, its inverse, lengths and the control block (base = 0, all_done = 0,
  // active_tiles = MT, done/steps/status = 0, max_steps) in one launch, as kernel arguments
  {
    TacoSetup ta{};
    ta.B = B;
    ta.MT = W.MT;
    for (int i = 0; i < B; ++i) {
      ta.perm[i] = perm[i];
      ta.inv[i] = inv[i];
      ta.lens[i] = h_lens[perm[i]];
      ta.max_steps[i] = h_max_steps[perm[i]];
    }
    taco_setup_kernel<<<1, 256, 0, s>>>(ta, W.map.i(), W.lens.i(), W.ctl.i(), fv ? x3_flag(c) : nullptr);
    HIP_OK(hipGetLastError());
  }
  int* d_map = W.map.i();
  W.thr = thr;
  // speaker vectors in decode order: external embeddings, or rows of the learned table
  TTS_CHECK(!M.variant() || use_persistent(c), "BN prenet / attention windowing / forward / Graves attention run on "
                                               "the persistent decoder only (<= 64 utterances per call on a 256-CU "
                                               "device)");
  if (M.spk_dim) {
    TTS_CHECK(d_spk_ids || d_spk_emb, "multi-speaker model: speaker ids or speaker embeddings are required");
    TTS_CHECK(use_persistent(c), "multi-speaker decoding runs on the persistent decoder only (<= 64 utterances "
                                 "per call on a 256-CU device)");
    if (d_spk_emb) {
      gather_rows<float>(d_spk_emb, W.spk.f(), d_map, M.spk_dim, B, s);
    } else {
      TTS_CHECK(M.num_spk > 0, "model has no speaker_embedding table: pass speaker embeddings");
      gather_rows<int64_t>(d_spk_ids, reinterpret_cast<int64_t*>(W.spkid.p), d_map, 1, B, s);
      launch_embed_gather(reinterpret_cast<const int64_t*>(W.spkid.p), 1, M.spk_table.f(), M.num_spk, M.spk_dim,
                          W.lens.i(), B, W.spk.f(), s);
    }
  }
  // encoder + processed inputs
  run_encoder(c, ids, B, T_max, W.enc.f(), s, d_map);
  {
    ConvCall cc;
    cc.lens = W.lens.i();
    cc.B = B;
    cc.oflow = x3_flag(c);
    cc.max_q = T_max;
    cc.s[0] = src_of(W.enc.f(), (long)T_max * 512, 1, 512, 512, 0);
    cc.out = W.penc.f();
    cc.ob = (long)T_max * 128;
    cc.oc = 1;
    cc.ot = 128;
    run_conv(M.penc, cc, s);
  }
  // decoder state
  const int Bp = W.MT * 16;
  const bool persist = use_persistent(c);
  if (persist && !W.pslot_cal) {  // ordered after the caller's work (enter above) and this call's encoder
    pick_barrier_blocks(reinterpret_cast<unsigned*>(W.pbar.p), PBAR_CAND, PMAX_LAUNCH, W.pslot, s);
    W.pslot_cal = true;
  }
  {
    FillList f;  // decoder state and outputs zeroed in one launch (the postnet output too)
    f.add(W.catt.p, (size_t)Bp * 1024 * 4);
    f.add(W.hatt.p, (size_t)Bp * 1024 * 4);
    f.add(W.hdec0.p, (size_t)Bp * 1024 * 4);
    f.add(W.hdec1.p, (size_t)Bp * 1024 * 4);
    f.add(W.cdec.p, (size_t)Bp * 1024 * 4);
    f.add(W.ctx.p, (size_t)Bp * 512 * 4);
    f.add(W.y.p, (size_t)Bp * 80 * M.r_init * 4);
    f.add(W.alpha.p, (size_t)B * T_max * 4);
    f.add(W.acum.p, (size_t)B * T_max * 4);
    f.add(W.dec.p, (size_t)B * S_cap * r * 80 * 4);
    f.add(W.align.p, (size_t)B * S_cap * T_max * 4);
    f.add(W.stop.p, (size_t)B * S_cap * 4);
    f.add(W.acnt.p, BMAX * sizeof(unsigned));
    f.add(W.post.p, (size_t)B * S_cap * r * 80 * 4);
    if (persist)
      for (int li = 0; li < W.MT; ++li) add_barrier_fills(f, reinterpret_cast<unsigned*>(W.pbar.p) + BAR_WORDS * W.pslot[li], 1);
    launch_fills(f, s);
  }
  bcast_rows_kernel<<<256, 256, 0, s>>>(M.att_bias.f(), 4096, W.gatt.f(), Bp);
  HIP_OK(hipGetLastError());
  c->dec_path = persist ? 1 : 0;
  if (persist) {
    run_persistent(c, r, thr, s);
  } else {
  // step graphs, cached per configuration / buffer generation
  if (W.graph_gen != W.gen || W.gB != B || W.gT != T_max || W.gS != S_cap || W.gr != r || W.gthr != thr) {
    for (auto& ge : W.graphs)
      if (ge) {
        HIP_OK(hipGraphExecDestroy(ge));
        ge = nullptr;
      }
    W.graph_gen = W.gen;
    W.gB = B;
    W.gT = T_max;
    W.gS = S_cap;
    W.gr = r;
    W.gthr = thr;
  }
  for (int mt = 1; mt <= W.MT; ++mt) step_graph(c, mt, s);
  // run chunks until every utterance is done (checked one chunk behind) or t > max steps; drop
  // to fewer batch tiles once the trailing rows have all finished
  const int chunks_max = max_ms / CHUNK + 1;  // covers t = max_ms (stop of the last step)
  bool done = false;
  int mt = W.MT;
  for (int ch = 0; ch < chunks_max && !done; ++ch) {
    HIP_OK(hipGraphLaunch(W.graphs[mt], s));
    HIP_OK(hipMemcpyAsync(&c->pinned[2 * (ch & 1)], &reinterpret_cast<DecCtl*>(W.ctl.p)->all_done, 8,
                          hipMemcpyDeviceToHost, s));
    HIP_OK(hipEventRecord(c->ev_chunk[ch & 1], s));
    if (ch >= 1) {
      HIP_OK(hipEventSynchronize(c->ev_chunk[(ch - 1) & 1]));
      const int* pv = &c->pinned[2 * ((ch - 1) & 1)];
      if (pv[0]) done = true;
      else if (pv[1] >= 1 && pv[1] < mt) mt = pv[1];
    }
  }
  }
  // postnet over each row's own frames: lengths from the decoder results on the device, grid sized
  // by S_cap (tiles past a row's length exit at entry), so the decode needs no host round trip
  taco_mlens_kernel<<<1, 64, 0, s>>>(W.ctl.i(), B, r, W.mlens.i());
  HIP_OK(hipGetLastError());
  const long fb = (long)S_cap * r * 80;  // W.post was zeroed with the decoder state
  run_postnet(c, W.dec.f(), fb, W.mlens.i(), B, S_cap * r, S_cap * r, W.post.f(), fb, s);
  // scatter back to the caller's row order: output row b <- decode row inv[b]
  gather4_rows(Gather4{{W.post.f(), W.dec.f(), W.align.f(), W.stop.f()}, {d_post, d_dec, d_align, d_stop},
                       {fb, fb, (long)S_cap * T_max, (long)S_cap}},
               d_map + BMAX, B, s);
  // one host round trip per call: barrier error words, per-row results, range flag, launch steps
  {
    const unsigned* lc = reinterpret_cast<const unsigned*>(W.lc.p);
    taco_status_kernel<<<1, 256, 0, s>>>(W.enc_persist ? lc : nullptr, W.enc_ndom,
                                         persist ? reinterpret_cast<const unsigned*>(W.pbar.p) : nullptr,
                                         DecSlots{{W.pslot[0], W.pslot[1], W.pslot[2], W.pslot[3]}}, c->dec_nlaunch, W.ctl.i(), c->gemm_x3 ? x3_flag(c) : nullptr, W.stat.i(),
                                         B, d_map + BMAX, r, fv ? fv->Lmin : 0, fv ? fv->vlens : nullptr);
    HIP_OK(hipGetLastError());
    int* pin = c->pinned;
    HIP_OK(hipMemcpyAsync(pin + TS_ENC, W.stat.i() + TS_ENC, (TS_N - TS_ENC) * 4, hipMemcpyDeviceToHost, s));
    if (fv) {  // the vocoder goes in behind the status words; the host waits for the words only
      HIP_OK(hipEventRecord(c->ev_status, s));
      fv->enqueue();
      HIP_OK(hipEventSynchronize(c->ev_status));
    } else {
      HIP_OK(hipStreamSynchronize(s));
    }
    TTS_CHECK(!W.enc_persist || (pin[TS_ENC] == 0 && pin[TS_ENC + 1] == 0 && pin[TS_ENC + 2] == 0 && pin[TS_ENC + 3] == 0),
              "persistent BiLSTM: grid barrier timed out (workgroups not co-resident) or preempted past "
              "TTS_BARRIER_TIMEOUT_MS; retrying the call is safe)");
    TTS_CHECK(!persist || (pin[TS_DEC] == 0 && pin[TS_DEC + 1] == 0 && pin[TS_DEC + 2] == 0 && pin[TS_DEC + 3] == 0),
              "persistent decoder: grid barrier timed out (workgroups not co-resident) or preempted past "
              "TTS_BARRIER_TIMEOUT_MS; retrying the call is safe)");
    if (c->gemm_x3) {  // with_x3_fallback reads the flag from here
      pin[12] = pin[TS_FLAG];
      c->flag_read = true;
    }
    for (int i = 0; i < PMAX_LAUNCH; ++i) c->dec_end[i] = persist && i < c->dec_nlaunch ? pin[TS_END + i] : 0;
    TTS_CHECK(!fv || pin[TS_VERR] == 0, VOC_SHORT_MSG);
  }
  const int* res = c->pinned + TS_RES;
  for (int i = 0; i < B; ++i) {
    TTS_CHECK(res[i] == 1, "decoder did not finish an utterance (internal error)");
    const int b = perm[i];
    h_steps[b] = res[BMAX + i];
    h_status[b] = res[2 * BMAX + i];
  }
  if (fv)  // the caller's stream waits for the decode's outputs here, for the vocoder at finish
    HIP_OK(hipStreamWaitEvent((hipStream_t)stream, c->ev_status, 0));
  else
    leave(c, stream);
  c->last_B = B;
  c->last_T = T_max;
  c->last_S = S_cap;
  c->last_r = r;
}

// ---------------------------------------------------------------- MelGAN -------------
std::vector<float> wn_weight(const HostMap& m, const std::string& name, std::vector<int64_t> shape) {
  auto itw = m.find(name + ".weight");
  if (itw != m.end()) return need(m, name + ".weight", shape).d;
  const auto& v = need(m, name + ".weight_v", shape).d;
  std::vector<int64_t> gshape(shape.size(), 1);
  gshape[0] = shape[0];
  const auto& g = need(m, name + ".weight_g", gshape).d;
  const size_t per = v.size() / shape[0];
  std::vector<float> w(v.size());
  for (int64_t o = 0; o < shape[0]; ++o) {
    double n = 0;
    for (size_t i = 0; i < per; ++i) n += (double)v[o * per + i] * v[o * per + i];
    n = std::sqrt(n);
    const double sc = g[o] / n;
    for (size_t i = 0; i < per; ++i) w[o * per + i] = (float)(v[o * per + i] * sc);
  }
  return w;
}

void melgan_finalize(tts_ctx* c, int in_ch, int out_ch, int base, const int32_t* ups, int n_up, int nres,
                     int use_pqmf) {
  auto& G = c->mg;
  const auto& m = c->mg_host;
  G.ready = false;
  TTS_CHECK(nres >= 1 && nres <= 4, "num_res_blocks must be in [1, 4] (dilation <= 27)");
  G.in_ch = in_ch;
  G.out_ch = out_ch;
  G.base = base;
  G.nres = nres;
  G.pqmf = use_pqmf;
  G.ups.assign(ups, ups + n_up);
  G.convT.clear();
  G.dconv.clear();
  G.fused.clear();
  G.convT.resize(n_up);
  G.convTm.clear();
  G.convTm.resize(n_up);
  G.dconv.resize((size_t)n_up * nres);
  G.fused.resize((size_t)n_up * nres);
  G.rb_wd16.clear();
  G.rb_wf16.clear();
  G.rb_wd16.resize((size_t)n_up * nres);
  G.rb_wf16.resize((size_t)n_up * nres);
  G.rb_wd16p.clear();
  G.rb_wd16p.resize((size_t)n_up * nres);
  int pl3[8] = {3}, pl0[8] = {0};
  {
    auto w = wn_weight(m, "layers.1", {base, in_ch, 7});
    pack_conv(G.conv_in, w, need(m, "layers.1.bias", {base}).d, in_ch, base, 7, 1, 1, pl3);
  }
  int idx = 2, C = base;
  for (int i = 0; i < n_up; ++i) {
    const int u = ups[i];
    TTS_CHECK(u % 2 == 0 && u <= 8, "upsample factors must be even and <= 8");
    const int cin = base >> i, cout = base >> (i + 1);
    const int p = u / 2;
    const std::string nm = "layers." + std::to_string(idx + 1);
    auto wt = wn_weight(m, nm, {cin, cout, 2 * u});  // ConvTranspose1d weight (Cin, Cout, K)
    std::vector<float> Wm((size_t)u * cout * cin * 2);
    int pls[8] = {0};
    for (int ph = 0; ph < u; ++ph) {
      const int dmax = (ph + p) / u, dmin = dmax - 1;
      pls[ph] = -dmin;
      for (int co = 0; co < cout; ++co)
        for (int ci = 0; ci < cin; ++ci)
          for (int jj = 0; jj < 2; ++jj) {
            const int delta = dmin + jj;
            const int k = ph + p - delta * u;
            Wm[(((size_t)ph * cout + co) * cin + ci) * 2 + jj] = wt[((size_t)ci * cout + co) * (2 * u) + k];
          }
    }
    pack_conv(G.convT[i], Wm, need(m, nm + ".bias", {cout}).d, cin, cout, 2, 1, u, pls);
    bool wm_in_range = true;
    for (float v : Wm) wm_in_range &= std::fabs(v) < F16_RANGE;
    // the merged GEMM has u * cout rows, so it is covered even where cout alone is not (full-band 64 -> 32)
    if (wm_in_range && conv_x3_supported(cin, u * cout, 2, 1)) {
      const auto& bias = need(m, nm + ".bias", {cout}).d;
      std::vector<float> bm((size_t)u * cout);
      for (size_t r = 0; r < bm.size(); ++r) bm[r] = bias[r / u];
      pack_conv_x3_only(G.convTm[i], merge_convT_phases(Wm, u, cin, cout), bm, cin, u * cout, 2);
    }
    C = cout;
    for (int bk = 0; bk < nres; ++bk) {
      const int d = 1;
      int dil = 1;
      for (int q = 0; q < bk; ++q) dil *= 3;
      (void)d;
      const std::string bn = "layers." + std::to_string(idx + 2) + ".blocks." + std::to_string(bk);
      auto wd = wn_weight(m, bn + ".2", {C, C, 3});
      int pld[8] = {dil};
      pack_conv(G.dconv[(size_t)i * nres + bk], wd, need(m, bn + ".2.bias", {C}).d, C, C, 3, dil, 1, pld);
      auto w1 = wn_weight(m, bn + ".4", {C, C, 1});
      const std::string sn = "layers." + std::to_string(idx + 2) + ".shortcuts." + std::to_string(bk);
      auto ws = wn_weight(m, sn, {C, C, 1});
      std::vector<float> Wf((size_t)C * 2 * C), bf(C);
      const auto& b1 = need(m, bn + ".4.bias", {C}).d;
      const auto& bs = need(m, sn + ".bias", {C}).d;
      for (int co = 0; co < C; ++co) {
        std::memcpy(&Wf[(size_t)co * 2 * C], &w1[(size_t)co * C], C * 4);
        std::memcpy(&Wf[(size_t)co * 2 * C + C], &ws[(size_t)co * C], C * 4);
        bf[co] = b1[co] + bs[co];
      }
      pack_conv(G.fused[(size_t)i * nres + bk], Wf, bf, 2 * C, C, 1, 1, 1, pl0);
      if (resblock_x3_supported(C)) {
        std::vector<uint16_t> wd16, wf16;
        pack_resblock_x3(wd, Wf, C, wd16, wf16);
        G.rb_wd16[(size_t)i * nres + bk].upload(wd16);
        G.rb_wf16[(size_t)i * nres + bk].upload(wf16);
        if (C % 32 == 16) {
          pack_resblock_x3p(wd, C, wd16);
          G.rb_wd16p[(size_t)i * nres + bk].upload(wd16);
        }
      }
    }
    idx += 3;
  }
  {
    const std::string nm = "layers." + std::to_string(idx + 2);
    auto w = wn_weight(m, nm, {out_ch, C, 7});
    const auto& bo = need(m, nm + ".bias", {out_ch}).d;
    pack_conv(G.conv_out, w, bo, C, out_ch, 7, 1, 1, pl3);
    G.C_last = C;
    if (out_ch == 4) {
      std::vector<float> wo((size_t)C * 7 * 4);
      for (int o = 0; o < 4; ++o)
        for (int ci = 0; ci < C; ++ci)
          for (int k = 0; k < 7; ++k) wo[((size_t)ci * 7 + k) * 4 + o] = w[((size_t)o * C + ci) * 7 + k];
      G.out_w.upload(wo);
      G.out_b.upload(bo);
    } else if (out_ch == 1) {  // full-band: [c][k] for launch_out_conv1
      G.out_w.upload(w);
      G.out_b.upload(bo);
    }
  }
  if (use_pqmf) {
    const auto& g = need(m, "pqmf_layer.G", {}).d;
    auto it = m.find("pqmf_layer.G");
    TTS_CHECK(it->second.shape.size() == 3 && it->second.shape[1] == out_ch, "pqmf_layer.G shape");
    G.taps = (int)it->second.shape[2] - 1;
    G.G.upload(g);
  }
  HIP_OK(hipDeviceSynchronize());
  G.ready = true;
}

// blocks 0-2 of a C = 48 ResidualStack as one kernel (TTS_STACK_FUSE=0: block by block, for A/B)
static bool stack_fuse_on() {
  static const bool on = [] {
    const char* e = std::getenv("TTS_STACK_FUSE");
    return !e || std::atoi(e) != 0;
  }();
  return on;
}
// the C = 96 stack in one launch: off by default since round 5 (TTS_STACK_FUSE96=1 turns it on).
// Same-box A/B over 4 bench runs each (profiles/r05/v17_stack96_ab.txt): vocoder 2.958 ms fused
// against 2.922 ms with blocks 0-2 as three resblock_x3 launches; the stack kernel's halo
// recompute (up to 24 extra rows per 96-position tile) now costs more than the two HBM round trips
// of x it saves at this width, while at C = 48 (with the fused ConvTranspose) fusing still wins
static bool stack_fuse96_on() {
  static const bool on = [] {
    const char* e = std::getenv("TTS_STACK_FUSE96");
    return e && std::atoi(e) != 0;
  }();
  return on;
}
// the last upsample's ConvTranspose inside the C = 48 stack kernel (resstack_x3.hip CTU = 2);
// TTS_CT_FUSE=0 keeps the separate conv_x3 launch
static bool ct_fuse_on() {
  static const bool on = [] {
    const char* e = std::getenv("TTS_CT_FUSE");
    return !e || std::atoi(e) != 0;
  }();
  return on;
}

// returns total upsampling factor; writes bands (B, out_ch, up*(M_max+2pad)) into `out`
// dev_lens: W.lens already holds the lengths on the device (a fused call's decode wrote them,
// checked there against vocoder_min_len); h_lens are then per-row upper bounds, used for tile counts
int run_generator(tts_ctx* c, const float* mel, const int32_t* h_lens, int B, int M_max, int pad, float* out,
                  hipStream_t s, GenTail* tail = nullptr, const int64_t* mel_strides = nullptr, bool dev_lens = false) {
  auto& G = c->mg;
  auto& W = c->mws;
  TTS_CHECK(G.ready, "melgan weights not finalized");
  TTS_CHECK(B >= 1, "B >= 1");
  for (int b = 0; b < B && !dev_lens; ++b) {
    TTS_CHECK(h_lens[b] >= 1 && h_lens[b] <= M_max, "mel lens out of range");
    TTS_CHECK(h_lens[b] + 2 * pad >= 4, "ReflectionPad1d(3): mel frames + 2*padding must be >= 4");
    for (int k = 0; k < G.nres && !G.ups.empty(); ++k)  // ResidualStack ReflectionPad1d(dilation), stage 0
      TTS_CHECK((long)(h_lens[b] + 2 * pad) * G.ups[0] > G.dconv[k].dil,
                "ReflectionPad1d: a residual stack's dilation must be < the first stage's length");
  }
  const int Lb = M_max + 2 * pad;
  int up = 1;
  for (int u : G.ups) up *= u;
  size_t maxelems = (size_t)G.base * Lb;
  {
    int mul = 1, Cc = G.base;
    for (int u : G.ups) {
      mul *= u;
      Cc /= 2;
      maxelems = std::max(maxelems, (size_t)Cc * Lb * mul);
    }
  }
  // device lengths: the ticket slot's (a fused submission's vocoder) or the workspace's
  int* vld = c->vlens_override;
  if (!vld) {
    W.lens.ensure(B * 4);
    vld = W.lens.i();
  }
  W.xa.ensure((size_t)B * maxelems * 4);
  W.xb.ensure((size_t)B * maxelems * 4);
  std::vector<int> lens(h_lens, h_lens + B);
  if (!dev_lens) HIP_OK(hipMemcpyAsync(vld, lens.data(), B * 4, hipMemcpyHostToDevice, s));
  else TTS_CHECK(c->vlens_override || W.lens.bytes >= (size_t)B * 4, "vocoder lengths buffer");
  ConvCall cc;
  cc.lens = vld;
  cc.B = B;
  cc.oflow = x3_flag(c);
  cc.len_add = 2 * pad;
  // layers[0..1]: replicate pad (inference_padding) + ReflectionPad1d(3) + Conv1d(k7)
  if (mel_strides) {
    TTS_CHECK(mel_strides[1] >= 1 && mel_strides[2] >= 1 && mel_strides[1] < (1L << 31) && mel_strides[2] < (1L << 31) &&
                  (mel_strides[0] >= 1 || B == 1) && mel_strides[0] >= 0,
              "mel strides must be positive");
    TTS_CHECK(mel_strides[1] != 1 || (mel_strides[2] % 4 == 0 && (reinterpret_cast<uintptr_t>(mel) & 15) == 0),
              "channel stride 1 needs a frame stride divisible by 4 and a 16-byte aligned mel");
    cc.s[0] = src_of(mel, (long)mel_strides[0], (int)mel_strides[1], (int)mel_strides[2], G.in_ch, 0);
  } else {
    cc.s[0] = src_of(mel, (long)G.in_ch * M_max, M_max, 1, G.in_ch, 0);
  }
  cc.pad_mode = 1;
  cc.rep_pad = pad;
  cc.in_mul = cc.q_mul = 1;
  cc.max_q = Lb;
  float* x = W.xa.f();
  float* xo = W.xb.f();
  int C = G.base, mul = 1;
  long Ls = Lb;
  cc.out = x;
  cc.ob = (long)C * Ls;
  cc.oc = Ls;
  cc.ot = 1;
  run_conv(G.conv_in, cc, s);
  cc.rep_pad = 0;
  // blocks 0-2 of stage i as one resstack_x3 launch (x: the stage input; with ct, x is the
  // ConvTranspose input and the kernel computes the stage input per tile): false if not covered
  auto stack3 = [&](size_t i, int Cs, long Lss, int muls, const float* xs, float* ys, const ConvLayer* ct,
                    const float* xin, int Cin, long Lin) {
    if (!(cc.oflow && G.nres >= 3 && stack_fuse_on() && G.rb_wd16[i * G.nres].p)) return false;
    if (Cs == 96 && !stack_fuse96_on()) return false;
    int dil[3];
    for (int k = 0; k < 3; ++k) dil[k] = G.dconv[i * G.nres + k].dil;
    if (!resstack_x3_supported(Cs, dil, 3)) return false;
    StackArgs sa{};
    sa.B = B;
    sa.x = xs;
    sa.y = ys;
    sa.sb = (long)Cs * Lss;
    sa.Ls = (int)Lss;
    sa.lens = vld;
    sa.len_add = 2 * pad;
    sa.mul = muls;
    for (int k = 0; k < 3; ++k) {
      sa.dil[k] = dil[k];
      sa.wd16[k] = Cs % 32 == 16 ? G.rb_wd16p[i * G.nres + k].p : G.rb_wd16[i * G.nres + k].p;
      sa.wf16[k] = G.rb_wf16[i * G.nres + k].p;
      sa.bd[k] = G.dconv[i * G.nres + k].bias.f();
      sa.bf[k] = G.fused[i * G.nres + k].bias.f();
    }
    sa.oflow = cc.oflow;
    if (ct) {
      sa.xin = xin;
      sa.sb_in = (long)Cin * Lin;
      sa.Ls_in = (int)Lin;
      sa.ct16 = ct->W16.p;
      sa.ct_bias = ct->bias.f();
    }
    if (!resstack_x3_fits(sa, lens.data())) return false;
    launch_resstack_x3(sa, lens.data(), Cs, s);
    return true;
  };
  for (size_t i = 0; i < G.ups.size(); ++i) {
    const int u = G.ups[i];
    int bk0 = 0;
    if (u == 2 && C == 96 && ct_fuse_on() && cc.oflow && G.convTm[i].W16.p &&
        stack3(i, C / 2, Ls * u, mul * u, nullptr, xo, &G.convTm[i], x, C, Ls)) {
      // LeakyReLU + ConvTranspose1d + blocks 0-2 in one launch (resstack_x3.hip CTU = 2)
      std::swap(x, xo);
      C /= 2;
      Ls *= u;
      mul *= u;
      bk0 = 3;
    }
    // LeakyReLU + ConvTranspose1d as u polyphase 2-tap convs
    ConvCall t = cc;
    t.s[0] = src_of(x, (long)C * Ls, Ls, 1, C, 1);
    t.pad_mode = 0;
    t.in_mul = t.q_mul = mul;
    t.max_q = Lb * mul;
    t.out_mul = u;
    const int Cn = C / 2;
    const long Ln = Ls * u;
    t.out = xo;
    t.ob = (long)Cn * Ln;
    t.oc = Ln;
    t.ot = 1;
    if (bk0 == 0) {
      if (t.oflow && G.convTm[i].W16.p) {  // all u phases as one GEMM over input positions 0 .. L
        t.out_mul = 1;
        t.max_q = Lb * mul + 1;
        t.merged_u = u;
        run_conv(G.convTm[i], t, s);
      } else {
        run_conv(G.convT[i], t, s);
      }
      std::swap(x, xo);
      C = Cn;
      Ls = Ln;
      mul *= u;
      // blocks 0-2 in one pass over the stage (resstack_x3.hip)
      if (stack3(i, C, Ls, mul, x, xo, nullptr, nullptr, 0, 0)) {
        std::swap(x, xo);
        bk0 = 3;
      }
    }
    for (int bk = bk0; bk < G.nres; ++bk) {  // fused ResidualStack blocks (resblock.hip)
      const ConvLayer& dl = G.dconv[i * G.nres + bk];
      const ConvLayer& fl = G.fused[i * G.nres + bk];
      ResArgs ra{};
      ra.x = x;
      ra.y = xo;
      ra.sb = (long)C * Ls;
      ra.Ls = (int)Ls;
      ra.lens = vld;
      ra.len_add = 2 * pad;
      ra.mul = mul;
      ra.dil = dl.dil;
      ra.Wd = dl.W.f();
      ra.bd = dl.bias.f();
      ra.Wf = fl.W.f();
      ra.bf = fl.bias.f();
      ra.max_q = Lb * mul;
      ra.B = B;
      const DevBuf& w16 = G.rb_wd16[i * G.nres + bk];
      if (cc.oflow && w16.p) {
        ra.Wd16 = w16.p;
        ra.Wf16 = G.rb_wf16[i * G.nres + bk].p;
        ra.oflow = cc.oflow;
        launch_resblock_x3(ra, lens.data(), C, s);
      } else {
        launch_resblock(ra, C, s);
      }
      std::swap(x, xo);
    }
  }
  if (tail) {
    tail->x = x;
    tail->C = C;
    tail->Ls = Ls;
    tail->mul = mul;
    return up;
  }
  if (G.out_ch == 1) {  // full-band output stage on the VALU (melgan_out.hip)
    HIP_OK(hipMemsetAsync(out, 0, (size_t)B * Ls * 4, s));
    launch_out_conv1(x, (long)C * Ls, Ls, C, G.out_w.f(), G.out_b.f(), vld, 2 * pad, mul, (int)(Lb * mul), B,
                     out, Ls, s);
    return up;
  }
  ConvCall o = cc;
  o.s[0] = src_of(x, (long)C * Ls, Ls, 1, C, 1);
  o.pad_mode = 1;
  o.in_mul = o.q_mul = mul;
  o.max_q = Lb * mul;
  o.epi = 2;
  o.out = out;
  o.ob = (long)G.out_ch * Ls;
  o.oc = Ls;
  o.ot = 1;
  HIP_OK(hipMemsetAsync(out, 0, (size_t)B * G.out_ch * Ls * 4, s));
  run_conv(G.conv_out, o, s);
  return up;
}

// Runs fn, which enqueues vocoder kernels on c->s; split-f16 kernels among them raise the
// workspace's range flag when an operand falls outside the f16 range (split16.h). If it was
// raised, fn runs again on the fp32 kernels, so results are always fp32-accurate. Costs one
// stream synchronisation per call while split-f16 is on. fn must be re-runnable (it rewrites
// all of its outputs).
template <class F>
void with_x3_fallback(tts_ctx* c, F&& fn) {
  if (!c->gemm_x3) {
    fn();
    return;
  }
  unsigned* flag = x3_flag(c);
  HIP_OK(hipMemsetAsync(flag, 0, 4, c->s));
  c->flag_read = false;
  fn();
  if (!c->flag_read) {  // fn may have fetched it with its own status words (taco_infer)
    HIP_OK(hipMemcpyAsync(&c->pinned[12], flag, 4, hipMemcpyDeviceToHost, c->s));
    HIP_OK(hipStreamSynchronize(c->s));
  }
  c->flag_read = false;
  if (c->pinned[12]) {
    c->x3_fallbacks++;
    c->gemm_x3 = false;
    try {
      fn();
    } catch (...) {
      c->gemm_x3 = true;
      throw;
    }
    c->gemm_x3 = true;
  }
}

template <class F>
int guarded(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    tts_set_error(e.what());
    return 1;
  } catch (...) {
    tts_set_error("unknown error");
    return 1;
  }
}

// Entry points that take a context hold its mutex for the whole call: a context owns one
// workspace, one internal stream, cached graphs and pinned polling words, so two host threads
// (ctypes releases the GIL) must not interleave inside it. Recursive so that helpers may re-enter.
template <class F>
int guarded_ctx(tts_ctx* c, F&& f) {
  if (!c) {
    tts_set_error("null ctx");
    return 1;
  }
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  return guarded(std::forward<F>(f));
}

// (B, T, D) -> (B, T, Dp) with zero channels D..Dp-1 (the conv staging reads 16-channel chunks)
__global__ void pad_channels_kernel(const float* __restrict__ x, int D, int Dp, long n_rows, float* __restrict__ y) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n_rows * Dp; i += (long)gridDim.x * blockDim.x) {
    const long r = i / Dp;
    const int c = (int)(i - r * Dp);
    y[i] = c < D ? x[r * D + c] : 0.f;
  }
}

// one workgroup per sequence: v = last frame (with_proj) or relu(W h_last + b), then
// F.normalize(v, p=2, dim=1) = v / max(||v||, 1e-12)  (model.py:58-63)
__global__ __launch_bounds__(256) void ge2e_final_kernel(const float* __restrict__ src, long sb, int width,
                                                         const int* lens, int T_max, const float* __restrict__ W,
                                                         const float* __restrict__ bias, int P,
                                                         float* __restrict__ out) {
  __shared__ float v[1024], red[4];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* last = src + b * sb + (long)(lens[b] - 1) * width;
  for (int i = tid; i < P; i += blockDim.x) {
    float x;
    if (W) {
      float acc = bias[i];
      for (int k = 0; k < width; ++k) acc = fmaf(W[(long)i * width + k], last[k], acc);
      x = fmaxf(acc, 0.f);
    } else {
      x = last[i];
    }
    v[i] = x;
  }
  __syncthreads();
  float ss = 0.f;
  for (int i = tid; i < P; i += blockDim.x) ss = fmaf(v[i], v[i], ss);
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float nrm = fmaxf(sqrtf(red[0] + red[1] + red[2] + red[3]), 1e-12f);
  for (int i = tid; i < P; i += blockDim.x) out[(long)b * P + i] = v[i] / nrm;
}

void ge2e_finalize(tts_ctx* c, int in_dim, int proj, int lstm, int nl, int with_proj) {
  auto& G = c->ge2e;
  const auto& h = c->ge2e_host;
  G.ready = false;
  TTS_CHECK(lstm == 768, "speaker encoder: lstm_dim must be 768 (the persistent LSTM kernel's width)");
  TTS_CHECK(nl >= 1 && nl <= 4 && in_dim >= 1 && in_dim <= 1024 && proj >= 1 && proj <= 1024, "speaker encoder sizes");
  G.in_dim = in_dim;
  G.in_pad = (in_dim + 15) / 16 * 16;
  G.proj = proj;
  G.H = lstm;
  G.nl = nl;
  G.with_proj = with_proj;
  const int H = lstm;
  int pl0[8] = {0};
  for (int l = 0; l < nl; ++l) {
    const std::string pfx = with_proj ? "layers." + std::to_string(l) + ".lstm." : "layers.lstm.";
    const std::string sfx = with_proj ? "_l0" : "_l" + std::to_string(l);
    const int din = l == 0 ? in_dim : (with_proj ? proj : H);
    const int dpad = l == 0 ? G.in_pad : din;
    TTS_CHECK(dpad % 16 == 0, "speaker encoder: layer input width must be a multiple of 16");
    const auto& wih = need(h, pfx + "weight_ih" + sfx, {4 * H, din}).d;
    const auto& whh = need(h, pfx + "weight_hh" + sfx, {4 * H, H}).d;
    const auto& bih = need(h, pfx + "bias_ih" + sfx, {4 * H}).d;
    const auto& bhh = need(h, pfx + "bias_hh" + sfx, {4 * H}).d;
    std::vector<float> wt = lstm_tile_rows(wih, H, din), w2((size_t)4 * H * dpad, 0.f);
    for (int r = 0; r < 4 * H; ++r)
      for (int k = 0; k < din; ++k) w2[(size_t)r * dpad + k] = wt[(size_t)r * din + k];
    std::vector<float> bs(4 * H);
    for (int i = 0; i < 4 * H; ++i) bs[i] = bih[i] + bhh[i];
    pack_conv(G.gin[l], w2, lstm_tile_rows(bs, H, 1), dpad, 4 * H, 1, 1, 1, pl0);
    G.whh[l].upload(swz(lstm_tile_rows(whh, H, H), 4 * H, H));
    upload_split_rows(G.whh16[l], lstm_tile_rows(whh, H, H), 4 * H, H);
    if (with_proj) {
      const auto& wl = need(h, "layers." + std::to_string(l) + ".linear.weight", {proj, H}).d;
      pack_conv(G.proj_l[l], wl, std::vector<float>(proj, 0.f), H, proj, 1, 1, 1, pl0);
    }
  }
  if (!with_proj) {
    G.lin_w.upload(need(h, "layers.linear.weight", {proj, H}).d);
    G.lin_b.upload(need(h, "layers.linear.bias", {proj}).d);
  }
  G.pipe_ok = G.whh16[0].p != nullptr;
  for (int l = 1; l < nl && G.pipe_ok; ++l) {
    const std::string pfx = with_proj ? "layers." + std::to_string(l) + ".lstm." : "layers.lstm.";
    const std::string sfx = with_proj ? "_l0" : "_l" + std::to_string(l);
    const int din = with_proj ? proj : H;
    const auto& wih = need(h, pfx + "weight_ih" + sfx, {4 * H, din}).d;
    const auto& whh = need(h, pfx + "weight_hh" + sfx, {4 * H, H}).d;
    const auto& bih = need(h, pfx + "bias_ih" + sfx, {4 * H}).d;
    const auto& bhh = need(h, pfx + "bias_hh" + sfx, {4 * H}).d;
    std::vector<float> win;
    if (with_proj) {  // the previous layer's Linear (no bias, model.py:22) folded into W_ih
      const auto& wl = need(h, "layers." + std::to_string(l - 1) + ".linear.weight", {proj, H}).d;
      win.assign((size_t)4 * H * H, 0.f);
      std::vector<double> acc(H);
      for (int r = 0; r < 4 * H; ++r) {
        std::fill(acc.begin(), acc.end(), 0.0);
        for (int j = 0; j < proj; ++j) {
          const double a = wih[(size_t)r * proj + j];
          const float* wr = &wl[(size_t)j * H];
          for (int k = 0; k < H; ++k) acc[k] += a * wr[k];
        }
        for (int k = 0; k < H; ++k) win[(size_t)r * H + k] = (float)acc[k];
      }
    } else {
      win = wih;
    }
    const auto t1 = lstm_tile_rows(whh, H, H), t2 = lstm_tile_rows(win, H, H);
    std::vector<float> wc((size_t)4 * H * 2 * H);
    for (int r = 0; r < 4 * H; ++r) {
      std::memcpy(&wc[(size_t)r * 2 * H], &t1[(size_t)r * H], H * 4);
      std::memcpy(&wc[(size_t)r * 2 * H + H], &t2[(size_t)r * H], H * 4);
    }
    upload_split_rows(G.wpipe[l], wc, 4 * H, 2 * H);
    std::vector<float> bs(4 * H);
    for (int i = 0; i < 4 * H; ++i) bs[i] = bih[i] + bhh[i];
    G.bpipe[l].upload(lstm_tile_rows(bs, H, 1));
    G.pipe_ok = G.wpipe[l].p != nullptr;
  }
  HIP_OK(hipDeviceSynchronize());
  G.ready = true;
}

void ge2e_infer(tts_ctx* c, const float* d_x, const int32_t* h_lens, int B, int T_max, float* d_out) {
  auto& G = c->ge2e;
  auto& W = c->gws;
  TTS_CHECK(G.ready, "speaker encoder weights not finalized");
  TTS_CHECK(B >= 1 && B <= 64, "speaker encoder: B must be in [1, 64]");
  TTS_CHECK(T_max >= 1 && T_max <= 100000, "speaker encoder: bad T_max");
  for (int b = 0; b < B; ++b) TTS_CHECK(h_lens[b] >= 1 && h_lens[b] <= T_max, "speaker encoder: lens out of range");
  hipStream_t s = c->s;
  const int H = G.H;
  long gen = 0;
  grow<float>(W.x, (size_t)B * T_max * G.in_pad, gen);
  grow<int>(W.lens, 64, gen);
  grow<float>(W.g, (size_t)B * T_max * 4 * H, gen);
  grow<float>(W.o, (size_t)B * T_max * H, gen);
  grow<float>(W.p, (size_t)B * T_max * G.proj, gen);
  grow<unsigned>(W.bar, BAR_WORDS, gen);
  grow<float>(W.hbuf, (size_t)2 * 64 * H, gen);
  std::vector<int> lens(h_lens, h_lens + B);
  HIP_OK(hipMemcpyAsync(W.lens.p, lens.data(), B * 4, hipMemcpyHostToDevice, s));
  pad_channels_kernel<<<1024, 256, 0, s>>>(d_x, G.in_dim, G.in_pad, (long)B * T_max, W.x.f());
  HIP_OK(hipGetLastError());
  const float* in = W.x.f();
  int din = G.in_pad;
  // all layers in one persistent launch (encoder.hip ge2e_pipe_kernel); TTS_GE2E_PIPE=0 keeps
  // one launch per layer with the input projections as convs
  static const bool pipe_env = [] {
    const char* e = std::getenv("TTS_GE2E_PIPE");
    return !(e && std::string(e) == "0");
  }();
  bool piped = false;
  if (pipe_env && c->gemm_x3 && G.pipe_ok && B <= 16) {
    ConvCall cc;  // layer-0 input gates
    cc.lens = W.lens.i();
    cc.B = B;
    cc.oflow = x3_flag(c);
    cc.max_q = T_max;
    cc.s[0] = src_of(in, (long)T_max * din, 1, din, din, 0);
    cc.out = W.g.f();
    cc.ob = (long)T_max * 4 * H;
    cc.oc = 1;
    cc.ot = 4 * H;
    run_conv(G.gin[0], cc, s);
    const uint16_t* w16[4] = {nullptr, nullptr, nullptr, nullptr};
    const float* bias[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int l = 0; l < G.nl; ++l) {
      w16[l] = l == 0 ? G.whh16[0].h() : G.wpipe[l].h();
      bias[l] = l == 0 ? nullptr : G.bpipe[l].f();
    }
    piped = launch_ge2e_pipe(w16, bias, G.nl, W.g.f(), W.lens.i(), T_max, B, W.hbuf.f(),
                             reinterpret_cast<unsigned*>(W.bar.p), W.o.f(), s);
    if (piped && G.with_proj) {  // the last layer's Linear
      ConvCall cp;
      cp.lens = W.lens.i();
      cp.B = B;
      cp.oflow = x3_flag(c);
      cp.max_q = T_max;
      cp.s[0] = src_of(W.o.f(), (long)T_max * H, 1, H, H, 0);
      cp.out = W.p.f();
      cp.ob = (long)T_max * G.proj;
      cp.oc = 1;
      cp.ot = G.proj;
      run_conv(G.proj_l[G.nl - 1], cp, s);
    }
  }
  for (int l = 0; l < G.nl && !piped; ++l) {
    ConvCall cc;  // gates_in = x W_ih^T + b  (time-major rows, K = 1)
    cc.lens = W.lens.i();
    cc.B = B;
    cc.oflow = x3_flag(c);
    cc.max_q = T_max;
    cc.s[0] = src_of(in, (long)T_max * din, 1, din, din, 0);
    cc.out = W.g.f();
    cc.ob = (long)T_max * 4 * H;
    cc.oc = 1;
    cc.ot = 4 * H;
    run_conv(G.gin[l], cc, s);
    const bool ok = launch_lstm768_persist(W.g.f(), G.whh[l].f(), c->gemm_x3 ? G.whh16[l].h() : nullptr, W.lens.i(),
                                           T_max, B, W.hbuf.f(),
                                           reinterpret_cast<unsigned*>(W.bar.p), W.o.f(), s);
    TTS_CHECK(ok, "speaker encoder: cooperative launch unavailable");
    if (G.with_proj) {
      ConvCall cp;
      cp.lens = W.lens.i();
      cp.B = B;
      cp.oflow = x3_flag(c);
      cp.max_q = T_max;
      cp.s[0] = src_of(W.o.f(), (long)T_max * H, 1, H, H, 0);
      cp.out = W.p.f();
      cp.ob = (long)T_max * G.proj;
      cp.oc = 1;
      cp.ot = G.proj;
      run_conv(G.proj_l[l], cp, s);
      in = W.p.f();
      din = G.proj;
    } else {
      in = W.o.f();
      din = H;
    }
  }
  if (G.with_proj)
    ge2e_final_kernel<<<B, 256, 0, s>>>(W.p.f(), (long)T_max * G.proj, G.proj, W.lens.i(), T_max, nullptr, nullptr,
                                        G.proj, d_out);
  else
    ge2e_final_kernel<<<B, 256, 0, s>>>(W.o.f(), (long)T_max * H, H, W.lens.i(), T_max, G.lin_w.f(), G.lin_b.f(),
                                        G.proj, d_out);
  HIP_OK(hipGetLastError());
  HIP_OK(hipStreamSynchronize(s));
  unsigned err = 0;
  HIP_OK(hipMemcpy(&err, reinterpret_cast<unsigned*>(W.bar.p) + 16, 4, hipMemcpyDeviceToHost));
  TTS_CHECK(err == 0, "speaker encoder: grid barrier timed out (workgroups not co-resident) or preempted past TTS_BARRIER_TIMEOUT_MS; retrying the call is safe)");
}

// ------------------------------------------------------------------------------------ Glow-TTS
// rows (r, half + r) -> (2r, 2r + 1) of a (2 * half, rowlen) weight and its bias
static std::pair<std::vector<float>, std::vector<float>> interleave_halves(const std::vector<float>& w,
                                                                           const std::vector<float>& b, int half,
                                                                           int rowlen) {
  std::vector<float> wo(w.size()), bo(b.size());
  for (int r = 0; r < 2 * half; ++r) {
    const int src = (r & 1) ? half + r / 2 : r / 2;
    std::copy(w.begin() + (size_t)src * rowlen, w.begin() + (size_t)(src + 1) * rowlen, wo.begin() + (size_t)r * rowlen);
    bo[r] = b[src];
  }
  return {wo, bo};
}

void glow_finalize(tts_ctx* c, int num_chars, int enc_layers, int flows, int wn_layers) {
  auto& G = c->glow;
  const auto& h = c->glow_host;
  G.ready = false;
  const int H = G.H, C = G.C, F = G.Fdp, C2 = 2 * C;
  TTS_CHECK(enc_layers >= 1 && enc_layers <= 32 && flows >= 1 && flows <= 32 && wn_layers >= 1 && wn_layers <= 8,
            "glow: layer counts");
  G.num_chars = num_chars;
  G.enc_layers = enc_layers;
  G.flows = flows;
  G.wn_layers = wn_layers;
  int p2[8] = {2}, p1[8] = {1}, p0[8] = {0};
  {
    auto e = need(h, "encoder.emb.weight", {num_chars, H}).d;
    const float sc = std::sqrt((float)H);  // encoder.py:107, x * math.sqrt(hidden) in fp32
    for (auto& v : e) v *= sc;
    G.emb.upload(e);
  }
  G.enc_conv.clear();
  G.enc_g.clear();
  G.enc_b.clear();
  G.tdsep = h.count("encoder.encoder.layers.0.time_conv.weight") > 0;
  G.tfm = h.count("encoder.encoder.attn_layers.0.conv_q.weight") > 0;
  if (G.tdsep || G.tfm) {
    G.pre_conv.clear();
    G.pre_conv.resize(3);
    G.pre_g.clear();
    G.pre_g.resize(3);
    G.pre_b.clear();
    G.pre_b.resize(3);
    for (int i = 0; i < 3; ++i) {
      const std::string q = "encoder.pre.";
      pack_conv(G.pre_conv[i], need(h, q + "conv_layers." + std::to_string(i) + ".weight", {H, H, 5}).d,
                need(h, q + "conv_layers." + std::to_string(i) + ".bias", {H}).d, H, H, 5, 1, 1, p2);
      G.pre_g[i].upload(need(h, q + "norm_layers." + std::to_string(i) + ".gamma", {1, H, 1}).d);
      G.pre_b[i].upload(need(h, q + "norm_layers." + std::to_string(i) + ".beta", {1, H, 1}).d);
    }
    pack_conv(G.pre_proj, need(h, "encoder.pre.proj.weight", {H, H, 1}).d, need(h, "encoder.pre.proj.bias", {H}).d, H,
              H, 1, 1, 1, p0);
  }
  if (G.tfm) {  // transformer.py:265-319, num_layers = enc_layers
    for (auto* v : {&G.tfm_qkv, &G.tfm_o, &G.tfm_f1, &G.tfm_f2}) {
      v->clear();
      v->resize(enc_layers);
    }
    for (auto* v : {&G.tfm_g1, &G.tfm_b1, &G.tfm_g2, &G.tfm_b2}) {
      v->clear();
      v->resize(enc_layers);
    }
    const int Fc = 768;
    for (int i = 0; i < enc_layers; ++i) {
      const std::string a = "encoder.encoder.attn_layers." + std::to_string(i) + ".";
      std::vector<float> wqkv, bqkv;
      for (const char* n : {"q", "k", "v"}) {
        const auto& w = need(h, a + "conv_" + n + ".weight", {H, H, 1}).d;
        const auto& bb = need(h, a + "conv_" + n + ".bias", {H}).d;
        wqkv.insert(wqkv.end(), w.begin(), w.end());
        bqkv.insert(bqkv.end(), bb.begin(), bb.end());
      }
      pack_conv(G.tfm_qkv[i], wqkv, bqkv, H, 3 * H, 1, 1, 1, p0);
      pack_conv(G.tfm_o[i], need(h, a + "conv_o.weight", {H, H, 1}).d, need(h, a + "conv_o.bias", {H}).d, H, H, 1, 1,
                1, p0);
      const std::string f = "encoder.encoder.ffn_layers." + std::to_string(i) + ".";
      pack_conv(G.tfm_f1[i], need(h, f + "conv_1.weight", {Fc, H, 3}).d, need(h, f + "conv_1.bias", {Fc}).d, H, Fc, 3,
                1, 1, p1);
      pack_conv(G.tfm_f2[i], need(h, f + "conv_2.weight", {H, Fc, 3}).d, need(h, f + "conv_2.bias", {H}).d, Fc, H, 3,
                1, 1, p1);
      const std::string n1 = "encoder.encoder.norm_layers_1." + std::to_string(i) + ".";
      const std::string n2 = "encoder.encoder.norm_layers_2." + std::to_string(i) + ".";
      G.tfm_g1[i].upload(need(h, n1 + "gamma", {1, H, 1}).d);
      G.tfm_b1[i].upload(need(h, n1 + "beta", {1, H, 1}).d);
      G.tfm_g2[i].upload(need(h, n2 + "gamma", {1, H, 1}).d);
      G.tfm_b2[i].upload(need(h, n2 + "beta", {1, H, 1}).d);
    }
  }
  if (G.tdsep) {
    // eval BatchNorm: y = (x - mean) * w / sqrt(var + 1e-5) + b, folded in double
    auto bn_fold = [&](const std::string& name, int n, std::vector<float>& W, std::vector<float>& bias, int rowlen) {
      const auto& w = need(h, name + ".weight", {n}).d;
      const auto& bb = need(h, name + ".bias", {n}).d;
      const auto& mu = need(h, name + ".running_mean", {n}).d;
      const auto& var = need(h, name + ".running_var", {n}).d;
      for (int r = 0; r < n; ++r) {
        const double sc = (double)w[r] / std::sqrt((double)var[r] + 1e-5);
        for (int k = 0; k < rowlen; ++k) W[(size_t)r * rowlen + k] = (float)(W[(size_t)r * rowlen + k] * sc);
        bias[r] = (float)(((double)bias[r] - mu[r]) * sc + bb[r]);
      }
    };
    G.tds_tc.clear();
    G.tds_tc.resize(enc_layers);
    G.tds_tc2.clear();
    G.tds_tc2.resize(enc_layers);
    G.tds_dw.clear();
    G.tds_dw.resize(enc_layers);
    G.tds_dwb.clear();
    G.tds_dwb.resize(enc_layers);
    for (int i = 0; i < enc_layers; ++i) {
      const std::string q = "encoder.encoder.layers." + std::to_string(i) + ".";
      auto w1 = need(h, q + "time_conv.weight", {2 * H, H, 1}).d;
      auto b1 = need(h, q + "time_conv.bias", {2 * H}).d;
      bn_fold(q + "norm1", 2 * H, w1, b1, H);
      auto [w1i, b1i] = interleave_halves(w1, b1, H, H);  // (a_c, g_c) pairs for the GLU epilogue
      pack_conv(G.tds_tc[i], w1i, b1i, H, 2 * H, 1, 1, 1, p0);
      auto wd = need(h, q + "depth_conv.weight", {H, 1, 5}).d;
      auto bd = need(h, q + "depth_conv.bias", {H}).d;
      bn_fold(q + "norm2", H, wd, bd, 5);
      G.tds_dw[i].upload(wd);
      G.tds_dwb[i].upload(bd);
      auto w2 = need(h, q + "time_conv2.weight", {H, H, 1}).d;
      auto b2 = need(h, q + "time_conv2.bias", {H}).d;
      bn_fold(q + "norm3", H, w2, b2, H);
      pack_conv(G.tds_tc2[i], w2, b2, H, H, 1, 1, 1, p0);
    }
  }
  const bool gated = !G.tdsep && !G.tfm;
  G.enc_conv.resize(gated ? enc_layers : 0);
  G.enc_g.resize(gated ? enc_layers : 0);
  G.enc_b.resize(gated ? enc_layers : 0);
  for (int i = 0; i < (gated ? enc_layers : 0); ++i) {
    const std::string pf = "encoder.encoder.";
    pack_conv(G.enc_conv[i], need(h, pf + "conv_layers." + std::to_string(i) + ".weight", {2 * H, H, 5}).d,
              need(h, pf + "conv_layers." + std::to_string(i) + ".bias", {2 * H}).d, H, 2 * H, 5, 1, 1, p2);
    G.enc_g[i].upload(need(h, pf + "norm_layers." + std::to_string(i) + ".gamma", {1, 2 * H, 1}).d);
    G.enc_b[i].upload(need(h, pf + "norm_layers." + std::to_string(i) + ".beta", {1, 2 * H, 1}).d);
  }
  pack_conv(G.proj_m, need(h, "encoder.proj_m.weight", {C, H, 1}).d, need(h, "encoder.proj_m.bias", {C}).d, H, C, 1, 1,
            1, p0);
  const std::string dp = "encoder.duration_predictor.";
  {
    auto it = h.find(dp + "conv_1.weight");
    TTS_CHECK(it != h.end() && it->second.shape.size() == 3, "missing tensor: " + dp + "conv_1.weight");
    G.c_in = (int)it->second.shape[1] - H;
    TTS_CHECK(G.c_in >= 0 && G.c_in <= 4096, "glow: duration predictor input channels");
  }
  const int cin = G.c_in, cpad = (cin + 15) / 16 * 16;
  G.c_pad = cpad;
  {
    // [x; g] input of conv_1, g's channels zero-padded to c_pad
    const auto& w = need(h, dp + "conv_1.weight", {F, H + cin, 3}).d;
    std::vector<float> wp((size_t)F * (H + cpad) * 3, 0.f);
    for (int o = 0; o < F; ++o)
      std::copy(w.begin() + (size_t)o * (H + cin) * 3, w.begin() + (size_t)(o + 1) * (H + cin) * 3,
                wp.begin() + (size_t)o * (H + cpad) * 3);
    pack_conv(G.dp1, wp, need(h, dp + "conv_1.bias", {F}).d, H + cpad, F, 3, 1, 1, p1);
  }
  G.n_spk = 0;
  G.emb_g.reset();
  if (h.count("emb_g.weight")) {
    auto it = h.find("emb_g.weight");
    TTS_CHECK(it->second.shape.size() == 2 && it->second.shape[1] == cin && it->second.shape[0] >= 1,
              "glow: emb_g.weight must be (num_speakers, c_in_channels)");
    G.n_spk = (int)it->second.shape[0];
    if (cin > 0) G.emb_g.upload(it->second.d);
  }
  pack_conv(G.dp2, need(h, dp + "conv_2.weight", {F, F, 3}).d, need(h, dp + "conv_2.bias", {F}).d, F, F, 3, 1, 1, p1);
  pack_conv(G.dp_proj, need(h, dp + "proj.weight", {1, F, 1}).d, need(h, dp + "proj.bias", {1}).d, F, 1, 1, 1, 1, p0);
  G.dp_g1.upload(need(h, dp + "norm_1.gamma", {1, F, 1}).d);
  G.dp_b1.upload(need(h, dp + "norm_1.beta", {1, F, 1}).d);
  G.dp_g2.upload(need(h, dp + "norm_2.gamma", {1, F, 1}).d);
  G.dp_b2.upload(need(h, dp + "norm_2.beta", {1, F, 1}).d);
  G.start.clear();
  G.start.resize(flows);
  G.end.clear();
  G.end.resize(flows);
  G.invtab.clear();
  G.invtab.resize(flows);
  G.wn_in.clear();
  G.wn_in.resize(flows * wn_layers);
  G.wn_rs.clear();
  G.wn_rs.resize(flows * wn_layers);
  std::vector<float> cond_w(cin > 0 ? (size_t)flows * wn_layers * 2 * H * cpad : 0, 0.f);
  std::vector<float> cond_b(cin > 0 ? (size_t)flows * wn_layers * 2 * H : 0, 0.f);
  for (int k = 0; k < flows; ++k) {
    const std::string an = "decoder.flows." + std::to_string(3 * k) + ".";
    const std::string ic = "decoder.flows." + std::to_string(3 * k + 1) + ".";
    const std::string cp = "decoder.flows." + std::to_string(3 * k + 2) + ".";
    pack_conv(G.start[k], wn_weight(h, cp + "start", {H, C, 1}), need(h, cp + "start.bias", {H}).d, C, H, 1, 1, 1, p0);
    // end rows interleaved (m_c, logs_c) for the conv's coupling-pair epilogue
    auto [we, be] = interleave_halves(need(h, cp + "end.weight", {C2, H, 1}).d, need(h, cp + "end.bias", {C2}).d, C, H);
    pack_conv(G.end[k], we, be, H, C2, 1, 1, 1, p0);
    for (int i = 0; i < wn_layers; ++i) {
      const std::string wi = cp + "wn.in_layers." + std::to_string(i);
      const std::string wr = cp + "wn.res_skip_layers." + std::to_string(i);
      // in rows interleaved (tanh_c, sigmoid_c) for the gate-pair epilogue
      auto [wg, bg] = interleave_halves(wn_weight(h, wi, {2 * H, H, 5}), need(h, wi + ".bias", {2 * H}).d, H, H * 5);
      pack_conv(G.wn_in[k * wn_layers + i], wg, bg, H, 2 * H, 5, 1, 1, p2);
      // rows [0, H): residual, [H, 2H): skip -- one conv into the [hidden | skip] buffer; the last
      // layer has the skip rows only
      const int rsc = i == wn_layers - 1 ? H : 2 * H;
      pack_conv(G.wn_rs[k * wn_layers + i], wn_weight(h, wr, {rsc, H, 1}), need(h, wr + ".bias", {rsc}).d, H, rsc, 1,
                1, 1, p0);
    }
    if (cin > 0) {  // cond_layer (2H * wn_layers, c_in): per layer slice interleaved like wn_in
      const int L2 = 2 * H * wn_layers;
      const auto w = wn_weight(h, cp + "wn.cond_layer", {L2, cin, 1});
      const auto& cb = need(h, cp + "wn.cond_layer.bias", {L2}).d;
      for (int i = 0; i < wn_layers; ++i) {
        std::vector<float> wl(w.begin() + (size_t)i * 2 * H * cin, w.begin() + (size_t)(i + 1) * 2 * H * cin);
        std::vector<float> bl(cb.begin() + (size_t)i * 2 * H, cb.begin() + (size_t)(i + 1) * 2 * H);
        auto [wi, bi] = interleave_halves(wl, bl, H, cin);
        const size_t r0 = ((size_t)k * wn_layers + i) * 2 * H;
        for (int r = 0; r < 2 * H; ++r) {
          std::copy(wi.begin() + (size_t)r * cin, wi.begin() + (size_t)(r + 1) * cin,
                    cond_w.begin() + (r0 + r) * cpad);
          cond_b[r0 + r] = bi[r];
        }
      }
    }
    // reverse of [ActNorm, InvConvNear] (glow.py:48-58, 184-201): output channel c' = i*C + 2j + k
    // (split s' = 2i + k) = (sum_s winv[s'][s] x[c_s] - bias[c']) * exp(-logs[c']), c_s = i_s*C + 2j + k_s
    const auto& w4 = need(h, ic + "weight", {4, 4}).d;
    double a[4][8];
    for (int r = 0; r < 4; ++r)
      for (int q = 0; q < 8; ++q) a[r][q] = q < 4 ? w4[r * 4 + q] : (q - 4 == r ? 1.0 : 0.0);
    for (int col = 0; col < 4; ++col) {  // Gauss-Jordan with partial pivoting
      int piv = col;
      for (int r = col + 1; r < 4; ++r)
        if (std::fabs(a[r][col]) > std::fabs(a[piv][col])) piv = r;
      for (int q = 0; q < 8; ++q) std::swap(a[col][q], a[piv][q]);
      TTS_CHECK(std::fabs(a[col][col]) > 1e-12, "glow: singular InvConvNear weight");
      const double d = a[col][col];
      for (int q = 0; q < 8; ++q) a[col][q] /= d;
      for (int r = 0; r < 4; ++r)
        if (r != col) {
          const double f = a[r][col];
          for (int q = 0; q < 8; ++q) a[r][q] -= f * a[col][q];
        }
    }
    // the reference inverts in fp32 and casts (glow.py:190-193): round the inverse to float
    const auto& logs = need(h, an + "logs", {1, C2, 1}).d;
    const auto& abias = need(h, an + "bias", {1, C2, 1}).d;
    std::vector<float> tab((size_t)C2 * 6);
    for (int cp2 = 0; cp2 < C2; ++cp2) {
      const int s2 = 2 * (cp2 / C) + cp2 % 2;
      for (int s1 = 0; s1 < 4; ++s1) tab[cp2 * 6 + s1] = (float)a[s2][4 + s1];
      tab[cp2 * 6 + 4] = abias[cp2];
      tab[cp2 * 6 + 5] = std::exp(-logs[cp2]);
    }
    G.invtab[k].upload(tab);
  }
  if (cin > 0) pack_conv(G.cond, cond_w, cond_b, cpad, flows * wn_layers * 2 * H, 1, 1, 1, p0);
  HIP_OK(hipDeviceSynchronize());
  G.ready = true;
}

// encoder + duration predictor + durations: h_ylens out (per-utterance frames)
void glow_encode(tts_ctx* c, const int64_t* d_ids, const int32_t* h_lens, const int32_t* h_spk, int B, int T,
                 float length_scale, int32_t* h_ylens) {
  auto& G = c->glow;
  auto& W = c->glws;
  TTS_CHECK(G.ready, "glow weights not finalized");
  TTS_CHECK(B >= 1 && B <= 64 && T >= 1 && T <= 4096, "glow: bad sizes");
  for (int b = 0; b < B; ++b) TTS_CHECK(h_lens[b] >= 1 && h_lens[b] <= T, "glow: lens out of range");
  if (h_spk) {
    // the reference looks g up in emb_g (absent unless num_speakers > 1) and feeds it to every WN
    // cond_layer (absent unless c_in_channels > 0): glow_tts.py:160, glow.py:119-120
    TTS_CHECK(G.n_spk > 1, "glow: speaker ids given but the model has no emb_g (num_speakers <= 1)");
    TTS_CHECK(G.c_in > 0, "glow: speaker ids given but the model has no cond_layer (c_in_channels = 0)");
    for (int b = 0; b < B; ++b) TTS_CHECK(h_spk[b] >= 0 && h_spk[b] < G.n_spk, "glow: speaker id out of range");
  } else {
    // without g the reference's duration predictor reads x alone (encoder.py:136), which its
    // conv_1 rejects when it was built for hidden + c_in_channels inputs
    TTS_CHECK(G.c_in == 0, "glow: this model's duration predictor expects speaker conditioning (c_in_channels > 0)");
  }
  hipStream_t s = c->s;
  const int H = G.H, C = G.C, F = G.Fdp;
  long gen = 0;
  grow<int>(W.lens, 64, gen);
  grow<int>(W.ylens, 64, gen);
  grow<int>(W.klens, 64, gen);
  grow<float>(W.xa, (size_t)B * 2 * H * T, gen);
  grow<float>(W.xb, (size_t)B * H * T, gen);
  grow<float>(W.h2, (size_t)B * 2 * H * T, gen);
  grow<float>(W.hdp, (size_t)B * F * T, gen);
  grow<float>(W.logw, (size_t)B * T, gen);
  grow<float>(W.cum, (size_t)B * T, gen);
  grow<float>(W.wceil, (size_t)B * T, gen);
  grow<float>(W.om, (size_t)B * C * T, gen);
  if (G.tfm) grow<float>(W.big, (size_t)B * 768 * T, gen);
  W.B = B;
  W.Tx = T;
  W.has_g = h_spk != nullptr;
  std::vector<int> lens(h_lens, h_lens + B);
  HIP_OK(hipMemcpyAsync(W.lens.p, lens.data(), B * 4, hipMemcpyHostToDevice, s));
  const int* dl = W.lens.i();
  if (W.has_g) {
    // g, then every WN layer's gate bias cond_layer(g) as one (B, flows * wn_layers * 2H) 1x1 conv
    // over a length-1 sequence
    const int NC = G.flows * G.wn_layers * 2 * H;
    grow<int>(W.spk, 64, gen);
    grow<float>(W.g, (size_t)B * G.c_pad, gen);
    grow<float>(W.gcond, (size_t)B * NC, gen);
    if (!W.ones.p) {
      std::vector<int> one(64, 1);
      W.ones.upload(one);
    }
    W.h_spk.assign(h_spk, h_spk + B);
    HIP_OK(hipMemcpyAsync(W.spk.p, W.h_spk.data(), B * 4, hipMemcpyHostToDevice, s));
    launch_glow_speaker(W.spk.i(), G.emb_g.f(), G.c_in, G.c_pad, W.g.f(), B, s);
    ConvCall cc;
    cc.lens = W.ones.i();
    cc.B = B;
    cc.oflow = x3_flag(c);
    cc.max_q = 1;
    cc.s[0] = src_of(W.g.f(), G.c_pad, 1, 1, G.c_pad, 0);
    cc.out = W.gcond.f();
    cc.ob = NC;
    cc.oc = 1;
    cc.ot = 1;
    run_conv(G.cond, cc, s);
  }
  float* x = W.xa.f();   // (B, H, T) current activations
  float* x2 = W.xb.f();  // ping-pong
  launch_glow_embed(d_ids, T, G.emb.f(), G.num_chars, H, dl, x, B, s);
  auto conv = [&](const ConvLayer& L, const float* in, int cin, float* out, int cout, int epi,
                  const float* resid = nullptr) {
    ConvCall cc;
    cc.lens = dl;
    cc.B = B;
    cc.oflow = x3_flag(c);
    cc.max_q = T;
    cc.s[0] = src_of(in, (long)cin * T, T, 1, cin, 0);
    cc.out = out;
    cc.ob = (long)cout * T;
    cc.oc = T;
    cc.ot = 1;
    cc.epi = epi;
    cc.resid = resid;
    cc.rb = (long)cout * T;
    cc.rc = T;
    cc.rt = 1;
    run_conv(L, cc, s);
  };
  if (G.tdsep || G.tfm) {
    // ConvLayerNorm prenet (glow.py:43-50): 3 x (conv k5 -> LayerNorm -> ReLU), x + proj(.)
    float* h0 = W.h2.f();
    float* h1 = W.hdp.f();
    conv(G.pre_conv[0], x, H, h0, H, 0);
    launch_ln(h0, (long)H * T, H, G.pre_g[0].f(), G.pre_b[0].f(), dl, B, T, s, true);
    conv(G.pre_conv[1], h0, H, h1, H, 0);
    launch_ln(h1, (long)H * T, H, G.pre_g[1].f(), G.pre_b[1].f(), dl, B, T, s, true);
    conv(G.pre_conv[2], h1, H, h0, H, 0);
    launch_ln(h0, (long)H * T, H, G.pre_g[2].f(), G.pre_b[2].f(), dl, B, T, s, true);
    conv(G.pre_proj, h0, H, x2, H, 0, x);
    std::swap(x, x2);
    // Transformer (transformer.py:307-319): x = LN1(x + o(attn(x))), x = LN2(x + FFN(x))
    for (int i = 0; i < (G.tfm ? G.enc_layers : 0); ++i) {
      float* big = W.big.f();
      conv(G.tfm_qkv[i], x, H, big, 3 * H, 0);
      launch_glow_mha(big, H, H / 96, T, dl, h0, B, s);
      conv(G.tfm_o[i], h0, H, x2, H, 0, x);
      launch_ln(x2, (long)H * T, H, G.tfm_g1[i].f(), G.tfm_b1[i].f(), dl, B, T, s);
      conv(G.tfm_f1[i], x2, H, big, 768, 1);
      conv(G.tfm_f2[i], big, 768, x, H, 0, x2);
      launch_ln(x, (long)H * T, H, G.tfm_g2[i].f(), G.tfm_b2[i].f(), dl, B, T, s);
    }
    // TimeDepthSeparableConvBlock (time_depth_sep_conv.py:51-63, 93-96)
    for (int i = 0; i < (G.tdsep ? G.enc_layers : 0); ++i) {
      conv(G.tds_tc[i], x, H, h0, H, 6);  // time_conv + BN + GLU -> H rows
      launch_tds_depthwise(h0, H, T, G.tds_dw[i].f(), G.tds_dwb[i].f(), dl, h1, B, s);
      conv(G.tds_tc2[i], h1, H, x2, H, 0, x);  // time_conv2 + BN + residual
      std::swap(x, x2);
    }
  }
  for (int i = 0; i < (G.tdsep || G.tfm ? 0 : G.enc_layers); ++i) {  // GatedConvBlock (gated_conv.py:31-42)
    conv(G.enc_conv[i], x, H, W.h2.f(), 2 * H, 0);
    launch_glu_ln_res(W.h2.f(), (long)2 * H * T, 2 * H, G.enc_g[i].f(), G.enc_b[i].f(), x, (long)H * T, x2,
                      (long)H * T, dl, B, T, s);
    std::swap(x, x2);
  }
  conv(G.proj_m, x, H, W.om.f(), C, 0);  // o_mean (encoder.py:125)
  // DurationPredictor (duration_predictor.py:29-40): conv -> relu -> LN, twice, then proj; the
  // input is [x; g] with g constant over time (encoder.py:131-135), masked like x by the conv
  if (G.c_pad > 0) {
    ConvCall cc;
    cc.lens = dl;
    cc.B = B;
    cc.max_q = T;
    cc.nsrc = 2;
    cc.s[0] = src_of(x, (long)H * T, T, 1, H, 0);
    cc.s[1] = src_of(W.g.f(), G.c_pad, 1, 0, G.c_pad, 0);
    cc.out = W.hdp.f();
    cc.ob = (long)F * T;
    cc.oc = T;
    cc.ot = 1;
    cc.epi = 1;
    // two sources: the fp32 conv (conv_x3 stages one source; this k3 conv over ~T x (H + c_pad)
    // inputs is a few microseconds of the call either way)
    run_conv(G.dp1, cc, s);
  } else {
    conv(G.dp1, x, H, W.hdp.f(), F, 1);
  }
  launch_ln(W.hdp.f(), (long)F * T, F, G.dp_g1.f(), G.dp_b1.f(), dl, B, T, s);
  conv(G.dp2, W.hdp.f(), F, W.h2.f(), F, 1);
  launch_ln(W.h2.f(), (long)F * T, F, G.dp_g2.f(), G.dp_b2.f(), dl, B, T, s);
  conv(G.dp_proj, W.h2.f(), F, W.logw.f(), 1, 0);
  launch_glow_durations(W.logw.f(), T, dl, length_scale, W.cum.f(), W.ylens.i(), W.wceil.f(), B, s);
  HIP_OK(hipMemcpyAsync(h_ylens, W.ylens.p, B * 4, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  int mx = 1;
  W.h_ylens.assign(h_ylens, h_ylens + B);
  W.h_klens.resize(B);
  for (int b = 0; b < B; ++b) mx = std::max(mx, (int)h_ylens[b]);
  W.Ty = mx;
}

// expand + noise + reverse flows after glow_encode: d_y (B, 80, 2*(Ty/2)), d_ymean (B, 80, Ty),
// d_attn (B, Ty, Tx), d_logw (B, Tx) = o_dur_log; d_noise (B, 80, Ty) standard normal or null
void glow_decode(tts_ctx* c, const float* d_noise, float noise_scale, int Ty, float* d_y, float* d_ymean,
                 float* d_attn, float* d_logw) {
  auto& G = c->glow;
  auto& W = c->glws;
  TTS_CHECK(W.B > 0 && Ty == W.Ty, "glow: decode after encode with Ty = max(y_lengths)");
  hipStream_t s = c->s;
  const int B = W.B, Tx = W.Tx, H = G.H, C = G.C, C2 = 2 * C, K = Ty / 2;
  long gen = 0;
  const int K1 = std::max(K, 1);
  grow<float>(W.z, (size_t)B * C * Ty, gen);
  grow<float>(W.sq, (size_t)B * C2 * K1, gen);
  grow<float>(W.sq2, (size_t)B * C2 * K1, gen);
  grow<float>(W.whs, (size_t)B * 2 * H * K1, gen);
  grow<float>(W.wacts, (size_t)B * H * K1, gen);
  launch_glow_expand(W.om.f(), C, Tx, W.lens.i(), W.cum.f(), W.ylens.i(), Ty, d_noise, noise_scale, d_ymean, W.z.f(),
                     d_attn, B, s);
  HIP_OK(hipMemcpyAsync(d_logw, W.logw.p, (size_t)B * Tx * 4, hipMemcpyDeviceToDevice, s));
  HIP_OK(hipMemsetAsync(d_y, 0, (size_t)B * C * 2 * K * 4, s));
  if (K == 0) return;
  // squeezed lengths floor(y_len / 2) (decoder.py:13-15); the staging vector lives in the
  // workspace so the async copy never reads a dead host buffer
  for (int b = 0; b < B; ++b) W.h_klens[b] = W.h_ylens[b] / 2;
  HIP_OK(hipMemcpyAsync(W.klens.p, W.h_klens.data(), B * 4, hipMemcpyHostToDevice, s));
  const int* kl = W.klens.i();
  launch_glow_squeeze(W.z.f(), C, Ty, W.ylens.i(), W.sq.f(), K, B, s);
  // every activation is (B, rows, K) with a per-buffer batch stride (in rows)
  auto conv = [&](const ConvLayer& L, const float* in, int in_rows, float* out, int out_rows, const float* resid,
                  int epi, int resid_rows = 0, const float* aux = nullptr) {
    ConvCall cc;
    cc.lens = kl;
    cc.B = B;
    cc.oflow = x3_flag(c);
    cc.max_q = K;
    cc.s[0] = src_of(in, (long)in_rows * K, K, 1, L.Cin, 0);
    cc.out = out;
    cc.ob = (long)out_rows * K;
    cc.oc = K;
    cc.ot = 1;
    cc.resid = resid;
    cc.rb = (long)out_rows * K;
    cc.rc = K;
    cc.rt = 1;
    cc.epi = epi;
    cc.resid_rows = resid_rows;
    cc.aux = aux;
    cc.auxb = (long)G.flows * G.wn_layers * 2 * H;  // epi 3: gcond's batch stride
    run_conv(L, cc, s);
  };
  float* x = W.sq.f();
  float* x2 = W.sq2.f();
  float* hid = W.whs.f();                 // [hidden | skip] (B, 2H, K)
  float* skip = W.whs.f() + (size_t)H * K;
  for (int k = G.flows - 1; k >= 0; --k) {
    // CouplingBlock reverse (glow.py:245-262): WN over start(x0), then z1 = (x1 - m) exp(-logs)
    conv(G.start[k], x, C2, hid, 2 * H, nullptr, 0);
    for (int i = 0; i < G.wn_layers; ++i) {  // WN (glow.py:118-138)
      const int li = k * G.wn_layers + i;
      // gate fused; with g, cond_layer(g)'s slice for this layer is a per-utterance gate bias
      conv(G.wn_in[li], hid, 2 * H, W.wacts.f(), H, nullptr, 3, 0, W.has_g ? W.gcond.f() + (size_t)li * 2 * H : nullptr);
      // skip rows start at the first layer's output (no accumulate), hidden rows add the residual
      if (i < G.wn_layers - 1) conv(G.wn_rs[li], W.wacts.f(), H, hid, 2 * H, hid, 0, i == 0 ? H : 0);
      else conv(G.wn_rs[li], W.wacts.f(), H, skip, 2 * H, i == 0 ? nullptr : skip, 0);
    }
    // end conv + coupling + inverse InvConvNear / ActNorm: reads x, writes the next x
    conv(G.end[k], skip, 2 * H, x2, C2, x, 5, 0, G.invtab[k].f());
    std::swap(x, x2);
  }
  launch_glow_unsqueeze(x, C2, K, W.ylens.i(), d_y, 2 * K, B, s);
  HIP_OK(hipStreamSynchronize(s));
}

void pwgan_finalize(tts_ctx* c, int layers, int stacks, const int32_t* ups, int n_up) {
  auto& P = c->pw;
  const auto& h = c->pw_host;
  P.ready = false;
  TTS_CHECK(layers >= 1 && layers <= 64 && stacks >= 1 && layers % stacks == 0, "pwgan: layers / stacks");
  TTS_CHECK(n_up >= 1 && n_up <= 6, "pwgan: upsample factors");
  const int R = 64, G = 128, A = 80, S = 64, K1 = 3 * R + A;
  P.layers = layers;
  P.stacks = stacks;
  P.ups.assign(ups, ups + n_up);
  P.first_w.upload(wn_weight(h, "first_conv", {R, 1, 1}));
  P.first_b.upload(need(h, "first_conv.bias", {R}).d);
  int p0[8] = {0};
  pack_conv(P.conv_in, wn_weight(h, "upsample_net.conv_in", {A, A, 1}), std::vector<float>(A, 0.f), A, A, 1, 1, 1,
            p0);
  P.up_h.clear();
  P.up_h.resize(n_up);
  for (int i = 0; i < n_up; ++i) {
    TTS_CHECK(ups[i] == 2 || ups[i] == 4 || ups[i] == 8, "pwgan: upsample factors must be 2, 4 or 8");
    P.up_h[i].upload(
        wn_weight(h, "upsample_net.upsample.up_layers." + std::to_string(2 * i + 1), {1, 1, 1, 2 * ups[i] + 1}));
  }
  P.W1.clear();
  P.W1.resize(layers);
  P.b1.clear();
  P.b1.resize(layers);
  P.W2.clear();
  P.W2.resize(layers);
  P.b2.clear();
  P.b2.resize(layers);
  P.W1x.clear();
  P.W1x.resize(layers);
  P.W2x.clear();
  P.W2x.resize(layers);
  for (int l = 0; l < layers; ++l) {
    const std::string q = "conv_layers." + std::to_string(l) + ".";
    const auto wd = wn_weight(h, q + "conv", {G, R, 3});
    const auto& bd = need(h, q + "conv.bias", {G}).d;
    const auto wa = wn_weight(h, q + "conv1x1_aux", {G, A, 1});
    // GEMM1 matrix (128 x 272): row r = gate row (r even: r/2, odd: 64 + r/2); column k = tap*64 + ch
    // for the dilated taps, 192 + ch for the aux features
    std::vector<float> m1((size_t)G * K1), bb1(G);
    for (int r = 0; r < G; ++r) {
      const int src = (r & 1) ? G / 2 + r / 2 : r / 2;
      for (int tap = 0; tap < 3; ++tap)
        for (int ch = 0; ch < R; ++ch) m1[(size_t)r * K1 + tap * R + ch] = wd[((size_t)src * R + ch) * 3 + tap];
      for (int ch = 0; ch < A; ++ch) m1[(size_t)r * K1 + 3 * R + ch] = wa[(size_t)src * A + ch];
      bb1[r] = bd[src];
    }
    std::vector<float> sw1((size_t)G * K1);
    swizzle_rows16(m1.data(), G, G, K1, sw1.data());
    P.W1[l].upload(sw1);
    P.b1[l].upload(bb1);
    const auto wo = wn_weight(h, q + "conv1x1_out", {R, G / 2, 1});
    const auto ws = wn_weight(h, q + "conv1x1_skip", {S, G / 2, 1});
    std::vector<float> m2((size_t)(R + S) * (G / 2)), bb2(R + S);
    std::copy(wo.begin(), wo.end(), m2.begin());
    std::copy(ws.begin(), ws.end(), m2.begin() + (size_t)R * (G / 2));
    const auto& bo = need(h, q + "conv1x1_out.bias", {R}).d;
    const auto& bs = need(h, q + "conv1x1_skip.bias", {S}).d;
    std::copy(bo.begin(), bo.end(), bb2.begin());
    std::copy(bs.begin(), bs.end(), bb2.begin() + R);
    std::vector<float> sw2(m2.size());
    swizzle_rows16(m2.data(), R + S, R + S, G / 2, sw2.data());
    P.W2[l].upload(sw2);
    P.b2[l].upload(bb2);
    bool in_range = true;
    for (float v : m1) in_range &= std::fabs(v) < F16_RANGE;
    for (float v : m2) in_range &= std::fabs(v) < F16_RANGE;
    if (in_range) {
      std::vector<uint16_t> w1x, w2x;
      pack_pw_layer_x3(m1, m2, w1x, w2x);
      P.W1x[l].upload(w1x);
      P.W2x[l].upload(w2x);
    }
  }
  P.W3.upload(wn_weight(h, "last_conv_layers.1", {S, S, 1}));
  P.b3.upload(need(h, "last_conv_layers.1.bias", {S}).d);
  P.w4.upload(wn_weight(h, "last_conv_layers.3", {1, S, 1}));
  P.b4.upload(need(h, "last_conv_layers.3.bias", {1}).d);
  HIP_OK(hipDeviceSynchronize());
  P.ready = true;
}

// ParallelWaveganGenerator.inference (parallel_wavegan_generator.py:120-125) for B mels of
// h_lens[b] frames: replicate pad p, upsample, WaveNet, output (B, 1, hop * (M_max + 2p)),
// row b zero past hop * (h_lens[b] + 2p). d_noise (B, 1, hop * (M_max + 2p)) standard normal.
void pwgan_infer(tts_ctx* c, const float* mel, const int32_t* h_lens, int B, int M_max, int pad, const float* noise,
                 float* out) {
  auto& P = c->pw;
  auto& W = c->pws;
  TTS_CHECK(P.ready, "pwgan weights not finalized");
  TTS_CHECK(B >= 1 && M_max >= 1 && pad >= 0 && pad <= 64, "pwgan: bad sizes");
  for (int b = 0; b < B; ++b) TTS_CHECK(h_lens[b] >= 1 && h_lens[b] <= M_max, "pwgan: mel lens out of range");
  hipStream_t s = c->s;
  int hop = 1;
  for (int u : P.ups) hop *= u;
  const int Lf = M_max + 2 * pad, Tmax = Lf * hop;
  W.lens.ensure(B * 4);
  W.ca.ensure((size_t)B * 80 * Tmax * 4);
  W.cb.ensure((size_t)B * 80 * Tmax * 4);
  W.xa.ensure((size_t)B * 64 * Tmax * 4);
  W.xb.ensure((size_t)B * 64 * Tmax * 4);
  W.skip.ensure((size_t)B * 64 * Tmax * 4);
  std::vector<int> lens(h_lens, h_lens + B);
  HIP_OK(hipMemcpyAsync(W.lens.p, lens.data(), B * 4, hipMemcpyHostToDevice, s));
  const int* dl = W.lens.i();
  // replicate pad + ConvUpsample.conv_in (1x1, frame rate)
  ConvCall cc;
  cc.lens = dl;
  cc.B = B;
  cc.len_add = 2 * pad;
  cc.s[0] = src_of(mel, (long)80 * M_max, M_max, 1, 80, 0);
  cc.oflow = x3_flag(c);
  cc.pad_mode = 2;
  cc.rep_pad = pad;
  cc.max_q = Lf;
  float* cin = W.cb.f();
  float* cout = W.ca.f();
  cc.out = cin;
  cc.ob = (long)80 * Lf;
  cc.oc = Lf;
  cc.ot = 1;
  run_conv(P.conv_in, cc, s);
  int L = Lf, mul = 1;
  for (size_t i = 0; i < P.ups.size(); ++i) {
    const int u = P.ups[i];
    launch_pw_upsample(cin, (long)80 * L, L, dl, 2 * pad, mul, u, P.up_h[i].f(), cout, (long)80 * L * u, L * u, 80, B,
                       s);
    std::swap(cin, cout);
    L *= u;
    mul *= u;
  }
  const float* cfeat = cin;  // (B, 80, Tmax)
  float* x = W.xa.f();
  float* xn = W.xb.f();
  launch_pw_first(noise, Tmax, P.first_w.f(), P.first_b.f(), dl, 2 * pad, hop, x, Tmax, B, s);
  if (!W.zeros.p) {
    W.zeros.ensure(256 * 4);
    HIP_OK(hipMemsetAsync(W.zeros.p, 0, 256 * 4, s));
  }
  // residual-block kernel: LDS-DMA ring (default) or register staging (TTS_PWGAN_STAGING=regs)
  static const int variant = [] {
    const char* e = std::getenv("TTS_PWGAN_STAGING");
    if (e && std::string(e) == "regs") return 0;
    if (e && std::string(e) == "ring4") return 2;
    return 1;
  }();
  const int per_stack = P.layers / P.stacks;
  unsigned* flag = x3_flag(c);
  for (int l = 0; l < P.layers; ++l) {
    if (flag && P.W1x[l].p)
      launch_pw_layer_x3(x, cfeat, xn, W.skip.f(), P.W1x[l].p, P.b1[l].f(), P.W2x[l].p, P.b2[l].f(), dl, h_lens,
                         2 * pad, hop, Tmax, 1 << (l % per_stack), l == 0, B, flag, s);
    else
      launch_pw_layer(x, cfeat, xn, W.skip.f(), P.W1[l].f(), P.b1[l].f(), P.W2[l].f(), P.b2[l].f(), dl, W.zeros.f(),
                      2 * pad, hop, Tmax, 1 << (l % per_stack), l == 0, B, variant, s);
    std::swap(x, xn);
  }
  launch_pw_out(W.skip.f(), std::sqrt(1.0f / P.layers), P.W3.f(), P.b3.f(), P.w4.f(), P.b4.f(), dl, 2 * pad, hop,
                Tmax, out, B, s);
  HIP_OK(hipStreamSynchronize(s));
}

void set_tensor(HostMap& m, const char* name, const float* h, const int64_t* shape, int ndim) {
  TTS_CHECK(name && (h || ndim == 0), "set_tensor: null argument");
  HostT t;
  size_t n = 1;
  for (int i = 0; i < ndim; ++i) {
    TTS_CHECK(shape[i] >= 0, "negative dim");
    t.shape.push_back(shape[i]);
    n *= (size_t)shape[i];
  }
  t.d.assign(h, h + n);
  m[name] = std::move(t);
}

}  // namespace

extern "C" {

int tts_version(void) { return 1; }
const char* tts_last_error(void) { return g_err.c_str(); }

int tts_ctx_create(int device, tts_ctx** out) {
  return guarded([&] {
    TTS_CHECK(out, "null out");
    int n = 0;
    HIP_OK(hipGetDeviceCount(&n));
    TTS_CHECK(device >= 0 && device < n, "invalid device");
    auto c = std::make_unique<tts_ctx>();
    c->device = device;
    if (const char* e = std::getenv("TTS_GEMM")) c->gemm_x3 = std::string(e) != "f32";
    DeviceGuard g(device);
    HIP_OK(hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking));
    const char* vs = std::getenv("TTS_VOC_STREAM");
    if (vs && std::atoi(vs) == 0) c->sv = c->s;
    else HIP_OK(hipStreamCreateWithFlags(&c->sv, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&c->ev_sv, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&c->ev_chunk[0], hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&c->ev_chunk[1], hipEventDisableTiming));
    for (auto& e : c->ev_dec) HIP_OK(hipEventCreate(&e));
    HIP_OK(hipEventCreateWithFlags(&c->ev_status, hipEventDisableTiming));
    for (auto& t : c->vt) HIP_OK(hipEventCreateWithFlags(&t.ev, hipEventDisableTiming));
    HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&c->pinned), 1024, hipHostMallocDefault));
    std::memset(c->pinned, 0, 1024);
    *out = c.release();
  });
}

int tts_ctx_destroy(tts_ctx* c) {
  return guarded([&] {
    if (!c) return;
    { std::lock_guard<std::recursive_mutex> lk(c->mu); }  // a call still inside the context ends first
    {
      DeviceGuard g(c->device);
      (void)hipStreamSynchronize(c->sv);
      (void)hipStreamSynchronize(c->s);
      for (auto& ge : c->tws.graphs)
        if (ge) {
          (void)hipGraphExecDestroy(ge);
          ge = nullptr;
        }
    }
    int dev = c->device;
    {
      DeviceGuard g(dev);
      hipStream_t s = c->s, sv = c->sv;
      std::vector<hipEvent_t> e = {c->ev_in, c->ev_out, c->ev_chunk[0], c->ev_chunk[1], c->ev_sv};
      for (auto ev : c->ev_dec) e.push_back(ev);
      e.push_back(c->ev_status);
      for (auto& t : c->vt) e.push_back(t.ev);
      int* pin = c->pinned;
      delete c;
      for (auto ev : e) (void)hipEventDestroy(ev);
      if (sv && sv != s) (void)hipStreamDestroy(sv);
      (void)hipStreamDestroy(s);
      (void)hipHostFree(pin);
    }
  });
}

int tts_taco_set_tensor(tts_ctx* c, const char* name, const float* h, const int64_t* shape, int ndim) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c, "null ctx");
    set_tensor(c->taco_host, name, h, shape, ndim);
  });
}

// finalize consumes the tensors staged by *_set_tensor, so the next model starts from an empty map
struct HostMapConsumer {
  HostMap& m;
  ~HostMapConsumer() { m.clear(); }
};

int tts_taco_finalize(tts_ctx* c, int num_chars, int r_init, int attn_norm) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c, "null ctx");
    TTS_CHECK(attn_norm == 0 || attn_norm == 1, "attn_norm must be 0 (sigmoid) or 1 (softmax)");
    TTS_CHECK(r_init >= 1 && r_init <= 16, "r_init out of range");
    DeviceGuard g(c->device);
    HostMapConsumer consume{c->taco_host};  // staged tensors are consumed, even on failure
    taco_finalize(c, num_chars, r_init, attn_norm);
  });
}

int tts_taco_infer(tts_ctx* c, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max, int r,
                   const int32_t* h_max_steps, int S_cap, float thr, float* d_dec, float* d_post, float* d_align,
                   float* d_stop, int32_t* h_steps, int32_t* h_status, void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && d_ids && h_lens && h_max_steps && d_dec && d_post && d_align && d_stop && h_steps && h_status,
              "null argument");
    DeviceGuard g(c->device);
    with_x3_fallback(c, [&] {
      taco_infer(c, d_ids, h_lens, B, T_max, r, h_max_steps, S_cap, thr, d_dec, d_post, d_align, d_stop, h_steps,
                 h_status, stream);
    });
  });
}

int tts_taco_infer_spk(tts_ctx* c, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max, int r,
                       const int32_t* h_max_steps, int S_cap, float thr, const int64_t* d_spk_ids,
                       const float* d_spk_emb, float* d_dec, float* d_post, float* d_align, float* d_stop,
                       int32_t* h_steps, int32_t* h_status, void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && d_ids && h_lens && h_max_steps && d_dec && d_post && d_align && d_stop && h_steps && h_status,
              "null argument");
    DeviceGuard g(c->device);
    with_x3_fallback(c, [&] {
      taco_infer(c, d_ids, h_lens, B, T_max, r, h_max_steps, S_cap, thr, d_dec, d_post, d_align, d_stop, h_steps,
                 h_status, stream, d_spk_ids, d_spk_emb);
    });
  });
}

int tts_taco_set_options(tts_ctx* c, int windowing, int forward_attn, int forward_attn_mask) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c, "null ctx");
    c->taco.windowing = windowing != 0;
    c->taco.forward_attn = forward_attn != 0;
    c->taco.forward_attn_mask = forward_attn_mask != 0;
  });
}

int tts_taco_speaker_dim(tts_ctx* c, int* spk_dim, int* num_speakers) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && spk_dim && num_speakers, "null argument");
    TTS_CHECK(c->taco.ready, "tacotron2 weights not finalized");
    *spk_dim = c->taco.spk_dim;
    *num_speakers = c->taco.num_spk;
  });
}

int tts_taco_encoder(tts_ctx* c, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max, float* d_out,
                     void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && d_ids && h_lens && d_out, "null argument");
    TTS_CHECK(c->taco.ready, "tacotron2 weights not finalized");
    TTS_CHECK(B >= 1 && B <= BMAX && T_max >= 1, "bad sizes");
    for (int b = 0; b < B; ++b) TTS_CHECK(h_lens[b] >= 1 && h_lens[b] <= T_max, "lens out of range");
    DeviceGuard g(c->device);
    taco_workspace(c, B, T_max, std::max(1, c->tws.S_cap), std::max(1, c->tws.r));
    enter(c, stream);
    std::vector<int> lens(h_lens, h_lens + B);
    HIP_OK(hipMemcpyAsync(c->tws.lens.p, lens.data(), B * 4, hipMemcpyHostToDevice, c->s));
    with_x3_fallback(c, [&] { run_encoder(c, d_ids, B, T_max, d_out, c->s); });
    check_encoder_barrier(c);
    leave(c, stream);
  });
}

int tts_taco_postnet(tts_ctx* c, const float* d_dec, const int32_t* h_lens, int B, int M_max, float* d_out,
                     void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && d_dec && h_lens && d_out, "null argument");
    TTS_CHECK(c->taco.ready, "tacotron2 weights not finalized");
    TTS_CHECK(B >= 1 && B <= BMAX && M_max >= 1, "bad sizes");
    DeviceGuard g(c->device);
    auto& W = c->tws;
    long gen = W.gen;
    grow<int>(W.mlens, BMAX, gen);
    grow<float>(W.pa, (size_t)B * 512 * M_max, gen);
    grow<float>(W.pbb, (size_t)B * 512 * M_max, gen);
    W.gen = gen;
    int maxM = 0;
    for (int b = 0; b < B; ++b) {
      TTS_CHECK(h_lens[b] >= 1 && h_lens[b] <= M_max, "lens out of range");
      maxM = std::max(maxM, (int)h_lens[b]);
    }
    enter(c, stream);
    std::vector<int> lens(h_lens, h_lens + B);
    HIP_OK(hipMemcpyAsync(W.mlens.p, lens.data(), B * 4, hipMemcpyHostToDevice, c->s));
    HIP_OK(hipMemsetAsync(d_out, 0, (size_t)B * M_max * 80 * 4, c->s));
    with_x3_fallback(c, [&] {
      run_postnet(c, d_dec, (long)M_max * 80, W.mlens.i(), B, M_max, maxM, d_out, (long)M_max * 80, c->s);
    });
    HIP_OK(hipStreamSynchronize(c->s));
    leave(c, stream);
  });
}

int tts_taco_decoder_state(tts_ctx* c, int B, int T_max, float* d_att_h, float* d_att_c, float* d_dec_h,
                           float* d_dec_c, float* d_context, float* d_alpha, float* d_alpha_cum, void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c, "null ctx");
    TTS_CHECK(c->last_B > 0, "run tts_taco_infer first");
    TTS_CHECK(B == c->last_B && T_max == c->last_T,
              "decoder state: the buffers' (B, T_max) differ from the last decode on this context");
    TTS_CHECK(c->dec_path == 1 && c->dec_nlaunch >= 1, "decoder state: the last decode did not run the persistent "
                                                       "decoder (TTS_DECODER=graph or a non-256-CU device)");
    DeviceGuard g(c->device);
    auto& W = c->tws;
    // the last executed step t_end - 1 wrote h_dec into hdec[(t_end - 1) & 1 ? 0 : 1]
    // (decoder_persist.hip P5: hd_nxt = (t & 1) ? hdec0 : hdec1)
    const int t_end = c->dec_end[c->dec_nlaunch - 1];
    TTS_CHECK(t_end >= 1, "decoder state: no decoder step ran");
    const float* hdec = ((t_end - 1) & 1) ? W.hdec0.f() : W.hdec1.f();
    enter(c, stream);
    taco_state_kernel<<<dim3(4, c->last_B), 256, 0, c->s>>>(W.hatt.f(), W.catt.f(), hdec, W.cdec.f(), W.ctx.f(),
                                                            W.alpha.f(), W.acum.f(), W.map.i() + BMAX, c->last_T,
                                                            c->dec_presplit ? 1 : 0, d_att_h, d_att_c, d_dec_h, d_dec_c, d_context, d_alpha,
                                                            d_alpha_cum);
    HIP_OK(hipGetLastError());
    leave(c, stream);
  });
}

int tts_pwgan_set_tensor(tts_ctx* c, const char* name, const float* h, const int64_t* shape, int ndim) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c, "null ctx");
    set_tensor(c->pw_host, name, h, shape, ndim);
  });
}

int tts_pwgan_finalize(tts_ctx* c, int num_res_blocks, int stacks, const int32_t* upsample_factors, int n_up) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && upsample_factors, "null argument");
    DeviceGuard g(c->device);
    HostMapConsumer consume{c->pw_host};
    pwgan_finalize(c, num_res_blocks, stacks, upsample_factors, n_up);
  });
}

int tts_pwgan_infer(tts_ctx* c, const float* d_mel, const int32_t* h_lens, int B, int M_max, int pad,
                    const float* d_noise, float* d_out, void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && d_mel && h_lens && d_noise && d_out, "null argument");
    DeviceGuard g(c->device);
    enter(c, stream);
    with_x3_fallback(c, [&] { pwgan_infer(c, d_mel, h_lens, B, M_max, pad, d_noise, d_out); });
    leave(c, stream);
  });
}

int tts_glow_set_tensor(tts_ctx* c, const char* name, const float* h, const int64_t* shape, int ndim) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c, "null ctx");
    set_tensor(c->glow_host, name, h, shape, ndim);
  });
}

int tts_glow_finalize(tts_ctx* c, int num_chars, int enc_layers, int num_flow_blocks, int num_block_layers) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c, "null ctx");
    DeviceGuard g(c->device);
    HostMapConsumer consume{c->glow_host};
    glow_finalize(c, num_chars, enc_layers, num_flow_blocks, num_block_layers);
  });
}

int tts_glow_encode(tts_ctx* c, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max, float length_scale,
                    int32_t* h_ylens, void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && d_ids && h_lens && h_ylens, "null argument");
    DeviceGuard g(c->device);
    enter(c, stream);
    with_x3_fallback(c, [&] { glow_encode(c, d_ids, h_lens, nullptr, B, T_max, length_scale, h_ylens); });
    leave(c, stream);
  });
}

int tts_glow_encode_spk(tts_ctx* c, const int64_t* d_ids, const int32_t* h_lens, const int32_t* h_speaker_ids, int B,
                        int T_max, float length_scale, int32_t* h_ylens, void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && d_ids && h_lens && h_ylens, "null argument");
    DeviceGuard g(c->device);
    enter(c, stream);
    with_x3_fallback(c, [&] { glow_encode(c, d_ids, h_lens, h_speaker_ids, B, T_max, length_scale, h_ylens); });
    leave(c, stream);
  });
}

int tts_glow_decode(tts_ctx* c, const float* d_noise, float noise_scale, int Ty, float* d_y, float* d_ymean,
                    float* d_attn, float* d_logw, void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && d_y && d_ymean && d_attn && d_logw, "null argument");
    DeviceGuard g(c->device);
    enter(c, stream);
    with_x3_fallback(c, [&] { glow_decode(c, d_noise, noise_scale, Ty, d_y, d_ymean, d_attn, d_logw); });
    leave(c, stream);
  });
}

int tts_ge2e_set_tensor(tts_ctx* c, const char* name, const float* h, const int64_t* shape, int ndim) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c, "null ctx");
    set_tensor(c->ge2e_host, name, h, shape, ndim);
  });
}

int tts_ge2e_finalize(tts_ctx* c, int input_dim, int proj_dim, int lstm_dim, int num_lstm_layers,
                      int use_lstm_with_projection) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c, "null ctx");
    DeviceGuard g(c->device);
    HostMapConsumer consume{c->ge2e_host};
    ge2e_finalize(c, input_dim, proj_dim, lstm_dim, num_lstm_layers, use_lstm_with_projection);
  });
}

int tts_ge2e_infer(tts_ctx* c, const float* d_x, const int32_t* h_lens, int B, int T_max, float* d_out,
                   void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && d_x && h_lens && d_out, "null argument");
    DeviceGuard g(c->device);
    enter(c, stream);
    with_x3_fallback(c, [&] { ge2e_infer(c, d_x, h_lens, B, T_max, d_out); });
    leave(c, stream);
  });
}

int tts_melgan_set_tensor(tts_ctx* c, const char* name, const float* h, const int64_t* shape, int ndim) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c, "null ctx");
    set_tensor(c->mg_host, name, h, shape, ndim);
  });
}

int tts_melgan_finalize(tts_ctx* c, int in_ch, int out_ch, int base, const int32_t* ups, int n_up, int nres,
                        int use_pqmf) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && ups && n_up >= 1 && n_up <= 6, "bad arguments");
    DeviceGuard g(c->device);
    HIP_OK(hipStreamSynchronize(c->sv));  // no submitted vocoder still reads the weights replaced here
    c->sv_live = false;
    HostMapConsumer consume{c->mg_host};
    melgan_finalize(c, in_ch, out_ch, base, ups, n_up, nres, use_pqmf);
  });
}

int tts_melgan_generator(tts_ctx* c, const float* d_mel, const int32_t* h_lens, int B, int M_max, int pad,
                         float* d_out, void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && d_mel && h_lens && d_out, "null argument");
    TTS_CHECK(pad >= 0, "pad >= 0");
    DeviceGuard g(c->device);
    enter(c, stream);
    with_x3_fallback(c, [&] { run_generator(c, d_mel, h_lens, B, M_max, pad, d_out, c->s); });
    leave(c, stream);
  });
}

// MultibandMelganGenerator.inference body on s (default c->s): generator, output conv and PQMF synthesis into
// d_wav (B, 1, hop * (M_max + 2 pad)), rows zero past their own length
static void mbmelgan_body(tts_ctx* c, const float* d_mel, const int64_t* mel_strides, const int32_t* h_lens, int B,
                          int M_max, int pad, float* d_wav, bool dev_lens = false, hipStream_t s = nullptr) {
  if (!s) s = c->s;
  auto& G = c->mg;
  int up = 1;
  for (int u : G.ups) up *= u;
  const long Ls = (long)(M_max + 2 * pad) * up;
  const bool fused = G.out_ch == 4 && G.taps == 62 && (G.C_last == 32 || G.C_last == 48);
  if (fused) {  // launch_out_pqmf writes the rows' zero padding itself
    GenTail t;
    run_generator(c, d_mel, h_lens, B, M_max, pad, nullptr, s, &t, mel_strides, dev_lens);
    TTS_CHECK(t.Ls == Ls, "generator length bookkeeping");
    const int* dl = c->vlens_override ? c->vlens_override : c->mws.lens.i();
    TTS_CHECK(launch_out_pqmf(t.x, (long)t.C * t.Ls, t.Ls, t.C, G.out_w.f(), G.out_b.f(), G.G.f(), G.out_ch,
                              G.taps, dl, 2 * pad, up, (int)Ls, B, d_wav, (long)G.out_ch * Ls, s),
              "fused output/PQMF shape not covered");
  } else {
    HIP_OK(hipMemsetAsync(d_wav, 0, (size_t)B * G.out_ch * Ls * 4, s));
    c->mws.bands.ensure((size_t)B * G.out_ch * Ls * 4);
    run_generator(c, d_mel, h_lens, B, M_max, pad, c->mws.bands.f(), s, nullptr, mel_strides, dev_lens);
    const int* dl = c->vlens_override ? c->vlens_override : c->mws.lens.i();
    launch_pqmf_synthesis(c->mws.bands.f(), (long)G.out_ch * Ls, Ls, G.G.f(), G.out_ch, G.taps, dl,
                          2 * pad, up, (int)Ls, B, d_wav, (long)G.out_ch * Ls, s);
  }
}

static int melgan_infer_impl(tts_ctx* c, const float* d_mel, const int64_t* mel_strides, const int32_t* h_lens, int B,
                      int M_max, int pad, float* d_wav, void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && d_mel && h_lens && d_wav, "null argument");
    TTS_CHECK(pad >= 0, "pad >= 0");
    auto& G = c->mg;
    TTS_CHECK(G.ready && G.pqmf, "melgan (with PQMF) not finalized");
    DeviceGuard g(c->device);
    enter(c, stream);
    with_x3_fallback(c, [&] { mbmelgan_body(c, d_mel, mel_strides, h_lens, B, M_max, pad, d_wav); });
    leave(c, stream);
  });
}

// the shortest mel (frames) the vocoder accepts at inference padding pad: run_generator's checks
static int vocoder_min_len(const MelganModel& G, int pad) {
  int L = std::max(1, 4 - 2 * pad);
  for (int k = 0; k < G.nres && !G.ups.empty(); ++k)
    while ((long)(L + 2 * pad) * G.ups[0] <= G.dconv[k].dil) ++L;
  return L;
}

// completes a submitted fused call: if its split-f16 vocoder raised the range flag, the vocoder
// runs again on the fp32 kernels from the postnet output (the two-call path's fallback); then the
// caller's stream is ordered after it
// the vocoder being enqueued uses a ticket slot's device lengths and range flag
struct VocSlot {
  tts_ctx* c;
  VocSlot(tts_ctx* c_, unsigned* flag, int* lens) : c(c_) {
    c->flag_override = flag;
    c->vlens_override = lens;
  }
  ~VocSlot() {
    c->flag_override = nullptr;
    c->vlens_override = nullptr;
  }
};
// the vocoder work just enqueued on sv: later entries join it (enter)
static void sv_mark(tts_ctx* c) {
  HIP_OK(hipEventRecord(c->ev_sv, c->sv));
  c->sv_live = c->sv != c->s;
}
static void sv_join(tts_ctx* c) {
  if (!c->sv_live) return;
  HIP_OK(hipStreamWaitEvent(c->s, c->ev_sv, 0));
  c->sv_live = false;
}

static void finish_ticket(tts_ctx* c, VocTicket& tk, void* stream) {
  if (!tk.pending) return;
  tk.pending = false;
  if (tk.x3) {
    HIP_OK(hipEventSynchronize(tk.ev));
    const int k = (int)(tk.id % NVT);
    if (c->pinned[TK_PIN + k]) {
      c->x3_fallbacks++;
      c->gemm_x3 = false;
      try {  // on sv, behind any later submission's vocoder; the slot's lengths from the host
        VocSlot vs(c, nullptr, vslot_lens(c, k));
        mbmelgan_body(c, tk.d_post, tk.st, tk.lens.data(), tk.B, tk.M, tk.pad, tk.d_wav, false, c->sv);
      } catch (...) {
        c->gemm_x3 = true;
        throw;
      }
      c->gemm_x3 = true;
      HIP_OK(hipEventRecord(tk.ev, c->sv));
      sv_mark(c);
    }
  }
  HIP_OK(hipStreamWaitEvent((hipStream_t)stream, tk.ev, 0));
}

// Tacotron2 decode + MB-MelGAN, submitted: the vocoder is launched on the device-side decoded
// lengths before the host waits for the decode's status words, and the call returns with the
// vocoder still running (ticket); finish_ticket completes it.
static int64_t taco_mbmelgan_submit(tts_ctx* c, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max, int r,
                                    const int32_t* h_max_steps, int S_cap, float thr, const int64_t* d_spk_ids,
                                    const float* d_spk_emb, float* d_dec, float* d_post, float* d_align,
                                    float* d_stop, int pad, float* d_wav, int32_t* h_steps, int32_t* h_status,
                                    void* stream) {
  TTS_CHECK(d_ids && h_lens && h_max_steps && d_dec && d_post && d_align && d_stop && d_wav && h_steps && h_status,
            "null argument");
  TTS_CHECK(pad >= 0, "pad >= 0");
  auto& G = c->mg;
  TTS_CHECK(G.ready && G.pqmf, "melgan (with PQMF) not finalized");
  TTS_CHECK(G.in_ch == 80, "vocoder input channels must be the decoder's 80 mel channels");
  TTS_CHECK(B >= 1 && B <= BMAX && r >= 1, "bad sizes");
  const int64_t id = c->next_ticket++;
  VocTicket& tk = c->vt[id % NVT];
  finish_ticket(c, tk, stream);  // the slot's previous submission completes first
  if (tk.id != 0) HIP_OK(hipStreamWaitEvent(c->s, tk.ev, 0));  // its vocoder is done with the slot
  tk.id = id;
  // per-row upper bounds of the decoded lengths (tile counts of the vocoder's persistent kernels)
  const int Lmin = vocoder_min_len(G, pad);
  std::vector<int32_t> bound(B);
  for (int b = 0; b < B; ++b) {
    TTS_CHECK(h_max_steps[b] >= 1 && h_max_steps[b] <= S_cap, "max_steps out of range");
    bound[b] = h_max_steps[b] * r;
    TTS_CHECK(bound[b] >= Lmin, VOC_SHORT_MSG);
  }
  const int64_t st[3] = {(int64_t)S_cap * r * 80, 1, 80};
  bool voc_x3 = false;
  const int k = (int)(id % NVT);
  int* slot = c->pinned + TK_PIN + k;
  int* vl = vslot_lens(c, k);
  unsigned* vf = vslot_flag(c, k);
  hipStream_t sv = c->sv;
  FusedVoc fv{vl, Lmin, [&] {
                voc_x3 = c->gemm_x3;
                // on sv behind the decode's status event (recorded just before), with the ticket
                // slot's lengths (the status kernel wrote them) and range flag; the vocoder's input
                // is the postnet output read in place, frame-major; rows are hop (S_cap r + 2 pad)
                // samples apart until the decoded lengths are on the host
                if (sv != c->s) HIP_OK(hipStreamWaitEvent(sv, c->ev_status, 0));
                if (voc_x3) HIP_OK(hipMemsetAsync(vf, 0, 4, sv));
                {
                  VocSlot vs(c, vf, vl);
                  mbmelgan_body(c, d_post, st, bound.data(), B, S_cap * r, pad, d_wav, /*dev_lens=*/true, sv);
                }
                if (voc_x3) HIP_OK(hipMemcpyAsync(slot, vf, 4, hipMemcpyDeviceToHost, sv));
                sv_mark(c);
              }};
  c->flag_read = false;
  c->in_submit = true;  // this submission's Tacotron2 does not wait for earlier vocoders on sv
  try {
    taco_infer(c, d_ids, h_lens, B, T_max, r, h_max_steps, S_cap, thr, d_dec, d_post, d_align, d_stop, h_steps,
               h_status, stream, d_spk_ids, d_spk_emb, &fv);
  } catch (...) {
    c->in_submit = false;
    throw;
  }
  c->in_submit = false;
  const bool taco_oflow = c->gemm_x3 && c->flag_read && c->pinned[12];
  c->flag_read = false;
  int S = 0;
  for (int b = 0; b < B; ++b) S = std::max(S, (int)h_steps[b]);
  std::vector<int32_t> mlens(B);
  for (int b = 0; b < B; ++b) mlens[b] = h_steps[b] * r;
  int up = 1;
  for (int u : G.ups) up *= u;
  const size_t row = (size_t)G.out_ch * up;  // hop: samples per mel frame
  if (taco_oflow) {
    // the decode left the f16 range: decode and vocoder again on the fp32 kernels (the split
    // vocoder already queued is overwritten), as the two separate calls would each have done
    c->x3_fallbacks++;
    c->gemm_x3 = false;
    sv_join(c);  // the split vocoder queued on sv writes d_wav before the fp32 one below
    try {
      taco_infer(c, d_ids, h_lens, B, T_max, r, h_max_steps, S_cap, thr, d_dec, d_post, d_align, d_stop, h_steps,
                 h_status, stream, d_spk_ids, d_spk_emb);
      S = 0;
      for (int b = 0; b < B; ++b) {
        S = std::max(S, (int)h_steps[b]);
        mlens[b] = h_steps[b] * r;
      }
      mbmelgan_body(c, d_post, st, mlens.data(), B, S * r, pad, d_wav);
    } catch (...) {
      c->gemm_x3 = true;
      throw;
    }
    c->gemm_x3 = true;
    leave(c, stream);
    return id;
  }
  if (S < S_cap) {  // pack the rows to hop (S r + 2 pad) samples apart, as the two calls return them
    const size_t P = row * ((size_t)S * r + 2 * pad), Pc = row * ((size_t)S_cap * r + 2 * pad);
    c->mws.bands.ensure((size_t)B * P * 4);
    HIP_OK(hipMemcpy2DAsync(c->mws.bands.p, P * 4, d_wav, Pc * 4, P * 4, B, hipMemcpyDeviceToDevice, sv));
    HIP_OK(hipMemcpyAsync(d_wav, c->mws.bands.p, (size_t)B * P * 4, hipMemcpyDeviceToDevice, sv));
  }
  HIP_OK(hipEventRecord(tk.ev, sv));
  sv_mark(c);
  tk.pending = true;
  tk.x3 = voc_x3;
  tk.d_post = d_post;
  std::copy(st, st + 3, tk.st);
  tk.lens = mlens;
  tk.B = B;
  tk.M = S * r;
  tk.pad = pad;
  tk.d_wav = d_wav;
  return id;
}

int tts_taco_mbmelgan_submit(tts_ctx* c, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max, int r,
                             const int32_t* h_max_steps, int S_cap, float thr, const int64_t* d_spk_ids,
                             const float* d_spk_emb, float* d_dec, float* d_post, float* d_align, float* d_stop,
                             int pad, float* d_wav, int32_t* h_steps, int32_t* h_status, int64_t* h_ticket,
                             void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && h_ticket, "null argument");
    DeviceGuard g(c->device);
    *h_ticket = taco_mbmelgan_submit(c, d_ids, h_lens, B, T_max, r, h_max_steps, S_cap, thr, d_spk_ids, d_spk_emb,
                                     d_dec, d_post, d_align, d_stop, pad, d_wav, h_steps, h_status, stream);
  });
}

int tts_taco_mbmelgan_finish(tts_ctx* c, int64_t ticket, void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c, "null ctx");
    TTS_CHECK(ticket >= 1 && ticket < c->next_ticket, "unknown ticket");
    DeviceGuard g(c->device);
    VocTicket& tk = c->vt[ticket % NVT];
    if (tk.id == ticket) finish_ticket(c, tk, stream);  // else a later submission already finished it
  });
}

int tts_taco_mbmelgan_infer(tts_ctx* c, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max, int r,
                            const int32_t* h_max_steps, int S_cap, float thr, const int64_t* d_spk_ids,
                            const float* d_spk_emb, float* d_dec, float* d_post, float* d_align, float* d_stop,
                            int pad, float* d_wav, int32_t* h_steps, int32_t* h_status, void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c, "null ctx");
    DeviceGuard g(c->device);
    const int64_t id = taco_mbmelgan_submit(c, d_ids, h_lens, B, T_max, r, h_max_steps, S_cap, thr, d_spk_ids,
                                            d_spk_emb, d_dec, d_post, d_align, d_stop, pad, d_wav, h_steps, h_status,
                                            stream);
    VocTicket& tk = c->vt[id % NVT];
    if (tk.id == id) finish_ticket(c, tk, stream);
    HIP_OK(hipStreamSynchronize(c->sv));  // returns with the call's work done, as before
    HIP_OK(hipStreamSynchronize(c->s));
  });
}

int tts_melgan_infer(tts_ctx* c, const float* d_mel, const int32_t* h_lens, int B, int M_max, int pad,
                     float* d_wav, void* stream) {
  return melgan_infer_impl(c, d_mel, nullptr, h_lens, B, M_max, pad, d_wav, stream);
}

int tts_melgan_infer_strided(tts_ctx* c, const float* d_mel, int64_t stride_b, int64_t stride_c, int64_t stride_t,
                             const int32_t* h_lens, int B, int M_max, int pad, float* d_wav, void* stream) {
  const int64_t st[3] = {stride_b, stride_c, stride_t};
  return melgan_infer_impl(c, d_mel, st, h_lens, B, M_max, pad, d_wav, stream);
}

int tts_pqmf_synthesis(tts_ctx* c, const float* d_x, int B, int N, int L, const float* d_G, int taps, float* d_y,
                       void* stream) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && d_x && d_G && d_y, "null argument");
    TTS_CHECK(B >= 1 && N >= 1 && N <= 8 && L >= 1 && taps >= 0, "bad sizes");
    DeviceGuard g(c->device);
    enter(c, stream);
    std::vector<int> lens(B, L);
    c->mws.lens.ensure(B * 4);
    HIP_OK(hipMemcpyAsync(c->mws.lens.p, lens.data(), B * 4, hipMemcpyHostToDevice, c->s));
    launch_pqmf_synthesis(d_x, (long)N * L, L, d_G, N, taps, c->mws.lens.i(), 0, 1, L, B, d_y, (long)N * L, c->s);
    HIP_OK(hipStreamSynchronize(c->s));
    leave(c, stream);
  });
}

int tts_set_gemm_mode(tts_ctx* c, int mode) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(mode == 0 || mode == 1, "gemm mode must be 0 (fp32) or 1 (split-f16)");
    c->gemm_x3 = mode == 1;
  });
}

int tts_test_stall_lstm(int recurrence) {
  g_test_stall_lstm.store(recurrence < 0 ? -1 : recurrence);
  return 0;
}

int tts_gemm_mode(tts_ctx* c, int* mode, int64_t* fallbacks) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(mode && fallbacks, "null argument");
    *mode = c->gemm_x3 ? 1 : 0;
    *fallbacks = c->x3_fallbacks;
  });
}

int tts_decoder_stats(tts_ctx* c, int* path, int* nlaunch, float* ms, int* steps) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && path && nlaunch && ms && steps, "bad arguments");
    TTS_CHECK(c->last_B > 0, "run tts_taco_infer first");
    *path = c->dec_path;
    *nlaunch = c->dec_path ? c->dec_nlaunch : 0;
    int prev = 0;
    for (int i = 0; i < *nlaunch; ++i) {
      HIP_OK(hipEventElapsedTime(&ms[i], c->ev_dec[i], c->ev_dec[i + 1]));
      steps[i] = c->dec_end[i] - prev;
      prev = c->dec_end[i];
    }
  });
}

int tts_time_decoder_kernel(tts_ctx* c, int which, int iters, float* ms_out) {
  return guarded_ctx(c, [&] {
    TTS_CHECK(c && ms_out && iters >= 1, "bad arguments");
    TTS_CHECK(c->last_B > 0 && c->tws.graphs[c->tws.MT], "run tts_taco_infer first");
    TTS_CHECK(c->tws.S_cap >= CHUNK + 2, "S_cap too small for timing");
    DeviceGuard g(c->device);
    auto& W = c->tws;
    hipStream_t s = c->s;
    // live state of the last decode, re-armed: base = 1, nothing done, unbounded max steps
    std::vector<int> ctl(4 + 4 * BMAX, 0);
    ctl[0] = 1;
    for (int b = 0; b < BMAX; ++b) ctl[4 + 3 * BMAX + b] = 1 << 30;
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipMemcpyAsync(W.ctl.p, ctl.data(), ctl.size() * 4, hipMemcpyHostToDevice, s));
    if (which == 0) enqueue_step(c, 0, 0, s, W.MT);  // warm-up
    else HIP_OK(hipGraphLaunch(W.graphs[W.MT], s));
    HIP_OK(hipMemcpyAsync(W.ctl.p, ctl.data(), ctl.size() * 4, hipMemcpyHostToDevice, s));
    HIP_OK(hipEventRecord(e0, s));
    for (int i = 0; i < iters; ++i) {
      if (which == 0) enqueue_step(c, 0, 0, s, W.MT);
      else {
        HIP_OK(hipGraphLaunch(W.graphs[W.MT], s));
      }
    }
    HIP_OK(hipEventRecord(e1, s));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    *ms_out = which == 0 ? ms / iters : ms / (iters * CHUNK);
    // leave the control block in a finished state
    ctl[1] = 1;
    HIP_OK(hipMemcpy(W.ctl.p, ctl.data(), ctl.size() * 4, hipMemcpyHostToDevice));
    HIP_OK(hipEventDestroy(e0));
    HIP_OK(hipEventDestroy(e1));
  });
}

}  // extern "C"
