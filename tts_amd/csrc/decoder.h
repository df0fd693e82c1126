// Decoder-step data structures shared by decoder.hip and api.hip.
#pragma once
#include "common.h"

enum { EPI_STORE = 0, EPI_LSTM = 1 };

// GEMM activations live in HBM in MFMA fragment order so that one wave's A-operand load of a
// 16 x 16 block is one contiguous 1 KiB (row-major rows made it 16 half-used cache lines per
// load, the dominant cost of the skinny GEMMs: tools/skinny_bench.hip):
//   element (m, k) of a (Bp x K) activation is at frag_idx(m, k, K)
//   = ((m/16 * K/16 + k/16) * 64 + (k%16)/4 * 16 + m%16) * 4 + k%4
__host__ __device__ inline long frag_idx(int m, int k, int K) {
  return ((long)((m >> 4) * (K >> 4) + (k >> 4)) * 64 + ((k & 15) >> 2) * 16 + (m & 15)) * 4 + (k & 3);
}

struct SkSeg {
  const float* ptr;  // fragment-order activation, at the segment's first 16-column chunk
  int ms;            // floats between 16-row blocks (= 16 * total columns of the activation)
  int K;             // multiple of 16
};

struct SkJob {
  SkSeg seg[3];
  int nseg;
  int K;
  const float* W;      // swizzled [tile][K/16][64][4]
  int ntiles;
  int epi;             // EPI_STORE | EPI_LSTM
  int act;             // store: 0 none, 1 relu
  const float* bias;   // per swizzled row (tile order)
  const float* addin;  // optional pre-activation addend [m][row]
  int addin_ld;
  float* out;          // store target [m][row] (out_frag: fragment order with out_ld columns)
  int out_ld;
  int out_frag;
  float* h_out;        // LSTM: h, fragment order with hc_ld columns
  float* c_state;      // LSTM: c[m][unit], updated in place
  int hc_ld;
  const float* WqT;    // optional: W_query^T [units][128] for partial query projection
  float* pq_part;      // [workgroup][Bp][128]
  int pq_cap;          // workgroup slots in pq_part (checked at launch)
  int frames_r;        // projection: write the first 80*r columns as frames of active utts
  // projection only: the stopnet logit is linear in [h_dec | ctx] once the projection is folded
  // in (stop = w_h.h + w_y.(W_p [h|ctx] + b_p) + b_s), so the folded 1536-vector is row 0 of a
  // leading weight tile (rows 1-15 zero) and its output, bias included, is the logit
  int lead_stop;         // tile 0 is the stopnet tile; outputs of later tiles shift by 16 rows
  float* stop_part;      // [Bp] stop logits
};

struct SkArgs {
  SkJob job[2];
  int njobs;
  int MT;  // batch tiles of 16 (Bp = 16*MT <= 64)
};

struct DecCtl {
  int base;          // step index of j = 0 in the current chunk
  int all_done;      // every utterance finished: all later kernels exit at entry
  int active_tiles;  // 1 + (largest unfinished row) / 16: the host drops to a smaller batch tile
  int pad1;
};

struct DecDev {
  DecCtl* ctl;
  int* done;
  int* steps;
  int* status;          // 1 = stopnet, 2 = max_decoder_steps
  const int* max_steps;
  const int* lens;      // encoder lengths T_b
  float* dec_out;       // (B, S_cap*r, 80)
  float* align_out;     // (B, S_cap, T_max)
  float* stop_out;      // (B, S_cap)
  int S_cap;
  int T_max;
  int B;
};

struct StopArgs {
  const float* part;  // stop logits [Bp] written by the projection kernel
  float threshold;
};

struct AttnArgs {
  const float* pq_part;  // [npq][Bp][128] partial query projections from the attention-LSTM kernel
  int npq;
  int Bp;
  float* alpha;       // (B, T_max) previous step weights, updated by the combining workgroup
  float* alpha_cum;   // (B, T_max)
  const float* Wloc;  // (32, 2, 31)
  const float* WdT;   // location_dense transposed (32, 128)
  const float* v;     // (128)
  float bv;
  const float* penc;  // (B, T_max, 128)
  float* energy;      // (B, T_max) raw energies
  const float* enc;   // (B, T_max, 512)
  float* ctx;         // (Bp, 512)
  float* part_s;      // (B, nchmax) chunk sums of sigmoid(e) / exp(e - m_chunk)
  float* part_m;      // (B, nchmax) chunk max (softmax)
  float* part_u;      // (B, nchmax, 512) chunk partial contexts
  unsigned* counter;  // (B) arrivals of the current step (zeroed per call; reset by the last arriver)
  int nchmax;
  int softmax;
};

// persistent decoder (decoder_persist.hip): every decoder tensor the loop touches
struct PArgs {
  const float* dec_w;   // [256][160][64][4] decoder_rnn [W_ih | W_hh] gate-interleaved tiles
  const float* dec_b;   // [4096]
  const float* apre_w;  // [256][96][64][4] attention_rnn [W_ih,ctx | W_hh]
  const float* apre_b;  // [4096] b_ih + b_hh
  const float* attp_w;  // [256][16][64][4] attention_rnn W_ih,prenet
  const uint16_t* attp_x3;  // the same weights split-f16 (split16.h pack_split_a [256][8][64][16]) or null
  unsigned* x3flag;         // raised when a split-f16 operand is outside the f16 range
  const uint16_t* dec_x3;   // dec_w split-f16 [256 tiles][80 k-steps][64][16] (with attp_x3)
  const uint16_t* apre_x3;  // apre_w split-f16 [256 tiles][48][64][16] (with attp_x3)
  const uint16_t* pj_x3;    // pj_w split-f16 [ntj tiles][48][64][16] (with attp_x3)
  const float* pj_w;    // [ntj][96][64][4] stop tile, 5r frame tiles, 16 folded prenet-1 tiles
  const float* pj_b;    // [ntj * 16]
  // per-row biases (api.hip spk_bias_kernel), row stride spk_ld: projection bias per row (always),
  // speaker parts W_s s of the attention_rnn / decoder_rnn gates and processed inputs (null
  // without speakers)
  const float* pjb_rows;
  const float* spk_att;
  const float* spk_dec;
  const float* spk_penc;
  int spk_ld;
  int spk_scale;  // Graves attention with speakers: speaker biases scale by the row's sum of weights
  // decoder variants (common_layers.py:25-74, 286-372): BN prenet biases (null = original prenet),
  // attention windowing, forward attention (+ transition agent)
  const float* pre1_b0;  // [256] layer-1 bias b1' (BN folded): the prenet input of step 0 is relu(b1')
  const float* pre2_b;   // [256] layer-2 bias b2'
  int win;
  int* win_idx;          // (B) previous argmax, -1 before the first step
  int fwd, trans, fwd_mask;
  float* fwd_u;          // (B) transition probability u, 0.5 before the first step
  float* part_f;         // (B, nchmax) chunk sums of the forward weights
  // Graves attention (VAR bit 2): N_a layer 1 tiles / bias, layer 2 (3K x 1024) / bias, hidden
  // (Bp x 1024, row-major), mixture means carried across steps (B x 16)
  int gK;
  const float *na1_w, *na1_b, *na2_w, *na2_b;
  float *gh, *gmu;
  const float* ta_w;     // [512 ctx | 1024 query]
  float ta_b;
  const float* pre2_w;  // [16][16][64][4]
  const float* WqT;     // [1024][128]
  const float* Wcomb;   // [64][128]: location_dense . location_conv as one 62-tap filter per dim
  const float* v;       // (128)
  float bv;
  int nt_proj, ntj, r;
  const float* penc;  // (B, T_max, 128)
  const float* enc;   // (B, T_max, 512)
  float* ypart;       // [2][64][ntj*16] projection halves
  float* pb;          // prenet output, fragment order (Bp, 256)
  float* gatt;        // [Bp][4096] attention_rnn ctx/h part + biases
  float* hatt;        // fragment order (Bp, 1024)
  float* catt;        // [Bp][1024]
  float* hdec0;       // fragment order (Bp, 1024), double-buffered on t & 1
  float* hdec1;
  float* cdec;        // [Bp][1024]
  float* ctx;         // fragment order (Bp, 512)
  float* pq;          // [128][Bp][128]
  float* alpha;       // (B, T_max)
  float* acum;
  float* energy;
  float* part_s;      // (B, nchmax)
  float* part_m;
  float* part_u;      // (B, nchmax, 512)
  unsigned* counter;  // (B)
  // deferred alignment pass (plain location attention, items per workgroup <= PDEF_MAXIT): the last
  // arriver publishes the step's normaliser S and max m per utterance here, and every item workgroup
  // writes alpha / alpha_cum / the alignment row of its own positions in P6
  float* anorm;       // (B, 2)
  int defer_align;
  int nchmax;
  int softmax;
  float thr;
  unsigned* bar;  // barrier words (zeroed before each launch): [0] global, [32] go, [64 + 32x] XCD x,
                  // [16] error
  int* base_out;  // optional: the step index at exit (launch statistics, read back with the status words)
  unsigned long long* trace;   // optional phase timestamps [8 steps][10][256] (TTS_PTRACE)
  unsigned long long* atrace;  // optional attention-item timestamps [8 steps][256][8]
  int trace_t0;
  unsigned* diag;  // optional (TTS_DIAG_XCC): the XCC id of every workgroup, written at launch
  DecDev D;
};

bool persist_supported(int device);
int persist_attn_tc();  // attention positions per work item (sizes the chunk-partial buffers)
bool persist_defer_ok(int nitems);  // the deferred alignment pass has room for this many items
bool persist_trace_built();          // phase stamps compiled in (-DTTS_PHASE_TRACE)
// time the flag barrier on `ncand` candidate blocks (BAR_WORDS apart from pool) and return the
// `nwant` fastest in slot[] (TTS_BAR_CALIBRATE=0: slots 0 .. nwant-1); one decoder grid per block
void pick_barrier_blocks(unsigned* pool, int ncand, int nwant, int* slot, hipStream_t s);
// arm: zero the barrier block first (false: the caller armed it, e.g. in its state fill)
// ev0 / ev1: optional timing events taken from the launch itself (before / after the kernel)
void launch_persist_decoder(const PArgs& a, int MT, hipStream_t s, bool arm = true, hipEvent_t ev0 = nullptr,
                            hipEvent_t ev1 = nullptr);
// whether that launch publishes h_att / ctx / h_dec pre-split (decoder_persist.hip presplit_of)
bool persist_presplit(const PArgs& a);

void launch_skinny(const SkArgs& a, const DecDev& d, int jstep, int NT, int KS, hipStream_t s);
// prenet layer 1 + layer 2 in one launch (16 workgroups) plus the stop workgroup
void launch_prenet_stop(const SkArgs& a, const DecDev& d, const StopArgs& st, int jstep, hipStream_t s);
void launch_attention(const AttnArgs& p, const DecDev& d, int jstep, hipStream_t s);
void launch_dec_advance(DecCtl* ctl, int n, hipStream_t s);
